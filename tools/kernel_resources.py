"""Per-kernel register, LDS and scratch use of libsed.so's gfx950 code objects (the AMDGPU metadata notes):
name, VGPRs, AGPRs, SGPRs, LDS bytes, scratch bytes per lane, and the waves per SIMD the VGPR count allows."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dot_hazard  # noqa: E402  (code-object extraction)

LLVM = dot_hazard.LLVM


def notes(lib_path):
    with tempfile.TemporaryDirectory() as wd:
        fat = os.path.join(wd, "fat.bin")
        subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib_path,
                               os.path.join(wd, "stripped.so")])
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(dot_hazard.BUNDLE), data)]
        out = []
        for k, s in enumerate(starts):
            part = os.path.join(wd, "b%d.bin" % k)
            with open(part, "wb") as f:
                f.write(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
            co = os.path.join(wd, "b%d.co" % k)
            subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                                   "--targets=" + dot_hazard.TARGET, "--input=" + part, "--output=" + co])
            if os.path.getsize(co):
                out.append(subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", co], text=True))
        return "\n".join(out)


def kernels(text):
    rows, cur = [], None
    for line in text.splitlines():
        line = line.strip()
        m = re.match(r"^- \.agpr_count:\s+(\d+)", line)
        if m:
            cur = {"agpr": int(m.group(1))}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key, name in ((".name:", "name"), (".vgpr_count:", "vgpr"), (".sgpr_count:", "sgpr"),
                          (".group_segment_fixed_size:", "lds"), (".private_segment_fixed_size:", "scratch"),
                          (".vgpr_spill_count:", "vspill"), (".sgpr_spill_count:", "sspill")):
            if line.startswith(key):
                v = line[len(key):].strip()
                cur[name] = v if name == "name" else int(v)
    return [r for r in rows if "name" in r and not r["name"].endswith(".kd")]


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(
        __file__))), "rna-sequence-diff-patch_amd", "libsed.so")
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    rows = kernels(notes(lib))
    filt = os.path.join(LLVM, "llvm-cxxfilt")
    names = subprocess.check_output([filt] if os.path.exists(filt) else ["c++filt"], input="\n".join(
        r["name"] for r in rows), text=True).splitlines() if rows else []
    for r, nm in zip(rows, names):
        if pat not in nm:
            continue
        v = r.get("vgpr", 0) + r.get("agpr", 0)
        waves = min(8, 512 // max(8, (v + 7) // 8 * 8)) if v else 8
        print("%-90s vgpr %3d agpr %3d sgpr %3d lds %6d scratch %4d spill v%d s%d waves/SIMD %d" % (
            nm[:90], r.get("vgpr", 0), r.get("agpr", 0), r.get("sgpr", 0), r.get("lds", 0), r.get("scratch", 0),
            r.get("vspill", 0), r.get("sspill", 0), waves))

#!/usr/bin/env python3
"""Static check of the v_dot4 result hazard in libsed.so's gfx950 code object.

The dot-key kernels issue the VOP3P v_dot4_i32_i8 as inline asm (sed_kernels.hip: dot_add), so the compiler's
hazard recognizer cannot insert the wait states a VALU reader of its result needs: the very next instruction
reads a stale value (tools/ubench/dot_dist.hip, profiles/r03/ubench_dot_dist.txt).  Correctness rests on the
asm ordering (volatile dots issued SED_DOT_AHEAD / 4 rows ahead, dot_fence next to each reader).  This check
makes that a build-time property: it extracts the gfx950 code object from libsed.so (llvm-objcopy +
clang-offload-bundler), disassembles it, and for every v_dot4_i32_i8 walks the straight-line code after it,
counting wait states the way LLVM's GCNHazardRecognizer does (every instruction 1, s_nop N = N + 1), until the
destination VGPR is read (a violation below `need` wait states), overwritten, or `need` wait states have passed.
A branch or the end of the program before that counts as a violation too (the target could read it at once).

    python tools/dot_hazard.py [libsed.so]     -> prints the summary, exit 1 on a violation
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
NEED = 3  # wait states: LLVM's DotWriteDifferentVALURead (gfx940 family); the microbenchmark shows 0 is stale
BUNDLE = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"

_LOADS = ("global_load", "buffer_load", "flat_load", "scratch_load", "ds_read", "ds_load")
_NODEST = ("global_store", "buffer_store", "flat_store", "scratch_store", "ds_write", "ds_store", "global_atomic",
           "buffer_atomic", "flat_atomic", "ds_add", "ds_or", "ds_and", "ds_max", "ds_min", "exp")
_ENDS = ("s_branch", "s_cbranch", "s_setpc", "s_swappc", "s_endpgm", "s_trap")


def _vgprs(op):
    """The VGPR numbers an operand names (v7, v[4:7])."""
    op = op.strip()
    m = re.fullmatch(r"v(\d+)", op)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def disassemble(lib_path, workdir):
    """gfx950 code objects of every offload bundle in lib_path's .hip_fatbin -> disassembly text."""
    fat = os.path.join(workdir, "fat.bin")
    subprocess.check_call([os.path.join(LLVM, "llvm-objcopy"), "--dump-section", ".hip_fatbin=" + fat, lib_path,
                           os.path.join(workdir, "stripped.so")])
    data = open(fat, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(BUNDLE), data)]
    texts = []
    for k, s in enumerate(starts):
        part = os.path.join(workdir, "b%d.bin" % k)
        with open(part, "wb") as f:
            f.write(data[s:starts[k + 1] if k + 1 < len(starts) else len(data)])
        co = os.path.join(workdir, "b%d.co" % k)
        subprocess.check_call([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                               "--targets=" + TARGET, "--input=" + part, "--output=" + co])
        if os.path.getsize(co) == 0:
            continue
        texts.append(subprocess.check_output([os.path.join(LLVM, "llvm-objdump"), "-d", co], text=True))
    return texts


def parse(text):
    """[(function, mnemonic, operands)] in program order."""
    out, fn = [], None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            fn = m.group(1)
            continue
        if not line.startswith("\t"):
            continue
        ins = line.split("//")[0].strip()
        if not ins:
            continue
        parts = ins.split(None, 1)
        ops = [o for o in re.split(r",\s*", parts[1])] if len(parts) > 1 else []
        out.append((fn, parts[0], ops))
    return out


def check(lib_path, need=NEED):
    """Returns (number of v_dot4_i32_i8, min wait states seen before a reader (None if none read early),
    violations [(function, index, dest, wait states, what)])."""
    with tempfile.TemporaryDirectory(prefix="dothaz_") as wd:
        texts = disassemble(lib_path, wd)
    return scan(texts, need)


def scan(texts, need=NEED):
    """check() over disassembly texts (llvm-objdump -d format)."""
    ndots, viol, closest = 0, [], None
    for text in texts:
        ins = parse(text)
        for k, (fn, mn, ops) in enumerate(ins):
            if mn != "v_dot4_i32_i8":
                continue
            ndots += 1
            dest = _vgprs(ops[0])
            waits = 0
            for fn2, mn2, ops2 in ins[k + 1:]:
                if waits >= need:
                    break
                if fn2 != fn or mn2.startswith(_ENDS):
                    viol.append((fn, k, ops[0], waits, "control flow leaves before %d wait states" % need))
                    break
                if mn2.startswith(_NODEST) or not (mn2.startswith("v_") or mn2.startswith(_LOADS)):
                    dst, srcs = set(), ops2
                else:
                    dst, srcs = _vgprs(ops2[0]) if ops2 else set(), ops2[1:]
                if any(_vgprs(o) & dest for o in srcs):
                    viol.append((fn, k, ops[0], waits, "%s %s" % (mn2, ", ".join(ops2))))
                    closest = waits if closest is None else min(closest, waits)
                    break
                if dst & dest and dst >= dest:
                    break  # overwritten before anyone read it
                waits += int(ops2[0], 0) + 1 if mn2 == "s_nop" else 1
    return ndots, closest, viol


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "rna-sequence-diff-patch_amd", "libsed.so")
    ndots, closest, viol = check(lib)
    print("%d v_dot4_i32_i8 in %s; %d read before %d wait states" % (ndots, os.path.basename(lib), len(viol), NEED))
    for v in viol[:20]:
        print("  %s #%d %s after %d wait states: %s" % v)
    return 1 if viol or ndots == 0 else 0


if __name__ == "__main__":
    sys.exit(main())

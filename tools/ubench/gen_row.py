"""Generate valu_row.hip: DP-row instruction schedules of the integer kernel written
as raw gfx950 asm loops (fixed registers), to measure which schedule issues fastest.
Rows: V[r] = v(0+r), mm[r] = v(16+r), tU = v(32+r), tL = v(48+r), tD = v(64+r);
ops acc v80, constants: v81 (DEL'), v82 (INS'), v83 (perm sel), tables v(84+r),
SGPRs s20 (DEL'), s21 (INS')."""
NR = 16


def row_basic(r, sg=False):
    up = (r - 1) % NR
    dl = "s20" if sg else "v81"
    il = "s21" if sg else "v82"
    return [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83",
            f"v_add_u32 v{32+r}, {dl}, v{up}",
            f"v_add_u32 v{48+r}, {il}, v{r}",
            f"v_add_u32 v{64+r}, v{64+r}, v{r}",
            f"v_min3_u32 v{16+r}, v{32+r}, v{48+r}, v{64+r}",
            f"v_alignbit_b32 v80, v{16+r}, v80, 2",
            f"v_and_b32 v{r}, -4, v{16+r}"]


def sched(name):
    L = []
    if name in ("S0", "S4"):
        for r in range(NR):
            L += row_basic(r, sg=(name == "S4"))
    elif name == "S1":
        L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83" for r in range(NR)]
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_add_u32 v{32+r}, v81, v{up}", f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{64+r}, v{64+r}, v{r}",
                  f"v_min3_u32 v{16+r}, v{32+r}, v{48+r}, v{64+r}", f"v_and_b32 v{r}, -4, v{16+r}"]
        L += [f"v_alignbit_b32 v80, v{16+r}, v80, 2" for r in range(NR)]
    elif name == "S2":
        L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83" for r in range(NR)]
        for r in range(NR):
            L += [f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{64+r}, v{64+r}, v{r}"]
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_add_u32 v{32+r}, v81, v{up}", f"v_min3_u32 v{16+r}, v{32+r}, v{48+r}, v{64+r}",
                  f"v_and_b32 v{r}, -4, v{16+r}"]
        L += [f"v_alignbit_b32 v80, v{16+r}, v80, 2" for r in range(NR)]
    elif name == "S3":
        # fast ops in pairs: (addL r, addD r) then chain; perm and alignbit of neighbouring rows between
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83",
                  f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{32+r}, v81, v{up}",
                  f"v_add_u32 v{64+r}, v{64+r}, v{r}",
                  f"v_min3_u32 v{16+r}, v{32+r}, v{48+r}, v{64+r}",
                  f"v_and_b32 v{r}, -4, v{16+r}",
                  f"v_alignbit_b32 v80, v{16+r}, v80, 2"]
    elif name == "S5":
        # only the 5 ops a distance-only kernel needs: perm, 3 add, min3
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83", f"v_add_u32 v{32+r}, v81, v{up}",
                  f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{64+r}, v{64+r}, v{r}",
                  f"v_min3_u32 v{r}, v{32+r}, v{48+r}, v{64+r}"]
    elif name == "S6":
        # distance only, perms hoisted
        L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83" for r in range(NR)]
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_add_u32 v{32+r}, v81, v{up}", f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{64+r}, v{64+r}, v{r}",
                  f"v_min3_u32 v{r}, v{32+r}, v{48+r}, v{64+r}"]
    elif name == "S7":
        # add3-free variant: alignbit replaced by a 16-bit shift-insert (v_lshl_or) -- same count, other op
        for r in range(NR):
            up = (r - 1) % NR
            L += [f"v_perm_b32 v{64+r}, v{84+r}, 6, v83", f"v_add_u32 v{32+r}, v81, v{up}",
                  f"v_add_u32 v{48+r}, v82, v{r}", f"v_add_u32 v{64+r}, v{64+r}, v{r}",
                  f"v_min3_u32 v{16+r}, v{32+r}, v{48+r}, v{64+r}", f"v_and_b32 v{r}, -4, v{16+r}",
                  f"v_and_b32 v{32+r}, 3, v{16+r}"]
    return L


NAMES = ["S0", "S1", "S2", "S3", "S4", "S5", "S6", "S7"]
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', '#define ITERS 256']
for k, nm in enumerate(NAMES):
    body = sched(nm)
    asm = "\\n".join(body)
    clob = ",".join(f'"v{i}"' for i in range(100))
    out.append(f'__global__ __launch_bounds__(256) void k{k}(uint32_t *o) {{')
    out.append('  asm volatile("s_mov_b32 s20, 0x30005\\n s_mov_b32 s21, 0x20004\\n v_mov_b32 v81, 0x30005\\n v_mov_b32 v82, 0x20004\\n v_mov_b32 v83, 0x0c040100\\n v_mov_b32 v80, 0" ::: "s20","s21","v80","v81","v82","v83");')
    out.append(f'  for (int it = 0; it < ITERS; ++it) asm volatile("{asm}" ::: {clob});')
    out.append('  uint32_t x; asm volatile("v_mov_b32 %0, v80" : "=v"(x)); if (x == 0x12345u) o[0] = x; }')
out.append('typedef void (*kfn)(uint32_t *);')
out.append('static kfn F[] = {' + ",".join(f"k{k}" for k in range(len(NAMES))) + '};')
out.append('static const int NI[] = {' + ",".join(str(len(sched(n))) for n in NAMES) + '};')
out.append('static const char *NM[] = {' + ",".join(f'"{n}"' for n in NAMES) + '};')
out.append('''int main() {
  uint32_t *d; (void)hipMalloc(&d, 4);
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  for (int wps : {4, 5}) for (int k = 0; k < (int)(sizeof(NI) / sizeof(NI[0])); ++k) {
    const int blocks = 256 * wps;
    hipLaunchKernelGGL(F[k], dim3(blocks), dim3(256), 0, 0, d); (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(F[k], dim3(blocks), dim3(256), 0, 0, d);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = 5.0 * blocks * 4.0 * ITERS * NI[k];
    const double cyc = (ms * 1e6) * 2.4 / (winstr / 1024.0);
    printf("waves/SIMD %d %s %3d instr/step  %.2f cycles/instr  %.2f cycles/row\\n", wps, NM[k], NI[k], cyc, cyc * NI[k] / 16);
  }
  return 0;
}''')
open(__file__.replace("gen_row.py", "valu_row.hip"), "w").write("\n".join(out) + "\n")

// The checkpoint traceback (sed_traceback_ck_kernel, config 4's script route) in a translation unit of its own, so it
// can be compiled with its own code-generation options (Makefile: CKTB_FLAGS).  A tile visit keeps its lane's code
// words in a uint32_t[NW] and the entry word's LDS inputs in two uint32_t[16]; by default the compiler promotes such
// arrays to single vector values of 12 / 16 registers (AMDGPUPromoteAlloca) and copies them whole at the joins between
// a visit's words (6 v_mov_b64 per word and per entry-word exit, ~60 VALU a visit against ~1320).  Built with promotion
// limited to 16-byte arrays, SROA splits them into separate registers after unrolling: no copies, same registers, no
// scratch.  The other kernels keep the default (several use more registers or scratch without the promotion).
#define SED_CKTB_TU 1
#include "sed_kernels.hip"

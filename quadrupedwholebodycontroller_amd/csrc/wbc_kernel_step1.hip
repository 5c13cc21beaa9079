// wbc_kernel_step1.hip — the stateful default step (wbc_update_solve_kernel<1>: history, hotstart),
// BASELINE configs[2]'s trot.  A translation unit of its own so that the Makefile can schedule it
// apart from the other kernels (STEP1_KFLAGS: DESIGN.md 4.24); the code is wbc_kernel.hip's, which
// WBC_STEP1_TU limits to this one kernel and its launcher.
#define WBC_STEP1_TU 1
#include "wbc_kernel.hip"

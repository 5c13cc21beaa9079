// wbc_kernel_step0.hip — the stateless default step of any mask mix (wbc_update_solve_kernel<0>:
// the four-contact stance form and the general 12-variable form in one kernel), e.g. BASELINE
// configs[3]'s rl_random batches.  A translation unit of its own so that the Makefile can schedule
// it apart from the other kernels (STEP0_KFLAGS: DESIGN.md 4.24); the code is wbc_kernel.hip's,
// which WBC_STEP0_TU limits to this one kernel and its launcher.
#define WBC_STEP0_TU 1
#include "wbc_kernel.hip"

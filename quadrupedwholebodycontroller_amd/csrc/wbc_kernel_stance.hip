// wbc_kernel_stance.hip — the stance-only default step (wbc_update_solve_kernel<0, true>): a
// stateless step whose QPs all have contact mask 15 (BASELINE configs[1], the headline), with the
// general 12-variable form compiled out.  A translation unit of its own so that the Makefile can
// schedule it apart from the mixed-form kernel (STANCE_KFLAGS: DESIGN.md 4.22); the code is
// wbc_kernel.hip's, which WBC_STANCE_TU limits to this one kernel and its launcher.
#define WBC_STANCE_TU 1
#include "wbc_kernel.hip"

// wbc_kernel_resident.hip — the resident B <= 4 control cycle (wbc_resident_kernel<0> and <1>,
// BASELINE configs[0]'s drop-in).  A translation unit of its own so that the Makefile can schedule
// it apart from the other kernels (RESIDENT_KFLAGS: DESIGN.md 4.24); the code is wbc_kernel.hip's,
// which WBC_RESIDENT_TU limits to these kernels and their launchers.
#define WBC_RESIDENT_TU 1
#include "wbc_kernel.hip"

// wbc_kernel_modes.hip — the mode loop (wbc_modes_kernel: contact-mode hypotheses with the update
// shared, BASELINE configs[4]).  A translation unit of its own so that the Makefile can schedule it
// apart from the other kernels (MODES_KFLAGS: DESIGN.md 4.24); the code is wbc_kernel.hip's, which
// WBC_MODES_TU limits to this one kernel and its launcher.
#define WBC_MODES_TU 1
#include "wbc_kernel.hip"

/* wbc_ref.h — TEST INFRASTRUCTURE ONLY: C restatement of the reference WBC path (see wbc_ref.c). */
#ifndef WBC_REF_H
#define WBC_REF_H
#include <stdint.h>

#include "wbc.h"

#ifdef __cplusplus
extern "C" {
#endif

enum { WBC_REF_OK = 0, WBC_REF_MAX_ITER = 1, WBC_REF_INFEASIBLE = 2, WBC_REF_NUMERIC = 3 };

typedef struct {
    double M[18 * 18], Cnu[18], foot_J[12 * 18], foot_pos[12], foot_vel[12], com[3], com_vel[3], RB[9];
} wbc_ref_kindyn_t;

/* per-robot state that survives between cycles (hpp:154-161) */
typedef struct {
    double old_T[18 * 18], old_Jc[12 * 18], old_Js[12 * 18], Tdot_inv[18 * 18], e_int[6];
    int contacts, first;
    int ws_n, ws_kap, cold_qp; /* working set of the last solve (hotstart, cpp:531); cold_qp: always init */
    int ws[42];
    /* QP method: 0 = the literal 42 x 70 QP (dense Goldfarb-Idnani), 1 = the engine's exact
     * 12-variable form of the same QP (its working set in ws12, row ids of that form) */
    int method, ws12_valid;
    unsigned long long ws12;
} wbc_ref_state;

typedef struct {
    double com[3], comvel[3], pose[6], vc[6], M[324], Cnu[18], Mbar_b[36], Mbar_j[144], Jbar[216], bbar[18], W[6],
        r1[12], rsw[12];
} wbc_ref_debug_t;

void wbc_ref_kindyn(const wbc_model* md, const double* pose, const double* nu, const double* qj, wbc_ref_kindyn_t* out);
void wbc_ref_state_init(wbc_ref_state* s);
int wbc_ref_step(const wbc_model* md, const wbc_params* pr, wbc_ref_state* st, const double* pose, const double* nu,
                 const double* qj, const double* ref, int contacts, int switching, double* tau, double* grf, double* x,
                 int* iters, wbc_ref_debug_t* dbg);
void wbc_ref_run_batch(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                       const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching, double* tau,
                       double* grf, double* x, int32_t* status, int32_t* iters);
/* the same with QP method `method` (wbc_ref_state::method) */
void wbc_ref_run_batch_method(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                              const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching,
                              double* tau, double* grf, double* x, int32_t* status, int32_t* iters, int method);
/* n stateful robots in one call: robot i (state st[i]) reads batch row idx[i], writes output row i */
void wbc_ref_step_states(const wbc_model* md, const wbc_params* pr, int n, wbc_ref_state* st, const int32_t* idx,
                         const double* pose, const double* nu, const double* qj, const double* ref,
                         const uint8_t* contacts, const uint8_t* switching, double* tau, double* grf, double* x,
                         int32_t* status, int32_t* iters, int threads);
int wbc_ref_gi(int n, const double* H, const double* g, int me, const double* CE, const double* ce, int mi, const double* CI,
               const double* ci, int max_iter, double* x, int* iters);

/* CPU baseline (bench.py cpu_baseline): oracle/wbc_fast.c, structure-exploiting, cold steps */
int wbc_fast_step(const wbc_model* md, const wbc_params* pr, const double* pose, const double* nu, const double* qj,
                  const double* ref, int contacts, double* tau, double* grf, int* iters);
void wbc_fast_run_batch(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                        const double* qj, const double* ref, const uint8_t* contacts, double* tau, double* grf,
                        int32_t* status, int32_t* iters, int threads);
void wbc_ref_run_batch_omp(const wbc_model* md, const wbc_params* pr, int B, const double* pose, const double* nu,
                           const double* qj, const double* ref, const uint8_t* contacts, const uint8_t* switching,
                           double* tau, double* grf, int32_t* status, int32_t* iters, int threads);

#ifdef __cplusplus
}
#endif
#endif

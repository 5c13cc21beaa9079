// wbc_layout.h — device-side record layouts shared by the HIP kernel and the host engine.
#ifndef WBC_LAYOUT_H
#define WBC_LAYOUT_H

#include "wbc.h"

namespace wbc {

// Per-robot history that survives between control cycles (stateful mode).  Compact form of
// the reference's finite-difference state (hpp:154-161): T_old (top rows only vary:
// [Ad^-1(r_old), Mbar_b^-1 A_j]), Jbar_old (com part [I, -S(p_f - c)] from d_old, joint part),
// Tdot_inv (top 6 rows), integralError_, the contacts of Jbar_old, a valid flag
// (0 right after setInitialState: T_old = I, J_old = 0, Tdot_inv = 0, cpp:84-104), and the
// working set of the previous QP (qpOASES SQProblem::hotstart, cpp:531).
enum HistOff {
    H_ROLD = 0,     // r_old = c - p_B of the previous cycle (3)
    H_MAOLD = 3,    // Mbar_b^-1 A_j of the previous cycle, 6x12 row-major (72)
    H_DOLD = 75,    // p_f - c, previous cycle (12)
    H_JBJOLD = 87,  // joint part of Jbar_feet, previous cycle, 12x12 (144)
    H_TDINV = 231,  // Tdot_inv top 6 rows, 6x18 row-major (108)
    H_EINT = 339,   // integralError_ (6)
    H_KOLD = 345,   // contact bitmask of the previous cycle (as double)
    H_VALID = 346,  // 0 after reset
    H_WSLO = 347,   // active inequality set of the previous solve, lanes 0..31 (bitmask as double)
    H_WSHI = 348,   //   lanes 32..63
    H_WSKAP = 349,  // contact mask that active set belongs to (hotstart only for the same mask)
    HIST_LEN = 350
};

// Assembled per-robot problem: written by the update phase, read by the solve phase
// (the HBM workspace between wbc_update and wbc_solve; kept in LDS by the fused step).
struct Prob {
    double m, inv_m;
    double Ic[9];
    double Icinv[9];
    double d[12];     // foot position minus CoM, LH, LF, RF, RH
    double Jbj[144];  // joint columns of Jbar_feet = J_feet T^-1, [row 0..11][joint 0..11]
    double Mbj[144];  // centroidMassMatrixJoints_
    double bbj[12];   // centroidGeneralizedBias_(6:18)
    double r1[12];    // R1 bound: -Jc_dot_com v_c - Jc_dot_j qdot (cpp:504)
    double rsw[12];   // R4/R5 bound: cmd - Js_dot_com v_c - Js_dot_j qdot (cpp:507,515)
    double W[6];      // computeDesiredWrench (cpp:426-445)
    double kappa;     // contact bitmask
    double flags;     // 1: non-finite input / intermediate, 2: slot Hessian not positive definite
};
static_assert(sizeof(Prob) % 16 == 0, "Prob must keep 16-byte alignment");
constexpr int PROB_LEN = sizeof(Prob) / sizeof(double);

// Slot factorisation formed at the end of the update kernel (presolve in wbc_kernel.hip), stored
// after the problem in the work row and read by the solve kernel from HBM / L2.
//
// Four-contact stance (kappa = 15) is solved in a smaller space: the 12 stance equalities
// (R1, cpp:494,504) Jbar_c,j qdd + G f = e are solved for qdd = q0 - P f in the update kernel,
// which leaves a 12-variable QP in the contact forces with Hessian H_f = P^T P + H_s and gradient
// g_s - P^T q0, and only inequality rows (16 friction faces, 24 torque rows tau = t0 - Nt f).
// Then Mi / xs hold the factor of H_f and the unconstrained f0, and the stance fields below are
// filled (wbc_kernel.hip stance_reduce).
struct Presolve {
    double Mi[78];    // M = L^-1 of the slot Hessian H_s = L L^T (H_f for stance), lower triangle row-major
    double xs[12];    // slot part of the unconstrained optimum x0 = -H^-1 g (f0 for stance)
    double presolved; // 1: Mi / xs hold the slot factorisation for this kappa; 0: the solve forms it
    double stance;    // 1: the stance elimination below is valid (Mi / xs then belong to H_f)
    double q0[12];    // stance: qdd = q0 - P f
    double t0[12];    //         tau = t0 - Nt f  (t0 = bbar_j + Mbar_j q0)
    double nsel[12];  //         |row|^2 of torque row j in the reference's 42-variable space
    double Nt[144];   //         Nt = Mbar_j P + Jbar_c,j^T, [joint j][force c]
    double Y[72];     //         P = Y B^T (rank 6): qdd = q0 - Y [F / m; I_c^-1 sum d_l x f_l], [joint][6]
};
static_assert(sizeof(Presolve) % 16 == 0, "Presolve must keep 16-byte alignment");
constexpr int PRE_LEN = sizeof(Presolve) / sizeof(double);
constexpr int WORK_LEN = PROB_LEN + PRE_LEN;  // work row: [Prob | Presolve]

// The step kernel's LDS image of the model and the friction-normal table, built once on the host
// (wbc_create) and copied into LDS by each workgroup as one contiguous block: each link record is
// padded to 29 doubles (at the API's 28, 224 B, lanes j and j + 8 of a segment read the same LDS
// banks for every field of their links), and the table holds face rr's normal for leg l as the 12
// doubles from FRIC_ROW(4 l + rr) (four 21-double bands: zeros, the face's three entries, zeros).
struct LdsLink {
    double R[9], p[3], axis[3], mass, com[3], inertia[9], pad_;
};
static_assert(sizeof(LdsLink) == sizeof(wbc_link) + sizeof(double), "LdsLink mirrors wbc_link");
struct LdsModel {
    double base_mass, base_com[3], base_inertia[9];
    LdsLink link[WBC_NUM_LEGS][3];
    double foot[WBC_NUM_LEGS][3];
    double total_mass;
};
constexpr int FRIC_LEN = 4 * 21;
#define FRIC_ROW(p) (((p) & 3) * 21 + 9 - 3 * ((p) >> 2))
struct LdsImage {
    LdsModel model;
    double fric[FRIC_LEN];
};
constexpr int LIMG_LEN = sizeof(LdsImage) / sizeof(double);
inline void build_lds_image(const wbc_model& m, double friction, LdsImage& o) {
    o.model.base_mass = m.base_mass;
    for (int i = 0; i < 3; ++i) o.model.base_com[i] = m.base_com[i];
    for (int i = 0; i < 9; ++i) o.model.base_inertia[i] = m.base_inertia[i];
    for (int l = 0; l < WBC_NUM_LEGS; ++l)
        for (int k = 0; k < 3; ++k) {
            const wbc_link& s = m.link[l][k];
            LdsLink& d = o.model.link[l][k];
            for (int i = 0; i < 9; ++i) { d.R[i] = s.R[i]; d.inertia[i] = s.inertia[i]; }
            for (int i = 0; i < 3; ++i) { d.p[i] = s.p[i]; d.axis[i] = s.axis[i]; d.com[i] = s.com[i]; }
            d.mass = s.mass;
            d.pad_ = 0.0;
        }
    for (int l = 0; l < WBC_NUM_LEGS; ++l)
        for (int i = 0; i < 3; ++i) o.model.foot[l][i] = m.foot[l][i];
    o.model.total_mass = m.total_mass;
    // face rr of a friction pyramid: [-1, 0, mu], [1, 0, mu], [0, -1, mu], [0, 1, mu] (force space)
    for (int e = 0; e < FRIC_LEN; ++e) {
        const int rr = e / 21, k = e % 21 - 9;
        const double fv = (k == 0) ? ((rr == 0) ? -1.0 : (rr == 1 ? 1.0 : 0.0))
                        : (k == 1) ? ((rr == 2) ? -1.0 : (rr == 3 ? 1.0 : 0.0)) : friction;
        o.fric[e] = (k >= 0 && k < 3) ? fv : 0.0;
    }
}

// The resident control cycle's mailbox (wbc_cycle with WBC_RESIDENT; pinned, coherent host memory):
// the host raises cmd (a sequence number, or WBC_RESIDENT_STOP), the resident wave answers with
// done = cmd once the cycle's outputs are visible, and sets exited = 1 when it ends (on
// WBC_RESIDENT_STOP or after its idle limit), so the host can tell a wave that ended by itself from
// one that is late.  cmd and the wave's words sit on separate 64-byte lines.
constexpr unsigned long long WBC_RESIDENT_STOP = ~0ull;
struct ResidentBox {
    unsigned long long cmd;
    unsigned long long pad0[7];
    unsigned long long done;
    unsigned long long exited;
    unsigned long long pad1[6];
};

// Kernel arguments (one struct, passed by value).
struct KernelArgs {
    const wbc_model* model;
    const wbc_params* params;
    const double* limg;  // LdsImage (model in the LDS layout + friction table), LIMG_LEN doubles
    const double* base_pose;
    const double* nu;
    const double* qj;
    const double* ref;
    const uint8_t* contacts;
    const uint8_t* switching;
    double* hist;       // [B][HIST_LEN]
    double* work;       // [B][WORK_LEN] (split update/solve): Prob, Presolve
    double* tau;
    double* grf;
    double* x;
    int32_t* status;
    int32_t* iters;
    double* dbg;        // [B][WBC_DBG_LEN]
    int32_t batch;
    int32_t stateful;   // read / write history
    int32_t debug;      // write debug records
    int32_t cold;       // stateful, but no QP hotstart (WBC_COLD)
    int32_t modes;      // contact-mode hypotheses per state (wbc_step_modes); 0 = one QP per input row
    const uint8_t* mode_masks;  // [modes]: contact mask of hypothesis k
    // Four-contact stance elimination (Presolve::stance) for this step's mask-15 QPs: the engine
    // turns it on when every QP of the step has mask 15 (then the stance solve kernel runs
    // instead of the general one).  QPs whose elimination did not happen (a near-singular leg)
    // are listed for the fallback solve: fb[parity] counts them, fb[2 ..] lists them (at most
    // fb_cap entries); the update kernel clears fb[parity ^ 1] for the next elimination update.
    // (The default step, wbc_update_solve_kernel, solves its fallbacks in place and uses neither.)
    int32_t elim;
    int32_t parity;
    int32_t* fb;
    int32_t fb_cap;
    // The default step's wave map (wbc_update_solve_kernel): entry e = qmap[4 w + seg] of segment
    // seg of workgroup w is (qp << 4 | mask) for a QP it solves (e >= 0), ~(qp << 4 | mask) for a
    // padding segment that recomputes QP qp without writing anything, QMAP_EMPTY when the whole
    // workgroup has nothing to do.  The mask travels in the entry, so the step reads one word before
    // the QP's inputs (not the word and then contacts[qp]).  The engine groups the QPs by contact
    // mask (qmap_build below, or wbc_qmap_kernel for device-bound masks), so the four segments of a
    // wave share one mask.  nullptr: QP 4 w + seg (every mask in the step is equal).
    // Under mode hypotheses the map is arithmetic (workgroup g K + k: states 4 g .. 4 g + 3 under
    // mask modes[k]) and qmap is unused.  nwaves: the step kernel's grid.
    const int32_t* qmap;
    int32_t nwaves;
    // Mode hypotheses with the state's update shared (wbc_modes_kernel): each wave holds four
    // states and a chunk of mloop hypotheses, solved one after another after one update; chunk c
    // runs hypotheses mode_order[c mloop .. c mloop + mloop - 1].  mloop = 0: one hypothesis per
    // segment (wbc_update_solve_kernel's arithmetic map).
    int32_t mloop;
    uint8_t mode_order[16];
    // the parameters by value: read from the kernel-argument segment (scalar loads of memory the
    // compiler knows is constant), not through `params`, whose global loads it must repeat after
    // every global store and wait for in turn
    wbc_params pv;
};

// ---------------------------------------------------------------------------------------
// Wave map of the default step: QPs grouped by contact mask, four to a wave (KernelArgs::qmap)
// ---------------------------------------------------------------------------------------
constexpr int32_t QMAP_EMPTY = (int32_t)0x80000000;
constexpr int QMAP_MAX_BATCH = (1 << 27) - 1;  // qp << 4 fits 31 bits
#ifdef __HIPCC__
#define WBC_HD __host__ __device__
#else
#define WBC_HD
#endif
WBC_HD inline int32_t qmap_entry(int qp, int mask) { return (int32_t)((qp << 4) | (mask & 15)); }
constexpr int QMAP_SEG = 4;  // QPs per wave (UPD_RPW of the kernel)
// Layout.  The general 12-variable form runs one instruction stream for every contact mask, so
// waves may mix masks at no cost; a stateless mask-15 QP takes the four-contact stance form, a
// different stream, so it never shares a wave with another mask.  Within that rule the map groups
// QPs of one mask (a wave runs its four QPs' largest pass count: QPs of one mask need similar counts)
// and uses at most one wave more than ceil(B / 4), so a batch that fills whole rounds of the chip
// does not spill a partial round:
//   region 0: the r15 = cnt[15] % 4 mask-15 QPs left over from whole waves, padded to one wave
//             (only when r15 > 0);
//   region 1: the other masks' leftovers (< 4 each, at most 45) in mixed waves, the last padded;
//   region 2: whole waves of one mask, buckets in QMAP_ORDER.
// Leftovers are a bucket's last QPs in batch order; a bucket's other QPs keep their batch order;
// padding segments recompute the bucket's first QP.  Buckets start with mask 15 (the most active-set
// passes on the bench batches: 8.9 per QP against 6.7 for three stance legs and 0.3 for none), then
// three stance legs, two, one, none: when a step has more waves than the chip holds at once, the
// hardware starts them in map order, so the costliest start first and the cheapest fill the end.
#ifndef WBC_QMAP_NATURAL_ORDER
constexpr uint8_t QMAP_ORDER[16] = {15, 7, 11, 13, 14, 3, 5, 6, 9, 10, 12, 1, 2, 4, 8, 0};
#else  // (A/B builds only)
constexpr uint8_t QMAP_ORDER[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
#endif
// capacity of the map for B QPs (entries): ceil(B / 4) + 1 waves
WBC_HD inline int qmap_capacity(int B) { return QMAP_SEG * ((B + QMAP_SEG - 1) / QMAP_SEG + 1); }
// The device builder's scratch after the map (wbc_qmap_count / _plan / _scatter): per block of
// QMAP_BLOCK QPs its 16 mask counts (then their exclusive prefixes over the blocks) and 16 first
// indices, then the plan
constexpr int QMAP_BLOCK = 1024;
WBC_HD inline int qmap_blocks(int B) { return (B + QMAP_BLOCK - 1) / QMAP_BLOCK; }
WBC_HD inline int qmap_scratch(int B) { return 32 * qmap_blocks(B) + 64; }
struct QmapPlan {
    int base1, base2, waves;  // region 1 / 2 starts (entries), total waves
    int full[16];             // QPs of bucket m in whole waves (4 * floor(cnt / 4))
    int off1[16], off2[16];   // bucket m's leftovers in region 1, its whole waves in region 2
    int pad0, pad1, end1;     // padding: region 0 [pad0, 4), region 1 [pad1, end1)
    int32_t v0, v1;           // their entries
};
// the plan from the bucket counts and each bucket's first QP (host and device builders alike)
WBC_HD inline void qmap_plan(const int* cnt, const int* first, QmapPlan& p) {
    const int r15 = cnt[15] % QMAP_SEG;
    p.base1 = r15 ? QMAP_SEG : 0;
    p.pad0 = r15;
    p.v0 = ~qmap_entry(first[15] < 0 ? 0 : first[15], 15);
    int o1 = 0, o2 = 0, last = -1;
#pragma unroll  // (device builder: bucket m a constant, the plan's fields registers)
    for (int k = 0; k < 16; ++k) {
        const int m = QMAP_ORDER[k];
        p.full[m] = cnt[m] - cnt[m] % QMAP_SEG;
        p.off2[m] = o2;
        o2 += p.full[m];
        p.off1[m] = o1;
        if (m != 15 && cnt[m] % QMAP_SEG) {
            o1 += cnt[m] % QMAP_SEG;
            last = m;
        }
    }
    p.pad1 = p.base1 + o1;
    p.end1 = p.base1 + QMAP_SEG * ((o1 + QMAP_SEG - 1) / QMAP_SEG);
    p.v1 = last < 0 ? 0 : ~qmap_entry(first[last], last);
    p.base2 = p.end1;
    p.waves = (p.base2 + o2) / QMAP_SEG;
}
// entry position of the j-th QP (batch order) of bucket m
WBC_HD inline int qmap_pos(const QmapPlan& p, int m, int j) {
    if (j < p.full[m]) return p.base2 + p.off2[m] + j;
    const int i = j - p.full[m];
    return (m == 15) ? i : p.base1 + p.off1[m] + i;
}
// Host form: returns the number of waves; 0 (map unused) when every mask is equal.
inline int qmap_build(const uint8_t* masks, int B, int32_t* map) {
    int cnt[16] = {0}, first[16];
    for (int m = 0; m < 16; ++m) first[m] = -1;
    for (int b = 0; b < B; ++b) {
        const int m = masks[b] & 15;
        if (first[m] < 0) first[m] = b;
        ++cnt[m];
    }
    for (int m = 0; m < 16; ++m)
        if (cnt[m] == B) return 0;
    QmapPlan p;
    qmap_plan(cnt, first, p);
    int j[16] = {0};
    for (int b = 0; b < B; ++b) {
        const int m = masks[b] & 15;
        map[qmap_pos(p, m, j[m]++)] = qmap_entry(b, m);
    }
    for (int e = p.pad0; p.base1 && e < QMAP_SEG; ++e) map[e] = p.v0;
    for (int e = p.pad1; e < p.end1; ++e) map[e] = p.v1;
    return p.waves;
}



// Mode hypotheses per wave (KernelArgs::mloop, wbc_modes_kernel) for K hypotheses over `groups`
// four-state groups on a device with `simds` SIMDs: the largest M dividing K that still gives
// every SIMD a wave (groups K / M >= simds), 1 (one hypothesis per segment) when even that leaves
// SIMDs idle; m_override (a divisor of K; 0 = none) replaces it.  order[c M .. c M + M - 1] are
// chunk c's hypotheses: longest first, each to the chunk with the least estimated work so far
// (LPT), the estimate a reduction and solve of 30 units plus 3 per expected working-set pass
// (0.3, 2.3, 4.5, 6.7, 8.9 passes for 0 .. 4 stance legs).  Returns M.
inline int mode_loop_plan(const uint8_t* modes, int K, int64_t groups, int64_t simds, int m_override,
                          uint8_t* order) {
    int M = 1;
    for (int m = K; m > 1; --m)
        if (K % m == 0 && groups * (K / m) >= simds) { M = m; break; }
    if (m_override >= 1 && m_override <= K && K % m_override == 0) M = m_override;
    static const double passes[5] = {0.3, 2.3, 4.5, 6.7, 8.9};
    const int C = K / M;
    int idx[16], fill[16] = {};
    double load[16] = {};
    for (int k = 0; k < K; ++k) idx[k] = k;
    auto cost = [&](int k) { return 30.0 + 3.0 * passes[__builtin_popcount(modes[k] & 15u)]; };
    for (int a = 1; a < K; ++a)  // stable insertion sort, costliest first
        for (int b = a; b > 0 && cost(idx[b]) > cost(idx[b - 1]); --b) {
            const int t = idx[b]; idx[b] = idx[b - 1]; idx[b - 1] = t;
        }
    uint8_t chunk[16][16];
    for (int t = 0; t < K; ++t) {
        int best = -1;
        for (int c = 0; c < C; ++c)
            if (fill[c] < M && (best < 0 || load[c] < load[best])) best = c;
        chunk[best][fill[best]++] = (uint8_t)idx[t];
        load[best] += cost(idx[t]);
    }
    for (int c = 0; c < C; ++c)
        for (int i = 0; i < M; ++i) order[c * M + i] = chunk[c][i];
    return M;
}
}  // namespace wbc
#endif

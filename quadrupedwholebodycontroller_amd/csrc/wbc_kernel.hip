// wbc_kernel.hip — batched whole-body-control step for gfx950 (MI355X), fp64.
//
// (Three translation units include this file to build one kernel each under its own schedule:
// wbc_kernel_stance.hip the stance-only default step, wbc_update_solve_kernel<0, true> (DESIGN.md
// 4.22); wbc_kernel_step0.hip the stateless default step, wbc_update_solve_kernel<0>; and
// wbc_kernel_modes.hip the mode loop, wbc_modes_kernel (4.24).  This file's own unit builds the rest.)
// The default step (wbc_update_solve_kernel, the mode loop wbc_modes_kernel and the resident B <= 4
// cycle wbc_resident_kernel) runs four robots per 64-lane wavefront, a 16-lane segment each, one
// workgroup = one wave, one wave per SIMD (≈ 400 registers, 40 KB of LDS), and solves each robot's
// QP in its exact 12-variable reduction (DESIGN.md 4.8, 4.4/4.6 for the stateless stance form).
// The split and fused forms (wbc_update_kernel + wbc_solve_kernel, wbc_step_kernel) run the
// 24-variable general QP described below one robot per wave at WBC_WAVES_PER_SIMD = 2 (<= 256
// VGPRs, spill-free, 20.3 KB of LDS); their 4-wave build spills and is slower
// (profiles/r01/variants_*.log).
//
//   update (≙ WholeBodyController::updateState, src/whole_body_controller.cpp:256-294)
//     stage A  lanes 0..11 = joints: sin/cos; lanes 0..3 = legs: forward kinematics chain
//              (3 links), joint-origin velocity and bias acceleration (iDynTree
//              KinDynComputations in MIXED representation, cpp:258-266,327-379,544-551)
//     stage B  lanes 0..12 = rigid bodies: com, world inertia, velocity, Newton-Euler bias force
//     stage C  lanes 0..11 = joints: centroidal momentum matrix columns, leg blocks of M, joint bias;
//              closed forms of T^-1, Mbar = T^-T M T^-1, Jbar = J T^-1, bbar (cpp:268-293) instead
//              of the reference's seven dense 18x18 LU inverses; finite differences against the
//              HBM history (cpp:384-402); desired wrench and swing commands (cpp:426-464).
//   solve (≙ solveQP + computeJointTorques, cpp:466-577), split and fused forms
//     The 42-variable / 70-row QP is reduced exactly to 24 variables and solved
//     with the Goldfarb-Idnani dual active-set method: lane p owns constraint p and its column
//     C[:,p] = J^T n_p (J = L^-T Q), so every product the method needs is lane-local; the chosen
//     column is broadcast with v_readlane; R^-1 (packed) lives in LDS; Householder reflections
//     add constraints; a drop re-adds the remaining active set.  The primal solution is recovered
//     from the final multipliers (y = x0 + H^-1 N_A u) with an LDS transpose-sum.
//
// 64-lane waves are assumed throughout (gfx950).
#include <hip/hip_runtime.h>

#include "wbc.h"
#include "wbc_layout.h"

#ifndef WBC_WAVES_PER_SIMD
#define WBC_WAVES_PER_SIMD 2
#endif

namespace wbc {

constexpr int NQ = 24;                  // reduced QP variables
constexpr int C0_LANES = 52;            // max constraints: 7 ns + 24 + 6 (4 - ns) <= 52

// Frames and bodies are read one per lane (lane = body): 25 doubles (50 dwords) apart puts 13
// consecutive lanes in distinct LDS banks, where 24 doubles (48 dwords) put every 4th lane in the
// same bank (PMC: ~2 300 bank-conflict cycles per update wave).
struct Frame {  // world frame of a body after stage A
    double R[9], o[3], w[3], al[3], ao[3], vo[3], pad;
};
struct Body {  // body quantities after stage B
    double c[3], I[9], F[3], N[3], pad[7];
};
static_assert(sizeof(Frame) == sizeof(Body), "frame / body union");

struct UpdScratch {
    double in[92];          // pose 7 | nu 18 | q 12 | ref 54
    double sc[12][2];       // sin, cos of q_j
    union {
        Frame fr[13];
        Body bd[13];
        struct {            // slot factorisation at the end of the update (presolve)
            double L[12][13];
            double ild[12];
            double xs[12];
        } ps;
        struct {            // four-contact stance elimination (stance_reduce), before the factorisation
            double W[12][6];    // rows of Jblk^-1 E
            double w[12];       // Jblk^-1 e
            // 6-row arrays padded to 9 columns (72 B): at 8 (64 B) rows r and r + 4, which lanes r
            // and r + 4 access together, share LDS banks
            double S[6][9];     // [I - K W | K w], then the rows of H^ = I + Mb^-2 + Mb^-1 Q Mb^-1
            double Si[6][9];    // S^-1 (rows)
            double Y[12][6];    // W S^-1
            double q0[12];
            double Q[6][9];     // [Y^T Y | Y^T q0]
        } sr;
    };
    double ja[12][3];       // joint axis (world)
    double jo[12][3];       // joint origin (world)
    double pf[4][3];
    double vf[4][3];
    double Jf[4][9];        // foot Jacobian joint columns of its leg: [row r][k]
    double A[12][6];        // centroidal momentum matrix joint columns (lin 3, ang about c 3)
    double KA[12][3];       // I_c^-1 A_ang
    double Mjj[12][3];      // leg block rows of M
    double hj[12];          // joint bias (C nu)_j
    double cen[40];         // uniform scratch (CEN_*)
    double yv[6];           // Tdot_inv nu exchange (segmented update kernel)
};

// The update kernel's inline solve (solve16) works in the robot's own UpdScratch and Prob, in
// arrays the update no longer reads once the reduction has formed the torque map: the factor
// (J mirror) and x0 stay where the factorisation leaves them (ps.L, ps.xs), the rest goes here.
// Two placements: the four-contact stance form (stance_reduce, stateless all-stance waves) and
// the general form of every contact mask (reduce_general, §4.8), whose torque map overwrites the
// problem's Jbar joint block and which keeps the maps back to the 42 variables for the outputs.
// friction normals, compact (LdsImage::fric, wbc_layout.h): face rr's row for leg l is 12 doubles
// from FRIC_ROW(4 l + rr) of a 21-double band per face, [9 zeros | -D[rr] (3) | 9 zeros]: the row
// starting 9 - 3 l doubles into the band has -D[rr] at 3 l .. 3 l + 2 and zeros elsewhere (84
// doubles instead of 16 x 12)
// row stride of the J mirror (over ps.L / ps.ild of the update scratch): 14 doubles (112 B) keeps
// rows 16-byte aligned for the b128 stores and puts no two of the 12 row lanes on the same banks
// (at 12 doubles, 96 B, rows r and r + 8 share them); 12 x 14 ends before ps.xs
constexpr int JMS = 14;
static_assert(11 * JMS + 12 <= (int)((offsetof(UpdScratch, ps) + offsetof(decltype(UpdScratch::ps), xs) -
                                      offsetof(UpdScratch, ps)) / 8), "J mirror ends before ps.xs");
struct St16 {
    double* Nt;    // [12][12] torque map rows: stance ja .. A (204 doubles); general P.Jbj
    double* Y;     // [12][6]  stance in; general sr.Y
    double* t0;    // [12]     stance in + 72; general pf
    double* q0;    // [12]     stance sc; general sr.q0
    double* nsel;  // [12]     sc + 12: |reference torque row|^2
    double* col;   // [16]     column exchange: d (12), slack, Givens pair (KA)
    double* f;     // [12]     primal (stance: cen; general: KA + 16)
    // general form only
    double* Bt;    // [12][6]  phi = B z: column j of B (ja, jo)
    double* Vt;    // [12][6]  leg row i: its coupling v_i to phi (in)
    double* rho0;  // [12]     leg row i at z = 0 (in + 72)
    double* J0;    // [12][12] copy of the initial J rows for a rejected hotstart (P.Mbj)
    const double* fric;  // friction normals, the workgroup's shared table (FRIC_ROW: row of face p)
    __device__ St16(UpdScratch& s, const double* fr)
        : Nt(&s.ja[0][0]), Y(&s.in[0]), t0(&s.in[72]), q0(&s.sc[0][0]), nsel(&s.sc[6][0]), col(&s.KA[0][0]),
          f(&s.cen[0]), Bt(nullptr), Vt(nullptr), rho0(nullptr), J0(nullptr), fric(fr) {}
    __device__ St16(UpdScratch& s, Prob& P, const double* fr)
        : Nt(&P.Jbj[0]), Y(&s.sr.Y[0][0]), t0(&s.pf[0][0]), q0(&s.sr.q0[0]), nsel(&s.sc[6][0]), col(&s.KA[0][0]),
          f(&s.KA[0][0] + 16), Bt(&s.ja[0][0]), Vt(&s.in[0]), rho0(&s.in[72]), J0(&P.Mbj[0]), fric(fr) {}
};
// row stride of Nt in the stance form: 13 doubles (26 dwords) puts the 12 row lanes of a segment on
// distinct LDS banks (at 12, rows r, r + 4 and r + 8 share them); the general form's Nt lies over
// P.Jbj (144 doubles, P.Mbj after it holds J0's copy) and keeps 12
constexpr int NTS_ST = 13;
static_assert(offsetof(UpdScratch, A) + sizeof(UpdScratch::A) - offsetof(UpdScratch, ja) >=
              (11 * NTS_ST + 12) * sizeof(double), "St16 Nt");
static_assert(offsetof(UpdScratch, jo) == offsetof(UpdScratch, ja) + sizeof(UpdScratch::ja), "St16 Bt");
static_assert(offsetof(UpdScratch, vf) == offsetof(UpdScratch, pf) + sizeof(UpdScratch::pf), "St16 t0");
static_assert(sizeof(UpdScratch::KA) >= 28 * sizeof(double), "St16 col / f");

struct QpScratch {
    static constexpr int N = NQ;
    double L[12][13];       // Cholesky factor of the slot Hessian (row-major, lower); then M = L^-1
    __device__ double (&Mi())[12][12] { return *reinterpret_cast<double(*)[12][12]>(&L[0][0]); }
    double xs[12];          // slot part of x0 = -H^-1 g
    double ild[12];         // 1 / L_kk
    union {
        double G[12][12];   // setup -> constraint normals: slot coupling Jc_com Mbar_b^-1 Jc_com^T
        double Rm[12][12];  // equality block: Rm[i][k] = R[k][i]
        double ucon[64];    // after the active-set loop: the primal y (24)
    };
    double colbuf[NQ];      // column broadcast (equality block)
    // initial constraint columns C0[:, p] = J0^T n_p (J0 = blkdiag(I, L^-T)), element k of lane p
    // at c0[k / 2][p].{x, y}: read back on a drop (no rebuild of the normals) and used by the
    // primal recovery (H^-1 n = J0 C0[:, p])
    double2 c0[NQ / 2][C0_LANES];
    // R^-1 (upper triangular, zero elsewhere): element (i, j) at Rv[j / 2][i].{x, y}[j % 2], so
    // lane i reads its row as 12 conflict-free ds_read_b128 and R^-1 d needs no masking
    double2 Rv[NQ / 2][NQ];
};

// Scratch of the four-contact stance solve (12 force variables, 40 inequality rows; wbc_layout.h)
struct StanceScratch {
    static constexpr int N = 12;
    static constexpr int MC = 40;  // 16 friction faces + 24 torque rows
    double M_[12][12];      // M = L^-1 of H_f (lower)
    __device__ double (&Mi())[12][12] { return M_; }
    double xs[12];          // f0 = -H_f^-1 g_f
    double colbuf[16];      // hotstart slot -> constraint exchange
    double ucon[24];        // after the loop: f (0..11), qdd (12..23)
    double2 c0[N / 2][MC];  // initial columns C0[:, p] = M n_p
    double2 Rv[N / 2][N];   // R^-1, as in QpScratch
};

struct Lds {
    Prob prob;
    union {
        UpdScratch u;
        QpScratch q;
    };
};

enum CenOff { CEN_C = 0, CEN_CD = 3, CEN_R = 6, CEN_HB = 9, CEN_POSE = 27, CEN_VC = 33 };

// ---------------------------------------------------------------------------------------
// wave helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x; }
__device__ __forceinline__ void wsync() { __syncthreads(); }  // one wave per workgroup
// Ordering point for lane-to-lane exchange through LDS inside the (single-wave) workgroup: LDS
// instructions of one wave execute in issue order, so only the compiler must not move LDS
// accesses across this point; a wavefront-scope fence is exactly that (no s_waitcnt, unlike
// __syncthreads, which also drains every outstanding global store).
__device__ __forceinline__ void lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

__device__ __forceinline__ double bcast(double v, int lane) {
    int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int bcast_i(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }
// Broadcast into VGPRs through the LDS crossbar (ds_bpermute; no LDS memory): the result is not
// known to be uniform, so it stays out of the SGPR file (readlane results are SGPRs, and a
// 24-vector of them overflows it into spill code)
__device__ __forceinline__ double vbcast(double v, int lane) {
    const int addr = lane << 2;
    const int lo = __builtin_amdgcn_ds_bpermute(addr, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(addr, __double2hiint(v));
    return __hiloint2double(hi, lo);
}

// DPP moves whose pattern reads a valid lane for every lane (quad_perm, row_ror, row_mirror,
// row_newbcast): v_mov_b32_dpp without an "old" operand (update_dpp(0, ...) makes the compiler
// zero the destination first, one extra move per 32-bit half)
// row_newbcast (0x150 + lane) is the one pattern gfx950 allows on 64-bit DPP: one v_mov_b64_dpp
// instead of two v_mov_b32_dpp
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
    if constexpr (CTRL >= 0x150 && CTRL <= 0x15F) {
        const long long b = __builtin_bit_cast(long long, v);
        const long long r = __builtin_amdgcn_mov_dpp(b, CTRL, 0xF, 0xF, false);
        return __builtin_bit_cast(double, r);
    } else {
        int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xF, 0xF, false);
        int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xF, 0xF, false);
        return __hiloint2double(hi, lo);
    }
}
// Lane j (a constant once the caller's loops are unrolled) of the robot's lane segment, to every
// lane of the segment: v_readlane for one robot per wave, DPP row_newbcast for 16-lane segments
// (one robot per DPP row: a VALU move, no SGPR round trip, no LDS), ds_bpermute for 32.
template <int SUB>
__device__ __forceinline__ double seg_bcast(double v, int j) {
    if constexpr (SUB == 64) {
        return bcast(v, j);
    } else if constexpr (SUB == 16) {
        switch (j) {
            case 0: return dpp_d<0x150>(v);
            case 1: return dpp_d<0x151>(v);
            case 2: return dpp_d<0x152>(v);
            case 3: return dpp_d<0x153>(v);
            case 4: return dpp_d<0x154>(v);
            case 5: return dpp_d<0x155>(v);
            case 6: return dpp_d<0x156>(v);
            case 7: return dpp_d<0x157>(v);
            case 8: return dpp_d<0x158>(v);
            case 9: return dpp_d<0x159>(v);
            case 10: return dpp_d<0x15A>(v);
            case 11: return dpp_d<0x15B>(v);
            case 12: return dpp_d<0x15C>(v);
            case 13: return dpp_d<0x15D>(v);
            case 14: return dpp_d<0x15E>(v);
            default: return dpp_d<0x15F>(v);
        }
    } else {
        return vbcast(v, ((int)threadIdx.x & ~(SUB - 1)) + j);
    }
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) { return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false); }

template <int CTRL>
__device__ __forceinline__ void argmin_step(double& v, int& i) {
    const double ov = dpp_d<CTRL>(v);
    const int oi = dpp_i<CTRL>(i);
    const bool take = (ov < v) || (ov == v && oi < i);
    v = take ? ov : v;
    i = take ? oi : i;
}
// argmin over the wave, ties to the lowest index; result uniform.  DPP within 16-lane rows
// (quad_perm, row_half_mirror, row_mirror), then the four row results via v_readlane.
__device__ __forceinline__ void wave_argmin(double& v, int& i) {
    argmin_step<0xB1>(v, i);   // quad_perm [1,0,3,2]
    argmin_step<0x4E>(v, i);   // quad_perm [2,3,0,1]
    argmin_step<0x141>(v, i);  // row_half_mirror
    argmin_step<0x140>(v, i);  // row_mirror
    double bv = bcast(v, 0);
    int bi = bcast_i(i, 0);
#pragma unroll
    for (int r = 16; r < 64; r += 16) {
        const double ov = bcast(v, r);
        const int oi = bcast_i(i, r);
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    v = bv;
    i = bi;
}
__device__ __forceinline__ bool wave_any(bool p) { return __any(p); }

// Wave argmin as a plain fp64 min: the lane index is written into the 6 low mantissa bits (as
// 63 - lane for negative values, so ties go to the lowest lane either way), then v_min_f64 over
// row_ror 8/4/2/1 and row_bcast 15/31 leaves the minimum in lane 63.  18 VALU + 2 readlanes
// instead of the compare/select ladder.  Returns the lane (uniform); callers re-read the exact
// value from that lane when they need it.  v must not be NaN.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_min(double v) {
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), CTRL, ROWMASK, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), CTRL, ROWMASK, 0xF, false);
    return fmin(v, __hiloint2double(hi, lo));
}
__device__ __forceinline__ int wave_argmin_lane(double v) {
    const int lane = lane_id();
    const int hi = __double2hiint(v);
    const int tag = (hi < 0) ? (63 - lane) : lane;
    v = __hiloint2double(hi, (__double2loint(v) & ~63) | tag);
    v = dpp_min<0x128, 0xF>(v);  // row_ror:8
    v = dpp_min<0x124, 0xF>(v);  // row_ror:4
    v = dpp_min<0x122, 0xF>(v);  // row_ror:2
    v = dpp_min<0x121, 0xF>(v);  // row_ror:1
    v = dpp_min<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v = dpp_min<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    const int mlo = __builtin_amdgcn_readlane(__double2loint(v), 63);
    const int mhi = __builtin_amdgcn_readlane(__double2hiint(v), 63);
    return (mhi < 0) ? (63 - (mlo & 63)) : (mlo & 63);
}

// The row to add in the one-robot-per-wave solves (solve_phase, solve_stance): the exact minimum m
// of v over the wave (the DPP min chain above without the lane tag), then the lowest lane whose v
// lies within WBC_TIE_BAND of it (include/wbc.h: near-ties are ties, decided by the row id, as the
// C oracle decides them).  v < 0 marks a violated row, 1e300 none; returns the lane (0 when m is
// 1e300) and m (uniform).
__device__ __forceinline__ int wave_select_band(double v, double& m) {
    double w = dpp_min<0x128, 0xF>(v);  // row_ror:8
    w = dpp_min<0x124, 0xF>(w);         // row_ror:4
    w = dpp_min<0x122, 0xF>(w);         // row_ror:2
    w = dpp_min<0x121, 0xF>(w);         // row_ror:1
    w = dpp_min<0x142, 0xA>(w);         // row_bcast:15 into rows 1, 3
    w = dpp_min<0x143, 0xC>(w);         // row_bcast:31 into rows 2, 3
    m = bcast(w, 63);
    const unsigned long long b = __ballot(v <= m * (1.0 - WBC_TIE_BAND));
    return b ? __builtin_ctzll(b) : 0;
}

// max |v| over the wave (uniform): the DPP min chain of wave_select_band on -|v|
__device__ __forceinline__ double wave_absmax(double v) {
    double w = dpp_min<0x128, 0xF>(-fabs(v));  // row_ror:8
    w = dpp_min<0x124, 0xF>(w);                 // row_ror:4
    w = dpp_min<0x122, 0xF>(w);                 // row_ror:2
    w = dpp_min<0x121, 0xF>(w);                 // row_ror:1
    w = dpp_min<0x142, 0xA>(w);                 // row_bcast:15 into rows 1, 3
    w = dpp_min<0x143, 0xC>(w);                 // row_bcast:31 into rows 2, 3
    return -bcast(w, 63);
}

// Sum over the 16 lanes of each DPP row (row_ror 8, 4, 2, 1); lane 0's value is broadcast so the
// result is uniform.  Used for the 13-body sums of the update phase (lanes >= 13 pass 0).
__device__ __forceinline__ double row0_sum(double v) {
    v += dpp_d<0x128>(v);
    v += dpp_d<0x124>(v);
    v += dpp_d<0x122>(v);
    v += dpp_d<0x121>(v);
    return bcast(v, 0);
}

// Segmented forms for the update kernel with several robots per wave (SUB lanes per robot, SUB in
// {16, 32, 64}): the row sum above, then the segment head's value to every lane of the segment
// (v_readlane for 64; DPP row_newbcast:0 for 16; ds_swizzle bitmask mode, lane & 0 within each
// 32-lane half, for 32), so every lane of a robot holds the same bits.
template <int AND>
__device__ __forceinline__ double swz_head(double v) {
    const int lo = __builtin_amdgcn_ds_swizzle(__double2loint(v), AND);
    const int hi = __builtin_amdgcn_ds_swizzle(__double2hiint(v), AND);
    return __hiloint2double(hi, lo);
}
template <int SUB>
__device__ __forceinline__ double seg_sum(double v) {
    static_assert(SUB == 16 || SUB == 32 || SUB == 64, "segment width");
    if constexpr (SUB == 64) {
        return row0_sum(v);
    } else {
        v += dpp_d<0x128>(v);
        v += dpp_d<0x124>(v);
        v += dpp_d<0x122>(v);
        v += dpp_d<0x121>(v);
        // 16: one robot per DPP row, row_newbcast:0 (a VALU move) instead of an LDS-pipe swizzle
        if constexpr (SUB == 16) return dpp_d<0x150>(v);
        else return swz_head<0x00>(v);
    }
}
template <int SUB>
__device__ __forceinline__ bool seg_any(bool p) {
    if constexpr (SUB == 64) {
        return __any(p);
    } else {
        const unsigned long long m = __ballot(p);
        const int seg = (int)threadIdx.x / SUB;
        return ((m >> (seg * SUB)) & ((1ull << SUB) - 1ull)) != 0ull;
    }
}

// v_min_f64 without fmin's quieting of its DPP-moved operand (a v_max_f64 x, x per step): the
// values reduced here are never NaN (1e300 marks "none"), and v_min_f64 is IEEE minNum anyway
__device__ __forceinline__ double vmin_f64(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// max(a, |b|) in one v_max_f64 (the source modifier), no quieting moves; operands never NaN here
__device__ __forceinline__ double vmaxabs_f64(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// max |S_rc| of a 6 x 6 matrix held as row r in lane r < 6 of the segment (lanes 6.. repeat row 5)
__device__ __forceinline__ double seg6_absmax(const double (&row)[6]) {
    double rm = 0.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) rm = vmaxabs_f64(rm, row[c]);
    double m = seg_bcast<16>(rm, 0);
#pragma unroll
    for (int k = 1; k < 6; ++k) m = vmaxabs_f64(m, seg_bcast<16>(rm, k));
    return m;
}
// One workgroup per robot: blockIdx -> robot.  (An XCD-aware remap, giving each XCD a contiguous
// robot range so that robot-major rows sharing a cache line stay in one L2, cut HBM traffic per
// launch 15.1 -> 11.4 MB but made the kernel 14 % slower at B = 4096, profiles/r01/variants_xcd_remap.log.)
__device__ __forceinline__ int xcd_robot() { return blockIdx.x; }

// ---------------------------------------------------------------------------------------
// small fp64 linear algebra (row-major 3x3)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void cross3(const double* a, const double* b, double* o) {
    double x = a[1] * b[2] - a[2] * b[1];
    double y = a[2] * b[0] - a[0] * b[2];
    double z = a[0] * b[1] - a[1] * b[0];
    o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ void mv3(const double* M, const double* v, double* o) {
    double x = M[0] * v[0] + M[1] * v[1] + M[2] * v[2];
    double y = M[3] * v[0] + M[4] * v[1] + M[5] * v[2];
    double z = M[6] * v[0] + M[7] * v[1] + M[8] * v[2];
    o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ void mm3(const double* A, const double* B, double* C) {
    double t[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) t[3 * i + j] = A[3 * i] * B[j] + A[3 * i + 1] * B[3 + j] + A[3 * i + 2] * B[6 + j];
#pragma unroll
    for (int k = 0; k < 9; ++k) C[k] = t[k];
}
__device__ __forceinline__ void rot_inertia(const double* R, const double* I, double* o) {  // R I R^T
    double t[9];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) t[3 * i + j] = R[3 * i] * I[j] + R[3 * i + 1] * I[3 + j] + R[3 * i + 2] * I[6 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) o[3 * i + j] = t[3 * i] * R[3 * j] + t[3 * i + 1] * R[3 * j + 1] + t[3 * i + 2] * R[3 * j + 2];
}
// Reciprocal and reciprocal square root: the hardware estimate (v_rcp_f64 / v_rsq_f64) plus two
// Newton steps (~1 ulp).  They replace IEEE division / sqrt sequences on the solver's sequential
// chains (Cholesky pivots, substitutions, Householder scalars), where latency is the cost.
__device__ __forceinline__ double fast_rcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ double fast_rsq(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    double e = fma(-h * y, y, 0.5);
    y = fma(y, e, y);
    e = fma(-h * y, y, 0.5);
    return fma(y, e, y);
}
__device__ __forceinline__ void inv3(const double* A, double* o) {
    double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
    double id = fast_rcp(A[0] * c00 + A[1] * c01 + A[2] * c02);
    o[0] = c00 * id; o[1] = (A[2] * A[7] - A[1] * A[8]) * id; o[2] = (A[1] * A[5] - A[2] * A[4]) * id;
    o[3] = c01 * id; o[4] = (A[0] * A[8] - A[2] * A[6]) * id; o[5] = (A[2] * A[3] - A[0] * A[5]) * id;
    o[6] = c02 * id; o[7] = (A[1] * A[6] - A[0] * A[7]) * id; o[8] = (A[0] * A[4] - A[1] * A[3]) * id;
}
// rotation about unit axis a by (s, c) = (sin q, cos q) (Rodrigues)
__device__ __forceinline__ void axis_rot(const double* a, double s, double c, double* R) {
    const double v = 1.0 - c;
    R[0] = c + a[0] * a[0] * v;        R[1] = a[0] * a[1] * v - a[2] * s; R[2] = a[0] * a[2] * v + a[1] * s;
    R[3] = a[1] * a[0] * v + a[2] * s; R[4] = c + a[1] * a[1] * v;        R[5] = a[1] * a[2] * v - a[0] * s;
    R[6] = a[2] * a[0] * v - a[1] * s; R[7] = a[2] * a[1] * v + a[0] * s; R[8] = c + a[2] * a[2] * v;
}
// Eigen::Quaterniond(w,x,y,z).toRotationMatrix() (cpp:209-213)
__device__ __forceinline__ void quat_R(double qx, double qy, double qz, double qw, double* R) {
    double tx = 2 * qx, ty = 2 * qy, tz = 2 * qz;
    double twx = tx * qw, twy = ty * qw, twz = tz * qw;
    double txx = tx * qx, txy = ty * qx, txz = tz * qx;
    double tyy = ty * qy, tyz = tz * qy, tzz = tz * qz;
    R[0] = 1 - (tyy + tzz); R[1] = txy - twz;       R[2] = txz + twy;
    R[3] = txy + twz;       R[4] = 1 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;       R[7] = tyz + twx;       R[8] = 1 - (txx + tyy);
}
// sin / cos of a joint angle: x = n pi/2 + r by a three-part FMA (Cody-Waite) reduction, |r| <=
// pi/4, and fdlibm's minimax kernels on r (< 1 ulp); ~40 instructions against the library
// sincos' ~150 (its general reduction).  |x| > 1e5 (no joint angle) takes the library call.
__device__ __forceinline__ void joint_sincos(double x, double* sn, double* cs) {
    const double n = __builtin_rint(x * 0.63661977236758134308);  // x * 2 / pi
    double r = fma(-n, 1.5707963267948966, x);                      // pi/2 in three parts
    r = fma(-n, 6.123233995736766e-17, r);
    r = fma(-n, -1.4973849048591698e-33, r);
    const double z = r * r;
    const double ps = fma(z, fma(z, fma(z, fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                        2.75573137070700676789e-06), -1.98412698298579493134e-04),
                          8.33333333332248946124e-03);
    const double sr = fma(z * r, fma(z, ps, -1.66666666666666324348e-01), r);
    const double pc = fma(z, fma(z, fma(z, fma(z, fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                               -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                 -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double cr = w + (((1.0 - w) - hz) + z * z * pc);
    const int q = (int)n & 3;
    const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
    *sn = (q & 2) ? -s0 : s0;
    *cs = ((q + 1) & 2) ? -c0 : c0;
    if (fabs(x) > 1e5) sincos(x, sn, cs);
}
// atan2 without branches (the pose angles, eulAnglesRPY cpp:12-20): t = min / max of |y|, |x| in
// [0, 1], atan t = atan c + atan((t - c) / (1 + c t)) with c = 0, 1/2 or 1 (|reduced| < 7/16) and
// fdlibm's atan kernel, then the octant / quadrant fix-ups; ~2 ulp (the division by fast_rcp)
__device__ __forceinline__ double atan2_br(double y, double x) {
    const double ax = fabs(x), ay = fabs(y);
    const double mx = fmax(ax, ay), mn = fmin(ax, ay);
    const double t = (mx > 0.0) ? mn * fast_rcp(mx) : 0.0;
    const bool c1 = t >= 0.6875, c5 = !c1 && t >= 0.4375;
    const double c = c1 ? 1.0 : (c5 ? 0.5 : 0.0);
    const double hi = c1 ? 7.85398163397448278999e-01 : (c5 ? 4.63647609000806093515e-01 : 0.0);
    const double lo = c1 ? 3.06161699786838301793e-17 : (c5 ? 2.26987774529616870924e-17 : 0.0);
    const double u = (t - c) * fast_rcp(fma(c, t, 1.0));
    const double z = u * u, w = z * z;
    const double s1 = z * fma(w, fma(w, fma(w, fma(w, fma(w, 1.62858201153657823623e-02, 4.97687799461593236017e-02),
                                                    6.66107313738753120669e-02), 9.09088713343650656196e-02),
                                     1.42857142725034663711e-01), 3.33333333333329318027e-01);
    const double s2 = w * fma(w, fma(w, fma(w, fma(w, -3.65315727442169155270e-02, -5.83357013379057348645e-02),
                                            -7.69187620504482999495e-02), -1.11111104054623557880e-01),
                              -1.99999999998764832476e-01);
    const double at = hi - ((u * (s1 + s2) - lo) - u);  // atan t
    double r = (ay > ax) ? 1.57079632679489655800e+00 - at : at;
    // quadrant from the sign bits (as std::atan2: atan2(+-0, x < 0) = +-pi, atan2(+-0, -0) = +-pi);
    // a comparison with 0.0 would treat -0 as +0 and return +pi for y = -0
    r = signbit(x) ? 3.14159265358979311600e+00 - r : r;
    return signbit(y) ? -r : r;
}
__device__ __forceinline__ double sel3(const double* v, int k) { return k == 0 ? v[0] : (k == 1 ? v[1] : v[2]); }
__device__ __forceinline__ double sel4d(int k, double a, double b, double c, double d) {
    return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d));
}
__device__ __forceinline__ double sel3d(int j, double a, double b, double c) { return j == 0 ? a : (j == 1 ? b : c); }

// Diagnostic build only (-DWBC_STAMPS): lane 0 records the shader clock at phase boundaries into
// the robot's debug record slots WBC_DBG_STAMPS.. (never read by the kernel, never an output).
#ifdef WBC_STAMPS
#define STAMP(a, rb, slot)                                                                             \
    do {                                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                                             \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();                                          \
        if (lane_id() == 0) (a).dbg[(size_t)(rb) * WBC_DBG_LEN + WBC_DBG_STAMPS + (slot)] = (double)t_; \
        __builtin_amdgcn_sched_barrier(0);                                                             \
    } while (0)
#else
#define STAMP(a, rb, slot) do { } while (0)
#endif
// Diagnostic build only (-DWBC_ISTAMPS): cycles spent in each sub-step of the active-set loop,
// summed over its iterations, written to debug slots 0..5 (never read by the kernel).
#ifdef WBC_ISTAMPS
#define IST_DECL                                          \
    unsigned long long ist_prev_ = __builtin_amdgcn_s_memtime(); \
    unsigned long long ist_acc_[6] = {0, 0, 0, 0, 0, 0}; \
    int ist_cnt_[2] = {0, 0}
#define IST_COUNT(i) (++ist_cnt_[i])
#define IST(i)                                                       \
    do {                                                             \
        __builtin_amdgcn_sched_barrier(0);                           \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
        ist_acc_[i] += t_ - ist_prev_;                               \
        ist_prev_ = t_;                                              \
        __builtin_amdgcn_sched_barrier(0);                           \
    } while (0)
#define IST_FLUSH(a, rb)                                                                          \
    do {                                                                                          \
        if (lane_id() == 0)                                                                       \
            for (int i_ = 0; i_ < 6; ++i_) (a).dbg[(size_t)(rb) * WBC_DBG_LEN + i_] = (double)ist_acc_[i_]; \
        if (lane_id() == 0)                                                                       \
            for (int i_ = 0; i_ < 2; ++i_) (a).dbg[(size_t)(rb) * WBC_DBG_LEN + 6 + i_] = (double)ist_cnt_[i_]; \
    } while (0)
// update-phase boundaries: absolute clock into debug slots 8.. (same build)
#define UST(a, rb, i)                                                                              \
    do {                                                                                           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
        const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                \
        if (lane_id() == 0) (a).dbg[(size_t)(rb) * WBC_DBG_LEN + 8 + (i)] = (double)t_;           \
        __builtin_amdgcn_sched_barrier(0);                                                         \
    } while (0)
#define EST(a, rb, i) UST(a, rb, 12 + (i))  // equality block / solve setup boundaries: slots 20..
#else
#define UST(a, rb, i) do { } while (0)
#define EST(a, rb, i) do { } while (0)
#define IST_DECL do { } while (0)
#define IST(i) do { } while (0)
#define IST_COUNT(i) do { } while (0)
#define IST_FLUSH(a, rb) do { } while (0)
#endif

// Row i (lane i < 12) of the slot coupling G = Jc_com Mbar_b^-1 Jc_com^T (unmasked; the constraint
// normals mask it).  With u_j = d_lj x e_rj: a . u_j = (a x d_lj)[rj], one cross product per leg.
__device__ __forceinline__ void g_row(const Prob& P, int i, double* grow) {
    const int li = i / 3, ri = i % 3;
    const double di[3] = {P.d[3 * li], P.d[3 * li + 1], P.d[3 * li + 2]};
    double e[3] = {ri == 0 ? 1.0 : 0.0, ri == 1 ? 1.0 : 0.0, ri == 2 ? 1.0 : 0.0}, ui[3], t[3];
    cross3(di, e, ui);
    mv3(P.Icinv, ui, t);
#pragma unroll
    for (int lj = 0; lj < 4; ++lj) {
        const double dj[3] = {P.d[3 * lj], P.d[3 * lj + 1], P.d[3 * lj + 2]};
        double gc[3];
        cross3(t, dj, gc);
#pragma unroll
        for (int rj = 0; rj < 3; ++rj) grow[3 * lj + rj] = (ri == rj ? P.inv_m : 0.0) + gc[rj];
    }
}

// The part of solveQP (cpp:466-515) that depends on the contact mask but not on the constraints:
// the slot Hessian H_s = I + Jc_com (I + Mbar_b^-2) Jc_com^T on stance slots (slack_weight I on
// swing slots; lane i < 12 of the robot's segment holds row i) and the slot gradient
// g_s = -Jc_com (W + [0, 0, g/m, 0, 0, 0]).
__device__ __forceinline__ void slot_hessian_row(const Prob& P, int kap, const wbc_params& pr, int lane,
                                                 double (&hrow)[12], double& gsv) {
    const double inv_m = P.inv_m;
    const int i = lane < 12 ? lane : 11, li = i / 3, ri = i % 3;
    const bool sti = (kap >> li) & 1;
    const double di[3] = {P.d[3 * li], P.d[3 * li + 1], P.d[3 * li + 2]};
    double e[3] = {ri == 0 ? 1.0 : 0.0, ri == 1 ? 1.0 : 0.0, ri == 2 ? 1.0 : 0.0}, ui[3];
    cross3(di, e, ui);
    double t[3], t2[3], Gu[3];
    mv3(P.Icinv, ui, t);
    mv3(P.Icinv, t, t2);
    Gu[0] = ui[0] + t2[0]; Gu[1] = ui[1] + t2[1]; Gu[2] = ui[2] + t2[2];
    const double ims = 1.0 + inv_m * inv_m;
#pragma unroll
    for (int lj = 0; lj < 4; ++lj) {
        const bool stj = (kap >> lj) & 1;
        const double dj[3] = {P.d[3 * lj], P.d[3 * lj + 1], P.d[3 * lj + 2]};
        double hc[3];
        cross3(Gu, dj, hc);
#pragma unroll
        for (int rj = 0; rj < 3; ++rj) {
            const int j = 3 * lj + rj;
            const double h = (i == j ? 1.0 : 0.0) + (ri == rj ? ims : 0.0) + hc[rj];
            hrow[j] = (sti && stj) ? h : ((!sti && i == j) ? pr.slack_weight : 0.0);
        }
    }
    gsv = sti ? -(P.W[ri] + (ri == 2 ? pr.gravity * inv_m : 0.0) + dot3(ui, &P.W[3])) : 0.0;
}

// Cholesky factor of a 12 x 12 SPD matrix (row i in lane i of the robot's segment, as hrow), its
// inverse M = L^-1 (lower, written over L) and x0 = -H^-1 g (g_i in lane i).  Returns false when
// the matrix is not positive definite.
template <int SUB>
__device__ bool factor12(double (&hrow)[12], double gsv, int lane, double (&L)[12][13], double* ild, double* xs,
                         [[maybe_unused]] const KernelArgs* ka = nullptr, [[maybe_unused]] int rb = 0) {
    // right-looking Cholesky, row i in lane i; L_jk broadcast from lane j of the segment
    bool chol_ok = true;
    double ildv = 1.0;  // lane k: 1 / L_kk
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const double dkk = seg_bcast<SUB>(hrow[k], k);
        chol_ok &= dkk > 0.0;
        const double il = fast_rsq(fmax(dkk, 1e-300));
        const double lkk = dkk * il;
        if (lane == k) ildv = il;
        hrow[k] = (lane == k) ? lkk : hrow[k] * il;   // L_ik for lanes i > k
        // trailing update, unmasked: lanes i < j only change their upper triangle, which is
        // never read (the factor is stored masked below)
#pragma unroll
        for (int j = k + 1; j < 12; ++j) hrow[j] = fma(-hrow[k], seg_bcast<SUB>(hrow[k], j), hrow[j]);
    }
    if (lane < 12) {
#pragma unroll
        for (int j = 0; j < 12; ++j) L[lane][j] = (j <= lane) ? hrow[j] : 0.0;
        ild[lane] = ildv;
    }
    lds_sync();  // L visible
    if (ka) UST(*ka, rb, 23);  // Cholesky
    // M = L^-1 (lower triangular), lane j forms column j by forward substitution; every later
    // use of the factor (C0 = L^-1 n_s, x0, primal recovery) is then a matvec without a chain
    double (&Mi)[12][12] = *reinterpret_cast<double(*)[12][12]>(&L[0][0]);
    {
        double m[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < i; ++k) a4[k & 3] += L[i][k] * m[k];
            m[i] = (((lane == i) ? 1.0 : 0.0) - ((a4[0] + a4[1]) + (a4[2] + a4[3]))) * ild[i];
        }
        lds_sync();  // all reads of L done: M overwrites it
        if (lane < 12) {
#pragma unroll
            for (int i = 0; i < 12; ++i) Mi[i][lane] = (i >= lane) ? m[i] : 0.0;
        }
    }
    lds_sync();
    if (ka) UST(*ka, rb, 24);  // M = L^-1
    // x0 = -H^-1 g = -M^T (M g): g_k and z_k broadcast from lane k
    {
        double gk[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) gk[k] = seg_bcast<SUB>(gsv, k);
        const int i = lane < 12 ? lane : 0;
        double z4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 12; ++k) z4[k & 3] += Mi[i][k] * gk[k];
        const double zi = (z4[0] + z4[1]) + (z4[2] + z4[3]);
        double x4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 12; ++k) x4[k & 3] += Mi[k][i] * seg_bcast<SUB>(zi, k);
        if (lane < 12) xs[lane] = -((x4[0] + x4[1]) + (x4[2] + x4[3]));
    }
    lds_sync();
    return chol_ok;
}

// The same factorisation for the inline solve of the general 12-variable form (§4.8), without the
// LDS round trips of factor12: the Cholesky as there (row i in lane i), then lane j forms column j of
// M = L^-1 by forward substitution with L's entries broadcast from their rows' lanes (DPP); column j
// of M is row j of J0 = L^-T, written straight into the J mirror (`Jm`, 12 x 12 row-major, J rows as
// solve16 keeps them); x0 = -H^-1 g = -J0 (J0^T g) (the mirror's columns, then the lane's own row).
// Returns false when H is not positive definite.
__device__ bool factor12_rows(double (&hrow)[12], double gsv, int lane, double* Jm, double* xs) {
    bool chol_ok = true;
    double ildv = 1.0;  // lane k: 1 / L_kk
#pragma unroll
    for (int k = 0; k < 12; ++k) {
        const double dkk = seg_bcast<16>(hrow[k], k);
        chol_ok &= dkk > 0.0;
        const double il = fast_rsq(fmax(dkk, 1e-300));
        const double lkk = dkk * il;
        if (lane == k) ildv = il;
        hrow[k] = (lane == k) ? lkk : hrow[k] * il;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) hrow[j] = fma(-hrow[k], seg_bcast<16>(hrow[k], j), hrow[j]);
    }
    // lane j: m = column j of M (m[i] = 0 for i < j); L[i][k] = hrow[k] of lane i
    double m[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < i; ++k) a4[k & 3] = fma(seg_bcast<16>(hrow[k], i), m[k], a4[k & 3]);
        m[i] = (((lane == i) ? 1.0 : 0.0) - ((a4[0] + a4[1]) + (a4[2] + a4[3]))) * seg_bcast<16>(ildv, i);
    }
    if (lane < 12) {
#pragma unroll
        for (int j = 0; j < 12; j += 2) *reinterpret_cast<double2*>(&Jm[lane * JMS + j]) = make_double2(m[j], m[j + 1]);
    }
    lds_sync();
    // z = J0^T g (lane i: column i of the mirror . g), x0_l = -(J0 row l) . z
    const int i = lane < 12 ? lane : 0;
    double z4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 12; ++k) z4[k & 3] = fma(Jm[k * JMS + i], seg_bcast<16>(gsv, k), z4[k & 3]);
    const double zi = (z4[0] + z4[1]) + (z4[2] + z4[3]);
    double x4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 12; ++k) x4[k & 3] = fma(m[k], seg_bcast<16>(zi, k), x4[k & 3]);
    if (lane < 12) xs[lane] = -((x4[0] + x4[1]) + (x4[2] + x4[3]));
    lds_sync();
    return chol_ok;
}

// Slot factorisation of the general solve: H_s, its factor, M = L^-1 and x0's slot part.  Runs
// at the end of the update (four robots per wave in the update kernel) or, under mode
// hypotheses, in the solve.  Returns false when H_s is not positive definite.
template <int SUB>
__device__ bool presolve(const Prob& P, int kap, const wbc_params& pr, int lane, double (&L)[12][13], double* ild,
                         double* xs) {
    double hrow[12], gsv;
    slot_hessian_row(P, kap, pr, lane, hrow, gsv);
    return factor12<SUB>(hrow, gsv, lane, L, ild, xs);
}

// Maximum over each 16-lane DPP row (row_ror 8/4/2/1 leaves it in every lane of the row).
__device__ __forceinline__ double seg16_max(double v) {
    v = fmax(v, dpp_d<0x128>(v));
    v = fmax(v, dpp_d<0x124>(v));
    v = fmax(v, dpp_d<0x122>(v));
    v = fmax(v, dpp_d<0x121>(v));
    return v;
}
// Index (within the row) of the lane of each 16-lane DPP row holding the largest v >= 0, ties to
// the lowest lane: the lane index is written into the 4 low mantissa bits before the max.
__device__ __forceinline__ int seg16_argmax(double v) {
    const int tag = 15 - ((int)threadIdx.x & 15);
    v = seg16_max(__hiloint2double(__double2hiint(v), (__double2loint(v) & ~15) | tag));
    return 15 - (__double2loint(v) & 15);
}

// Four-contact stance (kappa = 15): eliminate the 12 stance equalities Jbj qdd + G f = e (R1,
// cpp:494,504; G = E Mb^-1 E^T with E = Jc_com, rows [I, -S(d_l)]; e = r1 + g e_z) as qdd = q0 - P f.
// Jbj = Jblk - E K is the block-diagonal foot Jacobian (one 3x3 block per leg) minus a rank-6 term
// (K = Mb^-1 A_j), so by Woodbury, with W = Jblk^-1 E and S = I6 - K W:
//   Jbj^-1 E = W S^-1 = Y,   q0 = Jbj^-1 e = w + Y K w (w = Jblk^-1 e),   P = Y Mb^-1 E^T,
// and the force-space Hessian H_f = H_s + P^T P = I + E H^ E^T with H^ = I + Mb^-2 + Mb^-1 Y^T Y Mb^-1
// (H_s = I + E (I + Mb^-2) E^T).  Per robot that is four 3x3 inverses, one 6x6 inverse and a few
// 12 x 6 products; no 12-step elimination chain.  Also formed: the gradient g_f = g_s - P^T q0,
// the torque map Nt = Mbj P + Jbj^T and t0 = bbj + Mbj q0 (stored with Y, q0 and the torque
// rows' reference-space norms), H_f row i and g_f in hrow / gsv for factor12.  Returns false
// (nothing usable stored; the caller takes the general path) at a near-singular leg or S.
// Lane i < 12 of the segment is row i = 3 l + k; SUB = 16 only (one robot per DPP row).
// SOLVE (the update kernel's inline stance solve, wbc_update_solve_kernel): Nt, Y, q0, t0 and the
// norms stay in the robot's LDS scratch (St16) instead of going to the Presolve record.
template <bool SOLVE>
__device__ bool stance_reduce([[maybe_unused]] const KernelArgs& ka, [[maybe_unused]] int rb, const Prob& P,
                              const wbc_params& pr, int lane, bool wr, UpdScratch& s, double (&hrow)[12],
                              double& gsv, Presolve* pre) {
    auto& R = s.sr;
    const int i = lane < 12 ? lane : 11, l = i / 3, k = i % 3;
    const double dl[3] = {P.d[3 * l], P.d[3 * l + 1], P.d[3 * l + 2]};
    const double inv_m = P.inv_m;
    // row k of Jblk_l^-1 and the leg's conditioning
    double jr[3];
    bool ok;
    {
        const double* A = s.Jf[l];
        const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
        const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
        double amx = 0.0;
#pragma unroll
        for (int t = 0; t < 9; ++t) amx = fmax(amx, fabs(A[t]));
        ok = fabs(det) > 1e-9 * amx * amx * amx;
        const double id = fast_rcp(ok ? det : 1.0);
        const double r0[3] = {c00, A[2] * A[7] - A[1] * A[8], A[1] * A[5] - A[2] * A[4]};
        const double r1[3] = {c01, A[0] * A[8] - A[2] * A[6], A[2] * A[3] - A[0] * A[5]};
        const double r2[3] = {c02, A[1] * A[6] - A[0] * A[7], A[0] * A[4] - A[1] * A[3]};
#pragma unroll
        for (int t = 0; t < 3; ++t) jr[t] = ((k == 0) ? r0[t] : (k == 1) ? r1[t] : r2[t]) * id;
    }
    // W row i = [jr, d_l x jr], w_i = jr . e_l
    if (lane < 12) {
        double dxj[3];
        cross3(dl, jr, dxj);
        double wi = 0.0;
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            R.W[i][t] = jr[t];
            R.W[i][3 + t] = dxj[t];
            wi = fma(jr[t], P.r1[3 * l + t] + (t == 2 ? pr.gravity : 0.0), wi);
        }
        R.w[i] = wi;
    }
    lds_sync();
    UST(ka, rb, 19);  // leg inverses, W rows
    // [S | z] = [I - K W | K w], K[a][j] = A_j[a] / m (a < 3), (I_c^-1 A_ang)_j[a - 3]: 42 entries in
    // one round, lane < 12 -> row lane % 6, columns 0..2 or 3..6 (h = lane / 6), each entry summed
    // in the same order as a one-entry-per-lane loop
    {
        const int ra = lane % 6, h = (lane / 6) & 1;
        double acc[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        // both K entries loaded unconditionally and selected: a load under the lane-dependent
        // condition became a branch with its own LDS wait, 12 serialized round trips
        const int ra3 = ra < 3 ? ra : 0, rk3 = ra < 3 ? 0 : ra - 3;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double av = s.A[j][ra3], kv = s.KA[j][rk3];
            const double kj = (ra < 3) ? av * inv_m : kv;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c][j & 3] = fma(kj, R.W[j][3 * h + c], acc[c][j & 3]);
            acc[3][j & 3] = fma(kj, R.w[j], acc[3][j & 3]);
        }
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int cb = 3 * h + c;
                R.S[ra][cb] = (ra == cb ? 1.0 : 0.0) - ((acc[c][0] + acc[c][1]) + (acc[c][2] + acc[c][3]));
            }
            if (h) R.S[ra][6] = (acc[3][0] + acc[3][1]) + (acc[3][2] + acc[3][3]);
        }
    }
    lds_sync();
    UST(ka, rb, 20);  // S
    // S^-1 by Gauss-Jordan without pivoting (S is well conditioned: cond < 10 on the bench and
    // stress states, smallest pivot > 0.25 max|S|; a pivot below 1e-6 max|S| takes the general
    // path), row r in lane r < 6, pivot rows broadcast with DPP row_newbcast
    // Row r of S^-1 (ir) and z_r = S[r][6] stay in lane r's registers for the Y rows below, which
    // take them by DPP broadcast (LDS reads of S^-1 there waited ~19 times)
    double ir[6], zr;
    {
        const int r = lane < 6 ? lane : 5;
        double sr_[6];
        zr = R.S[r][6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            sr_[c] = R.S[r][c];
            ir[c] = (r == c) ? 1.0 : 0.0;
        }
        const double smx = seg6_absmax(sr_);  // max |S|: row maxima, then over the six row lanes
        double pmin = 1e300;
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
            const double pv = seg_bcast<16>(sr_[kk], kk);
            pmin = fmin(pmin, fabs(pv));
            const double ip = fast_rcp(pv);
            double prow[12];
#pragma unroll
            for (int c = kk + 1; c < 6; ++c) prow[c] = seg_bcast<16>(sr_[c], kk);
#pragma unroll
            for (int c = 0; c <= kk; ++c) prow[6 + c] = seg_bcast<16>(ir[c], kk);
            const double f = (lane == kk) ? 0.0 : sr_[kk] * ip;
            const double own = (lane == kk) ? ip : 1.0;
#pragma unroll
            for (int c = kk + 1; c < 6; ++c) sr_[c] = fma(-f, prow[c], sr_[c] * own);
#pragma unroll
            for (int c = 0; c <= kk; ++c) ir[c] = fma(-f, prow[6 + c], ir[c] * own);
        }
        ok = ok && pmin > 1e-6 * smx;
        UST(ka, rb, 12);  // leg inverses, S, S^-1
    }
    ok = !seg_any<16>(!ok);  // every leg and S usable (uniform over the robot)
    lds_sync();
    // Y row i = W_i S^-1, q0_i = w_i + Y_i z
    double yi[6], q = 0.0;  // row i of Y and q0_i, kept for the Nt stage's DPP broadcasts
    {
        double wrow[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) wrow[c] = R.W[i][c];
        q = R.w[i];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            double a4[2] = {0.0, 0.0};
#pragma unroll
            for (int t = 0; t < 6; ++t) a4[t & 1] = fma(wrow[t], seg_bcast<16>(ir[c], t), a4[t & 1]);
            yi[c] = a4[0] + a4[1];
            q = fma(yi[c], seg_bcast<16>(zr, c), q);
        }
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 6; ++c) R.Y[i][c] = yi[c];
            R.q0[i] = q;
        }
    }
    lds_sync();
    UST(ka, rb, 21);  // Y, q0
    // [Q | v] = [Y^T Y | Y^T q0]: 42 entries in one round, as S above
    {
        const int ra = lane % 6, h = (lane / 6) & 1;
        double acc[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double yj = R.Y[j][ra];
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c][j & 3] = fma(yj, R.Y[j][3 * h + c], acc[c][j & 3]);
            acc[3][j & 3] = fma(yj, R.q0[j], acc[3][j & 3]);
        }
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 3; ++c) R.Q[ra][3 * h + c] = (acc[c][0] + acc[c][1]) + (acc[c][2] + acc[c][3]);
            if (h) R.Q[ra][6] = (acc[3][0] + acc[3][1]) + (acc[3][2] + acc[3][3]);
        }
    }
    lds_sync();
    UST(ka, rb, 22);  // Q = Y^T Y
    // H^ rows (lane a < 6) over S: H^ = I + Mb^-2 + Mb^-1 Q Mb^-1, Mb^-1 = diag(I / m, I_c^-1)
    {
        const int ra = lane < 6 ? lane : 5;
        // T = Q Mb^-1, rows ra (lin) or 3..5 (ang, then I_c^-1 from the left)
        auto qm = [&](int row, double* o) {
#pragma unroll
            for (int c = 0; c < 3; ++c) o[c] = R.Q[row][c] * inv_m;
#pragma unroll
            for (int c = 0; c < 3; ++c)
                o[3 + c] = R.Q[row][3] * P.Icinv[c] + R.Q[row][4] * P.Icinv[3 + c] + R.Q[row][5] * P.Icinv[6 + c];
        };
        double hr[6];
        if (ra < 3) {
            qm(ra, hr);
#pragma unroll
            for (int c = 0; c < 6; ++c) hr[c] *= inv_m;
            hr[ra] += 1.0 + inv_m * inv_m;
        } else {
            double t3[3][6];
            qm(3, t3[0]); qm(4, t3[1]); qm(5, t3[2]);
            const int a3 = ra - 3;
            const double* ic = &P.Icinv[3 * a3];
#pragma unroll
            for (int c = 0; c < 6; ++c) hr[c] = ic[0] * t3[0][c] + ic[1] * t3[1][c] + ic[2] * t3[2][c];
            hr[ra] += 1.0;
#pragma unroll
            for (int c = 0; c < 3; ++c)  // (I_c^-2)[a3][c]
                hr[3 + c] += ic[0] * P.Icinv[c] + ic[1] * P.Icinv[3 + c] + ic[2] * P.Icinv[6 + c];
        }
        // v -> Mb^-1 v (uniform, every lane) for g_f
        lds_sync();  // all reads of S's z column done
        if (lane < 6) {
#pragma unroll
            for (int c = 0; c < 6; ++c) R.S[lane][c] = hr[c];
        }
    }
    double uv[6];
#pragma unroll
    for (int c = 0; c < 3; ++c) uv[c] = R.Q[c][6] * inv_m;
#pragma unroll
    for (int c = 0; c < 3; ++c) uv[3 + c] = P.Icinv[3 * c] * R.Q[3][6] + P.Icinv[3 * c + 1] * R.Q[4][6] + P.Icinv[3 * c + 2] * R.Q[5][6];
    lds_sync();
    // H_f row i = e_i + E H^ E_i^T: h = H^ E_i^T, then E_j . h = h[k_j] - (d_{l_j} x h_ang)[k_j]
    // (not needed by the inline solve's rank-6 factor)
    {
        if constexpr (!SOLVE) {
        double h[6];
#pragma unroll
        for (int ra = 0; ra < 6; ++ra) {
            // E_i = [e_k, -S(d_l) row k]: -S(d) rows (0, d2, -d1), (-d2, 0, d0), (d1, -d0, 0)
            const double e3 = (k == 0) ? 0.0 : (k == 1) ? -dl[2] : dl[1];
            const double e4 = (k == 0) ? dl[2] : (k == 1) ? 0.0 : -dl[0];
            const double e5 = (k == 0) ? -dl[1] : (k == 1) ? dl[0] : 0.0;
            const double hk = (k == 0) ? R.S[ra][0] : (k == 1) ? R.S[ra][1] : R.S[ra][2];
            h[ra] = hk + e3 * R.S[ra][3] + e4 * R.S[ra][4] + e5 * R.S[ra][5];
        }
#pragma unroll
        for (int lj = 0; lj < 4; ++lj) {
            const double dj[3] = {P.d[3 * lj], P.d[3 * lj + 1], P.d[3 * lj + 2]};
            double cr[3];
            cross3(dj, &h[3], cr);
#pragma unroll
            for (int kj = 0; kj < 3; ++kj) hrow[3 * lj + kj] = ((3 * lj + kj == i) ? 1.0 : 0.0) + h[kj] - cr[kj];
        }
        }
        // g_f = g_s - E_i Mb^-1 v,  g_s = -E_i (W + [0, 0, g / m, 0, 0, 0])
        double wv[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) wv[c] = P.W[c] + (c == 2 ? pr.gravity * inv_m : 0.0) + uv[c];
        double cw[3];
        cross3(dl, &wv[3], cw);
        gsv = -(((k == 0) ? wv[0] : (k == 1) ? wv[1] : wv[2]) - ((k == 0) ? cw[0] : (k == 1) ? cw[1] : cw[2]));
    }
    UST(ka, rb, 13);  // Y, H_f row, g_f
    // Nt row j = (Mbj Y)_j Mb^-1 E^T + Jbj column j; t0_j = bbj_j + Mbj row j . q0.  Row kk of Y and
    // q0_kk come from lane kk's registers by DPP (from LDS they were ~40 address adds, 40 reads and
    // their waits), and each of the six sums runs as two chains of six
    const int j = i;
    {
        double my[2][6] = {{0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}}, t4[2] = {0.0, 0.0}, s2 = 0.0;
#pragma unroll
        for (int kk = 0; kk < 12; ++kk) {
            const double mk = P.Mbj[j * 12 + kk], jc = P.Jbj[kk * 12 + j];
#pragma unroll
            for (int c = 0; c < 6; ++c) my[kk & 1][c] = fma(mk, seg_bcast<16>(yi[c], kk), my[kk & 1][c]);
            t4[kk & 1] = fma(mk, seg_bcast<16>(q, kk), t4[kk & 1]);
            s2 = fma(mk, mk, fma(jc, jc, s2));
        }
        double mm[6], ms[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) ms[c] = my[0][c] + my[1][c];
#pragma unroll
        for (int c = 0; c < 3; ++c) mm[c] = ms[c] * inv_m;
#pragma unroll
        for (int c = 0; c < 3; ++c) mm[3 + c] = P.Icinv[3 * c] * ms[3] + P.Icinv[3 * c + 1] * ms[4] + P.Icinv[3 * c + 2] * ms[5];
        double nt[12];
#pragma unroll
        for (int lj = 0; lj < 4; ++lj) {
            const double dj[3] = {P.d[3 * lj], P.d[3 * lj + 1], P.d[3 * lj + 2]};
            double cr[3];
            cross3(dj, &mm[3], cr);
#pragma unroll
            for (int kj = 0; kj < 3; ++kj) nt[3 * lj + kj] = mm[kj] - cr[kj] + P.Jbj[(3 * lj + kj) * 12 + j];
        }
        if constexpr (SOLVE) {
            const St16 V(s, nullptr);
            if (lane < 12) {
#pragma unroll
                for (int c = 0; c < 12; c += 2)
                    V.Nt[j * NTS_ST + c] = nt[c], V.Nt[j * NTS_ST + c + 1] = nt[c + 1];
#pragma unroll
                for (int c = 0; c < 6; c += 2) *reinterpret_cast<double2*>(&V.Y[j * 6 + c]) = make_double2(yi[c], yi[c + 1]);
                V.q0[j] = q;
                V.t0[j] = P.bbj[j] + (t4[0] + t4[1]);
                V.nsel[j] = s2;
            }
        } else if (ok && wr && lane < 12) {
#pragma unroll
            for (int c = 0; c < 12; c += 2)
                *reinterpret_cast<double2*>(&pre->Nt[j * 12 + c]) = make_double2(nt[c], nt[c + 1]);
#pragma unroll
            for (int c = 0; c < 6; c += 2) *reinterpret_cast<double2*>(&pre->Y[j * 6 + c]) = make_double2(yi[c], yi[c + 1]);
            pre->q0[j] = q;
            pre->t0[j] = P.bbj[j] + (t4[0] + t4[1]);
            pre->nsel[j] = s2;
        }
    }
    lds_sync();  // the scratch (aliasing the factor's L) is read completely before factor12 writes L
    UST(ka, rb, 14);  // Nt, t0, record stores
    return ok;
}

// ---------------------------------------------------------------------------------------
// Force-space factor for the inline solve without a 12-step Cholesky.  H_f = I + E Ĥ Eᵀ
// is the identity plus rank 6 (E = stacked [I, -S(d_l)], 12 x 6), and the dual method needs only
// some J0 with J0 J0ᵀ = H_f⁻¹ (its iterates do not depend on which).  With EᵀE = L_G L_Gᵀ and
// Q = E L_G⁻ᵀ (orthonormal columns), H_f = (I - QQᵀ) + Q (I + B) Qᵀ for B = L_Gᵀ Ĥ L_G, so with
// I + B = L6 L6ᵀ:  J0 = I + Q (L6⁻ᵀ - I) Qᵀ  and  f0 = -J0 J0ᵀ g.  EᵀE = [[4I, -S(D)], [S(D), Σ(|d|² I - d dᵀ)]]
// (D = Σ d_l) has the block factor L_G = [[2I, 0], [S(D)/2, L22]] with L22 = chol(Σ(|d|² I - d dᵀ) +
// S(D)²/4), and row i = 3 l + k of Q is [e_k / 2, L22⁻¹ p_k(d_l - D/4)] (p_k(v) = row k of -S(v)).
// Every lane forms the 6 x 6 quantities (uniform), lane i < 12 its row of J0 and f0_i; the rows go
// to the J mirror (over Ĥ's LDS, read first) and f0 to ps.xs.  False at a degenerate foot layout.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void pk3(int k, const double* v, double* o) {  // row k of -S(v)
    o[0] = (k == 0) ? 0.0 : (k == 1) ? -v[2] : v[1];
    o[1] = (k == 0) ? v[2] : (k == 1) ? 0.0 : -v[0];
    o[2] = (k == 0) ? -v[1] : (k == 1) ? v[0] : 0.0;
}
__device__ __forceinline__ bool rank6_factor(const Prob& P, UpdScratch& s, double gsv, int lane) {
    const int i = lane < 12 ? lane : 11, li = i / 3, ki = i % 3;
    double Hh[6][6];
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = 0; b < 6; ++b) Hh[a][b] = s.sr.S[a][b];
    double dl[4][3], D[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int c = 0; c < 3; ++c) { dl[l][c] = P.d[3 * l + c]; D[c] += dl[l][c]; }
    // M22 = sum_l (|d_l|^2 I - d_l d_l^T) + (D D^T - |D|^2 I) / 4, its six distinct entries: the
    // diagonal (a; b, c the other two axes) sum_l (d_lb^2 + d_lc^2) - (D_b^2 + D_c^2) / 4, the
    // off-diagonal D_a D_b / 4 - sum_l d_la d_lb
    double M22[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int b = (a + 1) % 3, c = (a + 2) % 3;
        double t = -0.25 * fma(D[b], D[b], D[c] * D[c]);
        double o = 0.25 * D[a] * D[b];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            t = fma(dl[l][b], dl[l][b], fma(dl[l][c], dl[l][c], t));
            o = fma(-dl[l][a], dl[l][b], o);
        }
        M22[a][a] = t;
        M22[a][b] = M22[b][a] = o;
    }
    // L22 = chol(M22), its reciprocal diagonal
    const double sc = fmax(M22[0][0], fmax(M22[1][1], M22[2][2]));
    const double p0 = M22[0][0], r0 = fast_rsq(fmax(p0, 1e-300));
    const double l00 = p0 * r0, l10 = M22[1][0] * r0, l20 = M22[2][0] * r0;
    const double p1 = M22[1][1] - l10 * l10, r1 = fast_rsq(fmax(p1, 1e-300));
    const double l11 = p1 * r1, l21 = (M22[2][1] - l20 * l10) * r1;
    const double p2 = M22[2][2] - l20 * l20 - l21 * l21, r2 = fast_rsq(fmax(p2, 1e-300));
    const double l22 = p2 * r2;
    const bool ok = p0 > 1e-10 * sc && p1 > 1e-10 * sc && p2 > 1e-10 * sc;
    const double L22[3][3] = {{l00, 0.0, 0.0}, {l10, l11, 0.0}, {l20, l21, l22}};
    const double SD[3][3] = {{0.0, -D[2], D[1]}, {D[2], 0.0, -D[0]}, {-D[1], D[0], 0.0}};  // S(D)
    // C6 = I + L_Gᵀ Ĥ L_G, one column per lane: lane cc < 6 forms column cc of X = Ĥ L_G (6 x 6
    // products with its column of L_G) and then column cc of C6 (L_Gᵀ's entries are uniform), and
    // the lower triangle goes to every lane of the segment by DPP (the 6 x 6 algebra in every lane
    // was ~250 instructions, the lane-parallel form ~90)
    double C[6][6];
    {
        const int cc = lane < 6 ? lane : 5;
        const bool lin = cc < 3;
        const int c3 = lin ? cc : cc - 3;
        // column cc of L_G = [[2I, 0], [S(D)/2, L22]]
        double gcol[6];
#pragma unroll
        for (int k = 0; k < 3; ++k) gcol[k] = (k == cc) ? 2.0 : 0.0;
#pragma unroll
        for (int m = 0; m < 3; ++m)
            gcol[3 + m] = lin ? 0.5 * sel3d(c3, SD[m][0], SD[m][1], SD[m][2]) : sel3d(c3, L22[m][0], L22[m][1], L22[m][2]);
        double Xc[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            double t0 = Hh[r][0] * gcol[0], t1 = Hh[r][3] * gcol[3];
            t0 = fma(Hh[r][1], gcol[1], t0);
            t1 = fma(Hh[r][4], gcol[4], t1);
            t0 = fma(Hh[r][2], gcol[2], t0);
            t1 = fma(Hh[r][5], gcol[5], t1);
            Xc[r] = t0 + t1;
        }
        double Cc[6];
#pragma unroll
        for (int a = 0; a < 6; ++a) {
            double t;
            if (a < 3) {
                t = 2.0 * Xc[a];
#pragma unroll
                for (int m = 0; m < 3; ++m)
                    if (m != a) t = fma(0.5 * SD[m][a], Xc[3 + m], t);
            } else {
                t = 0.0;
#pragma unroll
                for (int m = a - 3; m < 3; ++m) t = fma(L22[m][a - 3], Xc[3 + m], t);
            }
            Cc[a] = t + ((a == cc) ? 1.0 : 0.0);
        }
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int c = 0; c <= a; ++c) C[a][c] = seg_bcast<16>(Cc[a], c);
    }
    // L6 = chol(C6) in place (lower), id = 1 / diag; Li = L6⁻¹ (lower)
    double id[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const double ir = fast_rsq(C[k][k]);
        id[k] = ir;
        C[k][k] *= ir;
#pragma unroll
        for (int a = k + 1; a < 6; ++a) C[a][k] *= ir;
#pragma unroll
        for (int a = k + 1; a < 6; ++a)
#pragma unroll
            for (int b = k + 1; b <= a; ++b) C[a][b] = fma(-C[a][k], C[b][k], C[a][b]);
    }
    double Li[6][6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        Li[j][j] = id[j];
#pragma unroll
        for (int a = j + 1; a < 6; ++a) {
            double t = 0.0;
#pragma unroll
            for (int m = j; m < a; ++m) t = fma(C[a][m], Li[m][j], t);
            Li[a][j] = -t * id[a];
        }
    }
    // lane i: xb_i = L22⁻¹ p_ki(d_li - D/4) (Q_i = [e_ki / 2, xb_i])
    double ul[4][3];
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int c = 0; c < 3; ++c) ul[l][c] = dl[l][c] - 0.25 * D[c];
    auto l22solve = [&](const double* v, double* o) {  // L22 o = v
        o[0] = v[0] * r0;
        o[1] = (v[1] - l10 * o[0]) * r1;
        o[2] = (v[2] - l20 * o[0] - l21 * o[1]) * r2;
    };
    double xb[3];
    {
        const double u3[3] = {sel4d(li, ul[0][0], ul[1][0], ul[2][0], ul[3][0]), sel4d(li, ul[0][1], ul[1][1], ul[2][1], ul[3][1]),
                              sel4d(li, ul[0][2], ul[1][2], ul[2][2], ul[3][2])};
        double pv[3];
        pk3(ki, u3, pv);
        l22solve(pv, xb);
    }
    const double qt[3] = {ki == 0 ? 0.5 : 0.0, ki == 1 ? 0.5 : 0.0, ki == 2 ? 0.5 : 0.0};
    // a_i = Q_i T, T = Liᵀ - I: a[c] = sum_{r <= c} Q_i[r] Li[c][r] - Q_i[c]
    const double Qi[6] = {qt[0], qt[1], qt[2], xb[0], xb[1], xb[2]};
    double ai[6];
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        double t = -Qi[c];
#pragma unroll
        for (int r = 0; r <= c; ++r) t = fma(Qi[r], Li[c][r], t);
        ai[c] = t;
    }
    // b_i = L22⁻ᵀ a_i[3..5]; J0[i][j] = delta_ij + a_i[kj] / 2 + b_i . p_kj(u_lj)
    double bi[3];
    bi[2] = ai[5] * r2;
    bi[1] = (ai[4] - l21 * bi[2]) * r1;
    bi[0] = (ai[3] - l10 * bi[1] - l20 * bi[2]) * r0;
    // b_i . p_k(u) has two nonzero terms (p_k(u) = row k of -S(u)); written out, since x * 0.0 is
    // not folded (x may be inf)
    const double ha[3] = {0.5 * ai[0], 0.5 * ai[1], 0.5 * ai[2]};
    double J0[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        const double* u = ul[j / 3];
        const int k = j % 3;
        const double t = (k == 0) ? fma(bi[1], u[2], fma(-bi[2], u[1], ha[0]))
                       : (k == 1) ? fma(bi[2], u[0], fma(-bi[0], u[2], ha[1]))
                                  : fma(bi[0], u[1], fma(-bi[1], u[0], ha[2]));
        J0[j] = (i == j) ? t + 1.0 : t;
    }
    // f0 = -J0 J0ᵀ g: Eᵀ v = [sum_l v_l, sum_l d_l x v_l]; q6 = L_G⁻¹ Eᵀ v
    auto q6_of = [&](double vv, double* q6) {
        double top[3] = {0.0, 0.0, 0.0}, bot[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const double v3[3] = {seg_bcast<16>(vv, 3 * l), seg_bcast<16>(vv, 3 * l + 1), seg_bcast<16>(vv, 3 * l + 2)};
            double cr[3];
            cross3(dl[l], v3, cr);
#pragma unroll
            for (int c = 0; c < 3; ++c) { top[c] += v3[c]; bot[c] += cr[c]; }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) q6[c] = 0.5 * top[c];
        double dq[3], rhs[3];
        cross3(D, q6, dq);
#pragma unroll
        for (int c = 0; c < 3; ++c) rhs[c] = bot[c] - 0.5 * dq[c];
        l22solve(rhs, &q6[3]);
    };
    // f0 = J0 (J0ᵀ g), through the factor the loop uses: the shorter g + Q((I + B)⁻¹ - I)Qᵀ g
    // (one Eᵀ product less) leans on QᵀQ = I and moved x* by ~2e-8 relative on stress inputs
    double q6[6];
    q6_of(gsv, q6);
    double w[6];  // w = Tᵀ q6 = Li q6 - q6
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        double t = -q6[c];
#pragma unroll
        for (int r = 0; r <= c; ++r) t = fma(Li[c][r], q6[r], t);
        w[c] = t;
    }
    double y = gsv;
#pragma unroll
    for (int c = 0; c < 6; ++c) y = fma(Qi[c], w[c], y);
    q6_of(y, q6);
    double v[6];  // v = T q6 = Liᵀ q6 - q6
#pragma unroll
    for (int c = 0; c < 6; ++c) {
        double t = -q6[c];
#pragma unroll
        for (int r = c; r < 6; ++r) t = fma(Li[r][c], q6[r], t);
        v[c] = t;
    }
    double f0 = y;
#pragma unroll
    for (int c = 0; c < 6; ++c) f0 = fma(Qi[c], v[c], f0);
    lds_sync();  // every lane has read Ĥ before the mirror overwrites it
    if (lane < 12) {
        double* Jl = &s.ps.L[0][0];
#pragma unroll
        for (int j = 0; j < 12; j += 2) *reinterpret_cast<double2*>(&Jl[i * JMS + j]) = make_double2(J0[j], J0[j + 1]);
        s.ps.xs[i] = -f0;
    }
    lds_sync();
    return !seg_any<16>(!ok);
}

// ---------------------------------------------------------------------------------------
// General contact mask: the reference QP (cpp:466-515) reduced exactly to 12
// variables z, one 3-slot per leg (a swing leg's joint accelerations, a stance leg's force), with
// only inequality rows (the stance legs' friction faces and the 24 torque rows):
//   * a = Mb^-1 (E_S^T f - w_g) (R0, cpp:492);
//   * swing slacks: R4 / R5 (cpp:496-497, 507-515) say s_i >= |r_i|, r_i = Js_i [a; qdd] - rsw_i,
//     and s_i is in the objective only as 1/2 w s_i^2 (w = slack_weight), so s_i = |r_i| and the
//     row pair becomes the penalty 1/2 w r_i^2; a stance leg's pair is vacuous (s_i = |rsw_i|);
//   * stance equalities R1 (cpp:494, 504): Jbj_S qdd + G_S f = e_S, with Jbj = Jblk - E K, solved
//     for the stance joints by Woodbury as in stance_reduce: qdd_S = q0 + Y phi,
//     phi = K_W qdd_W - Mb^-1 E_S^T f = B z (column j of B: K_j for a swing slot, -Mb^-1 E_j^T for
//     a stance slot).
// The objective becomes 1/2 z^T H z + g^T z with H = I + P^T (I + Mb^-2) P + sum_i w_i Rho_i^T Rho_i,
// P z = E_S^T f and Rho the 12 "leg rows": a stance joint's acceleration q0_i + Y_i B z (w_i = 1)
// or a swing foot's task residual r_i = rho0_i + J_l[k] z_l + v_i B z (v_i = -S6^-T E_i^T,
// rho0_i = E_i c_psi - rsw_i, c_psi = -[0, 0, g, 0, 0, 0] - K_S q0; w_i = slack_weight).  With
// V = sum_i w_i v_i v_i^T (v_i = Y_i on stance rows), o_a = sum_i w_i own_ia v_i (own_i = J_l[k] on
// the swing leg's own slot) and blk = w J_l^T J_l (per swing leg):
//   H_aj = d_aj + blk_aj + (C_P P_a) . P_j + (V B_a + o_a) . B_j + B_a . o_j,
//   g_a  = -E_a (W + [0, 0, g / m, 0, 0, 0]) (stance) or w sum_k J_l[k][k_a] rho0_(l,k) (swing)
//          + B_a . gamma,   gamma = sum_i w_i v_i rho0_i.
// Torques: tau = t0 - Nt z, t0 = bbj + Mbj[:, S] q0, Nt[r][j] = -(Mbj[r, S] Y) . B_j + (stance j:
// Jbj[j][r]; swing j: -Mbj[r][j]).  Lane i < 12 of the robot's 16-lane segment is leg row / slot /
// joint i.  Returns false (nothing overwritten in the problem record: the caller takes the general
// 24-variable path) at a near-singular stance leg, S6 or factor; `vac` is the infeasibility of the
// swing legs' vacuous R1 rows (quirk A.12: 0 = r1).  Identical for every mask to the literal
// 42 x 70 QP (oracle/wbc_reduced.py, tests/test_oracle_reduced.py).
// ---------------------------------------------------------------------------------------
__device__ bool reduce_general([[maybe_unused]] const KernelArgs& ka, [[maybe_unused]] int rb, Prob& P,
                               const wbc_params& pr, int lane, int kap, UpdScratch& s, const St16& V, bool& vac) {
    static_assert(offsetof(UpdScratch, sr) + offsetof(decltype(UpdScratch::sr), Y) >=
                      offsetof(UpdScratch, ps) + sizeof(UpdScratch::ps), "Y / q0 survive the factorisation");
    auto& R = s.sr;
    const int i = lane < 12 ? lane : 11, l = i / 3, k = i % 3;
    const bool sti = (kap >> l) & 1;
    const double dl[3] = {P.d[3 * l], P.d[3 * l + 1], P.d[3 * l + 2]};
    const double inv_m = P.inv_m;
    const double wsw = pr.slack_weight;
    // vacuous rows: a swing leg's R1 row reads 0 = r1
    vac = seg_any<16>(lane < 12 && !sti && fabs(P.r1[i]) > 1e-9 * fmax(1.0, fabs(P.r1[i])));
    // R1: row k of J_l^-1 for a stance leg (W row i = [jr, d_l x jr], w_i = jr . e_l); swing rows 0
    bool ok;
    {
        const double* A = s.Jf[l];
        const double c00 = A[4] * A[8] - A[5] * A[7], c01 = A[5] * A[6] - A[3] * A[8], c02 = A[3] * A[7] - A[4] * A[6];
        const double det = A[0] * c00 + A[1] * c01 + A[2] * c02;
        double amx = 0.0;
#pragma unroll
        for (int t = 0; t < 9; ++t) amx = fmax(amx, fabs(A[t]));
        ok = !sti || fabs(det) > 1e-9 * amx * amx * amx;
        const double id = sti ? fast_rcp(ok ? det : 1.0) : 0.0;
        const double r0[3] = {c00, A[2] * A[7] - A[1] * A[8], A[1] * A[5] - A[2] * A[4]};
        const double r1[3] = {c01, A[0] * A[8] - A[2] * A[6], A[2] * A[3] - A[0] * A[5]};
        const double r2[3] = {c02, A[1] * A[6] - A[0] * A[7], A[0] * A[4] - A[1] * A[3]};
        double jr[3];
#pragma unroll
        for (int t = 0; t < 3; ++t) jr[t] = ((k == 0) ? r0[t] : (k == 1) ? r1[t] : r2[t]) * id;
        if (lane < 12) {
            double dxj[3];
            cross3(dl, jr, dxj);
            double wi = 0.0;
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                R.W[i][t] = jr[t];
                R.W[i][3 + t] = dxj[t];
                wi = fma(jr[t], P.r1[3 * l + t] + (t == 2 ? pr.gravity : 0.0), wi);
            }
            R.w[i] = wi;
        }
    }
    lds_sync();
    // R2: [S6 | z6] = [I - K W | K w] (42 entries in one round over 12 lanes, as stance_reduce)
    {
        const int ra = lane % 6, h = (lane / 6) & 1;
        double acc[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
        // both K entries loaded unconditionally and selected: a load under the lane-dependent
        // condition became a branch with its own LDS wait, 12 serialized round trips
        const int ra3 = ra < 3 ? ra : 0, rk3 = ra < 3 ? 0 : ra - 3;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double av = s.A[j][ra3], kv = s.KA[j][rk3];
            const double kj = (ra < 3) ? av * inv_m : kv;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c][j & 3] = fma(kj, R.W[j][3 * h + c], acc[c][j & 3]);
            acc[3][j & 3] = fma(kj, R.w[j], acc[3][j & 3]);
        }
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int cb = 3 * h + c;
                R.S[ra][cb] = (ra == cb ? 1.0 : 0.0) - ((acc[c][0] + acc[c][1]) + (acc[c][2] + acc[c][3]));
            }
            if (h) R.S[ra][6] = (acc[3][0] + acc[3][1]) + (acc[3][2] + acc[3][3]);
        }
    }
    lds_sync();
    // R3: S6^-1 by Gauss-Jordan without pivoting (S6 = I without stance legs; cond < 10 otherwise)
    // (row r of S6^-1 and z6_r stay in lane r's registers: R4 takes them by DPP broadcast)
    double ir[6], zr;
    {
        const int r = lane < 6 ? lane : 5;
        double sr_[6];
        zr = R.S[r][6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            sr_[c] = R.S[r][c];
            ir[c] = (r == c) ? 1.0 : 0.0;
        }
        const double smx = seg6_absmax(sr_);
        double pmin = 1e300;
#pragma unroll
        for (int kk = 0; kk < 6; ++kk) {
            const double pv = seg_bcast<16>(sr_[kk], kk);
            pmin = fmin(pmin, fabs(pv));
            const double ip = fast_rcp(pv);
            double prow[12];
#pragma unroll
            for (int c = kk + 1; c < 6; ++c) prow[c] = seg_bcast<16>(sr_[c], kk);
#pragma unroll
            for (int c = 0; c <= kk; ++c) prow[6 + c] = seg_bcast<16>(ir[c], kk);
            const double f = (lane == kk) ? 0.0 : sr_[kk] * ip;
            const double own = (lane == kk) ? ip : 1.0;
#pragma unroll
            for (int c = kk + 1; c < 6; ++c) sr_[c] = fma(-f, prow[c], sr_[c] * own);
#pragma unroll
            for (int c = 0; c <= kk; ++c) ir[c] = fma(-f, prow[6 + c], ir[c] * own);
        }
        ok = ok && pmin > 1e-6 * smx;
    }
    ok = !seg_any<16>(!ok);
    lds_sync();
    if (!ok) return false;
    // R4: Y_i = W_i S6^-1, q0_i = w_i + Y_i z6 (zero on swing rows); per lane: B_i, v_i, rho0_i
    double Bi[6], Ei[6];  // column i of B, E_i^T = [e_k; row k of -S(d_l)]
    double yi[6], q;      // Y_i, q0_i (kept for the torque map, R8)
    {
        double wrow[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) wrow[c] = R.W[i][c];
        q = R.w[i];
        double pkv[3];
        pk3(k, dl, pkv);
#pragma unroll
        for (int c = 0; c < 3; ++c) { Ei[c] = (c == k) ? 1.0 : 0.0; Ei[3 + c] = pkv[c]; }
        // Y_i = W_i S6^-1 and (S6^-T E_i^T)_c = sum_b S6^-1[b][c] E_i[b] in one pass over the
        // broadcast entries of S6^-1 (no LDS round trip)
        double sv[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            double a4[2] = {0.0, 0.0}, tv = 0.0;
#pragma unroll
            for (int t = 0; t < 6; ++t) {
                const double sb = seg_bcast<16>(ir[c], t);
                a4[t & 1] = fma(wrow[t], sb, a4[t & 1]);
                tv = fma(sb, Ei[t], tv);
            }
            yi[c] = a4[0] + a4[1];
            sv[c] = tv;
            q = fma(yi[c], seg_bcast<16>(zr, c), q);
        }
        double Ki[6];
#pragma unroll
        for (int c = 0; c < 3; ++c) { Ki[c] = s.A[i][c] * inv_m; Ki[3 + c] = s.KA[i][c]; }
        // c_psi = -[0, 0, g, 0, 0, 0] - sum over stance joints of K_j q0_j
        double cpsi[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) cpsi[c] = -seg_sum<16>(lane < 12 ? Ki[c] * q : 0.0) - (c == 2 ? pr.gravity : 0.0);
        double mpk[3];  // I_c^-1 (row k of -S(d_l))
        mv3(P.Icinv, pkv, mpk);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            Bi[c] = sti ? -Ei[c] * inv_m : Ki[c];
            Bi[3 + c] = sti ? -mpk[c] : Ki[3 + c];
        }
        // swing row: v_i = -S6^-T E_i^T, rho0_i = E_i c_psi - rsw_i
        double vi[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) vi[c] = sti ? yi[c] : -sv[c];
        double ec = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) ec = fma(Ei[c], cpsi[c], ec);
        const double rho = sti ? q : ec - P.rsw[i];
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 6; c += 2) {
                *reinterpret_cast<double2*>(&R.Y[i][c]) = make_double2(yi[c], yi[c + 1]);
                *reinterpret_cast<double2*>(&V.Vt[i * 6 + c]) = make_double2(vi[c], vi[c + 1]);
                *reinterpret_cast<double2*>(&V.Bt[i * 6 + c]) = make_double2(Bi[c], Bi[c + 1]);
            }
            R.q0[i] = q;
            V.rho0[i] = rho;
        }
    }
    lds_sync();
    UST(ka, rb, 20);
    // R5: [V | gamma] = sum_j w_j v_j [v_j^T | rho0_j] (42 entries in one round); slot a's o_a,
    // its blk row and its own gradient term (swing)
    {
        const int ra = lane % 6, h = (lane / 6) & 1;
        double acc[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double wj = ((kap >> (j / 3)) & 1) ? 1.0 : wsw;
            const double vj = wj * V.Vt[j * 6 + ra];
#pragma unroll
            for (int c = 0; c < 3; ++c) acc[c][j & 3] = fma(vj, V.Vt[j * 6 + 3 * h + c], acc[c][j & 3]);
            acc[3][j & 3] = fma(vj, V.rho0[j], acc[3][j & 3]);
        }
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 3; ++c) R.Q[ra][3 * h + c] = (acc[c][0] + acc[c][1]) + (acc[c][2] + acc[c][3]);
            if (h) R.Q[ra][6] = (acc[3][0] + acc[3][1]) + (acc[3][2] + acc[3][3]);
        }
    }
    double blk[3] = {0.0, 0.0, 0.0}, gown = 0.0;
    double Ci[6];  // C_a: P_a = E_a^T (stance slot) or o_a (swing slot), broadcast to the segment in R6
    {
        // o_a = w sum_r J_l[r][k] v_(l,r) (swing slot a = (l, k)); stance slot: C_a = P_a = E_a^T
        double oa[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double jrk = s.Jf[l][3 * r + k];
#pragma unroll
            for (int c = 0; c < 6; ++c) oa[c] = fma(jrk, V.Vt[(3 * l + r) * 6 + c], oa[c]);
#pragma unroll
            for (int kj = 0; kj < 3; ++kj) blk[kj] = fma(jrk, s.Jf[l][3 * r + kj], blk[kj]);
            gown = fma(jrk, V.rho0[3 * l + r], gown);
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) Ci[c] = sti ? Ei[c] : wsw * oa[c];
    }
    lds_sync();
    UST(ka, rb, 21);
    // R6: H row a = i and g_a
    double hrow[12], gsv;
    {
        double al[6], be[6];
        // alpha_a = (I + Mb^-2) P_a (stance), 0 (swing)
        {
            double t[3], t2[3];
            mv3(P.Icinv, &Ei[3], t);
            mv3(P.Icinv, t, t2);
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                al[c] = sti ? Ei[c] * (1.0 + inv_m * inv_m) : 0.0;
                al[3 + c] = sti ? Ei[3 + c] + t2[c] : 0.0;
            }
        }
        // beta_a = V B_a + o_a
#pragma unroll
        for (int c = 0; c < 6; ++c) {
            double t = sti ? 0.0 : Ci[c];
#pragma unroll
            for (int b = 0; b < 6; ++b) t = fma(R.Q[c][b], Bi[b], t);
            be[c] = t;
        }
#pragma unroll
        // B_j and C_j from lane j of the segment (DPP broadcasts: no LDS round trip per column,
        // which the register-bound schedule issued and waited for one at a time)
        for (int j = 0; j < 12; ++j) {
            const bool stj = (kap >> (j / 3)) & 1;
            double bj[6], cj[6];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                bj[c] = seg_bcast<16>(Bi[c], j);
                cj[c] = seg_bcast<16>(Ci[c], j);
            }
            double h = (i == j) ? 1.0 : 0.0;
            if (!sti && j / 3 == l) h = fma(wsw, sel3d(j % 3, blk[0], blk[1], blk[2]), h);
            double t1 = 0.0, ta = 0.0, tb = 0.0;  // both dots, one select (not one per component)
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                t1 = fma(be[c], bj[c], t1);
                ta = fma(al[c], cj[c], ta);
                tb = fma(Bi[c], cj[c], tb);
            }
            hrow[j] = h + t1 + (stj ? ta : tb);
        }
        double gam = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) gam = fma(Bi[c], R.Q[c][6], gam);
        double wv[6];
#pragma unroll
        for (int c = 0; c < 6; ++c) wv[c] = P.W[c] + (c == 2 ? pr.gravity * inv_m : 0.0);
        double ew = 0.0;
#pragma unroll
        for (int c = 0; c < 6; ++c) ew = fma(Ei[c], wv[c], ew);
        gsv = (sti ? -ew : wsw * gown) + gam;
    }
    UST(ka, rb, 22);
    // R7: H = L L^T, M = L^-1, x0 = -H^-1 g (ps.L, ps.xs: over W .. Si, all read by now)
    lds_sync();
    ok = factor12_rows(hrow, gsv, lane, &s.ps.L[0][0], s.ps.xs);
    UST(ka, rb, 23);  // R7 done (diagnostic build)
    if (!ok) return false;
    // R8: torque map row r = i, t0_r, the row's reference-space norm; then Nt over Jbj
    {
        const int r = i;
        double my[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0}, t4[2] = {0.0, 0.0}, s2 = 0.0, mrow[12];
        // Y, q0 and B from LDS (broadcast reads): kept in registers through the factorisation for
        // DPP broadcasts instead, they pushed ~250 AGPR moves into this stage
#pragma unroll
        for (int kk = 0; kk < 12; ++kk) {
            const double mk = P.Mbj[r * 12 + kk];
            const bool stk = (kap >> (kk / 3)) & 1;
            const double jcv = P.Jbj[kk * 12 + r];  // loaded, then masked (no load under the mask branch)
            const double jc = stk ? jcv : 0.0;
            mrow[kk] = stk ? jc : -mk;  // the slot's own term of Nt[r][kk]
#pragma unroll
            for (int c = 0; c < 6; ++c) my[c] = fma(mk, R.Y[kk][c], my[c]);
            t4[kk & 1] = fma(mk, R.q0[kk], t4[kk & 1]);
            s2 = fma(mk, mk, fma(jc, jc, s2));
        }
        double nt[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            double t = mrow[j];
#pragma unroll
            for (int c = 0; c < 6; ++c) t = fma(-my[c], V.Bt[j * 6 + c], t);
            nt[j] = t;
        }
        const double t0v = P.bbj[r] + (t4[0] + t4[1]);
        lds_sync();  // every lane has read Jbj / Mbj
        if (lane < 12) {
#pragma unroll
            for (int c = 0; c < 12; c += 2) *reinterpret_cast<double2*>(&V.Nt[r * 12 + c]) = make_double2(nt[c], nt[c + 1]);
            V.t0[r] = t0v;
            V.nsel[r] = s2;
        }
    }
    lds_sync();
    UST(ka, rb, 14);
    return true;
}

// ---------------------------------------------------------------------------------------
// inline stance solve: the 12-variable force-space QP of a four-contact robot whose equalities
// stance_reduce eliminated, solved by its own 16-lane segment of the update wave (four robots per
// wave) right after factor12, so that nothing of it passes through HBM.  The Goldfarb-Idnani
// method as solve_stance runs it (same selection by slack / |reference row|, ratio tests,
// Householder add, Givens drop, iteration count), but in the textbook J-form: with three of the
// 40 inequality rows per lane (lane l: friction face l, torque rows 16 + l and, for l < 8, 32 + l)
// keeping every transformed column C = J^T N up to date would cost three 12-long column updates
// per lane per step, so the segment keeps J = L^-T Q instead (row i in lane i < 12, mirrored in
// LDS for the column reads), forms d = J^T n+ and the primal direction z = J2 d2 once per step,
// and the slack rates n . z per row.  R^-1 lives in registers (lane i: row i); the primal x is
// updated with every step (no recovery pass).  Cold start only: the engine uses it for stateless
// all-stance steps.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ double seg16_min(double v) {
    v = vmin_f64(v, dpp_d<0x128>(v));
    v = vmin_f64(v, dpp_d<0x124>(v));
    v = vmin_f64(v, dpp_d<0x122>(v));
    v = vmin_f64(v, dpp_d<0x121>(v));
    return v;
}
// lane j of the caller's 16-lane segment (dynamic j; ds_bpermute, every lane of the segment active)
__device__ __forceinline__ double seg_shfl(double v, int j) { return vbcast(v, ((int)threadIdx.x & ~15) + (j & 15)); }
__device__ __forceinline__ int seg_shfl_i(int v, int j) {
    return __builtin_amdgcn_ds_bpermute((((int)threadIdx.x & ~15) + (j & 15)) << 2, v);
}

// ROWS: the J mirror already holds J0 by rows (rank6_factor); otherwise M = L^-1 (factor12).
// GEN: the general form of any contact mask (reduce_general, St16(s, P)): friction rows only for
// stance legs, the hotstart of stateful steps, the outputs mapped back through B, Y and the leg
// rows; otherwise the four-contact stance form (stateless).  qp = output row, hr = history row.
// STF: -1 stateful or not by KernelArgs::stateful at run time; 0 / 1 known at compile time (the
// default step's two instances, wbc_update_solve_kernel<STF>)
template <bool ROWS, bool GEN, int STF = -1>
__device__ void solve16(const KernelArgs& a, int rb, int qp, int l, bool wr, const Prob& P, UpdScratch& s,
                        const St16& V, int kap, int status0, double hws_lo = 0.0, double hws_hi = 0.0,
                        double hws_tag = 0.0) {
    constexpr int N = 12;
    constexpr int NTS = GEN ? 12 : NTS_ST;  // Nt row stride
    const wbc_params& pr = a.pv;
    double* Jl = &s.ps.L[0][0];  // M = L^-1 (row-major 12 x 12) on entry, then the LDS mirror of J
    const int i = l < N ? l : 0;
    int status = (P.flags != 0.0) ? WBC_QP_NUMERIC : status0;
    int iters = 0;
    lds_sync();

    // normals (force space) of the three slots, as solve_stance / build_normal
    const int fl = l >> 2, rr = l & 3, k1 = l >> 1, k2 = 8 + ((l & 7) >> 1);
    const bool v2 = l < 8;
    const bool fon = GEN ? (((kap >> fl) & 1) != 0) : true;  // friction faces exist for stance legs only
    const double sg = (l & 1) ? -1.0 : 1.0;
    double n0[N], n1[N], n2[N];
#pragma unroll
    for (int m = 0; m < N; ++m) {
        const int r = m % 3;
        const double fv = (r == 0) ? ((rr == 0) ? -1.0 : (rr == 1 ? 1.0 : 0.0))
                        : (r == 1) ? ((rr == 2) ? -1.0 : (rr == 3 ? 1.0 : 0.0)) : pr.friction;
        n0[m] = (m / 3 == fl) ? fv : 0.0;
        n1[m] = -sg * V.Nt[k1 * NTS + m];
        const double nt2 = V.Nt[k2 * NTS + m];  // (k2 is a valid row in every lane: loaded, then masked)
        n2[m] = v2 ? -sg * nt2 : 0.0;
    }
    const double bp1 = -pr.max_torque - sg * V.t0[k1], bp2 = -pr.max_torque - sg * V.t0[k2];
    const double tol0 = 1e-10;
    const double tol1 = 1e-10 * fmax(1.0, fabs(-pr.max_torque - sg * P.bbj[k1]));
    const double tol2 = 1e-10 * fmax(1.0, fabs(-pr.max_torque - sg * P.bbj[k2]));
    const double in0 = fast_rsq(fmax(1.0 + pr.friction * pr.friction, 1e-300));
    const double in1 = fast_rsq(fmax(V.nsel[k1], 1e-300)), in2 = fast_rsq(fmax(V.nsel[k2], 1e-300));
    double sp0, sp1, sp2;
    auto slacks = [&](const double* xv) {
        double q0[4] = {0.0, 0.0, 0.0, 0.0}, q1[4] = {0.0, 0.0, 0.0, 0.0}, q2[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < N; ++j) {
            q0[j & 3] += n0[j] * xv[j];
            q1[j & 3] += n1[j] * xv[j];
            q2[j & 3] += n2[j] * xv[j];
        }
        sp0 = ((q0[0] + q0[1]) + (q0[2] + q0[3])) - 0.0;
        sp1 = ((q1[0] + q1[1]) + (q1[2] + q1[3])) - bp1;
        sp2 = ((q2[0] + q2[1]) + (q2[2] + q2[3])) - bp2;
    };
    {
        double xv[N];
#pragma unroll
        for (int j = 0; j < N; ++j) xv[j] = s.ps.xs[j];
        slacks(xv);
    }
    // J = L^-T (row l of J = column l of M in lane l < 12), the primal x = x0 (x_l in lane l)
    double Jr[N];
#pragma unroll
    for (int j = 0; j < N; ++j) Jr[j] = (l < N) ? (ROWS ? Jl[i * JMS + j] : Jl[j * 12 + i]) : 0.0;
    double x = (l < N) ? s.ps.xs[i] : 0.0;
    lds_sync();  // every lane has read M before the mirror overwrites it
    auto mirror = [&]() {
        if (l < N) {
#pragma unroll
            for (int j = 0; j < N; j += 2) *reinterpret_cast<double2*>(&Jl[i * JMS + j]) = make_double2(Jr[j], Jr[j + 1]);
        }
        lds_sync();
    };
    if (!ROWS) mirror();
    UST(a, rb, 15);  // normals, slacks, J

    double rinv[N];  // row l of R^-1 (l < 12)
#pragma unroll
    for (int k = 0; k < N; ++k) rinv[k] = 0.0;
    int q = 0, pstar = -1, act = -1, ab = 0;  // ab: bit j = slot j of this lane active
    double u = 0.0, up = 0.0;
    bool done = (status != WBC_QP_OK);
    int max_wsr = pr.max_wsr;
    // held in a VGPR: left to the compiler it is re-loaded from the kernarg segment on every pass,
    // and that scalar load's wait drains the pass's outstanding LDS reads
    asm volatile("" : "+v"(max_wsr));

    // d = J^T n (lane j: dj = column j of the mirror . n), broadcast to every lane; d2 = rows >= pos;
    // r = R^-1 d (lane l < q), zn = |d2|^2, z = J2 d2 (lane k: z_k), dq = d[pos], jq = J[l][pos]
    auto dot_col = [&](const double* jc, const double* np) {
        double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < N; ++k) acc[k & 3] += jc[k] * np[k];
        return (l < N) ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.0;
    };
    // d is broadcast in its two parts, masked at the source lane (one select there instead of a mask
    // per element in every lane): d1 = rows < pos (the active part; rows of R^-1 are 0 beyond q =
    // pos anyway) and d2 = rows >= pos
    auto direction = [&](double dj, int pos, double* d2, double& rk, double& zn, double& zk, double& dq, double& jq) {
        const double dj2 = (l >= pos) ? dj : 0.0;
        const double dj1 = dj - dj2;
        double d1[N];
#pragma unroll
        for (int k = 0; k < N; ++k) {
            d1[k] = seg_bcast<16>(dj1, k);
            d2[k] = seg_bcast<16>(dj2, k);
        }
        // d[pos] and J[l][pos] (needed only by the Householder add, so their LDS latency is off
        // the chain): from lane pos of the segment and from the J mirror
        dq = seg_shfl(dj, pos);  // lane 12.. holds 0
        // loaded unconditionally from a clamped address, then masked (a load under the lane
        // condition is an exec-mask block with its own LDS wait)
        jq = (l >= N || pos >= N) ? 0.0 : Jl[i * JMS + (pos < N ? pos : 0)];
        {
            double acc[2] = {0.0, 0.0}, zz[2] = {0, 0};
#pragma unroll
            for (int j = 0; j < N; ++j) {
                acc[j & 1] += rinv[j] * d1[j];
                zz[j & 1] += d2[j] * d2[j];
            }
            rk = (l < N) ? acc[0] + acc[1] : 0.0;
            zn = zz[0] + zz[1];
        }
        {
            double acc[2] = {0.0, 0.0};
#pragma unroll
            for (int j = 0; j < N; ++j) acc[j & 1] += Jr[j] * d2[j];
            zk = acc[0] + acc[1];
        }
    };
    // Householder add at slot pos: J <- J H on columns pos.. (row l: v . J_l = z_l - alpha J_l[pos]);
    // R^-1 gains the column [-r / alpha; 1 / alpha]
    auto householder_add = [&](int pos, const double* d2, double rk, double zn, double zk, double dq, double jq) {
        const double rs = fast_rsq(zn);
        const double nrm2 = zn * rs;
        const double alpha = (dq >= 0.0) ? -nrm2 : nrm2;
        const double ia = (dq >= 0.0) ? -rs : rs;
        const double beta = fast_rcp(zn + nrm2 * fabs(dq));
        const double vw = (zk - alpha * jq) * beta, vwa = vw * alpha;
        // the unit vector e_pos, broadcast from the lanes (lane pos holds 1): one DPP move per
        // element instead of a compare + select + move per element in every lane
        const double epl = (l == pos) ? 1.0 : 0.0;
        double ep[N];
#pragma unroll
        for (int k = 0; k < N; ++k) ep[k] = seg_bcast<16>(epl, k);
#pragma unroll
        for (int k = 0; k < N; ++k) Jr[k] = fma(vwa, ep[k], fma(-vw, d2[k], Jr[k]));
        const double nv = (l == pos) ? ia : -rk * ia;
        // column pos of R^-1 is 0 before the add and nv is finite here (zn > 1e-14), so adding nv
        // under the 0 / 1 mask is exact
        const double nvw = (l <= pos) ? nv : 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) rinv[k] = fma(ep[k], nvw, rinv[k]);
    };

    // Hotstart (qpOASES SQProblem::hotstart, cpp:529-533): the previous solve's working set (row
    // ids of this numbering, tagged 16 + mask in H_WSKAP) minus the friction rows of legs that are
    // no longer in contact, re-added as a block without steps (the mirror's columns), then the
    // point where every warm row holds with equality: v = -R^-T s_A(x0), u = R^-1 v, x = x0 + J v.
    // A dependent warm row or a multiplier below -1e-10 rejects the set: cold start from x0.
    if constexpr (GEN) {
        if (!done && (STF < 0 ? a.stateful != 0 : STF == 1) && !a.cold) {
            // the previous set's words (H_WSLO, H_WSHI, H_WSKAP), loaded with the update's history
            // batch (update_phase load_hist): read here, their HBM round trip sat on the chain of
            // every stateful wave (~4 k ticks of the trot's ~7 k-tick hotstart stage)
            unsigned long long ws = (hws_tag >= 16.0) ? ((unsigned long long)(unsigned)hws_lo |
                                                         ((unsigned long long)(unsigned)hws_hi << 32))
                                                      : 0ull;
            unsigned long long keep = 0xFFFFFFull << 16;  // torque rows
#pragma unroll
            for (int lg = 0; lg < 4; ++lg)
                if ((kap >> lg) & 1) keep |= 0xFull << (4 * lg);
            ws &= keep;
            const int nw = __popcll(ws);
            // Direct check for a warm set of one or two rows (the trot's: 88 % of its QPs carry no
            // row, 12 % one, < 1 % two): the point where the rows hold, x = x0 + J0 D lambda with
            // D = J0^T N_A (the J mirror's columns still hold J0), G = D^T D, G lambda = -s_A(x0),
            // straight from the 1 x 1 / 2 x 2 system instead of Householder re-adds through the
            // mirror and 12 segment sums for R^-T s_A (~5 k ticks per stateful wave).  Accepted when
            // the rows are independent (the re-add's test), every multiplier >= -1e-10 (its
            // rejection rule) and no other row is violated at x: the set is then optimal, exactly
            // what the block below would find after its re-adds (iters 0, the same working set), so
            // the segment is done.  Anything else takes the block below unchanged.
            bool direct_ok = false, warm_pt = false, small_rej = false;
            double ua = 0.0, ub = 0.0, xw = 0.0;  // the direct point's multipliers and x (warm_pt)
            if (seg_any<16>(nw >= 1 && nw <= 2)) {
                const unsigned long long r1w = ws & (ws - 1ull);
                const int pa = __builtin_ctzll(ws | (1ull << 63)), pb = (nw == 2) ? __builtin_ctzll(r1w | (1ull << 63)) : pa;
                double jc[N];
#pragma unroll
                for (int k = 0; k < N; ++k) jc[k] = Jl[k * JMS + i];
                auto warm_row = [&](int p, double* np, double& nn) {
                    const bool frc = p < 16;
                    const int tq = p - 16;
                    const int fo = (int)(V.fric - V.Nt) + FRIC_ROW(p & 15), to = ((tq < 0 ? 0 : tq) >> 1) * NTS;
                    const double* nrow = V.Nt + (frc ? fo : to);
                    const double sgn = (frc || (tq & 1)) ? 1.0 : -1.0;
                    nn = 0.0;
#pragma unroll
                    for (int k = 0; k < N; ++k) { np[k] = sgn * nrow[k]; nn = fma(np[k], np[k], nn); }
                };
                double na[N], nb[N], nna, nnb;
                warm_row(pa, na, nna);
                warm_row(pb, nb, nnb);
                const double da = dot_col(jc, na), db = (nw == 2) ? dot_col(jc, nb) : 0.0;  // D[l][0..1]
                const double g11 = seg_sum<16>(da * da), g12 = seg_sum<16>(da * db), g22 = seg_sum<16>(db * db);
                const double s_a = seg_shfl(sel3d(pa >> 4, sp0, sp1, sp2), pa & 15);
                const double s_b = seg_shfl(sel3d(pb >> 4, sp0, sp1, sp2), pb & 15);
                double la, lb;
                bool ind;
                if (nw == 2) {
                    const double det = fma(g11, g22, -g12 * g12);
                    ind = g11 > 1e-26 * fmax(1.0, nna) && det > 1e-26 * fmax(1.0, nnb) * g11;
                    const double idt = fast_rcp(ind ? det : 1.0);
                    la = fma(s_b, g12, -s_a * g22) * idt;
                    lb = fma(s_a, g12, -s_b * g11) * idt;
                } else {
                    ind = g11 > 1e-26 * fmax(1.0, nna);
                    la = -s_a * fast_rcp(ind ? g11 : 1.0);
                    lb = 0.0;
                }
                bool ok = nw >= 1 && nw <= 2 && ind && la >= -1e-10 && lb >= -1e-10;
                // x = x0 + J0 e, e = D lambda (e_k in lane k)
                const double ek = fma(da, la, db * lb);
                double xd = 0.0;
                {
                    double a2[2] = {0.0, 0.0};
#pragma unroll
                    for (int k = 0; k < N; ++k) a2[k & 1] = fma(Jr[k], seg_bcast<16>(ek, k), a2[k & 1]);
                    xd = (l < N) ? x + (a2[0] + a2[1]) : 0.0;
                }
                const double t0s = sp0, t1s = sp1, t2s = sp2;
                {
                    double xv[N];
#pragma unroll
                    for (int j = 0; j < N; ++j) xv[j] = seg_bcast<16>(xd, j);
                    slacks(xv);
                }
                int abd = 0;
                if (l == (pa & 15)) abd |= 1 << (pa >> 4);
                if (nw == 2 && l == (pb & 15)) abd |= 1 << (pb >> 4);
                const bool viol = (fon && !(abd & 1) && sp0 < -tol0) || (!(abd & 2) && sp1 < -tol1) ||
                                  (v2 && !(abd & 4) && sp2 < -tol2);
                const bool any_viol = seg_any<16>(viol);
                direct_ok = ok && !any_viol;
                // rows violated at the warm point: the set's Householder re-adds (J and R for the loop)
                // below, but the point, its multipliers and slacks are these; a rejected set (dependent
                // rows or a multiplier < -1e-10) starts cold from x0, as the block below would after
                // its re-adds, without them
                warm_pt = ok && any_viol;
                small_rej = (nw >= 1 && nw <= 2) && !ok;
                if (direct_ok) {
                    x = xd;
                    ab = abd;
                    done = true;  // optimal: no row to add (iters 0, status OK)
                } else if (!warm_pt) {
                    sp0 = t0s; sp1 = t1s; sp2 = t2s;
                }
                ua = fmax(la, 0.0);
                ub = fmax(lb, 0.0);
                xw = xd;
            }
            if (nw > 0 && nw <= N && !direct_ok && !small_rej) {
                if (l < N) {  // J0 for a rejection
#pragma unroll
                    for (int j = 0; j < N; j += 2) *reinterpret_cast<double2*>(&V.J0[i * 12 + j]) = make_double2(Jr[j], Jr[j + 1]);
                }
                bool fail = false;
                unsigned long long rem = ws;
                for (int w = 0; w < nw; ++w) {
                    const int p = __builtin_ctzll(rem);
                    rem &= rem - 1ull;
                    const int ol = p & 15, js = p >> 4, pos = q;
                    double jc[N];
#pragma unroll
                    for (int k = 0; k < N; ++k) jc[k] = Jl[k * JMS + i];
                    // the row's normal from its id, as the loop below builds it (p numbers the rows
                    // as pstar does): a friction face from the shared table, a torque row as +-Nt;
                    // the same values lane ol holds as n0 / n1 / n2, without an LDS exchange
                    const bool frc = js == 0;
                    const int tq = frc ? 0 : p - 16;
                    const double* nrow = frc ? &V.fric[FRIC_ROW(p)] : &V.Nt[(tq >> 1) * NTS];
                    const double sgn = (frc || (tq & 1)) ? 1.0 : -1.0;
                    double np[N], nn = 0.0;
#pragma unroll
                    for (int k = 0; k < N; ++k) { np[k] = sgn * nrow[k]; nn = fma(np[k], np[k], nn); }
                    double d2[N], rk, zn, zk, dq, jq;
                    direction(dot_col(jc, np), pos, d2, rk, zn, zk, dq, jq);
                    if (!(zn > 1e-26 * fmax(1.0, nn))) { fail = true; break; }  // dependent: reject
                    householder_add(pos, d2, rk, zn, zk, dq, jq);
                    if (l == pos) act = p;
                    if (l == ol) ab |= 1 << js;
                    ++q;
                    mirror();
                }
                if (!fail && warm_pt) {  // the direct point: slots 0, 1 hold the rows in ctz order
                    if (l < q) u = (l == 0) ? ua : ub;
                    x = xw;
                } else if (!fail) {
                    // slack at x0 of the row in slot l (from its owner lane), then v, u, x
                    const int ow = act < 0 ? 0 : act & 15, jw = act < 0 ? 0 : act >> 4;
                    const double o0 = seg_shfl(sp0, ow), o1 = seg_shfl(sp1, ow), o2 = seg_shfl(sp2, ow);
                    const double sk = (l < q) ? sel3d(jw, o0, o1, o2) : 0.0;
                    double v[N];
#pragma unroll
                    for (int j = 0; j < N; ++j) v[j] = -seg_sum<16>(l < q ? rinv[j] * sk : 0.0);
                    double uu[4] = {0.0, 0.0, 0.0, 0.0}, xx[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int j = 0; j < N; ++j) {
                        uu[j & 3] = fma(rinv[j], v[j], uu[j & 3]);
                        xx[j & 3] = fma(Jr[j], v[j], xx[j & 3]);
                    }
                    const double uw = (uu[0] + uu[1]) + (uu[2] + uu[3]);
                    fail = seg_any<16>(l < q && uw < -1e-10);
                    if (!fail) {
                        if (l < q) u = fmax(uw, 0.0);
                        if (l < N) x += (xx[0] + xx[1]) + (xx[2] + xx[3]);
                        double xv[N];
#pragma unroll
                        for (int j = 0; j < N; ++j) xv[j] = seg_bcast<16>(x, j);
                        slacks(xv);
                    }
                }
                if (fail) {  // back to the cold start: J0, empty working set, x0 and its slacks
                    lds_sync();
#pragma unroll
                    for (int j = 0; j < N; ++j) Jr[j] = (l < N) ? V.J0[i * 12 + j] : 0.0;
#pragma unroll
                    for (int k = 0; k < N; ++k) rinv[k] = 0.0;
                    q = 0; act = -1; ab = 0; u = 0.0;
                    x = (l < N) ? s.ps.xs[i] : 0.0;
                    double xv[N];
#pragma unroll
                    for (int j = 0; j < N; ++j) xv[j] = s.ps.xs[j];
                    slacks(xv);
                    mirror();
                }
            }
        }
    }

    UST(a, rb, 25);  // hotstart block (stateful general form; immediate otherwise)
    // most violated row, by slack / |reference row| (ties to the lowest row); none: optimal.  Run
    // before the loop and then right after each add, where it overlaps the Householder update of J
    auto select = [&]() {
        const double w0 = (fon && !(ab & 1) && sp0 < -tol0) ? sp0 * in0 : 1e300;
        const double w1 = (!(ab & 2) && sp1 < -tol1) ? sp1 * in1 : 1e300;
        const double w2 = (v2 && !(ab & 4) && sp2 < -tol2) ? sp2 * in2 : 1e300;
        // the exact minimum, then the lowest row id within WBC_TIE_BAND of it (include/wbc.h:
        // near-ties are ties) from three ballots (friction rows 0..15 first, then 16 + l, then
        // 32 + l: the oracle's scan order)
        const double m = seg16_min(vmin_f64(w0, vmin_f64(w1, w2)));
        if (!(m < 1e299)) done = true;
        const double thr = m * (1.0 - WBC_TIE_BAND);  // m < 0 when a row is violated
        const int sh = (int)threadIdx.x & 48;
        const unsigned b0 = (unsigned)(__ballot(w0 <= thr) >> sh) & 0xFFFFu;
        const unsigned b1 = (unsigned)(__ballot(w1 <= thr) >> sh) & 0xFFFFu;
        const unsigned b2 = (unsigned)(__ballot(w2 <= thr) >> sh) & 0xFFFFu;
        // the three masks as one 49-bit word, lowest set bit first (as conditionals on b0 and b1
        // the compiler branched per segment)
        pstar = __builtin_ctzll((unsigned long long)b0 | ((unsigned long long)b1 << 16) |
                                ((unsigned long long)(b2 | 0x10000u) << 32));
        up = 0.0;
    };
    if (!done) select();

    IST_DECL;
    while (__any(!done)) {
        // column i of J from the mirror, issued first so that its LDS latency is off the chain
        double jc[N];
#pragma unroll
        for (int k = 0; k < N; ++k) jc[k] = Jl[k * JMS + i];
        {   // the working-set cap (++iters > max_wsr), as selects: branched, it cost two exec-mask
            // blocks per pass
            const bool hit = !done && iters >= max_wsr;
            iters += (done || hit) ? 0 : 1;
            status = hit ? WBC_QP_MAX_ITER : status;
            done = done || hit;
        }
        if (!done) {
            const int pos = q, ol = pstar & 15, js = pstar >> 4;
            // dj = column j of J . n for the chosen row, from the row id alone (no exchange of its
            // normal through the owner lane): a torque row is +-row of Nt, a friction face a row of
            // the workgroup's normal table (LDS, one address per segment); the slack from the owner
            // lane
            double dj;
            {
                const bool frc = pstar < 16;
                const int tq = pstar - 16;
                // the row as an offset from Nt, both candidates formed and one selected (a select
                // of the two addresses compiled to two exec-mask blocks)
                const int fo = (int)(V.fric - V.Nt) + FRIC_ROW(pstar), to = (tq >> 1) * NTS;
                const double* nrow = V.Nt + (frc ? fo : to);
                // two chains per dot in the pass (not four: the pass is issue-bound, and each
                // dot then ends in one add instead of three)
                double a2[2] = {0.0, 0.0};
#pragma unroll
                for (int k = 0; k < N; ++k) a2[k & 1] = fma(jc[k], nrow[k], a2[k & 1]);
                const double dn = a2[0] + a2[1];
                dj = ((l < N) ? ((frc || (tq & 1)) ? 1.0 : -1.0) : 0.0) * dn;
            }
            const double sps = seg_shfl(sel3d(js, sp0, sp1, sp2), ol);
            IST(0);  // the chosen row's normal
            double d2[N], rk, zn, zk, dq, jq;
            direction(dj, pos, d2, rk, zn, zk, dq, jq);
            IST(1);  // d = J^T n, R^-1 d, z
            // slack rates n . z of the lane's rows (z_m broadcast from lane m)
            double cz0, cz1, cz2;
            {
                double z0[2] = {0, 0}, z1[2] = {0, 0}, z2[2] = {0, 0};
#pragma unroll
                for (int m = 0; m < N; ++m) {
                    const double zm = seg_bcast<16>(zk, m);
                    z0[m & 1] += n0[m] * zm;
                    z1[m & 1] += n1[m] * zm;
                    z2[m & 1] += n2[m] * zm;
                }
                cz0 = z0[0] + z0[1];
                cz1 = z1[0] + z1[1];
                cz2 = z2[0] + z2[1];
            }
            IST(2);  // slack rates
            // step: t1 (drop an active slot) or t2 (the new row becomes active)
            const double vt = (l < q && rk > 1e-14) ? u * fast_rcp(rk) : 1e300;
            // the exact minimum (fmin returns one of its inputs), then its lowest lane from a
            // ballot of the lanes that hold it (one 4-step DPP chain; a 6-bit lane tag in the
            // mantissa needed a second chain to recover the exact value)
            const double t1 = seg16_min(vt);
            const double t2 = (zn > 1e-14) ? (-sps * fast_rcp(zn)) : 1e300;
            const double t = fmin(t1, t2);
            IST(3);  // step lengths
            if (!(t < 1e299)) {
                status = WBC_QP_INFEASIBLE;
                done = true;
            } else {
                const bool full = (t2 < 1e299 && t2 <= t1);
                // the primal and slack step only when the new row has a direction (t2 finite), as
                // a select: a zero step leaves them exactly as they were (branched, it cost an
                // exec-mask block per pass)
                const double ts = (t2 < 1e299) ? t : 0.0;
                sp0 += ts * cz0; sp1 += ts * cz1; sp2 += ts * cz2; x += ts * zk;
                if (l < q) u -= t * rk;
                up += t;
                if (full) {
                    if (l == q) { u = up; act = pstar; }
                    if (l == ol) ab |= 1 << js;
                    ++q;
                    select();  // the next row: slacks and active flags are final, J is not needed
                    householder_add(pos, d2, rk, zn, zk, dq, jq);
                    IST(4);  // select + Householder add
                } else {
                    // drop slot l1 (the lowest lane holding t1; only this path needs it): shift the
                    // active lists, then Givens deletion (givens_drop) with the rotation of step k
                    // from the R column of the row now in slot k: (J^T n)[k, k+1]
                    const int l1 = __builtin_ctzll((__ballot(vt == t1) >> ((int)threadIdx.x & 48)) & 0xFFFFull);
                    const int dropped = seg_shfl_i(act, l1);
                    if (l == (dropped & 15)) ab &= ~(1 << (dropped >> 4));
                    const double un = seg_shfl(u, l + 1);
                    const int an = seg_shfl_i(act, l + 1);
                    if (l >= l1 && l < q - 1) { u = un; act = an; }
                    if (l == q - 1) { u = 0.0; act = -1; }
                    --q;
#pragma unroll
                    for (int k = 0; k < N - 1; ++k) {
                        if (k >= l1 && k < q) {
                            const int pl = seg_shfl_i(act, k);
                            double nl;  // component i of row pl's normal
                            if (pl < 16) {
                                const int rp = pl & 3, r = i % 3;
                                const double fv = (r == 0) ? ((rp == 0) ? -1.0 : (rp == 1 ? 1.0 : 0.0))
                                                : (r == 1) ? ((rp == 2) ? -1.0 : (rp == 3 ? 1.0 : 0.0)) : pr.friction;
                                nl = (i / 3 == (pl >> 2)) ? fv : 0.0;
                            } else {
                                const int qt = pl - 16;
                                nl = ((qt & 1) ? 1.0 : -1.0) * V.Nt[(qt >> 1) * NTS + i];
                            }
                            const double a0 = seg_sum<16>(l < N ? Jr[k] * nl : 0.0);
                            const double b0 = seg_sum<16>(l < N ? Jr[k + 1] * nl : 0.0);
                            const double r2 = a0 * a0 + b0 * b0;
                            const double rh = (r2 > 0.0) ? fast_rsq(r2) : 0.0;
                            const double c = (r2 > 0.0) ? a0 * rh : 1.0, sn = b0 * rh;
                            double xa, ya;
                            xa = Jr[k]; ya = Jr[k + 1]; Jr[k] = fma(c, xa, sn * ya); Jr[k + 1] = fma(c, ya, -sn * xa);
                            xa = rinv[k]; ya = rinv[k + 1]; rinv[k] = fma(c, xa, sn * ya); rinv[k + 1] = fma(c, ya, -sn * xa);
                        }
                    }
                    const int src = l + ((l >= l1) ? 1 : 0);
#pragma unroll
                    for (int k = 0; k < N; ++k) {
                        const double v = seg_shfl(rinv[k], src);
                        rinv[k] = (l < q && k >= l && k < q) ? v : 0.0;
                    }
                    IST_COUNT(1);
                }
                mirror();
                IST(5);  // mirror (and the drop path)
                IST_COUNT(0);
            }
        }
    }
    IST_FLUSH(a, rb);
    UST(a, rb, 16);  // active-set loop
    UST(a, rb, 17);  // primal
    const bool ok = (status == WBC_QP_OK);
    const bool stl = GEN ? (((kap >> (i / 3)) & 1) != 0) : true;  // slot i is a stance force
    {  // tau_j = t0_j - Nt_j z (cpp:565-576), grf = f (cpp:556-563): z by DPP from its lanes (no
       // LDS round trip), the Nt row's reads issued alongside
        double zb[N];
#pragma unroll
        for (int c = 0; c < N; ++c) zb[c] = seg_bcast<16>(x, c);
        if (wr && l < N) {
            double t4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int c = 0; c < 12; ++c) t4[c & 3] = fma(V.Nt[l * NTS + c], zb[c], t4[c & 3]);
            const double tv = V.t0[l] - ((t4[0] + t4[1]) + (t4[2] + t4[3]));
            a.tau[(size_t)qp * 12 + l] = ok ? tv : 0.0;
            a.grf[(size_t)qp * 12 + l] = (ok && stl) ? x : 0.0;
        }
    }
    if (a.x) {  // the 42-vector's maps read z from LDS
        if (l < N) V.f[l] = x;
        lds_sync();
    }
    if (a.x && wr) {  // x (42, cpp:534-541): a = Mb^-1 (E_S^T f) - g e_z, qdd, f, slacks
        double F[3] = {0, 0, 0}, Mm[3] = {0, 0, 0};
#pragma unroll
        for (int ll = 0; ll < 4; ++ll) {
            const bool st = GEN ? (((kap >> ll) & 1) != 0) : true;
            const double fv[3] = {st ? V.f[3 * ll] : 0.0, st ? V.f[3 * ll + 1] : 0.0, st ? V.f[3 * ll + 2] : 0.0};
            const double dl[3] = {P.d[3 * ll], P.d[3 * ll + 1], P.d[3 * ll + 2]};
            double t[3];
            cross3(dl, fv, t);
#pragma unroll
            for (int c = 0; c < 3; ++c) { F[c] += fv[c]; Mm[c] += t[c]; }
        }
        double bf[6];  // Mb^-1 E_S^T f
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            bf[c] = F[c] * P.inv_m;
            bf[3 + c] = P.Icinv[3 * c] * Mm[0] + P.Icinv[3 * c + 1] * Mm[1] + P.Icinv[3 * c + 2] * Mm[2];
        }
        // phi = B z (general); the stance form's phi = -Mb^-1 E^T f
        double phi[6];
        if constexpr (GEN) {
#pragma unroll
            for (int c = 0; c < 6; ++c) phi[c] = 0.0;
#pragma unroll
            for (int j = 0; j < N; ++j) {
                const double zj = V.f[j];
#pragma unroll
                for (int c = 0; c < 6; ++c) phi[c] = fma(V.Bt[j * 6 + c], zj, phi[c]);
            }
        } else {
#pragma unroll
            for (int c = 0; c < 6; ++c) phi[c] = -bf[c];
        }
        if (l < 12) {
            double* xr = a.x + (size_t)qp * WBC_NV;
            if (l < 6) xr[l] = ok ? ((l < 3) ? sel3(bf, l < 3 ? l : 0) - (l == 2 ? pr.gravity : 0.0)
                                             : sel3(&bf[3], l < 3 ? 0 : l - 3)) : 0.0;
            double qv = V.q0[l];
#pragma unroll
            for (int c = 0; c < 6; ++c) qv = fma(V.Y[l * 6 + c], phi[c], qv);
            double sv = fabs(P.rsw[l]);
            if constexpr (GEN) {
                if (!stl) {  // swing: qdd_l is the variable, s = |r| of the foot's task row
                    qv = V.f[l];
                    const int lg = l / 3, kk = l % 3;
                    double r = V.rho0[l];
#pragma unroll
                    for (int c = 0; c < 3; ++c) r = fma(s.Jf[lg][3 * kk + c], V.f[3 * lg + c], r);
#pragma unroll
                    for (int c = 0; c < 6; ++c) r = fma(V.Vt[l * 6 + c], phi[c], r);
                    sv = fabs(r);
                }
            }
            xr[6 + l] = ok ? qv : 0.0;
            xr[18 + l] = (ok && stl) ? V.f[l] : 0.0;
            xr[30 + l] = ok ? sv : 0.0;
        }
    }
    if (wr && l == 0) {
        a.status[qp] = status;
        a.iters[qp] = iters;
    }
    if (GEN && (STF < 0 ? a.stateful != 0 : STF == 1) && wr) {  // working set for the next cycle's hotstart, this numbering
        const unsigned long long b0 = __ballot((ab & 1) != 0), b1 = __ballot((ab & 2) != 0), b2 = __ballot((ab & 4) != 0);
        const int sh = (int)threadIdx.x & 48;
        const unsigned long long ws = ((b0 >> sh) & 0xFFFFull) | (((b1 >> sh) & 0xFFFFull) << 16) |
                                      (((b2 >> sh) & 0xFFull) << 32);
        if (l == 0) {
            double* H = a.hist + (size_t)rb * HIST_LEN;
            H[H_WSLO] = ok ? (double)(unsigned)(ws & 0xffffffffull) : 0.0;
            H[H_WSHI] = ok ? (double)(unsigned)(ws >> 32) : 0.0;
            H[H_WSKAP] = 16.0 + (double)kap;
        }
    }
    UST(a, rb, 18);  // outputs
}

// ---------------------------------------------------------------------------------------
// update phase (≙ updateState, cpp:256-294, plus the per-cycle terms of solveQP that do not
// depend on the QP: computeDesiredWrench cpp:426-445, swing commands cpp:447-464, bounds cpp:503-515)
// ---------------------------------------------------------------------------------------
// SUB = lanes per robot (64: one robot per wave; 16 / 32: 4 / 2 robots per wave, each with its
// own scratch); lane = lane within the robot's segment; wr = false for a padding segment past the
// batch (computes a duplicate robot, writes nothing to HBM).  rb = the input / history row, kap its
// QP's contact mask (a hypothesis' mask under wbc_step_modes), qp = the output row.
// SOLVE (wbc_step_kernel16, the default wbc_step): the QP is reduced to 12 variables and solved
// here too (solve16: the four-contact stance form on stateless all-stance waves, the general form
// otherwise); returns false when the reduction was not usable (the caller writes the problem for
// the general fallback solve).  !SOLVE: the split update (Prob + Presolve records to HBM).
// the robot's 91 input doubles (pose | nu | q | ref), SUB lanes, element lane + it * SUB in v[it]
template <int SUB>
__device__ __forceinline__ void load_inputs(const KernelArgs& a, int rb, int lane, double (&v)[(91 + SUB - 1) / SUB]) {
    constexpr int NIT = (91 + SUB - 1) / SUB;
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int k = (lane + it * SUB < 91) ? lane + it * SUB : 90;
        const double* p = (k < 7) ? a.base_pose + (size_t)rb * 7 + k
                        : (k < 25) ? a.nu + (size_t)rb * 18 + (k - 7)
                        : (k < 37) ? a.qj + (size_t)rb * 12 + (k - 25)
                                   : a.ref + (size_t)rb * 54 + (k - 37);
        v[it] = *p;
    }
}

// Leg row i's two bounds under its contact flags (cpp:384-402 finite differences, 447-464 swing
// command): kr1 / ksw the row's R1 and swing masks (1 stance), ko the previous cycle's flag; one
// definition for the update and the mode loop, so both round alike
__device__ __forceinline__ void leg_bounds(double kr1, double ksw, double ko, double cur, double old, double cmd0,
                                           double rdt, bool switching, double& r1, double& rsw) {
    double jc_dot = 0.0, js_dot = 0.0;
    if (!switching) {
        jc_dot = (kr1 * cur - ko * old) * rdt;
        js_dot = ((1.0 - ksw) * cur - (1.0 - ko) * old) * rdt;
    }
    const double cmd = cmd0 * (1.0 - ksw);
    r1 = -jc_dot;
    rsw = cmd - js_dot;
}

template <int SUB, bool SOLVE = false, typename Model = wbc_model, bool MLOOP = false, int STF = -1, bool SONLY = false>
__device__ __forceinline__ bool update_phase(const KernelArgs& a, int rb, int qp, int kap, int lane, bool wr, UpdScratch& s, Prob& P,
                             Presolve* pre, const Model& md, const double* fric = nullptr,
                             const double* vin = nullptr, int chunk = 0, unsigned* fails = nullptr) {
    const wbc_params& pr = a.pv;
    const bool switching = a.switching[rb] != 0;
    const bool stateful = STF < 0 ? a.stateful != 0 : STF == 1;  // (STF: as solve16's)
    const bool debug = a.debug != 0;
    double* H = stateful ? a.hist + (size_t)rb * HIST_LEN : nullptr;
    UST(a, rb, 0);

    // inputs, one element per lane (robot-major arrays -> contiguous per wave); sin/cos per joint
    if constexpr (SUB == 64) {
        // both loads issued before either is used: lane k < 64 reads input k, lanes 0..26 also
        // read input 64 + k (all in the reference block)
        const double* p0 = (lane < 7) ? a.base_pose + (size_t)rb * 7 + lane
                         : (lane < 25) ? a.nu + (size_t)rb * 18 + (lane - 7)
                         : (lane < 37) ? a.qj + (size_t)rb * 12 + (lane - 25)
                                       : a.ref + (size_t)rb * 54 + (lane - 37);
        const bool two = lane + 64 < 91;
        const double v0 = *p0;
        const double v1 = two ? a.ref[(size_t)rb * 54 + (lane + 64 - 37)] : 0.0;

        const bool bad = !isfinite(v0) || !isfinite(v1);
        s.in[lane] = v0;
        if (two) s.in[lane + 64] = v1;
        if (lane >= 25 && lane < 37) {  // sin / cos of the joint angle this lane loaded
            double sn, cs;
            joint_sincos(v0, &sn, &cs);
            s.sc[lane - 25][0] = sn;
            s.sc[lane - 25][1] = cs;
        }
        const bool anybad = wave_any(bad);
        if (lane == 0) { P.flags = anybad ? 1.0 : 0.0; P.kappa = (double)kap; }
    } else {
        // all loads issued before any is used (addresses clamped to element 90, so every lane
        // loads); the joint angles' sin / cos come from LDS after the exchange.  vin: the caller
        // issued them already (load_inputs, before its own staging loads: one HBM round trip)
        constexpr int NIT = (91 + SUB - 1) / SUB;
        double v[NIT];
        if (vin) {
#pragma unroll
            for (int it = 0; it < NIT; ++it) v[it] = vin[it];
        } else {
            load_inputs<SUB>(a, rb, lane, v);
        }
        bool bad = false;
#pragma unroll
        for (int it = 0; it < NIT; ++it) {
            const int k = lane + it * SUB;
            if (k < 91) {
                bad = bad || !isfinite(v[it]);
                s.in[k] = v[it];
            }
        }
        const bool anybad = seg_any<SUB>(bad);
        if (lane == 0) { P.flags = anybad ? 1.0 : 0.0; P.kappa = (double)kap; }
        lds_sync();
        if (lane < 12) {
            double sn, cs;
            joint_sincos(s.in[25 + lane], &sn, &cs);
            s.sc[lane][0] = sn;
            s.sc[lane][1] = cs;
        }
    }
    lds_sync();
    UST(a, rb, 1);
    // The old history this lane reads, loaded in one batch (addresses clamped, so every lane loads
    // unconditionally).  Read where they are used, the loads sat in lane-dependent branches and
    // after history stores the compiler cannot order them against, so it issued and waited for
    // them group by group: about ten serialized memory round trips per stateful update.  The
    // stateful instance of the default step (STF = 1) issues the batch here, so that its HBM round
    // trip overlaps stages A-C; the others where the history is first used (after stage C).
    constexpr int NT = (18 + SUB - 1) / SUB;  // Tdot_inv columns per lane
    double hTd[18], hMa[NT][6], hR[3], hDo[3], hJo[12], hE = 0.0, hv = 0.0, hk = 15.0;
    double hWlo = 0.0, hWhi = 0.0, hWtag = 0.0;  // the previous working set (solve16's hotstart)
    // in two parts: the stateful default step issues them at the starts of stages B and Ic (all
    // ~55 at once, at stage A's start, stalled the wave on their issue: stage A took 6.6 k ticks
    // against 4.3 k without them, profiles/r05/hist_split/)
    auto load_hist_a = [&]() {
        const int l6 = lane < 6 ? lane : 5;
        hv = H[H_VALID];
        hk = H[H_KOLD];
        hWlo = H[H_WSLO];
        hWhi = H[H_WSHI];
        hWtag = H[H_WSKAP];
#pragma unroll
        for (int cc = 0; cc < 18; ++cc) hTd[cc] = H[H_TDINV + l6 * 18 + cc];
    };
    auto load_hist_b = [&]() {
        const int l6 = lane < 6 ? lane : 5, l12 = lane < 12 ? lane : 11;
#pragma unroll
        for (int i = 0; i < 3; ++i) hR[i] = H[H_ROLD + i];
#pragma unroll
        for (int it = 0; it < NT; ++it) {
            const int jj = lane + it * SUB - 6, j = jj < 0 ? 0 : (jj > 11 ? 11 : jj);
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) hMa[it][rr] = H[H_MAOLD + rr * 12 + j];
        }
#pragma unroll
        for (int k = 0; k < 3; ++k) hDo[k] = H[H_DOLD + 3 * (l12 / 3) + k];
#pragma unroll
        for (int j = 0; j < 12; ++j) hJo[j] = H[H_JBJOLD + l12 * 12 + j];
        hE = H[H_EINT + l6];
    };
    auto load_hist = [&]() {
        load_hist_a();
        load_hist_b();
    };
    const double* pB = &s.in[0];
    const double* vB = &s.in[7];
    const double* wB = &s.in[10];
    const double* qd = &s.in[13];
    const double* ref = &s.in[37];

    // stage A: the leg chains as prefix scans, one lane per joint: leg l, link k in lane 4 l + k
    // (k < 3) of the robot's first DPP row; lane 4 l + 3 holds the base's values, so that row_ror:1
    // hands link 0 the base as its parent.  The joint-local factors M_k = R_k^link axis_rot(q_k)
    // do not depend on the chain; the link rotations are R_0 = R_B M_0, R_1 = R_B (M_0 M_1),
    // R_2 = (R_B M_0)(M_1 M_2) (two rounds of 3x3 products instead of three in sequence), and the
    // velocities / accelerations are sums over the links above (row_ror:1 / :2 under 0/1 masks):
    //   w_k = w_B + sum_{m<=k} a_m qd_m, o_k = p_B + sum_{m<=k} rel_m, vo_k = v_B + sum_{m<=k} w_m^- x rel_m,
    //   al_k = sum_{m<=k} (w_m^- x a_m) qd_m, ao_k = sum_{m<=k} al_m^- x rel_m + w_m^- x (w_m^- x rel_m)
    // (rel_m = R_{m-1} p_m, a_m = R_{m-1} axis_m, ^- = before link m), the recursion of the
    // reference's forward kinematics at nu_dot = 0.  Lane 3 writes the base frame.
    static_assert(SUB == 16 || SUB == 64, "stage A uses the segment's first 16-lane DPP row");
    {
        const int l4 = (lane >> 2) & 3, k4 = lane & 3, kk = k4 < 3 ? k4 : 2, j = 3 * l4 + kk;
        const bool base = (k4 == 3);
        const auto& lk = md.link[l4][kk];
        const double m1 = (k4 >= 1 && !base) ? 1.0 : 0.0, m2 = (k4 >= 2 && !base) ? 1.0 : 0.0;
        auto ror1 = [](double v) { return dpp_d<0x121>(v); };
        auto ror2 = [](double v) { return dpp_d<0x122>(v); };
        double RB[9], M[9], axl[3];
        quat_R(s.in[3], s.in[4], s.in[5], s.in[6], RB);
        {
            double Rl[9];
            axis_rot(lk.axis, s.sc[j][0], s.sc[j][1], Rl);
            mm3(lk.R, Rl, M);
            mv3(lk.R, lk.axis, axl);
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) M[i] = base ? RB[i] : M[i];
        // X = (parent's M, or R_B) M: R_0 in link 0, M_0 M_1 in link 1, M_1 M_2 in link 2
        double P[9], X[9], R[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) P[i] = ror1(M[i]);
        mm3(P, M, X);
#pragma unroll
        for (int i = 0; i < 9; ++i) X[i] = base ? RB[i] : X[i];
        // R = (R_B, or X of link 0) X for links 1, 2; I X for link 0 and the base lanes (a select
        // of the left factor, not of the product: the compiler turns the latter into branches)
        const bool own = (k4 == 0 || base);
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            const double x2 = ror2(X[i]);
            P[i] = own ? ((i % 4 == 0) ? 1.0 : 0.0) : x2;
        }
        mm3(P, X, R);
        // parent rotation: rel = R_{k-1} p_k, a = R_{k-1} axis_k
        double rel[3], aj[3];
#pragma unroll
        for (int i = 0; i < 9; ++i) P[i] = ror1(R[i]);
        mv3(P, lk.p, rel);
        mv3(P, axl, aj);
        const double qdk = base ? 0.0 : qd[j];
        auto excl = [&](const double* v, double* o) {  // sum over the links above (0 for link 0)
#pragma unroll
            for (int i = 0; i < 3; ++i) o[i] = fma(m2, ror2(v[i]), m1 * ror1(v[i]));
        };
        double c3[3], wex[3], t[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) c3[i] = aj[i] * qdk;
        excl(c3, t);
#pragma unroll
        for (int i = 0; i < 3; ++i) wex[i] = wB[i] + t[i];
        double ope[3];
        excl(rel, ope);
        double tv[3], vex[3];
        cross3(wex, rel, tv);
        excl(tv, vex);
        double at[3], alx[3];
        cross3(wex, aj, at);
#pragma unroll
        for (int i = 0; i < 3; ++i) at[i] *= qdk;
        excl(at, alx);
        double ot[3], u3[3], aox[3];
        cross3(alx, rel, ot);
        cross3(wex, tv, u3);
#pragma unroll
        for (int i = 0; i < 3; ++i) ot[i] += u3[i];
        excl(ot, aox);
        if (lane < 16 && !base) {
            Frame& f = s.fr[1 + j];
#pragma unroll
            for (int i = 0; i < 9; ++i) f.R[i] = R[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const double op = pB[i] + ope[i] + rel[i];
                f.o[i] = op; f.w[i] = wex[i] + c3[i]; f.al[i] = alx[i] + at[i]; f.ao[i] = aox[i] + ot[i];
                f.vo[i] = vB[i] + vex[i] + tv[i];
                s.ja[j][i] = aj[i]; s.jo[j][i] = op;
            }
        } else if (lane == 3) {
            Frame& f = s.fr[0];
#pragma unroll
            for (int i = 0; i < 9; ++i) f.R[i] = RB[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) { f.o[i] = pB[i]; f.w[i] = wB[i]; f.al[i] = 0.0; f.ao[i] = 0.0; f.vo[i] = vB[i]; }
        }
    }
    lds_sync();

    UST(a, rb, 2);
    if constexpr (STF == 1) load_hist_a();
    // stage B: one lane per body: com, world inertia, com velocity, m a_com, I alpha + w x I w
    double c[3] = {0, 0, 0}, cd[3] = {0, 0, 0};  // CoM and its velocity (cpp:260-261)
    {
        double cb[3] = {0, 0, 0}, I[9], vc[3] = {0, 0, 0}, F[3], N[3], mb = 0.0;
        if (lane < 13) {
            const Frame& f = s.fr[lane];
            const double* com;
            const double* Il;
            if (lane == 0) { mb = md.base_mass; com = md.base_com; Il = md.base_inertia; }
            else {
                const auto& lk = md.link[(lane - 1) / 3][(lane - 1) % 3];
                mb = lk.mass; com = lk.com; Il = lk.inertia;
            }
            double R[9], o[3], w[3], al[3], ao[3], vo[3], rel[3], t[3], u[3];
#pragma unroll
            for (int i = 0; i < 9; ++i) R[i] = f.R[i];
#pragma unroll
            for (int i = 0; i < 3; ++i) { o[i] = f.o[i]; w[i] = f.w[i]; al[i] = f.al[i]; ao[i] = f.ao[i]; vo[i] = f.vo[i]; }
            mv3(R, com, rel);
#pragma unroll
            for (int i = 0; i < 3; ++i) cb[i] = o[i] + rel[i];
            rot_inertia(R, Il, I);
            cross3(w, rel, t);
            cross3(w, t, u);
            double a3[3];
            cross3(al, rel, a3);
#pragma unroll
            for (int i = 0; i < 3; ++i) { vc[i] = vo[i] + t[i]; F[i] = mb * (ao[i] + a3[i] + u[i]); }
            double Iw[3], Ia[3];
            mv3(I, w, Iw);
            mv3(I, al, Ia);
            cross3(w, Iw, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) N[i] = Ia[i] + t[i];
            if (lane >= 3 && (lane % 3) == 0) {  // SHANK bodies carry the foot frames (cpp:344-382)
                const int l = lane / 3 - 1;
                double pf[3], rf[3];
                mv3(R, md.foot[l], rf);
#pragma unroll
                for (int i = 0; i < 3; ++i) pf[i] = o[i] + rf[i];
                cross3(w, rf, t);
#pragma unroll
                for (int i = 0; i < 3; ++i) { s.pf[l][i] = pf[i]; s.vf[l][i] = vo[i] + t[i]; }
            }
        }
        lds_sync();  // every frame read before the union is overwritten
        if (lane < 13) {
            Body& bd = s.bd[lane];
#pragma unroll
            for (int i = 0; i < 3; ++i) { bd.c[i] = cb[i]; bd.F[i] = F[i]; bd.N[i] = N[i]; }
#pragma unroll
            for (int i = 0; i < 9; ++i) bd.I[i] = I[i];
        }
        // mass-weighted sums over the 13 bodies (lanes >= 13 hold mb = 0)
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            cd[i] = seg_sum<SUB>(mb * vc[i]);
            c[i] = seg_sum<SUB>(mb * cb[i]);
        }
    }
    lds_sync();
    UST(a, rb, 3);
    // foot Jacobian joint columns (getFrameFreeFloatingJacobian rows 0-2, cpp:327-341): a_k x (p_f - o_k)
    if (lane < 12) {
        const int l = lane / 3, k = lane % 3;
        double dd[3] = {s.pf[l][0] - s.jo[lane][0], s.pf[l][1] - s.jo[lane][1], s.pf[l][2] - s.jo[lane][2]}, col[3];
        cross3(s.ja[lane], dd, col);
#pragma unroll
        for (int r = 0; r < 3; ++r) s.Jf[l][3 * r + k] = col[r];
    }
    double m = md.base_mass;
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int k = 0; k < 3; ++k) m += md.link[l][k].mass;
    const double inv_m = fast_rcp(m);
#pragma unroll
    for (int i = 0; i < 3; ++i) { c[i] *= inv_m; cd[i] *= inv_m; }
    const double r[3] = {c[0] - pB[0], c[1] - pB[1], c[2] - pB[2]};
    UST(a, rb, 4);
    if constexpr (STF == 1) load_hist_b();
    double Ic[9], Icinv[9];
    {   // centroidal inertia: parallel-axis contributions of the 13 bodies, summed across lanes
        double t[6] = {0, 0, 0, 0, 0, 0};
        if (lane < 13) {
            const double mb = (lane == 0) ? md.base_mass : md.link[(lane - 1) / 3][(lane - 1) % 3].mass;
            const Body& bd = s.bd[lane];
            double d[3] = {bd.c[0] - c[0], bd.c[1] - c[1], bd.c[2] - c[2]};
            const double dd = dot3(d, d);
            t[0] = bd.I[0] + mb * (dd - d[0] * d[0]);
            t[1] = bd.I[4] + mb * (dd - d[1] * d[1]);
            t[2] = bd.I[8] + mb * (dd - d[2] * d[2]);
            t[3] = bd.I[1] - mb * d[0] * d[1];
            t[4] = bd.I[2] - mb * d[0] * d[2];
            t[5] = bd.I[5] - mb * d[1] * d[2];
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) t[k] = seg_sum<SUB>(t[k]);
        Ic[0] = t[0]; Ic[4] = t[1]; Ic[8] = t[2];
        Ic[1] = Ic[3] = t[3]; Ic[2] = Ic[6] = t[4]; Ic[5] = Ic[7] = t[5];
        inv3(Ic, Icinv);
    }
    double hb[6] = {0, 0, 0, 0, 0, 0};  // base bias: sum F ; sum (c_b - p_B) x F + N
    {
        if (lane < 13) {
            const Body& bd = s.bd[lane];
            double rb_[3] = {bd.c[0] - pB[0], bd.c[1] - pB[1], bd.c[2] - pB[2]}, t[3];
            cross3(rb_, bd.F, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) { hb[i] = bd.F[i]; hb[3 + i] = t[i] + bd.N[i]; }
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) hb[k] = seg_sum<SUB>(hb[k]);
    }
    UST(a, rb, 5);
    // stage C: per joint: centroidal momentum column (about c), leg block of M, joint bias (C nu)_j
    if (lane < 12) {
        const int j = lane, l = j / 3, k = j % 3;
        const double aj[3] = {s.ja[j][0], s.ja[j][1], s.ja[j][2]};
        const double oj[3] = {s.jo[j][0], s.jo[j][1], s.jo[j][2]};
        double Al[3] = {0, 0, 0}, Aa[3] = {0, 0, 0}, hsum[3] = {0, 0, 0}, Mrow[3] = {0, 0, 0};
        // every lane runs the three bodies of its leg, the ones above its joint weighted by 0: a
        // lane-dependent `if (kk >= k)` put each body's LDS loads in an exec-masked block with its
        // own wait
#pragma unroll
        for (int kk = 0; kk < 3; ++kk) {
            const bool below = kk >= k;
            {
                const int b = 1 + 3 * l + kk;
                const double mb = below ? md.link[l][kk].mass : 0.0;
                const double wI = below ? 1.0 : 0.0;  // the inertia and force terms
                const Body& bd = s.bd[b];
                const double cb[3] = {bd.c[0], bd.c[1], bd.c[2]};
                double rel[3] = {cb[0] - oj[0], cb[1] - oj[1], cb[2] - oj[2]}, v[3], t[3], Ia[3], fm[3];
                cross3(aj, rel, v);
                double dc[3] = {cb[0] - c[0], cb[1] - c[1], cb[2] - c[2]};
                cross3(dc, v, t);
                mv3(bd.I, aj, Ia);
                cross3(rel, bd.F, fm);
#pragma unroll
                for (int i = 0; i < 3; ++i) Ia[i] *= wI;
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    Al[i] += mb * v[i];
                    Aa[i] += mb * t[i] + Ia[i];
                    hsum[i] += wI * (fm[i] + bd.N[i]);
                }
#pragma unroll
                for (int k2 = 0; k2 < 3; ++k2) {
                    if (kk >= k2) {
                        const int j2 = 3 * l + k2;
                        const double a2[3] = {s.ja[j2][0], s.ja[j2][1], s.ja[j2][2]};
                        double rel2[3] = {cb[0] - s.jo[j2][0], cb[1] - s.jo[j2][1], cb[2] - s.jo[j2][2]}, v2[3];
                        cross3(a2, rel2, v2);
                        Mrow[k2] += mb * dot3(v, v2) + dot3(Ia, a2);
                    }
                }
            }
        }
        double KA[3];
        mv3(Icinv, Aa, KA);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            s.A[j][i] = Al[i]; s.A[j][3 + i] = Aa[i]; s.Mjj[j][i] = Mrow[i]; s.KA[j][i] = KA[i];
        }
        s.hj[j] = dot3(aj, hsum);
    }
    lds_sync();
    UST(a, rb, 6);


    // y = Tdot_inv(previous cycle) nu  (quirk A.3: nu, not T nu; one-cycle lag)
    double y[6] = {0, 0, 0, 0, 0, 0};
    bool hvalid = false;
    int kap_old = 15;
    if (stateful) {
        if constexpr (STF != 1) load_hist();
        hvalid = hv != 0.0;
        kap_old = (int)hk;
        if (hvalid) {
            double yl = 0.0;
            if (lane < 6) {
#pragma unroll
                for (int cc = 0; cc < 18; ++cc) yl += hTd[cc] * s.in[7 + cc];
            }
            if constexpr (SUB == 64) {
#pragma unroll
                for (int k = 0; k < 6; ++k) y[k] = bcast(yl, k);
            } else {
                if (lane < 6) s.yv[lane] = yl;
                lds_sync();
#pragma unroll
                for (int k = 0; k < 6; ++k) y[k] = s.yv[k];
            }
        }
    }
    // h' = C nu + M[:, 0:6] y ; M_bb = [[m I, -m S(r)], [m S(r), I_c - m S(r)^2]] ; zeta = Mbar_b^-1 Ad^T h'_b
    double hp[6], zeta[6];
    {
        double t[3], u[3], w[3], Icy[3];
        cross3(r, &y[3], t);
        cross3(r, t, u);
        mv3(Ic, &y[3], Icy);
        cross3(r, y, w);
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            hp[i] = hb[i] + m * (y[i] - t[i]);
            hp[3 + i] = hb[3 + i] + m * w[i] + Icy[i] - m * u[i];
        }
        double hca[3];
        cross3(r, hp, t);
        hca[0] = hp[3] - t[0]; hca[1] = hp[4] - t[1]; hca[2] = hp[5] - t[2];
        zeta[0] = hp[0] * inv_m; zeta[1] = hp[1] * inv_m; zeta[2] = hp[2] * inv_m;
        mv3(Icinv, hca, &zeta[3]);
    }
    {  // eulAnglesRPY (cpp:12-20): roll, pitch, yaw on lanes 0, 1, 2 in parallel (computed by
       // every lane, stored by three: no branch around the chain, so it interleaves with the rest)
        double RB[9];
        quat_R(s.in[3], s.in[4], s.in[5], s.in[6], RB);
        const double ya = (lane == 0) ? RB[7] : ((lane == 1) ? -RB[6] : RB[3]);
        const double xa = (lane == 0) ? RB[8] : ((lane == 1) ? sqrt(RB[7] * RB[7] + RB[8] * RB[8]) : RB[0]);
        const double ang = atan2_br(ya, xa);
        if (lane < 3) s.cen[CEN_POSE + 3 + lane] = ang;
    }
    if (lane == 0) {
        double* cen = s.cen;
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            cen[CEN_C + i] = c[i];
            cen[CEN_CD + i] = cd[i];
            cen[CEN_R + i] = r[i];
            cen[CEN_POSE + i] = c[i];   // currentPose_ = [c; eulAnglesRPY(R)] (cpp:262-264)
            cen[CEN_VC + i] = cd[i];    // centerOfMassVelocity_ = [c_dot; omega_B] (cpp:261, quirk A.4)
            cen[CEN_VC + 3 + i] = wB[i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) cen[CEN_HB + i] = hp[i];
        P.m = m; P.inv_m = inv_m;
#pragma unroll
        for (int i = 0; i < 9; ++i) { P.Ic[i] = Ic[i]; P.Icinv[i] = Icinv[i]; }
    }
    UST(a, rb, 7);
    // finite differences over dt = 1 / loop_rate (cpp:394): times loop_rate instead of divided by
    // dt (an IEEE division is ~10 dependent instructions; the two agree to an ulp)
    const double rdt = pr.loop_rate;

    if constexpr (SUB == 64) {  // the fused kernel (2 waves per SIMD): stores in the loops (no spills)
      if (lane < 12) {
        const int j = lane, lj = j / 3, kj = j % 3;
        const double Alj[3] = {s.A[j][0], s.A[j][1], s.A[j][2]}, Aaj[3] = {s.A[j][3], s.A[j][4], s.A[j][5]};
        const double KAj[3] = {s.KA[j][0], s.KA[j][1], s.KA[j][2]};
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            double d[3] = {s.pf[l][0] - c[0], s.pf[l][1] - c[1], s.pf[l][2] - c[2]}, t[3];
            cross3(d, KAj, t);
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                const double jf = (l == lj) ? s.Jf[l][3 * rr + kj] : 0.0;
                P.Jbj[(3 * l + rr) * 12 + j] = jf - Alj[rr] * inv_m + t[rr];
            }
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            double Mij = (i / 3 == lj) ? s.Mjj[j][i % 3] : 0.0;
            Mij -= (s.A[i][0] * Alj[0] + s.A[i][1] * Alj[1] + s.A[i][2] * Alj[2]) * inv_m;
            Mij -= s.A[i][3] * KAj[0] + s.A[i][4] * KAj[1] + s.A[i][5] * KAj[2];
            P.Mbj[i * 12 + j] = Mij;
        }
        double t[3];
        cross3(r, Alj, t);
        const double hpj = s.hj[j] + dot3(Alj, y) + (t[0] + Aaj[0]) * y[3] + (t[1] + Aaj[1]) * y[4] + (t[2] + Aaj[2]) * y[5];
        P.bbj[j] = hpj - (dot3(Alj, zeta) + dot3(Aaj, &zeta[3]));
        P.d[j] = s.pf[lj][kj] - sel3(c, kj);
      }
    } else
    // lane = joint column j: Jbar joint column, Mbar_j column, bbar_j.  The lane's own values are
    // loaded unconditionally and the stage's stores come after its loads: a load under a
    // lane-dependent condition became an exec-masked block with its own LDS wait, and a store
    // between loads kept the compiler from moving the later loads up (~50 LDS waits before)
    if (lane < 12) {
        const int j = lane, lj = j / 3, kj = j % 3;
        const double Alj[3] = {s.A[j][0], s.A[j][1], s.A[j][2]}, Aaj[3] = {s.A[j][3], s.A[j][4], s.A[j][5]};
        const double KAj[3] = {s.KA[j][0], s.KA[j][1], s.KA[j][2]};
        const double mjr[3] = {s.Mjj[j][0], s.Mjj[j][1], s.Mjj[j][2]};
        const double jfo[3] = {s.Jf[lj][kj], s.Jf[lj][3 + kj], s.Jf[lj][6 + kj]};  // own leg's column
        double jb[12];
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            double d[3] = {s.pf[l][0] - c[0], s.pf[l][1] - c[1], s.pf[l][2] - c[2]}, t[3];
            cross3(d, KAj, t);
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) jb[3 * l + rr] = ((l == lj) ? jfo[rr] : 0.0) - Alj[rr] * inv_m + t[rr];
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) P.Jbj[i * 12 + j] = jb[i];  // (before the M-bar loads: its live range ends)
        double mcol[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            double Mij = (i / 3 == lj) ? mjr[i % 3] : 0.0;
            Mij -= (s.A[i][0] * Alj[0] + s.A[i][1] * Alj[1] + s.A[i][2] * Alj[2]) * inv_m;
            Mij -= s.A[i][3] * KAj[0] + s.A[i][4] * KAj[1] + s.A[i][5] * KAj[2];
            mcol[i] = Mij;
        }
        double t[3];
        cross3(r, Alj, t);
        const double hpj = s.hj[j] + dot3(Alj, y) + (t[0] + Aaj[0]) * y[3] + (t[1] + Aaj[1]) * y[4] + (t[2] + Aaj[2]) * y[5];
        const double dj = s.pf[lj][kj] - sel3(c, kj);
#pragma unroll
        for (int i = 0; i < 12; ++i) P.Mbj[i * 12 + j] = mcol[i];
        P.bbj[j] = hpj - (dot3(Alj, zeta) + dot3(Aaj, &zeta[3]));
        P.d[j] = dj;
    }
    UST(a, rb, 8);
    // T_top = [Ad^-1(r), Mbar_b^-1 A_j]; Tdot_inv for the next cycle (cpp:291-293)
    double tcol[NT][6];
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
        for (int q = 0; q < 6; ++q) tcol[it][q] = 0.0;
    if (stateful) {
        double dr[3] = {0, 0, 0};
        if (!switching) {
#pragma unroll
            for (int i = 0; i < 3; ++i) dr[i] = (r[i] - hR[i]) * rdt;
        }
#pragma unroll
        for (int it = 0; it < NT; ++it) {
        const int ln = lane + it * SUB;
        // this lane's joint column (clamped, so every lane loads: the loads are not left inside the
        // lane-dependent branch below, where each waited for its own LDS round trip)
        const int jc = ln < 6 ? 0 : (ln > 17 ? 11 : ln - 6);
        double Aj[3], KAj[3];
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) { Aj[rr] = s.A[jc][rr]; KAj[rr] = s.KA[jc][rr]; }
        if (ln >= 3 && ln < 6) {  // lin rows, cols 3..5: S(dr)
            const int cc = ln - 3;
            double e[3] = {cc == 0 ? 1.0 : 0.0, cc == 1 ? 1.0 : 0.0, cc == 2 ? 1.0 : 0.0};
            cross3(dr, e, tcol[it]);
        } else if (ln >= 6 && ln < 18) {
            double Tj[6];
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                Tj[rr] = switching ? 0.0 : (Aj[rr] * inv_m - hMa[it][rr]) * rdt;
                Tj[3 + rr] = switching ? 0.0 : (KAj[rr] - hMa[it][3 + rr]) * rdt;
            }
            double t1[3], t2[3];
            cross3(dr, KAj, t1);
            cross3(r, &Tj[3], t2);
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                tcol[it][rr] = -(t1[rr] + Tj[rr] + t2[rr]);
                tcol[it][3 + rr] = -Tj[3 + rr];
            }
        }
        }
    }
    stateful ? wsync() : lds_sync();  // all reads of the old history done
    if (stateful && wr) {
#pragma unroll
        for (int it = 0; it < NT; ++it) {
            const int ln = lane + it * SUB;
            if (ln < 18) {
#pragma unroll
                for (int rr = 0; rr < 6; ++rr) H[H_TDINV + rr * 18 + ln] = tcol[it][rr];
            }
        }
        if (lane < 12) {
            const int j = lane;
#pragma unroll
            for (int rr = 0; rr < 3; ++rr) {
                H[H_MAOLD + rr * 12 + j] = s.A[j][rr] * inv_m;
                H[H_MAOLD + (3 + rr) * 12 + j] = s.KA[j][rr];
            }
        }
    }
    UST(a, rb, 9);
    // finite-difference bounds (cpp:384-402, 503-515); swing commands (cpp:447-464).  Leg row i's
    // terms stay in lane i for the mode loop, which re-masks them per hypothesis
    double lb_cur = 0.0, lb_old = 0.0, lb_ko = 1.0, lb_cmd = 0.0;
    if (lane < 12) {
        const int i = lane, l = i / 3, rr = i % 3;
        const double d[3] = {P.d[3 * l], P.d[3 * l + 1], P.d[3 * l + 2]};
        const double w3[3] = {s.cen[CEN_VC + 3], s.cen[CEN_VC + 4], s.cen[CEN_VC + 5]};
        double wxd[3];
        cross3(w3, d, wxd);
        double cur = s.cen[CEN_VC + rr] + sel3(wxd, rr);
#pragma unroll
        for (int j = 0; j < 12; ++j) cur += P.Jbj[i * 12 + j] * qd[j];
        double old = 0.0;
        if (stateful && hvalid) {
            const double dol[3] = {hDo[0], hDo[1], hDo[2]};
            double wxo[3];
            cross3(w3, dol, wxo);
            old = s.cen[CEN_VC + rr] + sel3(wxo, rr);
#pragma unroll
            for (int j = 0; j < 12; ++j) old += hJo[j] * qd[j];
        }
        // mode hypotheses (a.modes > 0, stateless): both bounds unmasked, the R1 bound as for a stance
        // leg and the swing bound as for a swing leg; the solve kernel masks them per hypothesis
        // (each is read only for legs of its own kind, so the masked values are bit-identical)
        const double kn = (kap >> l) & 1, ko = (kap_old >> l) & 1;
        const bool unmasked = a.modes && !SOLVE;  // the split update of mode hypotheses
        const double kr1 = unmasked ? 1.0 : kn, ksw = unmasked ? 0.0 : kn;
        const double cmd0 = ref[42 + i] + pr.kd_swing * (ref[30 + i] - s.vf[l][rr]) + pr.kp_swing * (ref[18 + i] - s.pf[l][rr]);
        leg_bounds(kr1, ksw, ko, cur, old, cmd0, rdt, switching, P.r1[i], P.rsw[i]);
        lb_cur = cur; lb_old = old; lb_ko = ko; lb_cmd = cmd0;
    }
    // desired wrench (cpp:426-445); integralError_ update after use (cpp:442)
    if (lane < 6) {
        const int k = lane;
        const double kp = (k == 2) ? pr.kp_z : pr.kp;
        const double eint = (stateful && hvalid) ? hE : 0.0;
        double mba;
        if (k < 3) mba = m * ref[12 + k];
        else mba = P.Ic[3 * (k - 3)] * ref[15] + P.Ic[3 * (k - 3) + 1] * ref[16] + P.Ic[3 * (k - 3) + 2] * ref[17];
        const double e = s.cen[CEN_POSE + k] - ref[k];
        P.W[k] = -kp * e - pr.kd * (s.cen[CEN_VC + k] - ref[6 + k]) - pr.ki * eint +
                 (k == 2 ? md.total_mass * pr.gravity : 0.0) + mba;
        if (stateful && wr) H[H_EINT + k] = eint + e * fast_rcp(pr.loop_rate);
    }
    // the default step's stateful instance only needs the LDS (P.Jbj) here: every read of the old
    // history finished at the first barrier above, and these stores do not overlap the ones just
    // issued, so waiting for those to complete (a full barrier's vmcnt(0)) only put a write round
    // trip on the chain
    (stateful && STF != 1) ? wsync() : lds_sync();
    if (stateful && wr) {
        for (int k = lane; k < 144; k += SUB) H[H_JBJOLD + k] = P.Jbj[k];
        if (lane < 12) H[H_DOLD + lane] = P.d[lane];
        if (lane < 3) H[H_ROLD + lane] = s.cen[CEN_R + lane];
        if (lane == 0) { H[H_KOLD] = (double)kap; H[H_VALID] = 1.0; }
    }
    UST(a, rb, 10);
    if (debug && wr) {
        double* D = a.dbg + (size_t)rb * WBC_DBG_LEN;
        if (lane < 3) {
            D[WBC_DBG_COM + lane] = s.cen[CEN_C + lane];
            D[WBC_DBG_COMVEL + lane] = s.cen[CEN_CD + lane];
        }
        if (lane < 6) {
            D[WBC_DBG_POSE + lane] = s.cen[CEN_POSE + lane];
            D[WBC_DBG_VC + lane] = s.cen[CEN_VC + lane];
            D[WBC_DBG_WRENCH + lane] = P.W[lane];
            const double* h6 = &s.cen[CEN_HB];
            double t[3];
            cross3(r, h6, t);
            D[WBC_DBG_BBAR + lane] = (lane < 3) ? h6[lane] : h6[lane] - sel3(t, lane - 3);  // Ad^T h'_b
        }
        auto Sr = [&](int aa, int bb) -> double {  // S(r) entry
            if (aa == bb) return 0.0;
            if (aa == 0) return bb == 1 ? -r[2] : r[1];
            if (aa == 1) return bb == 0 ? r[2] : -r[0];
            return bb == 0 ? -r[1] : r[0];
        };
        for (int e = lane; e < 324; e += SUB) {
            const int i = e / 18, j = e % 18;
            double v;
            if (i < 6 && j < 6) {
                if (i < 3 && j < 3) v = (i == j) ? m : 0.0;
                else if (i < 3) v = -m * Sr(i, j - 3);
                else if (j < 3) v = m * Sr(i - 3, j);
                else {
                    const int ii = i - 3, jj = j - 3;
                    v = P.Ic[3 * ii + jj] - m * (Sr(ii, 0) * Sr(0, jj) + Sr(ii, 1) * Sr(1, jj) + Sr(ii, 2) * Sr(2, jj));
                }
            } else if (i < 6 || j < 6) {
                const int bi = (i < 6) ? i : j, jj = (i < 6) ? j - 6 : i - 6;
                if (bi < 3) v = s.A[jj][bi];
                else {
                    double t[3];
                    cross3(r, s.A[jj], t);
                    v = sel3(t, bi - 3) + s.A[jj][bi];
                }
            } else {
                const int ji = i - 6, jj = j - 6;
                v = (ji / 3 == jj / 3) ? s.Mjj[ji][jj % 3] : 0.0;
            }
            D[WBC_DBG_M + e] = v;
        }
        for (int ln = lane; ln < 18; ln += SUB) {
            // register selects (a pointer select into hb[] would put hb in scratch memory)
            double v6 = hb[0];
#pragma unroll
            for (int k = 1; k < 6; ++k) v6 = (ln == k) ? hb[k] : v6;
            D[WBC_DBG_CNU + ln] = (ln < 6) ? v6 : s.hj[ln - 6];
        }
        for (int e = lane; e < 216; e += SUB) {
            const int i = e / 18, j = e % 18, l = i / 3, rr = i % 3;
            double v, vb;
            if (j < 3) {
                v = vb = (rr == j) ? 1.0 : 0.0;
            } else if (j < 6) {  // -S(p) e = e x p, row rr
                const double pfB[3] = {s.pf[l][0] - pB[0], s.pf[l][1] - pB[1], s.pf[l][2] - pB[2]};
                const double dl[3] = {P.d[3 * l], P.d[3 * l + 1], P.d[3 * l + 2]};
                double e3[3] = {j == 3 ? 1.0 : 0.0, j == 4 ? 1.0 : 0.0, j == 5 ? 1.0 : 0.0}, t[3], t2[3];
                cross3(e3, pfB, t);
                cross3(e3, dl, t2);
                v = sel3(t, rr);
                vb = sel3(t2, rr);
            } else {
                v = ((j - 6) / 3 == l) ? s.Jf[l][3 * rr + (j - 6) % 3] : 0.0;
                vb = P.Jbj[i * 12 + (j - 6)];
            }
            D[WBC_DBG_JFEET + e] = v;
            D[WBC_DBG_JBAR + e] = vb;
        }
        if (lane < 12) {
            D[WBC_DBG_PFEET + lane] = s.pf[lane / 3][lane % 3];
            D[WBC_DBG_VFEET + lane] = s.vf[lane / 3][lane % 3];
            D[WBC_DBG_R1 + lane] = P.r1[lane];
            D[WBC_DBG_RSW + lane] = P.rsw[lane];
            D[WBC_DBG_BBAR + 6 + lane] = P.bbj[lane];
        }
        for (int ln = lane; ln < 36; ln += SUB) {
            const int i = ln / 6, j = ln % 6;
            double v = 0.0;
            if (i < 3 && j < 3) v = (i == j) ? m : 0.0;
            else if (i >= 3 && j >= 3) v = P.Ic[3 * (i - 3) + (j - 3)];
            D[WBC_DBG_MBARB + ln] = v;
        }
        for (int e = lane; e < 144; e += SUB) D[WBC_DBG_MBARJ + e] = P.Mbj[e];
    }
    lds_sync();
    // the slot factorisation of the solve's start, here where the robot's own contact mask is
    // known: in the update kernel four robots share a wave, so this 12-lane work costs a quarter
    // of its one-robot-per-wave price.  Four-contact stance eliminates its equalities first
    // (stance_reduce) and factors the force-space Hessian instead.  Under mode hypotheses the
    // masks differ per QP: the stance elimination is formed for every state (the bounds are
    // written unmasked, i.e. as for stance legs, which is exactly the kappa = 15 hypothesis) and
    // the other hypotheses factor their slot Hessian in the solve.
    if constexpr (SOLVE && MLOOP) {
        // mode hypotheses, a.mloop of them per wave (wbc_modes_kernel): the state's update above once,
        // then each hypothesis of the wave's chunk reduced and solved in turn, as the per-QP step
        // below does it.  The reductions overwrite the update's P.Jbj (the general form's torque
        // map) and Jf | A | KA (the stance form's Nt, the exchange column): 288 doubles, 18 per lane,
        // kept in registers and restored before each later hypothesis (a copy through L2 instead
        // was 9.4 MB written per step at configs[4]'s shard).  Everything else they read
        // (the rest of P, the friction table) they leave alone.  A hypothesis whose reduction is not
        // usable writes its problem to work row qp and sets bit it of *fails (the caller drains them)
        static_assert(SUB == 16, "the inline solve runs in 16-lane segments");
        const int K = a.modes, M = a.mloop;
        double* flat = &s.Jf[0][0];
        static_assert(offsetof(UpdScratch, A) == offsetof(UpdScratch, Jf) + sizeof(UpdScratch::Jf) &&
                      offsetof(UpdScratch, KA) == offsetof(UpdScratch, A) + sizeof(UpdScratch::A) &&
                      sizeof(UpdScratch::Jf) + sizeof(UpdScratch::A) + sizeof(UpdScratch::KA) == 144 * sizeof(double),
                      "Jf | A | KA: one 144-double block");
        double kj[9], ks[9];
#pragma unroll
        for (int j = 0; j < 9; ++j) {
            kj[j] = P.Jbj[lane + 16 * j];
            ks[j] = flat[lane + 16 * j];
        }
        unsigned fl = 0;
        for (int it = 0; it < M; ++it) {
            const int k = a.mode_order[chunk * M + it];
            const int km = a.mode_masks[k] & 15;
            // the lane and row laundered per hypothesis: left loop-invariant, every address and
            // constant the reductions derive from them was hoisted out of the loop and held across it
            // (~180 spill instructions)
            int ln = lane, rw = rb;
            asm volatile("" : "+v"(ln), "+v"(rw));
            const int lane = ln, rb = rw;
            const int q = rb * K + k;
            lds_sync();  // the previous hypothesis is done with the problem and the scratch
            if (it > 0) {
#pragma unroll
                for (int j = 0; j < 9; ++j) {
                    P.Jbj[lane + 16 * j] = kj[j];
                    flat[lane + 16 * j] = ks[j];
                }
            }
            if (lane < 12) {
                const double kn = (km >> (lane / 3)) & 1;
                leg_bounds(kn, kn, lb_ko, lb_cur, lb_old, lb_cmd, rdt, switching, P.r1[lane], P.rsw[lane]);
            }
            if (lane == 0) P.kappa = (double)km;
            lds_sync();
            bool ok;
            if (km == 15) {  // stateless mask 15: the four-contact stance form
                double hrow[12], gsv = 0.0;
                ok = stance_reduce<true>(a, rb, P, pr, lane, wr, s, hrow, gsv, nullptr) && rank6_factor(P, s, gsv, lane);
                if (ok) solve16<true, false, STF>(a, rb, q, lane, wr, P, s, St16(s, fric), 15, WBC_QP_OK);
            } else {
                const St16 V(s, P, fric);
                bool vac = false;
                ok = reduce_general(a, rb, P, pr, lane, km, s, V, vac);
                if (ok) solve16<true, true, STF>(a, rb, q, lane, wr, P, s, V, km, vac ? WBC_QP_INFEASIBLE : WBC_QP_OK,
                                                 hWlo, hWhi, hWtag);
            }
            if (!ok && wr) {  // as wbc_update_solve_kernel's fallback record
                lds_sync();
                const double2* src = reinterpret_cast<const double2*>(&P);
                double* wrow = a.work + (size_t)q * WORK_LEN;
                double2* dst = reinterpret_cast<double2*>(wrow);
                for (int e = lane; e < PROB_LEN / 2; e += SUB) dst[e] = src[e];
                if (lane == 0) {
                    Presolve* pw = reinterpret_cast<Presolve*>(wrow + PROB_LEN);
                    pw->presolved = 0.0;
                    pw->stance = 0.0;
                }
                fl |= 1u << it;
            }
        }
        *fails = fl;
        return true;
    } else if constexpr (SOLVE) {
        static_assert(SUB == 16, "the inline solve runs in 16-lane segments");
        // a stateless QP of mask 15: the four-contact stance form (stance_reduce + the rank-6
        // factor, no Hessian to factor); every other QP: the general form (its own mask, a hotstart
        // on stateful steps).  The choice is the segment's own, so a QP's result never depends on
        // its wave-mates; the wave map (KernelArgs::qmap) gives every wave one mask, so the branch
        // does not diverge (a mixed wave, from unmapped device-bound masks, runs both forms)
        // SONLY (wbc_stance_step_kernel: a stateless step whose masks are all 15, which the host
        // knows): the stance form only, the general form compiled out
        if (SONLY || (!stateful && kap == 15)) {
            double hrow[12], gsv = 0.0;
            if (stance_reduce<true>(a, rb, P, pr, lane, wr, s, hrow, gsv, nullptr) && rank6_factor(P, s, gsv, lane)) {
                UST(a, rb, 11);
                solve16<true, false, STF>(a, rb, qp, lane, wr, P, s, St16(s, fric), 15, WBC_QP_OK);
                return true;
            }
            return false;
        }
        if constexpr (SONLY) return false;
        const St16 V(s, P, fric);
        bool vac = false;
        if (reduce_general(a, rb, P, pr, lane, kap, s, V, vac)) {
            UST(a, rb, 11);
            solve16<true, true, STF>(a, rb, qp, lane, wr, P, s, V, kap, vac ? WBC_QP_INFEASIBLE : WBC_QP_OK, hWlo, hWhi,
                                     hWtag);
            return true;
        }
        return false;
    }
    if (pre) {
        double hrow[12], gsv = 0.0;
        bool stance = false;
        if constexpr (SUB == 16) {
            if (a.elim && (kap == 15 || a.modes))
                stance = stance_reduce<false>(a, rb, P, pr, lane, wr, s, hrow, gsv, pre);
        }
        const bool fact = stance || !a.modes;
        if (fact) {
            if (!stance) slot_hessian_row(P, kap, pr, lane, hrow, gsv);
            const bool ok = factor12<SUB>(hrow, gsv, lane, s.ps.L, s.ps.ild, s.ps.xs, &a, rb);
            const double (&Mi)[12][12] = *reinterpret_cast<const double(*)[12][12]>(&s.ps.L[0][0]);
            if (wr) {
                for (int k = lane; k < 78; k += SUB) {
                    const int i = (int)((sqrt(8.0 * k + 1.0) - 1.0) * 0.5);
                    pre->Mi[k] = Mi[i][k - i * (i + 1) / 2];
                }
                if (lane < 12) pre->xs[lane] = s.ps.xs[lane];
            }
            if (lane == 0 && !ok && !a.modes) P.flags += 2.0;
            stance = stance && ok;  // (ok is uniform over the segment) modes: the kappa = 15 hypothesis factors H_s itself
        }
        if (lane == 0 && wr) {
            pre->presolved = (fact && !stance) ? 1.0 : 0.0;
            pre->stance = stance ? 1.0 : 0.0;
        }
        lds_sync();
        UST(a, rb, 11);  // slot 19; slots 20.. belong to the solve (EST)
        return stance;
    }
    UST(a, rb, 11);  // slot 19; slots 20.. belong to the solve (EST)
    return false;
}

// ---------------------------------------------------------------------------------------
// solve phase: reduced QP (24 variables), Goldfarb-Idnani, one constraint per lane
// ---------------------------------------------------------------------------------------
struct QpMap {
    int kap, ns, nsw, neq, nfr, ntq, m;
};

__device__ __forceinline__ QpMap make_map(int kap) {
    QpMap q;
    q.kap = kap & 15;
    q.ns = __builtin_popcount(q.kap);
    q.nsw = 4 - q.ns;
    q.neq = 3 * q.ns;
    q.nfr = 4 * q.ns;
    q.ntq = 24;
    q.m = q.neq + q.nfr + q.ntq + 6 * q.nsw;
    return q;
}
// index of the idx-th leg whose contact bit equals `want`
__device__ __forceinline__ int nth_leg(int kap, int idx, int want) {
    int cnt = 0, leg = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        if ((((kap >> l) & 1) == want)) {
            if (cnt == idx) leg = l;
            ++cnt;
        }
    }
    return leg;
}

// Normal n (24) and bound b of constraint p, as n^T y >= b (equalities: n^T y = b).
// y = [qdd (12); slot l = f_l (stance) or s_l (swing), l = 0..3].
// Branch-free over the constraint types (lanes hold different types, and divergent branches
// would make the wave execute every type's code): each type's contribution is computed on every
// lane and scaled by a per-lane 0 / +-1 factor (exact in fp64).
//   R1  stance rows       Jc_j qdd + Jc_com a = r1, a = Mbar_b^-1 (Jc^T f - gw)    (cpp:494,504)
//   R2  friction pyramid  -D_rr f_l >= 0                                          (cpp:404-424)
//   R3  torque limits     +-(Mbar_j qdd - Jc_j^T f) >= -tau_max -+ bbar_j          (cpp:495,506,513)
//   R4/R5 swing rows      +-(Js_j qdd + Js_com a) + s >= +-c'                     (cpp:496-497,507-515)
__device__ void build_normal(const Prob& P, const double (*G)[12], const QpMap& mp, const wbc_params& pr, int p,
                             double* n, double& b, bool& is_eq, double& nsel, double& tolv) {
    const int kap = mp.kap;
    const int t_fr = mp.neq, t_tq = mp.neq + mp.nfr, t_sw = t_tq + mp.ntq;
    const bool in = p < mp.m;
    const bool eq = in && p < t_fr;
    const bool fr = in && p >= t_fr && p < t_tq;
    const bool tq = in && p >= t_tq && p < t_sw;
    const bool sw = in && p >= t_sw;
    // per type: leg l, component k / friction face rr, row i, sign
    int l = 0, k = 0, rr = 0;
    double sg = 1.0;
    if (eq) { l = nth_leg(kap, p / 3, 1); k = p % 3; }
    if (fr) { const int q = p - t_fr; l = nth_leg(kap, q / 4, 1); rr = q % 4; }
    if (tq) { const int q = p - t_tq; k = q / 2; sg = (q & 1) ? -1.0 : 1.0; }
    if (sw) { const int q = p - t_sw; l = nth_leg(kap, q / 6, 0); k = (q % 6) / 2; sg = (q & 1) ? -1.0 : 1.0; }
    const int i = tq ? k : 3 * l + k;  // Jbj / Mbj row (torque: joint index)
    // qdd part: +-Jbj row i (R1, R4/R5) or +-Mbj row i (R3)
    const double* row = (tq ? P.Mbj : P.Jbj) + i * 12;
    const double sq = (eq ? 1.0 : 0.0) + ((tq || sw) ? sg : 0.0);
#pragma unroll
    for (int j = 0; j < 12; ++j) n[j] = sq * row[j];
    // slot part on stance slots: the coupling through a (R1, R4/R5: row 3 l + k of G, set up with
    // the slot Hessian) and -+ Jbj[3 mm + r][i] (R3); friction faces and swing slacks are unit rows
    const double scp = eq ? 1.0 : (sw ? sg : 0.0);
    const double stq = tq ? -sg : 0.0;
    const double* grow = G[3 * l + k];
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
        const bool st = (kap >> mm) & 1;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            double x = st ? fma(scp, grow[3 * mm + r], stq * P.Jbj[(3 * mm + r) * 12 + i]) : 0.0;
            // friction face rr of stance leg l: (-1 | 1 | 0, 0 | 0 | -1 | 1, mu)
            const double fv = (r == 0) ? ((rr == 0) ? -1.0 : (rr == 1 ? 1.0 : 0.0))
                            : (r == 1) ? ((rr == 2) ? -1.0 : (rr == 3 ? 1.0 : 0.0)) : pr.friction;
            if (fr && mm == l) x = fv;
            if (sw && mm == l && r == k) x = 1.0;  // the slack of swing leg l
            n[12 + 3 * mm + r] = x;
        }
    }
    const double g0 = pr.gravity;
    const double bj = P.bbj[tq ? k : 0];
    b = 0.0;
    if (eq) b = P.r1[i] + (k == 2 ? g0 : 0.0);
    if (tq) b = (sg > 0) ? (-pr.max_torque - bj) : (-pr.max_torque + bj);
    if (sw) b = sg * (P.rsw[i] + (k == 2 ? g0 : 0.0));
    is_eq = eq;
    // Selection scale and violation tolerance of the reference's own row (the 42-variable row of A
    // at cpp:492-515 that this reduced row restates, split two-sided as qpOASES' lbA / ubA): the
    // most violated constraint is chosen by slack / |row| in that space, as the oracle's dense
    // active set does, so both visit the same working sets and count the same iterations
    // (nWSR, cpp:517).  The slack itself is the same number in both spaces.
    //   R2 friction face: |(+-1, 0, -mu)|^2 = 1 + mu^2
    //   R3 torque row j:  |Mbar_j row j|^2 + sum over stance rows r of Jbar_c,j[r][j]^2
    //   R4/R5 swing row i = 3 l + k: |[e_k, -S(d_l) row k]|^2 + |Jbar_j row i|^2 + 1 (the slack)
    double s2 = 0.0;
    if (tq) {
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double mr = P.Mbj[i * 12 + j];
            const double jc = ((kap >> (j / 3)) & 1) ? P.Jbj[j * 12 + i] : 0.0;
            s2 = fma(mr, mr, fma(jc, jc, s2));
        }
    } else {
#pragma unroll
        for (int j = 0; j < 12; ++j) s2 = fma(row[j], row[j], s2);
        const double dl2 = P.d[3 * l] * P.d[3 * l] + P.d[3 * l + 1] * P.d[3 * l + 1] + P.d[3 * l + 2] * P.d[3 * l + 2];
        const double dk = P.d[3 * l + k];
        s2 += 2.0 + dl2 - dk * dk;
    }
    nsel = fr ? 1.0 + pr.friction * pr.friction : s2;
    const double bref = (sw && k == 2) ? b - sg * g0 : b;  // the reference row's own bound
    tolv = 1e-10 * fmax(1.0, fabs(bref));
}

// C0[:, p] = J0^T n_p with J0 = blkdiag(I12, L^-T), in place: qdd part n, slot part L^-1 n_slot
__device__ __forceinline__ void to_column(QpScratch& s, double* cc) {
    double t[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {  // slot part L^-1 n_s = M n_s (M read as a broadcast)
        double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k <= i; ++k) a4[k & 3] += s.Mi()[i][k] * cc[12 + k];
        t[i] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    }
#pragma unroll
    for (int i = 0; i < 12; ++i) cc[12 + i] = t[i];
}

// d = C[:, p] broadcast from lane p (uniform, v_readlane)
template <int N>
__device__ __forceinline__ void read_column(const double* cc, int p, double* d) {
#pragma unroll
    for (int k = 0; k < N; ++k) d[k] = vbcast(cc[k], p);  // ds_bpermute: 100.5 -> 95.4 us vs v_readlane (profiles/r01/variants_loop_bperm.log)
}
template <class S>
__device__ __forceinline__ void zero_rinv(S& s) {
    double2* r = &s.Rv[0][0];
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < (S::N / 2) * S::N; k += 64)
        if (k + lane < (S::N / 2) * S::N) r[k + lane] = make_double2(0.0, 0.0);
}
// r = R^-1 d (lane i < q holds r_i; rows >= q and columns >= q of R^-1 are zero)
template <class S>
__device__ __forceinline__ double rinv_times_d(const S& s, const double* d) {
    const int lane = lane_id();
    const int i = lane < S::N ? lane : 0;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // independent chains
#pragma unroll
    for (int jj = 0; jj < S::N / 2; ++jj) {
        const double2 v = s.Rv[jj][i];
        acc[(2 * jj) & 3] += v.x * d[2 * jj];
        acc[(2 * jj + 1) & 3] += v.y * d[2 * jj + 1];
    }
    return lane < S::N ? (acc[0] + acc[1]) + (acc[2] + acc[3]) : 0.0;
}
// add the constraint with column d at position q: Householder on rows q..23 of every C column
// (v = d with rows < q zeroed on entry, the Householder vector on exit; dq = d[q]); R^-1 gains the column [-r / alpha; 1 / alpha]
__device__ __forceinline__ double householder(int q, bool add, double zn, double dq, double* v, double* cc) {
    if (!add) { zn = 1.0; dq = 0.0; }  // no-op update: vw = 0 below leaves cc bit-identical
    const double rs = fast_rsq(zn);
    const double nrm2 = zn * rs;
    const double alpha = (dq >= 0.0) ? -nrm2 : nrm2;
    const double ia = (dq >= 0.0) ? -rs : rs;  // 1 / alpha
    const double beta = fast_rcp(zn + nrm2 * fabs(dq));
    const double vq = dq - alpha;
#pragma unroll
    for (int k = 0; k < NQ; ++k) v[k] = (k == q) ? vq : v[k];  // in place: d2 -> Householder vector
    double vp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < NQ; ++k) vp[k & 3] += v[k] * cc[k];
    const double vw = add ? ((vp[0] + vp[1]) + (vp[2] + vp[3])) * beta : 0.0;
#pragma unroll
    for (int k = 0; k < NQ; ++k) cc[k] -= vw * v[k];
    return ia;
}
template <class S>
__device__ __forceinline__ void store_rinv_column(S& s, int q, bool add, double ia, double rk) {
    const int lane = lane_id();
    if (add && lane <= q) {
        double* col = reinterpret_cast<double*>(&s.Rv[q >> 1][lane]) + (q & 1);
        *col = (lane == q) ? ia : -rk * ia;
    }
}
template <class S>
__device__ __forceinline__ void add_column(S& s, int q, bool add, double zn, double dq, double rk,
                                           double* v, double* cc) {
    store_rinv_column(s, q, add, householder(q, add, zn, dq, v, cc), rk);
}
// The same reflection without forming v: v = d2 - alpha e_q, so v^T c = cz - alpha c[q] and
// c -= vw v is c -= vw d2 plus vw alpha at row q.  d2 (the column masked to rows >= q), cz = c^T d2
// and cq = c[q] come in precomputed with fp64 0 / 1 row masks (one multiply or FMA per row instead
// of a two-instruction v_cndmask select per row for every dynamic-position insert and extract).
template <int N>
__device__ __forceinline__ double householder_masked(int q, bool add, double zn, double dq, double cz, double cq,
                                                     const double* d2, double* cc) {
    if (!add) { zn = 1.0; dq = 0.0; }
    const double rs = fast_rsq(zn);
    const double nrm2 = zn * rs;
    const double alpha = (dq >= 0.0) ? -nrm2 : nrm2;
    const double ia = (dq >= 0.0) ? -rs : rs;
    const double beta = fast_rcp(zn + nrm2 * fabs(dq));
    const double vw = add ? (cz - alpha * cq) * beta : 0.0;
    const double vwa = vw * alpha;
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const double ok = (k == q) ? 1.0 : 0.0;
        cc[k] = fma(vwa, ok, fma(-vw, d2[k], cc[k]));
    }
    return ia;
}

// Delete active slot l (Goldfarb-Idnani constraint drop, after the active lists were shifted and q
// decremented): slots l..q-1 now hold the old slots l+1..q, whose R columns (in the lanes act[k])
// have one sub-diagonal entry each.  Givens rotations G_k on rows (k, k+1), k = l..q-1, restore the
// triangle; they apply to every lane's column (J <- J G^T keeps C = J^T N consistent) and to the
// columns of R^-1, and the new R^-1 is R^-1 G^T without row l and column q (rows of the old inverse
// shift up by one).  Row and column loops are unrolled with wave-uniform guards, so every register
// index is static.
template <class S>
__device__ void givens_drop(S& s, int l, int q, int act, double* cc) {
    const int lane = lane_id();
    const int i = lane < S::N ? lane : 0;
    double rr[S::N];  // row i of R^-1
#pragma unroll
    for (int jj = 0; jj < S::N / 2; ++jj) {
        const double2 v = s.Rv[jj][i];
        rr[2 * jj] = v.x;
        rr[2 * jj + 1] = v.y;
    }
#pragma unroll
    for (int k = 0; k < S::N - 1; ++k) {
        if (k >= l && k < q) {
            const int pl = bcast_i(act, k);
            const double a0 = bcast(cc[k], pl), b0 = bcast(cc[k + 1], pl);
            const double r2 = a0 * a0 + b0 * b0;
            const double rh = (r2 > 0.0) ? fast_rsq(r2) : 0.0;
            const double c = (r2 > 0.0) ? a0 * rh : 1.0, sn = b0 * rh;
            const double x = cc[k], y = cc[k + 1];
            cc[k] = fma(c, x, sn * y);
            cc[k + 1] = fma(c, y, -sn * x);
            const double ra = rr[k], rb2 = rr[k + 1];
            rr[k] = fma(c, ra, sn * rb2);
            rr[k + 1] = fma(c, rb2, -sn * ra);
        }
    }
    // rows >= l take the next row; the triangle below the diagonal, row >= q and column >= q are 0
    const int src = lane + ((lane >= l) ? 1 : 0);
#pragma unroll
    for (int k = 0; k < S::N; ++k) {
        const double v = __shfl(rr[k], src & 63);
        rr[k] = (lane < q && k >= lane && k < q) ? v : 0.0;
    }
    if (lane < S::N) {
#pragma unroll
        for (int jj = 0; jj < S::N / 2; ++jj) s.Rv[jj][lane] = make_double2(rr[2 * jj], rr[2 * jj + 1]);
    }
}

// Multipliers and slacks of the point where every active constraint (slots 0..q-1, constraint
// act of slot lane) holds with equality, from the slacks sp0 at the unconstrained optimum x0:
// R^T v = -s_A (v_i = -column i of R^-1 . s_A), u = R^-1 v, s = sp0 + C[0:q]^T v.  This is the state
// the dual method reaches by adding those constraints with full steps (used by the hotstart).
template <class S>
__device__ void active_set_point(const S& s, int q, int act, double sp0, const double* cc, double& u,
                                 double& sp) {
    const int lane = lane_id();
    const int i = lane < S::N ? lane : 0;
    double a4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < S::N; ++j) {
        if (j < q) {
            const int aj = bcast_i(act, j);
            const double sa = bcast(sp0, aj < 0 ? 0 : aj);
            const double2 r = s.Rv[i >> 1][j];  // R^-1 (j, i)
            a4[j & 3] += ((i & 1) ? r.y : r.x) * sa;
        }
    }
    const double v = (lane < q) ? -((a4[0] + a4[1]) + (a4[2] + a4[3])) : 0.0;
    double u4[4] = {0.0, 0.0, 0.0, 0.0}, s4[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < S::N; ++j) {
        if (j < q) {
            const double vj = bcast(v, j);
            const double2 r = s.Rv[j >> 1][i];  // R^-1 (i, j)
            u4[j & 3] += ((j & 1) ? r.y : r.x) * vj;
            s4[j & 3] += cc[j] * vj;
        }
    }
    if (lane < q) u = (u4[0] + u4[1]) + (u4[2] + u4[3]);
    sp = sp0 + ((s4[0] + s4[1]) + (s4[2] + s4[3]));
}

// The Presolve record in registers: packed entry `lane` in v0 and 64 + lane in v1, loaded at the
// solve kernel's start so that its HBM round trip overlaps the problem copy
struct PreRegs {
    double v0, v1;
};
constexpr int PRE_FLAG = 90;  // packed index of Presolve::presolved
static_assert(offsetof(Presolve, presolved) == PRE_FLAG * sizeof(double), "PRE_FLAG");
static_assert(offsetof(Presolve, xs) == 78 * sizeof(double), "Presolve packing");

__device__ void solve_phase(const KernelArgs& a, int rb, const Prob& P, const PreRegs* pf, QpScratch& s) {
    const wbc_params& pr = a.pv;
    const int lane = lane_id();
    const int kap = (int)P.kappa;
    const QpMap mp = make_map(kap);
    int status = WBC_QP_OK;
    int iters = 0;
    if (P.flags != 0.0) status = WBC_QP_NUMERIC;
    {   // vacuous rows (quirk A.12): swing-leg rows of R1 read 0 = r1
        bool bad = false;
        if (lane < 12 && !((kap >> (lane / 3)) & 1)) bad = fabs(P.r1[lane]) > 1e-9 * fmax(1.0, fabs(P.r1[lane]));
        if (wave_any(bad) && status == WBC_QP_OK) status = WBC_QP_INFEASIBLE;
    }

    // slot coupling rows; the slot factor M = L^-1 and x0 come from the update (packed into the
    // problem) unless the contact mask is this QP's own (mode hypotheses): then formed here
    if (lane < 12) {
        double grow[12];
        g_row(P, lane, grow);
#pragma unroll
        for (int j = 0; j < 12; j += 2) *reinterpret_cast<double2*>(&s.G[lane][j]) = make_double2(grow[j], grow[j + 1]);
    }
    if (pf && bcast(pf->v1, PRE_FLAG - 64) != 0.0) {
        // unpack: packed p < 78 is M(i, j), p = i (i + 1) / 2 + j; 78..89 are xs
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int p = lane + 64 * h;
            const double v = h ? pf->v1 : pf->v0;
            if (p < 78) {
                const int i = (int)((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
                s.Mi()[i][p - i * (i + 1) / 2] = v;
            } else if (p < 90) {
                s.xs[p - 78] = v;
            }
        }
        for (int k = lane; k < 144; k += 64) {
            const int i = k / 12, j = k % 12;
            if (j > i) s.Mi()[i][j] = 0.0;
        }
    } else if (!presolve<64>(P, kap, pr, lane, s.L, s.ild, s.xs) && status == WBC_QP_OK) {
        status = WBC_QP_NUMERIC;
    }
    lds_sync();

    STAMP(a, rb, 2);
    double cc[NQ];
    double bp = 0.0, sp = 0.0, nn = 1.0, inrm = 1.0;  // |n_p|^2 (reduced), 1 / |row p| (reference space)
    double tolv = 0.0;  // violation tolerance of row p
    double sp0 = 0.0;  // slack at the unconstrained optimum x0
    bool is_eq = false, active = false;
    const bool is_con = lane < mp.m;
    {
        EST(a, rb, 5);
        double nsel;
        build_normal(P, s.G, mp, pr, lane, cc, bp, is_eq, nsel, tolv);
        EST(a, rb, 6);
        double np[4] = {0.0, 0.0, 0.0, 0.0}, sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NQ; ++k) np[k & 3] += cc[k] * cc[k];
#pragma unroll
        for (int k = 0; k < 12; ++k) sq[k & 3] += cc[12 + k] * s.xs[k];
        nn = (np[0] + np[1]) + (np[2] + np[3]);
        const double sx = (sq[0] + sq[1]) + (sq[2] + sq[3]);
        inrm = 1.0 / sqrt(fmax(nsel, 1e-300));  // selection by slack / |row| (the oracle's scale)
        sp = sx - bp;
        EST(a, rb, 7);
        to_column(s, cc);
        EST(a, rb, 8);
        sp0 = sp;
        if (lane < C0_LANES) {
#pragma unroll
            for (int k = 0; k < NQ; k += 2) s.c0[k / 2][lane] = make_double2(cc[k], cc[k + 1]);
        }
    }

    zero_rinv(s);
    lds_sync();
    STAMP(a, rb, 3);
    // Goldfarb-Idnani (wave-uniform control flow).  After a drop the loop re-adds the remaining
    // active set (rebuild mode) through the same add path, then resumes the pending constraint.
    int q = 0;         // active set size
    double u = 0.0;    // multiplier of active slot `lane`
    int act = -1;      // constraint id of active slot `lane`
    int neq_added = 0; // equalities occupy slots 0..neq_added-1
    int pstar = -1;
    int rbk = -1;      // rebuild cursor (>= 0 while re-adding active slot rbk)
    double up = 0.0;
    const double tiny = 1e-26;
    bool done = (status != WBC_QP_OK);

    // Equality block (R1 rows, lanes 0..neq-1).  The dual method adds the
    // equalities first with full steps; their result is the equality-constrained optimum, which
    // is computed here in one pass: Householder QR of the equality columns (column broadcast
    // through LDS), then R^-T v = -s_E, u = R^-1 v and s += C^T [v; 0] in closed form.
    // Redundant equalities (|d2| ~ 0) are skipped and must be consistent, as in the loop.
    EST(a, rb, 0);
    if (!done && mp.neq > 0) {
        int myslot = -1;
        bool redundant = false;
        int e0 = 0;
        // fast path, fully unrolled: while no equality has been redundant, equality e goes to slot
        // q = e, so every row mask below is a compile-time constant.
        // tn = |cc[e:]|^2, the tail norm of the lane's own column: lane e's is |d2|^2, so the
        // reflector scalars start while the column itself is being broadcast (v_readlane).  The
        // reflection keeps |cc[e:]|, so the next tail is tn - cc[e]^2 (one FMA instead of a 24 - e
        // term sum); when that cancels (below 2^-10 of tn) on a lane that can still be a pivot, the
        // tails are summed afresh.
        // rinv: row `lane` of R^-1, built column by column alongside the reflections
        // (R^-1 gains [-R^-1 r_e / alpha_e; 1 / alpha_e], r_e = rows < e of column e, final before
        // step e): an independent chain that overlaps the reflections' latency and replaces the
        // two 12-step substitutions after the block
        double rinv[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) rinv[k] = 0.0;
        double tn;
        {
            double zp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < NQ; ++k) zp[k & 3] += cc[k] * cc[k];
            tn = (zp[0] + zp[1]) + (zp[2] + zp[3]);
        }
#pragma unroll
        for (int e = 0; e < 12; ++e) {
            if (e < mp.neq && q == e) {
                const double zn = bcast(tn, e);
                double d[NQ];
#pragma unroll
                for (int k = 0; k < NQ; ++k) d[k] = (k >= e) ? bcast(cc[k], e) : 0.0;
                const bool add = !(zn <= tiny * fmax(1.0, bcast(nn, e)));
                // Householder reflection on rows e..23 (static q = e)
                {
                    const double dq = d[e];
                    const double zs = add ? zn : 1.0, dqs = add ? dq : 0.0;
                    const double rs = fast_rsq(zs);
                    const double nrm2 = zs * rs;
                    const double alpha = (dqs >= 0.0) ? -nrm2 : nrm2;
                    const double beta = fast_rcp(zs + nrm2 * fabs(dqs));
                    {
                        const double ia = (dqs >= 0.0) ? -rs : rs;  // 1 / alpha
                        double rk[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int k = 0; k < e; ++k) rk[k & 3] = fma(rinv[k], bcast(cc[k], e), rk[k & 3]);
                        rinv[e] = (lane == e) ? ia : -((rk[0] + rk[1]) + (rk[2] + rk[3])) * ia;
                    }
                    d[e] = dqs - alpha;
                    double vp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                    for (int k = e; k < NQ; ++k) vp[k & 3] += d[k] * cc[k];
                    const double vw = add ? ((vp[0] + vp[1]) + (vp[2] + vp[3])) * beta : 0.0;
#pragma unroll
                    for (int k = e; k < NQ; ++k) cc[k] -= vw * d[k];
                }
                if (e + 1 < 12) {
                    const double tr = fma(-cc[e], cc[e], tn);
                    if (wave_any(lane > e && lane < mp.neq && !(tr >= 0x1p-10 * tn))) {
                        double zp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                        for (int k = e + 1; k < NQ; ++k) zp[k & 3] += cc[k] * cc[k];
                        tn = (zp[0] + zp[1]) + (zp[2] + zp[3]);
                    } else {
                        tn = tr;
                    }
                }
                if (add) {
                    if (lane == e) { act = e; myslot = e; }
                    ++q;
                } else if (lane == e) {
                    redundant = true;
                }
                e0 = e + 1;
            }
        }
        EST(a, rb, 1);
        // general path (after a redundant equality): dynamic slot q
#pragma unroll 1
        for (int e = e0; e < mp.neq; ++e) {
            if (lane == e) {
#pragma unroll
                for (int k = 0; k < NQ; ++k) s.colbuf[k] = cc[k];
            }
            lds_sync();
            double d[NQ];
#pragma unroll
            for (int k = 0; k < NQ; ++k) d[k] = s.colbuf[k];
            double dq = 0.0, zp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < NQ; ++k) {
                dq = (k == q) ? d[k] : dq;
                d[k] = (k >= q) ? d[k] : 0.0;
                zp[k & 3] += d[k] * d[k];
            }
            const double zn = (zp[0] + zp[1]) + (zp[2] + zp[3]);
            const bool add = !(zn <= tiny * fmax(1.0, bcast(nn, e)));
            householder(q, add, zn, dq, d, cc);
            if (add) {
                if (lane == q) act = e;
                if (lane == e) myslot = q;
                ++q;
            } else if (lane == e) {
                redundant = true;
            }
            lds_sync();  // colbuf is rewritten next
        }
        neq_added = q;
        EST(a, rb, 2);
        if (!wave_any(redundant)) {
            // every equality went to slot = lane in the fast path: R^-1 rows are in rinv.
            // v = -R^-T s_E (uniform): v_j = -sum_k R^-1[k][j] s_k over the slots k < q (lanes
            // 0..11, one DPP row), u = R^-1 v, s += C[0:q]^T v
            double v[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) v[j] = -row0_sum((lane < q) ? rinv[j] * sp : 0.0);
            double uu[4] = {0.0, 0.0, 0.0, 0.0}, ds[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                uu[j & 3] = fma(rinv[j], v[j], uu[j & 3]);
                ds[j & 3] = fma(cc[j], v[j], ds[j & 3]);
            }
            if (lane < q) {
                u = (uu[0] + uu[1]) + (uu[2] + uu[3]);
#pragma unroll
                for (int jj = 0; jj < 6; ++jj) s.Rv[jj][lane] = make_double2(rinv[2 * jj], rinv[2 * jj + 1]);
            }
            sp += (ds[0] + ds[1]) + (ds[2] + ds[3]);
            lds_sync();
        } else {
        // R columns and equality slacks by slot
        if (myslot >= 0) {
#pragma unroll
            for (int k = 0; k < 12; ++k) s.Rm[myslot][k] = cc[k];
            s.colbuf[myslot] = sp;
        }
        lds_sync();
        // forward substitutions with R^T: v = -R^-T s_E (uniform) and, in lane i, row i of R^-1
        double v[12], y[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            double av[4] = {0.0, 0.0, 0.0, 0.0}, ay[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < j; ++k) {
                const double r = s.Rm[j][k];
                av[k & 3] += r * v[k];
                ay[k & 3] += r * y[k];
            }
            const bool in = j < q;
            const double ird = fast_rcp(in ? s.Rm[j][j] : 1.0);
            const double sj = in ? s.colbuf[j] : 0.0;
            v[j] = in ? (-sj - ((av[0] + av[1]) + (av[2] + av[3]))) * ird : 0.0;
            y[j] = in ? (((lane == j) ? 1.0 : 0.0) - ((ay[0] + ay[1]) + (ay[2] + ay[3]))) * ird : 0.0;
        }
        EST(a, rb, 3);
        double uu[4] = {0.0, 0.0, 0.0, 0.0}, ds[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            uu[j & 3] += y[j] * v[j];
            ds[j & 3] += cc[j] * v[j];
        }
        if (lane < q) {
            u = (uu[0] + uu[1]) + (uu[2] + uu[3]);
#pragma unroll
            for (int jj = 0; jj < 6; ++jj) s.Rv[jj][lane] = make_double2(y[2 * jj], y[2 * jj + 1]);
        }
        sp += (ds[0] + ds[1]) + (ds[2] + ds[3]);
        const bool bad = redundant && !(fabs(sp) <= 1e-9 * fmax(1.0, fabs(bp)));
        if (wave_any(bad)) { status = WBC_QP_INFEASIBLE; done = true; }
        lds_sync();
        }
    }
    EST(a, rb, 4);

    // Hotstart (qpOASES SQProblem::hotstart, cpp:523-535): in stateful mode, the inequalities that
    // were active at the end of the previous solve (same contact mask) are re-added as a block
    // (the loop's rebuild mode), then multipliers and slacks are set in closed form.  If any
    // re-added multiplier comes out negative, the warm set is dropped and the solve restarts
    // from the equality-constrained point, as a cold solve would.
    double* Hh = a.stateful ? a.hist + (size_t)rb * HIST_LEN : nullptr;
    int warm_phase = 0;  // 1: re-adding the warm set, 2: re-adding the equalities after rejecting it
    bool warm_fail = false;
    if (!done && Hh && !a.cold) {
        const unsigned long long ws = (unsigned long long)(unsigned)Hh[H_WSLO] |
                                      ((unsigned long long)(unsigned)Hh[H_WSHI] << 32);
        unsigned long long wm = ((int)Hh[H_WSKAP] == kap) ? ws : 0ull;
        wm &= ~((1ull << mp.neq) - 1ull);                        // inequalities only
        wm &= (mp.m >= 64) ? ~0ull : ((1ull << mp.m) - 1ull);
        const int nw = __popcll(wm);
        if (nw > 0 && neq_added + nw <= NQ) {
            const bool mine = (wm >> lane) & 1ull;
            const int slot = neq_added + __popcll(wm & ((1ull << lane) - 1ull));
            if (mine) s.colbuf[slot] = (double)lane;
            lds_sync();
            if (lane >= neq_added && lane < neq_added + nw) act = (int)s.colbuf[lane];
            if (mine) active = true;
            lds_sync();
            rbk = neq_added;
            q = neq_added + nw;
            warm_phase = 1;
        }
    }
    IST_DECL;
    const int max_wsr = pr.max_wsr;

    while (!done) {
        // compiler barrier: LDS reads of the problem (build_normal / to_column on the rare drop
        // path) stay inside the loop instead of being hoisted into registers for its whole length
        asm volatile("" ::: "memory");
        if (rbk >= q) {  // rebuild finished
            rbk = -1;
            if (warm_phase) {
                active_set_point(s, q, act, sp0, cc, u, sp);
                const bool neg = lane >= neq_added && lane < q && u < -1e-10;
                if (warm_phase == 1 && (warm_fail || wave_any(neg))) {
                    // reject the warm set: back to the equality slots, rebuilt from C0
                    const int pl = lane < C0_LANES ? lane : 0;
#pragma unroll
                    for (int k = 0; k < NQ; k += 2) {
                        const double2 c = s.c0[k / 2][pl];
                        cc[k] = lane < C0_LANES ? c.x : 0.0;
                        cc[k + 1] = lane < C0_LANES ? c.y : 0.0;
                    }
                    zero_rinv(s);
                    lds_sync();
                    if (lane >= neq_added) { act = -1; u = 0.0; }
                    if (!is_eq) active = false;
                    q = neq_added;
                    rbk = 0;
                    warm_phase = 2;
                    continue;
                }
                if (lane >= neq_added && lane < q && u < 0.0) u = 0.0;
                warm_phase = 0;
            }
        }
        const bool rebuild = rbk >= 0;
        int col, pos;
        if (rebuild) {
            col = bcast_i(act, rbk);
            pos = rbk;
        } else {
            if (pstar < 0) {  // most violated inequality (equalities are all active already)
                double v = 1e300;
                if (is_con && !is_eq && !active && sp < -tolv) v = sp * inrm;
                double vm;
                const int idx = wave_select_band(v, vm);
                if (!(vm < 1e299)) break;  // no violated constraint: optimal
                pstar = idx;
                up = 0.0;
            }
            if (++iters > max_wsr) { status = WBC_QP_MAX_ITER; iters = max_wsr; break; }
            col = pstar;
            pos = q;
        }
        IST(0);  // selection
        IST_COUNT(0);  // loop passes that reach the column broadcast (adds, drops, rebuild re-adds)
        double d[NQ];
        read_column<NQ>(cc, col, d);
        IST(1);  // column broadcast
        const double rk = rinv_times_d(s, d);
        // d2 = rows >= pos of d, cq = this lane's c[pos] (fp64 0 / 1 row masks, uniform)
        double czp[4] = {0.0, 0.0, 0.0, 0.0}, cqp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NQ; ++k) {
            const double mk = (k >= pos) ? 1.0 : 0.0, ok = (k == pos) ? 1.0 : 0.0;
            d[k] *= mk;
            czp[k & 3] += cc[k] * d[k];
            cqp[k & 3] += cc[k] * ok;
        }
        const double cz = (czp[0] + czp[1]) + (czp[2] + czp[3]);  // (C2^T d2)_p = n_p^T z
        const double cq = (cqp[0] + cqp[1]) + (cqp[2] + cqp[3]);  // exact: one non-zero term
        const double zn = bcast(cz, col);                   // |d2|^2: lane col holds d itself
        const double dq = bcast(cq, col);                   // d[pos]
        IST(2);  // R^-1 d, n^T z, |z|^2

        // step (skipped in rebuild mode: the active set is re-added as is)
        bool add = true, drop = false;
        int drop_slot = -1;
        if (rebuild && warm_phase == 1 && !(zn > tiny * fmax(1.0, bcast(nn, col)))) {
            add = false;  // a warm constraint dependent on the others: reject the warm set
            warm_fail = true;
            ++rbk;
        }
        if (!rebuild) {
            const double sps = bcast(sp, pstar);
            // partial step: keep active inequality multipliers >= 0
            double t1;
            int l1;
            {
                // an r_k at rounding level next to the largest |r| is no drop candidate (WBC_R_REL,
                // include/wbc.h; the C oracle's literal form applies the same rule)
                const double rthr = fmax(1e-14, WBC_R_REL * wave_absmax(lane < q ? rk : 0.0));
                double v = 1e300;
                if (lane < q && lane >= neq_added && rk > rthr) v = u * fast_rcp(rk);
                l1 = wave_argmin_lane(v);
                t1 = bcast(v, l1);
            }
            {
                // full step only along a direction the oracle also takes (zn = n^T z > 1e-14)
                const double t2 = (zn > 1e-14) ? (-sps * fast_rcp(zn)) : 1e300;
                const double t = fmin(t1, t2);
                if (!(t < 1e299)) { status = WBC_QP_INFEASIBLE; break; }
                const bool full = (t2 < 1e299 && t2 <= t1);
                if (t2 < 1e299) sp += t * cz;
                if (lane < q) u -= t * rk;
                up += t;
                if (!full) {
                    IST_COUNT(1);  // drops
                    add = false;
                    drop = true;
                    drop_slot = l1;
                    // drop active slot l1: shift the active list
                    const int dropped = bcast_i(act, l1);
                    if (lane == dropped) active = false;
                    const double un = __shfl(u, (lane + 1) & 63);
                    const int an = __shfl(act, (lane + 1) & 63);
                    if (lane >= l1 && lane < q - 1) { u = un; act = an; }
                    if (lane == q - 1) { u = 0.0; act = -1; }
                    --q;
                    // pstar stays pending (its slack was advanced)
                }
            }
        }
        IST(3);  // step length, multipliers
        // one in-place update site for every path (no second live copy of cc)
        store_rinv_column(s, pos, add, householder_masked<NQ>(pos, add, zn, dq, cz, cq, d, cc), rk);
        IST(4);  // Householder update
        if (add) {
            if (rebuild) {
                ++rbk;
            } else {
                if (lane == q) { u = up; act = pstar; }
                if (lane == pstar) active = true;
                ++q;
                pstar = -1;
            }
            lds_sync();
        }
        if (drop) {
            givens_drop(s, drop_slot, q, act, cc);
            lds_sync();
        }
        IST(5);  // bookkeeping, barrier, drop path
    }
    IST_FLUSH(a, rb);

    STAMP(a, rb, 4);
    // primal recovery: y = x0 + H^-1 N_A u = x0 + J0 w',  w' = sum_s u_s C0[:, a_s] (lane i < 24 forms
    // component i from the stored initial columns); qdd part: y = w'; slots: y_s = xs + L^-T w'_s
    double wi = 0.0;
    {
        // slots in groups of four under a uniform guard: the four column reads of a group are
        // independent (slots >= q have u = 0 and act = -1 -> column 0, a zero term)
        const int i = lane < NQ ? lane : 0;
        double w4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < NQ; k0 += 4) {
            if (k0 < q) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int ak = bcast_i(act, k0 + j);
                    const double2 c = s.c0[i >> 1][ak < 0 ? 0 : ak];
                    w4[j] = fma(bcast(u, k0 + j), (i & 1) ? c.y : c.x, w4[j]);
                }
            }
        }
        wi = lane < NQ ? (w4[0] + w4[1]) + (w4[2] + w4[3]) : 0.0;
    }
    double yv;
    {   // y_s = xs + M^T w'_s (lane i < 12: column i of M, w'_{12 + k} broadcast)
        const int i = lane < 12 ? lane : 0;
        double x4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < 12; ++k) x4[k & 3] += s.Mi()[k][i] * bcast(wi, 12 + k);
        yv = (lane < 12) ? s.xs[i] + ((x4[0] + x4[1]) + (x4[2] + x4[3])) : 0.0;
    }
    double* yq = s.ucon;  // y[0..23]: qdd then slots
    if (lane < 12) { yq[lane] = wi; yq[12 + lane] = yv; }
    lds_sync();

    STAMP(a, rb, 5);
    // outputs: x (42, cpp:534-541), grf = x[18:30] (cpp:556-563), tau (cpp:565-576)
    const bool ok = (status == WBC_QP_OK);
    if (a.x && lane < 42) {
        double xv;
        if (lane < 6) {  // a = Mbar_b^-1 (Jc_com^T f - gw)
            double F[3] = {0, 0, 0}, Mm[3] = {0, 0, 0};
#pragma unroll
            for (int l = 0; l < 4; ++l) {
                if ((kap >> l) & 1) {
                    const double fl[3] = {yq[12 + 3 * l], yq[13 + 3 * l], yq[14 + 3 * l]};
                    const double dl[3] = {P.d[3 * l], P.d[3 * l + 1], P.d[3 * l + 2]};
                    double t[3];
                    cross3(dl, fl, t);
#pragma unroll
                    for (int i = 0; i < 3; ++i) { F[i] += fl[i]; Mm[i] += t[i]; }
                }
            }
            if (lane < 3) xv = sel3(F, lane) * P.inv_m - (lane == 2 ? pr.gravity : 0.0);
            else {
                const int rr = lane - 3;
                xv = P.Icinv[3 * rr] * Mm[0] + P.Icinv[3 * rr + 1] * Mm[1] + P.Icinv[3 * rr + 2] * Mm[2];
            }
        } else if (lane < 18) {
            xv = yq[lane - 6];
        } else if (lane < 30) {
            const int i = lane - 18;
            xv = ((kap >> (i / 3)) & 1) ? yq[12 + i] : 0.0;
        } else {
            const int i = lane - 30;
            xv = ((kap >> (i / 3)) & 1) ? fabs(P.rsw[i]) : yq[12 + i];
        }
        a.x[(size_t)rb * WBC_NV + lane] = ok ? xv : 0.0;
    }
    if (lane < 12) {
        double tv = P.bbj[lane];
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            const double fi = ((kap >> (i / 3)) & 1) ? yq[12 + i] : 0.0;
            tv += P.Mbj[lane * 12 + i] * yq[i] - P.Jbj[i * 12 + lane] * fi;
        }
        const double fl = ((kap >> (lane / 3)) & 1) ? yq[12 + lane] : 0.0;
        a.tau[(size_t)rb * 12 + lane] = ok ? tv : 0.0;
        a.grf[(size_t)rb * 12 + lane] = ok ? fl : 0.0;
    }
    if (lane == 0) {
        a.status[rb] = status;
        a.iters[rb] = iters;
    }
    if (Hh) {  // working set for the next cycle's hotstart
        const unsigned long long am = __ballot(is_con && !is_eq && active);
        if (lane == 0) {
            Hh[H_WSLO] = ok ? (double)(unsigned)(am & 0xffffffffull) : 0.0;
            Hh[H_WSHI] = ok ? (double)(unsigned)(am >> 32) : 0.0;
            Hh[H_WSKAP] = (double)kap;
        }
    }
}

constexpr int PRE_STANCE = 91;  // packed index of Presolve::stance
static_assert(offsetof(Presolve, stance) == PRE_STANCE * sizeof(double), "PRE_STANCE");
static_assert(offsetof(Presolve, t0) == 104 * sizeof(double) && offsetof(Presolve, nsel) == 116 * sizeof(double),
              "Presolve stance packing (t0 / nsel in PreRegs::v1 lanes 40.. / 52..)");

// solveQP + computeJointTorques (cpp:466-577) for a four-contact stance robot whose equalities
// the update kernel eliminated (stance_reduce): Goldfarb-Idnani on the 12 contact forces with the
// 40 inequality rows, one per lane.  Lane p holds constraint 12 + p of the general numbering
// (friction faces 12..27, torque rows 28..51; the 12 equalities hold by construction), so the
// selection order, the reference-space row scales and the hotstart working-set bits are the
// general path's.  The dual iterates are those of the general solve after its equality block
// (same QP restricted to the equality manifold), which the iteration-parity tests check.
//   friction face rr of leg l:  -D_rr f_l >= 0                       (cpp:404-424)
//   torque row j, sign sg:      sg (t0_j - Nt_j f) >= -tau_max       (cpp:495,506,513)
__device__ void solve_stance(const KernelArgs& a, int rb, const Prob* Pg, const PreRegs& pf, const Presolve* rec,
                             StanceScratch& s) {
    const Prob& P = *Pg;  // the assembled problem in HBM / L2: only flags, bbar_j and the x-output fields are read
    constexpr int N = StanceScratch::N, MC = StanceScratch::MC, NEQ = 12;
    const wbc_params& pr = a.pv;
    const int lane = lane_id();
    STAMP(a, rb, 0);
    int status = (P.flags != 0.0) ? WBC_QP_NUMERIC : WBC_QP_OK;
    int iters = 0;
    // M (packed p < 78: M(i, j), p = i (i + 1) / 2 + j) and f0 (78..89) from the record registers
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int p = lane + 64 * h;
        const double v = h ? pf.v1 : pf.v0;
        if (p < 78) {
            const int i = (int)((sqrt(8.0 * p + 1.0) - 1.0) * 0.5);
            s.Mi()[i][p - i * (i + 1) / 2] = v;
        } else if (p < 90) {
            s.xs[p - 78] = v;
        }
    }
    for (int k = lane; k < 144; k += 64) {
        const int i = k / 12, j = k % 12;
        if (j > i) s.Mi()[i][j] = 0.0;
    }
    lds_sync();

    // this lane's row: normal n (force space), bound b (n^T f >= b), reference-space scale
    const bool is_con = lane < MC;
    const bool fr = lane < 16, tq = lane >= 16 && lane < MC;
    const int l = (lane >> 2) & 3, rr = lane & 3;
    const int qt = tq ? lane - 16 : 0, k = qt >> 1;
    const double sg = (qt & 1) ? -1.0 : 1.0;
    double cc[N];
    {
        const double2* nt = reinterpret_cast<const double2*>(rec->Nt + k * 12);
#pragma unroll
        for (int j = 0; j < N; j += 2) {
            const double2 v = nt[j / 2];
            cc[j] = tq ? -sg * v.x : 0.0;
            cc[j + 1] = tq ? -sg * v.y : 0.0;
        }
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
#pragma unroll
            for (int r = 0; r < 3; ++r) {
                // friction face rr: (-1 | 1 | 0, 0 | 0 | -1 | 1, mu), as build_normal
                const double fv = (r == 0) ? ((rr == 0) ? -1.0 : (rr == 1 ? 1.0 : 0.0))
                                : (r == 1) ? ((rr == 2) ? -1.0 : (rr == 3 ? 1.0 : 0.0)) : pr.friction;
                if (fr) cc[3 * mm + r] = (mm == l) ? fv : 0.0;
            }
        }
    }
    const double t0k = vbcast(pf.v1, 40 + k), nsk = vbcast(pf.v1, 52 + k);
    const double bj = P.bbj[k];
    const double bp = tq ? (-pr.max_torque - sg * t0k) : 0.0;
    const double bref = tq ? (-pr.max_torque - sg * bj) : 0.0;  // the reference row's own bound
    const double tolv = 1e-10 * fmax(1.0, fabs(bref));
    const double inrm = 1.0 / sqrt(fmax(fr ? 1.0 + pr.friction * pr.friction : nsk, 1e-300));
    double nn, sp;
    {
        double np[4] = {0.0, 0.0, 0.0, 0.0}, sq[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < N; ++j) {
            np[j & 3] += cc[j] * cc[j];
            sq[j & 3] += cc[j] * s.xs[j];
        }
        nn = (np[0] + np[1]) + (np[2] + np[3]);
        sp = ((sq[0] + sq[1]) + (sq[2] + sq[3])) - bp;
    }
    STAMP(a, rb, 1);  // unpack, normals, norms, slacks
    {   // C0[:, p] = M n_p (M read as a broadcast)
        double t[N];
#pragma unroll
        for (int i = 0; i < N; ++i) {
            double a4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int j = 0; j <= i; ++j) a4[j & 3] += s.Mi()[i][j] * cc[j];
            t[i] = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        }
#pragma unroll
        for (int i = 0; i < N; ++i) cc[i] = t[i];
    }
    const double sp0 = sp;
    if (is_con) {
#pragma unroll
        for (int j = 0; j < N; j += 2) s.c0[j / 2][lane] = make_double2(cc[j], cc[j + 1]);
    }
    zero_rinv(s);
    lds_sync();

    STAMP(a, rb, 2);  // C0, zero R^-1
    int q = 0;         // active set size
    double u = 0.0;    // multiplier of active slot `lane`
    int act = -1;      // constraint (lane) of active slot `lane`
    int pstar = -1;
    int rbk = -1;      // rebuild cursor (hotstart re-adds)
    double up = 0.0;
    bool active = false;
    const double tiny = 1e-26;
    bool done = (status != WBC_QP_OK);

    // hotstart (cpp:523-535): the previous working set, constraint ids 12.. -> lanes 0..
    double* Hh = a.stateful ? a.hist + (size_t)rb * HIST_LEN : nullptr;
    bool warm_fail = false;
    if (!done && Hh && !a.cold) {
        const unsigned long long ws = (unsigned long long)(unsigned)Hh[H_WSLO] |
                                      ((unsigned long long)(unsigned)Hh[H_WSHI] << 32);
        unsigned long long wm = ((int)Hh[H_WSKAP] == 15) ? (ws >> NEQ) : 0ull;
        wm &= (1ull << MC) - 1ull;
        const int nw = __popcll(wm);
        if (nw > 0 && nw <= N) {
            const bool mine = (wm >> lane) & 1ull;
            const int slot = __popcll(wm & ((1ull << lane) - 1ull));
            if (mine) s.colbuf[slot] = (double)lane;
            lds_sync();
            if (lane < nw) act = (int)s.colbuf[lane];
            if (mine) active = true;
            lds_sync();
            rbk = 0;
            q = nw;
        }
    }
    const int max_wsr = pr.max_wsr;

    while (!done) {
        asm volatile("" ::: "memory");
        if (rbk >= q) {  // hotstart re-adds finished
            rbk = -1;
            active_set_point(s, q, act, sp0, cc, u, sp);
            const bool neg = lane < q && u < -1e-10;
            if (warm_fail || wave_any(neg)) {
                // reject the warm set: cold start from the unconstrained optimum
                if (is_con) {
#pragma unroll
                    for (int j = 0; j < N; j += 2) {
                        const double2 c = s.c0[j / 2][lane];
                        cc[j] = c.x;
                        cc[j + 1] = c.y;
                    }
                }
                zero_rinv(s);
                lds_sync();
                act = -1;
                u = 0.0;
                active = false;
                q = 0;
                sp = sp0;
                continue;
            }
            if (lane < q && u < 0.0) u = 0.0;
        }
        const bool rebuild = rbk >= 0;
        int col, pos;
        if (rebuild) {
            col = bcast_i(act, rbk);
            pos = rbk;
        } else {
            if (pstar < 0) {  // most violated row, by slack / |reference row|
                double v = 1e300;
                if (is_con && !active && sp < -tolv) v = sp * inrm;
                double vm;
                const int idx = wave_select_band(v, vm);
                if (!(vm < 1e299)) break;  // no violated constraint: optimal
                pstar = idx;
                up = 0.0;
            }
            if (++iters > max_wsr) { status = WBC_QP_MAX_ITER; iters = max_wsr; break; }
            col = pstar;
            pos = q;
        }
        double d[N];
        read_column<N>(cc, col, d);
        const double rk = rinv_times_d(s, d);
        double czp[4] = {0.0, 0.0, 0.0, 0.0}, cqp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int j = 0; j < N; ++j) {
            const double mk = (j >= pos) ? 1.0 : 0.0, ok = (j == pos) ? 1.0 : 0.0;
            d[j] *= mk;
            czp[j & 3] += cc[j] * d[j];
            cqp[j & 3] += cc[j] * ok;
        }
        const double cz = (czp[0] + czp[1]) + (czp[2] + czp[3]);
        const double cq = (cqp[0] + cqp[1]) + (cqp[2] + cqp[3]);
        const double zn = bcast(cz, col);
        const double dq = bcast(cq, col);

        bool add = true, drop = false;
        int drop_slot = -1;
        if (rebuild && !(zn > tiny * fmax(1.0, bcast(nn, col)))) {
            add = false;  // a warm row dependent on the others: reject the warm set
            warm_fail = true;
            ++rbk;
        }
        if (!rebuild) {
            const double sps = bcast(sp, pstar);
            double t1;
            int l1;
            {
                double v = 1e300;
                if (lane < q && rk > 1e-14) v = u * fast_rcp(rk);
                l1 = wave_argmin_lane(v);
                t1 = bcast(v, l1);
            }
            const double t2 = (zn > 1e-14) ? (-sps * fast_rcp(zn)) : 1e300;
            const double t = fmin(t1, t2);
            if (!(t < 1e299)) { status = WBC_QP_INFEASIBLE; break; }
            const bool full = (t2 < 1e299 && t2 <= t1);
            if (t2 < 1e299) sp += t * cz;
            if (lane < q) u -= t * rk;
            up += t;
            if (!full) {
                add = false;
                drop = true;
                drop_slot = l1;
                const int dropped = bcast_i(act, l1);
                if (lane == dropped) active = false;
                const double un = __shfl(u, (lane + 1) & 63);
                const int an = __shfl(act, (lane + 1) & 63);
                if (lane >= l1 && lane < q - 1) { u = un; act = an; }
                if (lane == q - 1) { u = 0.0; act = -1; }
                --q;
            }
        }
        store_rinv_column(s, pos, add, householder_masked<N>(pos, add, zn, dq, cz, cq, d, cc), rk);
        if (add) {
            if (rebuild) {
                ++rbk;
            } else {
                if (lane == q) { u = up; act = pstar; }
                if (lane == pstar) active = true;
                ++q;
                pstar = -1;
            }
            lds_sync();
        }
        if (drop) {
            givens_drop(s, drop_slot, q, act, cc);
            lds_sync();
        }
    }

    STAMP(a, rb, 3);  // active-set loop
    // primal: f = f0 + H_f^-1 N_A u = f0 + M^T w',  w' = sum_s u_s C0[:, a_s]
    double wi;
    {
        const int i = lane < N ? lane : 0;
        double w4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k0 = 0; k0 < N; k0 += 4) {
            if (k0 < q) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int ak = bcast_i(act, k0 + j);
                    const double2 c = s.c0[i >> 1][ak < 0 ? 0 : ak];
                    w4[j] = fma(bcast(u, k0 + j), (i & 1) ? c.y : c.x, w4[j]);
                }
            }
        }
        wi = (w4[0] + w4[1]) + (w4[2] + w4[3]);
    }
    {
        const int i = lane < N ? lane : 0;
        double x4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k2 = 0; k2 < N; ++k2) x4[k2 & 3] += s.Mi()[k2][i] * bcast(wi, k2);
        if (lane < N) s.ucon[lane] = s.xs[i] + ((x4[0] + x4[1]) + (x4[2] + x4[3]));
    }
    lds_sync();
    STAMP(a, rb, 4);  // primal
    const bool ok = (status == WBC_QP_OK);
    // torques tau_j = t0_j - Nt_j f (cpp:565-576), grf = f (cpp:556-563)
    const double t0j = vbcast(pf.v1, 40 + (lane < 12 ? lane : 0));  // all lanes: ds_bpermute reads 0 from inactive ones
    if (lane < 12) {
        const int j = lane;
        const double2* nt = reinterpret_cast<const double2*>(rec->Nt + j * 12);
        double t4[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int c = 0; c < 12; c += 2) {
            const double2 nv = nt[c / 2];
            t4[c & 3] = fma(nv.x, s.ucon[c], t4[c & 3]);
            t4[(c + 1) & 3] = fma(nv.y, s.ucon[c + 1], t4[(c + 1) & 3]);
        }
        const double tv = t0j - ((t4[0] + t4[1]) + (t4[2] + t4[3]));
        a.tau[(size_t)rb * 12 + lane] = ok ? tv : 0.0;
        a.grf[(size_t)rb * 12 + lane] = ok ? s.ucon[j] : 0.0;
    }
    if (a.x) {  // x (42, cpp:534-541): a = Mb^-1 (E^T f - gw), qdd = q0 - Y Mb^-1 E^T f, f, slacks |rsw|
        double F[3] = {0, 0, 0}, Mm[3] = {0, 0, 0};
#pragma unroll
        for (int ll = 0; ll < 4; ++ll) {
            const double fl[3] = {s.ucon[3 * ll], s.ucon[3 * ll + 1], s.ucon[3 * ll + 2]};
            const double dl[3] = {P.d[3 * ll], P.d[3 * ll + 1], P.d[3 * ll + 2]};
            double t[3];
            cross3(dl, fl, t);
#pragma unroll
            for (int i = 0; i < 3; ++i) { F[i] += fl[i]; Mm[i] += t[i]; }
        }
        double bf[6];  // Mb^-1 E^T f
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            bf[i] = F[i] * P.inv_m;
            bf[3 + i] = P.Icinv[3 * i] * Mm[0] + P.Icinv[3 * i + 1] * Mm[1] + P.Icinv[3 * i + 2] * Mm[2];
        }
        if (lane < 42) {
            double xv;
            if (lane < 6) {
                // selects on scalars (sel3 on the local array was lowered to a scratch load)
                xv = sel3d(lane < 3 ? lane : 0, bf[0], bf[1], bf[2]);
                xv = (lane < 3) ? xv - (lane == 2 ? pr.gravity : 0.0) : sel3d(lane < 3 ? 0 : lane - 3, bf[3], bf[4], bf[5]);
            } else if (lane < 18) {
                const int j = lane - 6;
                const double* yr = rec->Y + j * 6;
                double qv = rec->q0[j];
#pragma unroll
                for (int c = 0; c < 6; ++c) qv = fma(-yr[c], bf[c], qv);
                xv = qv;
            } else if (lane < 30) {
                xv = s.ucon[lane - 18];
            } else {
                xv = a.modes ? 0.0 : fabs(P.rsw[lane - 30]);  // hypotheses mask the swing bound of stance legs
            }
            a.x[(size_t)rb * WBC_NV + lane] = ok ? xv : 0.0;
        }
    }
    if (lane == 0) {
        a.status[rb] = status;
        a.iters[rb] = iters;
    }
    STAMP(a, rb, 5);  // outputs
    if (Hh) {  // working set for the next cycle's hotstart, in the general numbering
        const unsigned long long am = __ballot(is_con && active) << NEQ;
        if (lane == 0) {
            Hh[H_WSLO] = ok ? (double)(unsigned)(am & 0xffffffffull) : 0.0;
            Hh[H_WSHI] = ok ? (double)(unsigned)(am >> 32) : 0.0;
            Hh[H_WSKAP] = 15.0;
        }
    }
}

// ---------------------------------------------------------------------------------------
// kernels: one 64-lane workgroup per robot
// ---------------------------------------------------------------------------------------
#define WBC_KERNEL_ATTR \
    __global__ __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(WBC_WAVES_PER_SIMD)))
// Split-mode update kernel: 16 lanes per robot, four robots per wave: the update phase keeps at
// most 13 lanes of a robot busy, so a 64-lane robot wastes 3/4 of every VALU issue.  Four robots'
// scratch (≈ 39 KB of LDS per workgroup) limits the kernel to one wave per SIMD; measured on
// MI355X it still beats the one-robot-per-wave update (which runs at 2 waves per SIMD) and the
// fused kernel: B = 4096 stance 110.0 -> 100.3 us per step, B = 16384 342 -> 310 us
// (profiles/r01/variants_update_sub.log).
#define WBC_UPDATE_KERNEL_ATTR \
    __global__ __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(1)))
constexpr int UPD_SUB = 16, UPD_RPW = 64 / UPD_SUB;
struct UpdLds {
    LdsModel model;   // staged once per wave (LdsImage): the kinematic chain reads it at lane-varying addresses
    double fric[FRIC_LEN];
    Prob prob[UPD_RPW];
    UpdScratch u[UPD_RPW];
};
// four workgroups per CU (one wave per SIMD): 160 KB of LDS
static_assert(4 * sizeof(UpdLds) <= 160 * 1024, "update_solve LDS budget");
static_assert(offsetof(UpdLds, fric) == offsetof(LdsImage, fric) && offsetof(UpdLds, model) == 0,
              "UpdLds starts with the LdsImage block");
struct SolveLds {
    Prob prob;
    QpScratch q;
};

// The one-kernel translation units (wbc_kernel_stance.hip, wbc_kernel_step0.hip,
// wbc_kernel_modes.hip) include this file under their own macro, which keeps only their kernel and
// its launcher; this file's own unit builds everything else
#if defined(WBC_STANCE_TU) || defined(WBC_STEP0_TU) || defined(WBC_STEP1_TU) || defined(WBC_MODES_TU) || \
    defined(WBC_RESIDENT_TU)
#define WBC_SINGLE_TU 1
#endif
#ifndef WBC_SINGLE_TU
WBC_KERNEL_ATTR void wbc_step_kernel(KernelArgs a) {
    __shared__ Lds L;
    const int rb = xcd_robot();
    if (rb >= a.batch) return;
    STAMP(a, rb, 0);
    update_phase<64>(a, rb, rb, a.contacts[rb], lane_id(), true, L.u, L.prob, nullptr, *a.model);
    STAMP(a, rb, 1);
    solve_phase(a, rb, L.prob, nullptr, L.q);
    STAMP(a, rb, 6);
}
#endif  // WBC_SINGLE_TU

// The update kernel, and (SOLVE) its form that also solves the four-contact stance QPs whose
// elimination succeeded (wbc_update_solve_kernel: stateless all-stance steps; the problem of such
// a robot never goes to HBM, only its outputs do).
// Copy N elements global -> LDS with every load issued before the first store: one memory round
// trip.  The plain strided loop (`for (k = lane; k < N; k += 64) dst[k] = src[k]`) has a
// lane-dependent trip count, so it is not unrolled and each iteration waits for its own load
// (s_waitcnt vmcnt(0) before the ds_write): N / 64 serialized round trips.
template <int N>
__device__ __forceinline__ void stage_to_lds(double* dst, const double* src, int t) {
    constexpr int IT = (N + 63) / 64;
    double v[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int k = t + 64 * it;
        v[it] = src[k < N ? k : N - 1];
    }
    __builtin_amdgcn_sched_barrier(0);  // the scheduler may not sink a load below the first store
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int k = t + 64 * it;
        dst[k < N ? k : N - 1] = v[it];  // branch-free: lanes past the end rewrite the last element, same value
    }
}
// the same for 16-byte elements (kept as two scalar arrays: a local array of double2 is not
// promoted to registers here and goes through scratch)
template <int N>
__device__ __forceinline__ void stage_to_lds(double2* dst, const double2* src, int t) {
    constexpr int IT = (N + 63) / 64;
    double vx[IT], vy[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int k = t + 64 * it;
        const double2 w = src[k < N ? k : N - 1];
        vx[it] = w.x;
        vy[it] = w.y;
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int k = t + 64 * it;
        dst[k < N ? k : N - 1] = make_double2(vx[it], vy[it]);
    }
}

#ifndef WBC_SINGLE_TU
// The split update (wbc_update, WBC_SPLIT, the update of wbc_step_modes' split form): Prob +
// Presolve records to HBM for wbc_solve_kernel / wbc_solve_stance_kernel.
WBC_UPDATE_KERNEL_ATTR void wbc_update_kernel(KernelArgs a) {
    __shared__ UpdLds L;
    const int seg = (int)threadIdx.x / UPD_SUB, lane = (int)threadIdx.x % UPD_SUB;
    int rb = (int)blockIdx.x * UPD_RPW + seg;
    const bool wr = rb < a.batch;  // a padding segment recomputes the last robot, writes nothing
    if (!wr) rb = a.batch - 1;
    stage_to_lds<LIMG_LEN>(reinterpret_cast<double*>(&L), a.limg, (int)threadIdx.x);
    lds_sync();
    // work row: [Prob | Presolve]; the Presolve record is stored by update_phase itself
    Presolve* pre = reinterpret_cast<Presolve*>(a.work + (size_t)rb * WORK_LEN + PROB_LEN);
    if (a.elim && blockIdx.x == 0 && threadIdx.x == 0) a.fb[a.parity ^ 1] = 0;  // for the next update
    const bool stance =
        update_phase<UPD_SUB, false>(a, rb, rb, a.contacts[rb], lane, wr, L.u[seg], L.prob[seg], pre, L.model);
    const double2* src = reinterpret_cast<const double2*>(&L.prob[seg]);
    double2* dst = reinterpret_cast<double2*>(a.work + (size_t)rb * WORK_LEN);
    if (wr) {
        for (int k = lane; k < PROB_LEN / 2; k += UPD_SUB) dst[k] = src[k];
    }
    // QPs whose elimination did not happen go to the fallback list (rare: one atomic each): every
    // one of them, whatever its mask, so that a wrong host decision (a mask the host counted as 15)
    // costs speed, never a QP left unsolved
    if (a.elim && wr && !stance) {
        const int K = a.modes;
        if (K ? lane < K : lane == 0) {
            const int idx = atomicAdd(&a.fb[a.parity], 1);
            if (idx < a.fb_cap) a.fb[2 + idx] = K ? rb * K + lane : rb;
        }
    }
}
#endif  // WBC_SINGLE_TU

// The default wbc_step (and wbc_step_modes): one kernel per step, four QPs per wave, 16 lanes
// each.  Segment seg of workgroup w is QP qp = 4 w + seg: its inputs and history are row qp, or,
// under K mode hypotheses, state qp / K with contact mask mode_masks[qp % K] (the state's
// dynamics are recomputed per hypothesis segment: four hypotheses of one state share a wave's
// instruction stream, and nothing passes through HBM).  update_phase reduces and solves the QP in
// place (§4.6, §4.8); a QP whose reduction is not usable (a near-singular stance leg) writes its
// problem to work row qp (no slot factor: presolved = 0), which the same wave then solves with the
// general 24-variable method (drain_fallbacks, modes = 0: the record carries the QP's own mask and
// masked bounds).
__device__ void solve_general_qp(const KernelArgs& a, int rb, SolveLds& L);
static_assert(sizeof(SolveLds) <= sizeof(UpdLds), "the drain reuses the update scratch");
// A call (the rare path stays out of the kernel's register allocation), handed the address of the
// kernel's arguments in its kernarg segment (passing the struct would pin a stack copy to the whole
// kernel; a callee has no kernarg pointer of its own).
// (One instance per calling kernel, TAG: a shared callee is allocated for the larger of its callers'
// register budgets, which raised the default step's to 512 registers and its scratch to 2.2 KB.)
template <int TAG>
__device__ __attribute__((noinline)) void drain_fallbacks(const KernelArgs* ka, unsigned long long fm, int qp,
                                                          SolveLds* L) {
    KernelArgs f = *ka;
    f.modes = 0;
    f.elim = 0;
    __threadfence_block();  // the records written above are read back by the whole wave
    while (fm) {
        const int seg = __builtin_ctzll(fm) / UPD_SUB;
        fm &= fm - 1ull;
        wsync();
        solve_general_qp(f, __builtin_amdgcn_readlane(qp, seg * UPD_SUB), *L);
    }
}
// Workgroups are dispatched to the 8 XCDs round-robin (block b on XCD b % 8), each with its own
// L2.  Under mode hypotheses the K / 4 workgroups of one state read the same input rows, so each
// XCD gets a contiguous range of logical blocks: a state's workgroups share one L2 and its inputs
// come from HBM once.
__device__ __forceinline__ int xcd_block(int b, int n) {
    const int x = b & 7, i = b >> 3, per = n >> 3, rem = n & 7;  // XCD x runs per + (x < rem) blocks
    return x * per + min(x, rem) + i;
}
// Two instances: STF = 0 for stateless steps (no history code at all), 1 for stateful ones
template <int STF, bool SONLY = false>
WBC_UPDATE_KERNEL_ATTR void wbc_update_solve_kernel(KernelArgs a) {
    __shared__ UpdLds L;
    const int seg = (int)threadIdx.x / UPD_SUB, lane = (int)threadIdx.x % UPD_SUB;
    const int K = a.modes;
    int qp, row, kap;
    bool wr, empty = false;
    if (K) {
        // workgroup g K + k: states 4 g .. 4 g + 3 under mask modes[k] (one mask per wave); the K
        // workgroups of a state group are consecutive, and xcd_block keeps them on one XCD
        const int blk = xcd_block((int)blockIdx.x, (int)gridDim.x);
        const int S = a.batch / K, g = blk / K, k = blk - g * K;
        row = 4 * g + seg;
        wr = row < S;  // a padding segment recomputes the last state, writes nothing
        if (!wr) row = S - 1;
        qp = row * K + k;
        kap = a.mode_masks[k] & 15;
    } else {
        // the wave map groups the QPs by contact mask (KernelArgs::qmap): the workgroup's four
        // entries as one uniform 16-byte (scalar) load
        int e = (int)blockIdx.x * UPD_RPW + seg;
        if (a.qmap) {
            const int4 e4 = reinterpret_cast<const int4*>(a.qmap)[blockIdx.x];
            e = (seg == 0) ? e4.x : (seg == 1) ? e4.y : (seg == 2) ? e4.z : e4.w;
        }
        if (a.qmap) {
            empty = e == QMAP_EMPTY;
            wr = e >= 0;
            const int v = empty ? qmap_entry(a.batch - 1, 15) : (wr ? e : ~e);
            qp = v >> 4;
            kap = v & 15;
            row = qp;
        } else {
            wr = e < a.batch;
            qp = wr ? e : a.batch - 1;
            row = qp;
            kap = a.contacts[row] & 15;
        }
    }
    UST(a, qp, 30);  // kernel entry (diagnostic build)
#ifdef WBC_ISTAMPS
    // placement and the constant clock, for the wave-schedule probe (tools/wave_sched.py): slots
    // 39 / 40 / 41 = s_memrealtime at entry, HW_ID, XCC_ID; 42 / 43 = s_memrealtime, s_memtime at the
    // end; 44 = the workgroup's index
    if (lane_id() == 0) {
        a.dbg[(size_t)qp * WBC_DBG_LEN + 39] = (double)__builtin_amdgcn_s_memrealtime();
        a.dbg[(size_t)qp * WBC_DBG_LEN + 40] = (double)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
        a.dbg[(size_t)qp * WBC_DBG_LEN + 41] = (double)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);
        a.dbg[(size_t)qp * WBC_DBG_LEN + 44] = (double)blockIdx.x;
    }
#endif
    // the robot's inputs (HBM) are requested before the model staging waits for its own loads
    double vin[(91 + UPD_SUB - 1) / UPD_SUB];
    load_inputs<UPD_SUB>(a, row, lane, vin);
    // the model and friction table: the host-built LDS image (wbc_layout.h), one contiguous copy
    stage_to_lds<LIMG_LEN>(reinterpret_cast<double*>(&L), a.limg, (int)threadIdx.x);
    if (__all(empty)) return;  // the unused tail of a device-built map (uniform)
    lds_sync();
    const bool solved = update_phase<UPD_SUB, true, LdsModel, false, STF, SONLY>(a, row, qp, kap, lane, wr, L.u[seg], L.prob[seg], nullptr,
                                                                         L.model, &L.fric[0], vin);
    // a QP whose reduction was not usable: its problem goes to work row qp, and the wave solves it
    // with the general 24-variable method right here (drain_fallbacks, the rare path; the wave's
    // LDS is reused once the four segments are done)
    const bool fb = wr && !solved;
    if (fb) {
        const double2* src = reinterpret_cast<const double2*>(&L.prob[seg]);
        double* wrow = a.work + (size_t)qp * WORK_LEN;
        double2* dst = reinterpret_cast<double2*>(wrow);
        for (int k = lane; k < PROB_LEN / 2; k += UPD_SUB) dst[k] = src[k];
        if (lane == 0) {
            Presolve* pre = reinterpret_cast<Presolve*>(wrow + PROB_LEN);
            pre->presolved = 0.0;
            pre->stance = 0.0;
        }
    }
    const unsigned long long fm = __ballot(fb && lane == 0);
    if (fm)
        drain_fallbacks<2 + STF>((const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr(), fm, qp,
                           reinterpret_cast<SolveLds*>(&L));
#ifdef WBC_ISTAMPS
    if (lane_id() == 0) {
        a.dbg[(size_t)qp * WBC_DBG_LEN + 42] = (double)__builtin_amdgcn_s_memrealtime();
        a.dbg[(size_t)qp * WBC_DBG_LEN + 43] = (double)__builtin_amdgcn_s_memtime();
    }
#endif
}

// The resident control cycle (wbc_cycle with WBC_RESIDENT, B <= 4: one wave): the step above,
// looped in one workgroup that stays on the GPU between control cycles, so a cycle costs no kernel
// launch and no stream synchronisation.  The host packs the cycle's inputs into
// the pinned input block, then raises box->cmd; the wave polls it (one lane, relaxed system-scope
// atomic loads, which bypass the caches, s_sleep between polls), copies the pinned input block
// into the engine's own device input block with the same loads (no acquire fence: a system-scope
// acquire invalidates the L2 and, polled, left the step's code and model to be fetched from HBM
// again every cycle), runs the step on it, writing the outputs to the pinned output block, and
// publishes box->done = cmd after a system-scope release of those stores.  Every wave of the loop
// ends: on WBC_RESIDENT_STOP, or when no command arrives within idle_ticks of the 100 MHz constant
// clock (s_memrealtime), so a host that stops posting (or exits) never leaves the wave spinning;
// the host relaunches it after any pause of half that time.
template <int STF>
WBC_UPDATE_KERNEL_ATTR void wbc_resident_kernel(KernelArgs args, ResidentBox* box, const unsigned long long* pin_in,
                                                unsigned long long* own_in, int in_words, unsigned long long seq0,
                                                unsigned long long idle_ticks) {
    __shared__ UpdLds L;
    // the loop's own state lives in LDS, re-read after every barrier: kept in registers across the
    // step body it was spilled to scratch (the body needs every register it has)
    __shared__ struct {
        ResidentBox* box;
        const unsigned long long* pin;
        unsigned long long *own, last, idle, cmd;
        int words;
    } C;
    (void)args;
    if (threadIdx.x == 0) {
        C.box = box;
        C.pin = pin_in;
        C.own = own_in;
        C.last = seq0;
        C.idle = idle_ticks;
        C.words = in_words;
    }
    for (;;) {
        __syncthreads();
        if (threadIdx.x == 0) {
            ResidentBox* bx = C.box;
            const unsigned long long last = C.last, idle = C.idle;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            unsigned long long c;
            for (;;) {
                c = __hip_atomic_load(&bx->cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (c != last) break;
                const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t0;
                if (dt > idle) { c = WBC_RESIDENT_STOP; break; }
                // polls over PCIe: every ~30 ns for the first 100 us after a cycle (a control loop's
                // next cycle usually comes sooner), then every ~0.5 us
                if (dt < 10000ull) __builtin_amdgcn_s_sleep(1);
                else __builtin_amdgcn_s_sleep(16);
            }
            C.cmd = c;
        }
        __syncthreads();
        if (C.cmd == WBC_RESIDENT_STOP) break;
        // the cycle's inputs: the pinned block's words (loads in one batch: two per lane covers B <= 1,
        // the loop the rest) into the engine's device block, which update_phase reads (KernelArgs'
        // input pointers point there)
        {
            const unsigned long long* pin = C.pin;
            unsigned long long* own = C.own;
            const int t = (int)threadIdx.x, nw = C.words;
            const int k0 = t < nw ? t : nw - 1, k1 = t + 64 < nw ? t + 64 : nw - 1;
            const unsigned long long w0 = __hip_atomic_load(&pin[k0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            const unsigned long long w1 = __hip_atomic_load(&pin[k1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            own[k0] = w0;
            own[k1] = w1;
            for (int k = t + 128; k < nw; k += 64)
                own[k] = __hip_atomic_load(&pin[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        // the step's arguments and lane ids are re-derived every cycle through an opaque copy: loop-
        // invariant, the compiler hoisted their derived values out of the loop and spilled them
        const KernelArgs* ap = (const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        int tid = (int)threadIdx.x;
        asm volatile("" : "+s"(ap), "+v"(tid));
        const KernelArgs& a = *ap;
        const int seg = tid / UPD_SUB, lane = tid % UPD_SUB;
        const int e = seg;
        const bool wr = e < a.batch;
        const int qp = wr ? e : a.batch - 1, row = qp;
        const int kap = a.contacts[row] & 15;
        double vin[(91 + UPD_SUB - 1) / UPD_SUB];
        load_inputs<UPD_SUB>(a, row, lane, vin);
        stage_to_lds<LIMG_LEN>(reinterpret_cast<double*>(&L), a.limg, tid);
        lds_sync();
        const bool solved = update_phase<UPD_SUB, true, LdsModel, false, STF>(a, row, qp, kap, lane, wr, L.u[seg], L.prob[seg],
                                                                            nullptr, L.model, &L.fric[0], vin);
        const bool fb = wr && !solved;
        if (fb) {
            const double2* src = reinterpret_cast<const double2*>(&L.prob[seg]);
            double* wrow = a.work + (size_t)qp * WORK_LEN;
            double2* dst = reinterpret_cast<double2*>(wrow);
            for (int k = lane; k < PROB_LEN / 2; k += UPD_SUB) dst[k] = src[k];
            if (lane == 0) {
                Presolve* pre = reinterpret_cast<Presolve*>(wrow + PROB_LEN);
                pre->presolved = 0.0;
                pre->stance = 0.0;
            }
        }
        const unsigned long long fm = __ballot(fb && lane == 0);
        if (fm)
            drain_fallbacks<4 + STF>(ap, fm, qp,
                                     reinterpret_cast<SolveLds*>(&L));
        // outputs (pinned host memory) and history (HBM) stored, then the cycle published
        __syncthreads();
        __threadfence_system();
        if (threadIdx.x == 0) {
            const unsigned long long cmd = C.cmd;
            __hip_atomic_store(&C.box->done, cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            C.last = cmd;
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(&C.box->exited, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef WBC_MODES_TU  // (wbc_kernel_modes.hip)
// Mode hypotheses with the update shared (KernelArgs::mloop = M > 1): workgroup g C + c (C = K / M
// chunks, xcd_block order, so a state group's chunks share an L2) runs states 4 g .. 4 g + 3, each
// segment through one update and then the M hypotheses of chunk c (update_phase's mode loop);
// the update's share of a hypothesis falls from one whole update to 1 / M of one.  Outputs,
// fallbacks and their records are the per-hypothesis step's.
WBC_UPDATE_KERNEL_ATTR void wbc_modes_kernel(KernelArgs a) {
    __shared__ UpdLds L;
    const int seg = (int)threadIdx.x / UPD_SUB, lane = (int)threadIdx.x % UPD_SUB;
    const int K = a.modes, M = a.mloop, C = K / M;
    const int blk = xcd_block((int)blockIdx.x, (int)gridDim.x);
    const int S = a.batch / K, g = blk / C, c = blk - g * C;
    int row = 4 * g + seg;
    const bool wr = row < S;  // a padding segment recomputes the last state, writes nothing
    if (!wr) row = S - 1;
    const int k0 = a.mode_order[c * M];
    double vin[(91 + UPD_SUB - 1) / UPD_SUB];
    load_inputs<UPD_SUB>(a, row, lane, vin);
    stage_to_lds<LIMG_LEN>(reinterpret_cast<double*>(&L), a.limg, (int)threadIdx.x);
    lds_sync();
    unsigned fails = 0;
    update_phase<UPD_SUB, true, LdsModel, true, 0>(a, row, row * K + k0, a.mode_masks[k0] & 15, lane, wr, L.u[seg],
                                                L.prob[seg], nullptr, L.model, &L.fric[0], vin, c, &fails);
    for (int it = 0; it < M; ++it) {
        const unsigned long long fm = __ballot(wr && lane == 0 && ((fails >> it) & 1u));
        if (fm)
            drain_fallbacks<1>((const KernelArgs*)__builtin_amdgcn_kernarg_segment_ptr(), fm,
                               row * K + a.mode_order[c * M + it], reinterpret_cast<SolveLds*>(&L));
    }
}

#endif  // WBC_MODES_TU
// Four-contact QP whose equalities the update kernel eliminated (its Presolve::stance flag, in
// the record registers): wbc_solve_stance_kernel's; every other QP is wbc_solve_kernel's.
__device__ __forceinline__ int qp_mask(const KernelArgs& a, int rb, int row) {
    return a.modes ? (a.mode_masks[rb - row * a.modes] & 15) : (a.contacts[rb] & 15);
}

__device__ void solve_general_qp(const KernelArgs& a, int rb, SolveLds& L);

#ifndef WBC_SINGLE_TU
WBC_KERNEL_ATTR void wbc_solve_kernel(KernelArgs a) {
    __shared__ SolveLds L;
    const int rb = xcd_robot();
    if (rb >= a.batch) return;
    solve_general_qp(a, rb, L);
}

// The general solve of the elimination fallbacks (mask-15 QPs with a near-singular leg), after
// the stance kernel: a few workgroups stride over the list, whose length the host does not know
// (usually 0).  The loop keeps the kernel arguments live through the solve (spills): this is the
// rare path; wbc_solve_kernel is the straight-line one.
WBC_KERNEL_ATTR void wbc_solve_fallback_kernel(KernelArgs a) {
    __shared__ SolveLds L;
    const int n = min(a.fb[a.parity], a.fb_cap);
    for (int w = blockIdx.x; w < n; w += gridDim.x) {
        const int rb = a.fb[2 + w];
        wsync();
        solve_general_qp(a, rb, L);
    }
}

#endif  // WBC_SINGLE_TU

__device__ void solve_general_qp(const KernelArgs& a, int rb, SolveLds& L) {
    // mode hypotheses: QP rb is hypothesis rb % modes of state rb / modes (one assembled problem
    // per state, read by all of its hypotheses)
    const int row = a.modes ? rb / a.modes : rb;
    // the Presolve record goes to registers, its loads issued before the problem copy's
    const double* prow = a.work + (size_t)row * WORK_LEN + PROB_LEN;
    PreRegs pf;
    pf.v0 = prow[lane_id()];
    pf.v1 = prow[64 + lane_id()];
    const int kap_qp = a.elim ? qp_mask(a, rb, row) : 0;
    stage_to_lds<PROB_LEN / 2>(reinterpret_cast<double2*>(&L.prob),
                               reinterpret_cast<const double2*>(a.work + (size_t)row * WORK_LEN), lane_id());
    // the stance kernel's QP: checked after the problem copy is issued, so that a general QP's
    // loads all go out together (one HBM round trip)
    if (a.elim && kap_qp == 15 && bcast(pf.v1, PRE_STANCE - 64) != 0.0) return;  // (kap_qp read only with elim)
    if (a.modes) {  // this hypothesis' contact mask on the unmasked bounds (update_phase)
        const int kap = a.mode_masks[rb - row * a.modes] & 15;
        const int lane = lane_id();
        wsync();
        if (lane < 12) {
            if ((kap >> (lane / 3)) & 1) L.prob.rsw[lane] = 0.0;
            else L.prob.r1[lane] = 0.0;
        }
        if (lane == 0) L.prob.kappa = (double)kap;
    }
    wsync();
    solve_phase(a, rb, L.prob, &pf, L.q);
}

#ifndef WBC_SINGLE_TU
// Four-contact stance QPs whose equalities the update kernel eliminated (Presolve::stance) are
// solved here, in the 12-variable force space; wbc_solve_kernel skips them.  A kernel of its own
// so that its register and LDS budgets (no 24-variable state, no LDS copy of the problem) allow
// WBC_STANCE_WAVES waves per SIMD instead of the general solve's 2.
#ifndef WBC_STANCE_WAVES
#define WBC_STANCE_WAVES 3  // 2 and 3 time the same; 4 spills (profiles/r02/d)
#endif
__global__ __attribute__((amdgpu_flat_work_group_size(64, 64), amdgpu_waves_per_eu(WBC_STANCE_WAVES)))
void wbc_solve_stance_kernel(KernelArgs a) {
    __shared__ StanceScratch S;
    const int rb = blockIdx.x;
    if (rb >= a.batch) return;
    const int row = a.modes ? rb / a.modes : rb;
    const double* prow = a.work + (size_t)row * WORK_LEN + PROB_LEN;
    PreRegs pf;
    pf.v0 = prow[lane_id()];
    pf.v1 = prow[64 + lane_id()];
    // the engine turns the elimination on only when every QP has mask 15; an elimination
    // fallback (near-singular leg, Presolve::stance = 0) is wbc_solve_fallback_kernel's
    if (bcast(pf.v1, PRE_STANCE - 64) == 0.0 || (a.modes && qp_mask(a, rb, row) != 15)) return;
    solve_stance(a, rb, reinterpret_cast<const Prob*>(a.work + (size_t)row * WORK_LEN), pf,
                 reinterpret_cast<const Presolve*>(prow), S);
}

// The default step's wave map for device-bound contact masks (KernelArgs::qmap, under WBC_GROUP):
// the layout of qmap_build (wbc_layout.h qmap_plan / qmap_pos), then QMAP_EMPTY up to the capacity,
// so the step launches qmap_capacity(B) / 4 workgroups without reading the masks back.  Three
// launches over blocks of QMAP_BLOCK QPs (the first version, one workgroup walking every mask
// twice, took 20 us at B = 8192 and 130 us at B = 65536, more than the grouping saved there,
// profiles/r05/qmap):
//   wbc_qmap_count    per block: the count and first QP of each mask (one ballot per mask and wave
//                     round of 64 QPs);
//   wbc_qmap_plan     one workgroup: each mask's exclusive prefix over the blocks, the totals and the
//                     plan (qmap_plan);
//   wbc_qmap_scatter  per block: each QP's rank in its mask's bucket (its block's prefix, the earlier
//                     waves' and rounds' counts, its ballot's mbcnt) and its entry at qmap_pos; the
//                     padding entries and QMAP_EMPTY up to the capacity.
// Buckets keep batch order, as the host builder's (tests/test_gpu_grouping.py: bit-identical steps).
constexpr int QMAP_THREADS = 256;
static_assert(sizeof(QmapPlan) <= 64 * sizeof(int), "the plan fits the scratch tail (qmap_scratch)");
static_assert(QMAP_BLOCK == 4 * QMAP_THREADS, "four rounds of 64 QPs per wave");
// per wave of the block: its 256 QPs in four rounds of 64, ballot per mask; counts and the first QP
__device__ __forceinline__ void qmap_wave_counts(const uint8_t* masks, int B, int b0, int* c, int* f) {
    const int l = (int)threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k < 16; ++k) { c[k] = 0; f[k] = -1; }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int b = b0 + 64 * r + l;
        const int m = b < B ? (masks[b] & 15) : 16;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const unsigned long long bal = __ballot(m == k);
            c[k] += __popcll(bal);
            if (f[k] < 0 && bal) f[k] = b0 + 64 * r + __builtin_ctzll(bal);
        }
    }
}
__global__ __launch_bounds__(QMAP_THREADS) void wbc_qmap_count(const uint8_t* masks, int B, int* scr) {
    __shared__ int wc[4][16], wf[4][16];
    const int w = (int)threadIdx.x >> 6, l = (int)threadIdx.x & 63;
    int c[16], f[16];
    qmap_wave_counts(masks, B, (int)blockIdx.x * QMAP_BLOCK + 256 * w, c, f);
    if (l == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) { wc[w][k] = c[k]; wf[w][k] = f[k]; }
    }
    __syncthreads();
    const int t = (int)threadIdx.x;
    if (t < 16) {
        int n = 0, fi = -1;
        for (int ww = 0; ww < 4; ++ww) {
            n += wc[ww][t];
            if (fi < 0) fi = wf[ww][t];
        }
        scr[blockIdx.x * 32 + t] = n;
        scr[blockIdx.x * 32 + 16 + t] = fi;
    }
}
__global__ __launch_bounds__(QMAP_THREADS) void wbc_qmap_plan(int B, int* scr) {
    __shared__ int col[16][QMAP_THREADS];  // per-thread sums, then inclusive prefixes over the threads
    __shared__ int first[16];
    const int t = (int)threadIdx.x, nb = qmap_blocks(B);
    const int C = (nb + QMAP_THREADS - 1) / QMAP_THREADS, j0 = min(t * C, nb), j1 = min(j0 + C, nb);
    if (t < 16) first[t] = -1;
    // this thread's blocks: counts and the first QP of each mask (its lowest block holding the mask).
    // One block per thread up to 256 blocks: all 32 loads issued together (a load, a wait and an LDS
    // atomic per mask took 10-25 us, profiles/r05/qmap)
    int own[16], fst[16];
    if (j1 - j0 == 1) {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            own[m] = scr[j0 * 32 + m];
            fst[m] = scr[j0 * 32 + 16 + m];
        }
    } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) { own[m] = 0; fst[m] = -1; }
        for (int j = j0; j < j1; ++j) {
#pragma unroll
            for (int m = 0; m < 16; ++m) {
                const int n = scr[j * 32 + m], f = scr[j * 32 + 16 + m];
                if (fst[m] < 0 && n > 0) fst[m] = f;
                own[m] += n;
            }
        }
    }
#pragma unroll
    for (int m = 0; m < 16; ++m) col[m][t] = own[m];
    __syncthreads();
    for (int d = 1; d < QMAP_THREADS; d <<= 1) {  // Hillis-Steele, all masks per step
        int v[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) v[m] = (t >= d) ? col[m][t - d] : 0;
        __syncthreads();
#pragma unroll
        for (int m = 0; m < 16; ++m) col[m][t] += v[m];
        __syncthreads();
    }
    // the first thread holding mask m (exclusive prefix 0, own count > 0) holds its first QP; the
    // blocks' exclusive prefixes go in place of their counts (no re-read for one block per thread)
#pragma unroll
    for (int m = 0; m < 16; ++m) {
        const int ex = col[m][t] - own[m];
        if (own[m] > 0 && ex == 0) first[m] = fst[m];
    }
    if (j1 - j0 == 1) {
#pragma unroll
        for (int m = 0; m < 16; ++m) scr[j0 * 32 + m] = col[m][t] - own[m];
    } else {
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            int run = col[m][t] - own[m];
            for (int j = j0; j < j1; ++j) {
                const int n = scr[j * 32 + m];
                scr[j * 32 + m] = run;
                run += n;
            }
        }
    }
    __syncthreads();
    if (t == 0) {
        int tot[16], f[16];
#pragma unroll
        for (int m = 0; m < 16; ++m) {
            tot[m] = col[m][QMAP_THREADS - 1];
            f[m] = first[m];
        }
        QmapPlan p;
        qmap_plan(tot, f, p);
        *reinterpret_cast<QmapPlan*>(scr + 32 * nb) = p;
    }
}
__global__ __launch_bounds__(QMAP_THREADS) void wbc_qmap_scatter(const uint8_t* masks, int B, const int* scr,
                                                                 int32_t* map, int cap) {
    __shared__ int wc[4][16];
    const int w = (int)threadIdx.x >> 6, l = (int)threadIdx.x & 63, nb = qmap_blocks(B);
    const QmapPlan& plan = *reinterpret_cast<const QmapPlan*>(scr + 32 * nb);
    const int b0 = (int)blockIdx.x * QMAP_BLOCK + 256 * w;
    int c[16], f[16];
    qmap_wave_counts(masks, B, b0, c, f);
    if (l == 0) {
#pragma unroll
        for (int k = 0; k < 16; ++k) wc[w][k] = c[k];
    }
    __syncthreads();
    int base[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        int n = scr[blockIdx.x * 32 + k];
        for (int ww = 0; ww < w; ++ww) n += wc[ww][k];
        base[k] = n;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int b = b0 + 64 * r + l;
        const int m = b < B ? (masks[b] & 15) : 16;
        int j = 0;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const unsigned long long bal = __ballot(m == k);
            const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
            if (m == k) j = base[k] + below;
            base[k] += __popcll(bal);
        }
        if (b < B) map[qmap_pos(plan, m, j)] = qmap_entry(b, m);
    }
    const int gt = (int)blockIdx.x * QMAP_THREADS + (int)threadIdx.x;
    if (gt < QMAP_SEG && plan.base1 && gt >= plan.pad0) map[gt] = plan.v0;
    if (gt >= QMAP_SEG && gt < 2 * QMAP_SEG && plan.pad1 + gt - QMAP_SEG < plan.end1) map[plan.pad1 + gt - QMAP_SEG] = plan.v1;
    for (int p = 4 * plan.waves + gt; p < cap; p += (int)gridDim.x * QMAP_THREADS) map[p] = QMAP_EMPTY;
}

__global__ void wbc_reset_kernel(double* hist, const uint8_t* mask, int batch) {
    const int rb = xcd_robot();
    if (rb >= batch) return;
    if (mask && !mask[rb]) return;
    double* H = hist + (size_t)rb * HIST_LEN;
    for (int k = threadIdx.x; k < HIST_LEN; k += blockDim.x) H[k] = (k == H_KOLD) ? 15.0 : 0.0;
}
#endif  // WBC_SINGLE_TU

}  // namespace wbc

#ifdef WBC_STANCE_TU
// The stance-only default step (wbc_kernel_stance.hip): built in a translation unit of its own so
// that its schedule can be chosen apart from the mixed-form kernel's (Makefile STANCE_KFLAGS)
extern "C" hipError_t wbc_launch_stance_step(const wbc::KernelArgs* a, hipStream_t st) {
    if (a->nwaves <= 0 || a->stateful || a->modes || a->qmap) return hipErrorInvalidValue;
    hipLaunchKernelGGL((wbc::wbc_update_solve_kernel<0, true>), dim3(a->nwaves), dim3(64), 0, st, *a);
    return hipGetLastError();
}
#elif defined(WBC_STEP0_TU)
// The stateless default step of any mask mix (wbc_kernel_step0.hip: both forms, its own schedule,
// Makefile STEP0_KFLAGS; wbc_launch_update_solve below forwards its stateless steps here)
extern "C" hipError_t wbc_launch_update_solve0(const wbc::KernelArgs* a, hipStream_t st) {
    if (a->nwaves <= 0 || a->stateful) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wbc::wbc_update_solve_kernel<0>, dim3(a->nwaves), dim3(64), 0, st, *a);
    return hipGetLastError();
}
#elif defined(WBC_MODES_TU)
// The mode loop (wbc_kernel_modes.hip, Makefile MODES_KFLAGS)
extern "C" hipError_t wbc_launch_modes(const wbc::KernelArgs* a, hipStream_t st) {
    if (a->nwaves <= 0 || a->modes <= 0 || a->mloop <= 0 || a->modes % a->mloop != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wbc::wbc_modes_kernel, dim3(a->nwaves), dim3(64), 0, st, *a);
    return hipGetLastError();
}
#elif defined(WBC_STEP1_TU)
// The stateful default step (wbc_kernel_step1.hip, Makefile STEP1_KFLAGS; wbc_launch_update_solve
// below forwards its stateful steps here)
extern "C" hipError_t wbc_launch_update_solve1(const wbc::KernelArgs* a, hipStream_t st) {
    if (a->nwaves <= 0 || !a->stateful) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wbc::wbc_update_solve_kernel<1>, dim3(a->nwaves), dim3(64), 0, st, *a);
    return hipGetLastError();
}
#elif defined(WBC_RESIDENT_TU)
// (wbc_kernel_resident.hip, Makefile RESIDENT_KFLAGS)
// The resident control cycle (one workgroup, B <= 4), until WBC_RESIDENT_STOP or idle_ticks without a command
extern "C" hipError_t wbc_launch_resident(const wbc::KernelArgs* a, wbc::ResidentBox* box, const void* pin_in,
                                          void* own_in, int in_words, unsigned long long seq0, unsigned long long idle_ticks,
                                          hipStream_t st) {
    // B <= 4: the 2 B mask bytes fit the one word after the 91 B doubles
    if (a->batch <= 0 || a->batch > wbc::UPD_RPW || a->qmap || a->modes || in_words != 91 * a->batch + 1)
        return hipErrorInvalidValue;
    const auto* pin = static_cast<const unsigned long long*>(pin_in);
    auto* own = static_cast<unsigned long long*>(own_in);
    if (a->stateful)
        hipLaunchKernelGGL(wbc::wbc_resident_kernel<1>, dim3(1), dim3(64), 0, st, *a, box, pin, own, in_words, seq0, idle_ticks);
    else
        hipLaunchKernelGGL(wbc::wbc_resident_kernel<0>, dim3(1), dim3(64), 0, st, *a, box, pin, own, in_words, seq0, idle_ticks);
    return hipGetLastError();
}
// Loads the resident kernels' code now (small engines: the B = 1 drop-in), so that the first resident
// cycle does not pay the code object's lazy load (~10 ms, which showed in the control loop's mean)
extern "C" hipError_t wbc_preload_resident() {
    hipFuncAttributes at;
    hipError_t e = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&wbc::wbc_resident_kernel<1>));
    if (e == hipSuccess) e = hipFuncGetAttributes(&at, reinterpret_cast<const void*>(&wbc::wbc_resident_kernel<0>));
    return e;
}
#else
extern "C" hipError_t wbc_launch_update_solve0(const wbc::KernelArgs* a, hipStream_t st);
extern "C" hipError_t wbc_launch_update_solve1(const wbc::KernelArgs* a, hipStream_t st);

// Launchers used by the engine (wbc_engine.cpp); grid = one 64-lane workgroup per robot.
extern "C" hipError_t wbc_launch_step(const wbc::KernelArgs* a, hipStream_t st) {
    hipLaunchKernelGGL(wbc::wbc_step_kernel, dim3(a->batch), dim3(64), 0, st, *a);
    return hipGetLastError();
}
// map: qmap_capacity(batch) entries followed by qmap_scratch(batch) ints of scratch
extern "C" hipError_t wbc_launch_qmap(const uint8_t* masks, int batch, int32_t* map, hipStream_t st) {
    if (batch <= 0) return hipErrorInvalidValue;
    const int cap = wbc::qmap_capacity(batch), nb = wbc::qmap_blocks(batch);
    int* scr = map + cap;
    hipLaunchKernelGGL(wbc::wbc_qmap_count, dim3(nb), dim3(wbc::QMAP_THREADS), 0, st, masks, batch, scr);
    hipLaunchKernelGGL(wbc::wbc_qmap_plan, dim3(1), dim3(wbc::QMAP_THREADS), 0, st, batch, scr);
    hipLaunchKernelGGL(wbc::wbc_qmap_scatter, dim3(nb), dim3(wbc::QMAP_THREADS), 0, st, masks, batch,
                       static_cast<const int*>(scr), map, cap);
    return hipGetLastError();
}
extern "C" hipError_t wbc_launch_update(const wbc::KernelArgs* a, hipStream_t st) {
    hipLaunchKernelGGL(wbc::wbc_update_kernel, dim3((a->batch + wbc::UPD_RPW - 1) / wbc::UPD_RPW), dim3(64), 0, st, *a);
    return hipGetLastError();
}
// The split step's solve: the general kernel (one workgroup per QP), or, when the engine turned
// the stance elimination on, the stance kernel (one workgroup per QP) and the fallback kernel.
extern "C" hipError_t wbc_launch_solve_general(const wbc::KernelArgs* a, hipStream_t st) {
    hipLaunchKernelGGL(wbc::wbc_solve_kernel, dim3(a->batch), dim3(64), 0, st, *a);
    return hipGetLastError();
}
extern "C" hipError_t wbc_launch_solve_stance(const wbc::KernelArgs* a, hipStream_t st) {
    hipLaunchKernelGGL(wbc::wbc_solve_stance_kernel, dim3(a->batch), dim3(64), 0, st, *a);
    hipLaunchKernelGGL(wbc::wbc_solve_fallback_kernel, dim3(16), dim3(64), 0, st, *a);
    return hipGetLastError();
}
// The default step in one launch: the update kernel reducing and solving every QP inline, and the
// QPs whose reduction was not usable with the general method in the same wave (drain_fallbacks:
// their records carry their own mask and bounds, so the general solve runs them with modes = 0).
extern "C" hipError_t wbc_launch_update_solve(const wbc::KernelArgs* a, hipStream_t st) {
    static_assert(wbc::UPD_RPW == wbc::QMAP_SEG, "the wave map's segments are the kernel's");
    if (a->nwaves <= 0) return hipErrorInvalidValue;
    return a->stateful ? wbc_launch_update_solve1(a, st) : wbc_launch_update_solve0(a, st);
}
extern "C" hipError_t wbc_launch_reset(double* hist, const uint8_t* mask, int batch, hipStream_t st) {
    hipLaunchKernelGGL(wbc::wbc_reset_kernel, dim3(batch), dim3(64), 0, st, hist, mask, batch);
    return hipGetLastError();
}
#endif  // the one-kernel units

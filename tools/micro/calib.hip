// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE for the step kernel's own HBM access pattern
// (VERDICT r04 item 4).  MI355X_MICROARCH.md calibrates FETCH_SIZE only for wide coalesced streaming
// reads (16 B per lane: counted at half the bytes); the step reads robot-major rows of 56 / 144 / 96 /
// 432 B (base pose, nu, qj, ref: wbc_kernel.hip load_inputs, 8 B per lane, 16 lanes per robot, four
// robots per wave, scattered over the batch by the wave map) and writes 96 + 96 + 4 + 4 B per QP.
// Each kernel below reproduces one of the engine's patterns with nothing else in it, so its bytes
// are known exactly; a --pmc pass over this program gives FETCH_SIZE / WRITE_SIZE per launch, and
// known / counted is the factor for that pattern (tools/calib_summary.py).
//
//   calib_rows_stance   B = 4096, waves take four consecutive robots (no map): configs[1]
//   calib_rows_rl       B = 8192, the wave map of uniform random masks (qmap_build): configs[3]'s shard
//   calib_rows_modes    1024 states x 16 masks, four hypotheses per wave (wbc_modes_kernel's grid and
//                       xcd_block order; a state's row read by its K / M = 4 workgroups): configs[4]
//   calib_image         the LDS model image staged per workgroup (1024 workgroups): not algorithmic
//   calib_stream16      a 16 B/lane coalesced stream of the same bytes as calib_rows_stance: the
//                       guide's calibrated case, as a check of the method on this box
//
// Build: hipcc -O3 --offload-arch=gfx950 -I../../include -I../../quadrupedwholebodycontroller_amd/csrc calib.hip -o calib
// Run:   ./calib [launches]  (prints the known bytes per launch of every kernel as one JSON line)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "wbc_layout.h"

namespace {
constexpr int SUB = 16, RPW = 4, NIN = 91;

struct Rows {
    const double *pose, *nu, *qj, *ref;
    const uint8_t *contacts, *switching;
    double *tau, *grf;
    int32_t *status, *iters;
};

// one robot's 91 input doubles, as load_inputs<16> reads them (k = lane + 16 it, clamped to 90)
__device__ __forceinline__ double read_row(const Rows& r, int rb, int lane) {
    double acc = 0.0;
#pragma unroll
    for (int it = 0; it < (NIN + SUB - 1) / SUB; ++it) {
        const int k = (lane + it * SUB < NIN) ? lane + it * SUB : NIN - 1;
        const double* p = (k < 7) ? r.pose + (size_t)rb * 7 + k
                        : (k < 25) ? r.nu + (size_t)rb * 18 + (k - 7)
                        : (k < 37) ? r.qj + (size_t)rb * 12 + (k - 25)
                                   : r.ref + (size_t)rb * 54 + (k - 37);
        acc += *p;
    }
    return acc + (double)r.switching[rb];
}
__device__ __forceinline__ double seg_sum16(double v) {
#pragma unroll
    for (int o = 8; o >= 1; o >>= 1) v += __shfl_xor(v, o, 16);
    return v;
}
// one QP's outputs, as the step writes them (lanes 0..11: tau and grf; lane 0: status and iters)
__device__ __forceinline__ void write_out(const Rows& r, int qp, int lane, double v) {
    if (lane < 12) {
        r.tau[(size_t)qp * 12 + lane] = v + lane;
        r.grf[(size_t)qp * 12 + lane] = v - lane;
    }
    if (lane == 0) {
        r.status[qp] = (int32_t)v & 3;
        r.iters[qp] = (int32_t)v & 7;
    }
}

__global__ __launch_bounds__(64) void calib_rows_stance(Rows r, int B) {
    const int seg = threadIdx.x / SUB, lane = threadIdx.x % SUB;
    int rb = blockIdx.x * RPW + seg;
    const bool wr = rb < B;
    if (!wr) rb = B - 1;
    const int kap = r.contacts[rb] & 15;
    const double v = seg_sum16(read_row(r, rb, lane)) + kap;
    if (wr) write_out(r, rb, lane, v);
}

__global__ __launch_bounds__(64) void calib_rows_rl(Rows r, const int32_t* qmap) {
    const int seg = threadIdx.x / SUB, lane = threadIdx.x % SUB;
    const int4 e4 = reinterpret_cast<const int4*>(qmap)[blockIdx.x];
    const int e = (seg == 0) ? e4.x : (seg == 1) ? e4.y : (seg == 2) ? e4.z : e4.w;
    const bool wr = e >= 0;
    const int v0 = wr ? e : ~e, qp = v0 >> 4;
    const double v = seg_sum16(read_row(r, qp, lane)) + (v0 & 15);
    if (wr) write_out(r, qp, lane, v);
}

// wbc_kernel.hip xcd_block: a contiguous range of logical blocks per XCD
__device__ __forceinline__ int xcd_block(int b, int n) {
    const int x = b & 7, i = b >> 3, per = n >> 3, rem = n & 7;
    return x * per + min(x, rem) + i;
}
__global__ __launch_bounds__(64) void calib_rows_modes(Rows r, int S, int K, int M) {
    const int seg = threadIdx.x / SUB, lane = threadIdx.x % SUB;
    const int C = K / M, blk = xcd_block(blockIdx.x, gridDim.x), g = blk / C, c = blk - g * C;
    int row = 4 * g + seg;
    const bool wr = row < S;
    if (!wr) row = S - 1;
    const double v = seg_sum16(read_row(r, row, lane));
    for (int h = 0; h < M; ++h)
        if (wr) write_out(r, row * K + c * M + h, lane, v + h);
}

// A long straight-line body with no data reads: 24576 dependent v_fma_f64 on
// registers, ~96 KB of code, 1024 workgroups.  Its FETCH_SIZE is the instruction fetch a launch makes
// from HBM (each XCD's L2 misses the code once); the known bytes are 8 x its symbol size
// (tools/calib_summary.py reads the size from this binary's code object).
#define CODE_F1 a = fma(a, b, a);
#define CODE_F8 CODE_F1 CODE_F1 CODE_F1 CODE_F1 CODE_F1 CODE_F1 CODE_F1 CODE_F1
#define CODE_F64 CODE_F8 CODE_F8 CODE_F8 CODE_F8 CODE_F8 CODE_F8 CODE_F8 CODE_F8
#define CODE_F512 CODE_F64 CODE_F64 CODE_F64 CODE_F64 CODE_F64 CODE_F64 CODE_F64 CODE_F64
#define CODE_F4096 CODE_F512 CODE_F512 CODE_F512 CODE_F512 CODE_F512 CODE_F512 CODE_F512 CODE_F512
__global__ __launch_bounds__(64) void calib_code(double seed, double* out) {
    double a = seed + (double)threadIdx.x, b = seed * 0.5;
    CODE_F4096 CODE_F4096 CODE_F4096 CODE_F4096 CODE_F4096 CODE_F4096  // straight-line: a loop would be a few hundred bytes of code
    if (a == 12345.0) out[blockIdx.x] = a;  // never true: no write bytes
}

__global__ __launch_bounds__(64) void calib_image(const double* limg, double* out) {
    double acc = 0.0;
    for (int k = threadIdx.x; k < wbc::LIMG_LEN; k += 64) acc += limg[k];
    for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
    if (threadIdx.x == 0 && acc == 12345.0) out[blockIdx.x] = acc;  // never true: no write bytes
}

__global__ __launch_bounds__(256) void calib_stream16(const double2* src, double* out, size_t n2) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    double acc = 0.0;
    if (i < n2) {
        const double2 w = src[i];
        acc = w.x + w.y;
    }
    if (acc == 12345.0) out[0] = acc;  // never true: no write bytes
}

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(2);                                                             \
        }                                                                             \
    } while (0)

Rows alloc_rows(size_t B, size_t Bout) {
    Rows r{};
    double* d;
    CK(hipMalloc(&d, B * 91 * sizeof(double)));
    CK(hipMemset(d, 0, B * 91 * sizeof(double)));
    r.pose = d;
    r.nu = d + B * 7;
    r.qj = d + B * 25;
    r.ref = d + B * 37;
    uint8_t* m;
    CK(hipMalloc(&m, 2 * B));
    CK(hipMemset(m, 15, 2 * B));
    r.contacts = m;
    r.switching = m + B;
    CK(hipMalloc(&r.tau, Bout * 12 * sizeof(double)));
    CK(hipMalloc(&r.grf, Bout * 12 * sizeof(double)));
    CK(hipMalloc(&r.status, Bout * sizeof(int32_t)));
    CK(hipMalloc(&r.iters, Bout * sizeof(int32_t)));
    return r;
}
}  // namespace

int main(int argc, char** argv) {
    const int launches = argc > 1 ? std::atoi(argv[1]) : 20;
    // configs[1]: 4096 stance robots, no map
    const int B1 = 4096;
    Rows r1 = alloc_rows(B1, B1);
    // configs[3]'s shard: 8192 robots, uniform random masks, the host wave map
    const int B2 = 8192;
    Rows r2 = alloc_rows(B2, B2);
    std::vector<uint8_t> masks(B2);
    unsigned long long s = 0x9E3779B97F4A7C15ull;
    for (int b = 0; b < B2; ++b) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        masks[b] = (uint8_t)((s >> 33) & 15);
    }
    std::vector<int32_t> map(wbc::qmap_capacity(B2));
    const int waves2 = wbc::qmap_build(masks.data(), B2, map.data());
    int32_t* dmap;
    CK(hipMalloc(&dmap, map.size() * sizeof(int32_t)));
    CK(hipMemcpy(dmap, map.data(), map.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    // configs[4]'s shard: 1024 states x 16 masks, M = 4 hypotheses per wave
    const int S = 1024, K = 16, M = 4;
    Rows r3 = alloc_rows(S, (size_t)S * K);
    const int waves3 = (S / 4) * (K / M);
    // the LDS image (model + friction table)
    double *limg, *sink;
    CK(hipMalloc(&limg, wbc::LIMG_LEN * sizeof(double)));
    CK(hipMemset(limg, 0, wbc::LIMG_LEN * sizeof(double)));
    CK(hipMalloc(&sink, 4096 * sizeof(double)));
    // a 16 B/lane stream of calib_rows_stance's input bytes
    const size_t n2 = (size_t)B1 * 91 / 2;
    double2* src;
    CK(hipMalloc(&src, n2 * sizeof(double2)));
    CK(hipMemset(src, 0, n2 * sizeof(double2)));
    for (int i = 0; i < launches; ++i) {
        hipLaunchKernelGGL(calib_rows_stance, dim3(B1 / 4), dim3(64), 0, 0, r1, B1);
        hipLaunchKernelGGL(calib_rows_rl, dim3(waves2), dim3(64), 0, 0, r2, dmap);
        hipLaunchKernelGGL(calib_rows_modes, dim3(waves3), dim3(64), 0, 0, r3, S, K, M);
        hipLaunchKernelGGL(calib_image, dim3(1024), dim3(64), 0, 0, limg, sink);
        hipLaunchKernelGGL(calib_code, dim3(1024), dim3(64), 0, 0, 1e-9, sink);
        hipLaunchKernelGGL(calib_stream16, dim3((unsigned)((n2 + 255) / 256)), dim3(256), 0, 0, src, sink, n2);
    }
    CK(hipDeviceSynchronize());
    // known bytes per launch: each robot row once (91 doubles + contacts + switching byte; the map
    // words 16 B per wave), outputs 96 + 96 + 4 + 4 B per QP
    const double in_row = 91 * 8 + 2, in_row_nocon = 91 * 8 + 1, out_qp = 200;
    std::printf("{\"launches\": %d, "
                "\"calib_rows_stance\": {\"read\": %.0f, \"write\": %.0f, \"qps\": %d}, "
                "\"calib_rows_rl\": {\"read\": %.0f, \"write\": %.0f, \"qps\": %d, \"waves\": %d}, "
                "\"calib_rows_modes\": {\"read\": %.0f, \"write\": %.0f, \"qps\": %d, \"waves\": %d}, "
                "\"calib_image\": {\"read_per_workgroup\": %.0f, \"workgroups\": 1024, \"write\": 0}, "
                "\"calib_code\": {\"workgroups\": 1024, \"write\": 0, \"code\": \"8 x the symbol size\"}, "
                "\"calib_stream16\": {\"read\": %.0f, \"write\": 0}}\n",
                launches, B1 * in_row, B1 * out_qp, B1, B2 * in_row_nocon + waves2 * 16.0, B2 * out_qp, B2, waves2,
                S * in_row_nocon, (double)S * K * out_qp, S * K, waves3, wbc::LIMG_LEN * 8.0, n2 * 16.0);
    return 0;
}

// SIMD throughput with 1..4 waves per SIMD on a loaded chip: 256 blocks of 4 w waves (w per SIMD of
// each CU), every wave timed (s_memtime at its start and end; s_memrealtime beside it converts ticks
// to ns), after a warm-up launch that brings the clocks up.  Reported: the median wave's ticks per
// instruction and the chip aggregate (all waves' instructions over [first start, last end] per SIMD).
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 16
#define REP 256
template <int OP>
__global__ void k(double* out, unsigned long long* ts, double a, double b, int ia) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    double r[N]; int q[N];
#pragma unroll
    for (int u = 0; u < N; ++u) { r[u] = l + u; q[u] = l * u; }
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
#pragma unroll 1
    for (int i = 0; i < REP; ++i) {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            if constexpr (OP == 0) r[u] = fma(r[u], a, b);
            if constexpr (OP == 1) q[u] = q[u] + ia;
            if constexpr (OP == 2) {
                long long bb = __builtin_bit_cast(long long, r[u]);
                r[u] = __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(bb, 0x153, 0xF, 0xF, false));
            }
        }
#pragma unroll
        for (int u = 0; u < N; ++u) { asm volatile("" : "+v"(r[u])); asm volatile("" : "+v"(q[u])); }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int u = 0; u < N; ++u) s += r[u] + q[u];
    out[threadIdx.x] = s;
    const int g = blockIdx.x * (blockDim.x >> 6) + w;
    if (l == 0) { ts[4 * g] = t0; ts[4 * g + 1] = t1; ts[4 * g + 2] = r0; ts[4 * g + 3] = r1; }
}
#include <vector>
#include <algorithm>
int main() {
    const int NB = 256;
    double* out; unsigned long long* ts;
    (void)hipMalloc(&out, NB * 1024 * sizeof(double));
    (void)hipMalloc(&ts, 4 * 16 * NB * sizeof(unsigned long long));
    std::vector<unsigned long long> h(4 * 16 * NB);
    const char* names[] = {"fma f64", "add u32", "mov_b64_dpp"};
    for (int i = 0; i < 200; ++i) hipLaunchKernelGGL(k<0>, dim3(NB), dim3(64 * 16), 0, 0, out, ts, 0.999, 1e-3, 3);  // warm-up
    (void)hipDeviceSynchronize();
    for (int op = 0; op < 3; ++op) {
        for (int waves = 4; waves <= 16; waves += 4) {
            for (int rep = 0; rep < 5; ++rep) {
                if (op == 0) hipLaunchKernelGGL(k<0>, dim3(NB), dim3(64 * waves), 0, 0, out, ts, 0.999, 1e-3, 3);
                if (op == 1) hipLaunchKernelGGL(k<1>, dim3(NB), dim3(64 * waves), 0, 0, out, ts, 0.999, 1e-3, 3);
                if (op == 2) hipLaunchKernelGGL(k<2>, dim3(NB), dim3(64 * waves), 0, 0, out, ts, 0.999, 1e-3, 3);
            }
            const int nw = NB * waves;
            (void)hipMemcpy(h.data(), ts, sizeof(unsigned long long) * 4 * nw, hipMemcpyDeviceToHost);
            unsigned long long s0 = ~0ull, s1 = 0, q0 = ~0ull, q1 = 0;
            std::vector<double> per(nw);
            for (int w = 0; w < nw; ++w) {
                s0 = std::min(s0, h[4 * w]); s1 = std::max(s1, h[4 * w + 1]);
                q0 = std::min(q0, h[4 * w + 2]); q1 = std::max(q1, h[4 * w + 3]);
                per[w] = double(h[4 * w + 1] - h[4 * w]);
            }
            std::sort(per.begin(), per.end());
            const double ninst = double(REP) * N;
            printf("%-12s %d per SIMD: median wave %.2f ticks/instr (min %.2f), chip aggregate %.2f ticks/instr per SIMD, "
                   "%.3f ticks per ns\n", names[op], waves / 4, per[nw / 2] / ninst, per[0] / ninst,
                   double(s1 - s0) / (ninst * nw / 1024.0), double(s1 - s0) / (double(q1 - q0) * 10.0));
        }
    }
    return 0;
}

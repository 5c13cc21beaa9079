// Issue-rate microbenchmarks (one wave): 16 independent chains of one op type.
#include <hip/hip_runtime.h>
#include <cstdio>
#define N 16
#define REP 128
template <int OP>
__global__ void k(double* out, unsigned long long* cyc, double a, double b, int ia) {
    const int l = threadIdx.x;
    double r[N]; float f[N]; int q[N];
#pragma unroll
    for (int u = 0; u < N; ++u) { r[u] = l + u; f[u] = l + u; q[u] = l * u; }
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < REP; ++i) {
#pragma unroll
        for (int u = 0; u < N; ++u) {
            if constexpr (OP == 0) r[u] = fma(r[u], a, b);
            if constexpr (OP == 1) f[u] = fmaf(f[u], (float)a, (float)b);
            if constexpr (OP == 2) q[u] = q[u] * ia + 3;
            if constexpr (OP == 3) q[u] = q[u] + ia;
            if constexpr (OP == 4) {
                long long bb = __builtin_bit_cast(long long, r[u]);
                r[u] = __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(bb, 0x153, 0xF, 0xF, false));
            }
            if constexpr (OP == 5) r[u] = r[u] * a;
            if constexpr (OP == 6) r[u] = r[u] + a;
            if constexpr (OP == 7) q[u] = (q[u] > ia) ? q[u] : ia + u;
        }
#pragma unroll
        for (int u = 0; u < N; ++u) { asm volatile("" : "+v"(r[u])); asm volatile("" : "+v"(f[u])); asm volatile("" : "+v"(q[u])); }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int u = 0; u < N; ++u) s += r[u] + f[u] + q[u];
    out[l] = s;
    if (l == 0) cyc[OP] = t1 - t0;
}
int main() {
    double* out; unsigned long long* cyc;
    (void)hipMalloc(&out, 64 * 64 * sizeof(double));
    (void)hipMalloc(&cyc, 16 * sizeof(unsigned long long));
    unsigned long long h[16];
    const char* names[] = {"fma f64", "fma f32", "mul_lo u32", "add u32", "mov_b64_dpp", "mul f64", "add f64", "max/sel i32"};
    for (int waves = 1; waves <= 16; waves *= 2) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k<0>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<1>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<2>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<3>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<4>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<5>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<6>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            hipLaunchKernelGGL(k<7>, dim3(1), dim3(64 * waves), 0, 0, out, cyc, 0.999, 1e-3, 3);
            (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        }
        for (int i = 0; i < 8; ++i)
            if (i == 0 || i == 3 || i == 4)
                printf("block of %2d waves (%d per SIMD): %-12s %.2f cyc/instr (wave 0)\n", waves, (waves + 3) / 4, names[i],
                       h[i] / double(REP * N));
    }
    return 0;
}

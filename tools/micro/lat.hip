// Latency microbenchmarks (one wave): cycles per op of dependent fp64 FMA chains, independent
// chains, 64-bit DPP broadcast chains, LDS write->read round trips and broadcast reads.
#include <hip/hip_runtime.h>
#include <cstdio>

__device__ __forceinline__ double bc(double v) {
    long long b = __builtin_bit_cast(long long, v);
    return __builtin_bit_cast(double, (long long)__builtin_amdgcn_mov_dpp(b, 0x153, 0xF, 0xF, false));
}

__global__ void k(double* out, unsigned long long* cyc, double a, double b) {
    __shared__ double lds[1024];
    const int l = threadIdx.x;
    double x = l * 1e-3, y = x + 1, z = x + 2, w = x + 3;
    unsigned long long t0, t1;
    // 1: dependent fma chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) x = fma(x, a, b);
    }
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[0] = t1 - t0;
    // 2: four independent chains
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
#pragma unroll
        for (int u = 0; u < 2; ++u) { x = fma(x, a, b); y = fma(y, a, b); z = fma(z, a, b); w = fma(w, a, b); }
    }
    asm volatile("" : "+v"(x), "+v"(y), "+v"(z), "+v"(w));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[1] = t1 - t0;
    // 3: dependent dpp broadcast + add chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) x = bc(x) * a;
    }
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[2] = t1 - t0;
    // 4: LDS write -> read round trip chain (lane-owned address)
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
        lds[l] = x;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        x = lds[(l + 1) & 63] * a;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
    asm volatile("" : "+v"(x));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[3] = t1 - t0;
    // 5: dependent LDS read chain (address from the previous value, broadcast)
    for (int i = l; i < 1024; i += 64) lds[i] = (double)((i * 7 + 3) & 1023);
    __syncthreads();
    double p = 0;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) p = lds[(int)p];
    asm volatile("" : "+v"(p));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[4] = t1 - t0;
    // 6: rcp f64 dependent chain
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 256; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) y = __builtin_amdgcn_rcp(y) + a;
    }
    asm volatile("" : "+v"(y));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[5] = t1 - t0;
    // 7: 32 independent fmas per iteration (issue rate)
    double r[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) r[u] = x + u;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 1
    for (int i = 0; i < 128; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u) r[u] = fma(r[u], a, b);
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) asm volatile("" : "+v"(r[u]));
    t1 = __builtin_amdgcn_s_memtime();
    if (l == 0) cyc[6] = t1 - t0;
    double s = x + y + z + w + p;
#pragma unroll
    for (int u = 0; u < 16; ++u) s += r[u];
    out[l] = s;
}

int main() {
    double* out; unsigned long long* cyc;
    hipMalloc(&out, 64 * sizeof(double));
    hipMalloc(&cyc, 16 * sizeof(unsigned long long));
    unsigned long long h[16];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, out, cyc, 0.999, 1e-3);
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    }
    printf("dep fma       %.2f cyc/op\n", h[0] / 2048.0);
    printf("4 indep fma   %.2f cyc/op\n", h[1] / 2048.0);
    printf("dpp64 bcast*a %.2f cyc/(bcast+mul)\n", h[2] / 2048.0);
    printf("lds wr->rd    %.2f cyc/round trip\n", h[3] / 256.0);
    printf("lds dep read  %.2f cyc/read\n", h[4] / 256.0);
    printf("rcp+add dep   %.2f cyc/(rcp+add)\n", h[5] / 2048.0);
    printf("16 indep fma  %.2f cyc/op\n", h[6] / 2048.0);
    return 0;
}

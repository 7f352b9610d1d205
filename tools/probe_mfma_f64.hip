// Sweep of the fp64 MFMA issue rate: v_mfma_f64_16x16x4_f64 back to back with NACC
// independent accumulators per wave, WPS waves per SIMD on every CU, 2 s of launches;
// prints TFLOP/s and the in-kernel clock (s_memtime / s_memrealtime).  Diagnostic for
// the training leg's roofline peak (sml_probe_mfma_f64 uses NACC 8, WPS 2).
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_mfma_f64 tools/probe_mfma_f64.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k(int iters, double *sink, long long *st) {
    d4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    long long c0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) sink[0] = s;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = clock64() - c0;
        st[2 * blockIdx.x + 1] = wall_clock64() - r0;
    }
}

template <int NACC>
__global__ __launch_bounds__(256) void k4(int iters, double *sink, long long *st) {
    double acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    long long c0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    if (s == 12345.678) sink[0] = s;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = clock64() - c0;
        st[2 * blockIdx.x + 1] = wall_clock64() - r0;
    }
}

// a GEMM-like issue pattern: 4 A x 4 B operand registers, 16 accumulators, every
// MFMA a different (a, b) pair (the training kernels' inner loop)
template <int NACC>
__global__ __launch_bounds__(256) void k4g(int iters, double *sink, long long *st) {
    double acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = 0.0;
    double a[4], b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = 1.0 + (threadIdx.x + i) * 1e-9;
        b[i] = 1.0 - (threadIdx.x + i) * 1e-9;
    }
    long long c0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = __builtin_amdgcn_mov_dpp(0, 0, 0xf, 0xf, false) * 0.0 + a[i];
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) s += acc[i][j];
    if (s == 12345.678) sink[0] = s;
    if (threadIdx.x == 0) {
        st[2 * blockIdx.x] = clock64() - c0;
        st[2 * blockIdx.x + 1] = wall_clock64() - r0;
    }
}

template <int NACC, int kKind = 0>
void run(int ncu, int wps) {
    constexpr bool kSmall = kKind != 0;
    const int blocks = ncu * wps;  // 256 threads = 1 wave per SIMD per block
    double *sink;
    long long *st;
    hipMalloc(&sink, 8);
    hipMalloc(&st, 2 * blocks * sizeof(long long));
    const int iters = 20000;
    auto kern = kKind == 2 ? k4g<NACC> : kKind == 1 ? k4<NACC> : k<NACC>;
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters / 10, sink, st);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, sink, st);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(2 * blocks);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> f;
    for (int i = 0; i < blocks; ++i)
        if (h[2 * i + 1] > 0) f.push_back((double)h[2 * i] / h[2 * i + 1] * 0.1);
    std::sort(f.begin(), f.end());
    const double flops = (double)blocks * 4 * iters * NACC * 2.0 * 16 * 16 * 4;  // 4x4x4 x 16 blocks: the same 2048
    printf("%s NACC %2d  waves/SIMD %d: %7.2f TFLOP/s, clock %.3f GHz, %.1f clk per MFMA per SIMD\n",
           kKind == 2 ? "4x4x4 g" : kSmall ? "4x4x4  " : "16x16x4", NACC, wps, flops / (ms * 1e-3) / 1e12, f[f.size() / 2],
           (double)ms * 1e-3 * f[f.size() / 2] * 1e9 / ((double)iters * NACC * wps));
    hipFree(sink);
    hipFree(st);
}

int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int wps : {1, 2, 4}) {
        run<4>(ncu, wps);
        run<8>(ncu, wps);
        run<16>(ncu, wps);
        run<8, 1>(ncu, wps);
        run<16, 1>(ncu, wps);
        run<16, 2>(ncu, wps);
    }
    return 0;
}

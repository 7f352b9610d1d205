// probe: the Gram kernel's inner loop alone -- operands from an LDS stage, no global
// loads, no barriers -- 16x16x4 (a[4] x b[4], 16 MFMAs per k-step) against 4x4x4
// (a[4] x b[16] broadcast, 64 MFMAs per k-step), 256-thread blocks, WPS blocks per CU
//   hipcc --offload-arch=gfx950 -O3 -o tools/probe_lds_mfma tools/probe_lds_mfma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int LD = 144, KC = 16;
template <bool M4>
__global__ __launch_bounds__(256, 2) void k(int iters, double *sink, long long *st) {
    __shared__ double sA[KC][LD], sB[KC][LD];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1, l16 = lane & 15, kk = lane >> 4, l4 = lane & 3;
    for (int i = tid; i < KC * LD; i += 256) { (&sA[0][0])[i] = 1.0 + i * 1e-9; (&sB[0][0])[i] = 1.0 - i * 1e-9; }
    __syncthreads();
    d4 acc[4][4];
    double acc4[4][16];
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) acc[i][j] = d4{0, 0, 0, 0};
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 16; ++j) acc4[i][j] = 0;
    long long c0 = clock64(), r0 = wall_clock64();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int s = 0; s < KC / 4; ++s) {
            if (M4) {
                double a[4], b[16];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = sA[4 * s + kk][wr * 64 + i * 16 + l16];
#pragma unroll
                for (int c = 0; c < 16; ++c) b[c] = sB[4 * s + kk][wc * 64 + 4 * c + l4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int c = 0; c < 16; ++c) acc4[i][c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a[i], b[c], acc4[i][c], 0, 0, 0);
            } else {
                double a[4], b[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = sA[4 * s + kk][wr * 64 + i * 16 + l16];
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = sB[4 * s + kk][wc * 64 + j * 16 + l16];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[i], b[j], acc[i][j], 0, 0, 0);
            }
        }
    }
    double s = 0;
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 4; ++j) s += acc[i][j][0] + acc[i][j][3];
    for (int i = 0; i < 4; ++i) for (int j = 0; j < 16; ++j) s += acc4[i][j];
    if (s == 12345.678) sink[0] = s;
    if (tid == 0) { st[2 * blockIdx.x] = clock64() - c0; st[2 * blockIdx.x + 1] = wall_clock64() - r0; }
}
template <bool M4>
void run(int ncu, int wps) {
    const int blocks = ncu * wps;
    double *sink; long long *st;
    hipMalloc(&sink, 8); hipMalloc(&st, 2 * blocks * sizeof(long long));
    const int iters = 4000;
    hipLaunchKernelGGL((k<M4>), dim3(blocks), dim3(256), 0, 0, iters / 10, sink, st);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<M4>), dim3(blocks), dim3(256), 0, 0, iters, sink, st);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(2 * blocks);
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> f;
    for (int i = 0; i < blocks; ++i) if (h[2 * i + 1] > 0) f.push_back((double)h[2 * i] / h[2 * i + 1] * 0.1);
    std::sort(f.begin(), f.end());
    const double flops = (double)blocks * 4 * iters * (KC / 4) * 16 * 2048.0;  // both: 32K flop per k-step per wave
    printf("%s blocks/CU %d: %7.2f TFLOP/s (%.3f of 78.6), clock %.3f GHz\n", M4 ? "4x4x4  " : "16x16x4", wps,
           flops / (ms * 1e-3) / 1e12, flops / (ms * 1e-3) / 1e12 / 78.6, f[f.size() / 2]);
    hipFree(sink); hipFree(st);
}
int main() {
    int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int wps : {1, 2}) { run<false>(ncu, wps); run<true>(ncu, wps); }
    return 0;
}

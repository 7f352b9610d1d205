// Diagnostic: cycles per f64 VALU instruction for one wave per SIMD vs two (and four)
// waves per SIMD -- decides whether splitting one FFT's butterflies over two waves of
// a SIMD can shorten it.  Build: hipcc --offload-arch=gfx950 -O3 tools/probe_f64_issue.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int CH>
__global__ void k_chain(double *out, long long *cyc, int iters) {
    double a[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = threadIdx.x * 1e-3 + c;
    const double b = 1.0000001, d = 1e-9;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) a[c] = a[c] * b + d;  // (contracted to one v_fma_f64)
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

int main() {
    double *out;
    long long *cyc;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 1 << 16);
    const int iters = 4096;
    for (int threads : {64, 256, 512, 1024}) {
        for (int rep = 0; rep < 2; ++rep) {
            hipLaunchKernelGGL(k_chain<8>, dim3(1), dim3(threads), 0, 0, out, cyc, iters);
            hipDeviceSynchronize();
        }
        std::vector<long long> c(threads / 64);
        hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
        long long mx = 0;
        for (auto v : c) mx = v > mx ? v : mx;
        printf("8 indep chains, %4d threads (%d waves/SIMD): %.2f cycles per f64 FMA per wave\n", threads,
               threads / 256 > 0 ? threads / 256 : 1, (double)mx / (iters * 8.0));
    }
    for (int threads : {64, 256, 512}) {
        hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(threads), 0, 0, out, cyc, iters);
        hipDeviceSynchronize();
        hipLaunchKernelGGL(k_chain<1>, dim3(1), dim3(threads), 0, 0, out, cyc, iters);
        hipDeviceSynchronize();
        long long c0;
        hipMemcpy(&c0, cyc, 8, hipMemcpyDeviceToHost);
        printf("1 dependent chain, %4d threads: %.2f cycles per f64 FMA\n", threads, (double)c0 / iters);
    }
    return 0;
}

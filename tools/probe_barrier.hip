// Probe: the per-step floor of a 128-step LDS publish / barrier / read loop, as the
// diagonal-factor kernels (k_chol_diag / k_chol_diag_reg) run it, one 512-thread block
// per CU on 144 CUs.  Variants: plain s_barrier with LDS-only fences; __syncthreads;
// plus a dependent f64 sqrt / divide per step; plus a 32-way select chain per step.
//   hipcc --offload-arch=gfx950 -O3 tools/probe_barrier.hip -o tools/probe_barrier
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int kMode>  // 0 lds barrier, 1 __syncthreads, 2 + sqrt/div, 3 + select chain
__global__ __launch_bounds__(512) void k_probe(double *out, int steps) {
    __shared__ double w[2][128];
    const int tid = threadIdx.x, i = tid & 127;
    double acc = 1.0 + tid, a[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) a[m] = m + tid;
    for (int j = 0; j < steps; ++j) {
        const int p = j & 1;
        if ((tid >> 7) == (j & 3)) {
            double v = acc;
            if constexpr (kMode == 3) {
#pragma unroll
                for (int m = 0; m < 32; ++m) v = m == (j >> 2) ? a[m] : v;
            }
            w[p][i] = v;
        }
        if constexpr (kMode == 1)
            __syncthreads();
        else
            lds_barrier();
        double d = w[p][j & 127];
        if constexpr (kMode >= 2) d = 1.0 / sqrt(d * d + 1.0);
        acc += d * w[p][i];
        a[j & 31] += d;
    }
    double s = acc;
#pragma unroll
    for (int m = 0; m < 32; ++m) s += a[m];
    out[blockIdx.x * 512 + tid] = s;
}

int main() {
    double *out = nullptr;
    CK(hipMalloc(&out, 144 * 512 * sizeof(double)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[4] = {"lds-only barrier", "__syncthreads", "+ sqrt/div", "+ select chain"};
    for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 3; ++rep) {
            CK(hipEventRecord(e0, 0));
            for (int it = 0; it < 10; ++it) {
                if (mode == 0) hipLaunchKernelGGL(k_probe<0>, dim3(144), dim3(512), 0, 0, out, 128);
                if (mode == 1) hipLaunchKernelGGL(k_probe<1>, dim3(144), dim3(512), 0, 0, out, 128);
                if (mode == 2) hipLaunchKernelGGL(k_probe<2>, dim3(144), dim3(512), 0, 0, out, 128);
                if (mode == 3) hipLaunchKernelGGL(k_probe<3>, dim3(144), dim3(512), 0, 0, out, 128);
            }
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms = 0;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 2) std::printf("%-18s %.3f us per 128-step launch, %.3f us per step\n", names[mode], ms * 100.0,
                                      ms * 100.0 / 128.0);
        }
    }
    CK(hipFree(out));
    return 0;
}

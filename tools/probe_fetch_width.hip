// Calibration probe for rocprofv3's FETCH_SIZE at the access widths the state update
// (k_res_update_bal) issues: coalesced 4-B and 8-B loads per lane (the ELL slot pairs'
// u16 column pairs and f32 value pairs, W_in's f32 values, the f64 state), and the
// 16-B loads whose factor the guide states (MI355X_MICROARCH.md, HBM: FETCH_SIZE
// reports 1/2 of a wide coalesced streaming read; other widths uncalibrated).
// Each kernel reads a known byte count once (2 GiB, past the 256 MiB Infinity Cache)
// and writes one double per block; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- tools/probe_fetch_width
// and divide each kernel's FETCH_SIZE (KB) by the bytes printed here.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_fetch_width.hip -o tools/probe_fetch_width
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

typedef double dv2 __attribute__((ext_vector_type(2)));

template <typename T>
__device__ inline double val(const T &v);
template <>
__device__ inline double val<unsigned>(const unsigned &v) { return (double)v; }
template <>
__device__ inline double val<double>(const double &v) { return v; }
template <>
__device__ inline double val<dv2>(const dv2 &v) { return v.x + v.y; }

// grid-stride coalesced read of n elements of T (consecutive lanes, consecutive elements)
template <typename T>
__global__ __launch_bounds__(256) void k_read(const T *__restrict__ p, size_t n, double *__restrict__ sink) {
    double s = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += val<T>(__builtin_nontemporal_load(p + i));
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < 256; ++i) t += red[i];
        sink[blockIdx.x] = t;
    }
}

// the update's mix per row pass: one 4-B and one 8-B load per lane from two arrays
__global__ __launch_bounds__(256) void k_read_pair(const unsigned *__restrict__ c, const double *__restrict__ v, size_t n,
                                                  double *__restrict__ sink) {
    double s = 0.0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        s += (double)__builtin_nontemporal_load(c + i) * __builtin_nontemporal_load(v + i);
    __shared__ double red[256];
    red[threadIdx.x] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int i = 0; i < 256; ++i) t += red[i];
        sink[blockIdx.x] = t;
    }
}

int main() {
    const size_t bytes = (size_t)2 << 30;  // 2 GiB per kernel
    char *buf = nullptr;
    double *sink = nullptr;
    CK(hipMalloc(&buf, bytes + (bytes / 3)));
    CK(hipMemset(buf, 1, bytes + (bytes / 3)));
    const int blocks = 256 * 8;
    CK(hipMalloc(&sink, blocks * sizeof(double)));
    CK(hipDeviceSynchronize());
    hipLaunchKernelGGL(k_read<unsigned>, dim3(blocks), dim3(256), 0, 0, (const unsigned *)buf, bytes / 4, sink);
    hipLaunchKernelGGL(k_read<double>, dim3(blocks), dim3(256), 0, 0, (const double *)buf, bytes / 8, sink);
    hipLaunchKernelGGL(k_read<dv2>, dim3(blocks), dim3(256), 0, 0, (const dv2 *)buf, bytes / 16, sink);
    // the pair: n elements of 4 B + 8 B = 12 n bytes ~ 2 GiB
    const size_t np = bytes / 12;
    hipLaunchKernelGGL(k_read_pair, dim3(blocks), dim3(256), 0, 0, (const unsigned *)buf,
                       (const double *)(buf + ((np * 4 + 255) & ~(size_t)255)), np, sink);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::printf("{\"k_read<unsigned>\": %zu, \"k_read<double>\": %zu, \"k_read<double2>\": %zu, \"k_read_pair\": %zu}\n",
                bytes, bytes, bytes, np * 12);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}

// Diagnostic partners for tools/probe_phase_contention.py: a streaming read of a
// buffer with non-temporal loads (as the reservoir's W_out / A streams) or plain
// loads (L2-allocating), 16 B per lane, launched on the caller's stream.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/stream_partner.hip -o tools/libstream_partner.so
#include <hip/hip_runtime.h>

typedef double dv2 __attribute__((ext_vector_type(2)));

template <bool kNT>
__global__ __launch_bounds__(256) void k_read(const dv2 *src, size_t n, double *sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const dv2 v = kNT ? __builtin_nontemporal_load(src + i) : src[i];
        acc += v.x + v.y;
    }
    if (acc == 12345.678) sink[0] = acc;  // (never: keeps the loads)
}

extern "C" int sp_read(const void *src, size_t bytes, double *sink, int nt, int blocks, void *stream) {
    const size_t n = bytes / sizeof(dv2);
    if (nt)
        hipLaunchKernelGGL(k_read<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const dv2 *)src, n, sink);
    else
        hipLaunchKernelGGL(k_read<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const dv2 *)src, n, sink);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}

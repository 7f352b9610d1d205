// Diagnostic: the latency of a dependency between two CU-masked streams on one
// device, from in-kernel wall-clock stamps (100 MHz).  Producer on CUs [0, 64),
// consumer on [64, 224), the hybrid step's layout.  Each case: producer kernel
// (busy 200 us so the host has queued everything) -> dependency -> consumer's
// first instruction; the figure is consumer start - producer end.
//   hipcc --offload-arch=gfx950 -O2 tools/probe_hop.hip -o tools/probe_hop && tools/probe_hop
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

typedef unsigned long long u64;

__global__ void k_work(u64 ticks, u64 *stamp, u64 *flag, u64 val) {
    const u64 t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        stamp[blockIdx.x] = wall_clock64();
        if (flag) {
            __threadfence();
            __hip_atomic_fetch_add(flag, val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// producer that also leaves `n` doubles written (how = 0: plain stores, 1: non-temporal,
// 2: agent-scope relaxed atomic stores, which write through L2)
__global__ void k_write(u64 ticks, u64 *stamp, double *buf, int n, int how) {
    const u64 t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (how == 0) buf[i] = (double)i;
        else if (how == 1) __builtin_nontemporal_store((double)i, buf + i);
        else __hip_atomic_store(buf + i, (double)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (threadIdx.x == 0) stamp[blockIdx.x] = wall_clock64();
}

__global__ void k_stamp(u64 *stamp) {
    if (threadIdx.x == 0) stamp[blockIdx.x] = wall_clock64();
}

// pre-launched consumer: waits for the flag to reach `target` (bounded: 0.5 s)
__global__ void k_wait(const u64 *flag, u64 target, u64 *stamp) {
    if (threadIdx.x == 0) {
        const u64 t0 = wall_clock64();
        while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 50000000ull) break;
        }
        stamp[blockIdx.x] = wall_clock64();
    }
    __syncthreads();
}

static hipStream_t cu_stream(int first, int n) {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = first; c < first + n && c < ncu; ++c) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    return s;
}

int main() {
    hipStream_t sa = cu_stream(0, 64), sb = cu_stream(64, 160);
    u64 *d_st, *d_flag;
    const int kReps = 24, kPB = 48, kCB = 48;
    CK(hipMalloc(&d_st, sizeof(u64) * 2 * 64));
    CK(hipMalloc(&d_flag, sizeof(u64)));
    CK(hipMemset(d_flag, 0, sizeof(u64)));
    hipEvent_t ev_nt, ev_t;
    CK(hipEventCreateWithFlags(&ev_nt, hipEventDisableTiming));
    CK(hipEventCreate(&ev_t));
    std::vector<u64> h(2 * 64);
    u64 flagv = 0;
    const u64 busy = 20000;  // 200 us
    const char *names[] = {"same stream (consumer on the producer's stream)", "event, timing disabled",
                           "event, timing enabled", "stream write/wait value", "pre-launched spin on a flag"};
    for (int mode = 0; mode < 5; ++mode) {
        std::vector<double> gaps;
        for (int r = 0; r < kReps; ++r) {
            CK(hipDeviceSynchronize());
            u64 *ps = d_st, *cs = d_st + 64;
            hipStream_t cons = mode == 0 ? sa : sb;
            if (mode == 4) {
                hipLaunchKernelGGL(k_wait, dim3(kCB), dim3(64), 0, cons, d_flag, (flagv + 1) * kPB, cs);
                hipLaunchKernelGGL(k_work, dim3(kPB), dim3(256), 0, sa, busy, ps, d_flag, 1ull);
                ++flagv;
            } else {
                hipLaunchKernelGGL(k_work, dim3(kPB), dim3(256), 0, sa, busy, ps, (u64 *)nullptr, 0ull);
                if (mode == 1 || mode == 2) {
                    hipEvent_t e = mode == 1 ? ev_nt : ev_t;
                    CK(hipEventRecord(e, sa));
                    CK(hipStreamWaitEvent(cons, e, 0));
                } else if (mode == 3) {
                    ++flagv;
                    CK(hipStreamWriteValue64(sa, d_flag, flagv * kPB, 0));
                    CK(hipStreamWaitValue64(cons, d_flag, flagv * kPB, hipStreamWaitValueGte, ~0ull));
                }
                hipLaunchKernelGGL(k_stamp, dim3(kCB), dim3(64), 0, cons, cs);
            }
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h.data(), d_st, sizeof(u64) * 128, hipMemcpyDeviceToHost));
            u64 pend = 0, cstart = ~0ull;
            for (int b = 0; b < kPB; ++b) pend = std::max(pend, h[b]);
            for (int b = 0; b < kCB; ++b) cstart = std::min(cstart, h[64 + b]);
            if (r >= 4) gaps.push_back(((double)cstart - (double)pend) * 0.01);
        }
        std::sort(gaps.begin(), gaps.end());
        std::printf("%-50s median %7.2f us  min %7.2f  max %7.2f\n", names[mode], gaps[gaps.size() / 2], gaps[0],
                    gaps.back());
    }
    // kernel boundary on one stream after the producer wrote `mb` MB
    double *d_buf;
    CK(hipMalloc(&d_buf, 64ull << 20));
    const char *hows[] = {"plain stores", "non-temporal stores", "agent-scope atomic stores"};
    for (int mb : {0, 1, 2, 8}) {
        for (int how = 0; how < 3; ++how) {
            std::vector<double> gaps;
            for (int r = 0; r < kReps; ++r) {
                CK(hipDeviceSynchronize());
                hipLaunchKernelGGL(k_write, dim3(kPB), dim3(256), 0, sa, busy, d_st, d_buf, mb << 17, how);
                hipLaunchKernelGGL(k_stamp, dim3(kCB), dim3(64), 0, sa, d_st + 64);
                CK(hipGetLastError());
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(h.data(), d_st, sizeof(u64) * 128, hipMemcpyDeviceToHost));
                u64 pend = 0, cstart = ~0ull;
                for (int b = 0; b < kPB; ++b) pend = std::max(pend, h[b]);
                for (int b = 0; b < kCB; ++b) cstart = std::min(cstart, h[64 + b]);
                if (r >= 4) gaps.push_back(((double)cstart - (double)pend) * 0.01);
            }
            std::sort(gaps.begin(), gaps.end());
            std::printf("same stream after %d MB of %-26s median %7.2f us  min %7.2f  max %7.2f\n", mb, hows[how],
                        gaps[gaps.size() / 2], gaps[0], gaps.back());
        }
    }
    return 0;
}

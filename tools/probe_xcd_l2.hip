// Diagnostic: does an XCD's L2 keep data across a kernel boundary for a reader on
// the same XCD, and where do SPEEDY's blocks land?  Stream on CUs [0, 64) (the
// window's), 62 blocks of 512 threads (one per CU, as k_st_spec).  Kernel W: block b
// writes chunk b (40 KB, plain stores) and records its XCC_ID; kernel R (next launch,
// same stream): block b reads chunk b and stamps the time from its first load to the
// loaded data (wall_clock64, 100 MHz), records its XCC_ID.  Over many launches the
// dispatcher puts reader and writer on the same or on different XCDs; the latency is
// reported per case, alone and beside a streaming read on CUs [64, 256).
//   hipcc --offload-arch=gfx950 -O3 tools/probe_xcd_l2.hip -o tools/probe_xcd_l2 && tools/probe_xcd_l2
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef unsigned long long u64;
constexpr int kBlocks = 62, kThreads = 512, kChunk = 5120;  // doubles per chunk (40 KB)

__device__ inline unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ __launch_bounds__(kThreads) void k_write(double *buf, int *wx, double val) {
    __shared__ double pad[18000];  // one block per CU (LDS), as the window's kernels
    pad[threadIdx.x] = val;
    double *c = buf + (size_t)blockIdx.x * kChunk;
    for (int i = threadIdx.x; i < kChunk; i += kThreads) c[i] = val + i + pad[threadIdx.x & 7] * 0.0;
    if (threadIdx.x == 0) wx[blockIdx.x] = (int)xcc_id();
}

__global__ __launch_bounds__(kThreads) void k_read(const double *buf, int *rx, u64 *lat, double *sink, int shift) {
    __shared__ double pad[18000];
    const double *c = buf + (size_t)((blockIdx.x + shift) % kBlocks) * kChunk;
    __syncthreads();
    const u64 t0 = wall_clock64();
    double s = 0.0;
    double v[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) v[q] = c[threadIdx.x + q * kThreads];
#pragma unroll
    for (int q = 0; q < 10; ++q) s += v[q];
    pad[threadIdx.x] = s;
    __syncthreads();
    const u64 t1 = wall_clock64();
    if (threadIdx.x == 0) {
        rx[blockIdx.x] = (int)xcc_id();
        lat[blockIdx.x] = t1 - t0;
        sink[blockIdx.x] = pad[5];
    }
}

// busy for `ticks` of the 100-MHz clock (the rest of a step between two reads)
__global__ void k_spin(u64 ticks) {
    const u64 t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) {
    }
}

typedef double dv4 __attribute__((ext_vector_type(4)));
__global__ void k_stream(const dv4 *src, size_t n, double *sink) {
    double acc = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const dv4 v = __builtin_nontemporal_load(src + i);
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.0) sink[0] = acc;
}

// mask of logical CUs c with pred(c)
template <class P>
static hipStream_t cu_stream(P pred) {
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = 0; c < ncu; ++c)
        if (pred(c)) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    return s;
}

static double median(std::vector<double> v) {
    if (v.empty()) return -1.0;
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

// one layout: placement, the 40-KB read of the previous kernel's output (own chunk =
// same block index, i.e. the same XCD if placement is stable; a neighbour's chunk),
// and the write -> read launch pair, alone and beside the partner stream
static void run(hipStream_t sa, hipStream_t sb, const char *name) {
    double *buf, *sink;
    int *wx, *rx;
    u64 *lat;
    CK(hipMalloc(&buf, sizeof(double) * kChunk * kBlocks));
    CK(hipMalloc(&sink, sizeof(double) * 64));
    CK(hipMalloc(&wx, sizeof(int) * 64));
    CK(hipMalloc(&rx, sizeof(int) * 64));
    CK(hipMalloc(&lat, sizeof(u64) * 64));
    const size_t nbig = (size_t)3 << 30;  // 3 GB partner stream
    dv4 *big;
    CK(hipMalloc(&big, nbig));
    CK(hipMemset(big, 0, nbig));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<int> hw(64), hr(64);
    std::vector<u64> hl(64);
    std::printf("== %s\n", name);
    for (int partner = 0; partner < 2; ++partner) {
        // shift -1: the chunks were written once, long ago; each rep spins 30 us on the
        // window's CUs and then re-reads its own chunk (L2 retention beside a stream)
        for (int shift : {0, 1, 5, -1}) {
            std::map<int, int> placement;  // xcc -> blocks
            std::vector<double> same, other, pair;
            int stable = 0, total = 0;
            std::vector<int> prev(64, -1);
            for (int rep = 0; rep < 150; ++rep) {
                if (partner && hipStreamQuery(sb) == hipSuccess)  // keep the partner stream running
                    hipLaunchKernelGGL(k_stream, dim3(192 * 8), dim3(256), 0, sb, big, nbig / sizeof(dv4), sink);
                CK(hipEventRecord(e0, sa));
                if (shift >= 0 || rep == 0)
                    hipLaunchKernelGGL(k_write, dim3(kBlocks), dim3(kThreads), 0, sa, buf, wx, (double)rep);
                if (shift < 0) hipLaunchKernelGGL(k_spin, dim3(kBlocks), dim3(64), 0, sa, 3000ull);
                hipLaunchKernelGGL(k_read, dim3(kBlocks), dim3(kThreads), 0, sa, buf, rx, lat, sink, shift < 0 ? 0 : shift);
                CK(hipEventRecord(e1, sa));
                CK(hipGetLastError());
                CK(hipStreamSynchronize(sa));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemcpy(hw.data(), wx, sizeof(int) * 64, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hr.data(), rx, sizeof(int) * 64, hipMemcpyDeviceToHost));
                CK(hipMemcpy(hl.data(), lat, sizeof(u64) * 64, hipMemcpyDeviceToHost));
                if (rep < 4) continue;
                pair.push_back(ms * 1e3);
                for (int b = 0; b < kBlocks; ++b) {
                    placement[hr[b]]++;
                    const int w = hw[(b + (shift < 0 ? 0 : shift)) % kBlocks];
                    (w == hr[b] ? same : other).push_back(hl[b] * 0.01);
                    if (prev[b] >= 0) {
                        ++total;
                        stable += prev[b] == hr[b];
                    }
                    prev[b] = hr[b];
                }
            }
            CK(hipDeviceSynchronize());
            std::printf("%s, reader of chunk b + %d: blocks per XCC:", partner ? "beside a stream" : "alone", shift);
            for (auto &kv : placement) std::printf(" %d:%d", kv.first, kv.second);
            std::printf("; same XCC as last launch %d/%d\n", stable, total);
            std::printf("  40-KB read of the previous kernel's output: writer on the same XCC %.2f us (n=%zu), "
                        "another XCC %.2f us (n=%zu); write+read pair %.2f us\n",
                        median(same), same.size(), median(other), other.size(), median(pair));
        }
    }
    CK(hipFree(buf));
    CK(hipFree(big));
    CK(hipFree(sink));
    CK(hipFree(wx));
    CK(hipFree(rx));
    CK(hipFree(lat));
}

int main(int argc, char **argv) {
    // layout 0: the window's CUs [0, 64) (interleaved over the XCDs), partner [64, 256)
    // layout 1: the window on the logical CUs c % 8 in {0, 1} (2 whole XCDs if c % 8 is the XCD)
    // layout 2: the window on the logical CUs with (c / 8) % 8 in {0, 1}: observed
    //   [0, 64) = 8 CUs on each XCD, so c / 8 mod 8 would be the XCD
    const char *names[] = {"window on CUs [0, 64)", "window on c % 8 in {0,1}", "window on (c / 8) % 8 in {0,1}"};
    for (int layout = 0; layout < 3; ++layout) {
        if (argc > 1 && std::atoi(argv[1]) != layout) continue;
        auto inA = [&](int c) { return layout == 0 ? c < 64 : layout == 1 ? (c % 8) < 2 : ((c / 8) % 8) < 2; };
        hipStream_t sa = cu_stream(inA), sb = cu_stream([&](int c) { return !inA(c); });
        run(sa, sb, names[layout]);
        CK(hipStreamDestroy(sa));
        CK(hipStreamDestroy(sb));
    }
    return 0;
}

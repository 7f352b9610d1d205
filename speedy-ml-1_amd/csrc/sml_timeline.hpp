// sml_timeline.hpp -- per-launch start / end times of the hybrid step's kernels, for
// the step accounting (tools/step_accounting.py).  Profiling build
// only: compiled in with -DSML_TL (tools/build_variant.sh tl 'EXTRA=-DSML_TL'); the
// product build has empty macros and no buffer.
//
// Each instrumented kernel's thread 0 of every block records the block's start and end
// (wall_clock64, 100 MHz) in a per-(kind, launch, block) slot with plain stores; the
// host takes a launch's start / end as the min / max over its blocks.  Untraced and
// inside the window graph alike: no launch argument changes.
#pragma once
#include <cstdint>

namespace sml {
namespace tl {
enum Kind {
    kEntrySpecx = 0,  // iogrid(30)'s entry specx (waits in-kernel for the assembled grid)
    kIoEntry,         // k_io_entry
    kRow,             // k_st_gridspec_p
    kSpec,            // k_st_spec
    kExitGridx,       // run_model's exit (iogrid(31)'s gridx + q floor)
    kExitStore,       // the forecast hop's store behind the exit
    kFinish,          // the v_p finish (+ local-model tiling, + one-rank assembly)
    kHopSignal,       // a hop's one-lane signal kernel
    kTileFeedback,    // k_tile_feedback
    kUpdate,          // the balanced state update
    kReadout,         // the W_out readout
    kFordate,         // k_fordate
    kCheckMinmax,     // the safety check's min / max
    kAssemble,        // k_assemble (the exchanged outvecs into the global grids, world > 1)
    kKinds
};
// per kind: launches kept (a ring) and blocks recorded per launch (blocks past it are
// not recorded; every grid of the step fits)
constexpr int kRingOf[kKinds] = {1024, 1024, 16384, 16384, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024};
constexpr int kBlocksOf[kKinds] = {64, 64, 64, 64, 64, 1, 2048, 1, 1024, 2048, 8192, 32, 4, 1024};
constexpr int kMaxBlocks = 8192;
// the log of a kind: [ring][blocks] of (start, end) wall_clock64 (100 MHz), the shader
// clock's counter (clock64, s_memtime) at the same two points -- their ratio is the
// clock the block ran at -- and the launch's grid size (block b's record count advances
// only in launches with more than b blocks: the host walks block 0's records and the
// grid sizes to match the other blocks' records to launches)
constexpr int kWords = 5;
constexpr long long log_offset(int kind) {
    long long o = 0;
    for (int k = 0; k < kind; ++k) o += (long long)kRingOf[k] * kBlocksOf[k] * kWords;
    return o;
}
constexpr long long kLogWords = log_offset(kKinds);
struct Buf {
    unsigned cnt[kKinds][kMaxBlocks];  // launches of the kind each block index has recorded
    unsigned long long log[kLogWords];
};
}  // namespace tl

// host: attach a buffer to every translation unit's kernels (sml_dbg_timeline)
int tl_attach_dynamics(tl::Buf *b);
int tl_attach_spectral(tl::Buf *b);
int tl_attach_reservoir(tl::Buf *b);
int tl_attach_hybrid(tl::Buf *b);
}  // namespace sml

#ifdef __HIPCC__
#ifdef SML_TL
// one pointer per translation unit (no relocatable device code), set by tl_attach_*;
// SML_TL_SCOPE(kind) at a kernel's start (or after its in-kernel wait): thread 0 of
// block b reads how many launches of the kind block b has recorded (launches of one
// kind run in order on one stream: no other writer) and its start time; its destructor
// -- at whatever return thread 0 takes -- stores (start, end) into that launch's slot
// and the count + 1: plain stores, no atomics, no wait at the block's end.
// kind < 0: not recorded (a shared kernel in another role)
#define SML_TL_DEFINE(unit)                                                                    \
    namespace {                                                                                \
    __device__ sml::tl::Buf *g_tl = nullptr;                                                   \
    struct TlScope {                                                                           \
        int kind;                                                                              \
        unsigned c = 0;                                                                        \
        unsigned long long s = 0, sc = 0;                                                      \
        __device__ explicit TlScope(int k) : kind(k) {                                         \
            const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);      \
            if (kind >= 0 && (threadIdx.x != 0 || !g_tl || b >= sml::tl::kBlocksOf[kind])) kind = -1; \
            if (kind >= 0) {                                                                   \
                c = g_tl->cnt[kind][b];                                                        \
                s = wall_clock64();                                                            \
                sc = clock64();                                                                \
            }                                                                                  \
        }                                                                                      \
        __device__ ~TlScope() {                                                                \
            if (kind < 0) return;                                                              \
            const int b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);      \
            const unsigned long long e = wall_clock64(), ec = clock64();                       \
            unsigned long long *l = g_tl->log + sml::tl::log_offset(kind) +                    \
                                    sml::tl::kWords * ((long long)(c % sml::tl::kRingOf[kind]) * sml::tl::kBlocksOf[kind] + b); \
            l[0] = s;                                                                          \
            l[1] = e;                                                                          \
            l[2] = sc;                                                                         \
            l[3] = ec;                                                                         \
            l[4] = gridDim.x * gridDim.y * gridDim.z;                                          \
            g_tl->cnt[kind][b] = c + 1;                                                        \
        }                                                                                      \
    };                                                                                         \
    }                                                                                          \
    int sml::tl_attach_##unit(sml::tl::Buf *b) {                                               \
        return hipMemcpyToSymbol(HIP_SYMBOL(g_tl), &b, sizeof b) == hipSuccess ? 0 : -2;       \
    }
#define SML_TL_SCOPE(kind) TlScope sml_tl_scope_(kind)
#else
#define SML_TL_DEFINE(unit) \
    int sml::tl_attach_##unit(sml::tl::Buf *) { return -1; }
#define SML_TL_SCOPE(kind) (void)0
#endif
#endif

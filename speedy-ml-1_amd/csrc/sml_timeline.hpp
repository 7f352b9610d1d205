// sml_timeline.hpp -- per-launch start / end times of the hybrid step's kernels, for
// the step accounting (tools/step_accounting.py).  Profiling build
// only: compiled in with -DSML_TL (tools/build_variant.sh tl 'EXTRA=-DSML_TL'); the
// product build has empty macros and no buffer.
//
// Each instrumented kernel's thread 0 of every block reads the kind's launch number at
// its start (launches of one kind run on one stream, in order, so every block of a
// launch reads the same number), and at its end folds its block's start and end
// wall_clock64 (100 MHz) into that launch's slot -- min of the starts, max of the ends
// -- then counts its arrival; the launch's last block bumps the number.  Untraced and
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
    kKinds
};
constexpr int kRing = 16384;
struct Buf {
    unsigned long long seq[kKinds];
    unsigned arrivals[kKinds];
    unsigned long long t0[kKinds][kRing];  // min of the blocks' starts (init ~0)
    unsigned long long t1[kKinds][kRing];  // max of the blocks' ends (init 0)
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
// SML_TL_SCOPE(kind) at a kernel's start (or after its in-kernel wait): thread 0 of the
// block reads the launch number and its start time, and its destructor -- at whatever
// return thread 0 takes -- folds the block's start / end in and counts the arrival.
// kind < 0: not recorded (a shared kernel in another role)
#define SML_TL_DEFINE(unit)                                                                    \
    namespace {                                                                                \
    __device__ sml::tl::Buf *g_tl = nullptr;                                                   \
    struct TlScope {                                                                           \
        int kind;                                                                              \
        unsigned long long seq = 0, s = 0;                                                     \
        __device__ explicit TlScope(int k) : kind(k) {                                         \
            if (threadIdx.x == 0 && g_tl && kind >= 0) {                                       \
                seq = __hip_atomic_load(&g_tl->seq[kind], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
                s = wall_clock64();                                                            \
            }                                                                                  \
        }                                                                                      \
        __device__ ~TlScope() {                                                                \
            if (threadIdx.x == 0 && g_tl && kind >= 0) {                                       \
                const unsigned long long e = wall_clock64();                                   \
                const int slot = (int)(seq % sml::tl::kRing);                                  \
                atomicMin(&g_tl->t0[kind][slot], s);                                           \
                atomicMax(&g_tl->t1[kind][slot], e);                                           \
                const unsigned n = gridDim.x * gridDim.y * gridDim.z;                          \
                if (atomicAdd(&g_tl->arrivals[kind], 1u) == n - 1) {                           \
                    g_tl->arrivals[kind] = 0;                                                  \
                    __hip_atomic_store(&g_tl->seq[kind], seq + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); \
                }                                                                              \
            }                                                                                  \
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

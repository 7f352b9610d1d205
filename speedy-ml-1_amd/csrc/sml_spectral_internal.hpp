// sml_spectral_internal.hpp -- library-internal access to the spectral context
// (used by the dynamics step; not part of the C ABI).
#pragma once
#include <hip/hip_runtime.h>

#include "sml_spectral_tables.hpp"

struct sml_spectral;

namespace sml {

// per-field sizes of the batched spectral buffers: spectral [nx][mx2], Fourier [il][mx2]
constexpr int kSpecField = kMX2 * kNX;  // 1984
constexpr int kVarmField = kMX2 * kIL;  // 2976

struct SpectralDev {
    const double *gradx, *uvdx, *uvdym, *uvdyp, *vddym, *vddyp;  // [n][m] (gradx [m])
    const double *el2, *trfilt;                                   // [n][m]
    const double *cosgr, *cosgr2, *wt;                            // [48], [48], [24]
    // the transform matrices (layouts in sml_spectral.hip): Legendre inverse
    // [m][n][32 lat], forward [m][n][24 lat]; Fourier inverse [64 c][96 lon],
    // forward [96 lon][64 c]
    const double *pinv, *pfwd, *dinv, *dfwd;
    const double *wa;  // FFTPACK twiddles for n = 96 (sml_fft.hpp)
};

const SpectralTables &spectral_host_tables(const sml_spectral *s);
SpectralDev spectral_dev(const sml_spectral *s);
// launches on `stream`; nf fields back to back
int spectral_gridy(sml_spectral *s, const double *spec, double *varm, int nf, hipStream_t st);
int spectral_gridx(sml_spectral *s, const double *varm, double *grid, int nf, int kcos, hipStream_t st);
// one launch over fields of both kinds: the first ncos1 kcos = 1, the rest kcos = 2
int spectral_gridx_split(sml_spectral *s, const double *varm, double *grid, int nf, int ncos1, hipStream_t st);
// kcos = 2 (x cosgr) for the fields c0 <= f < c1, kcos = 1 for the others
int spectral_gridx_range(sml_spectral *s, const double *varm, double *grid, int nf, int c0, int c1, hipStream_t st);
// iogrid(30)'s entry / iogrid(31)'s exit: specx from / gridx into variables3d and
// logp directly (real(4) copies and the q clip on entry).  gridx_io: the 33 Fourier fields [u v t q | ps] (kcos = 2 for the first
// nwind) straight into variables3d(4, ix, il, kx) and logp(ix, il)
// wait (optional): a cross-stream hand-off the kernel waits for in-kernel before it
// reads g4 / logp (*flag >= value; ~4 s, then *late is set and it goes on)
struct HopWait {
    const uint64_t *flag = nullptr;
    uint64_t value = 0;
    unsigned *late = nullptr;
    // signal at the kernel's start: lane 0 of each block adds 1 (the kernel's input
    // grid was released by the kernel before it on the stream; the chain on SPEEDY's
    // stream hands the assembled grid to the main stream's re-tiling this way)
    uint64_t *sig = nullptr;
    // give-up time of the poll in wall_clock64 ticks (100 MHz; default ~4 s); on a
    // timeout the kernel marks *late (system scope: a host-visible word) and reads NaN
    // instead of the grid it did not get, so nothing downstream passes for a forecast
    long long timeout = 400000000ll;
    // the value to wait for, from device memory instead of `value` (a wait captured in a
    // graph keeps its arguments: the kernel before it on the stream writes this word)
    const uint64_t *vptr = nullptr;
};
int spectral_specx_io_blocks();
int spectral_specx_io(sml_spectral *s, const double *g4, const double *logp, double *varm, int nwind,
                      hipStream_t st, HopWait wait = {});
int spectral_gridx_io(sml_spectral *s, const double *varm, double *g4, double *logp, int nwind, hipStream_t st);

// run_model's exit (src/mpires.f90:1605-1628) around iogrid(31): the forecast's q is
// floored at 1e-6 (:1614-1616), and when iogrid(30)'s safety check failed agcm_main
// skipped the integration (at_gcm.f90:37), so the forecast is run_model's copy of
// its input grid, q floored the same way (:1550-1553, :1586).  mm: the 8 min/max
// values of the check (device); in4 / inlp: the window's input grids.
struct IoExit {
    double qfloor;
    const double *mm, *in4, *inlp;
    // the check's hand-off without a stream hop (sml_dynamics chk_flag): mm is final
    // once *cnt >= target (the check's min/max blocks each add 1 after their sc1
    // stores); a hand-off that does not arrive within ~1 s sets *late and goes on
    const unsigned *cnt = nullptr;
    unsigned target = 0;
    unsigned *late = nullptr;
    long long timeout = 100000000ll;  // ~1 s; on a timeout the check counts as unsafe (NaN min / max)
    // the count to wait for, from device memory instead of `target` (xa[0], written by
    // this run_model's k_io_entry): an exit replayed inside a graph keeps its arguments
    const uint64_t *xa = nullptr;
};
int spectral_gridx_run_model_exit(sml_spectral *s, const double *varm, double *g4, double *logp, int nwind,
                                  IoExit ex, hipStream_t st);

// is_safe_to_run_speedy from the re-gridded entry state's min/max (ppo_iogrid.f90:
// 563-577; thresholds u +-150, v +-120, t 160..330, q -6..30).  A NaN anywhere makes
// the state unsafe (the reference's minval/maxval with NaN are processor-dependent
// under -ffast-math; stopping is the conservative reading).
__host__ __device__ inline bool io_state_safe(const double *mm) {
    const double lo[4] = {-150.0, -120.0, 160.0, -6.0}, hi[4] = {150.0, 120.0, 330.0, 30.0};
    for (int v = 0; v < 4; ++v)
        if (!(mm[2 * v] >= lo[v]) || !(mm[2 * v + 1] <= hi[v])) return false;
    return true;
}
// scale: 0 none, 1 x cosgr(lat), 2 x cosgr2(lat) (vdspec's prescaling)
int spectral_specx(sml_spectral *s, const double *grid, double *varm, int nf, int scale, hipStream_t st);
// one launch: the first nscaled fields x cosgr(lat) (vdspec kcos = 2), the rest plain
int spectral_specx_split(sml_spectral *s, const double *grid, double *varm, int nf, int nscaled, hipStream_t st);
int spectral_specy(sml_spectral *s, const double *varm, double *spec, int nf, hipStream_t st);

}  // namespace sml

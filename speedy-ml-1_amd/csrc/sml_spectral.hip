// sml_spectral.hip -- batched T30 spherical-harmonic transforms on gfx950.
//
// The reference transforms one field per call (grid / spec, spe_spectral.f90:389-414):
// a Legendre sum per latitude (gridy/specy, :454-538) and a 96-point FFTPACK real
// FFT per latitude row (gridx/specx, spe_subfft_fftpack.f90:15-87).  Here every
// call transforms a batch of fields and both stages are fp64 MFMA GEMMs
// (v_mfma_f64_16x16x4_f64):
//
//   Legendre (per zonal wavenumber m):  C[(field,Re/Im)][lat] = A[(field,Re/Im)][n] * P_m[n][lat]
//     16 rows = 8 fields x {Re, Im}; K = the 16 n of one parity (odd n build the
//     hemispherically symmetric part, even n the antisymmetric part, as gridy does);
//     N = 24 Gaussian latitudes (padded to 32).  P_m tiles come from a masked
//     table (the triangular T30 mask nsh2 is baked in as exact zeros).
//   Fourier (per latitude row): FFTPACK's real FFT (rfftb / rfftf for n = 96,
//     sml_fft.hpp) in the reference's operation order, many rows x fields per block
//     in LDS -- bit-identical to the reference's gridx / specx, and ~7x fewer flops
//     than a dense DFT.
//
// MFMA f64 16x16x4 operand map (cdna_hip_programming.md section 3): lane l holds
// A[l&15][l>>4] and B[l>>4][l&15]; the 4 results per lane are
// C[(l>>4) + 4q][l&15], q = 0..3.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <vector>

#include "sml_fft.hpp"
#include "sml_dynamics_tables.hpp"  // (+ sml_spectral_tables.hpp): kx for the iogrid exit layout
#include "sml_spectral_internal.hpp"  // IoExit, io_state_safe
#include "sml_timeline.hpp"

SML_TL_DEFINE(spectral)

using namespace sml;

typedef double d4 __attribute__((ext_vector_type(4)));

#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

constexpr int kGridField = kIX * kIL;   // 4608
constexpr int kJPad = 32;

struct sml_spectral {
    SpectralTables t;
    int device;
    double *d_pinv;   // [m][n][32]: P_mn(lat j) masked (ll <= ntrun1), j padded to 32
    double *d_pfwd;   // [m][n][24]: masked (ll <= ntrun1 and n <= ntrun1-1)
    double *d_dinv;   // [64][96]
    double *d_dfwd;   // [96][64]
    double *d_wa;     // FFTPACK twiddles for n = 96 (rffti1)
    double *d_wt;     // [24]
    double *d_cosgr;  // [48]
    double *d_cosgr2; // [48]
    double *d_coef;   // gradx[31] | uvdx | uvdym | uvdyp | vddym | vddyp ([32][31] each)
    double *d_el2;    // el2[32][31] | trfilt[32][31]
    double *d_work;   // varm workspace
    size_t work_fields;
    double *d_hbuf;   // staging for the host convenience calls
    size_t hbuf_doubles;
};

namespace {

// ------------------------------------------------------------------ kernels
// gridy: spec[f][n][62] -> varm[f][lat][62]  (one wave per (m, 8-field tile))
__global__ __launch_bounds__(64) void k_gridy(const double *__restrict__ spec, double *__restrict__ varm,
                                              const double *__restrict__ pinv, int nf) {
    const int m = blockIdx.x;
    const int f0 = blockIdx.y * 8;
    const int l = threadIdx.x, r = l & 15, kk = l >> 4;
    const int fa = f0 + (r >> 1);
    const bool ok = fa < nf;
    const double *sp = spec + (size_t)(ok ? fa : 0) * kSpecField + 2 * m + (r & 1);
    const double *pm = pinv + (size_t)m * kNX * kJPad;
    d4 acc00 = {0, 0, 0, 0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int n_odd = 2 * (4 * s + kk);  // n = 1,3,.. (1-based): symmetric part
        const int n_even = n_odd + 1;        // n = 2,4,..: antisymmetric part
        const double a0 = ok ? sp[n_odd * kMX2] : 0.0;
        const double a1 = ok ? sp[n_even * kMX2] : 0.0;
        acc00 = MFMA64(a0, pm[n_odd * kJPad + r], acc00);
        acc01 = MFMA64(a0, pm[n_odd * kJPad + 16 + r], acc01);
        acc10 = MFMA64(a1, pm[n_even * kJPad + r], acc10);
        acc11 = MFMA64(a1, pm[n_even * kJPad + 16 + r], acc11);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = kk + 4 * q;
        const int f = f0 + (row >> 1);
        if (f >= nf) continue;
        double *vr = varm + (size_t)f * kVarmField + 2 * m + (row & 1);
        {   // latitudes j = r (southern half), mirror j1 = 47 - j (northern)
            const int j = r;
            const double s = acc00[q], d = acc10[q];
            vr[(kIL - 1 - j) * kMX2] = s + d;
            vr[j * kMX2] = s - d;
        }
        const int j = 16 + r;
        if (j < kIY) {
            const double s = acc01[q], d = acc11[q];
            vr[(kIL - 1 - j) * kMX2] = s + d;
            vr[j * kMX2] = s - d;
        }
    }
}

// gridx / specx: FFTPACK's real FFT along each latitude row, one (field, row)
// transform per thread pair, each thread one n = 48 half held in registers
// (sml_fft.hpp rfftb96_half / rfftf48_reg + rfftf96_combine: FFTPACK's operations).
constexpr int kFftThreads = 64;

// gridx (spe_subfft_fftpack.f90:15-51): fvar(1) = varm(1) (Im of m = 0 dropped),
// fvar(m-1) = varm(m) for m = 3..mx2, 0 beyond; rfftb; x cosgr(j) for kcos = 2 (the
// fields c0 <= f < c1).  With g4 set, the 33 fields [u v t q (kx each) | ps] go
// straight into iogrid(31)'s variables3d(4, ix, il, kx) (var = T, u, v, q) and logp
// instead of grid (ppo_iogrid.f90:590-595); ex.mm set: run_model's exit on top
// (sml_spectral_internal.hpp IoExit: q floor, the unsafe window's pass-through)
// transform t -> (field f, latitude j) of the FFT kernels.  For iogrid's 33 fields
// of the (var, x, y, z)-ordered grid the four variables of one (level, latitude) are
// neighbouring transforms, so a wave's 8-B loads / stores of grid point e cover 64-B
// runs (4 variables x the pair's 2 points) instead of 64 scattered words; else
// consecutive transforms are consecutive latitudes of one field
__device__ inline void fft_fj(int t, bool io, int &f, int &j) {
    if (io && t < 4 * kKX * kIL) {
        const int q = t >> 2;
        f = (t & 3) * kKX + q % kKX;
        j = q / kKX;
    } else {
        f = t / kIL;
        j = t % kIL;
    }
}

// k_gridx's transform and stores of one thread (rfftb half h of transform (f, j))
__device__ __attribute__((always_inline)) inline void gridx_store(const double (&xi)[kMX2 - 1], int h, int f, int j,
                                                                  const double *was, const double *__restrict__ cosgr,
                                                                  int c0, int c1, double *__restrict__ grid,
                                                                  double *__restrict__ g4, double *__restrict__ logp,
                                                                  const IoExit &ex, const double (&mmv)[8]) {
    double y[kFftN / 2];
    fft::rfftb96_half([&](int e) { return e <= kMX2 - 2 ? xi[e] : 0.0; }, h, y, was);
    const bool k2 = f >= c0 && f < c1;
    const double cj = k2 ? cosgr[j] : 1.0;
    double *g = grid + (size_t)f * kGridField + j * kIX;
    int gs = 1;
    if (g4) {
        const int grp = f / kKX, k = f % kKX;
        size_t o;
        if (grp < 4) {
            const int var = grp == 0 ? 1 : grp == 1 ? 2 : grp == 2 ? 0 : 3;
            o = var + 4 * ((size_t)kGridField * k + j * kIX);
            g = g4 + o;
            gs = 4;
        } else {
            o = (size_t)j * kIX;
            g = logp + o;
        }
        if (ex.mm) {  // run_model's exit (uniform across the launch: every thread reads the same flag)
            const bool q = grp == 3;
            if (!io_state_safe(mmv)) {  // integration skipped: the input grid comes back
                const double *src = grp < 4 ? ex.in4 + o : ex.inlp + o;
#pragma unroll
                for (int qq = 0; qq < kFftN / 2; ++qq) {
                    const int e = 2 * qq + h;
                    const double vv = src[e * gs];
                    g[e * gs] = (q && vv < ex.qfloor) ? ex.qfloor : vv;
                }
                return;
            }
#pragma unroll
            for (int qq = 0; qq < kFftN / 2; ++qq) {
                const double vv = k2 ? y[qq] * cj : y[qq];
                g[(2 * qq + h) * gs] = (q && vv < ex.qfloor) ? ex.qfloor : vv;
            }
            return;
        }
    }
#pragma unroll
    for (int qq = 0; qq < kFftN / 2; ++qq) g[(2 * qq + h) * gs] = k2 ? y[qq] * cj : y[qq];
}

__global__ __launch_bounds__(kFftThreads) void k_gridx(const double *__restrict__ varm, double *__restrict__ grid,
                                                       const double *__restrict__ wa, const double *__restrict__ cosgr,
                                                       int nf, int c0, int c1, double *__restrict__ g4,
                                                       double *__restrict__ logp, IoExit ex) {
    SML_TL_SCOPE(ex.mm ? sml::tl::kExitGridx : -1);
    __shared__ double was[kFftWa];  // twiddles: LDS broadcast reads inside the FFT
    // transform (f, j) on the thread pair 2 t, 2 t + 1: thread h does half h of
    // FFTPACK's rfftb (sml_fft.hpp rfftb96_half), the grid points 2 q + h.  The
    // coefficients (and the exit's min/max) are loaded before the twiddles are staged:
    // one memory round trip for both
    const int id = blockIdx.x * kFftThreads + threadIdx.x;
    const bool act = id < 2 * nf * kIL;
    const int t = id >> 1, h = id & 1;
    int f = 0, j = 0;
    if (act) fft_fj(t, g4 && nf == 4 * kKX + 1, f, j);
    double xi[kMX2 - 1];
    if (act) {
        const double *v = varm + (size_t)f * kVarmField + j * kMX2;
        xi[0] = v[0];
#pragma unroll
        for (int e = 1; e <= kMX2 - 2; ++e) xi[e] = v[e + 1];
    }
    double mmv[8];
    if (ex.mm && ex.cnt) {
        // the safety check ran on another stream: wait for its hand-off counter (one
        // relaxed sc1 poll per step of lane 0, MI355X_MICROARCH.md inter-workgroup
        // visibility: the producer stored mm sc1 and drained before its atomic add),
        // then read mm with sc1 loads
        __shared__ int gave_up;
        if (threadIdx.x == 0) {
            gave_up = 0;
            const long long t0 = wall_clock64();
            const unsigned target = ex.xa ? (unsigned)ex.xa[0] : ex.target;
            while (__hip_atomic_load(ex.cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(2);
                if (wall_clock64() - t0 > ex.timeout) {  // never hang the queue
                    // the mark names the check given up on (its counter target, >= 4), so
                    // sml_dyn_last_safe fails that window only, not every later one
                    __hip_atomic_store(ex.late, target, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    gave_up = 1;
                    break;
                }
            }
        }
        __syncthreads();
        // a check that did not arrive counts as unsafe (NaN fails every threshold): the
        // forecast is then the window's input, as agcm_main skips an unsafe window
#pragma unroll
        for (int q = 0; q < 8; ++q)
            mmv[q] = gave_up ? __builtin_nan("") : __hip_atomic_load(ex.mm + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else if (ex.mm) {
#pragma unroll
        for (int q = 0; q < 8; ++q) mmv[q] = ex.mm[q];
    }
    if (threadIdx.x < kFftWa) was[threadIdx.x] = wa[threadIdx.x];
    if (threadIdx.x + kFftThreads < kFftWa) was[threadIdx.x + kFftThreads] = wa[threadIdx.x + kFftThreads];
    __syncthreads();
    if (act) gridx_store(xi, h, f, j, was, cosgr, c0, c1, grid, g4, logp, ex, mmv);
}

// specx (spe_subfft_fftpack.f90:55-87): fvar = vorg(:, j) (the first nscaled fields
// x scale_tab(j): vdspec's ug*cosgr(j) / ug*cosgr2(j), spe_spectral.f90:430-445);
// rfftf; varm(1) = fvar(1)/ix, varm(2) = 0, varm(m) = fvar(m-1)/ix
// With g4 set, the input is iogrid(30)'s variables3d(4, ix, il, kx) / logp: the 33
// fields [u v t q (kx each) | ps] as their real(4) copies, q < 0 -> 0 on the copy
// (ppo_iogrid.f90:503-518), instead of grid.
__global__ __launch_bounds__(kFftThreads) void k_specx(const double *__restrict__ grid, double *__restrict__ varm,
                                                       const double *__restrict__ wa,
                                                       const double *__restrict__ scale_tab, int nf, int nscaled,
                                                       const double *__restrict__ g4 = nullptr,
                                                       const double *__restrict__ logp = nullptr,
                                                       HopWait wait = {}) {
    __shared__ double was[kFftWa];
    __shared__ double S[kFftN * (kFftThreads / 2)];  // a pair's two n = 48 halves (E, O)
    if (wait.sig && threadIdx.x == 0) __hip_atomic_fetch_add(wait.sig, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // wait.flag: the grid comes from another stream (SML_HOP_KERNEL): the twiddles are
    // staged first, then one lane polls, acquires at agent scope and releases the
    // block (MI355X_MICROARCH.md inter-workgroup visibility, the consumer form)
    __shared__ int gave_up;
    if (wait.flag) {
        if (threadIdx.x < kFftWa) was[threadIdx.x] = wa[threadIdx.x];
        if (threadIdx.x + kFftThreads < kFftWa) was[threadIdx.x + kFftThreads] = wa[threadIdx.x + kFftThreads];
        if (threadIdx.x == 0) {
            gave_up = 0;
            const long long c0 = wall_clock64();
            const uint64_t want = wait.vptr ? *wait.vptr : wait.value;
            while (__hip_atomic_load(wait.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - c0 > wait.timeout) {
                    __hip_atomic_store(wait.late, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    gave_up = 1;
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    SML_TL_SCOPE(g4 ? sml::tl::kEntrySpecx : -1);  // (after the wait: when the grid arrived)
    const bool stale = wait.flag && gave_up;  // the grid never arrived: transform NaN, not stale values
    // transform (f, j) on the thread pair 2 t, 2 t + 1: thread h transforms the samples
    // 2 i + h (rfftf48), the pair meets in LDS for rfftf's last pass (rfftf96_combine).
    // The samples are loaded before the twiddles are staged (one memory round trip).
    const int id = blockIdx.x * kFftThreads + threadIdx.x;
    const bool act = id < 2 * nf * kIL;
    const int t = id >> 1, h = id & 1, pr = threadIdx.x >> 1;
    int f = 0, j = 0;
    if (act) fft_fj(t, g4 && nf == 4 * kKX + 1, f, j);
    double x[kFftN / 2];
    const bool sc = act && scale_tab && f < nscaled;
    double s0 = 1.0;
    if (act) {
        const double *g = grid + (size_t)f * kGridField + j * kIX + h;
        if (sc) s0 = scale_tab[j];
        if (g4) {
            const int grp = f / kKX, k = f % kKX;
            if (grp < 4) {
                const int var = grp == 0 ? 1 : grp == 1 ? 2 : grp == 2 ? 0 : 3;
                const double *src = g4 + var + 4 * ((size_t)kGridField * k + j * kIX + h);
#pragma unroll
                for (int i = 0; i < kFftN / 2; ++i) x[i] = src[8 * i];
            } else {
#pragma unroll
                for (int i = 0; i < kFftN / 2; ++i) x[i] = logp[j * kIX + 2 * i + h];
            }
        } else {
#pragma unroll
            for (int i = 0; i < kFftN / 2; ++i) x[i] = g[2 * i];
        }
    }
    if (stale) {
#pragma unroll
        for (int i = 0; i < kFftN / 2; ++i) x[i] = __builtin_nan("");
    }
    if (!wait.flag) {
        if (threadIdx.x < kFftWa) was[threadIdx.x] = wa[threadIdx.x];
        if (threadIdx.x + kFftThreads < kFftWa) was[threadIdx.x + kFftThreads] = wa[threadIdx.x + kFftThreads];
        __syncthreads();
    }
    if (act) {
        if (g4) {  // iogrid(30)'s real(4) copies, q < 0 -> 0 on the copy
            const bool qf = f / kKX == 3;
#pragma unroll
            for (int i = 0; i < kFftN / 2; ++i) {
                float v4 = (float)x[i];
                if (qf && v4 < 0.0f) v4 = 0.0f;
                x[i] = (double)v4;
            }
            if (sc) {
#pragma unroll
                for (int i = 0; i < kFftN / 2; ++i) x[i] = x[i] * s0;
            }
        } else if (sc) {
#pragma unroll
            for (int i = 0; i < kFftN / 2; ++i) x[i] = x[i] * s0;
        }
        fft::rfftf48_reg(x, was);
#pragma unroll
        for (int i = 0; i < kFftN / 2; ++i) S[(48 * h + i) * (kFftThreads / 2) + pr] = x[i];
    }
    __syncthreads();
    if (!act) return;
    auto E = [&](int i) { return S[i * (kFftThreads / 2) + pr]; };
    auto O = [&](int i) { return S[(48 + i) * (kFftThreads / 2) + pr]; };
    const double scale = 1. / (double)kIX;
    double *v = varm + (size_t)f * kVarmField + j * kMX2;
    auto out = [&](int m) {  // varm(2m+1..2m+2) = fvar(2m..2m+1) / ix
        double re, im;
        fft::rfftf96_combine(E, O, m, was, &re, &im);
        v[2 * m] = re * scale;
        v[2 * m + 1] = im * scale;
    };
    if (h == 0) {
        v[0] = (E(0) + O(0)) * scale;  // varm(1) = fvar(1) / ix, varm(2) = 0
        v[1] = 0.0;
#pragma unroll
        for (int m = 1; m <= 15; ++m) out(m);
    } else {
#pragma unroll
        for (int m = 16; m <= kMX - 1; ++m) out(m);
    }
}

// specy: varm[f][lat][62] -> spec[f][n][62]  (one wave per (m, 8-field tile));
// symmetric combinations x wt feed odd n, antisymmetric feed even n (specy :513-535)
__global__ __launch_bounds__(64) void k_specy(const double *__restrict__ varm, double *__restrict__ spec,
                                              const double *__restrict__ pfwd, const double *__restrict__ wt, int nf) {
    const int m = blockIdx.x;
    const int f0 = blockIdx.y * 8;
    const int l = threadIdx.x, r = l & 15, kk = l >> 4;
    const int fa = f0 + (r >> 1);
    const bool ok = fa < nf;
    const double *vr = varm + (size_t)(ok ? fa : 0) * kVarmField + 2 * m + (r & 1);
    const double *pm = pfwd + (size_t)m * kNX * kIY;
    d4 accS = {0, 0, 0, 0}, accD = accS;
#pragma unroll
    for (int s = 0; s < kIY / 4; ++s) {
        const int j = 4 * s + kk;
        double aS = 0.0, aD = 0.0;
        if (ok) {
            const double vn = vr[(kIL - 1 - j) * kMX2], vs = vr[j * kMX2];
            aS = (vn + vs) * wt[j];
            aD = (vn - vs) * wt[j];
        }
        accS = MFMA64(aS, pm[(2 * r) * kIY + j], accS);
        accD = MFMA64(aD, pm[(2 * r + 1) * kIY + j], accD);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = kk + 4 * q;
        const int f = f0 + (row >> 1);
        if (f >= nf) continue;
        double *sp = spec + (size_t)f * kSpecField + 2 * m + (row & 1);
        sp[(2 * r) * kMX2] = accS[q];
        sp[(2 * r + 1) * kMX2] = accD[q];
    }
}

// spectral-space operators on complex(mx,nx) = real(2,mx,nx); one thread per
// (field, m, n) complex coefficient.
struct Coef {
    const double *gradx, *uvdx, *uvdym, *uvdyp, *vddym, *vddyp;
};

__device__ inline int c3(int k, int m, int n) { return k + 2 * (m + kMX * n); }

// vds (spe_spectral.f90:307-349): (u cos, v cos) spectral -> (vor, div)
__global__ void k_vds(const double *__restrict__ ucos, const double *__restrict__ vcos, double *__restrict__ vor,
                      double *__restrict__ div, Coef cf, int nf) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nf * kMX * kNX) return;
    const int f = idx / (kMX * kNX), mn = idx % (kMX * kNX), n = mn / kMX, m = mn % kMX;
    const double *u = ucos + (size_t)f * kSpecField, *v = vcos + (size_t)f * kSpecField;
    double *vo = vor + (size_t)f * kSpecField, *dv = div + (size_t)f * kSpecField;
    const double gx = cf.gradx[m];
    double zp[2], zc[2];
    zp[1] = gx * u[c3(0, m, n)];
    zp[0] = -gx * u[c3(1, m, n)];
    zc[1] = gx * v[c3(0, m, n)];
    zc[0] = -gx * v[c3(1, m, n)];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        double a, b;
        if (n == 0) {
            const double yp = cf.vddyp[m];
            a = zc[k] - yp * u[c3(k, m, 1)];
            b = zp[k] + yp * v[c3(k, m, 1)];
        } else if (n == kNX - 1) {
            const double ym = cf.vddym[n * kMX + m];
            a = ym * u[c3(k, m, kNTRUN1 - 1)];
            b = -ym * v[c3(k, m, kNTRUN1 - 1)];
        } else {
            const double ym = cf.vddym[n * kMX + m], yp = cf.vddyp[n * kMX + m];
            a = ym * u[c3(k, m, n - 1)] - yp * u[c3(k, m, n + 1)] + zc[k];
            b = -ym * v[c3(k, m, n - 1)] + yp * v[c3(k, m, n + 1)] + zp[k];
        }
        vo[c3(k, m, n)] = a;
        dv[c3(k, m, n)] = b;
    }
}

// uvspec (spe_spectral.f90:351-387): (vor, div) -> (u cos, v cos)
__global__ void k_uvspec(const double *__restrict__ vor, const double *__restrict__ div, double *__restrict__ ucos,
                         double *__restrict__ vcos, Coef cf, int nf) {
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= nf * kMX * kNX) return;
    const int f = idx / (kMX * kNX), mn = idx % (kMX * kNX), n = mn / kMX, m = mn % kMX;
    const double *vo = vor + (size_t)f * kSpecField, *dv = div + (size_t)f * kSpecField;
    double *u = ucos + (size_t)f * kSpecField, *v = vcos + (size_t)f * kSpecField;
    const double ux = cf.uvdx[n * kMX + m];
    double zp[2], zc[2];
    zp[1] = ux * vo[c3(0, m, n)];
    zp[0] = -ux * vo[c3(1, m, n)];
    zc[1] = ux * dv[c3(0, m, n)];
    zc[0] = -ux * dv[c3(1, m, n)];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
        double a, b;
        if (n == 0) {
            const double yp = cf.uvdyp[m];
            a = zc[k] - yp * vo[c3(k, m, 1)];
            b = zp[k] + yp * dv[c3(k, m, 1)];
        } else if (n == kNX - 1) {
            const double ym = cf.uvdym[n * kMX + m];
            a = ym * vo[c3(k, m, kNTRUN1 - 1)];
            b = -ym * dv[c3(k, m, kNTRUN1 - 1)];
        } else {
            const double ym = cf.uvdym[n * kMX + m], yp = cf.uvdyp[n * kMX + m];
            b = -ym * dv[c3(k, m, n - 1)] + yp * dv[c3(k, m, n + 1)] + zp[k];
            a = ym * vo[c3(k, m, n - 1)] - yp * vo[c3(k, m, n + 1)] + zc[k];
        }
        u[c3(k, m, n)] = a;
        v[c3(k, m, n)] = b;
    }
}

Coef coef_of(const sml_spectral *s) {
    Coef c;
    const size_t tab = (size_t)kNX * kMX;
    c.gradx = s->d_coef;
    c.uvdx = s->d_coef + kMX;
    c.uvdym = c.uvdx + tab;
    c.uvdyp = c.uvdym + tab;
    c.vddym = c.uvdyp + tab;
    c.vddyp = c.vddym + tab;
    return c;
}

int ensure_work(sml_spectral *s, size_t fields) {
    if (fields <= s->work_fields) return SML_OK;
    if (s->d_work) SML_HIP(hipFree(s->d_work));
    s->d_work = nullptr;
    size_t nf = fields < 64 ? 64 : fields;
    // varm for 2*nf fields plus 2*nf spectral fields (vdspec transforms u and v
    // together and keeps their spectral coefficients for vds)
    SML_HIP(hipMalloc(&s->d_work, 2 * nf * (size_t)(kVarmField + kSpecField) * sizeof(double)));
    s->work_fields = nf;
    return SML_OK;
}

int check_ctx(const sml_spectral *s, int nf) {
    SML_REQUIRE(s != nullptr, "null spectral context");
    SML_REQUIRE(nf >= 0, "nfields must be >= 0 (got %d)", nf);
    return SML_OK;
}

}  // namespace

// ------------------------------------------------------------------ API
extern "C" int sml_spectral_create(double radius, sml_spectral **out) {
    SML_REQUIRE(out != nullptr, "out is null");
    SML_REQUIRE(radius > 0.0, "radius must be positive");
    *out = nullptr;
    sml_spectral *s = new (std::nothrow) sml_spectral();
    if (!s) return fail(SML_ERR_NOMEM, "host allocation failed");
    build_spectral_tables(radius, &s->t);
    SML_HIP(hipGetDevice(&s->device));
    const SpectralTables &t = s->t;
    std::vector<double> pinv((size_t)kMX * kNX * kJPad, 0.0), pfwd((size_t)kMX * kNX * kIY, 0.0);
    for (int m = 0; m < kMX; ++m)
        for (int n = 0; n < kNX; ++n)
            for (int j = 0; j < kIY; ++j) {
                const bool in_tri = m + n <= kNTRUN1;  // 2m < nsh2(n) (parmtr :82-107)
                if (in_tri) pinv[((size_t)m * kNX + n) * kJPad + j] = t.poly[j][n][m];
                if (in_tri && n < kNTRUN1) pfwd[((size_t)m * kNX + n) * kIY + j] = t.poly[j][n][m];
            }
    std::vector<double> coef(kMX + 5 * (size_t)kNX * kMX);
    std::memcpy(coef.data(), t.gradx, sizeof t.gradx);
    std::memcpy(coef.data() + kMX, t.uvdx, sizeof t.uvdx);
    std::memcpy(coef.data() + kMX + 1 * kNX * kMX, t.uvdym, sizeof t.uvdym);
    std::memcpy(coef.data() + kMX + 2 * kNX * kMX, t.uvdyp, sizeof t.uvdyp);
    std::memcpy(coef.data() + kMX + 3 * kNX * kMX, t.vddym, sizeof t.vddym);
    std::memcpy(coef.data() + kMX + 4 * kNX * kMX, t.vddyp, sizeof t.vddyp);
    std::vector<double> el2trf(2 * (size_t)kNX * kMX);
    for (int n = 0; n < kNX; ++n)
        for (int m = 0; m < kMX; ++m) {
            el2trf[n * kMX + m] = t.el2[n][m];
            el2trf[kNX * kMX + n * kMX + m] = (m + n <= kNTRUN) ? 1.0 : 0.0;  // trfilt (parmtr :103-107)
        }
    double wa[kFftWa];
    sml_fft_twiddles(wa);
    auto up = [](double **d, const void *h, size_t bytes) -> int {
        SML_HIP(hipMalloc(d, bytes));
        SML_HIP(hipMemcpy(*d, h, bytes, hipMemcpyHostToDevice));
        return SML_OK;
    };
    int rc;
    if ((rc = up(&s->d_pinv, pinv.data(), pinv.size() * 8)) || (rc = up(&s->d_pfwd, pfwd.data(), pfwd.size() * 8)) ||
        (rc = up(&s->d_dinv, t.dinv, sizeof t.dinv)) || (rc = up(&s->d_dfwd, t.dfwd, sizeof t.dfwd)) ||
        (rc = up(&s->d_wt, t.wt, sizeof t.wt)) || (rc = up(&s->d_cosgr, t.cosgr, sizeof t.cosgr)) ||
        (rc = up(&s->d_cosgr2, t.cosgr2, sizeof t.cosgr2)) || (rc = up(&s->d_coef, coef.data(), coef.size() * 8)) ||
        (rc = up(&s->d_el2, el2trf.data(), el2trf.size() * 8)) || (rc = up(&s->d_wa, wa, sizeof wa)) ||
        (rc = ensure_work(s, 64))) {
        sml_spectral_destroy(s);
        return rc;
    }
    *out = s;
    return SML_OK;
}

extern "C" int sml_spectral_destroy(sml_spectral *s) {
    if (!s) return SML_OK;
    double *ptrs[] = {s->d_pinv,   s->d_pfwd, s->d_dinv, s->d_dfwd, s->d_wt,   s->d_cosgr,
                      s->d_cosgr2, s->d_coef, s->d_el2,  s->d_work, s->d_hbuf, s->d_wa};
    for (double *p : ptrs)
        if (p) (void)hipFree(p);
    delete s;
    return SML_OK;
}

extern "C" int sml_spectral_tables(const sml_spectral *s, double *sia, double *wt, double *cpol, int *nsh2) {
    SML_REQUIRE(s != nullptr, "null spectral context");
    const SpectralTables &t = s->t;
    if (sia) std::memcpy(sia, t.sia, sizeof t.sia);
    if (wt) std::memcpy(wt, t.wt, sizeof t.wt);
    if (nsh2) std::memcpy(nsh2, t.nsh2, sizeof t.nsh2);
    if (cpol)  // cpol(mx2, nx, iy) column-major (mod_spectral.f90:29)
        for (int j = 0; j < kIY; ++j)
            for (int n = 0; n < kNX; ++n)
                for (int m = 0; m < kMX; ++m)
                    cpol[(j * kNX + n) * kMX2 + 2 * m] = cpol[(j * kNX + n) * kMX2 + 2 * m + 1] = t.poly[j][n][m];
    return SML_OK;
}

extern "C" int sml_gridy_batched(sml_spectral *s, const double *d_spec, double *d_varm, int nf, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    hipLaunchKernelGGL(k_gridy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, (hipStream_t)stream, d_spec, d_varm, s->d_pinv,
                       nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_gridx_batched(sml_spectral *s, const double *d_varm, double *d_grid, int nf, int kcos,
                                 void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    hipLaunchKernelGGL(k_gridx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, (hipStream_t)stream,
                       d_varm, d_grid, s->d_wa, s->d_cosgr, nf, kcos == 1 ? nf : 0, nf, nullptr, nullptr, IoExit{});
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_specx_batched(sml_spectral *s, const double *d_grid, double *d_varm, int nf, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    hipLaunchKernelGGL(k_specx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, (hipStream_t)stream,
                       d_grid, d_varm, s->d_wa, (const double *)nullptr, nf, 0);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_specy_batched(sml_spectral *s, const double *d_varm, double *d_spec, int nf, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    hipLaunchKernelGGL(k_specy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, (hipStream_t)stream, d_varm, d_spec, s->d_pfwd,
                       s->d_wt, nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_grid_batched(sml_spectral *s, const double *d_spec, double *d_grid, int nf, int kcos,
                                void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    if (int rc = ensure_work(s, nf)) return rc;
    if (int rc = sml_gridy_batched(s, d_spec, s->d_work, nf, stream)) return rc;
    return sml_gridx_batched(s, s->d_work, d_grid, nf, kcos, stream);
}

extern "C" int sml_spec_batched(sml_spectral *s, const double *d_grid, double *d_spec, int nf, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    if (int rc = ensure_work(s, nf)) return rc;
    if (int rc = sml_specx_batched(s, d_grid, s->d_work, nf, stream)) return rc;
    return sml_specy_batched(s, s->d_work, d_spec, nf, stream);
}

extern "C" int sml_vdspec_batched(sml_spectral *s, const double *d_ug, const double *d_vg, double *d_vor,
                                  double *d_div, int nf, int kcos, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    if (int rc = ensure_work(s, nf)) return rc;
    hipStream_t st = (hipStream_t)stream;
    const double *scale = (kcos == 2) ? s->d_cosgr : s->d_cosgr2;
    double *um = s->d_work, *vm = s->d_work + (size_t)nf * kVarmField;
    double *uc = s->d_work + 2 * s->work_fields * (size_t)kVarmField, *vc = uc + (size_t)nf * kSpecField;
    const dim3 fg((2 * nf * kIL + kFftThreads - 1) / kFftThreads), fb(kFftThreads);
    hipLaunchKernelGGL(k_specx, fg, fb, 0, st, d_ug, um, s->d_wa, scale, nf, nf);
    hipLaunchKernelGGL(k_specx, fg, fb, 0, st, d_vg, vm, s->d_wa, scale, nf, nf);
    hipLaunchKernelGGL(k_specy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, st, um, uc, s->d_pfwd, s->d_wt, nf);
    hipLaunchKernelGGL(k_specy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, st, vm, vc, s->d_pfwd, s->d_wt, nf);
    SML_HIP(hipGetLastError());
    const int total = nf * kMX * kNX;
    hipLaunchKernelGGL(k_vds, dim3((total + 255) / 256), dim3(256), 0, st, uc, vc, d_vor, d_div, coef_of(s), nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_uvspec_batched(sml_spectral *s, const double *d_vor, const double *d_div, double *d_ucos,
                                  double *d_vcos, int nf, void *stream) {
    if (int rc = check_ctx(s, nf)) return rc;
    if (nf == 0) return SML_OK;
    const int total = nf * kMX * kNX;
    hipLaunchKernelGGL(k_uvspec, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, d_vor, d_div, d_ucos,
                       d_vcos, coef_of(s), nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

static int ensure_hbuf(sml_spectral *s, size_t doubles) {
    if (doubles <= s->hbuf_doubles) return SML_OK;
    if (s->d_hbuf) SML_HIP(hipFree(s->d_hbuf));
    s->d_hbuf = nullptr;
    SML_HIP(hipMalloc(&s->d_hbuf, doubles * sizeof(double)));
    s->hbuf_doubles = doubles;
    return SML_OK;
}

extern "C" int sml_grid_host(sml_spectral *s, const double *spec, double *grid, int nf, int kcos) {
    if (int rc = check_ctx(s, nf)) return rc;
    SML_REQUIRE(spec && grid, "null host buffer");
    if (nf == 0) return SML_OK;
    if (int rc = ensure_hbuf(s, (size_t)nf * (kSpecField + kGridField))) return rc;
    double *ds = s->d_hbuf, *dg = s->d_hbuf + (size_t)nf * kSpecField;
    SML_HIP(hipMemcpy(ds, spec, (size_t)nf * kSpecField * 8, hipMemcpyHostToDevice));
    if (int rc = sml_grid_batched(s, ds, dg, nf, kcos, nullptr)) return rc;
    SML_HIP(hipMemcpy(grid, dg, (size_t)nf * kGridField * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_spec_host(sml_spectral *s, const double *grid, double *spec, int nf) {
    if (int rc = check_ctx(s, nf)) return rc;
    SML_REQUIRE(spec && grid, "null host buffer");
    if (nf == 0) return SML_OK;
    if (int rc = ensure_hbuf(s, (size_t)nf * (kSpecField + kGridField))) return rc;
    double *ds = s->d_hbuf, *dg = s->d_hbuf + (size_t)nf * kSpecField;
    SML_HIP(hipMemcpy(dg, grid, (size_t)nf * kGridField * 8, hipMemcpyHostToDevice));
    if (int rc = sml_spec_batched(s, dg, ds, nf, nullptr)) return rc;
    SML_HIP(hipMemcpy(spec, ds, (size_t)nf * kSpecField * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

// ------------------------------------------------------------------ internal API
#include "sml_spectral_internal.hpp"

namespace sml {

const SpectralTables &spectral_host_tables(const sml_spectral *s) { return s->t; }

SpectralDev spectral_dev(const sml_spectral *s) {
    SpectralDev d;
    const Coef c = coef_of(s);
    d.gradx = c.gradx;
    d.uvdx = c.uvdx;
    d.uvdym = c.uvdym;
    d.uvdyp = c.uvdyp;
    d.vddym = c.vddym;
    d.vddyp = c.vddyp;
    d.el2 = s->d_el2;
    d.trfilt = s->d_el2 + kNX * kMX;
    d.cosgr = s->d_cosgr;
    d.cosgr2 = s->d_cosgr2;
    d.wt = s->d_wt;
    d.pinv = s->d_pinv;
    d.pfwd = s->d_pfwd;
    d.dinv = s->d_dinv;
    d.dfwd = s->d_dfwd;
    d.wa = s->d_wa;
    return d;
}

int spectral_gridy(sml_spectral *s, const double *spec, double *varm, int nf, hipStream_t st) {
    if (nf <= 0) return SML_OK;
    hipLaunchKernelGGL(k_gridy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, st, spec, varm, s->d_pinv, nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_gridx(sml_spectral *s, const double *varm, double *grid, int nf, int kcos, hipStream_t st) {
    return spectral_gridx_range(s, varm, grid, nf, kcos == 1 ? nf : 0, nf, st);
}

int spectral_gridx_split(sml_spectral *s, const double *varm, double *grid, int nf, int ncos1, hipStream_t st) {
    return spectral_gridx_range(s, varm, grid, nf, ncos1, nf, st);
}

int spectral_gridx_range(sml_spectral *s, const double *varm, double *grid, int nf, int c0, int c1, hipStream_t st) {
    if (nf <= 0) return SML_OK;
    hipLaunchKernelGGL(k_gridx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, st, varm, grid, s->d_wa,
                       s->d_cosgr, nf, c0, c1, nullptr, nullptr, IoExit{});
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_gridx_io(sml_spectral *s, const double *varm, double *g4, double *logp, int nwind, hipStream_t st) {
    return spectral_gridx_run_model_exit(s, varm, g4, logp, nwind, IoExit{}, st);
}


int spectral_gridx_run_model_exit(sml_spectral *s, const double *varm, double *g4, double *logp, int nwind,
                                  IoExit ex, hipStream_t st) {
    constexpr int nf = 4 * kKX + 1;
    hipLaunchKernelGGL(k_gridx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, st, varm, nullptr,
                       s->d_wa, s->d_cosgr, nf, 0, nwind, g4, logp, ex);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_specx(sml_spectral *s, const double *grid, double *varm, int nf, int scale, hipStream_t st) {
    if (nf <= 0) return SML_OK;
    const double *sc = scale == 1 ? s->d_cosgr : scale == 2 ? s->d_cosgr2 : nullptr;
    hipLaunchKernelGGL(k_specx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, st, grid, varm, s->d_wa,
                       sc, nf, nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_specx_split(sml_spectral *s, const double *grid, double *varm, int nf, int nscaled, hipStream_t st) {
    if (nf <= 0) return SML_OK;
    hipLaunchKernelGGL(k_specx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, st, grid, varm, s->d_wa,
                       s->d_cosgr, nf, nscaled);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_specx_io_blocks() { return (2 * (4 * kKX + 1) * kIL + kFftThreads - 1) / kFftThreads; }

int spectral_specx_io(sml_spectral *s, const double *g4, const double *logp, double *varm, int nwind,
                      hipStream_t st, HopWait wait) {
    constexpr int nf = 4 * kKX + 1;
    hipLaunchKernelGGL(k_specx, dim3((2 * nf * kIL + kFftThreads - 1) / kFftThreads), dim3(kFftThreads), 0, st, nullptr, varm,
                       s->d_wa, s->d_cosgr, nf, nwind, g4, logp, wait);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int spectral_specy(sml_spectral *s, const double *varm, double *spec, int nf, hipStream_t st) {
    if (nf <= 0) return SML_OK;
    hipLaunchKernelGGL(k_specy, dim3(kMX, (nf + 7) / 8), dim3(64), 0, st, varm, spec, s->d_pfwd, s->d_wt, nf);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

}  // namespace sml

// sml_dynamics.hip -- one SPEEDY dynamics time step on gfx950.
//
// Reference: step (src/dyn_step.f90:1-128) =
//   grtend  (src/dyn_grtend.f90:1-279): 50 inverse transforms of the j2 state,
//           grid-point dynamics, physics hook (phypar, :225), 73 forward transforms
//   sptend  (src/dyn_sptend.f90:1-67) + geop (src/dyn_geop.f90:1-33)
//   implic  (src/dyn_implic.f90:1-68)         (alph != 0)
//   hordif, stratospheric drag, tracer diffusion (dyn_step.f90:60-112, :130-151)
//   timint with trunct, Robert-Williams filter  (dyn_step.f90:114-127, :153-190)
//
// MI355X design: the reference's ~164 one-field transforms per step become 7
// batched MFMA transform launches (gridy on 50 fields, gridx kcos=1/2, specx
// scaled/unscaled, specy on 73 fields); the grid-point dynamics is one kernel
// with a thread per grid column (vertical recurrences in registers); everything
// after the forward transforms (vds/lap assembly, sptend, geop, implic, hordif,
// drag, timint) runs in two kernels with a thread per spectral coefficient (m, n)
// that owns all levels, variables and both time levels of that coefficient, so no
// stage needs a grid-wide synchronisation.
//
// Physics (phypar, dyn_grtend.f90:223-226) runs on the GPU when the context has
// boundary fields (sml_dyn_set_physics): grtend always evaluates it on time level 1
// (dyn_step.f90:45), so the step adds 41 inverse transforms of level 1 (ucos,
// vcos, t, q, geop(1), ps; phy_phypar.f90:54-66) to the same batched launches and
// one column-physics kernel (sml_physics.hpp) whose tendencies enter where phypar
// adds them (after the dynamical tendencies, before the spectral conversion).
// Without boundary fields the tendencies come from an optional input buffer (a
// host that keeps phypar on the CPU) or are zero.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "sml_dynamics_tables.hpp"
#include "sml_fft.hpp"
#include "sml_fft_wa96.hpp"
#include "sml_physics.hpp"
#include "sml_physics_pair.hpp"
#include "sml_spectral_internal.hpp"
#include "sml_timeline.hpp"

SML_TL_DEFINE(dynamics)

using namespace sml;

namespace {

constexpr int kSF = kMX2 * kNX;       // 1984 doubles per spectral field
constexpr int kGF = kIX * kIL;        // 4608 doubles per grid field
constexpr int kVF = kMX2 * kIL;       // 2976 doubles per Fourier field
constexpr int kNInv = 6 * kKX + 2;    // 50 inverse transforms per step (dynamics)
constexpr int kNInv1 = 4 * kKX;       // the first 32 are kcos = 1
// with the physics on the GPU: kcos = 1 fields [vor div t tr (j2) | t1 q1 phi1 (8 each) | ps1]
// then kcos = 2 fields [ucos vcos (j2) | psdx psdy | ucos1 vcos1]
constexpr int kNInv1P = kNInv1 + 3 * kKX + 1;  // 57
constexpr int kNInvP = kNInv1P + 4 * kKX + 2;  // 91 (= the reference's 91 grid calls per step)
constexpr int kPT1 = kNInv1, kPQ1 = kNInv1 + kKX, kPPhi1 = kNInv1 + 2 * kKX, kPPs1 = kNInv1 + 3 * kKX;
constexpr int kNInvMax = kNInvP;
constexpr int kNFwdScaled = 6 * kKX;  // 48 vdspec inputs (x 1/cos lat)
constexpr int kNFwd = 9 * kKX + 1;    // 73 forward transforms per step
constexpr int kMN = kMX * kNX;        // 992 complex coefficients
constexpr int kNstrad = 3;            // shortwave radiation every 3rd step (mod_tsteps.f90:65)

// state buffer: vor(mx,nx,kx,2) | div | t | tr(ntr=1) | ps(mx,nx,2) (reference layouts)
constexpr size_t kOffVor = 0, kOffDiv = 2 * kKX * kSF, kOffT = 4 * kKX * kSF, kOffTr = 6 * kKX * kSF,
                 kOffPs = 8 * kKX * kSF, kStateSize = 8 * kKX * kSF + 2 * kSF;
// tendency buffer: vordt | divdt | tdt | trdt (kx fields each) | psdt
constexpr size_t kTVor = 0, kTDiv = kKX * kSF, kTT = 2 * kKX * kSF, kTTr = 3 * kKX * kSF, kTPs = 4 * kKX * kSF,
                 kTendSize = 4 * kKX * kSF + kSF;

__device__ inline int ci(int p, int m, int n) { return p + 2 * (m + kMX * n); }
__device__ inline int mi(int m, int n) { return m + kMX * n; }

}  // namespace

struct sml_dynamics {
    sml_spectral *sp = nullptr;
    DynTables tab;
    DynTables *d_tab = nullptr;   // current impint slot (one of d_tabs)
    double *d_tabm = nullptr;     // per slot: TabM of every m (the fused spectral stage's per-m tables)
    DynTables *d_tabs = nullptr;  // kTabSlots device copies keyed by (dt, alph): stepone's
                                  // three impint calls per window become pointer switches
    double slot_key[4][2] = {};
    bool slot_used[4] = {};
    int slot_next = 0;
    double *d_state = nullptr;
    double *d_phis = nullptr, *d_tcorh = nullptr, *d_qcorh = nullptr, *d_phi = nullptr;
    double *d_specin = nullptr, *d_varm = nullptr, *d_grid = nullptr, *d_gfwd = nullptr, *d_sfwd = nullptr;
    double *d_vfm = nullptr;  // fused step: m-major forward Fourier coefficients [m][73][lat][2]
    double *d_pfl = nullptr;  // specy's MFMA B operands in lane order [m][k-step][lane][S, D] (k_pack_pfwd)
    double *d_sm = nullptr;   // fused step: m-major state [2][m][var 5][lev 2][kx][n p], ping-pong:
    int sm_cur = 0;           // k_st_spec reads buffer sm_cur and writes the other (see sm_buf)
    long long *d_dbg = nullptr;  // diagnostic phase stamps (SML_DYN_STAMPS=1)
    double *d_tend = nullptr;
    double *d_phys = nullptr;  // physics tendencies: staging for a host's, or the GPU phypar's output
    double *d_minmax = nullptr;  // iogrid(30) safety check: min/max of u, v, t, q
    double *d_io = nullptr;      // staging for the host iogrid calls (grid4d + logp)
    // iogrid(30)'s safety check (re-grid + min/max) runs on its own stream beside the
    // window: its inputs [kNIo][kSF], Fourier [kNIo][kVF] and grid [kNIo][kGF] buffers
    double *d_chk = nullptr;
    hipStream_t chk_stream = nullptr;
    hipEvent_t ev_fork = nullptr, ev_chk = nullptr;
    bool chk_pending = false;  // work on chk_stream that the next user of d_chk must wait for
    // run_model's exit learns the check's result from a device counter instead of an
    // event wait on its stream: the check's k_io_minmax adds 4 per check, the exit polls
    // for 4 * chk_count (an event wait only where the check is not counted: capture)
    unsigned *d_chk_cnt = nullptr;
    // the exit's hand-off timed out: a pinned, host-visible word holding the counter
    // target of the check it gave up on (read without a copy by sml_dyn_last_safe and
    // sml::dyn_check_late, reset when reported); the exit's give-up time in ticks
    unsigned *d_chk_late = nullptr;
    long long chk_timeout = 100000000ll;
    // the next run_model's entry waits in-kernel for its input grids (sml::dyn_run_model_wait)
    HopWait entry_wait;
    // the next run_model's entry signals its input grid in-kernel (sml::dyn_run_model_entry_signal)
    uint64_t *entry_sig = nullptr;
    unsigned chk_count = 0;
    bool chk_counted = false;  // the last launch_io_check added to the counter
    // host copy of the last check's min/max (pinned; written behind the check on its
    // stream, ev_mm marks it): run_speedy for a host loop without a device sync
    double *h_mm = nullptr;
    hipEvent_t ev_mm = nullptr;
    bool mm_issued = false;
    const double *mm_last = nullptr;  // device min/max of the last from_grid
    bool impint_done = false;
    // GPU physics (phypar): tables, boundary fields [kNBc][ngp], radiation state
    PhysTables ptab;
    PhysTables *d_ptab = nullptr;
    double *d_pbc = nullptr, *d_rad = nullptr, *d_pio = nullptr;
    bool phys_on = false;
    // ini_sea's hybrid block (cpl_sea.f90:38-46): the coupler's sst_am as set_physics
    // gave it, sea-ice fraction / temperature, and the hybrid SST grid last applied
    // (sml_dyn_set_hybrid_sst; re-applied when set_physics brings a new sst_am)
    double *d_sst_cpl = nullptr, *d_sice = nullptr, *d_tice = nullptr;
    const double *hyb_sst = nullptr;
    double hyb_bias = 0.0;
    // agcm_init's per-window forcing (sml_dyn_fordate): inbcon's surface fields
    // [3][ngp] = fmask_l, fmask_s, alb0; the coupler's monthly climatologies
    // [5][12][ngp] = stl12, snowd12, soilw12, sst12, sice12 (optional); the two grid
    // fields of tcorh / qcorh and their Fourier coefficients
    double *d_surf = nullptr, *d_clim = nullptr, *d_ford = nullptr;
    bool surf_on = false, clim_on = false;
    // fordate's inputs change with the date or a setter: the generation of the
    // setters' inputs and the date of the last fordate (recomputed only on a change)
    long long ford_gen = 1, ford_done = 0;
    int ford_date[2] = {0, 0};
    int ford_count = 0;  // fordate recomputations issued (sml_dyn_fordate_count)
    // step kernels: the fused form (default: 2-3 launches per chained step, FMA
    // contraction) or the 8/9-launch form whose transforms are FFTPACK's separate
    // multiplies and adds (sml_dyn_set_fused; the two agree to rounding)
    bool fused = true;
    bool nograph = false;  // SML_DYN_NOGRAPH=1: the window's launches issued directly, not replayed
    // mod_lflags lradsw (module default .true.) and stloop's istep (at_gcm.f90:81)
    bool lradsw = true;
    int istep = 1;
    // leapfrog replay: one step(2, 2, ...) captured as a hipGraph per lradsw value
    hipStream_t cap_stream = nullptr;
    struct Replay {
        hipGraphExec_t exec = nullptr;
        double key[4] = {0, 0, 0, 0};
        const double *phys = nullptr;
        const DynTables *tab = nullptr;
        bool phys_on = false;
    } replay[2];
    // whole-window replay (sml_dyn_window): stepone + nleap leapfrog steps, one graph
    struct WindowReplay {
        hipGraphExec_t exec = nullptr;
        double key[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        DynTables *tab[3] = {nullptr, nullptr, nullptr};
        // run_model's exit captured behind the window, and with it the entry (iogrid(30)'s
        // specx + k_io_entry) in front of it: their arguments (the per-launch values come
        // from d_xa, written before each launch)
        bool has_exit = false;
        const void *exit_key[16] = {};
    };
    // [prepared entry (sml_dyn_run_model)][entry lradsw] x kReplayWays graphs each, so a
    // caller alternating its forecast / input buffers (ping-pong) replays one graph per
    // buffer set instead of re-capturing the window every call; round-robin eviction
    static constexpr int kReplayWays = 4;
    WindowReplay wreplay[4][kReplayWays];
    int wreplay_next[4] = {0, 0, 0, 0};
    // the next run_model's exit is followed by a store of exit_store_value to
    // *exit_store (sml::dyn_run_model_exit_store: the hybrid loop's forecast hop)
    uint64_t *exit_store = nullptr;
    uint64_t exit_store_value = 0;
    // a graph-captured run_model's per-launch values: [0] the check count the exit waits
    // for, [1] the hop value its store writes, [2] the hop value the entry specx waits for,
    // [3] the window's number, which its first row kernel hands the safety check
    // (k_set_xa right before the graph; k_io_entry when only the exit is captured)
    uint64_t *d_xa = nullptr;
    // the entry inside the window graph (run_model, no capture of the caller's, not under
    // serialised dispatch): the safety check then waits on its own stream for *d_go >=
    // the window's number, which the window's first row kernel stores as it starts
    // (k_io_entry's outputs are released by then) -- no event fork after k_io_entry
    bool entry_graph = true;
    bool serialized = false;  // AMD_SERIALIZE_KERNEL / rocprofv3's counter collection at create
    uint64_t *d_go = nullptr;
    uint64_t go_count = 0;
    // the next fused step's row kernel hands *go_src to *go_dst at its start (one launch)
    const uint64_t *go_src_next = nullptr;
    uint64_t *go_dst_next = nullptr;
    // while a run_model window is captured: the Fourier buffer its last k_st_spec fills
    // with iogrid(31)'s gridy (spectral layout), else null
    double *io_exit = nullptr;
};

namespace {

// uvspec(vor, div) -> (ucos, vcos) at coefficient (m, n), both parts
// (spe_spectral.f90:351-387)
__device__ inline void uvspec_at(const double *vor, const double *div, const DynTables *T, int m, int n, double *uc,
                                 double *vc) {
    const double ux = T->uvdx[n][m];
    double zp[2], zc[2];
    zp[1] = ux * vor[ci(0, m, n)];
    zp[0] = -ux * vor[ci(1, m, n)];
    zc[1] = ux * div[ci(0, m, n)];
    zc[0] = -ux * div[ci(1, m, n)];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        double a, b;
        if (n == 0) {
            a = zc[p] - T->uvdyp[0][m] * vor[ci(p, m, 1)];
            b = zp[p] + T->uvdyp[0][m] * div[ci(p, m, 1)];
        } else if (n == kNX - 1) {
            a = T->uvdym[n][m] * vor[ci(p, m, kNTRUN1 - 1)];
            b = -T->uvdym[n][m] * div[ci(p, m, kNTRUN1 - 1)];
        } else {
            b = -T->uvdym[n][m] * div[ci(p, m, n - 1)] + T->uvdyp[n][m] * div[ci(p, m, n + 1)] + zp[p];
            a = T->uvdym[n][m] * vor[ci(p, m, n - 1)] - T->uvdyp[n][m] * vor[ci(p, m, n + 1)] + zc[p];
        }
        uc[ci(p, m, n)] = a;
        vc[ci(p, m, n)] = b;
    }
}

// geop(1) at level k of one real coefficient c = 2 (m + mx n) + p (dyn_geop.f90:16-32):
// the hydrostatic sum from the bottom, then the free-troposphere lapse-rate
// correction of the zonal-mean row; t = level-1 temperature, all kx levels
__device__ inline double geop_at(const double *t, const double *phis, const DynTables *T, int c, int m, int k) {
    double phi = phis[c] + T->xgeop1[kKX - 1] * t[(size_t)(kKX - 1) * kSF + c];
    for (int kk = kKX - 2; kk >= k; --kk)
        phi = phi + T->xgeop2[kk + 1] * t[(size_t)(kk + 1) * kSF + c] + T->xgeop1[kk] * t[(size_t)kk * kSF + c];
    if (m == 0 && k >= 1 && k <= kKX - 2)
        phi = phi + T->corf[k] * (t[(size_t)(k + 1) * kSF + c] - t[(size_t)(k - 1) * kSF + c]);
    return phi;
}

// ---------------------------------------------------------------- kernels
// prep: inputs of the inverse transforms from time level j2 (grtend :60-99),
// [vor 8 | div 8 | t 8 | tr 8] then at o2 [ucos 8 | vcos 8 | psdx | psdy]; with
// phys, also the level-1 inputs of phypar (phy_phypar.f90:54-66): t1, q1, geop(1),
// ps1 at kPT1.. and ucos1, vcos1 at o2 + 18.  One thread per (m, n).
__global__ void k_dyn_prep(const double *__restrict__ st, double *__restrict__ sin_, const DynTables *__restrict__ T,
                           const double *__restrict__ phis, int j2, int o2, int phys) {
    const int mn = blockIdx.x * blockDim.x + threadIdx.x;
    if (mn >= kMN) return;
    const int k = blockIdx.y;
    const int m = mn % kMX, n = mn / kMX;
    const size_t lev = (size_t)(j2 - 1) * kKX;
    if (k < kKX) {
        const double *vor = st + kOffVor + (lev + k) * kSF, *div = st + kOffDiv + (lev + k) * kSF;
        const double *t = st + kOffT + (lev + k) * kSF, *tr = st + kOffTr + (lev + k) * kSF;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int c = ci(p, m, n);
            sin_[(size_t)k * kSF + c] = vor[c];
            sin_[(size_t)(kKX + k) * kSF + c] = div[c];
            sin_[(size_t)(2 * kKX + k) * kSF + c] = t[c];
            sin_[(size_t)(3 * kKX + k) * kSF + c] = tr[c];
        }
        uvspec_at(vor, div, T, m, n, sin_ + (size_t)(o2 + k) * kSF, sin_ + (size_t)(o2 + kKX + k) * kSF);
        if (phys) {
            const double *vor1 = st + kOffVor + (size_t)k * kSF, *div1 = st + kOffDiv + (size_t)k * kSF;
            const double *t1 = st + kOffT, *tr1 = st + kOffTr + (size_t)k * kSF;
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                const int c = ci(p, m, n);
                sin_[(size_t)(kPT1 + k) * kSF + c] = t1[(size_t)k * kSF + c];
                sin_[(size_t)(kPQ1 + k) * kSF + c] = tr1[c];
                sin_[(size_t)(kPPhi1 + k) * kSF + c] = geop_at(t1, phis, T, c, m, k);
            }
            uvspec_at(vor1, div1, T, m, n, sin_ + (size_t)(o2 + 2 * kKX + 2 + k) * kSF,
                      sin_ + (size_t)(o2 + 3 * kKX + 2 + k) * kSF);
        }
    } else {
        if (phys) {
#pragma unroll
            for (int p = 0; p < 2; ++p) sin_[(size_t)kPPs1 * kSF + ci(p, m, n)] = st[kOffPs + ci(p, m, n)];
        }
        // grad(ps(j2)) -> (psdx, psdy)  (spe_spectral.f90:271-305)
        const double *ps = st + kOffPs + (size_t)(j2 - 1) * kSF;
        double *dx = sin_ + (size_t)(o2 + 2 * kKX) * kSF, *dy = sin_ + (size_t)(o2 + 2 * kKX + 1) * kSF;
        dx[ci(1, m, n)] = T->gradx[m] * ps[ci(0, m, n)];
        dx[ci(0, m, n)] = -T->gradx[m] * ps[ci(1, m, n)];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            double v;
            if (n == 0)
                v = T->gradyp[0][m] * ps[ci(p, m, 1)];
            else if (n == kNX - 1)
                v = -T->gradym[n][m] * ps[ci(p, m, kNTRUN1 - 1)];
            else
                v = -T->gradym[n][m] * ps[ci(p, m, n - 1)] + T->gradyp[n][m] * ps[ci(p, m, n + 1)];
            dy[ci(p, m, n)] = v;
        }
    }
}

// the grid-point dynamics' per-level constants and the Coriolis row (the DynTables
// fields gridpoint_column reads), for an LDS copy in the row kernel
struct GpTab {
    double dhs[kKX], dhsr[kKX], fsgr[kKX], tref[kKX], tref3[kKX], coriol[kIL];
};

// grid-point dynamics of one column (grtend :60-217 and the products of :233-275).
// g(f) = inverse-transformed field f at the column (layout of k_dyn_prep, kcos = 2
// group at o2); hasP: add phypar's tendencies pu/pv/pt/pq [kx] where phypar adds
// them (:225); put(f, v) receives the 73 forward-transform inputs
//   [utend 8 | -u*tgg 8 | -u*trg 8 | vtend 8 | -v*tgg 8 | -v*trg 8]  (x 1/cos in specx)
//   [0.5(u^2+v^2) 8 | ttend 8 | trtend 8 | -umean*px - vmean*py]
template <class GetF, class PutF, class TT>
__device__ inline void gridpoint_products(int o2, GetF g, PutF put, const TT *T);

// products = false: the products of :239-271 are left to gridpoint_products (the row
// kernel runs them on the lane that has slack)
template <class GetF, class PutF, class TT>
__device__ inline void gridpoint_column(int j, int o2, GetF g, bool hasP, const double *pu, const double *pv,
                                        const double *pt, const double *pq, PutF put, const TT *T,
                                        bool products = true) {
    double ug[kKX], vg[kKX], vorg[kKX], divg[kKX], tg[kKX], trg[kKX];
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        vorg[k] = g(k) + T->coriol[j];
        divg[k] = g(kKX + k);
        tg[k] = g(2 * kKX + k);
        trg[k] = g(3 * kKX + k);
        ug[k] = g(o2 + k);
        vg[k] = g(o2 + kKX + k);
    }
    double px = g(o2 + 2 * kKX), py = g(o2 + 2 * kKX + 1);
    double umean = 0.0, vmean = 0.0, dmean = 0.0;
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        umean = umean + ug[k] * T->dhs[k];
        vmean = vmean + vg[k] * T->dhs[k];
        dmean = dmean + divg[k] * T->dhs[k];
    }
    put(kNFwd - 1, -umean * px - vmean * py);  // psdt source (:95-97)
    double puv[kKX], sigdt[kKXP], sigm[kKXP], tgg[kKX], temp[kKXP];
#pragma unroll
    for (int k = 0; k < kKX; ++k) puv[k] = (ug[k] - umean) * px + (vg[k] - vmean) * py;
    sigdt[0] = 0.0;
    sigm[0] = 0.0;
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        sigdt[k + 1] = sigdt[k] - T->dhs[k] * (puv[k] + divg[k] - dmean);
        sigm[k + 1] = sigm[k] - T->dhs[k] * puv[k];
    }
#pragma unroll
    for (int k = 0; k < kKX; ++k) tgg[k] = tg[k] - T->tref[k];
    px = kRgas * px;
    py = kRgas * py;
    // zonal wind tendency
    temp[0] = 0.0;
    temp[kKX] = 0.0;
#pragma unroll
    for (int k = 1; k < kKX; ++k) temp[k] = sigdt[k] * (ug[k] - ug[k - 1]);
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        double u = vg[k] * vorg[k] - tgg[k] * px - (temp[k + 1] + temp[k]) * T->dhsr[k];
        if (hasP) u = u + pu[k];
        put(k, u);
    }
    // meridional wind tendency
#pragma unroll
    for (int k = 1; k < kKX; ++k) temp[k] = sigdt[k] * (vg[k] - vg[k - 1]);
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        double v = -ug[k] * vorg[k] - tgg[k] * py - (temp[k + 1] + temp[k]) * T->dhsr[k];
        if (hasP) v = v + pv[k];
        put(3 * kKX + k, v);
    }
    // temperature tendency
#pragma unroll
    for (int k = 1; k < kKX; ++k)
        temp[k] = sigdt[k] * (tgg[k] - tgg[k - 1]) + sigm[k] * (T->tref[k] - T->tref[k - 1]);
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        double tt = tgg[k] * divg[k] - (temp[k + 1] + temp[k]) * T->dhsr[k] +
                    T->fsgr[k] * tgg[k] * (sigdt[k + 1] + sigdt[k]) + T->tref3[k] * (sigm[k + 1] + sigm[k]) +
                    kAkap * (tg[k] * puv[k] - tgg[k] * dmean);
        if (hasP) tt = tt + pt[k];
        put(7 * kKX + k, tt);
    }
    // tracer tendency: no vertical advection between the top three layers (:179-188)
#pragma unroll
    for (int k = 1; k < kKX; ++k) temp[k] = sigdt[k] * (trg[k] - trg[k - 1]);
    temp[1] = 0.0;
    temp[2] = 0.0;
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        double q = trg[k] * divg[k] - (temp[k + 1] + temp[k]) * T->dhsr[k];
        if (hasP) q = q + pq[k];
        put(8 * kKX + k, q);
    }
    // products for the spectral conversion (:239-271)
    if (products) gridpoint_products(o2, g, put, T);
}

template <class GetF, class PutF, class TT>
__device__ inline void gridpoint_products(int o2, GetF g, PutF put, const TT *T) {
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        const double ug = g(o2 + k), vg = g(o2 + kKX + k), trg = g(3 * kKX + k);
        const double tgg = g(2 * kKX + k) - T->tref[k];
        put(kKX + k, -ug * tgg);
        put(4 * kKX + k, -vg * tgg);
        put(2 * kKX + k, -ug * trg);
        put(5 * kKX + k, -vg * trg);
        put(6 * kKX + k, 0.5 * (ug * ug + vg * vg));
    }
}

// grid-point dynamics, one thread per grid column; G = the inverse-transformed
// fields, P = optional physics tendencies [u 8 | v 8 | t 8 | q 8] in grid space,
// F = the 73 forward-transform inputs (gridpoint_column)
__global__ __launch_bounds__(256) void k_dyn_gridpoint(const double *__restrict__ G, const double *__restrict__ P,
                                                       double *__restrict__ F, const DynTables *__restrict__ T,
                                                       int o2) {
    const int pt = blockIdx.x * blockDim.x + threadIdx.x;
    if (pt >= kGF) return;
    double pu[kKX], pv[kKX], ptt[kKX], pq[kKX];
    if (P) {
#pragma unroll
        for (int k = 0; k < kKX; ++k) {
            pu[k] = P[(size_t)k * kGF + pt];
            pv[k] = P[(size_t)(kKX + k) * kGF + pt];
            ptt[k] = P[(size_t)(2 * kKX + k) * kGF + pt];
            pq[k] = P[(size_t)(3 * kKX + k) * kGF + pt];
        }
    }
    gridpoint_column(
        pt / kIX, o2, [&](int f) { return G[(size_t)f * kGF + pt]; }, P != nullptr, pu, pv, ptt, pq,
        [&](int f, double v) { F[(size_t)f * kGF + pt] = v; }, T);
}

// phypar's physics, one thread per grid column (sml_physics.hpp): level fields
// [kx][ngp] in, tendencies P = [u 8 | v 8 | t 8 | q 8] x ngp out
__global__ __launch_bounds__(64) void k_phys(const double *__restrict__ ug1, const double *__restrict__ vg1,
                                             const double *__restrict__ tg1, const double *__restrict__ qg1,
                                             const double *__restrict__ phig1, const double *__restrict__ pslg1,
                                             const double *__restrict__ bc, double *__restrict__ rad,
                                             const PhysTables *__restrict__ PT, int lradsw, double *__restrict__ P) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= kNGP) return;
    double ua[kKX], va[kKX], ta[kKX], qa[kKX], phi[kKX], ut[kKX], vt[kKX], tt[kKX], qt[kKX];
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        ua[k] = ug1[(size_t)k * kNGP + j];
        va[k] = vg1[(size_t)k * kNGP + j];
        ta[k] = tg1[(size_t)k * kNGP + j];
        qa[k] = qg1[(size_t)k * kNGP + j];
        phi[k] = phig1[(size_t)k * kNGP + j];
    }
    phys_column(j, ua, va, ta, qa, phi, pslg1[j], bc, rad, PT, &PT->fband[0][0], lradsw != 0, ut, vt, tt, qt);
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        P[(size_t)k * kNGP + j] = ut[k];
        P[(size_t)(kKX + k) * kNGP + j] = vt[k];
        P[(size_t)(2 * kKX + k) * kNGP + j] = tt[k];
        P[(size_t)(3 * kKX + k) * kNGP + j] = qt[k];
    }
}

// Table access for the spectral-space stages of one zonal wavenumber m: GTab reads
// the DynTables in device memory (unfused kernels), LTab a per-m copy staged in LDS
// (TabM, the fused k_st_spec).  Vectors by level k, per-(n, m) tables by n, and
// xj(n, k1, k) = xj[m + n - 1][k1][k] (implic's matrix of ll = m + n).
struct TabM {
    double dhs[kKX], dhsr[kKX], fsgr[kKX], tref[kKX], tref1[kKX], tref2[kKX], tref3[kKX];
    double xgeop1[kKX], xgeop2[kKX], corf[kKX], tcorv[kKX], qcorv[kKX], dhsx[kKX];
    double xc[kKX][kKX], xd[kKX][kKX];
    double el2[kNX], elz[kNX], dmp[kNX], dmp1[kNX], dmpd[kNX], dmp1d[kNX], dmps[kNX], dmp1s[kNX], trfilt[kNX];
    double vddym[kNX], vddyp[kNX], gradym[kNX], gradyp[kNX], uvdx[kNX], uvdym[kNX], uvdyp[kNX];
    double gradx, pad_;
    double xj[kKX][kKX][kNX];  // [k1][k][n]: n fastest, so a wave's lanes (one n each) hit distinct LDS banks
};
constexpr int kTabMDoubles = (int)(sizeof(TabM) / sizeof(double));
constexpr int kTabMPad = 2048;  // d_tabm tail: k_st_spec stages whole 16-B rows of 512 threads
static_assert(kTabMDoubles % 2 == 0, "TabM is copied in 16-B pieces");

#define SML_TAB_VEC(X) \
    X(dhs) X(dhsr) X(fsgr) X(tref) X(tref1) X(tref2) X(tref3) X(xgeop1) X(xgeop2) X(corf) X(tcorv) X(qcorv) X(dhsx)
#define SML_TAB_NM(X)                                                                                       \
    X(el2) X(elz) X(dmp) X(dmp1) X(dmpd) X(dmp1d) X(dmps) X(dmp1s) X(trfilt) X(vddym) X(vddyp) X(gradym) \
        X(gradyp) X(uvdx) X(uvdym) X(uvdyp)

struct GTab {
    const DynTables *T;
    int m;
#define X(name) \
    __device__ double name(int k) const { return T->name[k]; }
    SML_TAB_VEC(X)
#undef X
#define X(name) \
    __device__ double name##_n(int n) const { return T->name[n][m]; }
    SML_TAB_NM(X)
#undef X
    __device__ double gradx_m() const { return T->gradx[m]; }
    __device__ double xc(int k1, int k) const { return T->xc[k1][k]; }
    __device__ double xd(int k1, int k) const { return T->xd[k1][k]; }
    __device__ double xj(int n, int k1, int k) const { return T->xj[m + n - 1][k1][k]; }
};

struct LTab {
    const TabM *t;
#define X(name) \
    __device__ double name(int k) const { return t->name[k]; }
    SML_TAB_VEC(X)
#undef X
#define X(name) \
    __device__ double name##_n(int n) const { return t->name[n]; }
    SML_TAB_NM(X)
#undef X
    __device__ double gradx_m() const { return t->gradx; }
    __device__ double xc(int k1, int k) const { return t->xc[k1][k]; }
    __device__ double xd(int k1, int k) const { return t->xd[k1][k]; }
    __device__ double xj(int n, int k1, int k) const { return t->xj[k1][k][n]; }
};

// the value at flat index i of m's TabM, read from the DynTables (host: the per-slot
// TabM copies built at impint time)
__host__ __device__ inline double tabm_value(const DynTables *__restrict__ T, int m, int i) {
    const TabM *z = nullptr;
    const size_t off = (size_t)i * sizeof(double);
#define X(name)                                                                             \
    {                                                                                       \
        const size_t a = offsetof(TabM, name), b = a + sizeof(z->name);                      \
        if (off >= a && off < b) return T->name[(off - a) / sizeof(double)];                 \
    }
    SML_TAB_VEC(X)
#undef X
#define X(name)                                                                             \
    {                                                                                       \
        const size_t a = offsetof(TabM, name), b = a + sizeof(z->name);                      \
        if (off >= a && off < b) return T->name[(off - a) / sizeof(double)][m];              \
    }
    SML_TAB_NM(X)
#undef X
    if (off >= offsetof(TabM, xc) && off < offsetof(TabM, xc) + sizeof(z->xc))
        return (&T->xc[0][0])[(off - offsetof(TabM, xc)) / sizeof(double)];
    if (off >= offsetof(TabM, xd) && off < offsetof(TabM, xd) + sizeof(z->xd))
        return (&T->xd[0][0])[(off - offsetof(TabM, xd)) / sizeof(double)];
    if (off == offsetof(TabM, gradx)) return T->gradx[m];
    if (off >= offsetof(TabM, xj)) {
        const int q = (int)((off - offsetof(TabM, xj)) / sizeof(double));
        const int k1 = q / (kKX * kNX), k = (q / kNX) % kKX, n = q % kNX;
        return m + n >= 1 ? T->xj[m + n - 1][k1][k] : 0.0;
    }
    return 0.0;
}

// vds (spe_spectral.f90:307-349) divergence / vorticity of one coefficient;
// u(pp, nn), v(pp, nn) read part pp of coefficient (m, nn)
template <class U, class V, class TB>
__device__ inline void vds_gen(U u, V v, const TB &tb, int n, int p, double *vor, double *div) {
    const double gx = tb.gradx_m();
    // zp(2)=gradx*u(1), zp(1)=-gradx*u(2); zc likewise from v
    const double ux = u(1 - p, n), vx = v(1 - p, n);
    const double zp = p == 1 ? gx * ux : -gx * ux;
    const double zc = p == 1 ? gx * vx : -gx * vx;
    // the n == 1 / n == ntrun+2 / interior cases all formed (neighbours clamped into
    // the row), then selected: the reference's values without divergent branches,
    // whose dependent reads cost a round trip per case where u, v live in LDS
    static_assert(kNTRUN1 - 1 == kNX - 2, "vds's last row reads n - 1");
    const int nm = n > 0 ? n - 1 : 0, np = n < kNX - 1 ? n + 1 : kNX - 1;
    const double um = u(p, nm), up = u(p, np), vm = v(p, nm), vp = v(p, np);
    const double dym = tb.vddym_n(n), dyp = tb.vddyp_n(n);
    const double vor0 = zc - dyp * up, div0 = zp + dyp * vp;
    const double vorl = dym * um, divl = -dym * vm;
    const double vori = dym * um - dyp * up + zc, divi = -dym * vm + dyp * vp + zp;
    *vor = n == 0 ? vor0 : n == kNX - 1 ? vorl : vori;
    *div = n == 0 ? div0 : n == kNX - 1 ? divl : divi;
}

__device__ inline void vds_at(const double *u, const double *v, const DynTables *T, int m, int n, int p, double *vor,
                              double *div) {
    vds_gen([&](int pp, int nn) { return u[ci(pp, m, nn)]; }, [&](int pp, int nn) { return v[ci(pp, m, nn)]; },
            GTab{T, m}, n, p, vor, div);
}

// combine: spectral tendencies of grtend (:229-278) from the 73 forward transforms
__global__ void k_dyn_combine(const double *__restrict__ S, double *__restrict__ Td, const DynTables *__restrict__ T) {
    const int mn = blockIdx.x * blockDim.x + threadIdx.x;
    if (mn >= kMN) return;
    const int k = blockIdx.y;
    const int m = mn % kMX, n = mn / kMX;
    auto fld = [&](int f) { return S + (size_t)f * kSF; };
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int c = ci(p, m, n);
        double vo, dv, d0, dq, dummy;
        vds_at(fld(k), fld(3 * kKX + k), T, m, n, p, &vo, &dv);              // vdspec(utend, vtend)
        const double lapv = -(fld(6 * kKX + k)[c] * T->el2[n][m]);          // lap(spec(0.5(u2+v2)))
        Td[kTVor + (size_t)k * kSF + c] = vo;
        Td[kTDiv + (size_t)k * kSF + c] = dv - lapv;
        vds_at(fld(kKX + k), fld(4 * kKX + k), T, m, n, p, &dummy, &d0);     // vdspec(-u tgg, -v tgg)
        Td[kTT + (size_t)k * kSF + c] = d0 + fld(7 * kKX + k)[c];
        vds_at(fld(2 * kKX + k), fld(5 * kKX + k), T, m, n, p, &dummy, &dq); // vdspec(-u trg, -v trg)
        Td[kTTr + (size_t)k * kSF + c] = dq + fld(8 * kKX + k)[c];
        if (k == 0) Td[kTPs + c] = (m == 0 && n == 0) ? 0.0 : fld(kNFwd - 1)[c];  // psdt(1,1) = 0
    }
}

// tail: sptend + geop + implic + hordif + drag + timint of one real coefficient c
// (= Re/Im of (m, n)) at level k, given grtend's spectral tendencies of (c, k).
// The CW coefficients x 8 levels of a block share sh[3][kx][CW] (LDS) for the
// vertical couplings (dmeanc, sigdtc, geop, implic's level matrices); every sum
// runs over k in the reference's order.  The whole block must call it (barriers).
template <int CW, class SA, class TB>
__device__ inline void tail_coef(SA S, double *__restrict__ Td, double *__restrict__ phi_out,
                                 const double *__restrict__ phis, const double *__restrict__ tcorh,
                                 const double *__restrict__ qcorh, int fc, const TB &tb,
                                 double (*sh)[kKX][CW], int cc, int k, int c, int m, int n, double vordt, double divdt,
                                 double tdt, double trdt, double psdt, int j1, int j4, double dt, double alph,
                                 double rob, double wil) {
    // S(var, lev, kk): the state of coefficient c (var 0..4 = vor, div, t, tr, ps at
    // kk = 0; lev 1 or 2), updated in place; phis / tcorh / qcorh at index fc
    // ---- sptend(divdt, tdt, psdt, j4)  (dyn_sptend.f90:29-66)
    sh[0][k][cc] = S(1, j4, k);
    sh[1][k][cc] = S(2, j4, k);
    __syncthreads();
    double dmeanc = 0.0;
#pragma unroll
    for (int kk = 0; kk < kKX; ++kk) dmeanc = dmeanc + sh[0][kk][cc] * tb.dhs(kk);
    psdt = psdt - dmeanc;
    if (m == 0 && n == 0) psdt = 0.0;  // psdt(1,1) = 0
    double sig_k = 0.0, sig_k1 = 0.0;  // sigdtc(k), sigdtc(k+1); sigdtc(1) = sigdtc(kxp) = 0
    {
        double sg = 0.0;
#pragma unroll
        for (int kk = 0; kk < kKX - 1; ++kk) {
            const double nx_ = sg - tb.dhs(kk) * (sh[0][kk][cc] - dmeanc);
            if (kk == k - 1) sig_k = nx_;
            if (kk == k) sig_k1 = nx_;
            sg = nx_;
        }
    }
    // (neighbour levels clamped and the edge cases selected: no branch around a read)
    const int km = k > 0 ? k - 1 : 0, kp = k < kKX - 1 ? k + 1 : kKX - 1;
    const double trk = tb.tref(k), trm = tb.tref(km), trp = tb.tref(kp);
    const double dumk_k = (k == 0) ? 0.0 : sig_k * (trk - trm);
    const double dumk_k1 = (k == kKX - 1) ? 0.0 : sig_k1 * (trp - trk);
    tdt = tdt - (dumk_k1 + dumk_k) * tb.dhsr(k) + tb.tref3(k) * (sig_k1 + sig_k) - tb.tref2(k) * dmeanc;
    // geop(j4)  (dyn_geop.f90:16-32)
    // (every level's term formed, the ones below k selected away: the sum and its
    // order are the reference's, and the LDS reads issue together instead of one
    // dependent round trip per level of a runtime-bounded loop)
    double phi = phis[fc] + tb.xgeop1(kKX - 1) * sh[1][kKX - 1][cc];
#pragma unroll
    for (int kk = kKX - 2; kk >= 0; --kk) {
        const double nx = phi + tb.xgeop2(kk + 1) * sh[1][kk + 1][cc] + tb.xgeop1(kk) * sh[1][kk][cc];
        phi = kk >= k ? nx : phi;
    }
    {
        const double pc = phi + tb.corf(k) * (sh[1][kp][cc] - sh[1][km][cc]);
        if (m == 0 && k >= 1 && k <= kKX - 2) phi = pc;
    }
    if (phi_out) phi_out[(size_t)k * kSF + c] = phi;
    {
        const double d1 = phi + kRgas * tb.tref(k) * S(4, j4, 0);
        const double lapd = -(d1 * tb.el2_n(n));
        divdt = divdt - lapd;
    }
    // ---- implic(divdt, tdt, psdt)  (dyn_implic.f90:22-67)
    if (alph != 0.0) {
        // tdt into the third plane: sptend's reads of sh[0] need no barrier of their
        // own before it (sh[1]'s geop reads end at the next one, before yf is written)
        sh[2][k][cc] = tdt;
        __syncthreads();
        double ye = 0.0;
#pragma unroll
        for (int k1 = 0; k1 < kKX; ++k1) ye = ye + tb.xd(k1, k) * sh[2][k1][cc];
        ye = ye + tb.tref1(k) * psdt;
        sh[1][k][cc] = divdt + tb.elz_n(n) * ye;  // yf
        __syncthreads();
        divdt = 0.0;
        const int ll = m + n;
        if (ll != 0) {
#pragma unroll
            for (int k1 = 0; k1 < kKX; ++k1) divdt = divdt + tb.xj(n, k1, k) * sh[1][k1][cc];
        }
        sh[0][k][cc] = divdt;
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kKX; ++kk) psdt = psdt - sh[0][kk][cc] * tb.dhsx(kk);
#pragma unroll
        for (int k1 = 0; k1 < kKX; ++k1) tdt = tdt + tb.xc(k1, k) * sh[0][k1][cc];
    }
    // ---- horizontal diffusion (dyn_step.f90:60-112, hordif :130-151)
    const double dmp = tb.dmp_n(n), dmp1 = tb.dmp1_n(n), dmpd = tb.dmpd_n(n), dmp1d = tb.dmp1d_n(n);
    vordt = (vordt - dmp * S(0, 1, k)) * dmp1;
    divdt = (divdt - dmpd * S(1, 1, k)) * dmp1d;
    const double ctmp = S(2, 1, k) + tcorh[fc] * tb.tcorv(k);
    tdt = (tdt - dmp * ctmp) * dmp1;
    if (k == 0) {
        if (m == 0) {  // stratospheric drag on the zonal mean, top level (:78-82)
            const double sdrag = 1. / (kTdrs * 3600.);
            vordt = vordt - sdrag * S(0, 1, 0);
            divdt = divdt - sdrag * S(1, 1, 0);
        }
        const double dmps = tb.dmps_n(n), dmp1s = tb.dmp1s_n(n);
        vordt = (vordt - dmps * S(0, 1, 0)) * dmp1s;
        divdt = (divdt - dmps * S(1, 1, 0)) * dmp1s;
        tdt = (tdt - dmps * ctmp) * dmp1s;
    }
    {
        const double cq = S(3, 1, k) + qcorh[fc] * tb.qcorv(k);
        trdt = (trdt - dmpd * cq) * dmp1d;
    }
    if (dt <= 0.0) {  // tendencies only (dyn_step.f90:109)
        if (!Td) return;
        Td[kTVor + (size_t)k * kSF + c] = vordt;
        Td[kTDiv + (size_t)k * kSF + c] = divdt;
        Td[kTT + (size_t)k * kSF + c] = tdt;
        Td[kTTr + (size_t)k * kSF + c] = trdt;
        if (k == 0) Td[kTPs + c] = psdt;
        return;
    }
    // ---- timint with the Robert-Williams filter (dyn_step.f90:153-190)
    const double eps = (j1 == 1) ? 0.0 : rob;
    const double trf = tb.trfilt_n(n);
    auto timint = [&](int var, int kk, double fdt) {
        fdt = fdt * trf;  // trunct
        double &f1 = S(var, 1, kk);
        double &f2 = S(var, 2, kk);
        const double fj1_old = (j1 == 1) ? f1 : f2;
        const double fnew = f1 + dt * fdt;
        const double f1new = fj1_old + wil * eps * (f1 - 2 * fj1_old + fnew);
        const double fj1_new = (j1 == 1) ? f1new : fj1_old;
        f2 = fnew - (1 - wil) * eps * (f1new - 2 * fj1_new + fnew);
        f1 = f1new;
    };
    if (k == 0) timint(4, 0, psdt);
    timint(0, k, vordt);
    timint(1, k, divdt);
    timint(2, k, tdt);
    timint(3, k, trdt);
}

// the barriers tail_coef executes, for threads of a block that hold no coefficient
// (keep in step with tail_coef: 1 in sptend, 3 in implic when alph != 0)
__device__ inline void tail_coef_barriers(double alph) {
    __syncthreads();
    if (alph != 0.0) {
        __syncthreads();
        __syncthreads();
        __syncthreads();
    }
}

// tail kernel of the unfused step: a block owns 32 real coefficients x 8 levels
constexpr int kTailC = 32;
__global__ __launch_bounds__(256) void k_dyn_tail(double *__restrict__ st, double *__restrict__ Td,
                                                  double *__restrict__ phi_out, const double *__restrict__ phis,
                                                  const double *__restrict__ tcorh, const double *__restrict__ qcorh,
                                                  const DynTables *__restrict__ T, int j1, int j4, double dt,
                                                  double alph, double rob, double wil) {
    __shared__ double sh[3][kKX][kTailC];
    const int cc = threadIdx.x & (kTailC - 1), k = threadIdx.x / kTailC;
    const int c = blockIdx.x * kTailC + cc;  // 0 .. 1983 = 2 * (m + mx n) + p
    const int mn = c >> 1, m = mn % kMX, n = mn / kMX;
    auto S = [&](int var, int lev, int kk) -> double & {  // reference layout; ps has one level
        if (var == 4) return st[kOffPs + (size_t)(lev - 1) * kSF + c];
        const size_t off = var == 0 ? kOffVor : var == 1 ? kOffDiv : var == 2 ? kOffT : kOffTr;
        return st[off + ((size_t)(lev - 1) * kKX + kk) * kSF + c];
    };
    tail_coef<kTailC>(S, Td, phi_out, phis, tcorh, qcorh, c, GTab{T, m}, sh, cc, k, c, m, n, Td[kTVor + (size_t)k * kSF + c],
                      Td[kTDiv + (size_t)k * kSF + c], Td[kTT + (size_t)k * kSF + c], Td[kTTr + (size_t)k * kSF + c],
                      Td[kTPs + c], j1, j4, dt, alph, rob, wil);
}

// ======================================================= fused step
// The step's stages regrouped at the all-to-all seams of the spectral transform
// (spectral <-> Fourier per zonal wavenumber m, Fourier <-> grid per latitude row):
//   k_st_rows   (latitude row j, no GPU physics): gridx (FFT) -> LDS -> grid-point
//               dynamics -> LDS -> specx (FFT)
//   k_st_gridspec_p (with GPU physics): gridx, the grid-point dynamics beside phypar
//               (its roles on waves of their own), specx, in one launch per row
//   k_st_spec   (zonal wavenumber m, 512 threads = 64 coefficients x 8 levels):
//               specy -> combine (vds, lap) -> sptend / geop / implic / hordif /
//               timint -> the NEXT step's inverse-transform inputs from the new
//               state (uvspec, grad, geop) -> gridy
//   k_st_inv    (m): the inverse-transform inputs + gridy from the state in memory,
//               for a step that follows no fused step (window start)
// A leapfrog step is 2 launches (with GPU physics: k_st_gridspec_p + k_st_spec)
// instead of 8 / 9.  Each block first stages everything it reads -- the m's slice of
// the state, the row's Fourier coefficients -- in LDS with coalesced loads: the
// fused step keeps its own m-major copies of the state ([m][var][lev][k][n p],
// k_state_to_m before a run of fused steps; the run's last k_st_spec writes the
// reference layout back) and of the forward Fourier coefficients ([m][lat][f][p]),
// so each block's slice is contiguous.  Every stage keeps the unfused kernels'
// arithmetic, operand order and MFMA tiling: results are bit-identical to them
// (tests/test_physics_gpu.py).
typedef double d4 __attribute__((ext_vector_type(4)));
#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

// one 16-B store of a (Re, Im) pair: the inter-kernel hand-offs of the fused step (vfm,
// the next step's varm and state).  (Stored write-through, sc1, the kernel boundary
// got cheaper but the stores far slower: measured and removed)
__device__ __attribute__((always_inline)) inline void store2(double *base, size_t idx, double a, double b) {
    *reinterpret_cast<double2 *>(base + idx) = double2{a, b};
}

constexpr int kCW = 2 * kNX;                  // real coefficients (n, p) of one m
// iogrid's field-major work layout, both directions: [u 8 | v 8 | t 8 | q 8 | ps]
constexpr int kNIo = 4 * kKX + 1;
constexpr int kNIoWind = 2 * kKX;
constexpr int kSM = 5 * 2 * kKX * kCW;        // m-major state slice: [var 5][lev 2][k][cc] (ps at k = 0)
// m-major Fourier coefficients, [m][lat][f][p]: a latitude row's fields are contiguous
// per m (the row kernels' 16-B stores / loads coalesce across the fields' lanes) and
// each m's slice is contiguous (the spectral kernels stage it with coalesced loads)
constexpr int kVLs = 2 * kNFwd;               // forward: latitude stride
constexpr int kVFm = kIL * kVLs;              // forward: per-m slice
constexpr int kVIl = 2 * kNInvMax;            // inverse: latitude stride
constexpr int kVIm = kIL * kVIl;              // inverse: per-m slice
__device__ inline int smi(int var, int lev, int k, int cc) { return ((var * 2 + lev - 1) * kKX + k) * kCW + cc; }

// diagnostic phase stamps (SML_DYN_STAMPS=1 at creation): thread 0 of each block
// writes wall_clock64() (100 MHz) at phase boundaries, [kernel][block][8]
constexpr int kStampKernels = 4, kStampBlocks = 96, kStamps = 8;  // kernels: grid/rows, spec, specx, last spec
__device__ inline void stamp(long long *dbg, int kern, int i) {
    if (dbg && threadIdx.x == 0) dbg[((size_t)kern * kStampBlocks + blockIdx.x) * kStamps + i] = wall_clock64();
}

// reference state layout <-> the fused step's m-major copy
__global__ void k_state_to_m(const double *__restrict__ st, double *__restrict__ sm) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kMX * kSM) return;
    const int m = e / kSM, i = e % kSM;
    const int cc = i % kCW, k = (i / kCW) % kKX, lev = (i / (kCW * kKX)) % 2, var = i / (2 * kKX * kCW);
    const int c = ci(cc & 1, m, cc >> 1);
    double v = 0.0;
    if (var < 4) {
        const size_t off = var == 0 ? kOffVor : var == 1 ? kOffDiv : var == 2 ? kOffT : kOffTr;
        v = st[off + ((size_t)lev * kKX + k) * kSF + c];
    } else if (k == 0) {
        v = st[kOffPs + (size_t)lev * kSF + c];
    }
    sm[e] = v;
}

// element i of m's slice (smi layout) into the reference-layout state
__device__ inline void put_state(double *__restrict__ st, int m, int i, double v) {
    const int cc = i % kCW, k = (i / kCW) % kKX, lev = (i / (kCW * kKX)) % 2, var = i / (2 * kKX * kCW);
    const int c = ci(cc & 1, m, cc >> 1);
    if (var < 4) {
        const size_t off = var == 0 ? kOffVor : var == 1 ? kOffDiv : var == 2 ? kOffT : kOffTr;
        st[off + ((size_t)lev * kKX + k) * kSF + c] = v;
    } else if (k == 0) {
        st[kOffPs + (size_t)lev * kSF + c] = v;
    }
}


// uvspec (spe_spectral.f90:351-387) of coefficient (n, p) at level k, time level lev,
// from an m's state slice Sst (smi layout) -> ucos (u), vcos (v).  Branch-free: every
// case's operands read (neighbour indices clamped) and its expression formed, then the
// case selected -- the reference's n == 1 / n == ntrun+2 / interior values without a
// divergent branch and its dependent LDS round trip per case (n and p vary across a
// wave's lanes)
template <class TB>
__device__ inline void uvspec_sel(const double *Sst, const TB &tb, int lev, int k, int n, int p, double *u,
                                  double *v) {
    static_assert(kNTRUN1 - 1 == kNX - 2, "uvspec's last row reads n - 1");
    const int nm = n > 0 ? n - 1 : 0, np = n < kNX - 1 ? n + 1 : kNX - 1;
    const bool first = n == 0, last = n == kNX - 1;
    const double vor_m = Sst[smi(0, lev, k, 2 * nm + p)], vor_p = Sst[smi(0, lev, k, 2 * np + p)];
    const double div_m = Sst[smi(1, lev, k, 2 * nm + p)], div_p = Sst[smi(1, lev, k, 2 * np + p)];
    const double vor_x = Sst[smi(0, lev, k, 2 * n + 1 - p)], div_x = Sst[smi(1, lev, k, 2 * n + 1 - p)];
    const double ux = tb.uvdx_n(n), uvdym = tb.uvdym_n(n), uvdyp = tb.uvdyp_n(n);
    const double zc = p == 1 ? ux * div_x : -ux * div_x;
    const double u0 = zc - uvdyp * vor_p, ul = uvdym * vor_m, um = uvdym * vor_m - uvdyp * vor_p + zc;
    const double zp = p == 1 ? ux * vor_x : -ux * vor_x;
    const double v0 = zp + uvdyp * div_p, vl = -uvdym * div_m, vm = -uvdym * div_m + uvdyp * div_p + zp;
    *u = first ? u0 : last ? ul : um;
    *v = first ? v0 : last ? vl : vm;
}

// The inverse-transform inputs of one m (k_dyn_prep's fields, same expressions)
// from the m's state slice Sst (smi layout); writes In[f][kCW] for f < nin.  The
// whole block calls it.
template <class TB>
__device__ inline void inv_inputs(const double *Sst, double *In, const double *phis_m, const TB &tb, int m, int j2,
                                  int n1, int nin) {
    // one thread per (coefficient cc = 2 n + p, level k) (512 threads): the fields of
    // level k, in the same expressions as k_dyn_prep
    const bool phys = nin > kNInv;
    const int cc = threadIdx.x & (kCW - 1), k = threadIdx.x / kCW, n = cc >> 1, p = cc & 1;
    auto sv = [&](int var, int lev, int kk, int c2) { return Sst[smi(var, lev, kk, c2)]; };
    auto put = [&](int f, double v) { In[f * kCW + cc] = v; };
#pragma unroll
    for (int var = 0; var < 4; ++var) put(var * kKX + k, sv(var, j2, k, cc));
    // uvspec of level lev at k -> ucos (field fu), vcos (fv)
    const int nm = n > 0 ? n - 1 : 0, np = n < kNX - 1 ? n + 1 : kNX - 1;
    const bool first = n == 0, last = n == kNX - 1;
    auto uvspec = [&](int lev, int fu, int fv) {
        double u, v;
        uvspec_sel(Sst, tb, lev, k, n, p, &u, &v);
        put(fu, u);
        put(fv, v);
    };
    uvspec(j2, n1 + k, n1 + kKX + k);
    if (k == 0) {  // grad(ps(j2)) (wave-uniform branch; the n cases selected as in uvspec)
        const double ps_x = sv(4, j2, 0, 2 * n + 1 - p), ps_m = sv(4, j2, 0, 2 * nm + p), ps_p = sv(4, j2, 0, 2 * np + p);
        const double gx = tb.gradx_m(), gym = tb.gradym_n(n), gyp = tb.gradyp_n(n);
        put(n1 + 2 * kKX, p == 1 ? gx * ps_x : -gx * ps_x);
        const double v0 = gyp * ps_p, vl = -gym * ps_m, vm = -gym * ps_m + gyp * ps_p;
        put(n1 + 2 * kKX + 1, first ? v0 : last ? vl : vm);
    }
    if (!phys) return;
    // phypar's level-1 inputs: t1, q1, geop(1) (geop_at), ps1, ucos1, vcos1
    put(kPT1 + k, sv(2, 1, k, cc));
    put(kPQ1 + k, sv(3, 1, k, cc));
    double phi = phis_m[cc] + tb.xgeop1(kKX - 1) * sv(2, 1, kKX - 1, cc);
#pragma unroll
    for (int kk = kKX - 2; kk >= 0; --kk) {  // levels below k selected away (as in tail_coef)
        const double nx = phi + tb.xgeop2(kk + 1) * sv(2, 1, kk + 1, cc) + tb.xgeop1(kk) * sv(2, 1, kk, cc);
        phi = kk >= k ? nx : phi;
    }
    {
        const int km = k > 0 ? k - 1 : 0, kp = k < kKX - 1 ? k + 1 : kKX - 1;
        const double pc = phi + tb.corf(k) * (sv(2, 1, kp, cc) - sv(2, 1, km, cc));
        if (m == 0 && k >= 1 && k <= kKX - 2) phi = pc;
    }
    put(kPPhi1 + k, phi);
    if (k == 0) put(kPPs1, sv(4, 1, 0, cc));
    uvspec(1, n1 + 2 * kKX + 2 + k, n1 + 3 * kKX + 2 + k);
}

// gridy of In[f][kCW] (this m) -> vim[m][lat][f][p] (k_gridy's tiling: one wave per
// 8-field x Re/Im tile, waves of the block stride over the tiles)
// the Legendre operands of gridy_m for this lane (loaded once per wave)
struct GridyB {
    double b00[4], b01[4], b10[4], b11[4];
};
// the same operands from a copy of pinv's m-slice [n][32] (LDS)
__device__ inline GridyB gridy_operands_slice(const double *pm) {
    const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
    GridyB g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int n_odd = 2 * (4 * s + kk), n_even = n_odd + 1;
        g.b00[s] = pm[n_odd * 32 + r];
        g.b01[s] = pm[n_odd * 32 + 16 + r];
        g.b10[s] = pm[n_even * 32 + r];
        g.b11[s] = pm[n_even * 32 + 16 + r];
    }
    return g;
}

__device__ inline GridyB gridy_operands(const double *__restrict__ pinv, int m) {
    const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
    const double *pm = pinv + (size_t)m * kNX * 32;
    GridyB g;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int n_odd = 2 * (4 * s + kk), n_even = n_odd + 1;
        g.b00[s] = pm[n_odd * 32 + r];
        g.b01[s] = pm[n_odd * 32 + 16 + r];
        g.b10[s] = pm[n_even * 32 + r];
        g.b11[s] = pm[n_even * 32 + 16 + r];
    }
    return g;
}

__device__ inline void gridy_m(const double *In, const GridyB &gb, double *__restrict__ varm, int m, int nf,
                               int tile0 = 0, int tile1 = -1) {
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
    const int tend = tile1 < 0 ? (nf + 7) / 8 : tile1;
    // work unit u = (tile, latitude half): half 0 the rows j < 16 (b00 / b10), half 1
    // j >= 16 (b01 / b11).  Whole tiles left the SIMDs uneven (k_st_spec's 6 tiles on
    // 8 waves: 2 tiles on two SIMDs, 1 on the others); half tiles give every SIMD 1.5
    for (int u = wave; u < 2 * (tend - tile0); u += nw) {
        const int tile = tile0 + (u >> 1), half = u & 1;
        const int f0 = tile * 8;
        const int fa = f0 + (r >> 1), p = r & 1;
        const bool ok = fa < nf;
        const double *a = In + (ok ? fa : 0) * kCW + p;
        d4 accS = {0, 0, 0, 0}, accA = accS;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int n_odd = 2 * (4 * s + kk);  // n = 1,3,.. (1-based): symmetric part
            const int n_even = n_odd + 1;        // n = 2,4,..: antisymmetric part
            const double a0 = ok ? a[2 * n_odd] : 0.0;
            const double a1 = ok ? a[2 * n_even] : 0.0;
            // the transposed product (Legendre operand first: the same products summed
            // in the same order), so a lane's outputs are latitude rows kk + 4 q of
            // field-part column r: a store instruction writes 16 consecutive doubles of
            // 4 latitudes (4 lines) instead of 4 of 16 latitudes (16 lines)
            accS = MFMA64(half ? gb.b01[s] : gb.b00[s], a0, accS);
            accA = MFMA64(half ? gb.b11[s] : gb.b10[s], a1, accA);
        }
        if (!ok) continue;
        // m-major inverse Fourier coefficients vim[m][lat][f][p]: column r = 2 (fa - f0) + p
        double *vr = varm + (size_t)m * kVIm + fa * 2 + p;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int j = 16 * half + kk + 4 * q;
            if (j >= kIY) continue;
            const double sym = accS[q], asym = accA[q];
            vr[(kIL - 1 - j) * kVIl] = sym + asym;
            vr[j * kVIl] = sym - asym;
        }
    }
}

// gridy_m with the spectral module's Fourier layout [f][lat][2 m + p] (k_gridy's
// stores): iogrid(31)'s inverse Legendre of the io fields, fused into the window's
// last per-m kernel (run_model)
__device__ inline void gridy_io(const double *In, const GridyB &gb, double *__restrict__ varm, int m, int nf) {
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
    for (int tile = wave; tile < (nf + 7) / 8; tile += nw) {
        const int f0 = tile * 8;
        const int fa = f0 + (r >> 1), p = r & 1;
        const bool ok = fa < nf;
        const double *a = In + (ok ? fa : 0) * kCW + p;
        d4 acc00 = {0, 0, 0, 0}, acc01 = acc00, acc10 = acc00, acc11 = acc00;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int n_odd = 2 * (4 * s + kk);
            const int n_even = n_odd + 1;
            const double a0 = ok ? a[2 * n_odd] : 0.0;
            const double a1 = ok ? a[2 * n_even] : 0.0;
            acc00 = MFMA64(a0, gb.b00[s], acc00);
            acc01 = MFMA64(a0, gb.b01[s], acc01);
            acc10 = MFMA64(a1, gb.b10[s], acc10);
            acc11 = MFMA64(a1, gb.b11[s], acc11);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = kk + 4 * q;
            const int f = f0 + (row >> 1);
            if (f >= nf) continue;
            double *vr = varm + (size_t)f * kVarmField + 2 * m + (row & 1);
            {
                const int j = r;
                const double sym = acc00[q], asym = acc10[q];
                vr[(kIL - 1 - j) * kMX2] = sym + asym;
                vr[j * kMX2] = sym - asym;
            }
            const int j = 16 + r;
            if (j < kIY) {
                const double sym = acc01[q], asym = acc11[q];
                vr[(kIL - 1 - j) * kMX2] = sym + asym;
                vr[j * kMX2] = sym - asym;
            }
        }
    }
}

// iogrid(31)'s k_io_prep at (coefficient cc, level k) from time level 1 of an m-major
// state slice: uvspec of (vor, div), copies of t, tr, ps -> put(field, value) in the
// io layout [u 8 | v 8 | t 8 | q 8 | ps] (the same expressions as uvspec_at)
template <class TB, class Put>
__device__ inline void io_prep_m(const double *Sst, const TB &tb, int k, int cc, Put put) {
    const int n = cc >> 1, p = cc & 1;
    double a, b;
    uvspec_sel(Sst, tb, 1, k, n, p, &a, &b);
    put(k, a);
    put(kKX + k, b);
    put(2 * kKX + k, Sst[smi(2, 1, k, cc)]);
    put(3 * kKX + k, Sst[smi(3, 1, k, cc)]);
    if (k == 0) put(4 * kKX, Sst[smi(4, 1, 0, cc)]);
}

// stage the m's forcing (phis, tcorh, qcorh: reference layout) into Fm[3][kCW]
__device__ inline void load_forcing_m(double *Fm, const double *__restrict__ phis, const double *__restrict__ tcorh,
                                      const double *__restrict__ qcorh, int m) {
    for (int i = threadIdx.x; i < 3 * kCW; i += blockDim.x) {
        const int which = i / kCW, cc = i % kCW;
        const double *src = which == 0 ? phis : which == 1 ? tcorh : qcorh;
        Fm[i] = src[ci(cc & 1, m, cc >> 1)];
    }
}

constexpr int kSpecThreads = kCW * kKX;  // 512: one thread per (coefficient, level) of one m
constexpr int kSpecBlk = 512;             // k_st_spec's block (768: specy -0.6 us, staging +1.2 us, gridy unchanged)
constexpr int kSpecSplit = 2;             // k_st_spec blocks per m (the next step's gridy tiles split between them)
// k_st_spec's grid: block b takes m = b % kSpecStride, half = b / kSpecStride.  A
// launch on a stream places block b on the same XCD every time, the same for every
// kernel of the stream (tools/probe_xcd_l2.hip: XCD = (b + c) mod 8), so with a
// stride of 32 (two idle blocks) both blocks of an m share the XCD of the lead block
// that wrote the m's state in the previous step (and of k_io_entry's block m): the
// slice and the m's tables are L2 hits for both, and the second block's copy of the
// m's Fourier coefficients merges with the first's in that L2.  Stride 31 (62 blocks):
// the second block's reads cross XCDs; same-box A/B: window 0.822 -> 0.800 ms,
// 1006.6 / 1013.5 -> 1018.9 / 1032.2 steps/s (profiles/r03d).  Speed only: any
// placement gives the same results.
#ifndef SML_SPEC_STRIDE
#define SML_SPEC_STRIDE 32
#endif
#ifndef SML_SPEC_VFM_FIRST
#define SML_SPEC_VFM_FIRST 0
#endif
constexpr int kSpecStride = SML_SPEC_STRIDE;
static_assert(kSpecStride >= kMX, "k_st_spec grid stride");

// window start: the inverse transforms of step (.., j2) from the m-major state
__global__ __launch_bounds__(kSpecThreads) void k_st_inv(const double *__restrict__ sm, const double *__restrict__ phis,
                                                         const DynTables *__restrict__ T,
                                                         const double *__restrict__ pinv, double *__restrict__ varm,
                                                         int j2, int n1, int nin) {
    __shared__ double Sst[kSM];
    __shared__ double In[kNInvMax * kCW];
    __shared__ double Fm[kCW];
    const int m = blockIdx.x;
    const double *src = sm + (size_t)m * kSM;
    for (int i = threadIdx.x; i < kSM / 2; i += blockDim.x)
        reinterpret_cast<double2 *>(Sst)[i] = reinterpret_cast<const double2 *>(src)[i];
    for (int cc = threadIdx.x; cc < kCW; cc += blockDim.x) Fm[cc] = phis[ci(cc & 1, m, cc >> 1)];
    __syncthreads();
    inv_inputs(Sst, In, Fm, GTab{T, m}, m, j2, n1, nin);
    __syncthreads();
    gridy_m(In, gridy_operands(pinv, m), varm, m, nin);
}

// Fourier stage of one latitude row: FFTPACK's real FFT (sml_fft.hpp, the reference's
// rfftb / rfftf operation order), one transform per thread held in registers; the
// row's grid values meet the column-wise grid-point stage in LDS, element-major
// A[lon][f] (row stride kRowLd, odd: the column threads' reads spread over banks).
constexpr int kRowThreads = 128, kRowLd = 97;
static_assert(kNInvMax <= kRowThreads && kNFwd <= kRowThreads && kIX <= kRowThreads, "one thread per transform");

// gridx of field f, row j (spe_subfft_fftpack.f90:24-45): packing, rfftb, x cosgr(j)
// for kcos = 2; the 96 values into A[lon][f]
__device__ __attribute__((always_inline)) inline void row_gridx(double *A, const double *__restrict__ varm, const double *__restrict__ wa, int f,
                                 int j, bool kcos2, double cj) {
    // the m-major coefficients vim[m][lat][f][p] of (f, j): coefficient c = 2 m + p
    const double *v = varm + (size_t)j * kVIl + f * 2;
    auto V = [&](int c) { return v[(size_t)(c >> 1) * kVIm + (c & 1)]; };
    double x[kFftN];
    x[0] = V(0);
#pragma unroll
    for (int e = 1; e <= kMX2 - 2; ++e) x[e] = V(e + 1);
#pragma unroll
    for (int e = kMX2 - 1; e < kFftN; ++e) x[e] = 0.0;
    fft::rfftb96_reg(x, wa);
#pragma unroll
    for (int e = 0; e < kFftN; ++e) A[e * kRowLd + f] = kcos2 ? x[e] * cj : x[e];
}

// specx of field f, row j from x[96] (already x cosgr(j) where vdspec scales):
// rfftf, varm(1) = fvar(1)/ix, varm(2) = 0, varm(m) = fvar(m-1)/ix, into the m-major
// forward coefficients vfm[m][f][j][p]
__device__ __attribute__((always_inline)) inline void row_specx(double *x, double *__restrict__ vfm, const double *__restrict__ wa, int f, int j) {
    fft::rfftf96_reg(x, wa);
    const double scale = 1. / (double)kIX;
    double *o = vfm + (size_t)j * kVLs + f * 2;
    o[0] = x[0] * scale;
    o[1] = 0.0;
#pragma unroll
    for (int c = 2; c < kMX2; ++c) o[(size_t)(c >> 1) * kVFm + (c & 1)] = x[c - 1] * scale;
}

// The row kernel's transforms on lane pairs (sml_fft.hpp rfftb96_half /
// rfftf96_combine): lane h of a pair does half h of FFTPACK's n = 96 transform, so a
// lane's dependent chain is about half of a whole transform's.
// gridx half h of field f, row j: grid points 2 q + h into A (x cosgr where kcos2)
// FFTPACK's half-complex input of field f, row j: x[0] = a0, x[2m-1] = Re, x[2m] = Im
// (m <= 30), 0 beyond (x(e) is a compile-time zero there)
__device__ __attribute__((always_inline)) inline void row_gridx_load(const double *__restrict__ varm, int f, int j,
                                                                     double (&xi)[kMX2 - 1]) {
    const double *v = varm + (size_t)j * kVIl + f * 2;
    xi[0] = v[0];  // a0 (coefficient c = 0); x[e] = coefficient c = e + 1 for e >= 1
#pragma unroll
    for (int e = 1; e < kMX2 - 1; ++e) xi[e] = v[(size_t)((e + 1) >> 1) * kVIm + ((e + 1) & 1)];
    // every load in flight before the first use: left alone, the scheduler hoisted
    // radb2's first add (x(0) + a zero) between the loads, and its wait cost a
    // whole memory round trip before the remaining loads issued
    __builtin_amdgcn_sched_barrier(0);
}

__device__ __attribute__((always_inline)) inline void row_gridx_half(double *A, const double (&xi)[kMX2 - 1],
                                                                     const double *__restrict__ wa, int f,
                                                                     bool kcos2, double cj, int h) {
    double y[48];
    fft::rfftb96_half([&](int e) { return e <= kMX2 - 2 ? xi[e] : 0.0; }, h, y, wa);
#pragma unroll
    for (int q = 0; q < 48; ++q) A[(2 * q + h) * kRowLd + f] = kcos2 ? y[q] * cj : y[q];
}

// specx of transform f, row j, on a lane pair: lane h holds its rfftf48 result of the
// samples 2 i + h in x48; the pair meets in LDS (E = half 0, O = half 1, rows
// [48 h, 48 h + 48) of S, column f) for radf2(48, 1) (spe_subfft_fftpack2.f90:741-789)
// of the outputs m <= 30 (lane 0: m <= 15, lane 1: 16..30), scale 1/ix, into the
// m-major forward coefficients vfm[m][f][j][p].  The whole block calls it (barrier).
__device__ __attribute__((always_inline)) inline void row_specx_pair(const double *x48, double *S, bool act,
                                                                     double *__restrict__ vfm,
                                                                     const double *__restrict__ wa, int f, int j,
                                                                     int h) {
    if (act) {
#pragma unroll
        for (int i = 0; i < 48; ++i) S[(48 * h + i) * kRowLd + f] = x48[i];
    }
    __syncthreads();
    if (!act) return;
    auto E = [&](int i) { return S[i * kRowLd + f]; };
    auto O = [&](int i) { return S[(48 + i) * kRowLd + f]; };
    const double scale = 1. / (double)kIX;
    // lane h does m = 16 h + i, i = 0..15, with the operands of its m selected per lane
    // (the halves' different m ranges were divergent branches: each wave ran both);
    // every m's expressions are rfftf96_combine's: E(2s-1) +- tr2, ti2 +- E(2s) with
    // the sign taken as an exact negation, m = 0 and 24 special
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int m0 = i, m1 = 16 + i;  // lane h = 0 / 1
        const int s0 = m0, s1 = m1 < 24 ? m1 : 48 - m1;
        const int m = h ? m1 : m0, sv = h ? s1 : s0;
        if (m >= kMX) continue;  // (h = 1, i = 15)
        const int sa = sv > 0 ? sv : 1;  // (m = 0: operands unused)
        const double c = h ? wa[2 * (s1 > 0 ? s1 : 1) - 2] : wa[2 * (s0 > 0 ? s0 : 1) - 2];
        const double sn = h ? wa[2 * (s1 > 0 ? s1 : 1) - 1] : wa[2 * (s0 > 0 ? s0 : 1) - 1];
        const double e1 = E(2 * sa - 1), e2 = E(2 * sa), o1 = O(2 * sa - 1), o2 = O(2 * sa);
        const double tr2 = c * o1 + sn * o2;
        const double ti2 = c * o2 - sn * o1;
        const bool lo = m < 24;
        double re = lo ? e1 + tr2 : e1 - tr2;
        double im = lo ? e2 + ti2 : ti2 - e2;
        if (m == 0) {  // ch(1, 1) = cc(1, 1) + cc(1, 2); varm(2) = 0
            re = E(0) + O(0);
            im = 0.0;
        } else if (m == 24) {  // ido even: ch(ido, 1) = cc(ido, 1), ch(1, 2) = -cc(ido, 2)
            re = E(47);
            im = -O(47);
        }
        store2(vfm, (size_t)j * kVLs + f * 2 + (size_t)m * kVFm, re * scale, im * scale);
    }
}

// one latitude row without GPU physics: gridx of the 50 inverse transforms, grid-
// point dynamics of the row's 96 columns (+ a host's physics tendencies Pext
// [u|v|t|q][kx][ngp] if given) into LDS, specx straight to the m-major coefficients.
__global__ __launch_bounds__(kRowThreads) void k_st_rows(const double *__restrict__ varm, double *__restrict__ vfm,
                                                         const double *__restrict__ wa,
                                                         const double *__restrict__ cosgr,
                                                         const DynTables *__restrict__ T,
                                                         const double *__restrict__ Pext, long long *dbg) {
    __shared__ double A[kFftN * kRowLd], B[kFftN * kRowLd], was[kFftWa];
    constexpr int n1 = kNInv1, nin = kNInv;
    const int j = blockIdx.x, tid = threadIdx.x;
    if (tid < kFftWa) was[tid] = wa[tid];
    __syncthreads();
    const double cj = cosgr[j];
    stamp(dbg, 0, 0);
    stamp(dbg, 0, 1);
    // gridx: one field per thread
    if (tid < nin) row_gridx(A, varm, was, tid, j, tid >= n1, cj);
    __syncthreads();
    stamp(dbg, 0, 2);
    // one thread per grid column: grid-point dynamics, the forward-transform inputs into B
    if (tid < kIX) {
        const int i = tid, pt = j * kIX + i;
        auto g = [&](int f) { return A[i * kRowLd + f]; };
        double pu[kKX], pv[kKX], ptt[kKX], pq[kKX];
        if (Pext) {
#pragma unroll
            for (int k = 0; k < kKX; ++k) {
                pu[k] = Pext[(size_t)k * kGF + pt];
                pv[k] = Pext[(size_t)(kKX + k) * kGF + pt];
                ptt[k] = Pext[(size_t)(2 * kKX + k) * kGF + pt];
                pq[k] = Pext[(size_t)(3 * kKX + k) * kGF + pt];
            }
        }
        gridpoint_column(j, n1, g, Pext != nullptr, pu, pv, ptt, pq, [&](int f, double v) { B[i * kRowLd + f] = v; },
                         T);
    }
    __syncthreads();
    stamp(dbg, 0, 3);
    // specx: vdspec's x cosgr(j) on its inputs (spe_spectral.f90:430-445), rfftf
    if (tid < kNFwd) {
        double x[kFftN];
#pragma unroll
        for (int e = 0; e < kFftN; ++e) x[e] = tid < kNFwdScaled ? B[e * kRowLd + tid] * cj : B[e * kRowLd + tid];
        row_specx(x, vfm, was, tid, j);
    }
    __syncthreads();
    stamp(dbg, 0, 4);
}

// With GPU physics, one latitude row per block: the row kernel.  8 waves, two per SIMD.
// gridx of the row's 91 inverse transforms (the 50 level-j2 dynamics fields and
// phypar's 41 level-1 fields) on lane pairs; then waves 0-1 run the grid-point dynamics
// and products (one column per thread, F -> B), waves 2-3 phypar's moist part and
// vdifsc (one column per lane, its results handed over in B's spare columns), waves 4-6
// the longwave / surface chain -- on a shortwave step after its own moist part and the
// shortwave -- on two lanes per column (sml_physics_pair.hpp), which then sum the
// tendencies into F (phys_column's sums, four levels per lane); then specx of the 73
// forward transforms (F + P where grtend adds it, x cosgr(j) for vdspec's inputs) on
// lane pairs straight into the m-major coefficients.  Every expression and sum order is
// phys_column's (the one-lane-per-column form it replaced bit for bit, r05).
constexpr int kGpThreads = 512;
__global__ __launch_bounds__(kGpThreads) void k_st_gridspec_p(
    const double *__restrict__ varm, double *__restrict__ vfm, const double *__restrict__ wa,
    const double *__restrict__ cosgr, const DynTables *__restrict__ T, const double *__restrict__ bc,
    double *__restrict__ rad, const PhysTables *__restrict__ PT, int lradsw, const uint64_t *__restrict__ go_src,
    uint64_t *__restrict__ go_dst, long long *dbg) {
    SML_TL_SCOPE(sml::tl::kRow);
    // the window's first row kernel in a graph that holds the entry: the entry's outputs
    // (the safety check's inputs) were released by k_io_entry's end, so the check may go
    // (a relaxed agent-scope vector store, as k_hop_signal)
    if (go_dst && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(go_dst, *go_src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __shared__ double A[kFftN * kRowLd], B[kFftN * kRowLd];
    const double *was = kFftWa96;
    (void)wa;
    constexpr int kPtS = (int)(offsetof(PhysTables, fband) / sizeof(double)), kGpS = (int)(sizeof(GpTab) / 8);
    static_assert(kPtS + kGpS <= kGpThreads, "table staging: one value per thread");
    static_assert(kRowLd - kNFwd >= 24, "moist-side hand-over: 24 spare slots per column in B");
    __shared__ double ptl[kPtS];
    __shared__ GpTab gpt;
    __shared__ double fsr[4 * kIX];  // radlw(1)'s surface row per (column, band), sfc_fband
    constexpr int kMh = 3 + kKX;
    __shared__ double mhs[kIX * kMh];  // a shortwave step's moist-part hand-over (precnv, precls, itop, rh)
    constexpr int n1 = kNInv1P;
    constexpr int nphys = (n1 - kPT1) + (kNInvP - (n1 + 2 * kKX + 2));  // 25 + 16 = 41
    const int j = blockIdx.x, tid = threadIdx.x;
    const bool isp = tid >= 256 && tid < 256 + 2 * kIX;  // the longwave side's pairs
    const int pi = isp ? (tid - 256) >> 1 : 0, ph_ = tid & 1, ppt = j * kIX + pi;
    // a longwave-only step's radiation state of the pair lane (bands 2h, 2h + 1, its levels)
    auto pair_pre_load = [&](PairPre &pre) {
        if (lradsw) return;
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int k = 0; k < kKX; ++k)
                pre.tau[b][k] = rad[kRadTau2 + ((size_t)(2 * ph_ + b) * kKX + k) * kNGP + ppt];
        pre.strat0 = rad[kRadStratc + ppt];
        pre.strat1 = rad[kRadStratc + kNGP + ppt];
        pre.ssrd = rad[kRadSsrd + ppt];
#pragma unroll
        for (int s = 0; s < 4; ++s) pre.ttrsw[s] = rad[kRadTtRsw + (size_t)(4 * ph_ + s) * kNGP + ppt];
    };
    stamp(dbg, 0, 0);
    double rtab = 0.0;
    if (tid < kPtS) {
        rtab = reinterpret_cast<const double *>(PT)[tid];
    } else if (tid < kPtS + kGpS) {
        const int e = tid - kPtS, k = e % kKX;
        const int w = e / kKX;
        rtab = w == 0 ? T->dhs[k] : w == 1 ? T->dhsr[k] : w == 2 ? T->fsgr[k] : w == 3 ? T->tref[k]
             : w == 4 ? T->tref3[k] : T->coriol[e - 5 * kKX];
    }
    {
        const int t = tid >> 1, h = tid & 1;
        const bool act = t < kNInv + nphys;
        const int f = t < kNInv ? (t < kNInv1 ? t : n1 + (t - kNInv1))
                                : (t - kNInv < n1 - kPT1 ? kPT1 + (t - kNInv)
                                                         : n1 + 2 * kKX + 2 + (t - kNInv - (n1 - kPT1)));
        double xi[kMX2 - 1];
        if (act) row_gridx_load(varm, f, j, xi);
        if (tid < kPtS) ptl[tid] = rtab;
        else if (tid < kPtS + kGpS) reinterpret_cast<double *>(&gpt)[tid - kPtS] = rtab;
        __syncthreads();
        if (act) row_gridx_half(A, xi, was, f, false, 1.0, h);
        // the surface rows (two dependent loads), by the lanes gridx leaves idle
        for (int e = tid - 192; e >= 0 && e < 4 * kIX; e += kGpThreads - 192)
            fsr[e] = sfc_fband(bc, &PT->fband[0][0], j * kIX + (e >> 2), e & 3);
    }
    __syncthreads();
    stamp(dbg, 0, 1);
    const PhysTables *PTl = reinterpret_cast<const PhysTables *>(ptl);  // (fband stays in PT)
    const double cj = cosgr[j];
    PairOut po;
    SML_PST_T(8, 0);
    SML_PST_T(10, 128);
    SML_PST_T(14, 256);
    if (tid < kIX) {  // grid-point dynamics of column i -> F in B[i][f], then its products
        const int i = tid;
        auto g = [&](int f) { return f >= n1 ? A[i * kRowLd + f] * cj : A[i * kRowLd + f]; };
        double dummy[kKX];
        gridpoint_column(j, n1, g, false, dummy, dummy, dummy, dummy, [&](int f, double v) { B[i * kRowLd + f] = v; },
                         &gpt, false);
        // (the products below kNFwdScaled are vdspec inputs: x cosgr(j) here, not in specx)
        gridpoint_products(n1, g, [&](int f, double v) { B[i * kRowLd + f] = f < kNFwdScaled ? v * cj : v; }, &gpt);
        SML_PST_T(9, 0);
    }
    // the moist / diffusion part of column i's phypar (waves 2-3); on a shortwave step its
    // moist part's results go to the longwave side through mhs at a block barrier
    const bool ism = tid >= 128 && tid < 128 + kIX;
    const int mi = ism ? tid - 128 : 0;
    PhysThermo mth;
    double mtt[kKX], mqt[kKX], mph[kKX];
    int micnv = 0;
    if (ism) {
        const double *Ai = A + mi * kRowLd;
        double ta[kKX], qa[kKX];
#pragma unroll
        for (int k = 0; k < kKX; ++k) {
            ta[k] = Ai[kPT1 + k];
            qa[k] = Ai[kPQ1 + k];
            mph[k] = Ai[kPPhi1 + k];
        }
        phys_thermo(ta, qa, mph, Ai[kPPs1], PTl, mth);
        SML_PST_T(11, 128);
        double precnv, precls;
        int itop;
        phys_moist(mth, PTl, mtt, mqt, precnv, precls, itop, micnv);
        SML_PST_T(12, 128);
        if (lradsw) {
            double *m = mhs + mi * kMh;
            m[0] = precnv;
            m[1] = precls;
            m[2] = (double)itop;
#pragma unroll
            for (int k = 0; k < kKX; ++k) m[3 + k] = mth.rh[k];
        }
    }
    if (lradsw) __syncthreads();
    if (ism) {
        double ttv[kKX], qtv[kKX];
        phys_vdif(mth, mph, micnv, PTl, ttv, qtv);
        double *Bh = B + mi * kRowLd + kNFwd;
        // tt[0] is +0 always (convection and condensation leave the top level alone)
#pragma unroll
        for (int k = 1; k < kKX; ++k) Bh[k - 1] = mtt[k];
#pragma unroll
        for (int k = 0; k < kKX; ++k) Bh[7 + k] = ttv[k];
#pragma unroll
        for (int k = 0; k < kKX - 1; ++k) Bh[15 + k] = mqt[k] + qtv[k];  // final above the surface layer
        Bh[22] = mqt[kKX - 1];
        Bh[23] = qtv[kKX - 1];
        SML_PST_T(13, 128);
    } else if (isp) {  // the longwave / surface chain (and the shortwave) of column pi, two lanes
        PairPre pre;
        pair_pre_load(pre);  // (before gridx instead: the gridx lanes' registers spilled, gridx 3.3 -> 3.9 us)
        const double *Ai = A + pi * kRowLd;
        const double u7 = Ai[n1 + 2 * kKX + 2 + kKX - 1] * cj, v7 = Ai[n1 + 3 * kKX + 2 + kKX - 1] * cj;
        const double fs2[2] = {fsr[4 * pi + 2 * ph_], fsr[4 * pi + 2 * ph_ + 1]};
        phys_pair<kPT1, kPQ1, kPPhi1, kPPs1>(ph_, ppt, j, Ai, u7, v7, pre, bc, rad, PTl, &PT->fband[0][0], fs2,
                                             mhs + pi * kMh, lradsw != 0, po);
        SML_PST_T(18, 256);
        SML_PST_T(19, 384);
    }
    __syncthreads();
    SML_PST_T(20, 256);
    if (isp) {  // phys_column's sums (phy_phypar.f90:174-196), the pair lane's four levels
        const double *Bh = B + pi * kRowLd + kNFwd;
        double *Bi = B + pi * kRowLd;
        const double rps = po.rps;
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = 4 * ph_ + s;
            const double ttk = (k == 0 ? 0.0 : Bh[k > 0 ? k - 1 : 0]) + po.rsw[s] + po.rlw[s];
            double ttv = Bh[7 + k], utv = 0., vtv = 0.;
            double qtk;
            if (k == kKX - 1) {
                utv = utv + po.ust * rps * PTl->grdsig[kKX - 1];
                vtv = vtv + po.vst * rps * PTl->grdsig[kKX - 1];
                ttv = ttv + po.shf * rps * PTl->grdscp[kKX - 1];
                const double qtv = Bh[23] + po.evp * rps * PTl->grdsig[kKX - 1];
                qtk = Bh[22] + qtv;
            } else {
                qtk = Bh[15 + k];
            }
            // F + P where grtend adds phypar's tendencies (u 0..7, v 24..31, t 56..63, q 64..71)
            Bi[k] = (Bi[k] + (0. + utv)) * cj;  // (x cosgr(j): a vdspec input, scaled here for specx)
            Bi[3 * kKX + k] = (Bi[3 * kKX + k] + (0. + vtv)) * cj;
            Bi[7 * kKX + k] = Bi[7 * kKX + k] + (ttk + ttv);
            Bi[8 * kKX + k] = Bi[8 * kKX + k] + qtk;
        }
    }
    __syncthreads();
    stamp(dbg, 0, 2);
    // specx: transform f on lanes 2 f, 2 f + 1, lane h on the samples 2 i + h
    {
        const int f = tid >> 1, h = tid & 1;
        const bool act = f < kNFwd;
        double x[48];
        if (act) {
            const double *fr = B + f + h * kRowLd;
#pragma unroll
            for (int i = 0; i < 48; ++i) x[i] = fr[2 * i * kRowLd];
            fft::rfftf48_reg(x, was);
        }
        __syncthreads();  // A's P columns are read: A becomes the pairs' meeting place
        row_specx_pair(x, A, act, vfm, was, f, j, h);
    }
    stamp(dbg, 0, 3);
}

// specy's MFMA B operands in lane order: lane l = 16 kk + r of k-step s takes
// pfwd[m][n][j] at n = 2 r (S) and 2 r + 1 (D), j = 4 s + kk ([m][n 32][lat 24], the
// spectral context's forward Legendre table) -> pfl[m][s][l][2]
__global__ void k_pack_pfwd(const double *__restrict__ pfwd, double *__restrict__ pfl) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= kMX * (kIY / 4) * 64) return;
    const int l = e % 64, s = (e / 64) % (kIY / 4), m = e / (64 * (kIY / 4));
    const int r = l & 15, kk = l >> 4, j = 4 * s + kk;
    const double *pm = pfwd + (size_t)m * kNX * kIY;
    pfl[2 * (size_t)e] = pm[(2 * r) * kIY + j];
    pfl[2 * (size_t)e + 1] = pm[(2 * r + 1) * kIY + j];
}

// one zonal wavenumber m: specy of the 73 forward transforms, combine and tail of
// the m's 64 real coefficients x 8 levels (one thread each) on the m's state slice
// in LDS; with next_j2 > 0 the new state feeds the next step's inverse transforms
__global__ __launch_bounds__(kSpecBlk) void k_st_spec(
    const double *__restrict__ vfm, const double *__restrict__ pfl, const double *__restrict__ wt,
    const double *__restrict__ sm, double *__restrict__ sm_out, double *__restrict__ Td, double *__restrict__ phi_out,
    const double *__restrict__ phis,
    const double *__restrict__ tcorh, const double *__restrict__ qcorh, const DynTables *__restrict__ T, int j1,
    int j4, double dt, double alph, double rob, double wil, const double *__restrict__ pinv,
    double *__restrict__ varm_next, int next_j2, int n1, int nin, const double *__restrict__ tabm,
    double *__restrict__ state_out, double *__restrict__ io_varm, long long *dbg) {
    SML_TL_SCOPE(sml::tl::kSpec);
    __shared__ double V[kVFm];            // this m's tables (TabM)
    __shared__ double S[kNInvMax * kCW];  // specy output [f][2 n + p]; then the next step's inputs
    __shared__ double sh[3][kKX][kCW];
    __shared__ double Sst[kSM];           // this m's state, updated in place
    __shared__ double Fm[3 * kCW];        // phis, tcorh, qcorh of this m
    // kSpecSplit blocks per m: each repeats the m's specy, combine and tail (on CUs that
    // would idle), and takes its share of the next step's gridy tiles; the lead block
    // (half 0) alone writes the state, phi and the stamps
    const int m = blockIdx.x % kSpecStride, half = blockIdx.x / kSpecStride;
    if (m >= kMX) return;  // (block-uniform: the grid's idle blocks)
    const bool lead = half == 0;
    if (!lead) dbg = nullptr;
    const int wave = threadIdx.x >> 6, l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
    const int sk = next_j2 > 0 ? 1 : 3;
    stamp(dbg, sk, 0);
    // a) specy (k_specy's tiling: 8 fields x Re/Im per wave), the wave's A operands
    // read from vfm [lat][f][p] (per instruction 4 latitudes x 128 contiguous bytes)
    const double *vm = vfm + (size_t)m * kVFm;
    // at most two tiles per wave (10 tiles, 8 waves): both tiles' loads are issued
    // before the first MFMA, so the second tile costs no memory round trip of its own
    constexpr int kTiles = (kNFwd + 7) / 8, kWaves = kSpecBlk / 64;
    static_assert(kTiles <= 2 * kWaves, "specy: two tiles per wave at most");
    auto tile_load = [&](int tile, double (&vn)[kIY / 4], double (&vs)[kIY / 4]) {
        const int fa = tile * 8 + (r >> 1);
        const double *vr = vm + (fa < kNFwd ? fa : 0) * 2 + (r & 1);
#pragma unroll
        for (int s = 0; s < kIY / 4; ++s) {
            const int j = 4 * s + kk;
            vn[s] = vr[(kIL - 1 - j) * kVLs];
            vs[s] = vr[j * kVLs];
        }
    };
    // SML_SPEC_VFM_FIRST: specy's Fourier operands -- the hand-off from the row kernel,
    // the loads specy waits on -- issued before the state / table loads (needed only
    // after specy), so their memory round trip starts first
    double vn0[kIY / 4], vs0[kIY / 4], vn1[kIY / 4], vs1[kIY / 4];
    const bool two = wave + kWaves < kTiles;  // wave-uniform
#if SML_SPEC_VFM_FIRST
    tile_load(wave, vn0, vs0);
    if (two) tile_load(wave + kWaves, vn1, vs1);
#endif
    constexpr int RT = (kTabMDoubles / 2 + kSpecBlk - 1) / kSpecBlk;
    // three named registers, not an array: held across specy, an array was kept in scratch
    static_assert((RT == 2 || RT == 3) && 2 * RT * kSpecBlk <= kVFm && 2 * RT * kSpecBlk - kTabMDoubles <= kTabMPad,
                  "TabM staging");
    double2 rt0, rt1, rt2 = {0.0, 0.0};
    // the m's state slice and tables: loads issued first, stored to LDS after specy
    // (which reads its Fourier coefficients straight from vfm), so their latency
    // hides behind it
    constexpr int NS = kSM / 2, RS = (NS + kSpecBlk - 1) / kSpecBlk;
    static_assert(RS == 5 && NS % kSpecBlk == 0, "state staging: five whole rows of the block");
    double2 rs0, rs1, rs2, rs3, rs4;  // named registers (an array held across specy went to scratch)
    {
        const double2 *ss = reinterpret_cast<const double2 *>(sm + (size_t)m * kSM) + threadIdx.x;
        rs0 = ss[0];
        rs1 = ss[kSpecBlk];
        rs2 = ss[2 * kSpecBlk];
        rs3 = ss[3 * kSpecBlk];
        rs4 = ss[4 * kSpecBlk];
        // this m's tables (into V's space); past the slice: the next m's table or
        // d_tabm's tail pad (unused)
        const double2 *t = reinterpret_cast<const double2 *>(tabm + (size_t)m * kTabMDoubles) + threadIdx.x;
        rt0 = t[0];
        rt1 = t[kSpecBlk];
        if constexpr (RT > 2) rt2 = t[2 * kSpecBlk];
    }
    // the m's forcing (load_forcing_m's elements, one per thread) stays in a register
    // until specy is done: stored to LDS here, its wait would have cost a memory
    // round trip before specy's loads issued
    double rf = 0.0;
    if (threadIdx.x < 3 * kCW) {
        const int which = threadIdx.x / kCW, cf = threadIdx.x % kCW;
        const double *src = which == 0 ? phis : which == 1 ? tcorh : qcorh;
        rf = src[ci(cf & 1, m, cf >> 1)];
    }
    // gridy's Legendre slice of this m (8 KB, one 16-B load per thread), staged in V
    // behind the tables: each wave then reads its MFMA operands from LDS instead of
    // every wave fetching the same 8 KB from memory in the gridy phase
    constexpr int kPinvM = kNX * 32, kVPinv = 2 * RT * kSpecBlk;
    static_assert(kPinvM == 2 * kSpecBlk && kVPinv + kPinvM <= kVFm && kVPinv % 2 == 0, "pinv slice staging in V");
    const double2 rp = reinterpret_cast<const double2 *>(pinv + (size_t)m * kPinvM)[threadIdx.x];
    // specy operands: wave w's tiles all use this m's Legendre columns of its lanes,
    // packed in lane order (k_pack_pfwd): one contiguous 1-KB load per k-step instead
    // of two loads touching 16 lines each (the prologue is bound by its loads' lines)
    const double2 *pl = reinterpret_cast<const double2 *>(pfl) + (size_t)m * (kIY / 4) * 64 + l;
    double wv[kIY / 4], bS[kIY / 4], bD[kIY / 4];
#pragma unroll
    for (int s = 0; s < kIY / 4; ++s) {
        const double2 b = pl[s * 64];
        wv[s] = wt[4 * s + kk];
        bS[s] = b.x;
        bD[s] = b.y;
    }
    if (dbg) __syncthreads();
    stamp(dbg, sk, 1);
    auto tile_mma = [&](int tile, const double (&vn)[kIY / 4], const double (&vs)[kIY / 4]) {
        const int f0 = tile * 8;
        const bool ok = f0 + (r >> 1) < kNFwd;
        d4 accS = {0, 0, 0, 0}, accD = accS;
#pragma unroll
        for (int s = 0; s < kIY / 4; ++s) {
            double aS = 0.0, aD = 0.0;
            if (ok) {
                aS = (vn[s] + vs[s]) * wv[s];
                aD = (vn[s] - vs[s]) * wv[s];
            }
            accS = MFMA64(aS, bS[s], accS);
            accD = MFMA64(aD, bD[s], accD);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = kk + 4 * q;
            const int f = f0 + (row >> 1);
            if (f >= kNFwd) continue;
            S[f * kCW + 2 * (2 * r) + (row & 1)] = accS[q];
            S[f * kCW + 2 * (2 * r + 1) + (row & 1)] = accD[q];
        }
    };
    {
#if !SML_SPEC_VFM_FIRST
        tile_load(wave, vn0, vs0);
        if (two) tile_load(wave + kWaves, vn1, vs1);
#endif
        tile_mma(wave, vn0, vs0);
        if (two) tile_mma(wave + kWaves, vn1, vs1);
    }
    TabM *tm = reinterpret_cast<TabM *>(V);
    {
        double2 *v2 = reinterpret_cast<double2 *>(V) + threadIdx.x;  // (V holds kVFm >= 2 RT kSpecBlk doubles)
        v2[0] = rt0;
        v2[kSpecBlk] = rt1;
        if constexpr (RT > 2) v2[2 * kSpecBlk] = rt2;
        double2 *s2 = reinterpret_cast<double2 *>(Sst) + threadIdx.x;
        s2[0] = rs0;
        s2[kSpecBlk] = rs1;
        s2[2 * kSpecBlk] = rs2;
        s2[3 * kSpecBlk] = rs3;
        s2[4 * kSpecBlk] = rs4;
        if (threadIdx.x < 3 * kCW) Fm[threadIdx.x] = rf;
        reinterpret_cast<double2 *>(V + kVPinv)[threadIdx.x] = rp;
    }
    __syncthreads();  // S, Sst, Fm, the tables complete
    const LTab tb{tm};
    stamp(dbg, sk, 2);
    // b) combine (k_dyn_combine) for coefficient (n, p) at level k: threads 0..511
    const bool holds = threadIdx.x < kSpecThreads;
    const int cc = threadIdx.x & (kCW - 1), k = holds ? threadIdx.x / kCW : 0;
    const int n = cc >> 1, p = cc & 1;
    const int c = ci(p, m, n);
    auto fl = [&](int f) { return [=](int pp, int nn) { return S[f * kCW + 2 * nn + pp]; }; };
    double vo = 0.0, dv = 0.0, d0 = 0.0, dq = 0.0, dummy;
    vds_gen(fl(k), fl(3 * kKX + k), tb, n, p, &vo, &dv);  // vdspec(utend, vtend)
    const double lapv = -(fl(6 * kKX + k)(p, n) * tb.el2_n(n));
    vds_gen(fl(kKX + k), fl(4 * kKX + k), tb, n, p, &dummy, &d0);      // vdspec(-u tgg, -v tgg)
    vds_gen(fl(2 * kKX + k), fl(5 * kKX + k), tb, n, p, &dummy, &dq);  // vdspec(-u trg, -v trg)
    const double psdt = (m == 0 && n == 0) ? 0.0 : fl(kNFwd - 1)(p, n);
    const double tdt0 = d0 + fl(7 * kKX + k)(p, n), trdt0 = dq + fl(8 * kKX + k)(p, n);
    if (dbg) {
        __syncthreads();
        stamp(dbg, sk, 3);
    }
    // c) sptend / implic / diffusion / time integration on the LDS state
    auto SA = [&](int var, int lev, int kk2) -> double & { return Sst[smi(var, lev, kk2, cc)]; };
    if (holds)
        tail_coef<kCW>(SA, lead ? Td : nullptr, lead && next_j2 <= 0 ? phi_out : nullptr, Fm, Fm + kCW, Fm + 2 * kCW, cc, tb, sh, cc, k, c, m, n, vo, dv - lapv, tdt0,
                       trdt0, psdt, j1, j4, dt, alph, rob, wil);
    else
        tail_coef_barriers(alph);
    __syncthreads();  // S is free, Sst complete
    stamp(dbg, sk, 4);
    if (next_j2 <= 0) {  // the run of fused steps ends: the state straight into the reference layout
        if (!lead) return;  // block-uniform
        for (int i = threadIdx.x; i < kSM; i += kSpecBlk) put_state(state_out, m, i, Sst[i]);
        if (io_varm) {  // run_model: iogrid(31)'s k_io_prep + gridy of this m (block-uniform)
            if (holds) io_prep_m(Sst, tb, k, cc, [&](int f, double v) { S[f * kCW + cc] = v; });
            __syncthreads();
            gridy_io(S, gridy_operands_slice(V + kVPinv), io_varm, m, kNIo);
        }
        return;  // block-uniform
    }
    if (lead) {  // into the other buffer: this m's second block may still be reading sm
        // (five whole rows of the block, static_assert above: the LDS reads issue together)
        const double2 *src = reinterpret_cast<const double2 *>(Sst) + threadIdx.x;
        double2 v[RS];
#pragma unroll
        for (int q = 0; q < RS; ++q) v[q] = src[q * kSpecBlk];
#pragma unroll
        for (int q = 0; q < RS; ++q)
            store2(sm_out, (size_t)m * kSM + 2 * ((size_t)q * kSpecBlk + threadIdx.x), v[q].x, v[q].y);
    }
    // d) the next step's inverse-transform inputs (k_dyn_prep) and gridy
    if (holds) inv_inputs(Sst, S, Fm, tb, m, next_j2, n1, nin);
    __syncthreads();
    stamp(dbg, sk, 5);
    {
        const int nt = (nin + 7) / 8, per = (nt + kSpecSplit - 1) / kSpecSplit;
        gridy_m(S, gridy_operands_slice(V + kVPinv), varm_next, m, nin, half * per, min(nt, (half + 1) * per));
    }
    if (dbg) {  // (diagnostics only: the kernel ends here)
        __syncthreads();
        stamp(dbg, sk, 6);
    }
}

// ------------------------------------------------------------ iogrid(30/31)
// ppo_iogrid.f90:497-601.  grid4d = variables3d(4, ix, il, kx) (T, u, v, q), logp(ix, il).
// Field-major work layout of both directions: [u 8 | v 8 | t 8 | q 8 | ps] (33 fields).


// entry: vdspec's vds + spec, trunct, into time level 1 (:524-538)
__global__ void k_io_combine(const double *__restrict__ S, double *__restrict__ st, const DynTables *__restrict__ T) {
    const int mn = blockIdx.x * blockDim.x + threadIdx.x;
    if (mn >= kMN) return;
    const int k = blockIdx.y;
    const int m = mn % kMX, n = mn / kMX;
    const double trf = T->trfilt[n][m];
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int c = ci(p, m, n);
        double vo, dv;
        vds_at(S + (size_t)k * kSF, S + (size_t)(kKX + k) * kSF, T, m, n, p, &vo, &dv);
        st[kOffVor + (size_t)k * kSF + c] = vo * trf;
        st[kOffDiv + (size_t)k * kSF + c] = dv * trf;
        st[kOffT + (size_t)k * kSF + c] = S[(size_t)(2 * kKX + k) * kSF + c] * trf;
        st[kOffTr + (size_t)k * kSF + c] = S[(size_t)(3 * kKX + k) * kSF + c] * trf;
        if (k == 0) st[kOffPs + c] = S[(size_t)(4 * kKX) * kSF + c] * trf;
    }
}

// both directions: inverse-transform inputs from level 1 (:541-553 / :576-589):
// [ucos 8 | vcos 8 | t 8 | q 8 | ps]
__global__ void k_io_prep(const double *__restrict__ st, double *__restrict__ sin_, const DynTables *__restrict__ T) {
    const int mn = blockIdx.x * blockDim.x + threadIdx.x;
    if (mn >= kMN) return;
    const int k = blockIdx.y;
    const int m = mn % kMX, n = mn / kMX;
    const double *vor = st + kOffVor + (size_t)k * kSF, *div = st + kOffDiv + (size_t)k * kSF;
    uvspec_at(vor, div, T, m, n, sin_ + (size_t)k * kSF, sin_ + (size_t)(kKX + k) * kSF);
#pragma unroll
    for (int p = 0; p < 2; ++p) {
        const int c = ci(p, m, n);
        sin_[(size_t)(2 * kKX + k) * kSF + c] = st[kOffT + (size_t)k * kSF + c];
        sin_[(size_t)(3 * kKX + k) * kSF + c] = st[kOffTr + (size_t)k * kSF + c];
        if (k == 0) sin_[(size_t)(4 * kKX) * kSF + c] = st[kOffPs + c];
    }
}

// run_model's window entry in one launch per zonal wavenumber m (512 threads = 64
// coefficients x 8 levels), after iogrid(30)'s specx: the same operations as
//   specy (k_specy's tiling)  -> k_io_combine (vds / spec + trunct into level 1)
//   -> k_io_prep (the safety check's inputs) -> k_state_to_m -> k_st_inv (the first
//   step's inverse inputs + gridy)
// which all stay inside one m.  vio: the io Fourier coefficients, kNIo fields in the
// spectral module's layout; state: reference layout, level 1 written, level 2 read
// into the m-major slice sm; chk: k_io_prep's output; varm: gridy for step(1, 1).
__global__ __launch_bounds__(kSpecThreads) void k_io_entry(const double *__restrict__ vio,
                                                           const double *__restrict__ pfl,
                                                           const double *__restrict__ wt, double *__restrict__ state,
                                                           double *__restrict__ sm, double *__restrict__ chk,
                                                           const double *__restrict__ phis,
                                                           const double *__restrict__ tabm,
                                                           const double *__restrict__ pinv, double *__restrict__ varm,
                                                           int n1, int nin, uint64_t *__restrict__ xa, uint64_t xa0,
                                                           uint64_t xa1) {
    SML_TL_SCOPE(sml::tl::kIoEntry);
    // a graph-captured exit's per-launch values (sml_dyn_run_model): ordered before the
    // window graph by this kernel's end
    if (xa && blockIdx.x == 0 && threadIdx.x == 0) {
        xa[0] = xa0;
        xa[1] = xa1;
    }
    __shared__ double S[kNIo * kCW];  // specy output [f][2 n + p]
    __shared__ double Sst[kSM];       // this m's state slice
    __shared__ double In[kNInvMax * kCW];
    __shared__ double Fm[kCW];
    constexpr int RT = (kTabMDoubles / 2 + kSpecThreads - 1) / kSpecThreads;
    __shared__ double V[2 * RT * kSpecThreads];  // this m's tables (TabM), staged as k_st_spec does
    const int m = blockIdx.x, tid = threadIdx.x;
    const int wave = tid >> 6, l = tid & 63, r = l & 15, kk = l >> 4;
    // every global load of the entry is issued before the first wait (one memory round
    // trip): level 2 of the slice (k_state_to_m), phis(m), specy's operands and
    // gridy's Legendre columns.  Element i = tid + 512 q of the slice has lev = q % 2,
    // var = q / 2, k = tid / 64, cc = tid % 64.
    constexpr int kSI = kSM / kSpecThreads;
    static_assert(kSM % kSpecThreads == 0 && kSI == 10, "slice staging: ten rows of the block");
    double s2[kSI / 2];
#pragma unroll
    for (int q = 1; q < kSI; q += 2) {  // level 2 (lev index 1); level 1 comes from the combine
        const int cc = tid % kCW, k = tid / kCW, var = q / 2;
        const int c = ci(cc & 1, m, cc >> 1);
        double v = 0.0;
        if (var < 4) {
            const size_t off = var == 0 ? kOffVor : var == 1 ? kOffDiv : var == 2 ? kOffT : kOffTr;
            v = state[off + ((size_t)kKX + k) * kSF + c];
        } else if (k == 0) {
            v = state[kOffPs + (size_t)kSF + c];
        }
        s2[q / 2] = v;
    }
    const double phis_m = tid < kCW ? phis[ci(tid & 1, m, tid >> 1)] : 0.0;
    static_assert(2 * RT * kSpecThreads - kTabMDoubles <= kTabMPad, "TabM staging");
    double2 rt[RT];
    {
        const double2 *t = reinterpret_cast<const double2 *>(tabm + (size_t)m * kTabMDoubles) + tid;
#pragma unroll
        for (int q = 0; q < RT; ++q) rt[q] = t[q * kSpecThreads];
    }
    // a) specy of the io fields (k_specy: a wave per 8 fields x Re/Im)
    const bool spw = wave < (kNIo + 7) / 8;  // wave-uniform
    const int f0 = wave * 8, fa = f0 + (r >> 1);
    const bool ok = spw && fa < kNIo;
    double vn[kIY / 4], vs[kIY / 4], wv[kIY / 4], bS[kIY / 4], bD[kIY / 4];
    if (spw) {
        const double *vr = vio + (size_t)(ok ? fa : 0) * kVarmField + 2 * m + (r & 1);
        const double2 *pl = reinterpret_cast<const double2 *>(pfl) + (size_t)m * (kIY / 4) * 64 + l;
#pragma unroll
        for (int s = 0; s < kIY / 4; ++s) {
            const int j = 4 * s + kk;
            vn[s] = vr[(kIL - 1 - j) * kMX2];
            vs[s] = vr[j * kMX2];
            wv[s] = wt[j];
            const double2 b = pl[s * 64];  // the packed B operands (k_pack_pfwd)
            bS[s] = b.x;
            bD[s] = b.y;
        }
    }
    const GridyB gb = gridy_operands(pinv, m);
    __builtin_amdgcn_sched_barrier(0);
    // (the table stores first, in the loads' own block: behind a branch the loads
    // were sunk next to them, after the first wait)
#pragma unroll
    for (int q = 0; q < RT; ++q) reinterpret_cast<double2 *>(V)[tid + q * kSpecThreads] = rt[q];
#pragma unroll
    for (int q = 1; q < kSI; q += 2) Sst[tid + kSpecThreads * q] = s2[q / 2];
    if (tid < kCW) Fm[tid] = phis_m;
    if (spw) {
        d4 accS = {0, 0, 0, 0}, accD = accS;
#pragma unroll
        for (int s = 0; s < kIY / 4; ++s) {
            double aS = 0.0, aD = 0.0;
            if (ok) {
                aS = (vn[s] + vs[s]) * wv[s];
                aD = (vn[s] - vs[s]) * wv[s];
            }
            accS = MFMA64(aS, bS[s], accS);
            accD = MFMA64(aD, bD[s], accD);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int row = kk + 4 * q;
            const int f = f0 + (row >> 1);
            if (f >= kNIo) continue;
            S[f * kCW + 2 * (2 * r) + (row & 1)] = accS[q];
            S[f * kCW + 2 * (2 * r + 1) + (row & 1)] = accD[q];
        }
    }
    __syncthreads();
    // b) k_io_combine: vdspec's vds + spec, trunct, into level 1 (ppo_iogrid.f90:524-538)
    const LTab tb{reinterpret_cast<const TabM *>(V)};
    const int cc = tid & (kCW - 1), k = tid / kCW, n = cc >> 1, p = cc & 1, c = ci(p, m, n);
    {
        auto fl = [&](int f) { return [=](int pp, int nn) { return S[f * kCW + 2 * nn + pp]; }; };
        const double trf = tb.trfilt_n(n);
        double vo, dv;
        vds_gen(fl(k), fl(kKX + k), tb, n, p, &vo, &dv);
        const double v0 = vo * trf, v1 = dv * trf, v2 = S[(2 * kKX + k) * kCW + cc] * trf,
                     v3 = S[(3 * kKX + k) * kCW + cc] * trf;
        Sst[smi(0, 1, k, cc)] = v0;
        Sst[smi(1, 1, k, cc)] = v1;
        Sst[smi(2, 1, k, cc)] = v2;
        Sst[smi(3, 1, k, cc)] = v3;
        state[kOffVor + (size_t)k * kSF + c] = v0;
        state[kOffDiv + (size_t)k * kSF + c] = v1;
        state[kOffT + (size_t)k * kSF + c] = v2;
        state[kOffTr + (size_t)k * kSF + c] = v3;
        if (k == 0) {
            const double v4 = S[(4 * kKX) * kCW + cc] * trf;
            Sst[smi(4, 1, 0, cc)] = v4;
            state[kOffPs + c] = v4;
        } else {
            Sst[smi(4, 1, k, cc)] = 0.0;  // ps lives at k = 0 only (k_state_to_m)
        }
    }
    __syncthreads();
    // c) k_io_prep: uvspec of level 1 and copies -> the safety check's inputs
    {
        double a, b;
        uvspec_sel(Sst, tb, 1, k, n, p, &a, &b);
        chk[(size_t)k * kSF + c] = a;
        chk[(size_t)(kKX + k) * kSF + c] = b;
        chk[(size_t)(2 * kKX + k) * kSF + c] = Sst[smi(2, 1, k, cc)];
        chk[(size_t)(3 * kKX + k) * kSF + c] = Sst[smi(3, 1, k, cc)];
        if (k == 0) chk[(size_t)(4 * kKX) * kSF + c] = Sst[smi(4, 1, 0, cc)];
    }
    // d) the m-major slice for the window's first k_st_spec (k_state_to_m; whole rows
    // of the block, the LDS reads issued together)
    {
        static_assert(kSM / 2 % kSpecThreads == 0, "slice rows");
        constexpr int R = kSM / 2 / kSpecThreads;
        double2 *dst = reinterpret_cast<double2 *>(sm + (size_t)m * kSM) + tid;
        const double2 *src = reinterpret_cast<const double2 *>(Sst) + tid;
        double2 v[R];
#pragma unroll
        for (int q = 0; q < R; ++q) v[q] = src[q * kSpecThreads];
#pragma unroll
        for (int q = 0; q < R; ++q) dst[q * kSpecThreads] = v[q];
    }
    // e) k_st_inv: step(1, 1)'s inverse inputs (j2 = 1) and gridy
    inv_inputs(Sst, In, Fm, tb, m, 1, n1, nin);
    __syncthreads();
    gridy_m(In, gb, varm, m, nin);
}

// entry safety check (:556-571): min / max of the re-gridded u, v, t, q.  One
// block of 1024 threads per variable.
// NaN-sticky min / max (fmin / fmax would drop a NaN; a blown-up state must not
// pass the check, io_state_safe)
__device__ inline double nmin(double a, double b) { return (a != a || b != b) ? __builtin_nan("") : (b < a ? b : a); }
__device__ inline double nmax(double a, double b) { return (a != a || b != b) ? __builtin_nan("") : (b > a ? b : a); }

// cnt (may be null): the hand-off counter the run_model exit polls -- each block stores
// its min / max sc1, drains its stores and adds 1 (MI355X_MICROARCH.md, inter-workgroup
// visibility: an agent-scope atomic add per storing workgroup, sc1 stores and loads)
// the hybrid loop's forecast hop behind run_model's exit: one relaxed agent-scope
// vector store of the hop's sequence number, xa[1] (the exit's stores were released by
// its kernel's end; as sml_hybrid's k_hop_signal)
__global__ void k_flag_store_value(uint64_t *flag, uint64_t v) {
    SML_TL_SCOPE(sml::tl::kExitStore);
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// a graph-captured run_model's per-launch values (WindowReplay, sml_dynamics::d_xa),
// launched right before the graph on its stream: behind the previous window, off the
// chain (the graph's entry waits for its grid anyway)
__global__ void k_set_xa(uint64_t *xa, uint64_t v0, uint64_t v1, uint64_t v2, uint64_t v3) {
    if (threadIdx.x == 0) {
        xa[0] = v0;
        xa[1] = v1;
        xa[2] = v2;
        xa[3] = v3;
    }
}

// the safety check's go on its own stream when the entry is inside the window graph:
// one lane polls *go (stored by the window's first row kernel) and acquires at agent
// scope; the check's kernels follow on the stream.  Never spins forever: on a timeout it
// marks *late with late_value (the exit's target for this check, so sml_dyn_last_safe
// fails this window) and the check reads whatever d_chk holds
__global__ void k_check_go(const uint64_t *go, uint64_t want, unsigned *late, unsigned late_value, long long timeout) {
    if (threadIdx.x != 0) return;
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < want) {
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > timeout) {
            __hip_atomic_store(late, late_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

__global__ void k_flag_store(uint64_t *flag, const uint64_t *xa) {
    SML_TL_SCOPE(sml::tl::kExitStore);
    if (threadIdx.x == 0) __hip_atomic_store(flag, xa[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// late / self: a check whose go hand-off gave up (k_check_go stored self into *late)
// reports NaN, so the exit takes the window as unsafe instead of trusting inputs the
// entry may not have written yet
__global__ __launch_bounds__(1024) void k_io_minmax(const double *__restrict__ G, double *__restrict__ mm,
                                                     unsigned *__restrict__ cnt, const unsigned *__restrict__ late,
                                                     unsigned self) {
    SML_TL_SCOPE(sml::tl::kCheckMinmax);
    __shared__ double smin[16], smax[16];
    const int v = blockIdx.x;
    const double *f = G + (size_t)v * kKX * kGF;
    double lo = f[threadIdx.x], hi = lo;
    for (int i = threadIdx.x; i < kKX * kGF; i += blockDim.x) {
        lo = nmin(lo, f[i]);
        hi = nmax(hi, f[i]);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = nmin(lo, __shfl_xor(lo, o));
        hi = nmax(hi, __shfl_xor(hi, o));
    }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        smin[w] = lo;
        smax[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int i = 1; i < 16; ++i) {
            lo = nmin(lo, smin[i]);
            hi = nmax(hi, smax[i]);
        }
        if (late && __hip_atomic_load(late, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == self)
            lo = hi = __builtin_nan("");
        if (cnt) {
            __hip_atomic_store(mm + 2 * v, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(mm + 2 * v + 1, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            mm[2 * v] = lo;
            mm[2 * v + 1] = hi;
        }
    }
}

template <typename T>
int dalloc(T **p, size_t count) {
    *p = nullptr;
    SML_HIP(hipMalloc((void **)p, count * sizeof(T)));
    SML_HIP(hipMemset(*p, 0, count * sizeof(T)));
    return SML_OK;
}

}  // namespace

// ------------------------------------------------------------------ API
extern "C" int sml_dyn_destroy(sml_dynamics *d) {
    if (!d) return SML_OK;
    void *ptrs[] = {d->d_tabs, d->d_tabm, d->d_state, d->d_phis, d->d_tcorh, d->d_phi, d->d_specin,
                    d->d_varm, d->d_grid, d->d_gfwd, d->d_sfwd, d->d_tend, d->d_phys, d->d_minmax, d->d_io, d->d_vfm, d->d_pfl, d->d_sm, d->d_dbg,
                    d->d_ptab, d->d_pbc, d->d_rad, d->d_pio, d->d_sst_cpl, d->d_sice, d->d_tice, d->d_surf,
                    d->d_clim, d->d_ford};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    for (auto &r : d->replay)
        if (r.exec) (void)hipGraphExecDestroy(r.exec);
    for (auto &cls : d->wreplay)
        for (auto &r : cls)
            if (r.exec) (void)hipGraphExecDestroy(r.exec);
    if (d->d_xa) (void)hipFree(d->d_xa);
    if (d->d_go) (void)hipFree(d->d_go);
    if (d->cap_stream) (void)hipStreamDestroy(d->cap_stream);
    if (d->chk_stream) {
        (void)hipStreamSynchronize(d->chk_stream);
        (void)hipStreamDestroy(d->chk_stream);
    }
    if (d->ev_fork) (void)hipEventDestroy(d->ev_fork);
    if (d->ev_chk) (void)hipEventDestroy(d->ev_chk);
    if (d->ev_mm) (void)hipEventDestroy(d->ev_mm);
    if (d->h_mm) (void)hipHostFree(d->h_mm);
    if (d->d_chk) (void)hipFree(d->d_chk);
    if (d->d_chk_cnt) (void)hipFree(d->d_chk_cnt);
    if (d->d_chk_late) (void)hipHostFree(d->d_chk_late);
    if (d->sp) sml_spectral_destroy(d->sp);
    delete d;
    return SML_OK;
}

static int upload_tabm(sml_dynamics *d, int i);

extern "C" int sml_dyn_create(double radius, sml_dynamics **out) {
    SML_REQUIRE(out, "out is null");
    *out = nullptr;
    sml_dynamics *d = new (std::nothrow) sml_dynamics();
    if (!d) return fail(SML_ERR_NOMEM, "host allocation failed");
    int rc = sml_spectral_create(radius, &d->sp);
    if (rc) {
        delete d;
        return rc;
    }
    build_dyn_indyns(spectral_host_tables(d->sp), &d->tab);
    build_phys_tables(d->tab, &d->ptab);
    if (const char *e = std::getenv("SML_DYN_NOGRAPH")) d->nograph = *e && *e != '0';
    // dispatch serialised by the runtime or a profiler's counter passes: the check must
    // not wait for a kernel enqueued after it (launch_io_check's go hand-off)
    for (const char *v : {"AMD_SERIALIZE_KERNEL", "ROCPROF_COUNTER_COLLECTION"})
        if (const char *e = std::getenv(v)) d->serialized = d->serialized || (*e && std::strcmp(e, "0") != 0);
    if (const char *e = std::getenv("SML_DYN_STAMPS"))
        if (*e && *e != '0' && (rc = dalloc(reinterpret_cast<double **>(&d->d_dbg), kStampKernels * kStampBlocks * kStamps))) {
            sml_dyn_destroy(d);
            return rc;
        }
    if ((rc = dalloc(&d->d_tabs, 4)) || (rc = dalloc(&d->d_tabm, (size_t)4 * kMX * kTabMDoubles + kTabMPad)) || (rc = dalloc(&d->d_state, kStateSize)) || (rc = dalloc(&d->d_phis, kSF)) ||
        (rc = dalloc(&d->d_tcorh, 2 * kSF)) || (rc = dalloc(&d->d_phi, kKX * kSF)) ||
        (rc = dalloc(&d->d_specin, (size_t)kNInvMax * kSF)) ||
        (rc = dalloc(&d->d_varm, (size_t)(kNInvMax > kNFwd ? kNInvMax : kNFwd) * kVF)) ||
        (rc = dalloc(&d->d_grid, (size_t)kNInvMax * kGF)) || (rc = dalloc(&d->d_gfwd, (size_t)kNFwd * kGF)) ||
        (rc = dalloc(&d->d_sfwd, (size_t)kNFwd * kSF)) || (rc = dalloc(&d->d_tend, kTendSize)) ||
        (rc = dalloc(&d->d_vfm, (size_t)kMX * kVFm)) || (rc = dalloc(&d->d_sm, (size_t)2 * kMX * kSM)) ||
        (rc = dalloc(&d->d_pfl, (size_t)kMX * (kIY / 4) * 64 * 2)) ||
        (rc = dalloc(&d->d_phys, (size_t)4 * kKX * kGF)) || (rc = dalloc(&d->d_minmax, 8)) ||
        (rc = dalloc(&d->d_chk_cnt, 2)) ||
        (rc = dalloc(&d->d_io, (size_t)4 * kKX * kGF + kGF)) || (rc = dalloc(&d->d_ptab, 1)) ||
        (rc = dalloc(&d->d_chk, (size_t)kNIo * (kSF + kVF + kGF))) ||
        (rc = dalloc(&d->d_pbc, (size_t)kNBc * kNGP)) || (rc = dalloc(&d->d_rad, kRadSize)) ||
        (rc = dalloc(&d->d_pio, (size_t)(5 * kKX + 1 + 4 * kKX) * kNGP)) || (rc = dalloc(&d->d_sst_cpl, kNGP)) ||
        (rc = dalloc(&d->d_sice, kNGP)) || (rc = dalloc(&d->d_tice, kNGP)) ||
        (rc = dalloc(&d->d_surf, (size_t)3 * kNGP)) || (rc = dalloc(&d->d_ford, (size_t)2 * (kGF + kVF)))) {
        sml_dyn_destroy(d);
        return rc;
    }
    d->d_qcorh = d->d_tcorh + kSF;  // one allocation: fordate's spec writes both fields
    if (hipHostMalloc((void **)&d->d_chk_late, sizeof(unsigned), hipHostMallocCoherent) != hipSuccess) {
        d->d_chk_late = nullptr;
        sml_dyn_destroy(d);
        return fail(SML_ERR_NOMEM, "sml_dyn_create: pinned late word");
    }
    *d->d_chk_late = 0;
    d->d_tab = d->d_tabs;
    hipError_t e = hipMemcpy(d->d_tab, &d->tab, sizeof(DynTables), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(d->d_ptab, &d->ptab, sizeof(PhysTables), hipMemcpyHostToDevice);
    if (e == hipSuccess) {  // specy's packed B operands from the spectral context's forward Legendre table
        const int n = kMX * (kIY / 4) * 64;
        hipLaunchKernelGGL(k_pack_pfwd, dim3((n + 255) / 256), dim3(256), 0, 0, spectral_dev(d->sp).pfwd, d->d_pfl);
        e = hipGetLastError();
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    if (e != hipSuccess) {
        sml_dyn_destroy(d);
        return fail(SML_ERR_HIP, "sml_dyn_create: %s", hipGetErrorString(e));
    }
    // slot 0's per-m copy too: run_model's entry (k_io_entry) reads the current slot's
    // TabM, before any impint when it is the first call
    if (int rc = upload_tabm(d, 0)) {
        sml_dyn_destroy(d);
        return rc;
    }
    *out = d;
    return SML_OK;
}

// the per-m TabM copies of d->tab into slot i of d_tabm
static int upload_tabm(sml_dynamics *d, int i) {
    std::vector<double> tm((size_t)kMX * kTabMDoubles);
    for (int m = 0; m < kMX; ++m)
        for (int q = 0; q < kTabMDoubles; ++q) tm[(size_t)m * kTabMDoubles + q] = tabm_value(&d->tab, m, q);
    SML_HIP(hipMemcpy(d->d_tabm + (size_t)i * kMX * kTabMDoubles, tm.data(), tm.size() * 8, hipMemcpyHostToDevice));
    return SML_OK;
}

extern "C" int sml_dyn_impint(sml_dynamics *d, double dt, double alph) {
    SML_REQUIRE(d, "null context");
    for (int i = 0; i < 4; ++i)
        if (d->slot_used[i] && d->slot_key[i][0] == dt && d->slot_key[i][1] == alph) {
            d->d_tab = d->d_tabs + i;  // cached: no host work, no copy
            d->impint_done = true;
            return SML_OK;
        }
    const int i = d->slot_next;
    d->slot_next = (i + 1) % 4;
    build_dyn_impint(dt, alph, &d->tab);
    // the copy is ordered before later launches on the legacy stream; kernels still
    // reading an evicted slot were launched earlier and complete first
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(d->d_tabs + i, &d->tab, sizeof(DynTables), hipMemcpyHostToDevice));
    if (int rc = upload_tabm(d, i)) return rc;
    d->slot_key[i][0] = dt;
    d->slot_key[i][1] = alph;
    d->slot_used[i] = true;
    d->d_tab = d->d_tabs + i;
    d->impint_done = true;
    return SML_OK;
}

extern "C" int sml_dyn_set_forcing(sml_dynamics *d, const double *phis, const double *tcorh, const double *qcorh) {
    SML_REQUIRE(d, "null context");
    if (phis) SML_HIP(hipMemcpy(d->d_phis, phis, kSF * 8, hipMemcpyHostToDevice));
    if (tcorh) SML_HIP(hipMemcpy(d->d_tcorh, tcorh, kSF * 8, hipMemcpyHostToDevice));
    if (qcorh) SML_HIP(hipMemcpy(d->d_qcorh, qcorh, kSF * 8, hipMemcpyHostToDevice));
    ++d->ford_gen;  // a later sml_dyn_fordate recomputes what the host has just replaced
    return SML_OK;
}

extern "C" int sml_dyn_get_forcing(sml_dynamics *d, double *phis, double *tcorh, double *qcorh) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    if (phis) SML_HIP(hipMemcpy(phis, d->d_phis, kSF * 8, hipMemcpyDeviceToHost));
    if (tcorh) SML_HIP(hipMemcpy(tcorh, d->d_tcorh, kSF * 8, hipMemcpyDeviceToHost));
    if (qcorh) SML_HIP(hipMemcpy(qcorh, d->d_qcorh, kSF * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_set_state(sml_dynamics *d, const double *vor, const double *div, const double *t,
                                 const double *ps, const double *tr) {
    SML_REQUIRE(d && vor && div && t && ps && tr, "null argument");
    const size_t f3 = 2 * kKX * kSF * 8;
    SML_HIP(hipMemcpy(d->d_state + kOffVor, vor, f3, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_state + kOffDiv, div, f3, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_state + kOffT, t, f3, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_state + kOffTr, tr, f3, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_state + kOffPs, ps, 2 * kSF * 8, hipMemcpyHostToDevice));
    return SML_OK;
}

extern "C" int sml_dyn_get_state(sml_dynamics *d, double *vor, double *div, double *t, double *ps, double *tr) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    const size_t f3 = 2 * kKX * kSF * 8;
    if (vor) SML_HIP(hipMemcpy(vor, d->d_state + kOffVor, f3, hipMemcpyDeviceToHost));
    if (div) SML_HIP(hipMemcpy(div, d->d_state + kOffDiv, f3, hipMemcpyDeviceToHost));
    if (t) SML_HIP(hipMemcpy(t, d->d_state + kOffT, f3, hipMemcpyDeviceToHost));
    if (tr) SML_HIP(hipMemcpy(tr, d->d_state + kOffTr, f3, hipMemcpyDeviceToHost));
    if (ps) SML_HIP(hipMemcpy(ps, d->d_state + kOffPs, 2 * kSF * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_get_phi(sml_dynamics *d, double *phi) {
    SML_REQUIRE(d && phi, "null argument");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(phi, d->d_phi, kKX * kSF * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_get_tendencies(sml_dynamics *d, double *tend) {
    SML_REQUIRE(d && tend, "null argument");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(tend, d->d_tend, kTendSize * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_state_device(sml_dynamics *d, double **d_state, double **d_phys) {
    SML_REQUIRE(d, "null context");
    if (d_state) *d_state = d->d_state;
    if (d_phys) *d_phys = d->d_phys;
    return SML_OK;
}

namespace {

// the unfused launches of one step(j1, j2, dt, alph, rob, wil) on stream st: 7
// without GPU physics, 8 with it
int launch_step_unfused(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                        const double *d_phys, bool lradsw, hipStream_t st) {
    const DynTables *T = d->d_tab;
    const bool phys = d->phys_on;
    const int n1 = phys ? kNInv1P : kNInv1, nin = phys ? kNInvP : kNInv;
    // 1. grtend: inverse transforms of the j2 state (+ phypar's level-1 inputs)
    hipLaunchKernelGGL(k_dyn_prep, dim3((kMN + 127) / 128, kKX + 1), dim3(128), 0, st, d->d_state, d->d_specin, T,
                       d->d_phis, j2, n1, phys ? 1 : 0);
    SML_HIP(hipGetLastError());
    if (int rc = spectral_gridy(d->sp, d->d_specin, d->d_varm, nin, st)) return rc;
    if (int rc = spectral_gridx_split(d->sp, d->d_varm, d->d_grid, nin, n1, st)) return rc;
    // 2. physics (phypar on level 1), then grid-point dynamics + physics tendencies
    if (phys) {
        const double *G = d->d_grid;
        hipLaunchKernelGGL(k_phys, dim3(kNGP / 64), dim3(64), 0, st, G + (size_t)(n1 + 2 * kKX + 2) * kGF,
                           G + (size_t)(n1 + 3 * kKX + 2) * kGF, G + (size_t)kPT1 * kGF, G + (size_t)kPQ1 * kGF,
                           G + (size_t)kPPhi1 * kGF, G + (size_t)kPPs1 * kGF, d->d_pbc, d->d_rad, d->d_ptab,
                           lradsw ? 1 : 0, d->d_phys);
        SML_HIP(hipGetLastError());
        d_phys = d->d_phys;
    }
    hipLaunchKernelGGL(k_dyn_gridpoint, dim3((kGF + 255) / 256), dim3(256), 0, st, d->d_grid, d_phys, d->d_gfwd, T,
                       n1);
    SML_HIP(hipGetLastError());
    // 3. forward transforms: vdspec inputs x 1/cos (kcos = 2), the rest plain
    if (int rc = spectral_specx_split(d->sp, d->d_gfwd, d->d_varm, kNFwd, kNFwdScaled, st)) return rc;
    if (int rc = spectral_specy(d->sp, d->d_varm, d->d_sfwd, kNFwd, st)) return rc;
    hipLaunchKernelGGL(k_dyn_combine, dim3((kMN + 127) / 128, kKX), dim3(128), 0, st, d->d_sfwd, d->d_tend, T);
    SML_HIP(hipGetLastError());
    // 4. sptend / implic / diffusion / time integration
    const int j4 = (alph == 0.0) ? j2 : 1;
    hipLaunchKernelGGL(k_dyn_tail, dim3(kSF / kTailC), dim3(kTailC * kKX), 0, st, d->d_state, d->d_tend, d->d_phi,
                       d->d_phis, d->d_tcorh, d->d_qcorh, T, j1, j4, dt, alph, rob, wil);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

// the fused step: [k_state_to_m k_st_inv] (k_st_rows | k_st_gridspec) k_st_spec.
// chained: the previous launch_step's k_st_spec left the m-major state and this
// step's gridy output (its next_j2 was this j2); next_j2 > 0: this step's k_st_spec
// prepares step (.., next_j2) and the state stays m-major, else it writes the
// reference-layout state.

// buffer b of the m-major state (two, so k_st_spec's second block of an m never
// reads a slice its lead block already advanced)
double *sm_buf(sml_dynamics *d, int b) { return d->d_sm + (size_t)b * kMX * kSM; }

int launch_step_fused(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                      const double *d_phys, bool lradsw, hipStream_t st, bool chained, int next_j2) {
    const DynTables *T = d->d_tab;
    const bool phys = d->phys_on;
    const int n1 = phys ? kNInv1P : kNInv1, nin = phys ? kNInvP : kNInv;
    const SpectralDev sd = spectral_dev(d->sp);
    if (dt <= 0.0) next_j2 = 0;  // tendencies only: the state does not advance
    const int conv_blocks = (kMX * kSM + 255) / 256;
    if (!chained) {  // a chain starts in buffer 0 (so a captured window replays the same pointers)
        d->sm_cur = 0;
        hipLaunchKernelGGL(k_state_to_m, dim3(conv_blocks), dim3(256), 0, st, d->d_state, sm_buf(d, 0));
        SML_HIP(hipGetLastError());
        hipLaunchKernelGGL(k_st_inv, dim3(kMX), dim3(kSpecThreads), 0, st, sm_buf(d, 0), d->d_phis, T, sd.pinv,
                           d->d_varm, j2, n1, nin);
        SML_HIP(hipGetLastError());
    }
    if (phys) {
        hipLaunchKernelGGL(k_st_gridspec_p, dim3(kIL), dim3(kGpThreads), 0, st, d->d_varm, d->d_vfm, sd.wa, sd.cosgr, T,
                           d->d_pbc, d->d_rad, d->d_ptab, lradsw ? 1 : 0, d->go_src_next, d->go_dst_next, d->d_dbg);
        d->go_src_next = nullptr;  // one launch
        d->go_dst_next = nullptr;
        SML_HIP(hipGetLastError());
    } else {
        hipLaunchKernelGGL(k_st_rows, dim3(kIL), dim3(kRowThreads), 0, st, d->d_varm, d->d_vfm, sd.wa, sd.cosgr, T,
                           d_phys, d->d_dbg);
        SML_HIP(hipGetLastError());
    }
    const int j4 = (alph == 0.0) ? j2 : 1;
    const int cur = d->sm_cur;
    if (next_j2 > 0) d->sm_cur = 1 - cur;  // the next step reads what this one writes
    hipLaunchKernelGGL(k_st_spec, dim3(kSpecStride * kSpecSplit), dim3(kSpecBlk), 0, st, d->d_vfm, d->d_pfl, sd.wt,
                       sm_buf(d, cur), sm_buf(d, 1 - cur), d->d_tend,
                       d->d_phi, d->d_phis, d->d_tcorh, d->d_qcorh, T, j1, j4, dt, alph, rob, wil, sd.pinv, d->d_varm,
                       next_j2, n1, nin, d->d_tabm + (size_t)(d->d_tab - d->d_tabs) * kMX * kTabMDoubles, d->d_state,
                       next_j2 > 0 ? nullptr : d->io_exit, d->d_dbg);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int launch_step(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil, const double *d_phys,
                bool lradsw, hipStream_t st, bool chained = false, int next_j2 = 0) {
    return d->fused ? launch_step_fused(d, j1, j2, dt, alph, rob, wil, d_phys, lradsw, st, chained, next_j2)
                    : launch_step_unfused(d, j1, j2, dt, alph, rob, wil, d_phys, lradsw, st);
}

}  // namespace

extern "C" int sml_dyn_step(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                            const double *d_phys, void *stream) {
    SML_REQUIRE(d, "null context");
    SML_REQUIRE((j1 == 1 || j1 == 2) && (j2 == 1 || j2 == 2), "j1/j2 must be 1 or 2");
    SML_REQUIRE(!(d->phys_on && d_phys), "physics runs on the GPU (sml_dyn_set_physics): d_phys must be NULL");
    if (!d->impint_done) return fail(SML_ERR_STATE, "sml_dyn_impint must be called before sml_dyn_step");
    return launch_step(d, j1, j2, dt, alph, rob, wil, d_phys, d->lradsw, (hipStream_t)stream);
}

namespace {

// the step(2, 2, dt, ...) graph for one lradsw value, (re)captured when its inputs change
int leapfrog_graph(sml_dynamics *d, bool lradsw, const double key[4], const double *d_phys, hipGraphExec_t *out) {
    sml_dynamics::Replay &r = d->replay[lradsw ? 1 : 0];
    if (r.exec && std::memcmp(key, r.key, sizeof r.key) == 0 && d_phys == r.phys && d->d_tab == r.tab &&
        d->phys_on == r.phys_on) {
        *out = r.exec;
        return SML_OK;
    }
    if (r.exec) {
        SML_HIP(hipGraphExecDestroy(r.exec));
        r.exec = nullptr;
    }
    if (!d->cap_stream) SML_HIP(hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking));
    hipGraph_t g = nullptr;
    SML_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeThreadLocal));
    int rc = launch_step(d, 2, 2, key[0], key[1], key[2], key[3], d_phys, lradsw, d->cap_stream);
    hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
    if (rc) {
        if (g) (void)hipGraphDestroy(g);
        return rc;
    }
    if (e != hipSuccess) return fail(SML_ERR_HIP, "sml_dyn_leapfrog capture: %s", hipGetErrorString(e));
    e = hipGraphInstantiate(&r.exec, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (e != hipSuccess) {
        r.exec = nullptr;
        return fail(SML_ERR_HIP, "sml_dyn_leapfrog instantiate: %s", hipGetErrorString(e));
    }
    std::memcpy(r.key, key, sizeof r.key);
    r.phys = d_phys;
    r.tab = d->d_tab;
    r.phys_on = d->phys_on;
    *out = r.exec;
    return SML_OK;
}

}  // namespace

extern "C" int sml_dyn_leapfrog(sml_dynamics *d, int nsteps, double dt, double alph, double rob, double wil,
                                const double *d_phys, void *stream) {
    SML_REQUIRE(d && nsteps >= 0, "bad argument");
    SML_REQUIRE(!(d->phys_on && d_phys), "physics runs on the GPU (sml_dyn_set_physics): d_phys must be NULL");
    if (!d->impint_done) return fail(SML_ERR_STATE, "sml_dyn_impint must be called before sml_dyn_leapfrog");
    const double key[4] = {dt, alph, rob, wil};
    // stloop (dyn_stloop.f90:37-56): lradsw = (mod(istep, nstrad) == 1) before each step
    for (int i = 0; i < nsteps; ++i) {
        const bool lradsw = (d->istep % kNstrad == 1);
        hipGraphExec_t exec = nullptr;  // without GPU physics lradsw is irrelevant: one graph
        if (int rc = leapfrog_graph(d, d->phys_on && lradsw, key, d_phys, &exec)) return rc;
        SML_HIP(hipGraphLaunch(exec, (hipStream_t)stream));
        d->lradsw = lradsw;
        ++d->istep;
    }
    return SML_OK;
}

// One SPEEDY window after iogrid(30): stepone (ini_stepone.f90:19-34: step(1, 1,
// delt/2), step(1, 2, delt) with the lradsw the previous window left) and nleap x
// step(2, 2, 2 delt) with stloop's radiation clock restarted at istep = 1
// (dyn_stloop.f90:37-56, at_gcm.f90:81), captured once as ONE hipGraph per
// (entry lradsw, delt, alph, rob, wil, physics on, impint slots) and replayed with
// a single launch, so the host thread never waits on the window's ~200 kernels.
namespace {
// run_model's exit as window_impl captures it behind the window: iogrid(31)'s gridx
// (IoExit) and an optional one-lane store (the hybrid loop's forecast hop)
// and, with `entry`, run_model's entry in front of the window: iogrid(30)'s specx (its
// hop wait's value from d_xa) and k_io_entry, the first row kernel handing *go_src to the
// safety check's *go
struct EntrySpec {
    const double *g4, *logp;
    HopWait w;
    uint64_t *go;
    const uint64_t *go_src;
};
struct ExitSpec {
    const double *varm;
    double *fc4, *fc2;
    IoExit ex;
    uint64_t *store;
    uint64_t store_value;
    const EntrySpec *entry = nullptr;
};
int launch_entry(sml_dynamics *d, const double *d_grid4d, const double *d_logp, HopWait w, hipStream_t st,
                 uint64_t *xa, uint64_t xa0, uint64_t xa1);
int window_impl(sml_dynamics *d, int nleap, double delt, double alph, double rob, double wil, void *stream,
                bool prepared, const ExitSpec *exit = nullptr);
}  // namespace

extern "C" int sml_dyn_window(sml_dynamics *d, int nleap, double delt, double alph, double rob, double wil,
                              void *stream) {
    SML_REQUIRE(d && nleap >= 0 && delt > 0.0, "bad argument");
    return window_impl(d, nleap, delt, alph, rob, wil, stream, false);
}

namespace {
// prepared: the m-major state and step(1, 1)'s gridy output are already in place
// (k_io_entry, fused path of sml_dyn_run_model), so the graph starts at the row
// kernel of the first step
int window_impl(sml_dynamics *d, int nleap, double delt, double alph, double rob, double wil, void *stream,
                bool prepared, const ExitSpec *exit) {
    const double dts[3] = {0.5 * delt, delt, 2.0 * delt};
    DynTables *tab[3];
    for (int i = 0; i < 3; ++i) {  // 4 cached slots hold all three tables at once
        if (int rc = sml_dyn_impint(d, dts[i], alph)) return rc;
        tab[i] = d->d_tab;
    }
    const bool entry = d->lradsw;
    if (d->nograph) {  // the same launches, issued one by one on the stream (A/B: SML_DYN_NOGRAPH=1)
        hipStream_t st = (hipStream_t)stream;
        d->d_tab = tab[0];
        d->io_exit = prepared ? d->d_varm : nullptr;
        int rc = launch_step(d, 1, 1, dts[0], alph, rob, wil, nullptr, entry, st, prepared, 2);
        d->d_tab = tab[1];
        if (!rc) rc = launch_step(d, 1, 2, dts[1], alph, rob, wil, nullptr, entry, st, true, nleap > 0 ? 2 : 0);
        d->d_tab = tab[2];
        for (int i = 0; i < nleap && !rc; ++i)
            rc = launch_step(d, 2, 2, dts[2], alph, rob, wil, nullptr, (1 + i) % kNstrad == 1, st, true,
                             i + 1 < nleap ? 2 : 0);
        d->io_exit = nullptr;
        if (rc) return rc;
        d->istep = 1 + nleap;
        if (nleap > 0) d->lradsw = (nleap % kNstrad == 1);
        return SML_OK;
    }
    const int cls = (entry ? 1 : 0) + (prepared ? 2 : 0);
    const double key[8] = {(double)nleap, delt,  alph, rob, wil, d->phys_on ? 1.0 : 0.0, d->fused ? 1.0 : 0.0,
                           prepared ? 2.0 : 1.0};
    // the exit's (and entry's) fixed arguments (the counts and hop values change per
    // launch: d_xa)
    const void *exit_key[16] = {};
    if (exit) {
        const EntrySpec *en = exit->entry;
        const void *k[16] = {exit->varm,   exit->fc4,     exit->fc2,    exit->ex.mm,
                             exit->ex.in4, exit->ex.inlp, exit->ex.cnt, (const void *)(intptr_t)exit->ex.timeout,
                             exit->store,  en ? (const void *)1 : nullptr,
                             en ? en->w.flag : nullptr, en ? en->w.late : nullptr, en ? en->w.sig : nullptr,
                             en ? (const void *)(intptr_t)en->w.timeout : nullptr, en ? en->w.vptr : nullptr,
                             en ? en->go : nullptr};
        std::memcpy(exit_key, k, sizeof k);
    }
    auto same = [&](const sml_dynamics::WindowReplay &w) {
        return w.exec && w.has_exit == (exit != nullptr) &&
               (!exit || std::memcmp(exit_key, w.exit_key, sizeof exit_key) == 0) &&
               std::memcmp(key, w.key, sizeof key) == 0 && std::memcmp(tab, w.tab, sizeof tab) == 0;
    };
    sml_dynamics::WindowReplay *hit = nullptr;
    for (auto &w : d->wreplay[cls])
        if (same(w)) hit = &w;
    if (!hit) {  // capture into the class's next way
        hit = &d->wreplay[cls][d->wreplay_next[cls]];
        d->wreplay_next[cls] = (d->wreplay_next[cls] + 1) % sml_dynamics::kReplayWays;
    }
    sml_dynamics::WindowReplay &r = *hit;
    if (!same(r)) {
        if (r.exec) {
            SML_HIP(hipGraphExecDestroy(r.exec));
            r.exec = nullptr;
        }
        r.has_exit = false;
        if (!d->cap_stream) SML_HIP(hipStreamCreateWithFlags(&d->cap_stream, hipStreamNonBlocking));
        hipGraph_t g = nullptr;
        SML_HIP(hipStreamBeginCapture(d->cap_stream, hipStreamCaptureModeThreadLocal));
        // consecutive steps chained: each step's last kernel prepares the next one's
        // inverse transforms (j2 = 1 for step(1, 1), then 2)
        int rc = SML_OK;
        if (exit && exit->entry) {  // run_model's entry (specx + k_io_entry) in front of the window
            // (with the tables the entry read when it was launched before the graph: the
            // last impint's, 2 delt, as the previous window left them)
            const EntrySpec *en = exit->entry;
            rc = launch_entry(d, en->g4, en->logp, en->w, d->cap_stream, nullptr, 0, 0);
            d->go_src_next = en->go_src;  // the first row kernel lets the safety check go
            d->go_dst_next = en->go;
        }
        d->d_tab = tab[0];
        d->io_exit = prepared ? d->d_varm : nullptr;  // run_model: the exit's gridy in the last kernel
        if (!rc) rc = launch_step(d, 1, 1, dts[0], alph, rob, wil, nullptr, entry, d->cap_stream, prepared, 2);
        d->go_src_next = nullptr;
        d->go_dst_next = nullptr;
        d->d_tab = tab[1];
        if (!rc) rc = launch_step(d, 1, 2, dts[1], alph, rob, wil, nullptr, entry, d->cap_stream, true, nleap > 0 ? 2 : 0);
        d->d_tab = tab[2];
        for (int i = 0; i < nleap && !rc; ++i)
            rc = launch_step(d, 2, 2, dts[2], alph, rob, wil, nullptr, (1 + i) % kNstrad == 1, d->cap_stream, true,
                             i + 1 < nleap ? 2 : 0);
        if (!rc && exit) {  // iogrid(31)'s gridx and the hop's store behind the window
            rc = spectral_gridx_run_model_exit(d->sp, exit->varm, exit->fc4, exit->fc2, kNIoWind, exit->ex,
                                               d->cap_stream);
            if (!rc && exit->store) {
                hipLaunchKernelGGL(k_flag_store, dim3(1), dim3(64), 0, d->cap_stream, exit->store, exit->ex.xa);
                if (hipGetLastError() != hipSuccess) rc = fail(SML_ERR_HIP, "k_flag_store capture");
            }
        }
        hipError_t e = hipStreamEndCapture(d->cap_stream, &g);
        d->io_exit = nullptr;
        if (rc) {
            if (g) (void)hipGraphDestroy(g);
            return rc;
        }
        if (e != hipSuccess) return fail(SML_ERR_HIP, "sml_dyn_window capture: %s", hipGetErrorString(e));
        e = hipGraphInstantiate(&r.exec, g, nullptr, nullptr, 0);
        if (e != hipSuccess) {
            (void)hipGraphDestroy(g);
            r.exec = nullptr;
            return fail(SML_ERR_HIP, "sml_dyn_window instantiate: %s", hipGetErrorString(e));
        }
        (void)hipGraphDestroy(g);
        r.has_exit = exit != nullptr;
        std::memcpy(r.exit_key, exit_key, sizeof exit_key);
        std::memcpy(r.key, key, sizeof key);
        std::memcpy(r.tab, tab, sizeof tab);
    }
    SML_HIP(hipGraphLaunch(r.exec, (hipStream_t)stream));
    d->d_tab = tab[2];
    d->istep = 1 + nleap;
    if (nleap > 0) d->lradsw = (nleap % kNstrad == 1);
    return SML_OK;
}
}  // namespace

extern "C" int sml_dyn_set_clock(sml_dynamics *d, int istep, int lradsw) {
    SML_REQUIRE(d, "null context");
    d->istep = istep;
    d->lradsw = lradsw != 0;
    return SML_OK;
}

extern "C" int sml_dyn_get_clock(const sml_dynamics *d, int *istep, int *lradsw) {
    SML_REQUIRE(d, "null context");
    if (istep) *istep = d->istep;
    if (lradsw) *lradsw = d->lradsw ? 1 : 0;
    return SML_OK;
}

namespace {
// ini_sea's hybrid block (cpl_sea.f90:38-46) per grid point: where the coupler's
// (ice-blended) sst_am is less than 6 K above the hybrid SST take the hybrid SST, add
// the bias, blend with the sea ice as sea2atm does (cpl_sea.f90:197)
__global__ void k_hybrid_sst(const double *__restrict__ cpl, const double *__restrict__ hyb,
                             const double *__restrict__ sice, const double *__restrict__ tice, double bias,
                             double *__restrict__ sst_am) {
#pragma clang fp contract(off)  // the reference's separate multiply and add (this file contracts by default)
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kNGP) return;
    double s = cpl[p];
    if (hyb) {
        const double diff = s - hyb[p];
        if (diff < 6.0) s = hyb[p];
        s = s + bias;
        const double d = tice[p] - s;
        s = s + sice[p] * d;
    }
    sst_am[p] = s;
}
}  // namespace

// run_model's SST hand-over (mpires.f90:1576-1584: internal_state_vector%sst_hybrid)
// as agcm_init's ini_sea applies it to the window's sst_am (cpl_sea.f90:38-46):
// d_sst_grid(96, 48) device; NULL restores the coupler's sst_am.  On `stream`, so a
// loop orders it before its next window.
extern "C" int sml_dyn_set_hybrid_sst(sml_dynamics *d, const double *d_sst_grid, double sst_bias, void *stream) {
    SML_REQUIRE(d, "null context");
    SML_REQUIRE(d->phys_on, "sml_dyn_set_physics must provide the boundary fields first");
    d->hyb_sst = d_sst_grid;
    d->hyb_bias = sst_bias;
    ++d->ford_gen;
    hipLaunchKernelGGL(k_hybrid_sst, dim3((kNGP + 255) / 256), dim3(256), 0, (hipStream_t)stream, d->d_sst_cpl,
                       d_sst_grid, d->d_sice, d->d_tice, sst_bias, d->d_pbc + (size_t)kBcSst * kNGP);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_dyn_set_physics(sml_dynamics *d, const double *bc) {
    SML_REQUIRE(d, "null context");
    if (!bc) {
        d->phys_on = false;
        return SML_OK;
    }
    SML_HIP(hipDeviceSynchronize());  // steps in flight may still read the old fields
    SML_HIP(hipMemcpy(d->d_pbc, bc, (size_t)kNBc * kNGP * 8, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_sst_cpl, bc + (size_t)kBcSst * kNGP, kNGP * 8, hipMemcpyHostToDevice));
    d->phys_on = true;
    ++d->ford_gen;
    if (d->hyb_sst) {  // a hybrid SST is in force: ini_sea applies it to every new sst_am
        if (int rc = sml_dyn_set_hybrid_sst(d, d->hyb_sst, d->hyb_bias, nullptr)) return rc;
        SML_HIP(hipDeviceSynchronize());
    }
    return SML_OK;
}

// sea-ice fraction and temperature of the coupler (sice_am, tice_am; cpl_sea.f90:
// 190-194), host [ngp] each; NULL = no ice (zero fraction)
extern "C" int sml_dyn_set_sea_ice(sml_dynamics *d, const double *sice, const double *tice) {
    SML_REQUIRE(d && (sice == nullptr) == (tice == nullptr), "sice and tice go together");
    SML_HIP(hipDeviceSynchronize());
    if (sice) {
        SML_HIP(hipMemcpy(d->d_sice, sice, kNGP * 8, hipMemcpyHostToDevice));
        SML_HIP(hipMemcpy(d->d_tice, tice, kNGP * 8, hipMemcpyHostToDevice));
    } else {
        SML_HIP(hipMemset(d->d_sice, 0, kNGP * 8));
        SML_HIP(hipMemset(d->d_tice, 0, kNGP * 8));
    }
    ++d->ford_gen;
    if (d->hyb_sst) return sml_dyn_set_hybrid_sst(d, d->hyb_sst, d->hyb_bias, nullptr);
    return SML_OK;
}

extern "C" int sml_dyn_get_sea_ice(sml_dynamics *d, double *sice, double *tice) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    if (sice) SML_HIP(hipMemcpy(sice, d->d_sice, kNGP * 8, hipMemcpyDeviceToHost));
    if (tice) SML_HIP(hipMemcpy(tice, d->d_tice, kNGP * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

// the boundary fields as phypar reads them, host [kNBc][ngp] (sml_dyn_set_physics order)
extern "C" int sml_dyn_get_physics(sml_dynamics *d, double *bc) {
    SML_REQUIRE(d && bc, "null argument");
    SML_REQUIRE(d->phys_on, "no boundary fields (sml_dyn_set_physics)");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(bc, d->d_pbc, (size_t)kNBc * kNGP * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

// ------------------------------------------------------ per-window forcing (fordate)
// run_model hands SPEEDY the calendar date of every window (mpires.f90:1545, :1595-1598)
// and agcm_init rebuilds the date's forcing before stepone (ini_agcm_init.f90:57-89):
// newdate(0), ini_coupler(2) and fordate(0); agcm_1day runs fordate(1) again before the
// leapfrog loop (at_gcm.f90:84) with the same inputs (lco2 is .false., mod_lflags.f90:
// 16, so imode 1 changes nothing).  With the coupler flags of the reference
// (icland = 1, icsea = 0, icice = 1, isstan = 0; mod_cpl_flags.f90) and jday = 0:
//   land (cpl_land.f90:1-95)  stl_am = forin5(stl12), snowd_am = forint(snowd12),
//                             soilw_am = forint(soilw12)
//   sea  (cpl_sea.f90:1-200)  sst = forin5(sst12), sice = forint(sice12) adjusted over
//                             sea ice (:96-117, tice), sst_am = sst + sice (tice - sst),
//                             then ini_sea's hybrid block (:38-46, k_hybrid_sst)
//   fordate (ini_fordate.f90:50-113)  sol_oz(tyear), the surface albedo, tcorh =
//                             spec(gamlat phis0), qcorh = spec(refrh1 (qref - qsfc))
//                             from the current stl_am / sst_am
// One thread per grid point; then spec of the two correction fields.
namespace {
struct FordateArgs {
    double sol[5][kIL];  // sol_oz per latitude row: fsol, ozone, ozupp, zenit, stratz
    int m5[5];
    double w5[5];
    int mi[2];
    double wmon;
    int clim, hyb;
    double bias;
};

__global__ __launch_bounds__(256) void k_fordate(FordateArgs a, const double *__restrict__ surf,
                                                 const double *__restrict__ clim, const double *__restrict__ hyb,
                                                 double *__restrict__ pbc, double *__restrict__ sst_cpl,
                                                 double *__restrict__ sice_am, double *__restrict__ tice_am,
                                                 double *__restrict__ corh) {
#pragma clang fp contract(off)  // the reference's separate multiplies and adds
    SML_TL_SCOPE(sml::tl::kFordate);
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= kNGP) return;
    const int j = p / kIX;
    const double fmask_l = surf[p], fmask_s = surf[kNGP + p], alb0 = surf[2 * kNGP + p];
    double snowc, sice, cpl;
    if (a.clim) {
        auto field = [&](int f, int m) { return clim[((size_t)f * 12 + m) * kNGP + p]; };
        auto forin5 = [&](int f) {
            return a.w5[0] * field(f, a.m5[0]) + a.w5[1] * field(f, a.m5[1]) + a.w5[2] * field(f, a.m5[2]) +
                   a.w5[3] * field(f, a.m5[3]) + a.w5[4] * field(f, a.m5[4]);
        };
        auto forint = [&](int f) {
            const double f0 = field(f, a.mi[0]);
            return f0 + a.wmon * (field(f, a.mi[1]) - f0);
        };
        // land: atm2land(0), stl_lm = stlcl_ob (ini_land, istart 2), land2atm(0)
        const double stl = forin5(0), snowd = forint(1), soilw = forint(2);
        pbc[(size_t)kBcStl * kNGP + p] = stl;
        pbc[(size_t)kBcSoilw * kNGP + p] = soilw;
        snowc = fmin(1., snowd / 60.0);  // fordate: min(1, snowd_am / sd2sc), mod_surfcon sd2sc
        // sea: atm2sea(0) with the sea-ice adjustment of the climatology
        double sst = forin5(3), sic = forint(4), tic;
        const double sstfr = 273.2 - 1.8;
        if (sst > sstfr) {
            sic = fmin(0.5, sic);
            tic = sstfr;
            if (sic > 0.) sst = sstfr + (sst - sstfr) / (1. - sic);
        } else {
            sic = fmax(0.5, sic);
            tic = sstfr + (sst - sstfr) / sic;
            sst = sstfr;
        }
        // ini_sea: the ocean / ice model starts from the climatology; sea2atm(0):
        // icsea 0 -> sst_am = sstcl_ob (+ no anomaly), icice 1 -> the model's ice
        sst = sst + 0.0;
        sst = sst + sic * (tic - sst);
        sice_am[p] = sic;
        tice_am[p] = tic;
        sst_cpl[p] = sst;
        sice = sic;
        cpl = sst;
    } else {
        snowc = pbc[(size_t)kBcSnowc * kNGP + p];
        sice = sice_am[p];
        cpl = sst_cpl[p];
    }
    double sst_am = cpl;
    if (a.hyb) {  // ini_sea's hybrid block, as k_hybrid_sst
        const double h = hyb[p];
        const double diff = sst_am - h;
        if (diff < 6.0) sst_am = h;
        sst_am = sst_am + a.bias;
        sst_am = sst_am + sice * (tice_am[p] - sst_am);
    }
    pbc[(size_t)kBcSst * kNGP + p] = sst_am;
    // fordate 2: daily-mean radiative forcing and the surface albedo
    pbc[(size_t)kBcFsol * kNGP + p] = a.sol[0][j];
    pbc[(size_t)kBcOzone * kNGP + p] = a.sol[1][j];
    pbc[(size_t)kBcOzupp * kNGP + p] = a.sol[2][j];
    pbc[(size_t)kBcZenit * kNGP + p] = a.sol[3][j];
    pbc[(size_t)kBcStratz * kNGP + p] = a.sol[4][j];
    const double albsn = 0.60, albsea = 0.07, albice = 0.60;  // mod_radcon.f90:59-61
    const double alb_l = alb0 + snowc * (albsn - alb0);
    const double alb_s = albsea + sice * (albice - albsea);
    pbc[(size_t)kBcSnowc * kNGP + p] = snowc;
    pbc[(size_t)kBcAlbL * kNGP + p] = alb_l;
    pbc[(size_t)kBcAlbS * kNGP + p] = alb_s;
    pbc[(size_t)kBcAlbsfc * kNGP + p] = alb_s + fmask_l * (alb_l - alb_s);
    // fordate 3-4: the horizontal-diffusion corrections (setgam: gamlat = gamma / (1000 g))
    const double gamlat = 6.0 / (1000. * 9.81), rd = 287., refrh1 = 0.7;
    const double c = gamlat * pbc[(size_t)kBcPhis0 * kNGP + p];
    const double pexp = 1. / (rd * gamlat);
    const double tsfc = fmask_l * pbc[(size_t)kBcStl * kNGP + p] + fmask_s * sst_am;
    const double tref = tsfc + c;
    const double psfc = pow(tsfc / tref, pexp);
    // shtorh(0, .., tref, 1, -1, ..) and shtorh(0, .., tsfc, psfc, 1, ..) (phy_shtorh.f90:27-51)
    auto qsat = [](double ta, double ps) {
        const double e0 = 6.108e-3, c1 = 17.269, c2 = 21.875, t0 = 273.16, t1 = 35.86, t2 = 7.66;
        const double q = (ta >= t0) ? e0 * exp(c1 * (ta - t0) / (ta - t1)) : e0 * exp(c2 * (ta - t0) / (ta - t2));
        return 622. * q / (ps - 0.378 * q);
    };
    const double qref = qsat(tref, 1.0), qsfc = qsat(tsfc, 1. * psfc);
    corh[p] = c;
    corh[kGF + p] = refrh1 * (qref - qsfc);
}

}  // namespace

// inbcon's time-independent surface fields fordate reads (ini_inbcon.f90:38-70,
// 140-156): host [3][ngp] = fmask_l (mod_cli_land), fmask_s (mod_cli_sea), alb0
// (mod_surfcon); NULL switches sml_dyn_fordate off
extern "C" int sml_dyn_set_surface(sml_dynamics *d, const double *surf) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    d->surf_on = surf != nullptr;
    if (surf) SML_HIP(hipMemcpy(d->d_surf, surf, (size_t)3 * kNGP * 8, hipMemcpyHostToDevice));
    ++d->ford_gen;
    return SML_OK;
}

// the coupler's monthly climatologies (inbcon, ini_inbcon.f90:71-230): host
// [5][12][ngp] = stl12, snowd12, soilw12 (mod_cli_land), sst12, sice12 (mod_cli_sea),
// month 1 first; NULL: sml_dyn_fordate keeps the coupler fields the host set
// (sml_dyn_set_physics' stl_am / sst_am / soilw_am / snowc, sml_dyn_set_sea_ice)
extern "C" int sml_dyn_set_climatology(sml_dynamics *d, const double *clim) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    if (clim) {
        if (!d->d_clim) SML_HIP(hipMalloc(&d->d_clim, (size_t)5 * 12 * kNGP * 8));
        SML_HIP(hipMemcpy(d->d_clim, clim, (size_t)5 * 12 * kNGP * 8, hipMemcpyHostToDevice));
    }
    d->clim_on = clim != nullptr;
    ++d->ford_gen;
    return SML_OK;
}

// agcm_init's forcing for a window at (iyear, imonth, iday) on `stream`: coupler,
// hybrid SST, fordate (see k_fordate).  A no-op when neither the date nor any input
// changed since the last call (the window's forcing stays as computed); force != 0
// recomputes anyway.  Ordered on `stream`: the next window on that stream reads it.
extern "C" int sml_dyn_fordate_ex(sml_dynamics *d, int iyear, int imonth, int iday, int force, void *stream) {
    // the days of newdate's 365-day table (ini_fordate / mod_date), plus February 29,
    // which the reference calendar emits once its SAVEd February latch is set
    // (mod_calendar.f90:40, 61-63); a later day would extrapolate tmonth past the month
    static const int kMonthDays[12] = {31, 29, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    SML_REQUIRE(d && imonth >= 1 && imonth <= 12 && iday >= 1 && iday <= kMonthDays[imonth - 1],
                "bad date %d-%d-%d", iyear, imonth, iday);
    SML_REQUIRE(d->phys_on, "sml_dyn_set_physics must provide the boundary fields first");
    SML_REQUIRE(d->surf_on, "sml_dyn_set_surface must provide fmask_l, fmask_s and alb0 first");
    (void)iyear;  // only the co2 trend reads the year (lco2 = .false.)
    if (!force && d->ford_done == d->ford_gen && d->ford_date[0] == imonth && d->ford_date[1] == iday)
        return SML_OK;
    hipStream_t st = (hipStream_t)stream;
    ForDate fd;
    phys_fordate_weights(imonth, iday, &fd);
    FordateArgs a;
    phys_sol_oz_lat(d->ptab, fd.tyear, &a.sol[0][0]);
    for (int k = 0; k < 5; ++k) {
        a.m5[k] = fd.m5[k];
        a.w5[k] = fd.w5[k];
    }
    a.mi[0] = fd.mi[0];
    a.mi[1] = fd.mi[1];
    a.wmon = fd.wmon;
    a.clim = d->clim_on ? 1 : 0;
    a.hyb = d->hyb_sst ? 1 : 0;
    a.bias = d->hyb_bias;
    double *grid = d->d_ford, *varm = d->d_ford + 2 * kGF;
    hipLaunchKernelGGL(k_fordate, dim3((kNGP + 255) / 256), dim3(256), 0, st, a, d->d_surf, d->d_clim, d->hyb_sst,
                       d->d_pbc, d->d_sst_cpl, d->d_sice, d->d_tice, grid);
    SML_HIP(hipGetLastError());
    // spec (specx + specy) of corh -> tcorh, qcorh (contiguous)
    if (int rc = spectral_specx(d->sp, grid, varm, 2, 0, st)) return rc;
    if (int rc = spectral_specy(d->sp, varm, d->d_tcorh, 2, st)) return rc;
    d->ford_done = d->ford_gen;
    d->ford_date[0] = imonth;
    d->ford_date[1] = iday;
    ++d->ford_count;
    return SML_OK;
}

extern "C" int sml_dyn_fordate(sml_dynamics *d, int iyear, int imonth, int iday, void *stream) {
    return sml_dyn_fordate_ex(d, iyear, imonth, iday, 0, stream);
}

extern "C" int sml_dyn_fordate_count(const sml_dynamics *d, int *count) {
    SML_REQUIRE(d && count, "null argument");
    *count = d->ford_count;
    return SML_OK;
}

extern "C" int sml_dyn_set_rad_state(sml_dynamics *d, const double *rad) {
    SML_REQUIRE(d, "null context");
    SML_HIP(hipDeviceSynchronize());
    if (rad)
        SML_HIP(hipMemcpy(d->d_rad, rad, kRadSize * 8, hipMemcpyHostToDevice));
    else
        SML_HIP(hipMemset(d->d_rad, 0, kRadSize * 8));
    return SML_OK;
}

extern "C" int sml_dyn_get_rad_state(sml_dynamics *d, double *rad) {
    SML_REQUIRE(d && rad, "null argument");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(rad, d->d_rad, kRadSize * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_phypar(sml_dynamics *d, const double *d_ug1, const double *d_vg1, const double *d_tg1,
                              const double *d_qg1, const double *d_phig1, const double *d_pslg1, int lradsw,
                              double *d_tend, void *stream) {
    SML_REQUIRE(d && d_ug1 && d_vg1 && d_tg1 && d_qg1 && d_phig1 && d_pslg1 && d_tend, "null argument");
    SML_REQUIRE(d->phys_on, "sml_dyn_set_physics must provide the boundary fields first");
    hipLaunchKernelGGL(k_phys, dim3(kNGP / 64), dim3(64), 0, (hipStream_t)stream, d_ug1, d_vg1, d_tg1, d_qg1,
                       d_phig1, d_pslg1, d->d_pbc, d->d_rad, d->d_ptab, lradsw ? 1 : 0, d_tend);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_dyn_phypar_host(sml_dynamics *d, const double *ug1, const double *vg1, const double *tg1,
                                   const double *qg1, const double *phig1, const double *pslg1, int lradsw,
                                   double *tend) {
    SML_REQUIRE(d && ug1 && vg1 && tg1 && qg1 && phig1 && pslg1 && tend, "null argument");
    const size_t f3 = (size_t)kKX * kNGP;
    double *b = d->d_pio;
    const double *src[5] = {ug1, vg1, tg1, qg1, phig1};
    for (int i = 0; i < 5; ++i) SML_HIP(hipMemcpy(b + i * f3, src[i], f3 * 8, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(b + 5 * f3, pslg1, kNGP * 8, hipMemcpyHostToDevice));
    double *out = b + 5 * f3 + kNGP;
    if (int rc = sml_dyn_phypar(d, b, b + f3, b + 2 * f3, b + 3 * f3, b + 4 * f3, b + 5 * f3, lradsw, out, nullptr))
        return rc;
    SML_HIP(hipMemcpy(tend, out, 4 * f3 * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_sol_oz(const sml_dynamics *d, double tyear, double *fields5) {
    SML_REQUIRE(d && fields5, "null argument");
    phys_sol_oz(d->ptab, tyear, fields5);
    return SML_OK;
}

extern "C" int sml_phys_sflset(const double *phi0, double *forog) {
    SML_REQUIRE(phi0 && forog, "null argument");
    phys_sflset(phi0, forog);
    return SML_OK;
}

namespace {

// iogrid inverse half: level 1 -> G = [u 8 | v 8 | t 8 | q 8 | ps] grids
}  // namespace

namespace {
// the safety check of iogrid(30) (ppo_iogrid.f90:556-571) from its spectral inputs in
// d_chk (k_io_prep / k_io_entry, already on st): the re-grid and its min / max run on
// chk_stream beside the window.  A caller's d_minmax is ready in st's order; the
// internal one (nullptr) only for the next user of d_chk (which waits for it).
// go > 0 (the entry inside the window graph): instead of an event fork from st, the
// check's stream waits in-kernel for the window's first row kernel to store go
int launch_io_check(sml_dynamics *d, hipStream_t st, double *d_minmax, uint64_t go = 0) {
    double *cs = d->d_chk, *cv = cs + (size_t)kNIo * kSF, *cg = cv + (size_t)kNIo * kVF;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    SML_HIP(hipStreamIsCapturing(st, &cap));
    hipStream_t cst = st;
    if (cap == hipStreamCaptureStatusNone) {
        if (!d->chk_stream) {
            SML_HIP(hipStreamCreateWithFlags(&d->chk_stream, hipStreamNonBlocking));
            SML_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
            SML_HIP(hipEventCreateWithFlags(&d->ev_chk, hipEventDisableTiming));
        }
        cst = d->chk_stream;
        if (go) {
            hipLaunchKernelGGL(k_check_go, dim3(1), dim3(64), 0, cst, d->d_go, go, d->d_chk_late,
                               4u * (d->chk_count + 1), d->chk_timeout);
            SML_HIP(hipGetLastError());
        } else {
            SML_HIP(hipEventRecord(d->ev_fork, st));
            SML_HIP(hipStreamWaitEvent(d->chk_stream, d->ev_fork, 0));
        }
    } else if (go) {
        return fail(SML_ERR_STATE, "launch_io_check: a go hand-off while the stream is captured");
    }
    if (int rc = spectral_gridy(d->sp, cs, cv, kNIo, cst)) return rc;
    if (int rc = spectral_gridx_range(d->sp, cv, cg, kNIo, 0, kNIoWind, cst)) return rc;
    double *mm = d_minmax ? d_minmax : d->d_minmax;
    // on the check stream, for run_model's exit: the counter hand-off (4 adds per check)
    const bool counted = cst != st && !d_minmax;
    hipLaunchKernelGGL(k_io_minmax, dim3(4), dim3(1024), 0, cst, cg, mm, counted ? d->d_chk_cnt : nullptr,
                       go ? d->d_chk_late : nullptr, 4u * (d->chk_count + 1));
    SML_HIP(hipGetLastError());
    if (counted) ++d->chk_count;
    d->chk_counted = counted;
    d->mm_last = mm;
    d->mm_issued = false;
    if (cst != st) {  // a host copy for sml_dyn_last_safe, behind the check on its stream
        if (!d->h_mm) {
            SML_HIP(hipHostMalloc((void **)&d->h_mm, 8 * sizeof(double), hipHostMallocDefault));
            SML_HIP(hipEventCreateWithFlags(&d->ev_mm, hipEventDisableTiming));
        }
        SML_HIP(hipMemcpyAsync(d->h_mm, mm, 8 * sizeof(double), hipMemcpyDeviceToHost, cst));
        SML_HIP(hipEventRecord(d->ev_mm, cst));
        d->mm_issued = true;
        SML_HIP(hipEventRecord(d->ev_chk, cst));
        d->chk_pending = true;
        if (d_minmax) {
            SML_HIP(hipStreamWaitEvent(st, d->ev_chk, 0));
            d->chk_pending = false;
        }
    }
    return SML_OK;
}

// run_model's entry: iogrid(30)'s specx (waiting for its grid when w.flag) and the per-m
// k_io_entry (specy, the combine into level 1, the check's inputs, the m-major state,
// step(1, 1)'s gridy); xa: an exit captured in the window graph takes its per-launch
// values from there (k_io_entry stores xa0 / xa1), else null
int launch_entry(sml_dynamics *d, const double *d_grid4d, const double *d_logp, HopWait w, hipStream_t st,
                 uint64_t *xa, uint64_t xa0, uint64_t xa1) {
    if (int rc = spectral_specx_io(d->sp, d_grid4d, d_logp, d->d_vfm, kNIoWind, st, w)) return rc;
    const SpectralDev sd = spectral_dev(d->sp);
    const bool phys = d->phys_on;
    hipLaunchKernelGGL(k_io_entry, dim3(kMX), dim3(kSpecThreads), 0, st, d->d_vfm, d->d_pfl, sd.wt, d->d_state,
                       sm_buf(d, 0), d->d_chk, d->d_phis,
                       d->d_tabm + (size_t)(d->d_tab - d->d_tabs) * kMX * kTabMDoubles, sd.pinv, d->d_varm,
                       phys ? kNInv1P : kNInv1, phys ? kNInvP : kNInv, xa, xa0, xa1);
    SML_HIP(hipGetLastError());
    return SML_OK;
}
}  // namespace

extern "C" int sml_dyn_from_grid(sml_dynamics *d, const double *d_grid4d, const double *d_logp, double *d_minmax,
                                 void *stream) {
    SML_REQUIRE(d && d_grid4d && d_logp, "null argument");
    hipStream_t st = (hipStream_t)stream;
    const DynTables *T = d->d_tab;
    if (d->chk_pending) {  // the previous check still reads d_chk
        SML_HIP(hipStreamWaitEvent(st, d->ev_chk, 0));
        d->chk_pending = false;
    }
    // entry (:503-518): real(4) copies, q clip, then vdspec kcos = 2 (x cosgr) on the
    // winds and none on the rest: one specx launch reading variables3d / logp
    HopWait w = d->entry_wait;
    w.sig = d->entry_sig;
    d->entry_wait = HopWait{};  // one launch
    d->entry_sig = nullptr;
    if (int rc = spectral_specx_io(d->sp, d_grid4d, d_logp, d->d_varm, kNIoWind, st, w)) return rc;
    if (int rc = spectral_specy(d->sp, d->d_varm, d->d_sfwd, kNIo, st)) return rc;
    hipLaunchKernelGGL(k_io_combine, dim3((kMN + 127) / 128, kKX), dim3(128), 0, st, d->d_sfwd, d->d_state, T);
    SML_HIP(hipGetLastError());
    // the safety check (:556-571) reads the new state: its k_io_prep stays on st (the
    // window overwrites the state), the rest of it beside the window
    hipLaunchKernelGGL(k_io_prep, dim3((kMN + 127) / 128, kKX), dim3(128), 0, st, d->d_state, d->d_chk, T);
    SML_HIP(hipGetLastError());
    return launch_io_check(d, st, d_minmax);
}

extern "C" int sml_dyn_to_grid(sml_dynamics *d, double *d_grid4d, double *d_logp, void *stream) {
    SML_REQUIRE(d && d_grid4d && d_logp, "null argument");
    hipStream_t st = (hipStream_t)stream;
    // exit (:590-595): the state re-gridded (k_io_prep, gridy, gridx) with the gridx
    // writing variables3d / logp directly
    hipLaunchKernelGGL(k_io_prep, dim3((kMN + 127) / 128, kKX), dim3(128), 0, st, d->d_state, d->d_specin, d->d_tab);
    SML_HIP(hipGetLastError());
    if (int rc = spectral_gridy(d->sp, d->d_specin, d->d_varm, kNIo, st)) return rc;
    return spectral_gridx_io(d->sp, d->d_varm, d_grid4d, d_logp, kNIoWind, st);
}

extern "C" int sml_dyn_is_safe(const double *minmax) {
    if (!minmax) return 0;
    return io_state_safe(minmax) ? 1 : 0;  // u, v, t, q thresholds (ppo_iogrid.f90:563-577)
}

// run_model (src/mpires.f90:1516-1628) on the device: agcm_main's window entry
// iogrid(30) with its safety check, the window (integrated whatever the check says:
// the outcome is selected at the exit), iogrid(31), then run_model's q floor; when
// the entry state was unsafe agcm_main skipped the integration (at_gcm.f90:37) and
// the forecast is the input grid (q floored).  The check runs beside the window on
// the context's check stream; the exit waits for it.
extern "C" int sml_dyn_run_model(sml_dynamics *d, const double *d_grid4d, const double *d_logp, int nleap,
                                 double delt, double alph, double rob, double wil, double *d_fc4d, double *d_fc2d,
                                 void *stream) {
    SML_REQUIRE(d && d_grid4d && d_logp && d_fc4d && d_fc2d, "null argument");
    SML_REQUIRE(d_fc4d != d_grid4d && d_fc2d != d_logp, "the forecast must not overwrite the window's input");
    SML_REQUIRE(nleap >= 0 && delt > 0.0, "bad argument");
    hipStream_t st = (hipStream_t)stream;
    if (d->fused) {
        // iogrid(30)'s specx, then ONE per-m launch for specy, the combine into level 1,
        // the check's inputs, the m-major state and step(1, 1)'s gridy (k_io_entry);
        // the window graph then starts at the first row kernel
        if (d->chk_pending) {
            SML_HIP(hipStreamWaitEvent(st, d->ev_chk, 0));
            d->chk_pending = false;
        }
        HopWait w = d->entry_wait;
        w.sig = d->entry_sig;
        d->entry_wait = HopWait{};  // one launch
        d->entry_sig = nullptr;
        const bool phys = d->phys_on;
        d->sm_cur = 0;  // the window's chain starts in buffer 0
        // the exit inside the window graph: needs the check's counter hand-off (no event
        // wait between the window and the exit; the check below counts unless captured)
        // and the graph path.  Its per-launch values go through d_xa
        hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
        SML_HIP(hipStreamIsCapturing(st, &cap));
        const bool xg = !d->nograph && cap == hipStreamCaptureStatusNone;
        if (xg && !d->d_xa) SML_HIP(hipMalloc(&d->d_xa, 4 * sizeof(uint64_t)));
        // and the entry inside it too (r06): specx + k_io_entry as the graph's first
        // nodes, the safety check forked by the first row kernel's go store instead of an
        // event after k_io_entry -- one launch boundary fewer on the chain, and the graph's
        // launch hidden behind the entry's wait.  Not under serialised dispatch (the check,
        // enqueued after the graph, would run after the exit that waits for it)
        if (xg && phys && d->entry_graph && !d->serialized) {
            if (!d->d_go) {
                SML_HIP(hipMalloc(&d->d_go, sizeof(uint64_t)));
                SML_HIP(hipMemset(d->d_go, 0, sizeof(uint64_t)));
                SML_HIP(hipDeviceSynchronize());
                d->go_count = 0;
            }
            const uint64_t go = ++d->go_count;
            hipLaunchKernelGGL(k_set_xa, dim3(1), dim3(64), 0, st, d->d_xa, (uint64_t)(4u * (d->chk_count + 1)),
                               d->exit_store_value, w.value, go);
            SML_HIP(hipGetLastError());
            EntrySpec en{d_grid4d, d_logp, w, d->d_go, d->d_xa + 3};
            if (w.flag) en.w.vptr = d->d_xa + 2;
            ExitSpec es{d->d_varm, d_fc4d, d_fc2d, IoExit{0.000001, d->d_minmax, d_grid4d, d_logp}, d->exit_store,
                        0};
            es.ex.cnt = d->d_chk_cnt;
            es.ex.xa = d->d_xa;
            es.ex.late = d->d_chk_late;
            es.ex.timeout = d->chk_timeout;
            es.entry = &en;
            d->exit_store = nullptr;  // one launch
            if (int rc = window_impl(d, nleap, delt, alph, rob, wil, stream, true, &es)) return rc;
            // enqueued after the graph, so whatever queue it shares, its producer is ahead
            if (int rc = launch_io_check(d, st, nullptr, go)) return rc;
            if (!(d->chk_pending && d->chk_counted && d->mm_last == d->d_minmax))
                return fail(SML_ERR_STATE, "sml_dyn_run_model: the safety check did not take the counter hand-off");
            d->chk_pending = false;  // the exit waits for the check's counter itself
            return SML_OK;
        }
        if (int rc = launch_entry(d, d_grid4d, d_logp, w, st, xg ? d->d_xa : nullptr,
                                  (uint64_t)(4u * (d->chk_count + 1)), d->exit_store_value))
            return rc;
        if (int rc = launch_io_check(d, st, nullptr)) return rc;
        if (xg) {
            if (!(d->chk_pending && d->chk_counted))
                return fail(SML_ERR_STATE, "sml_dyn_run_model: the safety check did not take the counter hand-off");
            ExitSpec es{d->d_varm, d_fc4d, d_fc2d, IoExit{0.000001, d->mm_last, d_grid4d, d_logp}, d->exit_store,
                        0};
            es.ex.cnt = d->d_chk_cnt;
            es.ex.xa = d->d_xa;
            es.ex.late = d->d_chk_late;
            es.ex.timeout = d->chk_timeout;
            d->chk_pending = false;
            d->exit_store = nullptr;  // one launch
            return window_impl(d, nleap, delt, alph, rob, wil, stream, true, &es);
        }
        if (int rc = window_impl(d, nleap, delt, alph, rob, wil, stream, true)) return rc;
    } else {
        if (int rc = sml_dyn_from_grid(d, d_grid4d, d_logp, nullptr, stream)) return rc;
        if (int rc = sml_dyn_window(d, nleap, delt, alph, rob, wil, stream)) return rc;
    }
    IoExit ex{0.000001, d->mm_last, d_grid4d, d_logp};
    if (d->chk_pending && d->chk_counted) {
        // the exit kernel itself waits for the check's counter: no event wait (a
        // barrier packet with a cross-queue dependency) on the window's stream.  The
        // check is complete once the exit has run, so the next user of d_chk needs no
        // wait either
        ex.cnt = d->d_chk_cnt;
        ex.target = 4u * d->chk_count;
        ex.late = d->d_chk_late;
        ex.timeout = d->chk_timeout;
        d->chk_pending = false;
    } else if (d->chk_pending) {  // the exit reads the check's min/max
        SML_HIP(hipStreamWaitEvent(st, d->ev_chk, 0));
        d->chk_pending = false;
    }
    if (!d->fused) {  // the fused window's last kernel did iogrid(31)'s prep + gridy already
        hipLaunchKernelGGL(k_io_prep, dim3((kMN + 127) / 128, kKX), dim3(128), 0, st, d->d_state, d->d_specin,
                           d->d_tab);
        SML_HIP(hipGetLastError());
        if (int rc = spectral_gridy(d->sp, d->d_specin, d->d_varm, kNIo, st)) return rc;
    }
    if (int rc = spectral_gridx_run_model_exit(d->sp, d->d_varm, d_fc4d, d_fc2d, kNIoWind, ex, st)) return rc;
    if (d->exit_store) {
        hipLaunchKernelGGL(k_flag_store_value, dim3(1), dim3(64), 0, st, d->exit_store, d->exit_store_value);
        SML_HIP(hipGetLastError());
        d->exit_store = nullptr;  // one launch
    }
    return SML_OK;
}

extern "C" int sml_dyn_set_check_cus(sml_dynamics *d, int first_cu, int num_cus) {
    SML_REQUIRE(d && first_cu >= 0 && num_cus >= 0, "bad argument");
    if (d->chk_stream) {  // the old stream's check completes first
        SML_HIP(hipStreamSynchronize(d->chk_stream));
        SML_HIP(hipStreamDestroy(d->chk_stream));
        d->chk_stream = nullptr;
        d->chk_pending = false;
    }
    if (num_cus > 0) {
        void *s = nullptr;
        if (int rc = sml_stream_create_cu_range(first_cu, num_cus, &s)) return rc;
        d->chk_stream = (hipStream_t)s;
    } else {
        SML_HIP(hipStreamCreateWithFlags(&d->chk_stream, hipStreamNonBlocking));
    }
    if (!d->ev_fork) SML_HIP(hipEventCreateWithFlags(&d->ev_fork, hipEventDisableTiming));
    if (!d->ev_chk) SML_HIP(hipEventCreateWithFlags(&d->ev_chk, hipEventDisableTiming));
    return SML_OK;
}

// run_speedy of the last sml_dyn_from_grid / sml_dyn_run_model (is_safe_to_run_speedy,
// broadcast as run_speedy, src/mpires.f90:721, 1623): waits only for that check
extern "C" int sml_dyn_last_safe(sml_dynamics *d, int *safe, double *minmax) {
    SML_REQUIRE(d && safe, "null argument");
    double mm[8];
    if (d->mm_issued) {
        // a host loop polls this once per step (parallelmain.f90:268-270): spin on the
        // event rather than hipEventSynchronize, whose wait policy may yield the thread
        // on a loaded host and wake it late, stalling the next step's enqueue
        hipError_t q;
        while ((q = hipEventQuery(d->ev_mm)) == hipErrorNotReady) {
        }
        SML_HIP(q);
        std::memcpy(mm, d->h_mm, sizeof mm);
    } else if (d->mm_last) {  // issued on the caller's stream (capture): synchronous copy
        SML_HIP(hipDeviceSynchronize());
        SML_HIP(hipMemcpy(mm, d->mm_last, sizeof mm, hipMemcpyDeviceToHost));
    } else {
        return fail(SML_ERR_STATE, "sml_dyn_last_safe before any sml_dyn_from_grid");
    }
    *safe = sml_dyn_is_safe(mm);
    // an exit that gave up on this check took the window as unsafe (it did so before the
    // check completed, so the word is final here).  The word holds the counter target of
    // the check the exit gave up on (4 * its number): a late exit of an earlier window,
    // not yet reported through sml::dyn_check_late, does not make this one unsafe
    if (d->d_chk_late && d->chk_counted &&
        __atomic_load_n(d->d_chk_late, __ATOMIC_ACQUIRE) == 4u * d->chk_count)
        *safe = 0;
    if (minmax) std::memcpy(minmax, mm, sizeof mm);
    return SML_OK;
}

// the next run_model's entry specx waits in-kernel until *flag >= value; on a timeout
// (ticks) it marks *late and transforms NaN (the window's check then fails)
int sml::dyn_run_model_wait(sml_dynamics *d, const uint64_t *flag, uint64_t value, unsigned *late,
                            long long timeout) {
    SML_REQUIRE(d && flag && late, "null argument");
    d->entry_wait = HopWait{flag, value, late};
    d->entry_wait.timeout = timeout;
    return SML_OK;
}

int sml::dyn_set_check_timeout(sml_dynamics *d, long long timeout) {
    SML_REQUIRE(d && timeout >= 0, "bad argument");
    d->chk_timeout = timeout;
    return SML_OK;
}

extern "C" int sml_dyn_set_check_timeout(sml_dynamics *d, int64_t microseconds) {
    SML_REQUIRE(d && microseconds >= 0, "bad argument");
    if (d->chk_stream) SML_HIP(hipStreamSynchronize(d->chk_stream));
    return sml::dyn_set_check_timeout(d, (long long)std::min<int64_t>(microseconds, INT64_MAX / 100) * 100);
}

extern "C" int sml_dyn_set_fused(sml_dynamics *d, int fused) {
    SML_REQUIRE(d, "null context");
    d->fused = fused != 0;
    return SML_OK;
}

extern "C" int sml_dyn_check_stream(const sml_dynamics *d, void **stream) {
    SML_REQUIRE(d && stream, "null argument");
    *stream = d->chk_stream;
    return SML_OK;
}

// the event behind the last safety check issued on the check stream (null if none)
int sml::dyn_check_event(sml_dynamics *d, void **ev) {
    SML_REQUIRE(d && ev, "null argument");
    *ev = d->chk_stream ? (void *)d->ev_chk : nullptr;
    return SML_OK;
}

// the next run_model's entry kernel (iogrid(30)'s specx) adds *adds to *counter as it
// starts: its input grid is complete and released by then
int sml::dyn_run_model_entry_signal(sml_dynamics *d, uint64_t *counter, int *adds) {
    SML_REQUIRE(d && counter && adds, "null argument");
    d->entry_sig = counter;
    *adds = spectral_specx_io_blocks();
    return SML_OK;
}

// the next run_model's exit is followed (on its stream, inside the window graph when the
// exit is captured there) by a one-lane store of value to *flag; flag = NULL withdraws it
int sml::dyn_run_model_exit_store(sml_dynamics *d, uint64_t *flag, uint64_t value) {
    SML_REQUIRE(d, "null argument");
    d->exit_store = flag;
    d->exit_store_value = value;
    return SML_OK;
}

// a run_model exit that gave up waiting for its safety check (it then took the window
// as unsafe): reported once, then reset.  The word is host memory: no copy, no sync --
// callers read it once the exit has run (sml_hybrid_run_speedy, after the check's event)
int sml::dyn_check_late(sml_dynamics *d) {
    if (!d || !d->d_chk_late) return SML_OK;
    if (__atomic_load_n(d->d_chk_late, __ATOMIC_ACQUIRE)) {
        __atomic_store_n(d->d_chk_late, 0u, __ATOMIC_RELEASE);
        return fail(SML_ERR_STATE, "run_model's exit did not receive its safety check in time (window taken as unsafe)");
    }
    return SML_OK;
}

extern "C" int sml_dyn_from_grid_host(sml_dynamics *d, const double *grid4d, const double *logp, double *minmax,
                                      int *safe) {
    SML_REQUIRE(d && grid4d && logp, "null argument");
    const size_t n4 = (size_t)4 * kKX * kGF;
    SML_HIP(hipMemcpy(d->d_io, grid4d, n4 * 8, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(d->d_io + n4, logp, kGF * 8, hipMemcpyHostToDevice));
    if (int rc = sml_dyn_from_grid(d, d->d_io, d->d_io + n4, d->d_minmax, nullptr)) return rc;
    double mm[8];
    SML_HIP(hipMemcpy(mm, d->d_minmax, sizeof mm, hipMemcpyDeviceToHost));
    if (minmax) std::memcpy(minmax, mm, sizeof mm);
    if (safe) *safe = sml_dyn_is_safe(mm);
    return SML_OK;
}

extern "C" int sml_dyn_to_grid_host(sml_dynamics *d, double *grid4d, double *logp) {
    SML_REQUIRE(d && grid4d && logp, "null argument");
    const size_t n4 = (size_t)4 * kKX * kGF;
    if (int rc = sml_dyn_to_grid(d, d->d_io, d->d_io + n4, nullptr)) return rc;
    SML_HIP(hipMemcpy(grid4d, d->d_io, n4 * 8, hipMemcpyDeviceToHost));
    SML_HIP(hipMemcpy(logp, d->d_io + n4, kGF * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_dyn_step_host(sml_dynamics *d, int j1, int j2, double dt, double alph, double rob, double wil,
                                 const double *phys) {
    SML_REQUIRE(d, "null context");
    const double *dp = nullptr;
    if (phys) {
        SML_REQUIRE(!d->phys_on, "physics runs on the GPU (sml_dyn_set_physics): phys must be NULL");
        SML_HIP(hipMemcpy(d->d_phys, phys, (size_t)4 * kKX * kGF * 8, hipMemcpyHostToDevice));
        dp = d->d_phys;
    }
    if (int rc = sml_dyn_step(d, j1, j2, dt, alph, rob, wil, dp, nullptr)) return rc;
    SML_HIP(hipDeviceSynchronize());
    return SML_OK;
}

// diagnostic: the phase stamps of the last fused launches ([4][96][8] wall_clock64
// ticks, 100 MHz); not part of the ABI header
#ifdef SML_PSTAMPS
// the physics sub-phase stamps of the last row kernel (profiling build only)
extern "C" int sml_dbg_pst(long long *out) {
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pst), sizeof(long long) * kIL * 32, 0, hipMemcpyDeviceToHost));
    return SML_OK;
}
#endif

extern "C" int sml_dbg_dyn_stamps(sml_dynamics *d, long long *out) {
    SML_REQUIRE(d && out && d->d_dbg, "stamps not enabled (SML_DYN_STAMPS=1 at creation)");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(out, d->d_dbg, kStampKernels * kStampBlocks * kStamps * sizeof(long long), hipMemcpyDeviceToHost));
    return SML_OK;
}

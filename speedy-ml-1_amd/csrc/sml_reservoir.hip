// sml_reservoir.hip -- batched reservoir forward (predict) for every region of a
// rank, plus the device-side exchange/tiling that replaces sendrecievegrid's
// gather / scatter loops.
//
// Reference: predict (src/mod_reservoir.f90:1416-1487), per region on the host:
//     y = A x                (MKL_SPARSE_D_MV, COO, :1442)
//     temp = W_in feedback   (dense n x ninp matmul, :1443)
//     x = (1-a) x + a tanh(y + temp)
//     x~ = x with every 2nd node squared (:1448-1449)
//     outvec = W_out [local_model; x~]  (:1454), then unstandardize (:1469)
//
// MI355X design (DESIGN.md "Reservoir"):
//   * all regions of the rank run in two launches (update + readout), no host loop;
//   * A is CSR (rows in the file's entry order, so every row sums in the same order
//     as the reference's COO traversal) with 16-bit column indices;
//   * W_in is CSR too: the trained matrix has one entry per row (train_reservoir,
//     :260-278), so the 26.5 MB dense matmul per region becomes n gathers;
//   * W_out is stored transposed ([nout][ld], rows padded to 16 B) in the file
//     precision (fp32 by default: NF90_REAL, mod_io.f90:1282, exact widening);
//     the readout streams it from HBM once per step with fp64 accumulation and
//     wave-level reductions -- this kernel carries ~90 % of the step's bytes;
//   * unstandardize is fused into the readout's epilogue.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <type_traits>
#include <vector>

#include "sml_internal.hpp"
#include "sml_timeline.hpp"

SML_TL_DEFINE(reservoir)

#ifndef SML_READ_NT
#define SML_READ_NT 1
#endif
#ifndef SML_UPD_NT
#define SML_UPD_NT 1
#endif

using namespace sml;

namespace {

constexpr int kLdAlign = 32;    // W_out / x_aug row stride multiple (columns)
constexpr int kRows = 8;        // W_out rows per wave in the readout (nout_pad's multiple)
constexpr int kRowsWide = 17;   // rows per wave when nout_pad = 17 w (w <= 8 waves)
constexpr int kWideWaves = 2;   // waves per readout block with kRowsWide rows (a region = w / 2 blocks;
                                // 2 / 4 / 8 waves measured: one-pass 0.638 / 0.644 / 0.696 ms)
constexpr int kMaxNcs = 256;     // local-model length bound of the fused finish (132 in T30L8)
constexpr int kMeanStd = 36;    // mean/std vector length (mod_reservoir.f90:1815-1846)
constexpr int kTisrStride = 16; // packed tisr input: [nlocal][16]
constexpr int kSrcKeep = -1;    // feedback entry left untouched (sst)

constexpr int kEllA = 8;  // ELL slots reserved per row for A (makesparse rows hold floor(k/n) or +1 <= 8)
constexpr int kEllW = 1;  // ELL slots per row for W_in (the trained W_in has one entry per row)

// A's ELL copy (r04b): a_w "main" slots per row, stored as slot pairs, pair-major
// ([pair][n] of (col, col) u16 pairs and of (val, val) pairs: lane i's row is one
// 4-B + one 8-B load per pair, coalesced across the wave), a_w chosen per region to
// move the fewest bytes.  makesparse rows hold floor(k/n) or floor(k/n) + 1 entries
// (mod_linalg.f90:180-218): with a_ov the rows holding a_w + 1 keep their last entry
// in an overflow list instead of padding every row to the longest -- a bit per row
// (u64 words) + a count per word locate it.  The dominant 4x4+sst region (n 6048,
// 4.8 % of rows one longer) moves 36.5 B of A per row instead of 48.
struct RegionDev {
    int n, ninp, ld;
    int a_w, w_w;  // A's ELL main width in slots (0 = use the CSR copy); W_in ELL (1) or CSR (0)
    int a_ov;      // 1: rows of a_w + 1 entries, the last in the overflow list
    int w_q;       // > 0: W_in's column of row i is i / w_q = umulhi(i, w_magic), not stored
    uint32_t w_magic;
    int64_t a_rp, a_nz, w_rp, w_nz, wout, x, xaug, fb;
    int64_t wlm;  // W_out(:, 1:ncs) transposed, [ncs][nout_pad], in the W_out pool after the row-major blocks
    int64_t a_ell, w_ell;  // offsets into the ELL pools (A: pair-major as above; W_in: [n])
    int64_t a_om;          // overflow bit words / per-word counts: [ceil(n / 64)] each
    int64_t a_oe;          // overflow entries (col, val) in row order: [n] reserved
};

}  // namespace

struct sml_reservoirs {
    int numregions = 0, nlocal = 0, ncs = 0, nout = 0, nout_pad = 0, wdtype = SML_F32;
    // row stride of the outvec arrays (sml_res_set_outvec_ld): nout, or wider when the
    // hybrid loop carries the slab ocean's sst beside each outvec in its exchange rows
    int ov_ld = 0;
    double leakage = 1.0;
    std::vector<int> region_ids, n, k, ninp, ld;
    std::vector<unsigned char> sst, loaded;
    std::vector<RegionGeom> geom;
    std::vector<RegionDev> rd;
    int64_t tot_wlm = 0;  // elements of the transposed local-model blocks (pool d_wlm)
    void *d_wlm = nullptr;
    int64_t tot_a_rp = 0, tot_a_nz = 0, tot_w_rp = 0, tot_w_nz = 0, tot_wout = 0, tot_xaug = 0,
            tot_fb = 0;
    std::vector<int64_t> w_nz_cap;  // reserved W_in CSR nnz per region (n at create: one entry per row as
                                    // trained; grow_win_pool re-lays the pool for a denser W_in)
    int maxn = 0, maxninp = 0;
    int device = 0;
    // device buffers
    RegionDev *d_rd = nullptr;
    int32_t *d_a_rp = nullptr, *d_w_rp = nullptr;
    uint16_t *d_a_col = nullptr, *d_w_col = nullptr;
    void *d_a_val = nullptr, *d_w_val = nullptr, *d_wout = nullptr;
    // ELL copies (row-major per region), used when rows are short enough
    std::vector<int> a_ell_cap, w_ell_cap;  // slots per row reserved per region
    int64_t tot_a_ell = 0, tot_w_ell = 0, tot_a_om = 0, tot_a_oe = 0;
    uint16_t *d_a_ell_col = nullptr, *d_w_ell_col = nullptr;
    void *d_a_ell_val = nullptr, *d_w_ell_val = nullptr;
    uint64_t *d_a_om = nullptr;   // A's overflow bits, one word per 64 rows
    uint32_t *d_a_ob = nullptr;   // overflow entries before each word (region-local)
    uint16_t *d_a_oc = nullptr;   // overflow entries: column
    void *d_a_ov = nullptr;       //                   value
    void *d_zero = nullptr;       // 256 zero bytes: the target of the balanced update's unused loads
    bool no_ell = false;          // CSR copies only (sml_res_set_reference_paths)
    double *d_x[2] = {nullptr, nullptr};
    int cur = 0;
    double *d_meanstd = nullptr;
    double *d_part = nullptr;       // [nlocal][nout_pad] W_out(:, ncs+1:) x~ of the step in flight
    // cap on the waves of the v_ml readout (the half that runs beside SPEEDY's window;
    // 0: one wave per item).  Sharing CUs with SPEEDY, uncapped it takes ~6 TB/s and
    // SPEEDY's latency-bound kernels stall behind it; paced at 2048 waves (~4.7 TB/s)
    // the overlapped step is 1.75 ms instead of 1.98 (profiles/r01p).  On CUs of its
    // own the pacing does not matter: sml_res_set_read_waves(0).
    int read_waves = 2048;
    // sml_res_step_begin's form (sml_res_set_begin_mode): 0 the update grid then the
    // v_ml readout grid, 1 one fused launch (k_res_begin, 2 blocks per CU), 2 fused with
    // the readout's loads unrolled twice (1 block per CU)
    int begin_mode = 0;
    // the balanced update (k_res_update_bal; k_res_update per region where the layout
    // does not fit it, or forced by sml_res_set_reference_paths):
    // row0 [nlocal+1] = the regions' rows concatenated; blk_r0 [grid] = the region each
    // block's share starts in, for the grid it was built for (upd_grid: the CUs the
    // launches get, sml_res_set_update_cus; 0 = every CU of the device)
    bool upd_bal = true;
    // the v_p finish one thread per output (vp_sum) instead of in column groups: the
    // fallback when ncs does not fit the groups, or forced (sml_res_set_reference_paths)
    bool finish_ungrouped = false;
    // the next grid finish waits in-kernel for *fin_wflag >= fin_wval (sml::res_finish_wait)
    const uint64_t *fin_wflag = nullptr;
    uint64_t fin_wval = 0;
    unsigned *fin_wlate = nullptr;
    long long fin_wtimeout = 400000000ll;  // wall_clock64 ticks
    int upd_cus = 0, ncu = 0;
    // the balanced update's per-block first regions, one table per grid size G (a paced
    // begin and an uncapped step alternate two sizes): tables in one device buffer at
    // offset G (G - 1) / 2, built once per G; blk_off[G] = -1 until then
    std::vector<int32_t> blk_off;
    std::vector<std::vector<int32_t>> blk_host;  // the host tables (async copies' sources stay alive)
    int blk_cap = 0;  // largest G the buffer holds
    size_t max_lds = 0;  // the device's LDS per workgroup (hipDeviceAttributeMaxSharedMemoryPerBlock)
    int ell_ok = -1;  // every local region's A and W_in in ELL form (-1: recount after a load)
    int32_t *d_row0 = nullptr, *d_blk_r0 = nullptr;
    std::vector<int32_t> row0_h;
    bool begun = false;             // sml_res_step_begin issued, finish pending
    int8_t *d_outl = nullptr;
    int32_t *d_asm_dst = nullptr;   // [numregions*nout] -> concatenated grid index
    int32_t *d_fb_src = nullptr;    // [tot_fb]
    uint8_t *d_fb_l = nullptr;      // [tot_fb]
    uint16_t *d_fb_reg = nullptr;   // [tot_fb]
    // tisr entries of the feedback (get_tisr_by_date, mpires.f90:1644-1676): feedback
    // index, grid2d index of the overlap-tile point, local region
    int tot_tisr = 0;
    int32_t *d_tisr_fb = nullptr, *d_tisr_grid = nullptr;
    uint16_t *d_tisr_reg = nullptr;
    int32_t *d_lm_src = nullptr;    // [nlocal*ncs]
    uint8_t *d_lm_l = nullptr;
    double *d_io = nullptr;         // staging for sml_res_step_host
    size_t d_io_n = 0;
    std::vector<hipEvent_t> ev;     // 3 events per timed step (start, update done, readout done)
    int ev_cap = 0, ev_used = 0;
    bool timing = false;
    std::vector<double> meanstd_h;  // host copy [nlocal][72]
    // generic context (sml_res_create_generic: the slab-ocean reservoir): ninp given,
    // no exchange tables, every output unstandardized with the mean / std slot out_l[o]
    bool generic = false;
    std::vector<int8_t> out_l;
};

namespace {

// ------------------------------------------------------------------ kernels
// XCD-contiguous remap of a 1-D grid: consecutive hardware blocks are dealt
// round-robin to the 8 XCDs (MI355X_MICROARCH.md, workgroup dispatch); this
// bijection gives each XCD one contiguous range of logical blocks, so all blocks
// of a region share one L2 (speed only, never correctness).
__device__ inline int xcd_remap(int b, int nb) {
    const int q8 = nb / 8, rem = nb % 8, xcd = b % 8, idx = b / 8;
    return xcd * q8 + min(xcd, rem) + idx;
}

constexpr int kUpdThreads = 1024;  // threads per update block (one row per thread per pass)

struct Ell {
    const uint16_t *a_col;
    const void *a_val;
    const uint16_t *w_col;
    const void *w_val;
    const uint64_t *a_om;  // A's overflow bits / counts / entries (RegionDev::a_ov)
    const uint32_t *a_ob;
    const uint16_t *a_oc;
    const void *a_ov;
    const void *zero;  // 256 zero bytes
};

// Row loads of one pass, issued ahead of their use (software pipelining): A's main
// slots as up to 4 (col, col) / (val, val) pairs, W_in's entry, and -- for a region
// with an overflow list -- the row's overflow word and count, then (resolve_ovf, one
// stage later) its overflow entry.
template <typename WT>
struct RowRegs {
    uint32_t c[kEllA / 2];
    WT v[kEllA];
    uint32_t wc;
    WT wv;
    uint64_t om;
    uint32_t ob;
    uint32_t oc;
    WT ov;
    bool oh;
};

// A and W_in are streamed once per step: non-temporal loads (SML_UPD_NT), like the
// readout's W_out, so they do not evict the data of the SPEEDY window running beside
template <typename T>
__device__ inline T stream_load(const T *p) {
#if SML_UPD_NT
    return __builtin_nontemporal_load(p);
#else
    return *p;
#endif
}

template <typename WT>
struct Pair;
template <>
struct Pair<float> {
    typedef float N __attribute__((ext_vector_type(2)));
};
template <>
struct Pair<double> {
    typedef double N __attribute__((ext_vector_type(2)));
};

// pair p of row i (slots 2p, 2p + 1) from the pair-major ELL copy
template <typename WT>
__device__ inline void load_pair(RowRegs<WT> &q, int p, const uint32_t *cp, const WT *vp) {
    typedef typename Pair<WT>::N V2;
    q.c[p] = stream_load(cp);
    const V2 v = stream_load(reinterpret_cast<const V2 *>(vp));
    q.v[2 * p] = v.x;
    q.v[2 * p + 1] = v.y;
}

__device__ inline uint32_t win_col_implicit(const RegionDev &rg, int i) {
    return __umulhi((uint32_t)i, rg.w_magic);  // = i / w_q for every i < n (checked at load)
}

// every load of row i, branching on the region's widths (k_res_update, k_res_begin)
template <typename WT>
__device__ inline void load_row(RowRegs<WT> &q, const RegionDev &rg, const Ell &ell, int i, bool live) {
    if (live && rg.a_w > 0) {
        const uint32_t *cb = reinterpret_cast<const uint32_t *>(ell.a_col + rg.a_ell);
        const WT *vb = (const WT *)ell.a_val + rg.a_ell;
        const int np = (rg.a_w + 1) >> 1, n = rg.n;
#pragma unroll
        for (int p = 0; p < kEllA / 2; ++p)
            if (p < np) load_pair(q, p, cb + (size_t)p * n + i, vb + 2 * ((size_t)p * n + i));
        if (rg.a_ov) {
            q.om = stream_load(ell.a_om + rg.a_om + (i >> 6));
            q.ob = stream_load(ell.a_ob + rg.a_om + (i >> 6));
        }
    }
    if (live && rg.w_w > 0) {
        q.wc = rg.w_q > 0 ? win_col_implicit(rg, i) : (uint32_t)stream_load(ell.w_col + rg.w_ell + i);
        q.wv = stream_load((const WT *)ell.w_val + rg.w_ell + i);
    }
}

// the same loads for the balanced update: NP pairs from every region (pairs past a
// narrower region's own load the zero bytes, so the pair loads carry no branch); the
// overflow word / count and the stored W_in column only where the region has them --
// a branch uniform across the pass (a pass never straddles regions)
template <typename WT, int NP, bool OVF>
__device__ inline void load_row_fixed(RowRegs<WT> &q, const RegionDev &rg, const Ell &ell, int i) {
    const uint32_t *cb = reinterpret_cast<const uint32_t *>(ell.a_col + rg.a_ell);
    const WT *vb = (const WT *)ell.a_val + rg.a_ell;
    const uint32_t *zc = reinterpret_cast<const uint32_t *>(ell.zero);
    const WT *zv = reinterpret_cast<const WT *>(ell.zero);
    const int np = (rg.a_w + 1) >> 1, n = rg.n;
    if (OVF) {
        q.om = 0;
        q.ob = 0;
        if (rg.a_ov) {
            q.om = stream_load(ell.a_om + rg.a_om + (i >> 6));
            q.ob = stream_load(ell.a_ob + rg.a_om + (i >> 6));
        }
    }
#pragma unroll
    for (int p = 0; p < NP; ++p) {
        const bool in = p < np;
        load_pair(q, p, in ? cb + (size_t)p * n + i : zc, in ? vb + 2 * ((size_t)p * n + i) : zv);
    }
    if (rg.w_q > 0)
        q.wc = win_col_implicit(rg, i);
    else
        q.wc = stream_load(ell.w_col + rg.w_ell + i);
    q.wv = stream_load((const WT *)ell.w_val + rg.w_ell + i);
}

// row i's overflow entry, if any: its bit in the word, its index = the word's count +
// the bits below it (kFixed: the balanced update's streaming loads)
template <typename WT, bool kFixed>
__device__ inline void resolve_ovf(RowRegs<WT> &q, const RegionDev &rg, const Ell &ell, int i) {
    const int b = i & 63;
    const uint64_t below = b ? q.om << (64 - b) : 0ull;  // the bits of rows i - b .. i - 1
    q.oh = rg.a_ov && ((q.om >> b) & 1ull);
    const int64_t e = rg.a_oe + q.ob + __popcll(below);
    if (q.oh) {  // (the lanes of the rows one longer: 5-16 % of them where a region has any)
        q.oc = kFixed ? stream_load(ell.a_oc + e) : ell.a_oc[e];
        q.ov = kFixed ? stream_load((const WT *)ell.a_ov + e) : ((const WT *)ell.a_ov)[e];
    }
}

// the reservoir's activation, tanh (mod_reservoir.f90:1447).  OCML's tanh(double) is
// ~150 f64 instructions (a double-double exp and a compensated division): in the
// state update that is more VALU time per row than the row's bytes take to stream
// at 8 TB/s.  tanh(x) = em / (em + 2), em = expm1(2|x|), sign restored: expm1 keeps
// small |x| exact to an ulp (no 1 - 2 / (e + 1) cancellation), the division rounds
// once; |x| > 20 gives 1 (tanh(20) = 1 - 8.5e-18 rounds to 1).  Within 3 ulp of
// glibc's tanh (the oracle's; tests bound states at 1e-14), NaN and -0 preserved.
// Every state update form uses it, so they stay bitwise equal to each other.
__device__ __attribute__((always_inline)) inline double res_tanh(double x) {
    double a = fabs(x);
    a = a > 20.0 ? 20.0 : a;  // (NaN stays NaN)
    const double em = expm1(2.0 * a);
    return copysign(em / (em + 2.0), x);
}

template <typename WT>
__device__ inline int ell_col(const RowRegs<WT> &q, int s) {
    return (int)((q.c[s >> 1] >> (16 * (s & 1))) & 0xffffu);
}

// x_new(i) from the row's loads: y = A x over the main slots in order, then the
// overflow entry (the row's file order: makesparse's blocks, CSR-stable), temp =
// W_in u, tanh, leak -- one expression for every ELL form of the update
template <typename WT>
__device__ __attribute__((always_inline)) inline double ell_row_value(const RowRegs<WT> &q, const RegionDev &rg,
                                                                      const double *xs, const double *fs, int i,
                                                                      double leak) {
    double y = 0.0;
#pragma unroll
    for (int s = 0; s < kEllA; ++s)
        if (s < rg.a_w) y = y + (double)q.v[s] * xs[ell_col(q, s)];
    if (q.oh) y = y + (double)q.ov * xs[q.oc];
    double t = 0.0;
    t = t + (double)q.wv * fs[q.wc];
    const double xn = res_tanh(y + t);
    return (1.0 - leak) * xs[i] + leak * xn;
}

// update: logical block = (region, part); a part is a contiguous range of rows
// walked in passes of 1024 rows.  With kLds the region's state x and feedback u
// are staged once per block in LDS and the SpMV's random column gathers hit LDS
// instead of the L2 (one L2 transaction per gathered double otherwise).  A and
// W_in are read in ELL form when the region's rows are short (pair-major, RegionDev;
// padding slots hold 0 * x[0] after the row's real entries, so the file-order sum
// is unchanged), otherwise from the CSR copy.  The next pass's ELL loads are issued
// before the current pass computes (the overflow entry, when the region has a list,
// is fetched when the row is computed: this form is not the one the loop runs).
template <typename WT, bool kLds, int kThr = kUpdThreads>
__device__ __attribute__((always_inline)) inline void update_block(
    int lb, double *smem, const RegionDev *__restrict__ R, const int32_t *__restrict__ a_rp,
    const uint16_t *__restrict__ a_col, const WT *__restrict__ a_val, const int32_t *__restrict__ w_rp,
    const uint16_t *__restrict__ w_col, const WT *__restrict__ w_val, const Ell &ell,
    const double *__restrict__ x_old, double *__restrict__ x_new,
    const double *__restrict__ feedback, double leak, int parts, int lds_x) {
    const int r = lb / parts, part = lb % parts;
    const RegionDev rg = R[r];
    const int n = rg.n, tid = threadIdx.x;
    const int per = (n + parts - 1) / parts;
    const int beg = part * per, end = min(n, beg + per);
    if (beg >= end) return;  // block-uniform
    RowRegs<WT> cur, nxt;
    load_row(cur, rg, ell, beg + tid, beg + tid < end);
    const double *xo = x_old + rg.x;
    const double *fb = feedback + rg.fb;
    const double *xs = xo, *fs = fb;
    if (kLds) {
        double *sx = smem, *sf = smem + lds_x;
        for (int j = tid; j < n; j += kThr) sx[j] = xo[j];
        for (int j = tid; j < rg.ninp; j += kThr) sf[j] = fb[j];
        __syncthreads();
        xs = sx;
        fs = sf;
    }
    const int32_t *rp = a_rp + rg.a_rp;
    const uint16_t *ac = a_col + rg.a_nz;
    const WT *av = a_val + rg.a_nz;
    const int32_t *wp = w_rp + rg.w_rp;
    const uint16_t *wc = w_col + rg.w_nz;
    const WT *wv = w_val + rg.w_nz;
    for (int base = beg; base < end; base += kThr) {
        const int i = base + tid;
        const bool live = i < end;
        const int inext = i + kThr;
        if (base + kThr < end) load_row(nxt, rg, ell, inext, inext < end);
        if (live) {
            // y = A x, entries of row i in the file's order (COO semantics, duplicates add)
            double y = 0.0;
            if (rg.a_w > 0) {
                cur.oh = false;
                if (rg.a_ov) resolve_ovf<WT, false>(cur, rg, ell, i);
#pragma unroll
                for (int s = 0; s < kEllA; ++s)
                    if (s < rg.a_w) y = y + (double)cur.v[s] * xs[ell_col(cur, s)];
                if (cur.oh) y = y + (double)cur.ov * xs[cur.oc];  // the row's last entry (ell_row_value)
            } else {
                for (int e = rp[i], e1 = rp[i + 1]; e < e1; ++e) y = y + (double)av[e] * xs[ac[e]];
            }
            // temp = W_in feedback
            double t = 0.0;
            if (rg.w_w > 0) {
                t = t + (double)cur.wv * fs[cur.wc];
            } else {
                for (int e = wp[i], e1 = wp[i + 1]; e < e1; ++e) t = t + (double)wv[e] * fs[wc[e]];
            }
            const double xn = res_tanh(y + t);
            const double xv = (1.0 - leak) * xs[i] + leak * xn;
            x_new[rg.x + i] = xv;  // (x~ = x with x(2:n:2)**2: squared by the readout's loads, rd_x)
        }
        cur = nxt;
    }
}

// logical blocks (region, part) = nlog; with a grid smaller than nlog (the paced
// update that runs beside SPEEDY's window) each block takes logical blocks in rounds
// kMinW: waves per SIMD the registers must allow (4: one 1024-thread block per CU; 8:
// two, so one block's x staging and SpMV overlap the other's -- 64 VGPRs)
template <typename WT, bool kLds, int kMinW = 4>
__global__ __launch_bounds__(kUpdThreads, kMinW) void k_res_update(
    const RegionDev *__restrict__ R, const int32_t *__restrict__ a_rp, const uint16_t *__restrict__ a_col,
    const WT *__restrict__ a_val, const int32_t *__restrict__ w_rp, const uint16_t *__restrict__ w_col,
    const WT *__restrict__ w_val, Ell ell, const double *__restrict__ x_old, double *__restrict__ x_new,
    const double *__restrict__ feedback, double leak, int parts, int lds_x, int nlog) {
    SML_TL_SCOPE(sml::tl::kUpdate);
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int off = xcd_remap(blockIdx.x, gridDim.x);
    for (int base = 0; base < nlog; base += gridDim.x) {
        const int lb = base + off;
        if (lb < nlog)  // block-uniform
            update_block<WT, kLds>(lb, smem, R, a_rp, a_col, a_val, w_rp, w_col, w_val, ell, x_old, x_new,
                                   feedback, leak, parts, lds_x);
        if (base + (int)gridDim.x < nlog) __syncthreads();  // the block's LDS, reused next round
    }
}

// ---------------------------------------------------------------- balanced update
// k_res_update_bal: the same rows, the same arithmetic (bitwise k_res_update's ELL
// path), laid out for HBM instead of per region.  k_res_update runs a block per
// (region, part): at 1152 regions on 256 CUs (one 1024-thread block per CU: 71 VGPRs)
// that is 4.5 rounds of blocks -- the fifth a half-empty tail -- each block staging
// its region's x in LDS behind a barrier and then keeping one pass of A rows in
// flight (55 KB per CU: ~0.5 of 8 TB/s at the loaded latency).
// Here a persistent grid of one block per CU takes a contiguous, equal share of all
// the rank's rows (the regions concatenated; r0 of each block from a host table), so
// no block waits on a tail; a pass never straddles regions (a share is a run of
// segments, one per region it touches); the A / W_in rows of the next TWO passes are
// in flight while a pass computes (~110 KB per CU), whatever segment they belong to;
// and the next segment's x / feedback are loaded while the current segment's last
// pass computes and stored into the second of two LDS buffers, so a segment switch
// costs one barrier, not a memory round trip.  Needs every region in ELL form, n <=
// kStageX * 1024, ninp <= 1024 and two buffers in LDS; else k_res_update runs.
constexpr int kStageX = 7;

struct PassDesc {
    int r, base, end, seg;
    bool live;
};

struct StageRegs {
    double x[kStageX];
    double f;
};

template <typename WT, int NP, bool OVF, int kDepth = 2>
__global__ __launch_bounds__(kUpdThreads, 4) void k_res_update_bal(
    const RegionDev *__restrict__ R, const int32_t *__restrict__ row0, const int32_t *__restrict__ blk_r0, int nlocal,
    int64_t total, Ell ell, const double *__restrict__ x_old, double *__restrict__ x_new,
    const double *__restrict__ feedback, double leak, int lds_x, int lds_buf) {
    SML_TL_SCOPE(sml::tl::kUpdate);
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int G = gridDim.x;
    const int b = xcd_remap(blockIdx.x, G);
    const int g0 = (int)(total * b / G), g1 = (int)(total * (b + 1) / G);
    if (g0 >= g1) return;  // block-uniform
    const int tid = threadIdx.x;
    auto seg_at = [&](int r, int seg) -> PassDesc {
        const int a = row0[r], e = row0[r + 1];
        return PassDesc{r, max(g0, a) - a, min(g1, e) - a, seg, true};
    };
    auto succ = [&](const PassDesc &p) -> PassDesc {
        if (!p.live) return p;
        if (p.base + kUpdThreads < p.end) return PassDesc{p.r, p.base + kUpdThreads, p.end, p.seg, true};
        const int r = p.r + 1;
        if (r >= nlocal || row0[r] >= g1) return PassDesc{r, 0, 0, p.seg + 1, false};
        return seg_at(r, p.seg + 1);
    };
    // a lane past its segment's end loads row 0's data (in range, never used): the
    // same loads in every lane and every pass
    auto load = [&](RowRegs<WT> &q, const PassDesc &p) {
        if (!p.live) return;
        const RegionDev rg = R[p.r];
        const int i = p.base + tid;
        load_row_fixed<WT, NP, OVF>(q, rg, ell, i < p.end ? i : 0);
    };
    auto resolve = [&](RowRegs<WT> &q, const PassDesc &p) {
        q.oh = false;
        if (!OVF || !p.live) return;
        const RegionDev rg = R[p.r];
        if (!rg.a_ov) return;  // pass-uniform
        const int i = p.base + tid;
        resolve_ovf<WT, true>(q, rg, ell, i < p.end ? i : 0);
    };
    auto stage_load = [&](StageRegs &sr, int r) {
        const RegionDev rg = R[r];
        const double *xo = x_old + rg.x;
#pragma unroll
        for (int q = 0; q < kStageX; ++q) {
            const int j = tid + q * kUpdThreads;
            if (j < rg.n) sr.x[q] = xo[j];
        }
        if (tid < rg.ninp) sr.f = feedback[rg.fb + tid];
    };
    auto stage_store = [&](const StageRegs &sr, int r, double *buf) {
        const RegionDev rg = R[r];
#pragma unroll
        for (int q = 0; q < kStageX; ++q) {
            const int j = tid + q * kUpdThreads;
            if (j < rg.n) buf[j] = sr.x[q];
        }
        if (tid < rg.ninp) buf[lds_x + tid] = sr.f;
    };
    // kDepth passes in flight while one computes: L1 .. L{kDepth} (P1 .. P{kDepth})
    static_assert(kDepth == 2 || kDepth == 3, "update pipeline depth");
    PassDesc P0 = seg_at(blk_r0[b], 0);
    RowRegs<WT> L0, L1, L2, L3;
    load(L0, P0);
    resolve(L0, P0);
    PassDesc P1 = succ(P0);
    load(L1, P1);
    PassDesc P2 = succ(P1), P3 = P2;
    if constexpr (kDepth == 3) {
        load(L2, P2);
        P3 = succ(P2);
    }
    {
        StageRegs sr;
        stage_load(sr, P0.r);
        stage_store(sr, P0.r, smem);
    }
    __syncthreads();
    while (P0.live) {  // block-uniform
        // P1's overflow entries before the next pass's loads: compute(P1) then waits for
        // nothing issued after them (the in-order vmcnt), so kDepth passes stay in flight
        resolve(L1, P1);
        if constexpr (kDepth == 3)
            load(L3, P3);
        else
            load(L2, P2);
        const bool newseg = P1.live && P1.seg != P0.seg;
        StageRegs sr;
        if (newseg) stage_load(sr, P1.r);
        {  // the pass: update_block's ELL row, expression for expression
            const RegionDev rg = R[P0.r];
            const double *xs = smem + (size_t)(P0.seg & 1) * lds_buf, *fs = xs + lds_x;
            const int i = P0.base + tid;
            if (i < P0.end) x_new[rg.x + i] = ell_row_value(L0, rg, xs, fs, i, leak);
        }
        if (newseg) {  // the other buffer: its last reader (segment P0.seg - 1) finished before the last barrier
            stage_store(sr, P1.r, smem + (size_t)(P1.seg & 1) * lds_buf);
            __syncthreads();
        }
        P0 = P1;
        L0 = L1;
        P1 = P2;
        L1 = L2;
        if constexpr (kDepth == 3) {
            P2 = P3;
            L2 = L3;
            P3 = succ(P3);
        } else {
            P2 = succ(P2);
        }
    }
}

template <typename WT>
struct Vec4;
template <>
struct Vec4<float> {
    typedef float4 T;
    typedef float N __attribute__((ext_vector_type(4)));  // native vector (non-temporal loads)
};
template <>
struct Vec4<double> {
    typedef double4 T;
    typedef double N __attribute__((ext_vector_type(4)));
};

// readout: one wave per (region, 8-row group) item, 4 waves per block; blocks are
// remapped so that the items of one region stay on one XCD's L2 (x_aug reuse).
// The product W_out [local_model; x~] is split at column ncs as the reference's
// outvec_component_contribs does (v_p + v_ml, mod_reservoir.f90:1456-1459):
//   kReadML:     part = v_ml = W_out(:, ncs+1:) x~     (needs only this step's feedback)
//   kReadFinish: v = v_p + part, unstandardize (k_res_finish: one thread per output)
//   kReadFull:   v = v_p + v_ml in one pass (sml_res_step)
// v_ml is the wave's per-lane partial sums + butterfly over W_out's rows; v_p is a
// per-output sum over the ncs columns in order from the transposed block
// W_out(:, 1:ncs) = [ncs][nout_pad] (coalesced across outputs), the same code in
// both modes, so the split step and the one-pass step agree bit for bit; the split
// lets the ML part -- ~98 % of the bytes -- run before SPEEDY's local_model exists.
enum ReadMode { kReadML = 0, kReadFinish = 1, kReadFull = 2 };

// dot products of the wave's 8 W_out rows with x over columns [c0, c1) (16-B groups;
// lanes own columns c0 + 4 lane + 256 t), reduced across the wave; x values outside
// [x0, x1) are zero (fma(w, 0, s) == s), which matters only when ncs % 4 != 0
template <int R>
struct Rows {
    double v[R];
};

template <typename WT, int R, int kUnroll = 2, typename XF>
__device__ __attribute__((always_inline)) inline Rows<R> rows_dot(const WT *W, int ld, int lane, int c0, int c1,
                                                               XF xload) {
    typedef typename Vec4<WT>::N V;
    double acc[R];
#pragma unroll
    for (int q = 0; q < R; ++q) acc[q] = 0.0;
#pragma unroll kUnroll
    for (int j = c0 + lane * 4; j < c1; j += 256) {
        const double4 xv = xload(j);
        V w[R];
#pragma unroll
        for (int q = 0; q < R; ++q)  // streamed once per step: non-temporal, so W_out does not evict the
#if SML_READ_NT                          // window's data
            w[q] = __builtin_nontemporal_load(reinterpret_cast<const V *>(W + (size_t)q * ld + j));
#else
            w[q] = *reinterpret_cast<const V *>(W + (size_t)q * ld + j);
#endif
#pragma unroll
        for (int q = 0; q < R; ++q) {
            double s = acc[q];
            s = fma((double)w[q].x, xv.x, s);
            s = fma((double)w[q].y, xv.y, s);
            s = fma((double)w[q].z, xv.z, s);
            s = fma((double)w[q].w, xv.w, s);
            acc[q] = s;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
        for (int q = 0; q < R; ++q) acc[q] += __shfl_xor(acc[q], off, 64);
    Rows<R> out;
#pragma unroll
    for (int q = 0; q < R; ++q) out.v[q] = acc[q];
    return out;
}

// v_p = W_out(o, 1:ncs) local_model from the transposed block wl = [ncs][nout_pad] (a
// wave's lanes read neighbouring outputs of a column), summed in kFinGroups groups of
// consecutive columns -- each group a sequential fma chain from 0, the groups added in
// order -- so the finish can run the groups on different threads (k_res_finish_grid)
// and every other form (k_res_finish, the one-pass readout) gets the same bits
constexpr int kFinGroups = 7;
constexpr int kFinGsz = 19;  // the grouped finish's column-group bound (ncs 132: 6 x 19 + 18)
__device__ inline int fin_gsz(int ncs) { return (ncs + kFinGroups - 1) / kFinGroups; }

template <typename WT>
__device__ inline double vp_sum(const WT *__restrict__ wl, int nout_pad, const double *__restrict__ lm, int ncs,
                                int o) {
    // the kFinGroups chains advance together; each is still the sequential sum of its
    // own columns.  Every load of a round of kVpU columns per chain is issued before
    // the round's FMAs (indices past a chain's end clamped into the block, those FMAs
    // selected away): one memory round trip per round, not one per column
    constexpr int kVpU = 2;
    const int gsz = fin_gsz(ncs);
    double s[kFinGroups];
#pragma unroll
    for (int g = 0; g < kFinGroups; ++g) s[g] = 0.0;
    for (int jj0 = 0; jj0 < gsz; jj0 += kVpU) {
        double w[kVpU][kFinGroups], x[kVpU][kFinGroups];
#pragma unroll
        for (int u = 0; u < kVpU; ++u)
#pragma unroll
            for (int g = 0; g < kFinGroups; ++g) {
                const int jc = min(g * gsz + jj0 + u, ncs - 1);
                w[u][g] = (double)wl[(size_t)jc * nout_pad + o];
                x[u][g] = lm[jc];
            }
#pragma unroll
        for (int u = 0; u < kVpU; ++u)
#pragma unroll
            for (int g = 0; g < kFinGroups; ++g) {
                const int jj = jj0 + u, j = g * gsz + jj;
                const double t = fma(w[u][g], x[u][g], s[g]);
                s[g] = (jj < gsz && j < ncs) ? t : s[g];
            }
    }
    double v = s[0];
#pragma unroll
    for (int g = 1; g < kFinGroups; ++g) v = v + s[g];
    return v;
}

// unstandardize_state_vec_res: x*std + mean (two roundings) where the output has a slot
__device__ inline double unstd(double v, const double *ms, int l) {
    if (l >= 0) {
        const double t = v * ms[kMeanStd + l];
        v = t + ms[l];
    }
    return v;
}

// x~ over the columns j .. j + 3 of a region's ld-wide row (xr: the row's start; the
// state x sits from column ncs on): x_aug = [local_model; x~], x~ = x with its 1-based
// even entries squared (x_temp(2:n:2)**2, mod_reservoir.f90:1452-1455), the columns
// below ncs zero.  The squares are formed here, where x~ is consumed, instead of in a
// copy written by the update (the same multiply, so the same bits)
__device__ __attribute__((always_inline)) inline double4 rd_x(const double *xr, int j, int ncs) {
    double4 v = *reinterpret_cast<const double4 *>(xr + j);
    auto f = [&](double x, int c) {
        const int i = j + c - ncs;  // 0-based state index
        return i < 0 ? 0.0 : (i & 1) ? x * x : x;
    };
    return double4{f(v.x, 0), f(v.y, 1), f(v.z, 2), f(v.w, 3)};
}

template <typename WT, int kMode, int NR>
__global__ __launch_bounds__(512) void k_res_readout(const RegionDev *__restrict__ R, const WT *__restrict__ wout,
                                                     const WT *__restrict__ wlm,
                                                     const double *__restrict__ xst,
                                                     const double *__restrict__ local_model,
                                                     const double *__restrict__ meanstd,
                                                     const int8_t *__restrict__ outl, double *__restrict__ part,
                                                     double *__restrict__ outvec, int nout, int ov_ld, int nout_pad,
                                                     int ncs, int groups, int nitems, int ipw) {
    SML_TL_SCOPE(sml::tl::kReadout);
    // wave gw takes the items gw, gw + W, gw + 2W, .. (W waves; one item each unless
    // the launch is paced): the waves in flight together work on consecutive items.
    // NR = kRowsWide (17 rows a wave, 8 waves a region of 136 outputs): x_aug is read
    // 8 times per region instead of 17, the waves of a block together; NR = kRows:
    // 17 waves per region.  Either way a region's blocks are neighbours, kept on one
    // XCD's L2 by the remap
    const int bs = xcd_remap(blockIdx.x, gridDim.x);
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    const int gw = bs * wpb + (threadIdx.x >> 6), nw = gridDim.x * wpb;
    (void)ipw;
    for (int item = gw; item < nitems; item += nw) {
        const int r = item / groups, g = item % groups;
        const RegionDev rg = R[r];
        const int ld = rg.ld;
        const WT *W = wout + rg.wout + (size_t)(g * NR) * ld;
        Rows<NR> ml{};
        {   // v_ml: x~ from the state, columns ncs .. ld (zero below ncs from the aligned start)
            const double *xa = xst + rg.xaug;
            ml = rows_dot<WT, NR>(W, ld, lane, ncs & ~(kLdAlign - 1), ld, [=](int j) { return rd_x(xa, j, ncs); });
        }
        const int o0 = g * NR;
        if (kMode == kReadML) {  // every lane holds all 8 sums after the butterfly; lane 0 writes them
            if (lane == 0) {
    #pragma unroll
                for (int q = 0; q < NR; ++q) part[(size_t)r * nout_pad + o0 + q] = ml.v[q];
            }
        } else {  // kReadFull: lane q finishes row o0 + q with v_p (k_res_finish's sum) + v_ml
            const int o = o0 + lane;
            if (lane < NR && o < nout) {
                double vml = ml.v[0];  // static indices only: a lane-indexed pick would put the sums in scratch
    #pragma unroll
                for (int q = 1; q < NR; ++q)
                    if (lane == q) vml = ml.v[q];
                const double vp = vp_sum(wlm + rg.wlm, nout_pad, local_model + (size_t)r * ncs, ncs, o);
                outvec[(size_t)r * ov_ld + o] = unstd(vp + vml, meanstd + (size_t)r * 2 * kMeanStd, outl[o]);
            }
        }
    }
}

// sml_res_step_begin's two launches (k_res_update, then k_res_readout<kReadML>) as
// one, a block per region: the block updates its region's state (update_block, the
// same rows in the same order, kBeginThreads rows per pass) and then each of its
// waves forms one 17-row item of v_ml exactly as k_res_readout does (rows_dot: the
// same lanes, columns and butterfly), reading x~ back from x_aug, which this block
// has just written (same workgroup: visible after the barrier).  The update's
// latency-bound SpMV + tanh of one block then overlaps the W_out stream of the other
// blocks on its CU, instead of running as a grid of its own before the stream.
// Requires the wide readout (nout_pad = 17 g, g <= 8) and the LDS-staged update.
constexpr int kBeginThreads = 512;
template <typename WT, int kUnroll, int kMinWaves>
__global__ __launch_bounds__(kBeginThreads, kMinWaves) void k_res_begin(
    const RegionDev *__restrict__ R, const int32_t *__restrict__ a_rp, const uint16_t *__restrict__ a_col,
    const WT *__restrict__ a_val, const int32_t *__restrict__ w_rp, const uint16_t *__restrict__ w_col,
    const WT *__restrict__ w_val, Ell ell, const double *__restrict__ x_old, double *__restrict__ x_new,
    const double *__restrict__ feedback, int ncs, double leak, int lds_x, const WT *__restrict__ wout, double *__restrict__ part, int nout_pad, int groups) {
    extern __shared__ __attribute__((aligned(16))) double smem[];
    const int r = blockIdx.x;
    update_block<WT, true, kBeginThreads>(r, smem, R, a_rp, a_col, a_val, w_rp, w_col, w_val, ell, x_old, x_new,
                                          feedback, leak, 1, lds_x);
    __syncthreads();  // the region's new state complete (workgroup scope)
    const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    if (g >= groups) return;  // wave-uniform
    const RegionDev rg = R[r];
    const int ld = rg.ld;
    const WT *W = wout + rg.wout + (size_t)(g * kRowsWide) * ld;
    const double *xa = x_new + rg.xaug;
    // k_res_readout<kReadML>'s item (r, g): the same x~ loads (zero below ncs)
    const Rows<kRowsWide> ml = rows_dot<WT, kRowsWide, kUnroll>(W, ld, lane, ncs & ~(kLdAlign - 1), ld,
                                                                [=](int j) { return rd_x(xa, j, ncs); });
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < kRowsWide; ++q) part[(size_t)r * nout_pad + g * kRowsWide + q] = ml.v[q];
    }
}

// second half of the split readout (sml_res_step_finish): one thread per (region,
// output): v = v_p + v_ml (v_ml from k_res_readout<kReadML>), unstandardized --
// the same sums, in the same order, as k_res_readout<kReadFull>
// raw (may be NULL): the outputs before unstandardize as well -- predict_slab keeps
// them as its next local model (mod_slab_ocean_reservoir.f90:1235)
template <typename WT>
__global__ __launch_bounds__(256) void k_res_finish(const RegionDev *__restrict__ R, const WT *__restrict__ wlm,
                                                    const double *__restrict__ local_model,
                                                    const double *__restrict__ meanstd,
                                                    const int8_t *__restrict__ outl, const double *__restrict__ part,
                                                    double *__restrict__ outvec, int nout, int ov_ld, int nout_pad,
                                                    int ncs, int nlocal, double *__restrict__ raw = nullptr) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = t / nout_pad, o = t % nout_pad;
    if (r >= nlocal || o >= nout) return;
    const double vp = vp_sum(wlm + R[r].wlm, nout_pad, local_model + (size_t)r * ncs, ncs, o);
    const double v = vp + part[(size_t)r * nout_pad + o];
    if (raw) raw[(size_t)r * nout + o] = v;
    outvec[(size_t)r * ov_ld + o] = unstd(v, meanstd + (size_t)r * 2 * kMeanStd, outl[o]);
}

// sml_res_step_finish_grid: k_tile_local_model + k_res_finish in one launch, one
// block per region.  The region's local-model vector is tiled and standardized
// into LDS (and to d_lm when given) exactly as k_tile_local_model does, then each
// thread finishes one output with vp_sum over the LDS copy: the same values, sums
// and order as the two-launch form, one kernel boundary fewer on the hybrid step's
// critical path
// kAsm (sml_res_step_finish_assemble, one rank holding every region in order): each
// output is also scattered into the global grids with the root's clips, exactly as
// k_assemble does from the outvec (every grid point has one writer), so the
// assembly's own launch leaves the critical path
__device__ inline void assemble_one(int d, double v, double *__restrict__ g4, double *__restrict__ g2,
                                    double *__restrict__ pr) {
    if (d < 0) return;
    if (d < kGrid4d) {
        if ((d & 3) == 3 && v < 0.000001) v = 0.000001;  // mpires.f90:448-450
        g4[d] = v;
    } else if (d < kGrid4d + kGrid2d) {
        g2[d - kGrid4d] = v;
    } else {
        if (v < 0.00001) v = 0.0;  // mpires.f90:474-478
        pr[d - kGrid4d - kGrid2d] = v;
    }
}

template <typename WT>
struct Quad {
    WT v[4];
};
template <typename WT>
__device__ inline Quad<WT> load_quad(const WT *p) {
    Quad<WT> q;
    if constexpr (sizeof(WT) == 4) {
        const float4 a = *reinterpret_cast<const float4 *>(p);
        q.v[0] = a.x; q.v[1] = a.y; q.v[2] = a.z; q.v[3] = a.w;
    } else {
        const double2 a = *reinterpret_cast<const double2 *>(p), b = *reinterpret_cast<const double2 *>(p + 2);
        q.v[0] = a.x; q.v[1] = a.y; q.v[2] = b.x; q.v[3] = b.y;
    }
    return q;
}

// kGrouped (nout_pad <= 4 * 36, ncs <= kFinGroups * kFinGsz): thread t takes outputs
// 4 (t % nq) .. + 3 over column group t / nq, its W_out loads (one 16-B load per
// column) issued before the local-model gather, so they fly while the forecast is
// read; the kFinGroups partial sums meet in LDS and are added in group order
// (vp_sum's order).  Else one thread per output with vp_sum.
//
// wflag (may be null): the forecast grids come from another stream, whose one-lane
// signal kernel stores a sequence number >= wval behind SPEEDY's exit (SML_HOP_KERNEL;
// sml_hybrid.hip k_hop_signal).  The kernel then goes in ahead of the forecast: its
// W_out(:, 1:ncs) block, the gather's tables and mean / std are loaded while the window
// still runs, and only the forecast values wait -- one relaxed poll by one lane,
// one agent-scope acquire by that wave, a barrier (MI355X_MICROARCH.md
// inter-workgroup visibility, the consumer form), then plain loads.  The poll gives
// up after ~4 s, marks *wlate and goes on (sml_hybrid_sync reports it).
template <typename WT, bool kAsm = false, bool kGrouped = true>
__global__ __launch_bounds__(256) void k_res_finish_grid(
    const RegionDev *__restrict__ R, const WT *__restrict__ wlm, const int32_t *__restrict__ src,
    const uint8_t *__restrict__ lidx, const double *__restrict__ fc4, const double *__restrict__ fc2,
    double *__restrict__ lm_out, const double *__restrict__ meanstd, const int8_t *__restrict__ outl,
    const double *__restrict__ part, double *__restrict__ outvec, int nout, int ov_ld, int nout_pad, int ncs,
    const int32_t *__restrict__ asm_dst = nullptr, double *__restrict__ g4 = nullptr, double *__restrict__ g2 = nullptr,
    double *__restrict__ pr = nullptr, const uint64_t *__restrict__ wflag = nullptr, uint64_t wval = 0,
    unsigned *__restrict__ wlate = nullptr, long long wtimeout = 400000000ll) {
    __shared__ double slm[kMaxNcs];
    __shared__ int gave_up;
    __shared__ double red[kGrouped ? kFinGroups * 144 : 1];
    const int r = blockIdx.x, t = threadIdx.x;
    const double *ms = meanstd + (size_t)r * 2 * kMeanStd;
    const WT *wl = wlm + R[r].wlm;
    const int nq = nout_pad / 4, gsz = fin_gsz(ncs);
    const int q = t % nq, g = t / nq;
    const int j0 = g * gsz, j1 = min(ncs, j0 + gsz);
    Quad<WT> w[kFinGsz];
    if constexpr (kGrouped) {
        // every load issued, unpredicated (columns past the group's end clamped into the
        // block and not summed): one memory round trip for all of them
        const int gq = g < kFinGroups ? g : 0;
        const int jlast = max(ncs - 1, 0);
#pragma unroll
        for (int jj = 0; jj < kFinGsz; ++jj)
            w[jj] = load_quad(wl + (size_t)min(gq * gsz + jj, jlast) * nout_pad + 4 * q);
    }
    // the gather's tables and standardization (ncs <= kMaxNcs = blockDim: one entry per thread)
    const bool gj = t < ncs;
    int gs = 0;
    double gmean = 0.0, gstd = 1.0;
    if (gj) {
        const int e = r * ncs + t;
        gs = src[e];
        const int l = lidx[e];
        gmean = ms[l];
        gstd = ms[kMeanStd + l];
    }
    if (wflag) {
        if (t == 0) {
            gave_up = 0;
            const long long c0 = wall_clock64();
            while (__hip_atomic_load(wflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < wval) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - c0 > wtimeout) {  // default ~4 s at wall_clock64's 100 MHz
                    __hip_atomic_store(wlate, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    gave_up = 1;
                    break;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
    }
    SML_TL_SCOPE(sml::tl::kFinish);  // (after the wait: when the forecast arrived)
    if (gj) {
        // a forecast that never arrived reads as NaN: the outvecs, grids and the next
        // window's safety check then refuse it instead of predicting from stale values
        const double v = (wflag && gave_up) ? __builtin_nan("") : (gs < kGrid4d ? fc4[gs] : fc2[gs - kGrid4d]);
        const double d = v - gmean;
        const double x = d / gstd;
        slm[t] = x;
        if (lm_out) lm_out[r * ncs + t] = x;
    }
    __syncthreads();
    if constexpr (kGrouped) {
        // (keep the W_out quads in their storage precision until here: converted early
        // they would hold twice the registers across the gather)
        __builtin_amdgcn_sched_barrier(0);
        if (g < kFinGroups) {
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int jj = 0; jj < kFinGsz; ++jj)
                if (j0 + jj < j1) {
                    const double x = slm[j0 + jj];
#pragma unroll
                    for (int k = 0; k < 4; ++k) acc[k] = fma((double)w[jj].v[k], x, acc[k]);
                }
#pragma unroll
            for (int k = 0; k < 4; ++k) red[g * nout_pad + 4 * q + k] = acc[k];
        }
        __syncthreads();
    }
    for (int o = t; o < nout; o += blockDim.x) {
        double vp;
        if constexpr (kGrouped) {
            vp = red[o];
#pragma unroll
            for (int gg = 1; gg < kFinGroups; ++gg) vp = vp + red[gg * nout_pad + o];
        } else {
            vp = vp_sum(wl, nout_pad, slm, ncs, o);
        }
        const double v = unstd(vp + part[(size_t)r * nout_pad + o], ms, outl[o]);
        outvec[(size_t)r * ov_ld + o] = v;
        if constexpr (kAsm) assemble_one(asm_dst[(size_t)r * nout + o], v, g4, g2, pr);
    }
}

// assemble: all regions' outvecs -> global grids, with the root's clips
__global__ void k_assemble(const int32_t *__restrict__ dst, const double *__restrict__ ov, double *__restrict__ g4,
                           double *__restrict__ g2, double *__restrict__ pr, int total, int nout, int ov_ld) {
    SML_TL_SCOPE(sml::tl::kAssemble);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int d = dst[e];
    if (d < 0) return;
    assemble_one(d, ov_ld == nout ? ov[e] : ov[(size_t)(e / nout) * ov_ld + e % nout], g4, g2, pr);
}

__device__ inline double grid_at(int src, const double *g4, const double *g2, const double *pr) {
    if (src < kGrid4d) return g4[src];
    if (src < kGrid4d + kGrid2d) return g2[src - kGrid4d];
    return pr[src - kGrid4d - kGrid2d];
}

// tile feedback: overlap tiles of the global grids, standardized (x-mean)/std
__global__ void k_tile_feedback(const int32_t *__restrict__ src, const uint8_t *__restrict__ lidx,
                                const uint16_t *__restrict__ reg, const double *__restrict__ meanstd,
                                const double *__restrict__ g4, const double *__restrict__ g2,
                                const double *__restrict__ pr, const double *__restrict__ tisr,
                                double *__restrict__ feedback, int total) {
    SML_TL_SCOPE(sml::tl::kTileFeedback);
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int s = src[e];
    if (s == kSrcKeep) return;
    if (s < kSrcKeep) {  // tisr entry: -2 - packed index
        if (tisr) feedback[e] = tisr[-2 - s];
        return;
    }
    const double *ms = meanstd + (size_t)reg[e] * 2 * kMeanStd;
    const int l = lidx[e];
    const double t = grid_at(s, g4, g2, pr) - ms[l];
    feedback[e] = t / ms[kMeanStd + l];
}

// tisr entries from one hour's global tisr field (96, 48): get_tisr_by_date's
// full_tisr(:, :, hour) of the region's overlap tile (read_3d_file_parallel over the
// input extent), standardized with the region's tisr mean / std (l = 34,
// get_full_tisr, mod_reservoir.f90:888-906)
__global__ void k_tile_tisr(const int32_t *__restrict__ fbi, const int32_t *__restrict__ gi,
                            const uint16_t *__restrict__ reg, const double *__restrict__ meanstd,
                            const double *__restrict__ G, double *__restrict__ feedback, int total) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const double *ms = meanstd + (size_t)reg[e] * 2 * kMeanStd;
    const double t = G[gi[e]] - ms[33];
    feedback[fbi[e]] = t / ms[kMeanStd + 33];
}

// tile local_model: SPEEDY forecast at the region's own points, standardized
__global__ void k_tile_local_model(const int32_t *__restrict__ src, const uint8_t *__restrict__ lidx,
                                   const double *__restrict__ meanstd, const double *__restrict__ fc4,
                                   const double *__restrict__ fc2, double *__restrict__ lm, int ncs, int total) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= total) return;
    const int s = src[e];
    const double v = s < kGrid4d ? fc4[s] : fc2[s - kGrid4d];
    const double *ms = meanstd + (size_t)(e / ncs) * 2 * kMeanStd;
    const int l = lidx[e];
    const double t = v - ms[l];
    lm[e] = t / ms[kMeanStd + l];
}

// --------------------------------------------------------------- host helpers
template <typename T>
int dalloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) count = 1;
    SML_HIP(hipMalloc((void **)p, count * sizeof(T)));
    return SML_OK;
}

int dalloc_bytes(void **p, size_t bytes) {
    *p = nullptr;
    SML_HIP(hipMalloc(p, bytes ? bytes : 16));
    return SML_OK;
}

size_t wbytes(const sml_reservoirs *c) { return c->wdtype == SML_F32 ? 4 : 8; }

// mean/std index (0-based) of output o of the bottom-level 2x2 reservoir:
// atmo (var,x,y,z) -> (var-1)*8+z, logp -> 33, precip -> 35 (1-based; :1815-1846)
int out_std_index(int o, const RegionGeom &g) {
    const int res2d = g.resx * g.resy, natmo = kVars * res2d * kZGrid;
    if (o < natmo) {
        const int v = o % kVars, z = o / (kVars * res2d);
        return v * kZGrid + z;
    }
    if (o < natmo + res2d) return 32;
    if (o < natmo + 2 * res2d) return 34;
    return -1;
}

template <typename T>
int upload(T *dst, const std::vector<T> &src) {
    if (!src.empty()) SML_HIP(hipMemcpy(dst, src.data(), src.size() * sizeof(T), hipMemcpyHostToDevice));
    return SML_OK;
}

int build_tables(sml_reservoirs *c) {
    if (c->generic) {  // no exchange / tiling tables: only the unstandardize slots
        if (int rc = dalloc(&c->d_outl, c->nout)) return rc;
        SML_HIP(hipMemcpy(c->d_outl, c->out_l.data(), c->nout, hipMemcpyHostToDevice));
        return SML_OK;
    }
    // assemble: every region of the decomposition (outvec_all is global)
    std::vector<int32_t> dst((size_t)c->numregions * c->nout, -1);
    for (int r = 0; r < c->numregions; ++r) {
        RegionGeom g;
        region_geom(c->numregions, r, &g);
        const int rx = g.resx, ry = g.resy, natmo = kVars * rx * ry * kZGrid;
        for (int o = 0; o < c->nout; ++o) {
            int d = -1;
            if (o < natmo) {
                const int v = o % kVars, x = (o / kVars) % rx, y = (o / (kVars * rx)) % ry, z = o / (kVars * rx * ry);
                d = g4(v, g.res_xstart - 1 + x, g.res_ystart - 1 + y, z);
            } else if (o < natmo + rx * ry) {
                const int p = o - natmo;
                d = kGrid4d + g2(g.res_xstart - 1 + p % rx, g.res_ystart - 1 + p / rx);
            } else if (o < natmo + 2 * rx * ry) {
                const int p = o - natmo - rx * ry;
                d = kGrid4d + kGrid2d + g2(g.res_xstart - 1 + p % rx, g.res_ystart - 1 + p / rx);
            }
            dst[(size_t)r * c->nout + o] = d;
        }
    }
    // feedback tiles of the local regions (tile_4d_and_logp_to_local_state_input +
    // standardize_state_vec_input + precip standardisation + tisr + sst)
    std::vector<int32_t> fsrc(c->tot_fb);
    std::vector<uint8_t> fl(c->tot_fb, 0);
    std::vector<uint16_t> freg(c->tot_fb);
    std::vector<int32_t> lsrc((size_t)c->nlocal * std::max(c->ncs, 1), 0);
    std::vector<uint8_t> ll((size_t)c->nlocal * std::max(c->ncs, 1), 0);
    std::vector<int32_t> tfb, tgi;
    std::vector<uint16_t> treg;
    for (int i = 0; i < c->nlocal; ++i) {
        const RegionGeom &g = c->geom[i];
        const int ix = g.inx, iy = g.iny, in2d = ix * iy, natmo = kVars * in2d * kZGrid;
        const int64_t base = c->rd[i].fb;
        auto gx = [&](int lx) { return input_x(g, lx + 1) - 1; };
        for (int z = 0; z < kZGrid; ++z)
            for (int ly = 0; ly < iy; ++ly)
                for (int lx = 0; lx < ix; ++lx)
                    for (int v = 0; v < kVars; ++v) {
                        const int64_t e = base + v + kVars * (lx + ix * (ly + iy * z));
                        fsrc[e] = g4(v, gx(lx), g.in_ystart - 1 + ly, z);
                        fl[e] = (uint8_t)(v * kZGrid + z);
                    }
        for (int ly = 0; ly < iy; ++ly)
            for (int lx = 0; lx < ix; ++lx) {
                const int p = lx + ix * ly;
                fsrc[base + natmo + p] = kGrid4d + g2(gx(lx), g.in_ystart - 1 + ly);
                fl[base + natmo + p] = 32;  // logp (l = 33)
                fsrc[base + natmo + in2d + p] = kGrid4d + kGrid2d + g2(gx(lx), g.in_ystart - 1 + ly);
                fl[base + natmo + in2d + p] = 34;  // precip (l = 35)
            }
        int64_t off = base + natmo + 2 * in2d;
        if (c->sst[i]) {
            for (int p = 0; p < in2d; ++p) fsrc[off + p] = kSrcKeep;
            off += in2d;
        }
        for (int p = 0; p < in2d; ++p) {
            fsrc[off + p] = -2 - (i * kTisrStride + p);
            tfb.push_back((int32_t)(off + p));
            tgi.push_back(g2(gx(p % ix), g.in_ystart - 1 + p / ix));
            treg.push_back((uint16_t)i);
        }
        for (int64_t e = base; e < base + c->ninp[i]; ++e) freg[e] = (uint16_t)i;
        // local_model: the region's own points of the SPEEDY forecast grids
        const int rx = g.resx, ry = g.resy, na = kVars * rx * ry * kZGrid;
        for (int cidx = 0; cidx < c->ncs; ++cidx) {
            int s = 0, l = 0;
            if (cidx < na) {
                const int v = cidx % kVars, x = (cidx / kVars) % rx, y = (cidx / (kVars * rx)) % ry,
                          z = cidx / (kVars * rx * ry);
                s = g4(v, g.res_xstart - 1 + x, g.res_ystart - 1 + y, z);
                l = v * kZGrid + z;
            } else {
                const int p = cidx - na;
                s = kGrid4d + g2(g.res_xstart - 1 + p % rx, g.res_ystart - 1 + (p / rx) % ry);
                l = 32;
            }
            lsrc[(size_t)i * c->ncs + cidx] = s;
            ll[(size_t)i * c->ncs + cidx] = (uint8_t)l;
        }
    }
    std::vector<int8_t> outl(c->nout);
    for (int o = 0; o < c->nout; ++o) outl[o] = (int8_t)out_std_index(o, c->geom.empty() ? RegionGeom{} : c->geom[0]);
    int rc;
    if ((rc = dalloc(&c->d_asm_dst, dst.size())) || (rc = dalloc(&c->d_fb_src, fsrc.size())) ||
        (rc = dalloc(&c->d_fb_l, fl.size())) || (rc = dalloc(&c->d_fb_reg, freg.size())) ||
        (rc = dalloc(&c->d_lm_src, lsrc.size())) || (rc = dalloc(&c->d_lm_l, ll.size())) ||
        (rc = dalloc(&c->d_outl, outl.size())) || (rc = dalloc(&c->d_tisr_fb, tfb.size())) ||
        (rc = dalloc(&c->d_tisr_grid, tgi.size())) || (rc = dalloc(&c->d_tisr_reg, treg.size())))
        return rc;
    c->tot_tisr = (int)tfb.size();
    if ((rc = upload(c->d_tisr_fb, tfb)) || (rc = upload(c->d_tisr_grid, tgi)) || (rc = upload(c->d_tisr_reg, treg)))
        return rc;
    SML_HIP(hipMemcpy(c->d_asm_dst, dst.data(), dst.size() * 4, hipMemcpyHostToDevice));
    if (!fsrc.empty()) {
        SML_HIP(hipMemcpy(c->d_fb_src, fsrc.data(), fsrc.size() * 4, hipMemcpyHostToDevice));
        SML_HIP(hipMemcpy(c->d_fb_l, fl.data(), fl.size(), hipMemcpyHostToDevice));
        SML_HIP(hipMemcpy(c->d_fb_reg, freg.data(), freg.size() * 2, hipMemcpyHostToDevice));
    }
    SML_HIP(hipMemcpy(c->d_lm_src, lsrc.data(), lsrc.size() * 4, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(c->d_lm_l, ll.data(), ll.size(), hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(c->d_outl, outl.data(), outl.size(), hipMemcpyHostToDevice));
    return SML_OK;
}

// convert to the storage dtype; fp32 storage demands exact representability
template <typename S, typename D>
bool narrow(const S *src, size_t count, std::vector<D> &out) {
    out.resize(count);
    for (size_t i = 0; i < count; ++i) {
        out[i] = (D)src[i];
        if ((S)out[i] != src[i] && !(src[i] != src[i])) return false;
    }
    return true;
}

// W_in's CSR pool holds n entries per region at create (the trained W_in has one
// entry per row, mod_reservoir.f90:260-278).  A denser W_in -- up to the dense
// win(n, ninp) of the reference's matmul (:1443) -- re-lays the pool: region i gets
// room for wnz entries, the other regions' entries move device to device, every
// region's offset is re-uploaded.  The ELL copy stays one slot per row: such a region
// is read from the CSR form.
int grow_win_pool(sml_reservoirs *c, int i, int64_t wnz) {
    const size_t wb = wbytes(c);
    std::vector<int64_t> off(c->nlocal);
    int64_t tot = 0;
    for (int j = 0; j < c->nlocal; ++j) {
        off[j] = tot;
        tot += (j == i) ? wnz : c->w_nz_cap[j];
    }
    uint16_t *col = nullptr;
    void *val = nullptr;
    if (int rc = dalloc(&col, tot)) return rc;
    if (int rc = dalloc_bytes(&val, tot * wb)) {
        (void)hipFree(col);
        return rc;
    }
    SML_HIP(hipDeviceSynchronize());  // steps in flight read the old pool
    for (int j = 0; j < c->nlocal; ++j) {
        if (j == i || !c->loaded[j] || c->w_nz_cap[j] == 0) continue;
        SML_HIP(hipMemcpy(col + off[j], c->d_w_col + c->rd[j].w_nz, c->w_nz_cap[j] * 2, hipMemcpyDeviceToDevice));
        SML_HIP(hipMemcpy((char *)val + off[j] * wb, (char *)c->d_w_val + c->rd[j].w_nz * wb, c->w_nz_cap[j] * wb,
                          hipMemcpyDeviceToDevice));
    }
    SML_HIP(hipFree(c->d_w_col));
    SML_HIP(hipFree(c->d_w_val));
    c->d_w_col = col;
    c->d_w_val = val;
    c->w_nz_cap[i] = wnz;
    c->tot_w_nz = tot;
    for (int j = 0; j < c->nlocal; ++j) c->rd[j].w_nz = off[j];
    SML_HIP(hipMemcpy(c->d_rd, c->rd.data(), sizeof(RegionDev) * c->nlocal, hipMemcpyHostToDevice));
    return SML_OK;
}

template <typename SrcT, typename StoT>
int load_region_impl(sml_reservoirs *c, int i, const int *rows, const int *cols, const SrcT *vals, const SrcT *win,
                     const SrcT *wout, const double *mean, const double *std) {
    const int n = c->n[i], k = c->k[i], ninp = c->ninp[i], ld = c->ld[i], ncs = c->ncs, nout = c->nout;
    const RegionDev &rg = c->rd[i];
    // --- A: COO (1-based) -> CSR, stable in file order (mklsparse, mod_linalg.f90:10-25)
    std::vector<int32_t> rp(n + 1, 0);
    for (int e = 0; e < k; ++e) {
        SML_REQUIRE(rows[e] >= 1 && rows[e] <= n && cols[e] >= 1 && cols[e] <= n,
                    "region %d: A entry %d out of range (row %d col %d, n %d)", i, e, rows[e], cols[e], n);
        rp[rows[e]]++;
    }
    for (int r = 0; r < n; ++r) rp[r + 1] += rp[r];
    std::vector<int32_t> fill(rp.begin(), rp.end() - 1);
    std::vector<uint16_t> acol(k);
    std::vector<StoT> aval(k);
    for (int e = 0; e < k; ++e) {
        const int p = fill[rows[e] - 1]++;
        acol[p] = (uint16_t)(cols[e] - 1);
        aval[p] = (StoT)vals[e];
        SML_REQUIRE((SrcT)aval[p] == vals[e], "region %d: A value %d not representable in the storage dtype", i, e);
    }
    // --- W_in: dense win(n, ninp) column-major -> CSR by row, columns ascending
    std::vector<int32_t> wrp(n + 1, 0);
    for (int col = 0; col < ninp; ++col)
        for (int r = 0; r < n; ++r)
            if (win[(size_t)col * n + r] != (SrcT)0) wrp[r + 1]++;
    for (int r = 0; r < n; ++r) wrp[r + 1] += wrp[r];
    const int64_t wnz = wrp[n];
    if (wnz > c->w_nz_cap[i])  // a W_in denser than trained (up to the dense n x ninp matmul, :1443)
        if (int rc = grow_win_pool(c, i, wnz)) return rc;
    std::vector<int32_t> wfill(wrp.begin(), wrp.end() - 1);
    std::vector<uint16_t> wcol(wnz);
    std::vector<StoT> wval(wnz);
    for (int col = 0; col < ninp; ++col)
        for (int r = 0; r < n; ++r) {
            const SrcT v = win[(size_t)col * n + r];
            if (v == (SrcT)0) continue;
            const int p = wfill[r]++;
            wcol[p] = (uint16_t)col;
            wval[p] = (StoT)v;
            SML_REQUIRE((SrcT)wval[p] == v, "region %d: W_in value not representable in the storage dtype", i);
        }
    // --- W_out: wout(nout, ncs+n) column-major -> [nout_pad][ld] row-major
    std::vector<StoT> wt((size_t)c->nout_pad * ld, (StoT)0);
    for (int j = 0; j < ncs + n; ++j)
        for (int o = 0; o < nout; ++o) {
            const SrcT v = wout[(size_t)j * nout + o];
            StoT s = (StoT)v;
            SML_REQUIRE((SrcT)s == v || v != v, "region %d: W_out value not representable in the storage dtype", i);
            wt[(size_t)o * ld + j] = s;
        }
    // --- upload
    const size_t wb = sizeof(StoT);
    SML_HIP(hipMemcpy(c->d_a_rp + rg.a_rp, rp.data(), rp.size() * 4, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(c->d_a_col + rg.a_nz, acol.data(), acol.size() * 2, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy((char *)c->d_a_val + rg.a_nz * wb, aval.data(), aval.size() * wb, hipMemcpyHostToDevice));
    SML_HIP(hipMemcpy(c->d_w_rp + rg.w_rp, wrp.data(), wrp.size() * 4, hipMemcpyHostToDevice));
    if (wnz) {
        SML_HIP(hipMemcpy(c->d_w_col + rg.w_nz, wcol.data(), wcol.size() * 2, hipMemcpyHostToDevice));
        SML_HIP(hipMemcpy((char *)c->d_w_val + rg.w_nz * wb, wval.data(), wval.size() * wb, hipMemcpyHostToDevice));
    }
    SML_HIP(hipMemcpy((char *)c->d_wout + rg.wout * wb, wt.data(), wt.size() * wb, hipMemcpyHostToDevice));
    if (ncs > 0) {  // W_out(:, 1:ncs) as [ncs][nout_pad]: the file's own order (outputs fastest), padded
        std::vector<StoT> wl((size_t)ncs * c->nout_pad, (StoT)0);
        for (int j = 0; j < ncs; ++j)
            for (int o = 0; o < nout; ++o) wl[(size_t)j * c->nout_pad + o] = (StoT)wout[(size_t)j * nout + o];
        SML_HIP(hipMemcpy((char *)c->d_wlm + rg.wlm * wb, wl.data(), wl.size() * wb, hipMemcpyHostToDevice));
    }
    // --- ELL copies (RegionDev): A pair-major with the main width that moves the fewest
    // bytes, W_in one slot per row -- file order within a row, zero-padded after the
    // row's entries; a region whose rows do not fit keeps the CSR copies only
    RegionDev &rgm = c->rd[i];
    rgm.a_w = rgm.w_w = rgm.a_ov = rgm.w_q = 0;
    rgm.w_magic = 0;
    if (c->a_ell_cap[i] > 0) {
        int maxlen = 0, nmax = 0;
        for (int r = 0; r < n; ++r) maxlen = std::max(maxlen, rp[r + 1] - rp[r]);
        for (int r = 0; r < n; ++r) nmax += (rp[r + 1] - rp[r]) == maxlen;
        if (maxlen >= 1 && maxlen <= c->a_ell_cap[i]) {
            // bytes per row: the pairs (odd widths padded), + for an overflow list its bit
            // words / counts (12 B per 64 rows) and an entry per row of maxlen entries
            const double eb = 2.0 + (double)wb;
            auto cost = [&](int w, bool ov) {
                return 2 * ((w + 1) / 2) * eb * n + (ov ? 12.0 * ((n + 63) / 64) + eb * nmax : 0.0);
            };
            int w = maxlen;
            bool ov = false;
            if (maxlen >= 2 && cost(maxlen - 1, true) < cost(maxlen, false)) {
                w = maxlen - 1;
                ov = true;
            }
            const int np = (w + 1) / 2;
            std::vector<uint16_t> ec((size_t)2 * np * n, 0);
            std::vector<StoT> ev((size_t)2 * np * n, (StoT)0);
            const int nw = (n + 63) / 64;
            std::vector<uint64_t> om(ov ? nw : 0, 0ull);
            std::vector<uint32_t> ob(ov ? nw : 0, 0u);
            std::vector<uint16_t> oc;
            std::vector<StoT> ovv;
            for (int r = 0; r < n; ++r) {
                if (ov && (r & 63) == 0) ob[r >> 6] = (uint32_t)oc.size();
                for (int e = rp[r]; e < rp[r + 1]; ++e) {
                    const int s = e - rp[r];
                    if (s < w) {  // pair s / 2, half s % 2 of row r
                        const size_t at = (size_t)(s >> 1) * 2 * n + 2 * (size_t)r + (s & 1);
                        ec[at] = acol[e];
                        ev[at] = aval[e];
                    } else {  // s == w: the overflow entry
                        om[r >> 6] |= 1ull << (r & 63);
                        oc.push_back(acol[e]);
                        ovv.push_back(aval[e]);
                    }
                }
            }
            SML_HIP(hipMemcpy(c->d_a_ell_col + rgm.a_ell, ec.data(), ec.size() * 2, hipMemcpyHostToDevice));
            SML_HIP(hipMemcpy((char *)c->d_a_ell_val + rgm.a_ell * wb, ev.data(), ev.size() * wb,
                              hipMemcpyHostToDevice));
            if (ov) {
                SML_HIP(hipMemcpy(c->d_a_om + rgm.a_om, om.data(), om.size() * 8, hipMemcpyHostToDevice));
                SML_HIP(hipMemcpy(c->d_a_ob + rgm.a_om, ob.data(), ob.size() * 4, hipMemcpyHostToDevice));
                if (!oc.empty()) {
                    SML_HIP(hipMemcpy(c->d_a_oc + rgm.a_oe, oc.data(), oc.size() * 2, hipMemcpyHostToDevice));
                    SML_HIP(hipMemcpy((char *)c->d_a_ov + rgm.a_oe * wb, ovv.data(), ovv.size() * wb,
                                      hipMemcpyHostToDevice));
                }
            }
            rgm.a_w = w;
            rgm.a_ov = ov ? 1 : 0;
        }
    }
    if (c->w_ell_cap[i] > 0) {
        bool one = true;  // exactly one entry per row (train_reservoir's W_in, mod_reservoir.f90:260-278)
        for (int r = 0; r < n && one; ++r) one = wrp[r + 1] - wrp[r] == 1;
        if (one) {
            std::vector<uint16_t> ec(n);
            std::vector<StoT> ev(n);
            for (int r = 0; r < n; ++r) {
                ec[r] = wcol[wrp[r]];
                ev[r] = wval[wrp[r]];
            }
            // block-diagonal (rows (j-1) q + 1 .. j q read input j, q = n / ninp): the
            // column is i / q, computed as umulhi(i, magic), so only the value is read
            const int q = ninp > 0 && n % ninp == 0 ? n / ninp : 0;
            bool implicit = q > 0;
            const uint32_t magic = q > 0 ? (uint32_t)((0x100000000ull + q - 1) / q) : 0u;
            for (int r = 0; r < n && implicit; ++r)
                implicit = ec[r] == r / q && (uint32_t)(((uint64_t)r * magic) >> 32) == (uint32_t)(r / q);
            SML_HIP(hipMemcpy(c->d_w_ell_col + rgm.w_ell, ec.data(), ec.size() * 2, hipMemcpyHostToDevice));
            SML_HIP(hipMemcpy((char *)c->d_w_ell_val + rgm.w_ell * wb, ev.data(), ev.size() * wb,
                              hipMemcpyHostToDevice));
            rgm.w_w = 1;
            if (implicit) {
                rgm.w_q = q;
                rgm.w_magic = magic;
            }
        }
    }
    SML_HIP(hipMemcpy(c->d_rd + i, &rgm, sizeof(RegionDev), hipMemcpyHostToDevice));
    c->ell_ok = -1;
    double ms[2 * kMeanStd];
    std::memcpy(ms, mean, sizeof(double) * kMeanStd);
    std::memcpy(ms + kMeanStd, std, sizeof(double) * kMeanStd);
    std::memcpy(&c->meanstd_h[(size_t)i * 2 * kMeanStd], ms, sizeof ms);
    SML_HIP(hipMemcpy(c->d_meanstd + (size_t)i * 2 * kMeanStd, ms, sizeof ms, hipMemcpyHostToDevice));
    c->loaded[i] = 1;
    return SML_OK;
}

int check_region(const sml_reservoirs *c, int i) {
    SML_REQUIRE(c != nullptr, "null reservoir context");
    SML_REQUIRE(i >= 0 && i < c->nlocal, "local region index %d out of range [0,%d)", i, c->nlocal);
    return SML_OK;
}

}  // namespace

// ------------------------------------------------------------------ API
extern "C" int sml_res_destroy(sml_reservoirs *c) {
    if (!c) return SML_OK;
    void *ells[] = {c->d_a_ell_col, c->d_w_ell_col, c->d_a_ell_val, c->d_w_ell_val, c->d_a_om,
                    c->d_a_ob,      c->d_a_oc,      c->d_a_ov,      c->d_zero};
    for (void *p : ells)
        if (p) (void)hipFree(p);
    void *ptrs[] = {c->d_rd,    c->d_a_rp,    c->d_w_rp,   c->d_a_col,  c->d_w_col,  c->d_a_val,  c->d_w_val,
                    c->d_wout,  c->d_x[0],    c->d_x[1],   c->d_meanstd, c->d_outl,  c->d_asm_dst,
                    c->d_fb_src, c->d_fb_l,   c->d_fb_reg, c->d_lm_src, c->d_lm_l,   c->d_io,     c->d_part,
                    c->d_wlm,   c->d_tisr_fb, c->d_tisr_grid, c->d_tisr_reg, c->d_row0, c->d_blk_r0};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : c->ev)
        if (e) (void)hipEventDestroy(e);
    delete c;
    return SML_OK;
}

namespace {
int res_create_impl(int numregions, int nlocal, const int *region_ids, const unsigned char *sst_flags,
                    const int *n, const int *k, int chunk_speedy, int nout, int weight_dtype, double leakage,
                    const int *ninp_generic, const signed char *out_index, sml_reservoirs **out);
}

extern "C" int sml_res_create(int numregions, int nlocal, const int *region_ids, const unsigned char *sst_flags,
                              const int *n, const int *k, int chunk_speedy, int nout, int weight_dtype,
                              double leakage, sml_reservoirs **out) {
    return res_create_impl(numregions, nlocal, region_ids, sst_flags, n, k, chunk_speedy, nout, weight_dtype, leakage,
                           nullptr, nullptr, out);
}

extern "C" int sml_res_create_generic(int numregions, int nlocal, const int *region_ids, const int *ninp,
                                      const int *n, const int *k, int chunk_speedy, int nout,
                                      const signed char *out_index, int weight_dtype, double leakage,
                                      sml_reservoirs **out) {
    SML_REQUIRE(nlocal == 0 || (ninp && out_index), "null ninp / out_index");
    for (int o = 0; o < nout && out_index; ++o)
        SML_REQUIRE(out_index[o] >= -1 && out_index[o] < kMeanStd, "out_index[%d] = %d outside [-1, 36)", o,
                    out_index[o]);
    std::vector<unsigned char> sst(std::max(nlocal, 1), 0);
    return res_create_impl(numregions, nlocal, region_ids, sst.data(), n, k, chunk_speedy, nout, weight_dtype,
                           leakage, ninp, out_index, out);
}

namespace {
int res_create_impl(int numregions, int nlocal, const int *region_ids, const unsigned char *sst_flags,
                    const int *n, const int *k, int chunk_speedy, int nout, int weight_dtype, double leakage,
                    const int *ninp_generic, const signed char *out_index, sml_reservoirs **out) {
    SML_REQUIRE(out != nullptr, "out is null");
    *out = nullptr;
    int fx, fy;
    SML_REQUIRE(decompose(numregions, &fx, &fy), "numregions %d does not decompose the 96x48 grid", numregions);
    SML_REQUIRE(nlocal >= 0 && nlocal <= numregions && nlocal < 65536, "bad nlocal %d", nlocal);
    SML_REQUIRE(nlocal == 0 || (region_ids && sst_flags && n && k), "null per-region arrays");
    SML_REQUIRE(chunk_speedy >= 0 && nout > 0, "bad chunk sizes (%d, %d)", chunk_speedy, nout);
    SML_REQUIRE(weight_dtype == SML_F32 || weight_dtype == SML_F64, "weight_dtype must be SML_F32 or SML_F64");
    sml_reservoirs *c = new (std::nothrow) sml_reservoirs();
    if (!c) return fail(SML_ERR_NOMEM, "host allocation failed");
    c->numregions = numregions;
    c->nlocal = nlocal;
    c->ncs = chunk_speedy;
    c->nout = nout;
    c->nout_pad = (nout + kRows - 1) / kRows * kRows;
    c->ov_ld = nout;
    c->wdtype = weight_dtype;
    c->leakage = leakage;
    c->generic = ninp_generic != nullptr;
    if (c->generic) c->out_l.assign(out_index, out_index + nout);
    (void)hipGetDevice(&c->device);
    (void)hipDeviceGetAttribute(&c->ncu, hipDeviceAttributeMultiprocessorCount, c->device);
    {
        int lds = 0;
        (void)hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerBlock, c->device);
        c->max_lds = (size_t)std::max(lds, 0);
    }
    c->region_ids.assign(region_ids, region_ids + nlocal);
    c->sst.assign(sst_flags, sst_flags + nlocal);
    c->n.assign(n, n + nlocal);
    c->k.assign(k, k + nlocal);
    c->loaded.assign(nlocal, 0);
    c->meanstd_h.assign((size_t)nlocal * 2 * kMeanStd, 0.0);
    c->geom.resize(nlocal);
    c->ninp.resize(nlocal);
    c->ld.resize(nlocal);
    c->rd.resize(nlocal);
    c->w_nz_cap.resize(nlocal);
    for (int i = 0; i < nlocal; ++i) {
        if (!region_geom(numregions, region_ids[i], &c->geom[i])) {
            sml_res_destroy(c);
            return fail(SML_ERR_ARG, "region id %d out of range", region_ids[i]);
        }
        if (n[i] <= 0 || n[i] > 65535 || k[i] < 0) {
            sml_res_destroy(c);
            return fail(SML_ERR_ARG, "region %d: n=%d (1..65535) k=%d", i, n[i], k[i]);
        }
        const RegionGeom &g = c->geom[i];
        if (!c->generic && (kVars * g.resx * g.resy * kZGrid + 2 * g.resx * g.resy != nout ||
                            (chunk_speedy && chunk_speedy != kVars * g.resx * g.resy * kZGrid + g.resx * g.resy))) {
            sml_res_destroy(c);
            return fail(SML_ERR_ARG, "nout %d / chunk_speedy %d do not match the %dx%d region tiles", nout,
                        chunk_speedy, g.resx, g.resy);
        }
        c->ninp[i] = c->generic ? ninp_generic[i] : region_ninp(g, sst_flags[i] != 0);
        if (c->ninp[i] <= 0 || c->ninp[i] > 65535) {
            sml_res_destroy(c);
            return fail(SML_ERR_ARG, "region %d: ninp %d (1..65535)", i, c->ninp[i]);
        }
        // W_out rows (and x_aug) padded to 32 columns: with the streamed columns starting
        // at ncs & ~31, every 1 KB load of a wave is whole 128-B lines (no line fetched
        // by two neighbouring loads)
        c->ld[i] = (chunk_speedy + n[i] + kLdAlign - 1) / kLdAlign * kLdAlign;
        c->w_nz_cap[i] = n[i];
        RegionDev &r = c->rd[i];
        r.n = n[i];
        r.ninp = c->ninp[i];
        r.ld = c->ld[i];
        r.a_rp = c->tot_a_rp;
        c->tot_a_rp += n[i] + 1;
        r.a_nz = c->tot_a_nz;
        c->tot_a_nz += k[i];
        r.w_rp = c->tot_w_rp;
        c->tot_w_rp += n[i] + 1;
        r.w_nz = c->tot_w_nz;
        c->tot_w_nz += n[i];
        r.wout = c->tot_wout;
        c->tot_wout += (int64_t)c->nout_pad * c->ld[i];
        r.wlm = c->tot_wlm;
        c->tot_wlm += (int64_t)c->ncs * c->nout_pad;
        // the state's slot is the x~ column block of the region's ld-wide row (column
        // ncs on, 32-column aligned start, zero padding after n): the readout streams
        // x~ straight from the state the update wrote, squaring the even-numbered
        // entries as it loads them, so the update writes 8 B per row less
        r.xaug = c->tot_xaug;
        c->tot_xaug += c->ld[i];
        r.x = r.xaug + chunk_speedy;
        r.fb = c->tot_fb;
        c->tot_fb += c->ninp[i];
        c->maxn = std::max(c->maxn, n[i]);
        c->maxninp = std::max(c->maxninp, c->ninp[i]);
        // makesparse rows hold floor(k/n) or floor(k/n)+1 entries (per-block permutations)
        c->a_ell_cap.push_back(!c->no_ell && k[i] / n[i] + 1 <= kEllA ? kEllA : 0);
        c->w_ell_cap.push_back(c->no_ell ? 0 : kEllW);
        r.a_w = r.w_w = r.a_ov = r.w_q = 0;
        r.w_magic = 0;
        r.a_ell = c->tot_a_ell;
        c->tot_a_ell += (int64_t)c->a_ell_cap.back() * n[i];
        r.w_ell = c->tot_w_ell;
        c->tot_w_ell += (int64_t)c->w_ell_cap.back() * n[i];
        r.a_om = c->tot_a_om;
        c->tot_a_om += c->a_ell_cap.back() ? (n[i] + 63) / 64 : 0;
        r.a_oe = c->tot_a_oe;
        c->tot_a_oe += c->a_ell_cap.back() ? n[i] : 0;
    }
    const size_t wb = wbytes(c);
    int rc;
    if ((rc = dalloc(&c->d_a_ell_col, std::max<int64_t>(c->tot_a_ell, 1))) ||
        (rc = dalloc_bytes(&c->d_a_ell_val, std::max<int64_t>(c->tot_a_ell, 1) * wb)) ||
        (rc = dalloc(&c->d_w_ell_col, std::max<int64_t>(c->tot_w_ell, 1))) ||
        (rc = dalloc_bytes(&c->d_w_ell_val, std::max<int64_t>(c->tot_w_ell, 1) * wb)) ||
        (rc = dalloc(&c->d_a_om, std::max<int64_t>(c->tot_a_om, 1))) ||
        (rc = dalloc(&c->d_a_ob, std::max<int64_t>(c->tot_a_om, 1))) ||
        (rc = dalloc(&c->d_a_oc, std::max<int64_t>(c->tot_a_oe, 1))) ||
        (rc = dalloc_bytes(&c->d_a_ov, std::max<int64_t>(c->tot_a_oe, 1) * wb)) ||
        (rc = dalloc_bytes(&c->d_zero, 256))) {
        sml_res_destroy(c);
        return rc;
    }
    if ((rc = dalloc(&c->d_rd, nlocal)) || (rc = dalloc(&c->d_a_rp, c->tot_a_rp)) ||
        (rc = dalloc(&c->d_a_col, c->tot_a_nz)) || (rc = dalloc_bytes(&c->d_a_val, c->tot_a_nz * wb)) ||
        (rc = dalloc(&c->d_w_rp, c->tot_w_rp)) || (rc = dalloc(&c->d_w_col, c->tot_w_nz)) ||
        (rc = dalloc_bytes(&c->d_w_val, c->tot_w_nz * wb)) || (rc = dalloc_bytes(&c->d_wout, c->tot_wout * wb)) ||
        (rc = dalloc_bytes(&c->d_wlm, std::max<int64_t>(c->tot_wlm, 1) * wb)) ||
        (rc = dalloc(&c->d_x[0], c->tot_xaug)) || (rc = dalloc(&c->d_x[1], c->tot_xaug)) ||
        (rc = dalloc(&c->d_meanstd, (size_t)nlocal * 2 * kMeanStd)) ||
        (rc = dalloc(&c->d_part, (size_t)std::max(nlocal, 1) * c->nout_pad))) {
        sml_res_destroy(c);
        return rc;
    }
    hipError_t e = hipSuccess;
    if (e == hipSuccess) e = hipMemset(c->d_zero, 0, 256);
    if (e == hipSuccess) e = hipMemset(c->d_a_rp, 0, std::max<int64_t>(c->tot_a_rp, 1) * 4);
    if (e == hipSuccess) e = hipMemset(c->d_w_rp, 0, std::max<int64_t>(c->tot_w_rp, 1) * 4);
    if (e == hipSuccess) e = hipMemset(c->d_wout, 0, std::max<int64_t>(c->tot_wout * wb, 16));
    if (e == hipSuccess) e = hipMemset(c->d_wlm, 0, std::max<int64_t>(c->tot_wlm, 1) * wb);
    if (e == hipSuccess) e = hipMemset(c->d_x[0], 0, std::max<int64_t>(c->tot_xaug, 1) * 8);
    if (e == hipSuccess) e = hipMemset(c->d_x[1], 0, std::max<int64_t>(c->tot_xaug, 1) * 8);
    if (e == hipSuccess && nlocal)
        e = hipMemcpy(c->d_rd, c->rd.data(), sizeof(RegionDev) * nlocal, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        sml_res_destroy(c);
        return fail(SML_ERR_HIP, "sml_res_create: %s", hipGetErrorString(e));
    }
    // unit std / zero mean until loaded
    for (int i = 0; i < nlocal; ++i)
        for (int l = 0; l < kMeanStd; ++l) c->meanstd_h[(size_t)i * 2 * kMeanStd + kMeanStd + l] = 1.0;
    if (nlocal) {
        e = hipMemcpy(c->d_meanstd, c->meanstd_h.data(), c->meanstd_h.size() * 8, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            sml_res_destroy(c);
            return fail(SML_ERR_HIP, "sml_res_create: %s", hipGetErrorString(e));
        }
    }
    if ((rc = build_tables(c))) {
        sml_res_destroy(c);
        return rc;
    }
    c->row0_h.assign(nlocal + 1, 0);
    for (int i = 0; i < nlocal; ++i) c->row0_h[i + 1] = c->row0_h[i] + n[i];
    if ((rc = dalloc(&c->d_row0, nlocal + 1)) ||
        hipMemcpy(c->d_row0, c->row0_h.data(), (nlocal + 1) * 4, hipMemcpyHostToDevice) != hipSuccess) {
        sml_res_destroy(c);
        return rc ? rc : fail(SML_ERR_HIP, "row table");
    }
    *out = c;
    return SML_OK;
}
}  // namespace

// the row stride of every outvec array the context writes (sml_res_step*, the
// finish kernels) and of sml_exchange_assemble's input (>= nout)
extern "C" int sml_res_set_outvec_ld(sml_reservoirs *c, int ld) {
    SML_REQUIRE(c && ld >= c->nout, "bad outvec row stride %d", ld);
    SML_REQUIRE(!c->begun, "sml_res_set_outvec_ld inside a begun step");
    c->ov_ld = ld;
    return SML_OK;
}

extern "C" int sml_res_info(const sml_reservoirs *c, int *numregions, int *nlocal, int *chunk_speedy, int *nout,
                            int *region_ids) {
    SML_REQUIRE(c, "null context");
    if (numregions) *numregions = c->numregions;
    if (nlocal) *nlocal = c->nlocal;
    if (chunk_speedy) *chunk_speedy = c->ncs;
    if (nout) *nout = c->nout;
    if (region_ids) std::memcpy(region_ids, c->region_ids.data(), sizeof(int) * c->nlocal);
    return SML_OK;
}

extern "C" int sml_res_ninp(const sml_reservoirs *c, int i, int *ninp) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(ninp, "ninp is null");
    *ninp = c->ninp[i];
    return SML_OK;
}

// the mean / std (36 each) local region i standardizes with (host copy of the loaded ones)
extern "C" int sml_res_mean_std(const sml_reservoirs *c, int i, double *mean, double *std) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(mean && std, "null argument");
    std::memcpy(mean, &c->meanstd_h[(size_t)i * 2 * kMeanStd], kMeanStd * 8);
    std::memcpy(std, &c->meanstd_h[(size_t)i * 2 * kMeanStd + kMeanStd], kMeanStd * 8);
    return SML_OK;
}

extern "C" int sml_res_feedback_offsets(const sml_reservoirs *c, int64_t *offsets) {
    SML_REQUIRE(c && offsets, "null argument");
    for (int i = 0; i < c->nlocal; ++i) offsets[i] = c->rd[i].fb;
    offsets[c->nlocal] = c->tot_fb;
    return SML_OK;
}

extern "C" int sml_res_load_region_f32(sml_reservoirs *c, int i, const int *rows, const int *cols, const float *vals,
                                       const float *win, const float *wout, const double *mean, const double *std) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(win && wout && mean && std && (c->k[i] == 0 || (rows && cols && vals)), "null weight array");
    if (c->wdtype == SML_F32) return load_region_impl<float, float>(c, i, rows, cols, vals, win, wout, mean, std);
    return load_region_impl<float, double>(c, i, rows, cols, vals, win, wout, mean, std);
}

extern "C" int sml_res_load_region_f64(sml_reservoirs *c, int i, const int *rows, const int *cols,
                                       const double *vals, const double *win, const double *wout,
                                       const double *mean, const double *std) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(win && wout && mean && std && (c->k[i] == 0 || (rows && cols && vals)), "null weight array");
    if (c->wdtype == SML_F32) return load_region_impl<double, float>(c, i, rows, cols, vals, win, wout, mean, std);
    return load_region_impl<double, double>(c, i, rows, cols, vals, win, wout, mean, std);
}

extern "C" int sml_res_set_state(sml_reservoirs *c, int i, const double *x) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(x, "x is null");
    // a begun step read the state being replaced: it is discarded (sml_res_step_cancel)
    if (int rc = sml_res_step_cancel(c)) return rc;
    SML_HIP(hipMemcpy(c->d_x[c->cur] + c->rd[i].x, x, (size_t)c->n[i] * 8, hipMemcpyHostToDevice));
    return SML_OK;
}

extern "C" int sml_res_get_state(sml_reservoirs *c, int i, double *x) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(x, "x is null");
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpy(x, c->d_x[c->cur] + c->rd[i].x, (size_t)c->n[i] * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

namespace {
bool bal_usable(sml_reservoirs *c);
}

// the CUs the context's launches get (a CU-masked stream: the hybrid loop's reservoir
// stream); the balanced update runs one block per CU.  0 = every CU of the device.
extern "C" int sml_res_set_update_cus(sml_reservoirs *c, int cus) {
    SML_REQUIRE(c && cus >= 0, "bad argument");
    c->upd_cus = cus;
    return SML_OK;
}

// 1 when sml_res_step / _begin run the balanced update (k_res_update_bal), 0 for the
// per-region k_res_update (a region in CSR form, n > 7168, ninp > 1024, SML_RES_PATH_PER_REGION)
extern "C" int sml_res_update_balanced(sml_reservoirs *c, int *balanced) {
    SML_REQUIRE(c && balanced, "null argument");
    *balanced = bal_usable(c) ? 1 : 0;
    return SML_OK;
}

extern "C" int sml_res_ell_layout(sml_reservoirs *c, int i, int *a_width, int *a_overflow, int *win_q,
                                  int *win_ell) {
    if (int rc = check_region(c, i)) return rc;
    SML_REQUIRE(a_width && a_overflow && win_q && win_ell, "null argument");
    const RegionDev &r = c->rd[i];
    *a_width = r.a_w;
    *a_overflow = r.a_ov;
    *win_q = r.w_q;
    *win_ell = r.w_w;
    return SML_OK;
}

// the fallback paths forced for every region (bitwise the defaults, which take them
// only where a region's structure does not fit): SML_RES_PATH_CSR -- A and W_in from
// their CSR copies, no ELL layout (before any region is loaded); SML_RES_PATH_PER_REGION
// -- k_res_update, a block per (region, part), instead of the balanced update;
// SML_RES_PATH_UNGROUPED_FINISH -- the v_p finish one thread per output
extern "C" int sml_res_set_reference_paths(sml_reservoirs *c, int flags) {
    SML_REQUIRE(c && (flags & ~7) == 0, "bad argument");
    const bool csr = flags & SML_RES_PATH_CSR;
    if (csr != c->no_ell) {
        for (unsigned char l : c->loaded)
            SML_REQUIRE(!l, "sml_res_set_reference_paths(SML_RES_PATH_CSR) after a region was loaded");
        c->no_ell = csr;
        // (the ELL buffers stay sized for the default: a region is laid out in ELL only
        // while its cap is non-zero, at load)
        for (int i = 0; i < c->nlocal; ++i) {
            c->a_ell_cap[i] = !csr && c->k[i] / c->n[i] + 1 <= kEllA ? kEllA : 0;
            c->w_ell_cap[i] = csr ? 0 : kEllW;
        }
        c->ell_ok = -1;
    }
    c->upd_bal = !(flags & SML_RES_PATH_PER_REGION);
    c->finish_ungrouped = flags & SML_RES_PATH_UNGROUPED_FINISH;
    return SML_OK;
}

extern "C" int sml_res_set_read_waves(sml_reservoirs *c, int waves) {
    SML_REQUIRE(c && waves >= 0, "bad argument");
    c->read_waves = waves;
    return SML_OK;
}

namespace {
bool begin_fusable(const sml_reservoirs *c);
}

extern "C" int sml_res_set_begin_mode(sml_reservoirs *c, int mode) {
    SML_REQUIRE(c && mode >= 0 && mode <= 2, "bad argument");
    c->begin_mode = mode;
    return SML_OK;
}

extern "C" int sml_res_begin_fused(const sml_reservoirs *c, int *fused) {
    SML_REQUIRE(c && fused, "null argument");
    *fused = begin_fusable(c) ? 1 : 0;
    return SML_OK;
}

extern "C" int sml_res_enable_timing(sml_reservoirs *c, int capacity) {
    SML_REQUIRE(c, "null context");
    SML_REQUIRE(capacity >= 0, "capacity must be >= 0");
    while (c->ev_cap < capacity) {
        for (int q = 0; q < 3; ++q) {
            hipEvent_t e;
            SML_HIP(hipEventCreate(&e));
            c->ev.push_back(e);
        }
        ++c->ev_cap;
    }
    c->timing = capacity > 0;
    c->ev_used = 0;
    return SML_OK;
}

extern "C" int sml_res_kernel_times(sml_reservoirs *c, float *update_ms, float *readout_ms, int max_steps,
                                    int *count) {
    SML_REQUIRE(c && count, "null argument");
    const int n = std::min(c->ev_used, max_steps);
    for (int s = 0; s < n; ++s) {
        SML_HIP(hipEventSynchronize(c->ev[3 * s + 2]));
        float a = 0, b = 0;
        SML_HIP(hipEventElapsedTime(&a, c->ev[3 * s], c->ev[3 * s + 1]));
        SML_HIP(hipEventElapsedTime(&b, c->ev[3 * s + 1], c->ev[3 * s + 2]));
        if (update_ms) update_ms[s] = a;
        if (readout_ms) readout_ms[s] = b;
    }
    *count = n;
    c->ev_used = 0;
    return SML_OK;
}

namespace {
Ell make_ell(const sml_reservoirs *c) {
    return Ell{c->d_a_ell_col, c->d_a_ell_val, c->d_w_ell_col, c->d_w_ell_val, c->d_a_om,
               c->d_a_ob,      c->d_a_oc,      c->d_a_ov,      c->d_zero};
}

// x_new = (1 - leak) x + leak tanh(A x + W_in u) for every local region (+ x~, x_aug)
bool bal_usable(sml_reservoirs *c) {
    if (!c->upd_bal || c->nlocal == 0) return false;
    if (c->ell_ok < 0) {
        c->ell_ok = 1;
        for (int i = 0; i < c->nlocal; ++i)
            if (c->rd[i].a_w <= 0 || c->rd[i].w_w <= 0) c->ell_ok = 0;
    }
    const size_t lds = 2 * (size_t)((c->maxn + 1) / 2 * 2 + c->maxninp) * sizeof(double);
    return c->ell_ok == 1 && c->maxn <= kStageX * kUpdThreads && c->maxninp <= kUpdThreads && lds <= c->max_lds;
}

int launch_update_bal(sml_reservoirs *c, const double *xo, double *xn, const double *d_feedback, hipStream_t st) {
    const int64_t total = c->row0_h[c->nlocal];
    int G = c->upd_cus > 0 ? c->upd_cus : std::max(c->ncu, 1);  // one block per CU the launch gets
    G = (int)std::max<int64_t>(1, std::min<int64_t>(G, total));
    if (G > c->blk_cap) {  // (the buffer grows only past the largest grid seen: rare, synchronous)
        const int cap = std::max(G, std::max(c->ncu, c->upd_cus));
        if (c->d_blk_r0) {
            SML_HIP(hipDeviceSynchronize());
            SML_HIP(hipFree(c->d_blk_r0));
            c->d_blk_r0 = nullptr;
        }
        if (int rc = dalloc(&c->d_blk_r0, (size_t)cap * (cap + 1) / 2)) return rc;
        c->blk_off.assign(cap + 1, -1);
        c->blk_cap = cap;
    }
    if (c->blk_off[G] < 0) {  // each block's first region, for this grid: once per G
        std::vector<int32_t> r0(G);
        for (int b = 0; b < G; ++b) {
            const int64_t g0 = total * b / G;
            r0[b] = (int32_t)(std::upper_bound(c->row0_h.begin(), c->row0_h.end(), (int32_t)g0) - c->row0_h.begin() - 1);
        }
        c->blk_off[G] = G * (G - 1) / 2;
        c->blk_host.push_back(std::move(r0));  // ordered before the launch on st
        SML_HIP(hipMemcpyAsync(c->d_blk_r0 + c->blk_off[G], c->blk_host.back().data(), (size_t)G * 4,
                               hipMemcpyHostToDevice, st));
    }
    const int32_t *blk_r0 = c->d_blk_r0 + c->blk_off[G];
    const int lds_x = (c->maxn + 1) / 2 * 2, lds_buf = lds_x + c->maxninp;
    const size_t lds = 2 * (size_t)lds_buf * sizeof(double);
    const Ell ell = make_ell(c);
    // the pairs every pass loads (the widest region's; 2 at least) and whether any
    // region keeps an overflow list
    int np = 2;
    bool ovf = false;
    for (int i = 0; i < c->nlocal; ++i) {
        np = std::max(np, (c->rd[i].a_w + 1) / 2);
        ovf = ovf || c->rd[i].a_ov;
    }
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(G), dim3(kUpdThreads), lds, st, c->d_rd, c->d_row0, blk_r0, c->nlocal,
                           total, ell, xo, xn, d_feedback, c->leakage, lds_x, lds_buf);
    };
    // two passes of A / W_in rows in flight (a third measured slower: 114-124 VGPRs)
#define SML_BAL(WT)                                                                                         \
    do {                                                                                                    \
        if (np == 2) ovf ? go(k_res_update_bal<WT, 2, true, 2>) : go(k_res_update_bal<WT, 2, false, 2>);    \
        else if (np == 3) ovf ? go(k_res_update_bal<WT, 3, true, 2>) : go(k_res_update_bal<WT, 3, false, 2>); \
        else ovf ? go(k_res_update_bal<WT, 4, true, 2>) : go(k_res_update_bal<WT, 4, false, 2>);             \
    } while (0)
    if (c->wdtype == SML_F32)
        SML_BAL(float);
    else
        SML_BAL(double);
#undef SML_BAL
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int launch_update(sml_reservoirs *c, const double *xo, double *xn, const double *d_feedback, hipStream_t st) {
    if (bal_usable(c)) return launch_update_bal(c, xo, xn, d_feedback, st);
    // parts per region: enough blocks to fill the 512 resident 1024-thread block slots
    // (2 per CU with ~54 KB LDS each) once, each part at least one 1024-row pass.  Every
    // part stages the region's whole x, so more parts cost HBM traffic: measured on
    // 1152 regions, 1 part 119 us, 2 parts 128 us, 4 parts 165 us (profiles/r01m)
    const int max_parts = std::max(1, (c->maxn + kUpdThreads - 1) / kUpdThreads);
    const int parts = std::max(1, std::min(max_parts, (512 + c->nlocal - 1) / c->nlocal));
    const int lds_x = (c->maxn + 1) / 2 * 2;
    const size_t lds = (size_t)(lds_x + c->maxninp) * sizeof(double);
    const bool use_lds = lds <= 64 * 1024;
    const int bpr = parts;
    const int nlog = bpr * c->nlocal;
    const dim3 ug(nlog);
#define SML_UPD(WT, L)                                                                                            \
    hipLaunchKernelGGL((k_res_update<WT, L, 4>), ug, dim3(kUpdThreads),                                          \
                       L ? lds : 0, st, c->d_rd, c->d_a_rp, c->d_a_col, (const WT *)c->d_a_val, c->d_w_rp,        \
                       c->d_w_col, (const WT *)c->d_w_val, ell, xo, xn, d_feedback, c->leakage, bpr, lds_x, nlog)
    const Ell ell = make_ell(c);
    if (c->wdtype == SML_F32) {
        if (use_lds)
            SML_UPD(float, true);
        else
            SML_UPD(float, false);
    } else {
        if (use_lds)
            SML_UPD(double, true);
        else
            SML_UPD(double, false);
    }
#undef SML_UPD
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int begin_mode(const sml_reservoirs *c) { return c->begin_mode; }

// the fused begin needs the wide readout (8 waves of 17 rows per region at most)
// and the update's LDS staging (2 blocks per CU: <= 64 KB each)
bool begin_fusable(const sml_reservoirs *c) {
    const int lds_x = (c->maxn + 1) / 2 * 2;
    return begin_mode(c) > 0 && c->nout_pad % kRowsWide == 0 && c->nout_pad / kRowsWide <= kBeginThreads / 64 &&
           (size_t)(lds_x + c->maxninp) * sizeof(double) <= 64 * 1024;
}

int launch_begin(sml_reservoirs *c, const double *xo, double *xn, const double *d_feedback, hipStream_t st) {
    const int lds_x = (c->maxn + 1) / 2 * 2;
    const size_t lds = (size_t)(lds_x + c->maxninp) * sizeof(double);
    const int groups = c->nout_pad / kRowsWide;
    const Ell ell = make_ell(c);
    auto go = [&](auto wt_tag, auto kern) {
        using WT = decltype(wt_tag);
        hipLaunchKernelGGL(kern, dim3(c->nlocal), dim3(kBeginThreads), lds, st, c->d_rd, c->d_a_rp, c->d_a_col,
                           (const WT *)c->d_a_val, c->d_w_rp, c->d_w_col, (const WT *)c->d_w_val, ell, xo, xn,
                           d_feedback, c->ncs, c->leakage, lds_x, (const WT *)c->d_wout, c->d_part,
                           c->nout_pad, groups);
    };
    const bool two = begin_mode(c) == 2;
    if (c->wdtype == SML_F32) {
        if (two) go(float{}, k_res_begin<float, 2, 2>);
        else go(float{}, k_res_begin<float, 1, 4>);
    } else {
        if (two) go(double{}, k_res_begin<double, 2, 2>);
        else go(double{}, k_res_begin<double, 1, 4>);
    }
    SML_HIP(hipGetLastError());
    return SML_OK;
}

int check_loaded(const sml_reservoirs *c) {
    for (int i = 0; i < c->nlocal; ++i)
        if (!c->loaded[i]) return fail(SML_ERR_STATE, "local region %d has no weights loaded", i);
    return SML_OK;
}

// xs: the state the readout's x~ comes from (the one the update just wrote; unused
// by the finish)
template <int kMode>
void launch_readout(sml_reservoirs *c, const double *xs, const double *d_local_model, double *d_outvec,
                    hipStream_t st, double *d_raw = nullptr) {
    if constexpr (kMode == kReadFinish) {
        const int total = c->nlocal * c->nout_pad;
        if (c->wdtype == SML_F32)
            hipLaunchKernelGGL(k_res_finish<float>, dim3((total + 255) / 256), dim3(256), 0, st, c->d_rd,
                               (const float *)c->d_wlm, d_local_model, c->d_meanstd, c->d_outl, c->d_part, d_outvec,
                               c->nout, c->ov_ld, c->nout_pad, c->ncs, c->nlocal, d_raw);
        else
            hipLaunchKernelGGL(k_res_finish<double>, dim3((total + 255) / 256), dim3(256), 0, st, c->d_rd,
                               (const double *)c->d_wlm, d_local_model, c->d_meanstd, c->d_outl, c->d_part,
                               d_outvec, c->nout, c->ov_ld, c->nout_pad, c->ncs, c->nlocal, d_raw);
    } else {
        const bool wide = c->nout_pad % kRowsWide == 0 && c->nout_pad / kRowsWide <= 8;
        const int rows = wide ? kRowsWide : kRows;
        const int groups = c->nout_pad / rows;
        const int nitems = c->nlocal * groups;
        const int wpb = wide ? kWideWaves : 4;  // waves per block
        // the v_ml half runs beside SPEEDY's window: c->read_waves > 0 caps its waves
        // (each takes a run of items) so it leaves HBM headroom for the window
        int ipw = 1;
        if (kMode == kReadML && c->read_waves > 0 && c->read_waves < nitems)
            ipw = (nitems + c->read_waves - 1) / c->read_waves;
        const int nwaves = (nitems + ipw - 1) / ipw;
        const int nblocks = (nwaves + wpb - 1) / wpb;
        auto go = [&](auto wt_tag, auto r_tag) {
            using WT = decltype(wt_tag);
            constexpr int R = decltype(r_tag)::value;
            hipLaunchKernelGGL((k_res_readout<WT, kMode, R>), dim3(nblocks), dim3(64 * wpb), 0, st, c->d_rd,
                               (const WT *)c->d_wout, (const WT *)c->d_wlm, xs, d_local_model, c->d_meanstd,
                               c->d_outl, c->d_part, d_outvec, c->nout, c->ov_ld, c->nout_pad, c->ncs, groups, nitems, ipw);
        };
        using RW = std::integral_constant<int, kRowsWide>;
        using RN = std::integral_constant<int, kRows>;
        if (c->wdtype == SML_F32) {
            if (wide) go(float{}, RW{});
            else go(float{}, RN{});
        } else {
            if (wide) go(double{}, RW{});
            else go(double{}, RN{});
        }
    }
}
}  // namespace

extern "C" int sml_res_step_begin(sml_reservoirs *c, const double *d_feedback, void *stream) {
    SML_REQUIRE(c, "null context");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_feedback, "null device buffer");
    if (c->begun) return fail(SML_ERR_STATE, "sml_res_step_begin called twice without sml_res_step_finish");
    if (int rc = check_loaded(c)) return rc;
    hipStream_t st = (hipStream_t)stream;
    const double *xo = c->d_x[c->cur];
    double *xn = c->d_x[1 - c->cur];
    const bool rec = c->timing && c->ev_used < c->ev_cap;
    hipEvent_t *ev = rec ? &c->ev[3 * c->ev_used] : nullptr;
    if (rec) SML_HIP(hipEventRecord(ev[0], st));
    if (begin_fusable(c)) {  // one launch: the update's time is inside the readout's (update_ms 0)
        if (rec) SML_HIP(hipEventRecord(ev[1], st));
        if (int rc = launch_begin(c, xo, xn, d_feedback, st)) return rc;
    } else {
        if (int rc = launch_update(c, xo, xn, d_feedback, st)) return rc;  // beside SPEEDY's window
        if (rec) SML_HIP(hipEventRecord(ev[1], st));
        launch_readout<kReadML>(c, xn, nullptr, nullptr, st);
    }
    SML_HIP(hipGetLastError());
    if (rec) {
        SML_HIP(hipEventRecord(ev[2], st));
        ++c->ev_used;
    }
    c->cur = 1 - c->cur;
    c->begun = true;
    return SML_OK;
}

// discard a begun step (sml_res_step_begin without its finish): wait for it, then
// roll the state back -- the begin read x from one buffer and wrote the update into
// the other, so the old state is intact; x_aug and the v_ml partial sums are scratch
// that the next begin rewrites.  A no-op when no step is begun.
extern "C" int sml_res_step_cancel(sml_reservoirs *c) {
    SML_REQUIRE(c, "null context");
    if (!c->begun) return SML_OK;
    SML_HIP(hipDeviceSynchronize());
    c->cur = 1 - c->cur;
    c->begun = false;
    return SML_OK;
}

extern "C" int sml_res_step_begun(const sml_reservoirs *c, int *begun) {
    SML_REQUIRE(c && begun, "null argument");
    *begun = c->begun ? 1 : 0;
    return SML_OK;
}

extern "C" int sml_res_step_finish(sml_reservoirs *c, const double *d_local_model, double *d_outvec, void *stream) {
    SML_REQUIRE(c, "null context");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_outvec, "null device buffer");
    SML_REQUIRE(c->ncs == 0 || d_local_model, "hybrid context needs d_local_model");
    if (!c->begun) return fail(SML_ERR_STATE, "sml_res_step_finish without sml_res_step_begin");
    hipStream_t st = (hipStream_t)stream;
    launch_readout<kReadFinish>(c, nullptr, d_local_model, d_outvec, st);
    SML_HIP(hipGetLastError());
    c->begun = false;
    return SML_OK;
}

// predict_slab (src/mod_slab_ocean_reservoir.f90:1201-1249) for every local region
// of a generic context: x = tanh(A x + W_in feedback) (leakage as created; the
// reference's slab update has none, i.e. 1), outvec = W_out [local_model; x~], the
// raw outvec as the next local model (:1235), then x*std + mean per output slot.
// d_local_model_next must not alias d_local_model (the host ping-pongs them).
extern "C" int sml_res_step_slab(sml_reservoirs *c, const double *d_feedback, const double *d_local_model,
                                 double *d_local_model_next, double *d_outvec, void *stream) {
    SML_REQUIRE(c, "null context");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_feedback && d_outvec && d_local_model_next && (c->ncs == 0 || d_local_model), "null device buffer");
    SML_REQUIRE(d_local_model_next != d_local_model, "d_local_model_next must not alias d_local_model");
    SML_REQUIRE(c->ncs == c->nout, "predict_slab feeds its outvec back: chunk_speedy (%d) must equal nout (%d)",
                c->ncs, c->nout);
    if (int rc = sml_res_step_begin(c, d_feedback, stream)) return rc;
    launch_readout<kReadFinish>(c, nullptr, d_local_model, d_outvec, (hipStream_t)stream, d_local_model_next);
    SML_HIP(hipGetLastError());
    c->begun = false;
    return SML_OK;
}

namespace {
// the finish from SPEEDY's forecast grids (k_res_finish_grid), grouped when the shape
// allows (nout_pad <= 144 in quads, ncs <= kFinGroups * kFinGsz), with or without the
// assembly
template <bool kAsm>
void launch_finish_grid(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d, double *d_local_model,
                        double *d_outvec, double *d_grid4d, double *d_grid2d, double *d_precip, hipStream_t st) {
    const bool grouped = c->ncs > 0 && c->nout_pad % 4 == 0 && c->nout_pad <= 144 && c->nout_pad / 4 * kFinGroups <= 256 &&
                         (c->ncs + kFinGroups - 1) / kFinGroups <= kFinGsz && !c->finish_ungrouped;
    auto go = [&](auto wt_tag, auto grouped_tag) {
        using WT = decltype(wt_tag);
        hipLaunchKernelGGL((k_res_finish_grid<WT, kAsm, decltype(grouped_tag)::value>), dim3(c->nlocal), dim3(256), 0,
                           st, c->d_rd, (const WT *)c->d_wlm, c->d_lm_src, c->d_lm_l, d_fc4d, d_fc2d, d_local_model,
                           c->d_meanstd, c->d_outl, c->d_part, d_outvec, c->nout, c->ov_ld, c->nout_pad, c->ncs,
                           c->d_asm_dst, d_grid4d, d_grid2d, d_precip, c->fin_wflag, c->fin_wval, c->fin_wlate,
                           c->fin_wtimeout);
    };
    using G1 = std::integral_constant<bool, true>;
    using G0 = std::integral_constant<bool, false>;
    if (c->wdtype == SML_F32) {
        if (grouped) go(float{}, G1{});
        else go(float{}, G0{});
    } else {
        if (grouped) go(double{}, G1{});
        else go(double{}, G0{});
    }
    c->fin_wflag = nullptr;  // one launch
    c->fin_wlate = nullptr;
}
}  // namespace

int sml::res_finish_wait(sml_reservoirs *c, const uint64_t *flag, uint64_t value, unsigned *late,
                         long long timeout) {
    SML_REQUIRE(c && flag && late, "null argument");
    SML_REQUIRE(c->ncs <= 256, "the in-kernel wait needs ncs <= the finish block");
    c->fin_wflag = flag;
    c->fin_wval = value;
    c->fin_wlate = late;
    c->fin_wtimeout = timeout;
    return SML_OK;
}

extern "C" int sml_res_step_finish_grid(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d,
                                        double *d_local_model, double *d_outvec, void *stream) {
    SML_REQUIRE(c, "null context");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_outvec && (c->ncs == 0 || (d_fc4d && d_fc2d)), "null device buffer");
    SML_REQUIRE(!c->generic || c->ncs == 0, "a generic (slab) context has no local-model tiling");
    SML_REQUIRE(c->ncs <= kMaxNcs, "ncs %d exceeds %d", c->ncs, kMaxNcs);
    if (!c->begun) return fail(SML_ERR_STATE, "sml_res_step_finish_grid without sml_res_step_begin");
    launch_finish_grid<false>(c, d_fc4d, d_fc2d, d_local_model, d_outvec, nullptr, nullptr, nullptr,
                              (hipStream_t)stream);
    SML_HIP(hipGetLastError());
    c->begun = false;
    return SML_OK;
}

bool sml::res_in_global_order(const sml_reservoirs *c) {
    if (!c || c->generic || c->nlocal != c->numregions) return false;
    for (int i = 0; i < c->nlocal; ++i)
        if (c->region_ids[i] != i) return false;
    return true;
}

extern "C" int sml_res_step_finish_assemble(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d,
                                            double *d_local_model, double *d_outvec, double *d_grid4d,
                                            double *d_grid2d, double *d_precip, void *stream) {
    SML_REQUIRE(c, "null context");
    SML_REQUIRE(sml::res_in_global_order(c), "the fused assembly needs every region on this rank, in global order");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_outvec && d_grid4d && d_grid2d && d_precip && (c->ncs == 0 || (d_fc4d && d_fc2d)),
                "null device buffer");
    SML_REQUIRE(c->ncs <= kMaxNcs, "ncs %d exceeds %d", c->ncs, kMaxNcs);
    if (!c->begun) return fail(SML_ERR_STATE, "sml_res_step_finish_assemble without sml_res_step_begin");
    launch_finish_grid<true>(c, d_fc4d, d_fc2d, d_local_model, d_outvec, d_grid4d, d_grid2d, d_precip,
                             (hipStream_t)stream);
    SML_HIP(hipGetLastError());
    c->begun = false;
    return SML_OK;
}

extern "C" int sml_res_step(sml_reservoirs *c, const double *d_feedback, const double *d_local_model,
                            double *d_outvec, void *stream) {
    SML_REQUIRE(c, "null context");
    if (c->nlocal == 0) return SML_OK;
    SML_REQUIRE(d_feedback && d_outvec, "null device buffer");
    SML_REQUIRE(c->ncs == 0 || d_local_model, "hybrid context needs d_local_model");
    if (c->begun) return fail(SML_ERR_STATE, "sml_res_step inside a begun step");
    if (int rc = check_loaded(c)) return rc;
    hipStream_t st = (hipStream_t)stream;
    const bool rec = c->timing && c->ev_used < c->ev_cap;
    hipEvent_t *ev = rec ? &c->ev[3 * c->ev_used] : nullptr;
    if (rec) SML_HIP(hipEventRecord(ev[0], st));
    if (int rc = launch_update(c, c->d_x[c->cur], c->d_x[1 - c->cur], d_feedback, st)) return rc;
    if (rec) SML_HIP(hipEventRecord(ev[1], st));
    launch_readout<kReadFull>(c, c->d_x[1 - c->cur], d_local_model, d_outvec, st);
    SML_HIP(hipGetLastError());
    if (rec) {
        SML_HIP(hipEventRecord(ev[2], st));
        ++c->ev_used;
    }
    c->cur = 1 - c->cur;
    return SML_OK;
}

// synchronize (src/mod_reservoir.f90:1352-1378): `length` reservoir updates driven
// by a sequence of inputs, no readout -- the spin-up of start_prediction (:938-959).
// d_inputs: length blocks of the packed feedback layout (sml_res_feedback_offsets),
// block i at d_inputs + i * stride doubles.
extern "C" int sml_res_synchronize(sml_reservoirs *c, const double *d_inputs, int length, int64_t stride,
                                   void *stream) {
    SML_REQUIRE(c && length >= 0, "bad argument");
    if (c->nlocal == 0 || length == 0) return SML_OK;
    SML_REQUIRE(d_inputs && stride >= (int64_t)c->tot_fb, "stride smaller than the packed feedback size");
    if (c->begun) return fail(SML_ERR_STATE, "sml_res_synchronize inside a begun step");
    for (int i = 0; i < c->nlocal; ++i)
        if (!c->loaded[i]) return fail(SML_ERR_STATE, "local region %d has no weights loaded", i);
    hipStream_t st = (hipStream_t)stream;
    for (int t = 0; t < length; ++t) {
        if (int rc = launch_update(c, c->d_x[c->cur], c->d_x[1 - c->cur], d_inputs + (size_t)t * stride, st))
            return rc;
        c->cur = 1 - c->cur;
    }
    return SML_OK;
}

// start_prediction (src/mod_reservoir.f90:938-959): synchronize_print (:1381-1414,
// the same update loop as synchronize) over the first `length` input blocks, then
// the next block becomes the feedback (reservoir%feedback = predictiondata(:, L+1))
extern "C" int sml_res_start_prediction(sml_reservoirs *c, const double *d_inputs, int length, int64_t stride,
                                        double *d_feedback, void *stream) {
    SML_REQUIRE(c && d_inputs && d_feedback && length >= 0, "bad argument");
    if (int rc = sml_res_synchronize(c, d_inputs, length, stride, stream)) return rc;
    if (c->tot_fb)
        SML_HIP(hipMemcpyAsync(d_feedback, d_inputs + (size_t)length * stride, (size_t)c->tot_fb * 8,
                               hipMemcpyDeviceToDevice, (hipStream_t)stream));
    return SML_OK;
}

extern "C" int sml_res_step_host(sml_reservoirs *c, const double *feedback, const double *local_model,
                                 double *outvec) {
    SML_REQUIRE(c && feedback && outvec, "null argument");
    SML_REQUIRE(c->ncs == 0 || local_model, "hybrid context needs local_model");
    const size_t nfb = c->tot_fb, nlm = (size_t)c->nlocal * c->ncs, nov = (size_t)c->nlocal * c->ov_ld;
    if (c->d_io_n != nfb + nlm + nov) {  // sized for the current outvec stride
        if (c->d_io) SML_HIP(hipFree(c->d_io));
        c->d_io = nullptr;
        if (int rc = dalloc(&c->d_io, nfb + nlm + nov)) return rc;
        c->d_io_n = nfb + nlm + nov;
    }
    double *dfb = c->d_io, *dlm = dfb + nfb, *dov = dlm + nlm;
    SML_HIP(hipMemcpy(dfb, feedback, nfb * 8, hipMemcpyHostToDevice));
    if (nlm) SML_HIP(hipMemcpy(dlm, local_model, nlm * 8, hipMemcpyHostToDevice));
    if (int rc = sml_res_step(c, dfb, dlm, dov, nullptr)) return rc;
    SML_HIP(hipMemcpy2D(outvec, (size_t)c->nout * 8, dov, (size_t)c->ov_ld * 8, (size_t)c->nout * 8, c->nlocal,
                        hipMemcpyDeviceToHost));
    return SML_OK;
}

extern "C" int sml_res_footprint(const sml_reservoirs *c, int64_t *weight_bytes, int64_t *algo_bytes) {
    SML_REQUIRE(c, "null context");
    const int64_t wb = (int64_t)wbytes(c);
    int64_t w = 0, a = 0;
    for (int i = 0; i < c->nlocal; ++i) {
        const int64_t n = c->n[i], k = c->k[i], ninp = c->ninp[i];
        const int64_t wout = wb * c->nout * (c->ncs + n);     // unpadded W_out
        const int64_t amat = 4 * (n + 1) + (2 + wb) * k;      // CSR row ptr + col + val
        const int64_t winm = 4 * (n + 1) + (2 + wb) * n;      // CSR, one entry per row
        w += wout + amat + winm;
        // minimal traffic: weights once, state in + out, feedback, local model, outvec
        a += wout + amat + winm + 8 * n + 8 * n + 8 * ninp + 8 * c->ncs + 8 * c->nout;
    }
    if (weight_bytes) *weight_bytes = w;
    if (algo_bytes) *algo_bytes = a;
    return SML_OK;
}

extern "C" int sml_exchange_assemble(sml_reservoirs *c, const double *d_outvec_all, double *d_grid4d,
                                     double *d_grid2d, double *d_precip, void *stream) {
    SML_REQUIRE(c && d_outvec_all && d_grid4d && d_grid2d && d_precip, "null argument");
    SML_REQUIRE(!c->generic, "a generic (slab) context has no exchange tables");
    const int total = c->numregions * c->nout;
    hipLaunchKernelGGL(k_assemble, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, c->d_asm_dst,
                       d_outvec_all, d_grid4d, d_grid2d, d_precip, total, c->nout, c->ov_ld);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_res_tile_feedback(sml_reservoirs *c, const double *d_grid4d, const double *d_grid2d,
                                     const double *d_precip, const double *d_tisr, double *d_feedback, void *stream) {
    SML_REQUIRE(c && d_grid4d && d_grid2d && d_precip && d_feedback, "null argument");
    SML_REQUIRE(!c->generic, "a generic (slab) context has no exchange tables");
    if (c->tot_fb) {
        const int total = (int)c->tot_fb;
        hipLaunchKernelGGL(k_tile_feedback, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream, c->d_fb_src,
                           c->d_fb_l, c->d_fb_reg, c->d_meanstd, d_grid4d, d_grid2d, d_precip, d_tisr, d_feedback,
                           total);
        SML_HIP(hipGetLastError());
    }
    return SML_OK;
}

extern "C" int sml_res_tile_tisr_field(sml_reservoirs *c, const double *d_tisr_grid, double *d_feedback,
                                       void *stream) {
    SML_REQUIRE(c && d_tisr_grid && d_feedback, "null argument");
    SML_REQUIRE(!c->generic, "a generic (slab) context has no exchange tables");
    if (c->tot_tisr) {
        hipLaunchKernelGGL(k_tile_tisr, dim3((c->tot_tisr + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           c->d_tisr_fb, c->d_tisr_grid, c->d_tisr_reg, c->d_meanstd, d_tisr_grid, d_feedback,
                           c->tot_tisr);
        SML_HIP(hipGetLastError());
    }
    return SML_OK;
}

extern "C" int sml_res_tile_local_model(sml_reservoirs *c, const double *d_fc4d, const double *d_fc2d,
                                        double *d_local_model, void *stream) {
    SML_REQUIRE(c && d_fc4d && d_fc2d && d_local_model, "null argument");
    SML_REQUIRE(!c->generic, "a generic (slab) context has no exchange tables");
    if (c->ncs && c->nlocal) {
        const int total = c->nlocal * c->ncs;
        hipLaunchKernelGGL(k_tile_local_model, dim3((total + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                           c->d_lm_src, c->d_lm_l, c->d_meanstd, d_fc4d, d_fc2d, d_local_model, c->ncs, total);
        SML_HIP(hipGetLastError());
    }
    return SML_OK;
}

extern "C" int sml_res_tile_inputs(sml_reservoirs *c, const double *d_grid4d, const double *d_grid2d,
                                   const double *d_precip, const double *d_fc4d, const double *d_fc2d,
                                   const double *d_tisr, double *d_feedback, double *d_local_model, void *stream) {
    if (int rc = sml_res_tile_feedback(c, d_grid4d, d_grid2d, d_precip, d_tisr, d_feedback, stream)) return rc;
    if (c->ncs && d_fc4d && c->nlocal) return sml_res_tile_local_model(c, d_fc4d, d_fc2d, d_local_model, stream);
    return SML_OK;
}

// ---------------------------------------------------------------- CU-range streams
extern "C" int sml_stream_create_cu_range(int first_cu, int num_cus, void **out) {
    SML_REQUIRE(out && first_cu >= 0 && num_cus > 0, "bad argument");
    int dev = 0, ncu = 0;
    SML_HIP(hipGetDevice(&dev));
    SML_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    SML_REQUIRE(first_cu + num_cus <= ncu, "CU range [%d, %d) exceeds the device's %d CUs", first_cu,
                first_cu + num_cus, ncu);
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int c = first_cu; c < first_cu + num_cus; ++c) mask[c / 32] |= 1u << (c % 32);
    hipStream_t s = nullptr;
    SML_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *out = s;
    return SML_OK;
}

extern "C" int sml_stream_destroy(void *stream) {
    SML_REQUIRE(stream, "bad argument");
    SML_HIP(hipStreamDestroy((hipStream_t)stream));
    return SML_OK;
}

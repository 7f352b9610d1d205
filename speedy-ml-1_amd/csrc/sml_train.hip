// sml_train.hip -- W_out ridge training for a batch of regions on gfx950.
//
// Reference (per region, one vertical level):
//   chunking_matmul  src/mod_reservoir.f90:1643-1699
//       states_x_trainingdata_aug += targetdata * augmented_states^T   (136 x naug)
//       states_x_states_aug       += augmented_states * augmented_states^T  (DGEMM)
//     with augmented_states(naug = chunk_size_speedy + n, m) = [imperfect model ; x]
//   fit_chunk_hybrid src/mod_reservoir.f90:1233-1332 (fit_chunk_ml :1175-1231)
//       diag += beta_model (first chunk_size_speedy) / beta_res (rest), squared when
//       using_prior, prior(i,i) = prior_val * beta_model^2 added to b_trans
//   mldivide         src/mod_linalg.f90:109-151: dgesv(a_trans, b_trans), wout = b_trans^T
//
// MI355X design.  The Gram accumulation is the flop-heavy part (2 naug^2 m per
// batch, ~16 TFLOP per region over a full training run): one hand-written fp64
// MFMA kernel (v_mfma_f64_16x16x4_f64) computes, for every region of the batch,
// the lower-triangular 128x128 tiles of S S^T and the 136-row strip T S^T in one
// launch; S and T are read once per tile pair from HBM through LDS.  The solve is
// SPD (regularised Gram), so it is a Cholesky factorisation instead of dgesv's LU --
// the same solution up to rounding x cond(G) -- written here for the batch
// (right-looking, 128 x 128 blocks, in place on the padded column-major G):
//   per block column k: k_chol_diag_b factors the diagonal block in LDS and inverts
//   its triangle (one workgroup per region); k_chol_panel forms L_ik = A_ik L_kk^-T
//   as a GEMM against that inverse; k_chol_update subtracts L_ik L_jk^T from every
//   trailing tile (the n^3/3 flops, fp64 MFMA) -- then the two triangular solves
//   against the 136 right-hand sides, block by block with the same GEMM tile.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "sml_internal.hpp"

using namespace sml;

typedef double d4 __attribute__((ext_vector_type(4)));
typedef double d2 __attribute__((ext_vector_type(2)));
#define MFMA64(a, b, c) __builtin_amdgcn_mfma_f64_16x16x4f64((a), (b), (c), 0, 0, 0)

namespace {

constexpr int kTile = 128;  // C tile edge
constexpr int kKC = 16;     // time steps per LDS stage
constexpr int kLdsPad = 4;  // row padding (doubles) against bank conflicts
constexpr int kStrip = 2;   // tile rows of the T S^T strip (nout <= 256)
constexpr int kRhs = 144;   // right-hand sides of the solves: nout = 136 rounded up to the 16-wide MFMA tile
constexpr int kPanel = 8;   // block columns per Cholesky panel (default): trailing-update depth 1024

struct TrainRegion {
    long long s_off, t_off;  // offsets of S (naug x m) and T (nout x m) in the batch buffers
    int naug;
    int pad_;
};

// block columns of region r holding data: the batch's tiles are sized for its largest
// naug (npad); a region's blocks at or past ceil(naug / 128) are padding -- zero in S,
// identity in the regularised G -- so every kernel below skips them (adding exact zeros,
// or factoring / inverting an identity block, is all they would do: bitwise the same)
__device__ inline int live_blocks(const TrainRegion *regs, int r) { return (regs[r].naug + kTile - 1) / kTile; }

// tile index -> (bi, bj): lower triangle of the C x C Gram tiles first, then the
// kStrip x C strip tiles (rows = outputs).
__device__ inline bool tile_of(int idx, int C, int *bi, int *bj, bool *strip) {
    const int tri = C * (C + 1) / 2;
    if (idx < tri) {
        int i = (int)((sqrt(8.0 * idx + 1.0) - 1.0) * 0.5);
        while (i * (i + 1) / 2 > idx) --i;
        while ((i + 1) * (i + 2) / 2 <= idx) ++i;
        *bi = i;
        *bj = idx - i * (i + 1) / 2;
        *strip = false;
        return true;
    }
    idx -= tri;
    if (idx >= kStrip * C) return false;
    *bi = idx / C;
    *bj = idx % C;
    *strip = true;
    return true;
}

// The Gram and cross product: one workgroup (4 waves, 2 x 2) per (region, 128 x 128
// tile); wave (wr, wc) owns a 64 x 64 sub-tile = 4 x 4 MFMA 16x16 tiles.  K loop over
// the batch's time steps in stages of 16, register-prefetched one stage ahead into
// double-buffered LDS stages: one barrier per stage (the next stage's registers go to
// the other buffer while this one is read), the LDS rows padded to 144 doubles so the
// two 16-lane halves of a ds_read_b64 group (consecutive k) fall on disjoint banks (a
// 132-double row shifts by 8 banks: 2-way conflicts).  (The single-buffered form, two
// barriers per stage, measured slower: DESIGN.md §3.4.)
constexpr int kLdsLd2 = kTile + 16;

// One 16-B-per-lane global -> LDS copy (global_load_lds_dwordx4): lane l's 16 bytes from
// g land at LDS byte address lds + 16 l.  In inline asm (as the CDNA guide's recipe:
// M0 saved, set and restored in the one statement) because the builtin makes hipcc wait
// vmcnt(0) around every such load; hipcc does not count these loads, so their
// completion is waited for by hand (lds_dma_wait) before the barrier that publishes them.
__device__ __forceinline__ void lds_dma16(const void *g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(g), "s"(lds)
                 : "memory");
}
__device__ __forceinline__ void lds_dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ unsigned lds_addr(const double *p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) double *)p;
}
#ifndef SML_GDIAG
#define SML_GDIAG 0
#endif
__global__ __launch_bounds__(256, 2) void k_train_gram2(const double *__restrict__ S, const double *__restrict__ T,
                                                     const TrainRegion *__restrict__ regs, int m, int nout, int npad,
                                                     double *__restrict__ G, double *__restrict__ B) {
    __shared__ double sm[2][2][kKC][kLdsLd2];  // [stage buffer][A, B][time row][row]: one LDS object
    const int r = blockIdx.y;
    const TrainRegion R = regs[r];
    const int C = npad / kTile;
    int bi, bj;
    bool strip;
    if (!tile_of(blockIdx.x, C, &bi, &bj, &strip)) return;
    const int Cr = (R.naug + kTile - 1) / kTile;
    if ((strip ? bj : bi) >= Cr) return;  // padding (bi >= bj)
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1, l16 = lane & 15, kk = lane >> 4;
    const double *Sr = S + R.s_off, *Tr = T + R.t_off;
    const int naug = R.naug;
    // a wave whose 64 x 64 sub-tile holds no output (rows past naug / nout, columns
    // past naug, or above the diagonal of a diagonal tile) loads its share of the LDS
    // stages and skips its MFMAs, leaving the SIMD to the other block's waves
    const bool wlive = (bi * kTile + wr * 64 < (strip ? nout : naug)) && (bj * kTile + wc * 64 < naug) &&
                       !(!strip && bi == bj && wr < wc);
    // and inside a live wave, its 16-row / 16-column MFMA tiles past naug / nout
    const int ni = min(4, max(0, ((strip ? nout : naug) - bi * kTile - wr * 64 + 15) / 16));
    const int nj = min(4, max(0, (naug - bj * kTile - wc * 64 + 15) / 16));
    const bool full = ni == 4 && nj == 4;
    // LDS staging: a thread moves row pairs (2 r2, 2 r2 + 1) of time rows tq + 4 q, one
    // 16-B load and one 16-B LDS store each (4 + 4 per stage: the stage's instruction
    // count is what bounds the kernel).  Rows and steps clamped into the
    // operand, so the loads are unconditional; the values past naug / nout / m are
    // selected to 0 at the store, after the load's wait (a select right after the load
    // would wait there, and the stage ahead would not be a prefetch) -- on the tiles at a
    // region's edge only
    const int r2 = tid & 63, tq = __builtin_amdgcn_readfirstlane(tid >> 6);  // the time row: per wave
    const int rowsA = strip ? nout : naug;
    const int ar = bi * kTile + 2 * r2, br = bj * kTile + 2 * r2;
    const int ac = min(ar, rowsA - 2), bc = min(br, naug - 2);  // nout, naug >= 2
    // a scalar base per time row plus the lane's row offset
    const double *pa = (strip ? Tr : Sr) + bi * kTile, *pb = Sr + bj * kTile;
    const int oa = ac - bi * kTile, ob = bc - bj * kTile;
    const long long lda = rowsA;
    const bool inner = __builtin_amdgcn_readfirstlane(bi * kTile + kTile <= rowsA && bj * kTile + kTile <= naug &&
                                                      m % kKC == 0);
#if SML_GDIAG == 1  // diagnostic: every block reads region 0's first 128 rows (L2-resident)
    pa = pb = S;
#endif
    d2 ra[kKC / 4], rb[kKC / 4];
    auto fetch = [&](int t0) {
#pragma unroll
        for (int q = 0; q < kKC / 4; ++q) {
            const long long tc = min(t0 + tq + 4 * q, m - 1);
#if SML_GDIAG == 2  // diagnostic: no global load
            ra[q] = rb[q] = d2{(double)(tc & 7), 1.0};
#else
            ra[q] = *(const d2 *)(pa + tc * lda + oa);
            rb[q] = *(const d2 *)(pb + tc * naug + ob);
#endif
        }
    };
    // the pair as loaded from the clamped start c, for rows (x, x + 1) of n
    auto pick = [](d2 v, int x, int c, int n, bool t_ok) {
        return d2{t_ok && x < n ? (x == c ? v.x : v.y) : 0.0, t_ok && x + 1 < n && x == c ? v.y : 0.0};
    };
    auto store = [&](int buf, int t0) {
#pragma unroll
        for (int q = 0; q < kKC / 4; ++q) {
            d2 va = ra[q], vb = rb[q];
            if (!inner) {
                const bool t_ok = t0 + tq + 4 * q < m;
                va = pick(va, ar, ac, rowsA, t_ok);
                vb = pick(vb, br, bc, naug, t_ok);
            }
            *(d2 *)&sm[buf][0][tq + 4 * q][2 * r2] = va;
            *(d2 *)&sm[buf][1][tq + 4 * q][2 * r2] = vb;
        }
    };
    d4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = d4{0, 0, 0, 0};
    auto compute = [&](int cur) {
        const double(*sA)[kLdsLd2] = sm[cur][0];
        const double(*sB)[kLdsLd2] = sm[cur][1];
        if (wlive && full) {  // wave-uniform; the stage's four k-steps one branch-free block,
                              // so step s + 1's LDS reads issue under step s's MFMAs
#pragma unroll
            for (int s = 0; s < kKC / 4; ++s) {
                double a[4], b[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = sA[4 * s + kk][wr * 64 + i * 16 + l16];
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = sB[4 * s + kk][wc * 64 + j * 16 + l16];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j) acc[i][j] = MFMA64(a[i], b[j], acc[i][j]);
            }
        } else if (wlive) {  // a tile at a region's edge
#pragma unroll
            for (int s = 0; s < kKC / 4; ++s) {
                double a[4], b[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) a[i] = sA[4 * s + kk][wr * 64 + i * 16 + l16];
#pragma unroll
                for (int j = 0; j < 4; ++j) b[j] = sB[4 * s + kk][wc * 64 + j * 16 + l16];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (i < ni && j < nj) acc[i][j] = MFMA64(a[i], b[j], acc[i][j]);
            }
        }
    };
    // inner tiles with 16-B-aligned operand rows: the stages filled by LDS-DMA (a wave
    // copies time rows 4 w .. 4 w + 3 of A and of B, one 1-KiB instruction each), the
    // next stage's copies issued before this stage's MFMAs
    const bool glds = inner && __builtin_amdgcn_readfirstlane((((size_t)pa | (size_t)pb) & 15) == 0 &&
                                                              (lda & 1) == 0 && (naug & 1) == 0);
    if (glds && SML_GDIAG == 0) {
        const int wu = __builtin_amdgcn_readfirstlane(w);
        auto dma = [&](int buf, int t0) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const long long t = t0 + 4 * wu + u;
                lds_dma16(pa + t * lda + 2 * lane, lds_addr(&sm[buf][0][4 * wu + u][0]));
                lds_dma16(pb + t * naug + 2 * lane, lds_addr(&sm[buf][1][4 * wu + u][0]));
            }
        };
        dma(0, 0);
        lds_dma_wait();
        __syncthreads();
        int cur = 0;
        for (int t0 = 0; t0 < m; t0 += kKC) {
            if (t0 + kKC < m) dma(cur ^ 1, t0 + kKC);
            compute(cur);
            lds_dma_wait();
            __syncthreads();
            cur ^= 1;
        }
    } else {
        fetch(0);
        store(0, 0);
        __syncthreads();
        if (kKC < m) fetch(kKC);
        int cur = 0;
        for (int t0 = 0; t0 < m; t0 += kKC) {
            compute(cur);
#if SML_GDIAG != 3  // diagnostic 3: the stages are never refilled
            if (t0 + kKC < m) {
                store(cur ^ 1, t0 + kKC);
                if (t0 + 2 * kKC < m) fetch(t0 + 2 * kKC);
            }
#endif
            __syncthreads();
            cur ^= 1;
        }
    }
    if (!wlive) return;
    double *Gr = G + (size_t)r * npad * npad;
    double *Br = B + (size_t)r * npad * nout;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = bi * kTile + wr * 64 + i * 16 + kk + 4 * q;
                const int col = bj * kTile + wc * 64 + j * 16 + l16;
                if (strip) {
                    if (row < nout) {
                        double *p = Br + (size_t)row * npad + col;
                        *p = *p + acc[i][j][q];
                    }
                } else {
                    double *p = Gr + (size_t)col * npad + row;
                    *p = *p + acc[i][j][q];
                }
            }
}

// fit_chunk_hybrid regularisation on the padded, column-major Gram:
// diag(i) += beta_model (i < ncs) / beta_res (i < naug); padding diag = 1, prior on B
__global__ void k_train_regularise(double *__restrict__ G, double *__restrict__ B,
                                   const TrainRegion *__restrict__ regs, int npad, int nout, int ncs,
                                   double add_model, double add_res, double prior) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (i >= npad) return;
    const int naug = regs[r].naug;
    double *g = G + (size_t)r * npad * npad + (size_t)i * npad + i;
    if (i < naug)
        *g = *g + (i < ncs ? add_model : add_res);
    else
        *g = 1.0;
    if (prior != 0.0 && i < ncs && i < nout) {
        double *b = B + (size_t)r * npad * nout + (size_t)i * npad + i;  // b_trans(i, i)
        *b = *b + prior;
    }
}

// solution X(j, o) (npad x nout per region) -> wout(nout, naug) column-major: a
// transpose through LDS, 32 j per block -- read along j, write along o, both coalesced
constexpr int kWoutJ = 32;
__global__ __launch_bounds__(256) void k_train_wout(const double *__restrict__ X, const TrainRegion *__restrict__ regs,
                                                    int npad, int nout, const long long *__restrict__ wout_off,
                                                    double *__restrict__ wout) {
    __shared__ double tile[kWoutJ][kRhs + 1];
    const int j0 = blockIdx.x * kWoutJ, r = blockIdx.y, tid = threadIdx.x;
    const int naug = regs[r].naug;
    if (j0 >= naug) return;
    const double *x = X + (size_t)r * npad * nout;
    for (int idx = tid; idx < kWoutJ * nout; idx += 256) {
        const int o = idx / kWoutJ, jj = idx % kWoutJ;
        tile[jj][o] = j0 + jj < naug ? x[(size_t)o * npad + j0 + jj] : 0.0;
    }
    __syncthreads();
    double *w = wout + wout_off[r] + (size_t)j0 * nout;
    const int nj = min(kWoutJ, naug - j0);
    for (int idx = tid; idx < nj * nout; idx += 256) w[idx] = tile[idx / nout][idx % nout];
}

// ------------------------------------------------------------ batched Cholesky
// a wave's LDS operations complete in issue order: a fence for the compiler and a wave
// barrier order one lane's LDS writes before another lane's reads
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// One TR x TC output tile (4 waves, wave (wr, wc) owns (TR/2) x (TC/2) = (TR/32) x
// (TC/32) MFMA 16x16 tiles):
//   O(r, c) = (accumulate ? O(r, c) : 0) + alpha * sum_{l < K} A(r, l) B(c, l)
// A is TR x K, B is TC x K (K a multiple of 16), both column-major (A(r, l) at
// pa[l * lda + r]); rows >= arows / brows are not stored.  O is column-major: O(r, c) at
// po[c * ldo + r].  128 x 128 tiles for the wide trailing update, 64-wide ones for
// the narrow launches (panel, triangular solves), where one tile's MFMA chain is the
// launch's latency.
// lower: the tile is on the diagonal of a symmetric update and only its lower triangle
// is read later -- the wave above the diagonal (wr < wc) loads its share of the LDS
// stages and skips its MFMAs and stores.  KC: values of l per LDS stage (the MFMA chain
// of an element runs over l in the same order whatever KC)
// DMA (the 128 x 128 trailing update): the stages double-buffered and filled by LDS-DMA as
// k_train_gram2's inner tiles (a wave copies 4 time rows of A and of B per stage, one
// 1-KiB instruction each), the next stage's copies issued before this stage's MFMAs
// DW: lower's waves on the diagonal also skip their 16 x 16 tiles above it (a separate
// instance: in the trailing update the branch costs more registers than it saves)
template <int TR, int TC, int KC = kKC, bool DMA = false, bool DW = false>
__device__ __forceinline__ void gemm_tile(const double *__restrict__ pa, long long lda, int arows,
                                          const double *__restrict__ pb, long long ldb, int brows, double *po,
                                          long long ldo, double alpha, bool accumulate, int K = kTile,
                                          bool lower = false, bool te = false) {
    constexpr int NI = TR / 32, NJ = TC / 32, NB = DMA ? 2 : 1;
    static_assert(!DMA || (TR == 128 && TC == 128 && KC == 16), "LDS-DMA: one 128-row time row per instruction");
    __shared__ double sA_[NB][KC][TR + kLdsPad];
    __shared__ double sB_[NB][KC][TC + kLdsPad];
    double(*sA)[TR + kLdsPad] = sA_[0];
    double(*sB)[TC + kLdsPad] = sB_[0];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1, l16 = lane & 15, kk = lane >> 4;
    // LDS staging as k_train_gram2's: row pairs (2 p, 2 p + 1) of time rows u + TQ q, one
    // 16-B load and one 16-B LDS store each; every caller passes whole tiles (arows = TR,
    // brows = TC, the rows of G's / linv's blocks), so the loads are unmasked
    constexpr int RPA = TR / 2, RPB = TC / 2, TQA = 256 / RPA, TQB = 256 / RPB;
    constexpr int NQA = KC / TQA, NQB = KC / TQB;
    static_assert(NQA * TQA == KC && NQB * TQB == KC, "stage rows");
    const int pa2 = tid % RPA, pb2 = tid % RPB;
    const int ua = RPA == 64 ? __builtin_amdgcn_readfirstlane(tid / RPA) : tid / RPA;
    const int ub = RPB == 64 ? __builtin_amdgcn_readfirstlane(tid / RPB) : tid / RPB;
    d2 ra[NQA], rb[NQB];
    auto fetch = [&](int t0) {
#pragma unroll
        for (int q = 0; q < NQA; ++q) ra[q] = *(const d2 *)(pa + (long long)(t0 + ua + TQA * q) * lda + 2 * pa2);
#pragma unroll
        for (int q = 0; q < NQB; ++q) rb[q] = *(const d2 *)(pb + (long long)(t0 + ub + TQB * q) * ldb + 2 * pb2);
    };
    d4 acc[NI][NJ];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = d4{0, 0, 0, 0};
    // rows at or past arows (a region's last, partial block: padding, whose rows of L are
    // 0) take nothing from the GEMM: a wave whose rows all lie there skips its MFMAs, and
    // the epilogue does not store them -- bitwise what the full tile leaves there
    // lower, the waves on the diagonal (wr = wc): their 16 x 16 tiles above the diagonal
    // are not read later either, so they are skipped (left 0, stored as + 0)
    const bool wlive = !(lower && wr < wc) && wr * (TR / 2) < arows;
    const bool dw = DW && __builtin_amdgcn_readfirstlane(lower && wr == wc);
    auto compute = [&](const double(*cA)[TR + kLdsPad], const double(*cB)[TC + kLdsPad]) {
        if (!wlive) return;  // wave-uniform
        if (dw) {
            static_assert(TR != TC || NI == NJ, "square wave tiles");
#pragma unroll
            for (int s = 0; s < KC / 4; ++s) {
                double a[NI], b[NJ];
#pragma unroll
                for (int i = 0; i < NI; ++i) a[i] = cA[4 * s + kk][wr * (TR / 2) + i * 16 + l16];
#pragma unroll
                for (int j = 0; j < NJ; ++j) b[j] = cB[4 * s + kk][wc * (TC / 2) + j * 16 + l16];
#pragma unroll
                for (int i = 0; i < NI; ++i)
#pragma unroll
                    for (int j = 0; j <= i && j < NJ; ++j) acc[i][j] = MFMA64(a[i], b[j], acc[i][j]);
            }
            return;
        }
#pragma unroll
        for (int s = 0; s < KC / 4; ++s) {
            double a[NI], b[NJ];
#pragma unroll
            for (int i = 0; i < NI; ++i) a[i] = cA[4 * s + kk][wr * (TR / 2) + i * 16 + l16];
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = cB[4 * s + kk][wc * (TC / 2) + j * 16 + l16];
#pragma unroll
            for (int i = 0; i < NI; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = MFMA64(a[i], b[j], acc[i][j]);
        }
    };
    if constexpr (DMA) {
        const int wu = __builtin_amdgcn_readfirstlane(w);
        auto dma = [&](int buf, int t0) {
#pragma unroll
            for (int u = 0; u < KC / 4; ++u) {
                const long long t = t0 + 4 * wu + u;
                lds_dma16(pa + t * lda + 2 * lane, lds_addr(&sA_[buf][4 * wu + u][0]));
                lds_dma16(pb + t * ldb + 2 * lane, lds_addr(&sB_[buf][4 * wu + u][0]));
            }
        };
        __syncthreads();  // a previous tile's readers of these stages (k_chol_upanel's two calls)
        dma(0, 0);
        lds_dma_wait();
        __syncthreads();
        int cur = 0;
        for (int t0 = 0; t0 < K; t0 += KC) {
            if (t0 + KC < K) dma(cur ^ 1, t0 + KC);
            compute(sA_[cur], sB_[cur]);
            lds_dma_wait();
            __syncthreads();
            cur ^= 1;
        }
    } else {
    fetch(0);
    for (int t0 = 0; t0 < K; t0 += KC) {
        __syncthreads();
#pragma unroll
        for (int q = 0; q < NQA; ++q) *(d2 *)&sA[ua + TQA * q][2 * pa2] = ra[q];
#pragma unroll
        for (int q = 0; q < NQB; ++q) *(d2 *)&sB[ub + TQB * q][2 * pb2] = rb[q];
        __syncthreads();
        if (t0 + KC < K) fetch(t0 + KC);
        compute(sA, sB);
    }
    }
    if (te) {
        // each 16 x 16 tile transposed through the wave's LDS scratch (sA, free after the
        // last stage; gemm_rhs's te): a read-modify-write instruction covers 16 consecutive
        // rows of 4 columns, whole 128-B lines; the same expression per element
        static_assert(KC * (TR + kLdsPad) >= 4 * 16 * 17, "the waves' transpose scratch fits in sA");
        __syncthreads();
        if (lower && wr < wc) return;
        double *scr = &sA[0][0] + w * (16 * 17);
        const int a = lane >> 4, b = lane & 15;
#pragma unroll
        for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) scr[l16 * 17 + kk + 4 * q] = acc[i][j][q];
                wave_sync();
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int row = wr * (TR / 2) + i * 16 + b, col = wc * (TC / 2) + j * 16 + 4 * q + a;
                    const double v = scr[(4 * q + a) * 17 + b];
                    if (row < arows && col < brows) {
                        double *p = po + (long long)col * ldo + row;
                        *p = (accumulate ? *p : 0.0) + alpha * v;
                    }
                }
                wave_sync();
            }
        return;
    }
    if (lower && wr < wc) return;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = wr * (TR / 2) + i * 16 + kk + 4 * q;
                const int col = wc * (TC / 2) + j * 16 + l16;
                if (row < arows && col < brows) {
                    double *p = po + (long long)col * ldo + row;
                    *p = (accumulate ? *p : 0.0) + alpha * acc[i][j][q];
                }
            }
}

constexpr int kDiagThreads = 1024;            // 8 threads per row of the diagonal block
constexpr int kDiagLd = kTile + 1;            // LDS row stride (doubles)
constexpr int kDiagH = kDiagThreads / kTile;  // entries of a row per thread stride
constexpr size_t kDiagLds = (size_t)(kTile * kDiagLd + 2 * kTile) * sizeof(double);

// Diagonal block k of every region, A_kk = L_kk L_kk^T and X = L_kk^-1: L_kk goes back
// to G (lower triangle), L_kk^-1 (column-major, zeros above the diagonal) to linv for
// the panel GEMM and the triangular solves, and potrf's info (first non-positive
// pivot, 1-based global index) -- from the 128 x 128 block as sub-blocks of kSub
// columns.  Sub-block P: one wave factors its kSub x kSub diagonal block and inverts
// it (potrf's unblocked column steps restricted to the sub-block, no workgroup barrier: the wave's LDS operations complete in order); every wave then
// forms the rows below, L_IP = A_IP X_PP^T, and the trailing update inside the block,
// A_IJ -= L_IP L_JP^T, as 16 x 16 f64 MFMA tiles from LDS.  After the last sub-block
// the inverse's off-diagonal blocks, X_IJ = -X_II sum_{J <= K < I} L_IK X_KJ, row of
// blocks by row.  About 20 workgroup barriers instead of the column-by-column form's
// 256 (r05: 269 -> 122 us per launch); the same factorisation up to rounding (the
// update sums are blocked).
#ifndef SML_DIAG_SUB
#define SML_DIAG_SUB 16
#endif
constexpr int kSub = SML_DIAG_SUB;           // sub-block edge (16 or 32)
constexpr int kNS = kTile / kSub, kNT = kSub / 16;  // sub-blocks; 16-tiles per sub-block edge
constexpr int kSH = 64 / kSub;               // lanes per row in the sub-block steps
constexpr int kTs = kSub + 1;                // LDS stride of the T_J scratch blocks
constexpr size_t kDiagBLds = kDiagLds + (size_t)(kNS - 1) * kSub * kTs * sizeof(double);
static_assert(kSub == 16 || kSub == 32, "sub-block edge");

// phase stamps of k_chol_diag_b (profiling build, -DSML_DSTAMPS): thread 0 of block 0
// of the launch for block column g_dst_k records wall_clock64 at slot s
#ifdef SML_DSTAMPS
__device__ long long g_dst[32];
__device__ int g_dst_k = 0;
#define SML_DST(s)                                                                   \
    do {                                                                             \
        if (threadIdx.x == 0 && blockIdx.x == 0 && k == g_dst_k) g_dst[s] = wall_clock64(); \
    } while (0)
#else
#define SML_DST(s) \
    do {           \
    } while (0)
#endif

// one 16 x 16 tile of O = A B^T over K (a multiple of 4): fa(r, t), fb(c, t) for
// r, c < 16; acc[q] = O(kk + 4 q, l16) (lane = 16 kk + l16), gemm_tile's layout
template <class FA, class FB>
__device__ __forceinline__ d4 mfma_tile16(FA fa, FB fb, int K) {
    const int lane = threadIdx.x & 63, l16 = lane & 15, kk = lane >> 4;
    d4 acc = {0, 0, 0, 0};
    for (int t0 = 0; t0 < K; t0 += 4) acc = MFMA64(fa(l16, t0 + kk), fb(l16, t0 + kk), acc);
    return acc;
}

__global__ __launch_bounds__(kDiagThreads) void k_chol_diag_b(double *__restrict__ G, double *__restrict__ linv,
                                                              int npad, int k, int *__restrict__ info,
                                                              const TrainRegion *__restrict__ regs) {
    extern __shared__ double S[];  // S[i * kDiagLd + c]: L(i, c) for c < i, X(i, c) at S[c][i]
    double *ldg = S + kTile * kDiagLd, *xd = ldg + kTile, *Tb = xd + kTile;
    const int r = blockIdx.x, C = npad / kTile;
    if (k >= live_blocks(regs, r)) return;  // an identity block: L = L^-1 = I, already in G
    constexpr int ld = kDiagLd;
    const int tid = threadIdx.x, i = tid & (kTile - 1), h = tid >> 7;
    const int w = tid >> 6, lane = tid & 63, l16 = lane & 15, kk = lane >> 4;
    double *A = G + (size_t)r * npad * npad + (size_t)k * kTile * npad + (size_t)k * kTile;
    SML_DST(0);
    for (int c = h; c < kTile; c += kDiagH) S[i * ld + c] = c <= i ? A[(size_t)c * npad + i] : 0.0;
    // X(t, c) of the lower-triangular inverse (row t, column c; 0 above the diagonal)
    auto Xv = [&](int t, int c) { return t > c ? S[c * ld + t] : (t == c ? xd[t] : 0.0); };
    for (int P = 0; P < kNS; ++P) {
        const int o = P * kSub;
        __syncthreads();
        SML_DST(1 + 4 * P);
        if (w == 0) {  // the sub-block's column steps (potrf's unblocked ones, on rows / columns o..o+kSub-1)
            const int si = lane & (kSub - 1), sh = lane / kSub;
            for (int j = 0; j < kSub; ++j) {
                const double d = S[(o + j) * ld + o + j];
                const double inv = 1.0 / sqrt(d);
                if (lane == 0) {
                    ldg[o + j] = sqrt(d);
                    xd[o + j] = inv;
                    if (!(d > 0.0) && info[r] == 0) info[r] = k * kTile + o + j + 1;
                }
                if (sh == 0 && si > j) S[(o + si) * ld + o + j] *= inv;  // L(si, j)
                if (sh == kSH - 1 && si < j) S[(o + si) * ld + o + j] *= inv;  // X(j, c = si), stored at S[c][j]
                wave_sync();
                if (si > j) {
                    const double lij = S[(o + si) * ld + o + j];
                    double *Si = S + (o + si) * ld + o;
                    for (int l0 = j + 1 + sh; l0 <= si; l0 += 4 * kSH) {  // L(si, l) -= L(si, j) L(l, j)
                        double a[4], b[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int l = l0 + kSH * u;
                            if (l <= si) {
                                a[u] = Si[l];
                                b[u] = S[(o + l) * ld + o + j];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (l0 + kSH * u <= si) Si[l0 + kSH * u] = a[u] - lij * b[u];
                    }
                    for (int c0 = sh; c0 < j; c0 += 4 * kSH) {  // X(si, c) -= L(si, j) X(j, c)
                        double a[4], b[4];
#pragma unroll
                        for (int u = 0; u < 4; ++u) {
                            const int c = c0 + kSH * u;
                            if (c < j) {
                                a[u] = S[(o + c) * ld + o + si];
                                b[u] = S[(o + c) * ld + o + j];
                            }
                        }
#pragma unroll
                        for (int u = 0; u < 4; ++u)
                            if (c0 + kSH * u < j) S[(o + c0 + kSH * u) * ld + o + si] = a[u] - lij * b[u];
                    }
                    if (sh == kSH - 1) S[(o + j) * ld + o + si] -= lij * xd[o + j];  // X(si, j)
                }
                wave_sync();
            }
        }
        __syncthreads();
        SML_DST(2 + 4 * P);
        const int below = kTile - o - kSub;  // rows under the sub-block
        if (below == 0) break;
        // L_IP = A_IP X_PP^T (rows o+32.., columns o..o+31): every tile read before any is written
        const int ntp = kNT * (below / 16);
        d4 accp = {0, 0, 0, 0};
        int pr0 = 0, pc0 = 0;
        if (w < ntp) {
            pr0 = o + kSub + 16 * (w / kNT);
            pc0 = o + 16 * (w % kNT);
            accp = mfma_tile16([&](int rr, int t) { return S[(pr0 + rr) * ld + o + t]; },
                               [&](int cc, int t) { return Xv(pc0 + cc, o + t); }, kSub);
        }
        __syncthreads();
        if (w < ntp) {
#pragma unroll
            for (int q = 0; q < 4; ++q) S[(pr0 + kk + 4 * q) * ld + pc0 + l16] = accp[q];
        }
        __syncthreads();
        SML_DST(3 + 4 * P);
        // the trailing update inside the block: the lower-triangle 16-tiles (a >= b) of
        // rows / columns o+32..127, A(i, c) -= sum_t L(i, t) L(c, t), t in the sub-block
        const int nT = below / 16, ntu = nT * (nT + 1) / 2;
        for (int u = w; u < ntu; u += kDiagThreads / 64) {
            int a = 0, rem = u;
            while (rem > a) rem -= ++a;  // u = a (a + 1) / 2 + b
            const int b = rem;
            const int r0 = o + kSub + 16 * a, c0 = o + kSub + 16 * b;
            const d4 acc = mfma_tile16([&](int rr, int t) { return S[(r0 + rr) * ld + o + t]; },
                                       [&](int cc, int t) { return S[(c0 + cc) * ld + o + t]; }, kSub);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = r0 + kk + 4 * q, col = c0 + l16;
                if (a != b || col <= row) S[row * ld + col] -= acc[q];
            }
        }
    }
    SML_DST(17);
    // the inverse's off-diagonal blocks, block row I by block row:
    //   T_J = sum_{t in [32 J, 32 I)} L(32 I + u, t) X(t, 32 J + c);   X_IJ = -X_II T_J
    for (int I = 1; I < kNS; ++I) {
        const int oi = I * kSub;
        for (int u = w; u < kNT * kNT * I; u += kDiagThreads / 64) {
            const int J = u / (kNT * kNT), u0 = 16 * ((u / kNT) % kNT), c0 = 16 * (u % kNT), oj = J * kSub;
            const d4 acc = mfma_tile16([&](int rr, int t) { return S[(oi + u0 + rr) * ld + oj + t]; },
                                       [&](int cc, int t) { return Xv(oj + t, oj + c0 + cc); }, oi - oj);
#pragma unroll
            for (int q = 0; q < 4; ++q) Tb[J * kSub * kTs + (u0 + kk + 4 * q) * kTs + c0 + l16] = acc[q];
        }
        __syncthreads();
        for (int u = w; u < kNT * kNT * I; u += kDiagThreads / 64) {
            const int J = u / (kNT * kNT), u0 = 16 * ((u / kNT) % kNT), c0 = 16 * (u % kNT), oj = J * kSub;
            const double *TJ = Tb + J * kSub * kTs;
            const d4 acc = mfma_tile16([&](int rr, int v) { return Xv(oi + u0 + rr, oi + v); },
                                       [&](int cc, int v) { return TJ[v * kTs + c0 + cc]; }, kSub);
#pragma unroll
            for (int q = 0; q < 4; ++q) S[(oj + c0 + l16) * ld + oi + u0 + kk + 4 * q] = -acc[q];
        }
        __syncthreads();
    }
    SML_DST(18);
    double *Li = linv + ((size_t)r * C + k) * kTile * kTile;
    for (int c = h; c < kTile; c += kDiagH) {
        if (c <= i) A[(size_t)c * npad + i] = c < i ? S[i * ld + c] : ldg[i];
        Li[(size_t)c * kTile + i] = c < i ? S[c * ld + i] : (c == i ? xd[i] : 0.0);
    }
    __syncthreads();
    SML_DST(19);
}

// L_ik = A_ik L_kk^-T for the blocks i > k below the diagonal, in place: a block
// owns 64 rows x all 128 columns (it reads the whole rows it overwrites)
__global__ __launch_bounds__(256, 3) void k_chol_panel(double *__restrict__ G, const double *__restrict__ linv, int npad,
                                                    int k, const TrainRegion *__restrict__ regs, int te) {
    const int r = blockIdx.y, C = npad / kTile, i = k + 1 + (blockIdx.x >> 1), r0 = (blockIdx.x & 1) * 64;
    const int rows = min(64, regs[r].naug - i * kTile - r0);  // the slab's data rows
    if (rows <= 0) return;  // A_ik = 0: L_ik = 0 (padding)
    double *Gr = G + (size_t)r * npad * npad;
    double *A = Gr + (size_t)k * kTile * npad + (size_t)i * kTile + r0;
    const double *Li = linv + ((size_t)r * C + k) * kTile * kTile;
    gemm_tile<64, 128>(A, npad, rows, Li, kTile, kTile, A, npad, 1.0, false, kTile, false, te != 0);
}

#ifndef SML_UPD_DMA
#define SML_UPD_DMA 1
#endif
// A_ij -= sum_{k0 <= k < k0 + kw} L_ik L_jk^T for the lower-triangle tiles j <= i
// of block columns jlo <= j < jhi: one GEMM of depth 128 kw per tile (the block
// columns of L are contiguous in the column-major G).  KC: the GEMM's LDS stage depth
// (16; 32-deep stages spilled at two waves per SIMD)
template <int KC>
__global__ __launch_bounds__(256, 2) void k_chol_update(double *__restrict__ G, int npad, int k0, int kw, int jlo,
                                                     int jhi, const TrainRegion *__restrict__ regs) {
    const int r = blockIdx.y, C = npad / kTile;
    int idx = blockIdx.x, j = jlo;
    while (j < jhi && idx >= C - j) idx -= C - j++;
    if (j >= jhi) return;
    const int i = j + idx;
    if (i >= live_blocks(regs, r)) return;  // L_ik = 0 for the padding rows (i >= j > k)
    double *Gr = G + (size_t)r * npad * npad;
    const double *Lik = Gr + (size_t)k0 * kTile * npad + (size_t)i * kTile;
    const double *Ljk = Gr + (size_t)k0 * kTile * npad + (size_t)j * kTile;
    double *Aij = Gr + (size_t)j * kTile * npad + (size_t)i * kTile;
    const int rows = min(kTile, regs[r].naug - i * kTile);  // block row i's data rows
    gemm_tile<128, 128, KC, SML_UPD_DMA>(Lik, npad, rows, Ljk, npad, kTile, Aij, npad, -1.0, true, kw * kTile,
                                          i == j);
}

// Block column k > k0 of a panel below its diagonal, fused (k_chol_update then
// k_chol_panel as one launch): rows r0 .. r0 + 63 of block i take the left-looking
// update by the panel's earlier block columns k0 .. k - 1 (k_chol_update's GEMM, in place),
// then L_ik = A_ik L_kk^-T (k_chol_panel's GEMM) on the same rows, read back from L2 by the
// workgroup that wrote them -- one HBM read of the slab instead of two, one launch fewer
// per block column.  The same sums per element as the two launches (the tile shape does
// not change an element's MFMA chain), so the factor is bitwise the same.
__global__ __launch_bounds__(256, 3) void k_chol_upanel(double *__restrict__ G, const double *__restrict__ linv,
                                                     int npad, int k0, int k, const TrainRegion *__restrict__ regs,
                                                     int te) {
    const int r = blockIdx.y, C = npad / kTile, i = k + 1 + (blockIdx.x >> 1), r0 = (blockIdx.x & 1) * 64;
    const int rows = min(64, regs[r].naug - i * kTile - r0);  // the slab's data rows
    if (rows <= 0) return;  // A_ik = 0: L_ik = 0 (padding)
    double *Gr = G + (size_t)r * npad * npad;
    const double *Lip = Gr + (size_t)k0 * kTile * npad + (size_t)i * kTile + r0;
    const double *Lkp = Gr + (size_t)k0 * kTile * npad + (size_t)k * kTile;
    double *A = Gr + (size_t)k * kTile * npad + (size_t)i * kTile + r0;
    gemm_tile<64, 128>(Lip, npad, rows, Lkp, npad, kTile, A, npad, -1.0, true, (k - k0) * kTile, false, te != 0);
    __syncthreads();  // the slab's updated rows, stored by every wave, before any is read
    const double *Li = linv + ((size_t)r * C + k) * kTile * kTile;
    gemm_tile<64, 128>(A, npad, rows, Li, kTile, kTile, A, npad, 1.0, false, kTile, false, te != 0);
}

// The left-looking update of a panel's diagonal tile (k, k) by block columns k0 .. k - 1
// on the fused path, as three workgroups per region: the 64 x 64 quadrants (0, 0), (1, 0),
// (1, 1) -- exactly the waves k_chol_update's lower tile runs (its quadrant above the
// diagonal skipped), each quadrant's chain on four waves instead of one, three times
// the workgroups for a launch of one tile per region.  Bitwise the 128 x 128 form.
__global__ __launch_bounds__(256, 2) void k_chol_update_diag(double *__restrict__ G, int npad, int k0, int k,
                                                          const TrainRegion *__restrict__ regs, int te) {
    const int r = blockIdx.y, q = blockIdx.x, r0 = q == 0 ? 0 : 64, c0 = q == 2 ? 64 : 0;
    if (k >= live_blocks(regs, r)) return;  // (padding block columns are never factored)
    double *Gr = G + (size_t)r * npad * npad;
    const double *Lkp = Gr + (size_t)k0 * kTile * npad + (size_t)k * kTile;
    double *Akk = Gr + (size_t)k * kTile * npad + (size_t)k * kTile;
    gemm_tile<64, 64, kKC, false, true>(Lkp + r0, npad, 64, Lkp + c0, npad, 64, Akk + (size_t)c0 * npad + r0, npad,
                                        -1.0, true, (k - k0) * kTile, q != 1, te != 0);  // (0, 0), (1, 1): diagonal
}

static int update_tiles(int C, int jlo, int jhi) {
    int n = 0;
    for (int j = jlo; j < jhi; ++j) n += C - j;
    return n;
}

// One 128 x NC tile of the triangular solves (NC = kRhs: all right-hand sides at
// once, so a block of L is read once per pass; NC = kRhs / 3 for the latency-bound
// in-panel launches, three blocks per tile row): 4 waves stacked by rows, each 32
// rows x NC columns = 2 x NC / 16 MFMA tiles;
//   O(r, c) = (accumulate ? O(r, c) : 0) + alpha * sum_{l < K} A(r, l) B(c, l)
// A(r, l) at pa[l * lda + r] (AT = false) or pa[r * lda + l] (AT = true); B(c, l) at
// pb[c * ldb + l] (a row range of the right-hand sides), columns c >= nb read as zero
// and are not stored.
template <bool AT, int NC>
__device__ __forceinline__ void gemm_rhs(const double *__restrict__ pa, long long lda, const double *__restrict__ pb,
                                         long long ldb, int nb, double *po, long long ldo, double alpha,
                                         bool accumulate, int K = kTile, bool te = false, int arows = kTile) {
    constexpr int NJ = NC / 16;
    static_assert(NC % 16 == 0, "column group");
    __shared__ double sA[kKC][kTile + kLdsPad];
    __shared__ double sB[kKC][NC + kLdsPad];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, l16 = lane & 15, kk = lane >> 4;
    // 16-B loads as gemm_tile's.  A column-major (AT = false): row pairs of time rows;
    // transposed (AT = true, A(r, l) at pa[r * lda + l]): l pairs (2 lp, 2 lp + 1) of
    // rows ar + 32 q, two LDS stores each.  B: l pairs of columns c = idx / 8, the columns
    // past nb loaded from column nb - 1 and selected to 0 at the LDS store
    constexpr int NQA = 4, NPB = NC * kKC / 2, NQB = (NPB + 255) / 256;
    const int pa2 = tid & 63, ua = __builtin_amdgcn_readfirstlane(tid >> 6);  // AT = false
    const int lp = tid & 7, ar = tid >> 3;                                     // AT = true
    d2 ra[NQA], rb[NQB];
    auto fetch = [&](int t0) {
#pragma unroll
        for (int q = 0; q < NQA; ++q)
            ra[q] = AT ? *(const d2 *)(pa + (long long)(ar + 32 * q) * lda + t0 + 2 * lp)
                       : *(const d2 *)(pa + (long long)(t0 + ua + 4 * q) * lda + 2 * pa2);
#pragma unroll
        for (int q = 0; q < NQB; ++q) {
            const int idx = min(tid + 256 * q, NPB - 1), c = min(idx >> 3, nb - 1);
            rb[q] = *(const d2 *)(pb + (long long)c * ldb + t0 + 2 * (idx & 7));
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int q = 0; q < NQA; ++q) {
            if (AT) {
                sA[2 * lp][ar + 32 * q] = ra[q].x;
                sA[2 * lp + 1][ar + 32 * q] = ra[q].y;
            } else {
                *(d2 *)&sA[ua + 4 * q][2 * pa2] = ra[q];
            }
        }
#pragma unroll
        for (int q = 0; q < NQB; ++q) {
            const int idx = tid + 256 * q, c = idx >> 3;
            if (idx < NPB) {
                sB[2 * (idx & 7)][c] = c < nb ? rb[q].x : 0.0;
                sB[2 * (idx & 7) + 1][c] = c < nb ? rb[q].y : 0.0;
            }
        }
    };
    d4 acc[2][NJ];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = d4{0, 0, 0, 0};
    fetch(0);
    for (int t0 = 0; t0 < K; t0 += kKC) {
        __syncthreads();
        store();
        __syncthreads();
        if (t0 + kKC < K) fetch(t0 + kKC);
        if (w * 32 >= arows) continue;  // wave-uniform: rows of a partial last block's padding
#pragma unroll
        for (int s = 0; s < kKC / 4; ++s) {
            double a[2], b[NJ];
#pragma unroll
            for (int i = 0; i < 2; ++i) a[i] = sA[4 * s + kk][w * 32 + i * 16 + l16];
#pragma unroll
            for (int j = 0; j < NJ; ++j) b[j] = sB[4 * s + kk][j * 16 + l16];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NJ; ++j) acc[i][j] = MFMA64(a[i], b[j], acc[i][j]);
        }
    }
    if (te) {
        // each 16 x 16 tile transposed through the wave's LDS scratch (sA, free after the
        // last stage), so a read-modify-write instruction covers 16 consecutive rows of 4
        // columns (whole 128-B lines) instead of 4 rows of 16; the same expression per element
        __syncthreads();
        double *scr = &sA[0][0] + w * (16 * 17);
        const int a = lane >> 4, b = lane & 15;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
#pragma unroll
                for (int q = 0; q < 4; ++q) scr[l16 * 17 + kk + 4 * q] = acc[i][j][q];
                wave_sync();
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = 4 * q + a, row = w * 32 + i * 16 + b, col = j * 16 + c;
                    const double v = scr[c * 17 + b];
                    if (col < nb && row < arows) {
                        double *p = po + (long long)col * ldo + row;
                        *p = (accumulate ? *p : 0.0) + alpha * v;
                    }
                }
                wave_sync();
            }
        return;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int row = w * 32 + i * 16 + kk + 4 * q, col = j * 16 + l16;
                if (col < nb && row < arows) {
                    double *p = po + (long long)col * ldo + row;
                    *p = (accumulate ? *p : 0.0) + alpha * acc[i][j][q];
                }
            }
}

// Update of block rows ilo <= i < ihi by the solved block rows [k0, k0 + kw), one
// GEMM of depth 128 kw per block row:
//   forward:  B_i -= sum_k L_ik Y_k        backward: B_i -= sum_k L_ki^T X_k
template <bool upper, int NC>
__global__ __launch_bounds__(256, 2) void k_solve_update(const double *__restrict__ G, double *__restrict__ B, int npad,
                                                      int nout, int k0, int kw, int ilo,
                                                      const TrainRegion *__restrict__ regs, int te) {
    const int r = blockIdx.y, i = ilo + (int)blockIdx.x, c0 = NC * blockIdx.z;
    const int Cr = live_blocks(regs, r);
    // padding block rows stay 0; backward, solved rows k0.. past the data are 0
    if (i >= Cr || (upper && k0 >= Cr) || c0 >= nout) return;
    const double *Gr = G + (size_t)r * npad * npad;
    double *Br = B + (size_t)r * npad * nout + (size_t)c0 * npad;
    const int rows = min(kTile, regs[r].naug - i * kTile);  // block row i's data rows
    if constexpr (upper)  // A(rr, l) = L(k0 kTile + l, i kTile + rr): the transposed blocks (k, i)
        gemm_rhs<true, NC>(Gr + (size_t)i * kTile * npad + (size_t)k0 * kTile, npad, Br + (size_t)k0 * kTile, npad,
                           nout - c0, Br + (size_t)i * kTile, npad, -1.0, true, kw * kTile, te != 0, rows);
    else
        gemm_rhs<false, NC>(Gr + (size_t)k0 * kTile * npad + (size_t)i * kTile, npad, Br + (size_t)k0 * kTile, npad,
                            nout - c0, Br + (size_t)i * kTile, npad, -1.0, true, kw * kTile, te != 0, rows);
}

// A block row of a panel's triangular solve in one launch, left-looking (k_chol_upanel's
// form for the solves): the row's update by the panel's rows already solved, then its
// diagonal block -- forward (upper = 0) for block row i of panel [p0, p1):
//   B_i -= sum_{p0 <= k < i} L_ik Y_k,  Y_i = L_ii^-1 B_i
// backward (upper = 1): B_i -= sum_{i < k < p1} L_ki^T X_k,  X_i = L_ii^-T B_i.
// Each output column's sum is the right-looking form's, the depth-128 terms gathered
// into one GEMM (the same products, summed in one MFMA chain instead of several
// read-modify-writes: agrees to rounding); one launch per block row instead of two
// per block column, the update and the diagonal block on the same workgroup
template <bool upper, int NC>
__global__ __launch_bounds__(256, 2) void k_solve_lpanel(const double *__restrict__ linv, const double *__restrict__ G,
                                                      double *__restrict__ B, int npad, int nout, int p0, int p1,
                                                      int i, const TrainRegion *__restrict__ regs, int te) {
    const int r = blockIdx.y, C = npad / kTile, c0 = NC * blockIdx.z;
    const int Cr = live_blocks(regs, r);
    if (i >= Cr || c0 >= nout) return;  // padding block rows stay 0
    const double *Gr = G + (size_t)r * npad * npad;
    double *Br = B + (size_t)r * npad * nout + (size_t)c0 * npad;
    double *Bi = Br + (size_t)i * kTile;
    const int rows = min(kTile, regs[r].naug - i * kTile);  // block row i's data rows
    if constexpr (upper) {
        const int k1 = min(p1, Cr);  // solved rows i + 1 .. k1 - 1 (X past the data is 0)
        if (k1 > i + 1)
            gemm_rhs<true, NC>(Gr + (size_t)i * kTile * npad + (size_t)(i + 1) * kTile, npad,
                               Br + (size_t)(i + 1) * kTile, npad, nout - c0, Bi, npad, -1.0, true,
                               (k1 - 1 - i) * kTile, te != 0, rows);
    } else {
        if (i > p0)
            gemm_rhs<false, NC>(Gr + (size_t)p0 * kTile * npad + (size_t)i * kTile, npad, Br + (size_t)p0 * kTile,
                                npad, nout - c0, Bi, npad, -1.0, true, (i - p0) * kTile, te != 0, rows);
    }
    __syncthreads();  // the row's updated values, stored by every wave, before any is read
    const double *Li = linv + ((size_t)r * C + i) * kTile * kTile;
    gemm_rhs<upper, NC>(Li, kTile, Bi, npad, nout - c0, Bi, npad, 1.0, false, kTile, te != 0, rows);
}

}  // namespace

struct sml_train {
    int nlocal = 0, nout = 0, npad = 0, C = 0;
    int panel = kPanel;  // block columns per Cholesky panel (sml_train_set_panel)
    std::vector<int> naug;
    TrainRegion *d_regs = nullptr;
    double *d_G = nullptr, *d_B = nullptr;
    long long *d_wout_off = nullptr;
    double *d_linv = nullptr;  // L_kk^-1 per region and block column (C x 128 x 128)
    int *d_info = nullptr;
    long long s_total = 0, t_total = 0;
    int last_m = -1;
    // the forward substitution's stream (beside the factorisation, sml_train_solve) and
    // its fork / join events, created on the first solve
    hipStream_t fwd = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

static void set_offsets(sml_train *t, int m, std::vector<TrainRegion> &h) {
    long long so = 0, to = 0;
    for (int i = 0; i < t->nlocal; ++i) {
        h[i].s_off = so;
        h[i].t_off = to;
        h[i].naug = t->naug[i];
        so += (long long)t->naug[i] * m;
        to += (long long)t->nout * m;
    }
}

extern "C" int sml_train_destroy(sml_train *t) {
    if (!t) return SML_OK;
    void *ptrs[] = {t->d_regs, t->d_G, t->d_B, t->d_wout_off, t->d_info, t->d_linv};
    for (void *p : ptrs)
        if (p) (void)hipFree(p);
    if (t->ev_fork) (void)hipEventDestroy(t->ev_fork);
    if (t->ev_join) (void)hipEventDestroy(t->ev_join);
    if (t->fwd) (void)hipStreamDestroy(t->fwd);
    delete t;
    return SML_OK;
}

extern "C" int sml_train_create(int nlocal, const int *naug, int nout, sml_train **out) {
    SML_REQUIRE(out && naug && nlocal > 0, "bad argument");
    SML_REQUIRE(nout > 0 && nout <= kRhs, "nout must be in 1..144");
    *out = nullptr;
    sml_train *t = new (std::nothrow) sml_train();
    if (!t) return fail(SML_ERR_NOMEM, "host allocation failed");
    t->nlocal = nlocal;
    t->nout = nout;
    t->naug.assign(naug, naug + nlocal);
    int mx = 0;
    for (int i = 0; i < nlocal; ++i) {
        if (naug[i] <= 0) {
            delete t;
            return fail(SML_ERR_ARG, "naug[%d] = %d", i, naug[i]);
        }
        mx = naug[i] > mx ? naug[i] : mx;
    }
    t->npad = (mx + kTile - 1) / kTile * kTile;  // uniform padded size: one batched solve
    t->C = t->npad / kTile;
    const size_t g = (size_t)nlocal * t->npad * t->npad, b = (size_t)nlocal * t->npad * nout;
    hipError_t e;
    if ((e = hipMalloc(&t->d_G, g * 8)) != hipSuccess || (e = hipMalloc(&t->d_B, b * 8)) != hipSuccess ||
        (e = hipMalloc(&t->d_regs, nlocal * sizeof(TrainRegion))) != hipSuccess ||
        (e = hipMalloc(&t->d_wout_off, nlocal * sizeof(long long))) != hipSuccess ||
        (e = hipMalloc(&t->d_info, nlocal * sizeof(int))) != hipSuccess ||
        (e = hipMalloc(&t->d_linv, (size_t)nlocal * t->C * kTile * kTile * 8)) != hipSuccess) {
        sml_train_destroy(t);
        return fail(SML_ERR_NOMEM, "sml_train_create: %s (%.2f GB of Gram matrices)", hipGetErrorString(e),
                    g * 8e-9);
    }
    std::vector<long long> wo(nlocal);
    long long off = 0;
    for (int i = 0; i < nlocal; ++i) {
        wo[i] = off;
        off += (long long)nout * naug[i];
    }
    SML_HIP(hipMemcpy(t->d_wout_off, wo.data(), nlocal * sizeof(long long), hipMemcpyHostToDevice));
    static bool lds_set = false;
    if (!lds_set) {
        SML_HIP(hipFuncSetAttribute((const void *)k_chol_diag_b, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)kDiagBLds));
        lds_set = true;
    }
    *out = t;
    return sml_train_reset(t, nullptr);
}

extern "C" int sml_train_reset(sml_train *t, void *stream) {
    SML_REQUIRE(t, "null context");
    const size_t g = (size_t)t->nlocal * t->npad * t->npad, b = (size_t)t->nlocal * t->npad * t->nout;
    SML_HIP(hipMemsetAsync(t->d_G, 0, g * 8, (hipStream_t)stream));
    SML_HIP(hipMemsetAsync(t->d_B, 0, b * 8, (hipStream_t)stream));
    return SML_OK;
}

extern "C" int sml_train_accumulate(sml_train *t, const double *d_states, const double *d_targets, int m,
                                    void *stream) {
    SML_REQUIRE(t && d_states && d_targets && m > 0, "bad argument");
    if (m != t->last_m) {
        std::vector<TrainRegion> h(t->nlocal);
        set_offsets(t, m, h);
        SML_HIP(hipMemcpy(t->d_regs, h.data(), h.size() * sizeof(TrainRegion), hipMemcpyHostToDevice));
        t->last_m = m;
    }
    const int tiles = t->C * (t->C + 1) / 2 + kStrip * t->C;
    hipLaunchKernelGGL(k_train_gram2, dim3(tiles, t->nlocal), dim3(256), 0, (hipStream_t)stream, d_states, d_targets,
                       t->d_regs, m, t->nout, t->npad, t->d_G, t->d_B);
    SML_HIP(hipGetLastError());
    return SML_OK;
}

extern "C" int sml_train_solve(sml_train *t, int ncs, double beta_res, double beta_model, int using_prior,
                               double prior_val, double *d_wout, int *info, void *stream) {
    SML_REQUIRE(t && d_wout, "bad argument");
    SML_REQUIRE(ncs >= 0, "ncs must be >= 0");
    if (t->last_m < 0) {  // regions table (offsets unused by the solve)
        std::vector<TrainRegion> h(t->nlocal);
        set_offsets(t, 1, h);
        SML_HIP(hipMemcpy(t->d_regs, h.data(), h.size() * sizeof(TrainRegion), hipMemcpyHostToDevice));
        t->last_m = 1;
    }
    hipStream_t st = (hipStream_t)stream;
    const double add_model = using_prior ? beta_model * beta_model : beta_model;
    const double add_res = using_prior ? beta_res * beta_res : beta_res;
    const double prior = using_prior ? prior_val * beta_model * beta_model : 0.0;
    hipLaunchKernelGGL(k_train_regularise, dim3((t->npad + 255) / 256, t->nlocal), dim3(256), 0, st, t->d_G, t->d_B,
                       t->d_regs, t->npad, t->nout, ncs, add_model, add_res, prior);
    SML_HIP(hipGetLastError());
    SML_HIP(hipMemsetAsync(t->d_info, 0, t->nlocal * sizeof(int), st));
    const int C = t->C, nl = t->nlocal, npad = t->npad, nout = t->nout;
    // potrs, blocked by panels of P block rows: inside a panel, left-looking (block row i
    // of the panel takes the update by the panel's rows already solved, then its diagonal
    // inverse: k_solve_lpanel, latency-bound, one launch per row); then the rows beyond
    // the panel take the whole panel's update at depth 128 P (MFMA-bound).  The in-panel
    // launches in three column groups of the right-hand sides, their epilogues through an
    // LDS transpose (te); the wide ones whole, stored directly.
    //
    // The forward substitution L Y = B of panel p reads only the factor's block columns
    // of panels <= p (final once panel p's columns are done: later panels write columns
    // >= p1 only) and writes only B, which the factorisation never reads, so it runs on
    // a second stream forked after each panel's columns, beside the factorisation of the
    // later panels: its latency-bound in-panel launches fill the CUs the diagonal factors
    // (one workgroup per region) leave idle.  Every kernel and every element's sums are
    // the same as on one stream (bitwise); the backward substitution joins after both.
    constexpr int kG = kRhs / 3;
    const dim3 g1(1, nl, 3);
    const int te = 1;
    if (!t->fwd) {
        SML_HIP(hipStreamCreateWithFlags(&t->fwd, hipStreamNonBlocking));
        SML_HIP(hipEventCreateWithFlags(&t->ev_fork, hipEventDisableTiming));
        SML_HIP(hipEventCreateWithFlags(&t->ev_join, hipEventDisableTiming));
    }
    hipStream_t fw = t->fwd;
    auto forward_panel = [&](int p0, int p1) {  // L Y = B for block rows p0 .. p1 - 1
        for (int i = p0; i < p1; ++i)
            hipLaunchKernelGGL((k_solve_lpanel<false, kG>), g1, dim3(256), 0, fw, t->d_linv, t->d_G, t->d_B, npad,
                               nout, p0, p1, i, t->d_regs, te);
        if (p1 < C)
            hipLaunchKernelGGL((k_solve_update<false, kRhs>), dim3(C - p1, nl), dim3(256), 0, fw, t->d_G, t->d_B, npad,
                               nout, p0, p1 - p0, p1, t->d_regs, 0);
    };
    // potrf: G = L L^T over panels of t->panel block columns.  Inside a panel,
    // left-looking: block column k first takes the update from the panel's earlier
    // columns (depth 128 (k - p0)), then its diagonal factor and L_ik below it;
    // after the panel, one right-looking update of the whole trailing matrix at
    // depth 128 x panel.  Block column k > p0 of a panel: its diagonal tile's update
    // (three quadrant workgroups), the diagonal factor, then the update and L_ik of the
    // blocks below fused (k_chol_upanel); the panel's first column: the factor and
    // k_chol_panel.  The shallow launches store through an LDS transpose (cte).
    // (A lookahead split of the trailing update -- the next panel's columns on the chain,
    // the rest on a third stream beside the next panel's factorisation -- measured no
    // better, and slower on a default-priority chain: DESIGN.md §3.4.)
    const int P = t->panel, cte = 1;
    for (int p0 = 0; p0 < C; p0 += P) {
        const int p1 = std::min(C, p0 + P);
        for (int k = p0; k < p1; ++k) {
            const bool fused = k > p0;
            if (fused)
                hipLaunchKernelGGL(k_chol_update_diag, dim3(3, nl), dim3(256), 0, st, t->d_G, npad, p0, k, t->d_regs,
                                   cte);
            hipLaunchKernelGGL(k_chol_diag_b, dim3(nl), dim3(kDiagThreads), kDiagBLds, st, t->d_G, t->d_linv, npad, k,
                               t->d_info, t->d_regs);
            if (k < C - 1 && fused)
                hipLaunchKernelGGL(k_chol_upanel, dim3(2 * (C - 1 - k), nl), dim3(256), 0, st, t->d_G, t->d_linv,
                                   npad, p0, k, t->d_regs, cte);
            else if (k < C - 1)
                hipLaunchKernelGGL(k_chol_panel, dim3(2 * (C - 1 - k), nl), dim3(256), 0, st, t->d_G, t->d_linv,
                                   npad, k, t->d_regs, cte);
        }
        SML_HIP(hipGetLastError());
        // fork: panel p's forward substitution behind its columns (and, on fw, behind
        // the earlier panels' forward substitution)
        SML_HIP(hipEventRecord(t->ev_fork, st));
        SML_HIP(hipStreamWaitEvent(fw, t->ev_fork, 0));
        forward_panel(p0, p1);
        SML_HIP(hipGetLastError());
        if (p1 < C)  // the trailing update (the factorisation's largest launch)
            hipLaunchKernelGGL(k_chol_update<kKC>, dim3(update_tiles(C, p1, C), nl), dim3(256), 0, st, t->d_G, npad, p0,
                               p1 - p0, p1, C, t->d_regs);
    }
    // join: the backward substitution reads Y
    SML_HIP(hipEventRecord(t->ev_join, fw));
    SML_HIP(hipStreamWaitEvent(st, t->ev_join, 0));
    for (int p1 = C; p1 > 0; p1 -= P) {  // L^T X = Y, panels from the bottom
        const int p0 = std::max(0, p1 - P);
        for (int i = p1 - 1; i >= p0; --i)
            hipLaunchKernelGGL((k_solve_lpanel<true, kG>), g1, dim3(256), 0, st, t->d_linv, t->d_G, t->d_B, npad,
                               nout, p0, p1, i, t->d_regs, te);
        if (p0 > 0)
            hipLaunchKernelGGL((k_solve_update<true, kRhs>), dim3(p0, nl), dim3(256), 0, st, t->d_G, t->d_B, npad, nout,
                               p0, p1 - p0, 0, t->d_regs, 0);
    }
    SML_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_train_wout, dim3(t->npad / kWoutJ, t->nlocal), dim3(256), 0, st, t->d_B, t->d_regs,
                       t->npad, t->nout, t->d_wout_off, d_wout);
    SML_HIP(hipGetLastError());
    if (info) SML_HIP(hipMemcpyAsync(info, t->d_info, t->nlocal * sizeof(int), hipMemcpyDeviceToHost, st));
    return SML_OK;
}

// block columns per Cholesky panel (default 8): the trailing update's depth is 128 x P
extern "C" int sml_train_set_panel(sml_train *t, int panel) {
    SML_REQUIRE(t && panel >= 1, "bad argument");
    t->panel = panel;
    return SML_OK;
}

extern "C" int sml_train_npad(const sml_train *t, int *npad) {
    SML_REQUIRE(t && npad, "null argument");
    *npad = t->npad;
    return SML_OK;
}

extern "C" int sml_train_get_gram(sml_train *t, int i, double *G, double *B) {
    SML_REQUIRE(t && i >= 0 && i < t->nlocal, "bad region index");
    SML_HIP(hipDeviceSynchronize());
    const size_t g = (size_t)t->npad * t->npad, b = (size_t)t->npad * t->nout;
    if (G) SML_HIP(hipMemcpy(G, t->d_G + i * g, g * 8, hipMemcpyDeviceToHost));
    if (B) SML_HIP(hipMemcpy(B, t->d_B + i * b, b * 8, hipMemcpyDeviceToHost));
    return SML_OK;
}

// ------------------------------------------------------------------ measurement
// Back-to-back v_mfma_f64_16x16x4_f64 with 8 independent accumulators per wave on
// every SIMD: the chip's sustained fp64 MFMA rate, the `peak` of the training
// roofline (MI355X_MICROARCH.md lists no fp64 MFMA figure).
namespace {
// stamps (optional): thread 0 of each block records the core-clock counter
// (s_memtime) and the 100-MHz real-time counter (s_memrealtime) around its loop, so
// the host gets the clock the chip held under the load (MI355X_MICROARCH.md, DVFS
// give-back item 6: the in-kernel clock = d memtime / d memrealtime x 100 MHz)
__global__ __launch_bounds__(256) void k_probe_mfma_f64(int iters, double *sink, long long *stamps) {
    d4 acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = d4{0, 0, 0, 0};
    double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - threadIdx.x * 1e-9;
    long long c0 = 0, r0 = 0;
    if (stamps && threadIdx.x == 0) {
        c0 = clock64();
        r0 = wall_clock64();
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = MFMA64(a, b, acc[i]);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    if (s == 12345.678) sink[0] = s;  // keep the chain live
    if (stamps && threadIdx.x == 0) {
        stamps[2 * blockIdx.x] = clock64() - c0;
        stamps[2 * blockIdx.x + 1] = wall_clock64() - r0;
    }
}
}  // namespace

// the sustained fp64 MFMA rate and, when ghz is given, the median in-kernel core
// clock of the timed run (GHz)
extern "C" int sml_probe_mfma_f64_clock(int iters, double *tflops, double *ghz) {
    SML_REQUIRE(tflops && iters > 0, "bad argument");
    int dev = 0, ncu = 0;
    SML_HIP(hipGetDevice(&dev));
    SML_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const int blocks = ncu * 2;  // 8 waves per CU = 2 per SIMD
    double *sink = nullptr;
    long long *stamps = nullptr;
    SML_HIP(hipMalloc(&sink, 8));
    if (ghz) SML_HIP(hipMalloc(&stamps, (size_t)2 * blocks * sizeof(long long)));
    hipEvent_t e0, e1;
    SML_HIP(hipEventCreate(&e0));
    SML_HIP(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_probe_mfma_f64, dim3(blocks), dim3(256), 0, nullptr, iters / 10, sink, nullptr);  // warm-up
    SML_HIP(hipEventRecord(e0, nullptr));
    hipLaunchKernelGGL(k_probe_mfma_f64, dim3(blocks), dim3(256), 0, nullptr, iters, sink, stamps);
    SML_HIP(hipEventRecord(e1, nullptr));
    SML_HIP(hipEventSynchronize(e1));
    float ms = 0;
    SML_HIP(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(sink);
    const double flops = (double)blocks * 4 * iters * 8 * 2.0 * 16 * 16 * 4;
    *tflops = flops / (ms * 1e-3) / 1e12;
    if (ghz) {
        std::vector<long long> h((size_t)2 * blocks);
        SML_HIP(hipMemcpy(h.data(), stamps, h.size() * sizeof(long long), hipMemcpyDeviceToHost));
        (void)hipFree(stamps);
        std::vector<double> f;
        for (int b = 0; b < blocks; ++b)
            if (h[2 * b + 1] > 0) f.push_back((double)h[2 * b] / (double)h[2 * b + 1] * 0.1);  // 100 MHz -> GHz
        std::sort(f.begin(), f.end());
        *ghz = f.empty() ? 0.0 : f[f.size() / 2];
    }
    return SML_OK;
}

extern "C" int sml_probe_mfma_f64(int iters, double *tflops) { return sml_probe_mfma_f64_clock(iters, tflops, nullptr); }

#ifdef SML_DSTAMPS
// diagnostic (profiling build): the stamps of k_chol_diag_b's launch for block column k
extern "C" int sml_dbg_diag_stamps(int k, long long *out) {
    SML_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dst_k), &k, sizeof(int), 0, hipMemcpyHostToDevice));
    if (!out) return SML_OK;
    SML_HIP(hipDeviceSynchronize());
    SML_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dst), sizeof(long long) * 32, 0, hipMemcpyDeviceToHost));
    return SML_OK;
}
#endif

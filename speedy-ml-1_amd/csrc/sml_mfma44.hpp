// sml_mfma44.hpp -- a 16x16x4 fp64 MFMA step as four v_mfma_f64_4x4x4_f64.
//
// On gfx950 v_mfma_f64_16x16x4_f64 (2048 flop) issues once per ~105 clk per SIMD
// (47.9 TFLOP/s chip-wide at the 2.39 GHz the chip holds), while v_mfma_f64_4x4x4_f64
// (four independent 4x4x4 blocks, 512 flop) issues once per ~16.7 clk (75 TFLOP/s, 0.96
// of the nominal 78.6): tools/probe_mfma_f64.hip.  Its lanes (tools/probe_mfma44_layout.hip):
//   A: lane 16k + 4b + i = A_b[i][k]    B: lane 16k + 4b + j = B_b[k][j]    D: lane 16i + 4b + j = C_b[i][j]
// With the 16x16x4 operands as they are (a: lane l = A[l % 16][l / 16], b: lane l =
// B[l / 16][l % 16]), instruction q takes b rotated by 4q lanes within each row of 16
// (DPP), so block b of instruction q is the 4x4 tile (rows 4b.., columns
// 4((b + q) % 4)..) of the 16x16 product: the four instructions cover it once.  The
// accumulators stay in that form through the K loop; acc44_to_d4 re-lays them out
// once, at the end, as v_mfma_f64_16x16x4_f64's result (lane l, item q = C[l / 16 + 4q][l % 16]),
// so the kernels' epilogues are unchanged.
#pragma once
#include <hip/hip_runtime.h>

namespace sml {

typedef double mfma_d4 __attribute__((ext_vector_type(4)));

struct Acc44 {
    double q[4];
};

__device__ __forceinline__ Acc44 acc44_zero() { return Acc44{{0.0, 0.0, 0.0, 0.0}}; }

// DPP row_ror:N on a double (dst lane x = src lane x - N within its row of 16)
template <int N>
__device__ __forceinline__ double dpp_row_ror(double v) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const int lo = __builtin_amdgcn_mov_dpp((int)(unsigned)u, 0x120 + N, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), 0x120 + N, 0xf, 0xf, false);
    return __builtin_bit_cast(double, ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo);
}

// b rotated for instructions 1, 2, 3: lane x takes b from lane x + 4q (mod 16 within its row)
struct B44 {
    double r[4];
};
__device__ __forceinline__ B44 b44(double b) { return B44{{b, dpp_row_ror<12>(b), dpp_row_ror<8>(b), dpp_row_ror<4>(b)}}; }

__device__ __forceinline__ void mfma44(double a, const B44 &b, Acc44 &c) {
#pragma unroll
    for (int q = 0; q < 4; ++q) c.q[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b.r[q], c.q[q], 0, 0, 0);
}

// the 16x16 tile in v_mfma_f64_16x16x4_f64's result layout, through a wave-private
// LDS scratch of 256 doubles (the caller's block must not be using it)
__device__ __forceinline__ mfma_d4 acc44_to_d4(const Acc44 &c, double *scr) {
    const int L = threadIdx.x & 63, i = L >> 4, b = (L >> 2) & 3, j = L & 3;
#pragma unroll
    for (int q = 0; q < 4; ++q) scr[(4 * b + i) * 16 + 4 * ((b + q) & 3) + j] = c.q[q];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    mfma_d4 out;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[q] = scr[((L >> 4) + 4 * q) * 16 + (L & 15)];
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    return out;
}

}  // namespace sml

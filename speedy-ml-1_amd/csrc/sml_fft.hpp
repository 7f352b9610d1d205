// sml_fft.hpp -- the real FFT of SPEEDY's longitude axis (n = ix = 96) on gfx950,
// in FFTPACK's algorithm and operation order, so the Fourier stage of grid/spec is
// bit-identical to the reference's (gridx / specx call rfftb / rfftf,
// src/spe_subfft_fftpack.f90:15-87; the FFTPACK routines are
// src/spe_subfft_fftpack2.f90: rffti1 :36-100, rfftb1 :102-165, rfftf1 :167-231,
// radb2/3/4 :233-448, radf2/3/4 :741-950).
//
// rffti1 factors 96 as ifac = (4, 2, 4, 4, 3) (a 2 found after other factors moves
// to the front), so the backward transform is radb2(ido 48, l1 1) -> radb4(12, 2)
// -> radb4(3, 8) -> radb3(1, 32) and the forward one radf3(1, 32) -> radf4(3, 8) ->
// radf4(12, 2) -> radf2(48, 1), each pass between two buffers.
//
// GPU form: many transforms at once, each array held in LDS element-major
// (element e of transform f at buf[e * ld + f], so the lanes of a wave that work on
// neighbouring transforms touch neighbouring words); P threads share one transform
// and split each pass's independent butterflies (the reference's k / i loop
// iterations), with a block barrier between passes.  The twiddles wa are
// rffti1's (host: sml_fft_twiddles), in the order FFTPACK stores them.
#pragma once

#include <cmath>

namespace sml {

constexpr int kFftN = 96;
constexpr int kFftWa = 96;  // wa(1:94) used

// rffti1's twiddle table for n = 96 (wa(i-1) = cos, wa(i) = sin of fi * ld * 2 pi / n,
// in double like the reference's -fdefault-real-8 build)
inline void sml_fft_twiddles(double *wa) {
    const int ifac[4] = {2, 4, 4, 3};
    for (int i = 0; i < kFftWa; ++i) wa[i] = 0.0;
    const double tpi = 8. * std::atan(1.);
    const double argh = tpi / kFftN;
    int is = 0, l1 = 1;
    for (int k1 = 0; k1 < 3; ++k1) {  // nfm1 = nf - 1 = 3
        const int ip = ifac[k1], l2 = l1 * ip, ido = kFftN / l2;
        int ld = 0;
        for (int j = 1; j <= ip - 1; ++j) {
            ld += l1;
            int i = is;
            const double argld = ld * argh;
            double fi = 0.;
            for (int ii = 3; ii <= ido; ii += 2) {
                i += 2;
                fi = fi + 1.;
                const double arg = fi * argld;
                wa[i - 2] = std::cos(arg);  // wa(i-1), 1-based
                wa[i - 1] = std::sin(arg);  // wa(i)
            }
            is += ido;
        }
        l1 = l2;
    }
}

#if defined(__HIPCC__) || defined(SML_FFT_HOST)
#ifndef __HIPCC__  // host-only build (oracle/fft_check.cpp): plain functions
#define __device__
#define __host__
#endif
#ifdef __HIP_DEVICE_COMPILE__
#define SML_FFT_SYNC() __syncthreads()
#else
#define SML_FFT_SYNC() ((void)0)
#endif
namespace fft {

// Passes read one array and write the other: both are __restrict__ so the loads of
// later butterflies can be issued ahead of the stores of earlier ones; the item
// loops have compile-time trip counts (threads past the end skip the body) so they
// unroll.  Arrays are element-major: element e (1-based) of the transform at
// p[(e - 1) * ld].
#define SML_FFT_ITEMS(N, P, ...)                                        \
    _Pragma("unroll") for (int q_ = 0; q_ < ((N) + (P) - 1) / (P); ++q_) { \
        const int it = t + q_ * (P);                                    \
        if (it < (N)) __VA_ARGS__                                       \
    }

// radb2 (:233-281): cc(ido, 2, l1) -> ch(ido, l1, 2)
template <int IDO, int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radb2(const double *__restrict__ c, double *__restrict__ h, int ld,
                                      const double *__restrict__ wa1, int t) {
    auto cc = [&](int i, int j, int k) { return c[(i - 1 + IDO * ((j - 1) + 2 * (k - 1))) * ld]; };
    auto ch = [&](int i, int k, int j) -> double & { return h[(i - 1 + IDO * ((k - 1) + L1 * (j - 1))) * ld]; };
    constexpr int NB = (IDO - 1) / 2, NI = 1 + (IDO > 2 ? NB : 0) + (IDO % 2 == 0 ? 1 : 0);
    SML_FFT_ITEMS(NI * L1, P, {
        const int k = it / NI + 1, s = it % NI;
        if (s == 0) {
            ch(1, k, 1) = cc(1, 1, k) + cc(IDO, 2, k);
            ch(1, k, 2) = cc(1, 1, k) - cc(IDO, 2, k);
        } else if (IDO > 2 && s <= NB) {
            const int i = 2 * s + 1, ic = IDO + 2 - i;
            ch(i - 1, k, 1) = cc(i - 1, 1, k) + cc(ic - 1, 2, k);
            const double tr2 = cc(i - 1, 1, k) - cc(ic - 1, 2, k);
            ch(i, k, 1) = cc(i, 1, k) - cc(ic, 2, k);
            const double ti2 = cc(i, 1, k) + cc(ic, 2, k);
            ch(i - 1, k, 2) = wa1[i - 3] * tr2 - wa1[i - 2] * ti2;
            ch(i, k, 2) = wa1[i - 3] * ti2 + wa1[i - 2] * tr2;
        } else {  // ido even (:105-106)
            ch(IDO, k, 1) = cc(IDO, 1, k) + cc(IDO, 1, k);
            ch(IDO, k, 2) = -(cc(1, 2, k) + cc(1, 2, k));
        }
    })
}

// radb3 (:283-351) for ido = 1: cc(1, 3, l1) -> ch(1, l1, 3)
template <int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radb3_ido1(const double *__restrict__ c, double *__restrict__ h, int ld, int t) {
    const double taur = -.5, taui = .5 * sqrt(3.);
    SML_FFT_ITEMS(L1, P, {
        const int k = it + 1;
        auto cc = [&](int j) { return c[((j - 1) + 3 * (k - 1)) * ld]; };
        auto ch = [&](int j) -> double & { return h[((k - 1) + L1 * (j - 1)) * ld]; };
        const double tr2 = cc(2) + cc(2);
        const double cr2 = cc(1) + taur * tr2;
        ch(1) = cc(1) + tr2;
        const double ci3 = taui * (cc(3) + cc(3));
        ch(2) = cr2 - ci3;
        ch(3) = cr2 + ci3;
    })
}

// radb4 (:353-447): cc(ido, 4, l1) -> ch(ido, l1, 4)
template <int IDO, int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radb4(const double *__restrict__ c, double *__restrict__ h, int ld,
                                      const double *__restrict__ wa1, const double *__restrict__ wa2,
                                      const double *__restrict__ wa3, int t) {
    auto cc = [&](int i, int j, int k) { return c[(i - 1 + IDO * ((j - 1) + 4 * (k - 1))) * ld]; };
    auto ch = [&](int i, int k, int j) -> double & { return h[(i - 1 + IDO * ((k - 1) + L1 * (j - 1))) * ld]; };
    const double sqrt2 = sqrt(2.);
    constexpr int NB = (IDO - 1) / 2, NI = 1 + (IDO > 2 ? NB : 0) + (IDO % 2 == 0 ? 1 : 0);
    SML_FFT_ITEMS(NI * L1, P, {
        const int k = it / NI + 1, s = it % NI;
        if (s == 0) {
            const double tr1 = cc(1, 1, k) - cc(IDO, 4, k);
            const double tr2 = cc(1, 1, k) + cc(IDO, 4, k);
            const double tr3 = cc(IDO, 2, k) + cc(IDO, 2, k);
            const double tr4 = cc(1, 3, k) + cc(1, 3, k);
            ch(1, k, 1) = tr2 + tr3;
            ch(1, k, 2) = tr1 - tr4;
            ch(1, k, 3) = tr2 - tr3;
            ch(1, k, 4) = tr1 + tr4;
        } else if (IDO > 2 && s <= NB) {
            const int i = 2 * s + 1, ic = IDO + 2 - i;
            const double ti1 = cc(i, 1, k) + cc(ic, 4, k);
            const double ti2 = cc(i, 1, k) - cc(ic, 4, k);
            const double ti3 = cc(i, 3, k) - cc(ic, 2, k);
            const double tr4 = cc(i, 3, k) + cc(ic, 2, k);
            const double tr1 = cc(i - 1, 1, k) - cc(ic - 1, 4, k);
            const double tr2 = cc(i - 1, 1, k) + cc(ic - 1, 4, k);
            const double ti4 = cc(i - 1, 3, k) - cc(ic - 1, 2, k);
            const double tr3 = cc(i - 1, 3, k) + cc(ic - 1, 2, k);
            ch(i - 1, k, 1) = tr2 + tr3;
            const double cr3 = tr2 - tr3;
            ch(i, k, 1) = ti2 + ti3;
            const double ci3 = ti2 - ti3;
            const double cr2 = tr1 - tr4;
            const double cr4 = tr1 + tr4;
            const double ci2 = ti1 + ti4;
            const double ci4 = ti1 - ti4;
            ch(i - 1, k, 2) = wa1[i - 3] * cr2 - wa1[i - 2] * ci2;
            ch(i, k, 2) = wa1[i - 3] * ci2 + wa1[i - 2] * cr2;
            ch(i - 1, k, 3) = wa2[i - 3] * cr3 - wa2[i - 2] * ci3;
            ch(i, k, 3) = wa2[i - 3] * ci3 + wa2[i - 2] * cr3;
            ch(i - 1, k, 4) = wa3[i - 3] * cr4 - wa3[i - 2] * ci4;
            ch(i, k, 4) = wa3[i - 3] * ci4 + wa3[i - 2] * cr4;
        } else {  // ido even (:105-106)
            const double ti1 = cc(1, 2, k) + cc(1, 4, k);
            const double ti2 = cc(1, 4, k) - cc(1, 2, k);
            const double tr1 = cc(IDO, 1, k) - cc(IDO, 3, k);
            const double tr2 = cc(IDO, 1, k) + cc(IDO, 3, k);
            ch(IDO, k, 1) = tr2 + tr2;
            ch(IDO, k, 2) = sqrt2 * (tr1 - ti1);
            ch(IDO, k, 3) = ti2 + ti2;
            ch(IDO, k, 4) = -sqrt2 * (tr1 + ti1);
        }
    })
}

// radf2 (:741-789): cc(ido, l1, 2) -> ch(ido, 2, l1)
template <int IDO, int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radf2(const double *__restrict__ c, double *__restrict__ h, int ld,
                                      const double *__restrict__ wa1, int t) {
    auto cc = [&](int i, int k, int j) { return c[(i - 1 + IDO * ((k - 1) + L1 * (j - 1))) * ld]; };
    auto ch = [&](int i, int j, int k) -> double & { return h[(i - 1 + IDO * ((j - 1) + 2 * (k - 1))) * ld]; };
    constexpr int NB = (IDO - 1) / 2, NI = 1 + (IDO > 2 ? NB : 0) + (IDO % 2 == 0 ? 1 : 0);
    SML_FFT_ITEMS(NI * L1, P, {
        const int k = it / NI + 1, s = it % NI;
        if (s == 0) {
            ch(1, 1, k) = cc(1, k, 1) + cc(1, k, 2);
            ch(IDO, 2, k) = cc(1, k, 1) - cc(1, k, 2);
        } else if (IDO > 2 && s <= NB) {
            const int i = 2 * s + 1, ic = IDO + 2 - i;
            const double tr2 = wa1[i - 3] * cc(i - 1, k, 2) + wa1[i - 2] * cc(i, k, 2);
            const double ti2 = wa1[i - 3] * cc(i, k, 2) - wa1[i - 2] * cc(i - 1, k, 2);
            ch(i, 1, k) = cc(i, k, 1) + ti2;
            ch(ic, 2, k) = ti2 - cc(i, k, 1);
            ch(i - 1, 1, k) = cc(i - 1, k, 1) + tr2;
            ch(ic - 1, 2, k) = cc(i - 1, k, 1) - tr2;
        } else {  // ido even (:105-106)
            ch(1, 2, k) = -cc(IDO, k, 2);
            ch(IDO, 1, k) = cc(IDO, k, 1);
        }
    })
}

// radf3 (:791-857) for ido = 1: cc(1, l1, 3) -> ch(1, 3, l1)
template <int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radf3_ido1(const double *__restrict__ c, double *__restrict__ h, int ld, int t) {
    const double taur = -.5, taui = .5 * sqrt(3.);
    SML_FFT_ITEMS(L1, P, {
        const int k = it + 1;
        auto cc = [&](int j) { return c[((k - 1) + L1 * (j - 1)) * ld]; };
        auto ch = [&](int j) -> double & { return h[((j - 1) + 3 * (k - 1)) * ld]; };
        const double cr2 = cc(2) + cc(3);
        ch(1) = cc(1) + cr2;
        ch(3) = taui * (cc(3) - cc(2));
        ch(2) = cc(1) + taur * cr2;  // ch(ido, 2, k) with ido = 1
    })
}

// radf4 (:859-950): cc(ido, l1, 4) -> ch(ido, 4, l1)
template <int IDO, int L1, int P>
__host__ __device__ __attribute__((always_inline)) inline void radf4(const double *__restrict__ c, double *__restrict__ h, int ld,
                                      const double *__restrict__ wa1, const double *__restrict__ wa2,
                                      const double *__restrict__ wa3, int t) {
    auto cc = [&](int i, int k, int j) { return c[(i - 1 + IDO * ((k - 1) + L1 * (j - 1))) * ld]; };
    auto ch = [&](int i, int j, int k) -> double & { return h[(i - 1 + IDO * ((j - 1) + 4 * (k - 1))) * ld]; };
    const double hsqt2 = .5 * sqrt(2.);
    constexpr int NB = (IDO - 1) / 2, NI = 1 + (IDO > 2 ? NB : 0) + (IDO % 2 == 0 ? 1 : 0);
    SML_FFT_ITEMS(NI * L1, P, {
        const int k = it / NI + 1, s = it % NI;
        if (s == 0) {
            const double tr1 = cc(1, k, 2) + cc(1, k, 4);
            const double tr2 = cc(1, k, 1) + cc(1, k, 3);
            ch(1, 1, k) = tr1 + tr2;
            ch(IDO, 4, k) = tr2 - tr1;
            ch(IDO, 2, k) = cc(1, k, 1) - cc(1, k, 3);
            ch(1, 3, k) = cc(1, k, 4) - cc(1, k, 2);
        } else if (IDO > 2 && s <= NB) {
            const int i = 2 * s + 1, ic = IDO + 2 - i;
            const double cr2 = wa1[i - 3] * cc(i - 1, k, 2) + wa1[i - 2] * cc(i, k, 2);
            const double ci2 = wa1[i - 3] * cc(i, k, 2) - wa1[i - 2] * cc(i - 1, k, 2);
            const double cr3 = wa2[i - 3] * cc(i - 1, k, 3) + wa2[i - 2] * cc(i, k, 3);
            const double ci3 = wa2[i - 3] * cc(i, k, 3) - wa2[i - 2] * cc(i - 1, k, 3);
            const double cr4 = wa3[i - 3] * cc(i - 1, k, 4) + wa3[i - 2] * cc(i, k, 4);
            const double ci4 = wa3[i - 3] * cc(i, k, 4) - wa3[i - 2] * cc(i - 1, k, 4);
            const double tr1 = cr2 + cr4;
            const double tr4 = cr4 - cr2;
            const double ti1 = ci2 + ci4;
            const double ti4 = ci2 - ci4;
            const double ti2 = cc(i, k, 1) + ci3;
            const double ti3 = cc(i, k, 1) - ci3;
            const double tr2 = cc(i - 1, k, 1) + cr3;
            const double tr3 = cc(i - 1, k, 1) - cr3;
            ch(i - 1, 1, k) = tr1 + tr2;
            ch(ic - 1, 4, k) = tr2 - tr1;
            ch(i, 1, k) = ti1 + ti2;
            ch(ic, 4, k) = ti1 - ti2;
            ch(i - 1, 3, k) = ti4 + tr3;
            ch(ic - 1, 2, k) = tr3 - ti4;
            ch(i, 3, k) = tr4 + ti3;
            ch(ic, 2, k) = tr4 - ti3;
        } else {  // ido even (:105-106)
            const double ti1 = -hsqt2 * (cc(IDO, k, 2) + cc(IDO, k, 4));
            const double tr1 = hsqt2 * (cc(IDO, k, 2) - cc(IDO, k, 4));
            ch(IDO, 1, k) = tr1 + cc(IDO, k, 1);
            ch(IDO, 3, k) = cc(IDO, k, 1) - tr1;
            ch(1, 2, k) = ti1 - cc(IDO, k, 3);
            ch(1, 4, k) = ti1 + cc(IDO, k, 3);
        }
    })
}

// rfftb (rfftb1 :102-165) of the transform in column f of A (ld), B as scratch;
// the result is back in A.  All threads of the block call it (barriers); thread
// t of the P sharing transform f passes active = true.
template <int P>
__host__ __device__ inline void rfftb96(double *A, double *B, int ld, int f, int t, bool active,
                                        const double *__restrict__ wa) {
    double *a = A + f, *b = B + f;
    if (active) radb2<48, 1, P>(a, b, ld, wa + 0, t);
    SML_FFT_SYNC();
    if (active) radb4<12, 2, P>(b, a, ld, wa + 48, wa + 60, wa + 72, t);
    SML_FFT_SYNC();
    if (active) radb4<3, 8, P>(a, b, ld, wa + 84, wa + 87, wa + 90, t);
    SML_FFT_SYNC();
    if (active) radb3_ido1<32, P>(b, a, ld, t);
    SML_FFT_SYNC();
}

// rfftf (rfftf1 :167-231): the same shape of call; the result is back in A
template <int P>
__host__ __device__ inline void rfftf96(double *A, double *B, int ld, int f, int t, bool active,
                                        const double *__restrict__ wa) {
    double *a = A + f, *b = B + f;
    if (active) radf3_ido1<32, P>(a, b, ld, t);
    SML_FFT_SYNC();
    if (active) radf4<3, 8, P>(b, a, ld, wa + 84, wa + 87, wa + 90, t);
    SML_FFT_SYNC();
    if (active) radf4<12, 2, P>(a, b, ld, wa + 48, wa + 60, wa + 72, t);
    SML_FFT_SYNC();
    if (active) radf2<48, 1, P>(b, a, ld, wa + 0, t);
    SML_FFT_SYNC();
}

// One transform per thread in registers: x[96] in, x[96] out.  The passes are the
// same code with one thread per transform (P = 1, unit stride); every index is a
// compile-time constant after unrolling, so x and the scratch stay in VGPRs.
__host__ __device__ __attribute__((always_inline)) inline void rfftb96_reg(double *x, const double *__restrict__ wa) {
    double y[kFftN];
    radb2<48, 1, 1>(x, y, 1, wa + 0, 0);
    radb4<12, 2, 1>(y, x, 1, wa + 48, wa + 60, wa + 72, 0);
    radb4<3, 8, 1>(x, y, 1, wa + 84, wa + 87, wa + 90, 0);
    radb3_ido1<32, 1>(y, x, 1, 0);
}

__host__ __device__ __attribute__((always_inline)) inline void rfftf96_reg(double *x, const double *__restrict__ wa) {
    double y[kFftN];
    radf3_ido1<32, 1>(x, y, 1, 0);
    radf4<3, 8, 1>(y, x, 1, wa + 84, wa + 87, wa + 90, 0);
    radf4<12, 2, 1>(x, y, 1, wa + 48, wa + 60, wa + 72, 0);
    radf2<48, 1, 1>(y, x, 1, wa + 0, 0);
}

// n = 48 (rffti1's factors 4, 4, 3), one transform per thread in registers, for
// the decimated form of the n = 96 transform (two independent halves per lane
// pair).  Its twiddles are a sub-table of n = 96's: 2 pi ld / 48 = 2 pi (2 ld) / 96,
// so the n = 48 passes radb4(12, 1) / radb4(3, 4) use wa96 + 48 / 60 / 72 and
// wa96 + 84 / 87 / 90, exactly the n = 96 passes radb4(12, 2) / radb4(3, 8)'s.
// rfftb48: x[q] = Y_0 + 2 sum_k (Re Y_k cos - Im Y_k sin)(2 pi k q / 48) + Y_24 (-1)^q
// from the half-complex x = [Y_0, Re Y_1, Im Y_1, .., Re Y_23, Im Y_23, Y_24].
__host__ __device__ __attribute__((always_inline)) inline void rfftb48_reg(double *x, const double *__restrict__ wa96) {
    double y[48];
    radb4<12, 1, 1>(x, y, 1, wa96 + 48, wa96 + 60, wa96 + 72, 0);
    radb4<3, 4, 1>(y, x, 1, wa96 + 84, wa96 + 87, wa96 + 90, 0);
    radb3_ido1<16, 1>(x, y, 1, 0);
#pragma unroll
    for (int e = 0; e < 48; ++e) x[e] = y[e];
}

// rfftf48: the half-complex X_k = sum_q x_q e^{-2 pi i k q / 48} (unnormalised)
__host__ __device__ __attribute__((always_inline)) inline void rfftf48_reg(double *x, const double *__restrict__ wa96) {
    double y[48];
    radf3_ido1<16, 1>(x, y, 1, 0);
    radf4<3, 4, 1>(y, x, 1, wa96 + 84, wa96 + 87, wa96 + 90, 0);
    radf4<12, 1, 1>(x, y, 1, wa96 + 48, wa96 + 60, wa96 + 72, 0);
#pragma unroll
    for (int e = 0; e < 48; ++e) x[e] = y[e];
}

// The n = 96 transforms split over a lane pair.  rfftb96 starts with radb2(48, 1)
// (:233-281): its two output halves ch(., 1, 1) / ch(., 1, 2) -- which the later
// passes keep apart and which become the even / odd points -- are two independent
// n = 48 transforms; rfftf96 ends with radf2(48, 1) (:741-789) over the n = 48
// transforms of the even and the odd samples.  Half h of a pair does one of them,
// operation for operation as FFTPACK (fft_check.cpp checks it against the
// reference's compiled rfftb / rfftf, bit for bit).
// rfftb96_half: x(e) = the half-complex input (e < 96); y[q] = point 2 q + h.  Both
// halves' radb2 values are formed and one selected (no branch on h in a wave).
template <class XF>
__host__ __device__ __attribute__((always_inline)) inline void rfftb96_half(XF x, int h, double *y,
                                                                             const double *__restrict__ wa96) {
    const bool odd = h != 0;
    y[0] = odd ? x(0) - x(95) : x(0) + x(95);
#pragma unroll
    for (int s = 1; s <= 23; ++s) {
        const double c1 = x(2 * s - 1), c2 = x(2 * s), d1 = x(95 - 2 * s), d2 = x(96 - 2 * s);
        const double e1 = c1 + d1, e2 = c2 - d2;
        const double tr2 = c1 - d1, ti2 = c2 + d2;
        const double o1 = wa96[2 * s - 2] * tr2 - wa96[2 * s - 1] * ti2;
        const double o2 = wa96[2 * s - 2] * ti2 + wa96[2 * s - 1] * tr2;
        y[2 * s - 1] = odd ? o1 : e1;
        y[2 * s] = odd ? o2 : e2;
    }
    y[47] = odd ? -(x(48) + x(48)) : x(47) + x(47);
    rfftb48_reg(y, wa96);
}

// rfftf96's last pass for output m (0 <= m <= 48) from E = rfftf48 of the even
// samples and O = rfftf48 of the odd ones (accessors E(i), O(i), i < 48): the
// unnormalised half-complex coefficient (Re X_m, Im X_m) as rfftf96 leaves it
// (Im = 0 at m = 0 and 48)
template <class EF, class OF>
__host__ __device__ __attribute__((always_inline)) inline void rfftf96_combine(EF E, OF O, int m,
                                                                                const double *__restrict__ wa96,
                                                                                double *re, double *im) {
    if (m == 0 || m == 48) {  // ch(1, 1) = cc(1, 1) + cc(1, 2), ch(ido, 2) = cc(1, 1) - cc(1, 2)
        *re = m == 0 ? E(0) + O(0) : E(0) - O(0);
        *im = 0.0;
        return;
    }
    if (m == 24) {  // ido even: ch(ido, 1) = cc(ido, 1), ch(1, 2) = -cc(ido, 2)
        *re = E(47);
        *im = -O(47);
        return;
    }
    const int s = m < 24 ? m : 48 - m;
    const double c = wa96[2 * s - 2], sn = wa96[2 * s - 1];
    const double tr2 = c * O(2 * s - 1) + sn * O(2 * s);
    const double ti2 = c * O(2 * s) - sn * O(2 * s - 1);
    if (m < 24) {
        *re = E(2 * s - 1) + tr2;
        *im = E(2 * s) + ti2;
    } else {
        *re = E(2 * s - 1) - tr2;
        *im = ti2 - E(2 * s);
    }
}

}  // namespace fft
#endif

}  // namespace sml

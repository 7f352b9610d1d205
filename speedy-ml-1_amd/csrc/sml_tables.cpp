// sml_tables.cpp -- host-side initialisation of the T30 spectral operators and
// the library's error state.  Compiled with g++ (needs __float128).
//
// Restates parmtr/gaussl/lgndre (src/spe_spectral.f90:2-242) and the FFTPACK
// twiddles that inifft prepares (src/spe_subfft_fftpack.f90:1-11) as explicit
// real-DFT matrices.  The tables are computed once per context on the host and
// handed to the device (sml_spectral.hip); the reference recomputes them at every
// SPEEDY window (ini_indyns.f90:69), which this build does not need to.
#include "sml_spectral_tables.hpp"

#include <quadmath.h>

#include <cmath>
#include <cstring>
#include <string>

namespace sml {

static thread_local std::string g_error;

int fail(int code, const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_error = buf;
    return code;
}

void clear_error() { g_error.clear(); }

// gaussl (spe_spectral.f90:2-43): Newton iteration on P_n(z).  The reference's
// `double precision` work variables are real(16) under -fdefault-real-8, so the
// iteration runs in __float128.
static void gaussl(double *x, double *w, int m) {
    const __float128 eps = 3.0e-14Q;
    const int n = 2 * m;
    __float128 z1 = 2.0Q, pp = 0.0Q;
    for (int i = 1; i <= m; ++i) {
        __float128 z = cosq(3.141592654Q * ((__float128)i - 0.25Q) / ((__float128)n + 0.5Q));
        while (fabsq(z - z1) > eps) {
            __float128 p1 = 1.0Q, p2 = 0.0Q, p3;
            for (int j = 1; j <= n; ++j) {
                p3 = p2;
                p2 = p1;
                p1 = ((2.0Q * j - 1.0Q) * z * p2 - (j - 1.0Q) * p3) / j;
            }
            pp = n * (z * p1 - p2) / (z * z - 1.0Q);
            z1 = z;
            z = z1 - p1 / pp;
        }
        x[i - 1] = (double)z;
        w[i - 1] = (double)(2.0Q / ((1.0Q - z * z) * pp * pp));
    }
}

void build_spectral_tables(double a, SpectralTables *t) {
    std::memset(t, 0, sizeof *t);
    t->radius = a;
    gaussl(t->sia, t->wt, kIY);
    for (int j = 0; j < kIY; ++j) {
        const double cosqr = 1.0 - t->sia[j] * t->sia[j];
        t->coa[j] = std::sqrt(cosqr);
    }
    for (int j = 0; j < kIY; ++j) {
        const int jj = kIL - 1 - j;
        t->cosgr[j] = t->cosgr[jj] = 1.0 / t->coa[j];
        t->cosgr2[j] = t->cosgr2[jj] = 1.0 / (t->coa[j] * t->coa[j]);
    }
    // total wavenumber and triangular masks (parmtr, spe_spectral.f90:82-107)
    for (int n = 0; n < kNX; ++n) {
        t->nsh2[n] = 0;
        for (int m = 0; m < kMX; ++m) {
            const int ll = m + n;
            t->el2[n][m] = (double)(ll * (ll + 1)) * (1.0 / (a * a));
            if (ll <= kNTRUN1) t->nsh2[n] += 2;
        }
    }
    // recursion coefficients (spe_spectral.f90:120-141)
    double epsi[kNX + 1][kMX], repsi[kNX + 1][kMX], consq[kMX];
    for (int m = 0; m < kMX; ++m)
        for (int n = 0; n <= kNX; ++n) {
            const double emm = m, ell = n + m;
            const double emm2 = emm * emm, ell2 = ell * ell;
            if (n == kNX || (n == 0 && m == 0))
                epsi[n][m] = 0.0;
            else
                epsi[n][m] = std::sqrt((ell2 - emm2) / (4.0 * ell2 - 1.0));
            repsi[n][m] = epsi[n][m] > 0.0 ? 1.0 / epsi[n][m] : 0.0;
        }
    const double sqrhlf = std::sqrt(0.5);
    for (int m = 1; m < kMX; ++m) consq[m] = std::sqrt(0.5 * (2.0 * m + 1.0) / (double)m);
    // grad / uvspec / vds coefficients (spe_spectral.f90:145-170)
    for (int m = 0; m < kMX; ++m)
        for (int n = 0; n < kNX; ++n) {
            const double el1 = (double)(m + n);
            if (n == 0) {
                t->gradx[m] = (double)m / a;
                t->uvdx[0][m] = -a / (double)(m + 1);
                t->uvdym[0][m] = 0.0;
                t->vddym[0][m] = 0.0;
            } else {
                t->uvdx[n][m] = -a * (double)m / (el1 * (el1 + 1.0));
                t->gradym[n][m] = (el1 - 1.0) * epsi[n][m] / a;
                t->uvdym[n][m] = -a * epsi[n][m] / el1;
                t->vddym[n][m] = (el1 + 1.0) * epsi[n][m] / a;
            }
            t->gradyp[n][m] = (el1 + 2.0) * epsi[n + 1][m] / a;
            t->uvdyp[n][m] = -a * epsi[n + 1][m] / (el1 + 1.0);
            t->vddyp[n][m] = el1 * epsi[n + 1][m] / a;
        }
    // Legendre polynomials per Gaussian latitude (lgndre, spe_spectral.f90:194-242)
    for (int j = 0; j < kIY; ++j) {
        double alp[kNX][kMX];
        const double y = t->coa[j], x = t->sia[j];
        alp[0][0] = sqrhlf;
        for (int m = 1; m < kMX; ++m) alp[0][m] = consq[m] * y * alp[0][m - 1];
        for (int m = 0; m < kMX; ++m) alp[1][m] = (x * alp[0][m]) * repsi[1][m];
        for (int n = 2; n < kNX; ++n)
            for (int m = 0; m < kMX; ++m)
                alp[n][m] = (x * alp[n - 1][m] - epsi[n - 1][m] * alp[n - 2][m]) * repsi[n][m];
        for (int n = 0; n < kNX; ++n)
            for (int m = 0; m < kMX; ++m) t->poly[j][n][m] = std::fabs(alp[n][m]) <= 1.0e-30 ? 0.0 : alp[n][m];
    }
    // Real-DFT matrices equivalent to FFTPACK rfftb / rfftf + the gridx/specx
    // packing (spe_subfft_fftpack.f90:15-87): inverse x_i = a0 + 2 sum_k (Re_k cos
    // - Im_k sin), forward Re_k = (1/96) sum x cos, Im_k = -(1/96) sum x sin.
    const long double tpi = 8.0L * atanl(1.0L);
    for (int c = 0; c < kCPad; ++c)
        for (int i = 0; i < kIX; ++i) {
            double inv = 0.0, fwd = 0.0;
            if (c == 0) {
                inv = 1.0;
                fwd = 1.0 / (double)kIX;
            } else if (c >= 2 && c < kMX2) {
                const int k = c / 2;
                const long double arg = tpi * (long double)((k * i) % kIX) / (long double)kIX;
                if ((c & 1) == 0) {
                    inv = (double)(2.0L * cosl(arg));
                    fwd = (double)(cosl(arg) / (long double)kIX);
                } else {
                    inv = (double)(-2.0L * sinl(arg));
                    fwd = (double)(-sinl(arg) / (long double)kIX);
                }
            }
            t->dinv[c][i] = inv;
            t->dfwd[i][c] = fwd;
        }
}

}  // namespace sml

extern "C" const char *sml_last_error(void) { return sml::g_error.c_str(); }
extern "C" int sml_abi_version(void) { return 1; }

/*
 * oracle/speedy_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the SPEEDY-ML hybrid hot path (awikner/SPEEDY-ML-1), written
 * from the reference's behaviour.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library.
 *
 * Coverage:
 *   - spectral tables:  parmtr/gaussl/lgndre          (src/spe_spectral.f90:2-242)
 *   - Legendre:         gridy/specy                    (src/spe_spectral.f90:454-538)
 *   - Fourier:          gridx/specx (FFTPACK rfftb/f)  (src/spe_subfft_fftpack.f90:15-87)
 *   - composites:       grid/spec/vdspec/uvspec/vds/grad/lap/invlap/trunct
 *                                                      (src/spe_spectral.f90:244-551)
 *   - reservoir:        predict / predict_ml           (src/mod_reservoir.f90:1416-1533)
 *                       unstandardize_state_vec_res    (src/res_domain.f90:1402-1453)
 *   - tiling:           getxyresextent/getoverlapindices (src/res_domain.f90:123-204)
 *                       tile_full_grid_with_local_state_vec_res1d (res_domain.f90:769-804)
 *                       tileoverlapgrid4d + tile_4d_and_logp_to_local_state_input
 *                                                      (res_domain.f90:348-420,1059-1103)
 *                       tile_4d_and_logp_full_grid_to_local_res_vec (res_domain.f90:1000-1031)
 *                       standardize_state_vec_input/res (res_domain.f90:1189-1293)
 *                       sendrecievegrid clips           (src/mpires.f90:448-478,726-751)
 *
 * Pinning:
 *   - spectral functions are pinned against the reference Fortran compiled as-is
 *     (oracle/Makefile -> oracle/_ref/libspeedy_ref_spectral.so) through the golden
 *     fixtures in tests/golden/ (tests/golden/make_golden.py).
 *   - reservoir/tiling: PARITY UNPINNED by the reference itself: the reference's
 *     reservoir path (mod_reservoir/mod_linalg/res_domain/mod_utilities) needs MKL
 *     sparse BLAS, MPI and netCDF-Fortran, none of which exist in this image, so it
 *     is unbuildable here (DESIGN.md "Oracle").  The restatement follows the cited
 *     lines statement by statement.
 *
 * Layout conventions: every array uses the reference's Fortran column-major layout,
 * e.g. a spectral field v(mx2=62,nx=32) is v[n*62+m], a grid field g(ix=96,il=48) is
 * g[j*96+i] with j=0 the southernmost row.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <quadmath.h>

#define MX 31
#define NX 32
#define MX2 62
#define IX 96
#define IY 24
#define IL 48
#define NTRUN 30
#define NTRUN1 31
#define MXP 31
#define NXP 33

/* ------------------------------------------------------------------------- */
/* spectral tables (mod_spectral.f90:12-35)                                  */
/* ------------------------------------------------------------------------- */
static double el2[NX][MX], elm2[NX][MX], el4[NX][MX], trfilt[NX][MX];
static int nsh2[NX];
static double sia[IY], coa[IY], wt[IY], wght[IY];
static double cosg[IL], cosgr[IL], cosgr2[IL];
static double gradx[MX], gradym[NX][MX], gradyp[NX][MX];
static double sqrhlf, consq[MXP], epsi[NXP][MXP], repsi[NXP][MXP], emm[MXP], ell[NXP][MXP];
static double cpol[IY][NX][MX2];
static double uvdx[NX][MX], uvdym[NX][MX], uvdyp[NX][MX];
static double vddym[NX][MX], vddyp[NX][MX];
static int tables_ready = 0;

/* gaussl (spe_spectral.f90:2-43).  The reference declares the work variables
 * `double precision`; under its gfortran/flang build flag -fdefault-real-8 those
 * are promoted to real(16), so this restatement iterates in __float128. */
static void orc_gaussl(double *x, double *w, int m)
{
    const __float128 eps = 3.0e-14Q;
    int n = 2 * m;
    __float128 z, z1 = 2.0Q, p1, p2, p3, pp = 0;
    for (int i = 1; i <= m; ++i) {
        z = cosq(3.141592654Q * ((__float128)i - 0.25Q) / ((__float128)n + 0.5Q));
        while (fabsq(z - z1) > eps) {
            p1 = 1.0Q;
            p2 = 0.0Q;
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

/* lgndre (spe_spectral.f90:194-242): associated Legendre polynomials at sia(j). */
static void orc_lgndre(int j, double poly[NX][MX])
{
    double alp[NX][MXP];
    double y = coa[j], x = sia[j];
    alp[0][0] = sqrhlf;
    for (int m = 1; m < MXP; ++m) alp[0][m] = consq[m] * y * alp[0][m - 1];
    for (int m = 0; m < MXP; ++m) alp[1][m] = (x * alp[0][m]) * repsi[1][m];
    for (int n = 2; n < NX; ++n)
        for (int m = 0; m < MXP; ++m)
            alp[n][m] = (x * alp[n - 1][m] - epsi[n - 1][m] * alp[n - 2][m]) * repsi[n][m];
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MXP; ++m)
            if (fabs(alp[n][m]) <= 1.0e-30) alp[n][m] = 0.0;
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) poly[n][m] = alp[n][m];  /* isc = 1 */
}

/* parmtr (spe_spectral.f90:45-192) */
void orc_spectral_init(double a)
{
    double am2 = 1.0 / (a * a);
    orc_gaussl(sia, wt, IY);
    for (int j = 0; j < IY; ++j) {
        double cosqr = 1.0 - sia[j] * sia[j];
        coa[j] = sqrt(cosqr);
        wght[j] = wt[j] / (a * cosqr);
    }
    for (int j = 0; j < IY; ++j) {
        int jj = IL - 1 - j;
        cosg[j] = cosg[jj] = coa[j];
        cosgr[j] = cosgr[jj] = 1.0 / coa[j];
        cosgr2[j] = cosgr2[jj] = 1.0 / (coa[j] * coa[j]);
    }
    for (int n = 0; n < NX; ++n) {
        nsh2[n] = 0;
        for (int m = 0; m < MX; ++m) {
            int mm = m;                      /* mm(m) = isc*(m-1) */
            int ll = mm + n;                 /* ll(m,n) = mm + n - 1 (1-based n) */
            int l2 = ll * (ll + 1);
            el2[n][m] = (double)l2 * am2;
            el4[n][m] = el2[n][m] * el2[n][m];
            if (ll <= NTRUN1) nsh2[n] += 2;
            trfilt[n][m] = (ll <= NTRUN) ? 1.0 : 0.0;
        }
    }
    elm2[0][0] = 0.0;
    for (int m = 1; m < MX; ++m)
        for (int n = 0; n < NX; ++n) elm2[n][m] = 1.0 / el2[n][m];
    for (int n = 1; n < NX; ++n) elm2[n][0] = 1.0 / el2[n][0];

    for (int m = 0; m < MXP; ++m) {
        for (int n = 0; n < NXP; ++n) {
            emm[m] = (double)m;
            ell[n][m] = (double)(n + m);
            double emm2 = emm[m] * emm[m], ell2 = ell[n][m] * ell[n][m];
            if (n == NXP - 1)
                epsi[n][m] = 0.0;
            else if (n == 0 && m == 0)
                epsi[n][m] = 0.0;
            else
                epsi[n][m] = sqrt((ell2 - emm2) / (4.0 * ell2 - 1.0));
            repsi[n][m] = 0.0;
            if (epsi[n][m] > 0.0) repsi[n][m] = 1.0 / epsi[n][m];
        }
    }
    sqrhlf = sqrt(0.5);
    for (int m = 1; m < MXP; ++m) consq[m] = sqrt(0.5 * (2.0 * emm[m] + 1.0) / emm[m]);

    for (int m = 0; m < MX; ++m) {
        for (int n = 0; n < NX; ++n) {
            int m1 = m, m2 = m1 + 1;          /* 1-based index into epsi's m */
            double el1 = (double)(m + n);
            if (n == 0) {
                gradx[m] = (double)m1 / a;
                uvdx[0][m] = -a / (double)(m1 + 1);
                uvdym[0][m] = 0.0;
                vddym[0][m] = 0.0;
            } else {
                uvdx[n][m] = -a * (double)m1 / (el1 * (el1 + 1.0));
                gradym[n][m] = (el1 - 1.0) * epsi[n][m2 - 1] / a;
                uvdym[n][m] = -a * epsi[n][m2 - 1] / el1;
                vddym[n][m] = (el1 + 1.0) * epsi[n][m2 - 1] / a;
            }
            gradyp[n][m] = (el1 + 2.0) * epsi[n + 1][m2 - 1] / a;
            uvdyp[n][m] = -a * epsi[n + 1][m2 - 1] / (el1 + 1.0);
            vddyp[n][m] = el1 * epsi[n + 1][m2 - 1] / a;
        }
    }
    for (int j = 0; j < IY; ++j) {
        double poly[NX][MX];
        orc_lgndre(j, poly);
        for (int n = 0; n < NX; ++n)
            for (int m = 0; m < MX; ++m) cpol[j][n][2 * m] = cpol[j][n][2 * m + 1] = poly[n][m];
    }
    tables_ready = 1;
}

/* Table export for tests (lets tests compare the product's tables too). */
void orc_get_tables(double *out_sia, double *out_wt, double *out_cpol, int *out_nsh2)
{
    if (out_sia) memcpy(out_sia, sia, sizeof sia);
    if (out_wt) memcpy(out_wt, wt, sizeof wt);
    if (out_cpol) memcpy(out_cpol, cpol, sizeof cpol);
    if (out_nsh2) memcpy(out_nsh2, nsh2, sizeof nsh2);
}

/* ------------------------------------------------------------------------- */
/* Legendre (spe_spectral.f90:454-538)                                       */
/* ------------------------------------------------------------------------- */
/* gridy: v(mx2,nx) -> varm(mx2,il) */
void orc_gridy(const double *v, double *varm)
{
    for (int j = 0; j < IY; ++j) {
        int j1 = IL - 1 - j;
        double vm1[MX2], vm2[MX2];
        for (int m = 0; m < MX2; ++m) vm1[m] = vm2[m] = 0.0;
        for (int n = 0; n < NX; n += 2)          /* n = 1,3,... (1-based) */
            for (int m = 0; m < nsh2[n]; ++m) vm1[m] = vm1[m] + v[n * MX2 + m] * cpol[j][n][m];
        for (int n = 1; n < NX; n += 2)          /* n = 2,4,... */
            for (int m = 0; m < nsh2[n]; ++m) vm2[m] = vm2[m] + v[n * MX2 + m] * cpol[j][n][m];
        for (int m = 0; m < MX2; ++m) {
            varm[j1 * MX2 + m] = vm1[m] + vm2[m];
            varm[j * MX2 + m] = vm1[m] - vm2[m];
        }
    }
}

/* specy: varm(mx2,il) -> vorm(mx2,nx); rows n = 32 stay zero (ntrun1 = 31) */
void orc_specy(const double *varm, double *vorm)
{
    double svarm[IY][MX2], dvarm[IY][MX2];
    for (int i = 0; i < MX2 * NX; ++i) vorm[i] = 0.0;
    for (int j = 0; j < IY; ++j) {
        int j1 = IL - 1 - j;
        for (int m = 0; m < MX2; ++m) {
            svarm[j][m] = (varm[j1 * MX2 + m] + varm[j * MX2 + m]) * wt[j];
            dvarm[j][m] = (varm[j1 * MX2 + m] - varm[j * MX2 + m]) * wt[j];
        }
    }
    for (int j = 0; j < IY; ++j) {
        for (int n = 0; n < NTRUN1; n += 2)
            for (int m = 0; m < nsh2[n]; ++m) vorm[n * MX2 + m] = vorm[n * MX2 + m] + cpol[j][n][m] * svarm[j][m];
        for (int n = 1; n < NTRUN1; n += 2)
            for (int m = 0; m < nsh2[n]; ++m) vorm[n * MX2 + m] = vorm[n * MX2 + m] + cpol[j][n][m] * dvarm[j][m];
    }
}

/* ------------------------------------------------------------------------- */
/* Fourier (spe_subfft_fftpack.f90:15-87).  FFTPACK's rfftb/rfftf compute the  */
/* unnormalised real DFT in half-complex order r(1)=a0, r(2k)=Re_k,            */
/* r(2k+1)=Im_k; this restatement evaluates the same sums directly in long     */
/* double (O(n^2), exact up to rounding).                                      */
/* ------------------------------------------------------------------------- */
static long double twc[IX][IX], tws[IX][IX];
static int tw_ready = 0;
static void orc_twiddles(void)
{
    if (tw_ready) return;
    const long double tpi = 8.0L * atanl(1.0L);
    for (int k = 0; k < IX; ++k)
        for (int i = 0; i < IX; ++i) {
            long double arg = tpi * (long double)((k * i) % IX) / (long double)IX;
            twc[k][i] = cosl(arg);
            tws[k][i] = sinl(arg);
        }
    tw_ready = 1;
}

/* gridx: varm(mx2,il) -> vorg(ix,il); kcos==2 multiplies by 1/cos(lat) */
void orc_gridx(const double *varm, double *vorg, int kcos)
{
    orc_twiddles();
    for (int j = 0; j < IL; ++j) {
        /* fvar(1) = varm(1), fvar(m-1) = varm(m) for m = 3..mx2, the rest 0:
         * Im of wavenumber 0 is dropped, wavenumbers > 30 are zero. */
        const double *vr = varm + j * MX2;
        for (int i = 0; i < IX; ++i) {
            long double s = vr[0];
            for (int k = 1; k <= NTRUN; ++k)
                s += 2.0L * ((long double)vr[2 * k] * twc[k][i] - (long double)vr[2 * k + 1] * tws[k][i]);
            double f = (double)s;
            vorg[j * IX + i] = (kcos == 1) ? f : f * cosgr[j];
        }
    }
}

/* specx: vorg(ix,il) -> varm(mx2,il), scaled by 1/ix, varm(2) = 0 */
void orc_specx(const double *vorg, double *varm)
{
    orc_twiddles();
    const double scale = 1.0 / (double)IX;
    for (int j = 0; j < IL; ++j) {
        const double *g = vorg + j * IX;
        double *vr = varm + j * MX2;
        long double a0 = 0.0L;
        for (int i = 0; i < IX; ++i) a0 += g[i];
        vr[0] = (double)a0 * scale;
        vr[1] = 0.0;
        for (int k = 1; k <= NTRUN; ++k) {
            long double re = 0.0L, im = 0.0L;
            for (int i = 0; i < IX; ++i) {
                re += (long double)g[i] * twc[k][i];
                im -= (long double)g[i] * tws[k][i];
            }
            vr[2 * k] = (double)re * scale;
            vr[2 * k + 1] = (double)im * scale;
        }
    }
}

/* grid / spec (spe_spectral.f90:389-414) */
void orc_grid(const double *vorm, double *vorg, int kcos)
{
    double varm[IL * MX2];
    orc_gridy(vorm, varm);
    orc_gridx(varm, vorg, kcos);
}

void orc_spec(const double *vorg, double *vorm)
{
    double varm[IL * MX2];
    orc_specx(vorg, varm);
    orc_specy(varm, vorm);
}

/* Complex spectral arrays are (2,mx,nx): element (k,m,n) at k + 2*(m + mx*n). */
#define C3(k, m, n) ((k) + 2 * ((m) + MX * (n)))

/* vds (spe_spectral.f90:307-349) */
void orc_vds(const double *ucosm, const double *vcosm, double *vorm, double *divm)
{
    static double zc[2 * MX * NX], zp[2 * MX * NX];
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) {
            zp[C3(1, m, n)] = gradx[m] * ucosm[C3(0, m, n)];
            zp[C3(0, m, n)] = -gradx[m] * ucosm[C3(1, m, n)];
            zc[C3(1, m, n)] = gradx[m] * vcosm[C3(0, m, n)];
            zc[C3(0, m, n)] = -gradx[m] * vcosm[C3(1, m, n)];
        }
    for (int k = 0; k < 2; ++k)
        for (int m = 0; m < MX; ++m) {
            vorm[C3(k, m, 0)] = zc[C3(k, m, 0)] - vddyp[0][m] * ucosm[C3(k, m, 1)];
            vorm[C3(k, m, NX - 1)] = vddym[NX - 1][m] * ucosm[C3(k, m, NTRUN1 - 1)];
            divm[C3(k, m, 0)] = zp[C3(k, m, 0)] + vddyp[0][m] * vcosm[C3(k, m, 1)];
            divm[C3(k, m, NX - 1)] = -vddym[NX - 1][m] * vcosm[C3(k, m, NTRUN1 - 1)];
        }
    for (int k = 0; k < 2; ++k)
        for (int n = 1; n < NTRUN1; ++n)
            for (int m = 0; m < MX; ++m) {
                vorm[C3(k, m, n)] = vddym[n][m] * ucosm[C3(k, m, n - 1)] - vddyp[n][m] * ucosm[C3(k, m, n + 1)] + zc[C3(k, m, n)];
                divm[C3(k, m, n)] = -vddym[n][m] * vcosm[C3(k, m, n - 1)] + vddyp[n][m] * vcosm[C3(k, m, n + 1)] + zp[C3(k, m, n)];
            }
}

/* uvspec (spe_spectral.f90:351-387) */
void orc_uvspec(const double *vorm, const double *divm, double *ucosm, double *vcosm)
{
    static double zc[2 * MX * NX], zp[2 * MX * NX];
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) {
            zp[C3(1, m, n)] = uvdx[n][m] * vorm[C3(0, m, n)];
            zp[C3(0, m, n)] = -uvdx[n][m] * vorm[C3(1, m, n)];
            zc[C3(1, m, n)] = uvdx[n][m] * divm[C3(0, m, n)];
            zc[C3(0, m, n)] = -uvdx[n][m] * divm[C3(1, m, n)];
        }
    for (int k = 0; k < 2; ++k)
        for (int m = 0; m < MX; ++m) {
            ucosm[C3(k, m, 0)] = zc[C3(k, m, 0)] - uvdyp[0][m] * vorm[C3(k, m, 1)];
            ucosm[C3(k, m, NX - 1)] = uvdym[NX - 1][m] * vorm[C3(k, m, NTRUN1 - 1)];
            vcosm[C3(k, m, 0)] = zp[C3(k, m, 0)] + uvdyp[0][m] * divm[C3(k, m, 1)];
            vcosm[C3(k, m, NX - 1)] = -uvdym[NX - 1][m] * divm[C3(k, m, NTRUN1 - 1)];
        }
    for (int k = 0; k < 2; ++k)
        for (int n = 1; n < NTRUN1; ++n)
            for (int m = 0; m < MX; ++m) {
                vcosm[C3(k, m, n)] = -uvdym[n][m] * divm[C3(k, m, n - 1)] + uvdyp[n][m] * divm[C3(k, m, n + 1)] + zp[C3(k, m, n)];
                ucosm[C3(k, m, n)] = uvdym[n][m] * vorm[C3(k, m, n - 1)] - uvdyp[n][m] * vorm[C3(k, m, n + 1)] + zc[C3(k, m, n)];
            }
}

/* grad (spe_spectral.f90:271-305) */
void orc_grad(const double *psi, double *psdx, double *psdy)
{
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) {
            psdx[C3(1, m, n)] = gradx[m] * psi[C3(0, m, n)];
            psdx[C3(0, m, n)] = -gradx[m] * psi[C3(1, m, n)];
        }
    for (int k = 0; k < 2; ++k)
        for (int m = 0; m < MX; ++m) {
            psdy[C3(k, m, 0)] = gradyp[0][m] * psi[C3(k, m, 1)];
            psdy[C3(k, m, NX - 1)] = -gradym[NX - 1][m] * psi[C3(k, m, NTRUN1 - 1)];
        }
    for (int k = 0; k < 2; ++k)
        for (int n = 1; n < NTRUN1; ++n)
            for (int m = 0; m < MX; ++m)
                psdy[C3(k, m, n)] = -gradym[n][m] * psi[C3(k, m, n - 1)] + gradyp[n][m] * psi[C3(k, m, n + 1)];
}

/* vdspec (spe_spectral.f90:416-452) */
void orc_vdspec(const double *ug, const double *vg, double *vorm, double *divm, int kcos)
{
    static double ug1[IX * IL], vg1[IX * IL], um[MX2 * IL], vm[MX2 * IL];
    static double d1[MX2 * NX], d2[MX2 * NX];
    for (int j = 0; j < IL; ++j)
        for (int i = 0; i < IX; ++i) {
            double s = (kcos == 2) ? cosgr[j] : cosgr2[j];
            ug1[j * IX + i] = ug[j * IX + i] * s;
            vg1[j * IX + i] = vg[j * IX + i] * s;
        }
    orc_specx(ug1, um);
    orc_specx(vg1, vm);
    orc_specy(um, d1);
    orc_specy(vm, d2);
    orc_vds(d1, d2, vorm, divm);
}

/* lap / invlap / trunct (spe_spectral.f90:244-269,540-551) on complex(mx,nx) */
void orc_lap(const double *strm, double *vorm)
{
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m)
            for (int k = 0; k < 2; ++k) vorm[C3(k, m, n)] = -(strm[C3(k, m, n)] * el2[n][m]);
}
void orc_invlap(const double *vorm, double *strm)
{
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m)
            for (int k = 0; k < 2; ++k) strm[C3(k, m, n)] = -(vorm[C3(k, m, n)] * elm2[n][m]);
}
void orc_trunct(double *vor)
{
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m)
            for (int k = 0; k < 2; ++k) vor[C3(k, m, n)] = vor[C3(k, m, n)] * trfilt[n][m];
}

/* ------------------------------------------------------------------------- */
/* Domain decomposition (res_domain.f90:31-204,258-292) for 1152 regions of   */
/* 2x2 points on the 96x48 grid, overlap 1, one vertical level of 8 heights.  */
/* All indices returned 1-based as in the reference.                          */
/* ------------------------------------------------------------------------- */
#define XGRID 96
#define YGRID 48
#define ZGRID 8

typedef struct {
    int res_xstart, res_xend, res_ystart, res_yend, resxchunk, resychunk;
    int input_xstart, input_xend, input_ystart, input_yend, inputxchunk, inputychunk;
    int pole, periodic;
    int tdata_xstart, tdata_xend, tdata_ystart, tdata_yend;
} orc_region_geom;

/* domaindecomposition (res_domain.f90:258-280) */
static void orc_domaindecomposition(int numregions, int *fx, int *fy)
{
    int n = (XGRID * YGRID) / numregions;
    int fmax = (int)floor(sqrt((double)n));
    *fx = *fy = 0;
    for (int i = fmax; i >= 0; --i) {
        if (i == 0) break;
        if (YGRID % i == 0) {
            *fy = i;
            if (n % i == 0) {
                *fx = n / i;
                if (XGRID % *fx == 0) break;
            }
        }
    }
}

void orc_region_geometry(int numregions, int region, int overlap, orc_region_geom *g)
{
    int fx, fy;
    orc_domaindecomposition(numregions, &fx, &fy);
    /* getworkerlower_leftcorner (res_domain.f90:282-292) */
    int col = region % (YGRID / fy);
    int row = (int)floor((double)region / ((double)YGRID / (double)fy));
    g->resxchunk = fx;
    g->resychunk = fy;
    g->res_xstart = row * fx + 1;
    g->res_xend = (row + 1) * fx;
    g->res_ystart = col * fy + 1;
    g->res_yend = (col + 1) * fy;
    /* getoverlapindices (res_domain.f90:155-204) */
    g->inputxchunk = fx + 2 * overlap;
    g->inputychunk = fy + 2 * overlap;
    g->periodic = 0;
    g->pole = 0;
    if (g->res_xstart - overlap < 1) {
        g->input_xstart = XGRID - overlap + 1;
        g->periodic = 1;
    } else
        g->input_xstart = g->res_xstart - overlap;
    if (g->res_xend + overlap > XGRID) {
        g->input_xend = overlap;
        g->periodic = 1;
    } else
        g->input_xend = overlap + g->res_xend;
    if (g->res_ystart - overlap < 1) {
        g->input_ystart = 1;
        g->inputychunk = fy + overlap + (g->res_ystart - 1);
        g->pole = 1;
    } else
        g->input_ystart = g->res_ystart - overlap;
    if (g->res_yend + overlap > YGRID) {
        g->input_yend = YGRID;
        g->inputychunk = fy + overlap + (YGRID - g->res_yend);
        g->pole = 1;
    } else
        g->input_yend = overlap + g->res_yend;
    /* get_trainingdataindices (res_domain.f90:547-574) */
    g->tdata_xstart = 1 + overlap;
    g->tdata_xend = g->inputxchunk - overlap;
    if (g->res_ystart - overlap < 1) {
        g->tdata_ystart = 1 + (g->res_ystart - 1);
        g->tdata_yend = g->inputychunk - overlap;
    } else if (g->res_yend + overlap > YGRID) {
        g->tdata_ystart = 1 + overlap;
        g->tdata_yend = g->inputychunk - (YGRID - g->res_yend);
    } else {
        g->tdata_ystart = 1 + overlap;
        g->tdata_yend = g->inputychunk - overlap;
    }
}

/* Plain-int export of the geometry for ctypes: 18 ints in struct order. */
void orc_region_geometry_ints(int numregions, int region, int overlap, int *out)
{
    orc_region_geom g;
    orc_region_geometry(numregions, region, overlap, &g);
    memcpy(out, &g, sizeof g);
}

/* x index (1-based, global) of local input column lx (1-based) of
 * tileoverlapgrid4d (res_domain.f90:348-420): periodic wrap in x. */
static int orc_input_x(const orc_region_geom *g, int lx)
{
    if (!g->periodic) return g->input_xstart + lx - 1;
    if (g->res_xend > g->input_xend || g->input_xstart > g->res_xstart) {
        int nfirst = XGRID - (g->input_xstart - 1);
        if (lx <= nfirst) return g->input_xstart + lx - 1;
        return lx - nfirst;
    }
    return g->input_xstart + lx - 1;
}

/* get_radius_by_lat (res_domain.f90:1601-1638) with speedylat (mod_utilities.f90:23-29) */
static const double speedylat[48] = {
    -87.159, -83.479, -79.777, -76.070, -72.362, -68.652, -64.942, -61.232, -57.521, -53.810,
    -50.099, -46.389, -42.678, -38.967, -35.256, -31.545, -27.833, -24.122, -20.411, -16.700,
    -12.989, -9.278,  -5.567,  -1.856,  1.856,   5.567,   9.278,   12.989,  16.700,  20.411,
    24.122,  27.833,  31.545,  35.256,  38.967,  42.678,  46.389,  50.099,  53.810,  57.521,
    61.232,  64.942,  68.652,  72.362,  76.070,  79.777,  83.479,  87.159};

double orc_radius_by_region(int numregions, int region)
{
    orc_region_geom g;
    orc_region_geometry(numregions, region, 1, &g);
    double startlat = speedylat[g.res_ystart - 1], endlat = speedylat[g.res_yend - 1];
    const double highest_lat = 45.0, max_radius = 0.7, min_radius = 0.3;
    double smallest = fabs(fmin(startlat, endlat));
    (void)fabs(fmax(startlat, endlat));
    if (smallest >= highest_lat) return max_radius;
    return (max_radius - min_radius) / highest_lat + min_radius;
}

/* Reservoir sizes (mod_reservoir.f90:78-178 allocate_res_new, :1781-1884):
 * bottom level, logp+tisr+precip always on, sst per region.
 * out: [ninp, n, k, chunk_size_prediction(136), chunk_size_speedy(132)] */
void orc_reservoir_sizes(int numregions, int region, int sst, int m_nodes, int *out)
{
    orc_region_geom g;
    orc_region_geometry(numregions, region, 1, &g);
    int in2d = g.inputxchunk * g.inputychunk;
    int res2d = g.resxchunk * g.resychunk;
    int chunk = res2d * 4 * ZGRID + res2d + res2d;              /* atmo + logp + precip */
    int locality = in2d * ZGRID * 4 + in2d /*logp*/ + in2d /*precip*/ + in2d /*tisr*/ + (sst ? in2d : 0) - chunk;
    int ninp = chunk + locality;
    int nodes_per_input = (int)lround((double)m_nodes / (double)ninp);  /* NINT */
    int n = nodes_per_input * ninp;
    double density = 6.0 / (double)m_nodes;                     /* deg/m, :99 */
    int k = (int)(density * n * n);
    out[0] = ninp;
    out[1] = n;
    out[2] = k;
    out[3] = chunk;
    out[4] = res2d * 4 * ZGRID + res2d;
}

/* ------------------------------------------------------------------------- */
/* Reservoir forward: predict (mod_reservoir.f90:1416-1487) and               */
/* unstandardize_state_vec_res (res_domain.f90:1402-1453).                    */
/* ------------------------------------------------------------------------- */
/* outvec layout for the bottom-level 2x2 reservoir: atmo(4,2,2,8) | logp(2,2)
 * | precip(2,2).  mean/std index l = (var-1)*8 + level for atmo, 33 logp,
 * 35 precip (1-based; mod_reservoir.f90:1815-1846). */
void orc_unstandardize_res(double *outvec, int resx, int resy, int nlev, const double *mean, const double *std,
                           int logp, int precip, int logp_idx, int precip_idx)
{
    int natmo = 4 * resx * resy * nlev;
    for (int v = 0; v < 4; ++v)
        for (int z = 0; z < nlev; ++z) {
            int l = v * nlev + z;  /* 0-based */
            for (int y = 0; y < resy; ++y)
                for (int x = 0; x < resx; ++x) {
                    double *p = outvec + v + 4 * (x + resx * (y + resy * z));
                    double t = *p * std[l];
                    *p = t + mean[l];
                }
        }
    if (logp)
        for (int i = 0; i < resx * resy; ++i) {
            double t = outvec[natmo + i] * std[logp_idx - 1];
            outvec[natmo + i] = t + mean[logp_idx - 1];
        }
    if (precip)
        for (int i = 0; i < resx * resy; ++i) {
            double *p = outvec + natmo + resx * resy + i;
            double t = *p * std[precip_idx - 1];
            *p = t + mean[precip_idx - 1];
        }
}

/* predict for one region, reference arithmetic order:
 *   y = A x  (COO in file order, 1-based rows/cols: MKL_SPARSE_D_MV, :1442)
 *   temp = matmul(win, feedback)  (dense n x ninp column-major, :1443)
 *   x = (1-leak) x + leak tanh(y + temp)   (:1445-1446)
 *   x_temp(2:n:2) = x_temp(2:n:2)**2       (:1448-1449)
 *   x_aug = [local_model ; x_temp]         (:1451-1452)
 *   outvec = matmul(wout, x_aug)           (:1454; wout(nout, ncs+n) column-major)
 * then unstandardize (:1469).  chunk_speedy = 0 gives predict_ml (:1489-1533). */
void orc_predict(int n, int ninp, int k, const int *rows, const int *cols, const double *vals,
                 const double *win, const double *wout, int nout, int chunk_speedy, double leakage,
                 const double *feedback, const double *local_model, double *x, double *outvec,
                 const double *mean, const double *std, int unstd)
{
    double *y = (double *)calloc((size_t)n, sizeof(double));
    double *temp = (double *)calloc((size_t)n, sizeof(double));
    double *xa = (double *)malloc(sizeof(double) * (size_t)(n + chunk_speedy));
    for (int e = 0; e < k; ++e) y[rows[e] - 1] = y[rows[e] - 1] + vals[e] * x[cols[e] - 1];
    for (int jj = 0; jj < ninp; ++jj) {
        double fb = feedback[jj];
        const double *wc = win + (size_t)jj * n;
        for (int i = 0; i < n; ++i) temp[i] = temp[i] + wc[i] * fb;
    }
    for (int i = 0; i < n; ++i) {
        double xn = tanh(y[i] + temp[i]);
        x[i] = (1.0 - leakage) * x[i] + leakage * xn;
    }
    for (int i = 0; i < chunk_speedy; ++i) xa[i] = local_model[i];
    for (int i = 0; i < n; ++i) xa[chunk_speedy + i] = (i & 1) ? x[i] * x[i] : x[i];
    for (int o = 0; o < nout; ++o) outvec[o] = 0.0;
    for (int jj = 0; jj < n + chunk_speedy; ++jj) {
        double a = xa[jj];
        const double *wc = wout + (size_t)jj * nout;
        for (int o = 0; o < nout; ++o) outvec[o] = outvec[o] + wc[o] * a;
    }
    if (unstd) orc_unstandardize_res(outvec, 2, 2, ZGRID, mean, std, 1, 1, 33, 35);
    free(y);
    free(temp);
    free(xa);
}

/* The CPU baseline's reservoir leg (bench.py cpu_baseline): orc_predict -- the
 * reference's arithmetic, dense W_in matmul included -- for every region, OpenMP
 * over regions (each region as the reference's per-region predict call,
 * parallelmain.f90:225-234; the reference itself runs one region after another on
 * each MPI rank).  Per-region arrays are passed as pointer tables; outvecs
 * [nreg][nout]. */
void orc_predict_regions(int nreg, int nthreads, const int *n, const int *ninp, const int *k,
                         const int *const *rows, const int *const *cols, const double *const *vals,
                         const double *const *win, const double *const *wout, int nout, int chunk_speedy,
                         double leakage, const double *const *feedback, const double *const *local_model,
                         double *const *x, double *outvecs, const double *const *mean, const double *const *std)
{
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
    for (int r = 0; r < nreg; ++r)
        orc_predict(n[r], ninp[r], k[r], rows[r], cols[r], vals[r], win[r], wout[r], nout, chunk_speedy, leakage,
                    feedback[r], local_model[r], x[r], outvecs + (size_t)r * nout, mean[r], std[r], 1);
}

/* Same as orc_predict but W_in given in compressed form (one column index and
 * value per row, the structure train_reservoir writes, mod_reservoir.f90:260-278)
 * and float32 weights (the NetCDF file precision, mod_io.f90:1282); products
 * with the dense matrix's exact zeros contribute nothing, so this is the same
 * arithmetic.  Used for the CPU baseline on bounded samples. */
void orc_predict_f32(int n, int ninp, int k, const int *rows, const int *cols, const float *vals,
                     const int *win_col, const float *win_val, const float *wout, int nout, int chunk_speedy,
                     double leakage, const double *feedback, const double *local_model, double *x,
                     double *outvec, const double *mean, const double *std)
{
    double *y = (double *)calloc((size_t)n, sizeof(double));
    double *xa = (double *)malloc(sizeof(double) * (size_t)(n + chunk_speedy));
    (void)ninp;
    for (int e = 0; e < k; ++e) y[rows[e] - 1] = y[rows[e] - 1] + (double)vals[e] * x[cols[e] - 1];
    for (int i = 0; i < n; ++i) {
        double t = (double)win_val[i] * feedback[win_col[i]];
        double xn = tanh(y[i] + t);
        x[i] = (1.0 - leakage) * x[i] + leakage * xn;
    }
    for (int i = 0; i < chunk_speedy; ++i) xa[i] = local_model[i];
    for (int i = 0; i < n; ++i) xa[chunk_speedy + i] = (i & 1) ? x[i] * x[i] : x[i];
    for (int o = 0; o < nout; ++o) outvec[o] = 0.0;
    for (int jj = 0; jj < n + chunk_speedy; ++jj) {
        double a = xa[jj];
        const float *wc = wout + (size_t)jj * nout;
        for (int o = 0; o < nout; ++o) outvec[o] = outvec[o] + (double)wc[o] * a;
    }
    orc_unstandardize_res(outvec, 2, 2, ZGRID, mean, std, 1, 1, 33, 35);
    free(y);
    free(xa);
}

/* orc_predict_f32 over many regions, OpenMP over regions (tests: the oracle chain of
 * the full-size hybrid step).  Per-region arrays as pointer tables; outvecs [nreg][nout]. */
void orc_predict_f32_regions(int nreg, int nthreads, const int *n, const int *ninp, const int *k,
                             const int *const *rows, const int *const *cols, const float *const *vals,
                             const int *const *win_col, const float *const *win_val, const float *const *wout,
                             int nout, int chunk_speedy, double leakage, const double *const *feedback,
                             const double *const *local_model, double *const *x, double *outvecs,
                             const double *const *mean, const double *const *std)
{
#pragma omp parallel for num_threads(nthreads) schedule(dynamic, 1)
    for (int r = 0; r < nreg; ++r)
        orc_predict_f32(n[r], ninp[r], k[r], rows[r], cols[r], vals[r], win_col[r], win_val[r], wout[r], nout,
                        chunk_speedy, leakage, feedback[r], local_model[r], x[r], outvecs + (size_t)r * nout,
                        mean[r], std[r]);
}

/* predict_slab_ml (mod_slab_ocean_reservoir.f90:1251-1296): the slab-ocean reservoir's
 * ML-only step --
 *   y = A x (COO in file order), temp = matmul(win, feedback)  (:1274-1275)
 *   x = (1-leak) x + leak tanh(y + temp)                        (:1277-1278)
 *   x_augment = x with x(2:n:2)**2                              (:1280-1283)
 *   outvec = matmul(wout, x_augment) * std(sst) + mean(sst)     (:1285-1287)
 * W_in compressed (one entry per row), fp32 weights as in the file. */
void orc_predict_slab_ml_f32(int n, int k, const int *rows, const int *cols, const float *vals, const int *win_col,
                             const float *win_val, const float *wout, int nout, double leakage,
                             const double *feedback, double *x, double *outvec, double mean_sst, double std_sst)
{
    double *y = (double *)calloc((size_t)n, sizeof(double));
    for (int e = 0; e < k; ++e) y[rows[e] - 1] = y[rows[e] - 1] + (double)vals[e] * x[cols[e] - 1];
    for (int i = 0; i < n; ++i) {
        double t = (double)win_val[i] * feedback[win_col[i]];
        double xn = tanh(y[i] + t);
        x[i] = (1.0 - leakage) * x[i] + leakage * xn;
    }
    for (int o = 0; o < nout; ++o) outvec[o] = 0.0;
    for (int jj = 0; jj < n; ++jj) {
        double a = (jj & 1) ? x[jj] * x[jj] : x[jj];
        const float *wc = wout + (size_t)jj * nout;
        for (int o = 0; o < nout; ++o) outvec[o] = outvec[o] + (double)wc[o] * a;
    }
    for (int o = 0; o < nout; ++o) {
        double t = outvec[o] * std_sst;
        outvec[o] = t + mean_sst;
    }
    free(y);
}

/* ------------------------------------------------------------------------- */
/* Exchange + tiling (mpires.f90:sendrecievegrid 218-780)                     */
/* Global grids use the reference layout: grid4d(4,96,48,8) column-major,     */
/* grid2d(96,48), precip(96,48).                                              */
/* ------------------------------------------------------------------------- */
#define G4(v, x, y, z) ((v) + 4 * ((x) + XGRID * ((y) + YGRID * (z))))
#define G2(x, y) ((x) + XGRID * (y))

/* tile_full_grid_with_local_state_vec_res1d (res_domain.f90:769-804) for every
 * region, then the root clips of sendrecievegrid: q >= 1e-6 (mpires.f90:448-450),
 * precip < 1e-5 -> 0 (:474-478). outvecs: [numregions][136]. */
void orc_assemble(int numregions, const double *outvecs, int outlen, double *grid4d, double *grid2d, double *precip)
{
    memset(grid4d, 0, sizeof(double) * 4 * XGRID * YGRID * ZGRID);
    memset(grid2d, 0, sizeof(double) * XGRID * YGRID);
    memset(precip, 0, sizeof(double) * XGRID * YGRID);
    for (int r = 0; r < numregions; ++r) {
        orc_region_geom g;
        orc_region_geometry(numregions, r, 1, &g);
        const double *ov = outvecs + (size_t)r * outlen;
        int rx = g.resxchunk, ry = g.resychunk, natmo = 4 * rx * ry * ZGRID;
        for (int z = 0; z < ZGRID; ++z)
            for (int y = 0; y < ry; ++y)
                for (int x = 0; x < rx; ++x)
                    for (int v = 0; v < 4; ++v)
                        grid4d[G4(v, g.res_xstart - 1 + x, g.res_ystart - 1 + y, z)] = ov[v + 4 * (x + rx * (y + ry * z))];
        for (int y = 0; y < ry; ++y)
            for (int x = 0; x < rx; ++x) {
                grid2d[G2(g.res_xstart - 1 + x, g.res_ystart - 1 + y)] = ov[natmo + x + rx * y];
                precip[G2(g.res_xstart - 1 + x, g.res_ystart - 1 + y)] = ov[natmo + rx * ry + x + rx * y];
            }
    }
    for (int z = 0; z < ZGRID; ++z)
        for (int y = 0; y < YGRID; ++y)
            for (int x = 0; x < XGRID; ++x)
                if (grid4d[G4(3, x, y, z)] < 0.000001) grid4d[G4(3, x, y, z)] = 0.000001;
    for (int i = 0; i < XGRID * YGRID; ++i)
        if (precip[i] < 0.00001) precip[i] = 0.0;
}

/* Feedback for one region (mpires.f90:562-563 tile_4d_and_logp_to_local_state_input,
 * then :734-751 tisr / sst / standardize_state_vec_input / precip standardisation).
 * feedback order: atmo(4,ix,iy,8) | logp(ix,iy) | precip(ix,iy) | sst? | tisr.
 * tisr_std: standardized tisr for this region (pre-standardized table, :905).
 * sst_std:  standardized sst input (NULL when the region has no sst input);
 *           kept as-is (slab-ocean feedback is out of scope). */
void orc_tile_feedback(int numregions, int region, const double *grid4d, const double *grid2d, const double *precip,
                       const double *mean, const double *std, const double *tisr_std, const double *sst_std,
                       double *feedback)
{
    orc_region_geom g;
    orc_region_geometry(numregions, region, 1, &g);
    int ix = g.inputxchunk, iy = g.inputychunk, in2d = ix * iy;
    int natmo = 4 * in2d * ZGRID;
    for (int z = 0; z < ZGRID; ++z)
        for (int ly = 0; ly < iy; ++ly)
            for (int lx = 0; lx < ix; ++lx) {
                int gx = orc_input_x(&g, lx + 1) - 1, gy = g.input_ystart - 1 + ly;
                for (int v = 0; v < 4; ++v) {
                    int l = v * ZGRID + z;
                    double t = grid4d[G4(v, gx, gy, z)] - mean[l];
                    feedback[v + 4 * (lx + ix * (ly + iy * z))] = t / std[l];
                }
            }
    for (int ly = 0; ly < iy; ++ly)
        for (int lx = 0; lx < ix; ++lx) {
            int gx = orc_input_x(&g, lx + 1) - 1, gy = g.input_ystart - 1 + ly;
            double t = grid2d[G2(gx, gy)] - mean[32];
            feedback[natmo + lx + ix * ly] = t / std[32];
            double tp = precip[G2(gx, gy)] - mean[34];
            feedback[natmo + in2d + lx + ix * ly] = tp / std[34];
        }
    int off = natmo + 2 * in2d;
    if (sst_std) {
        for (int i = 0; i < in2d; ++i) feedback[off + i] = sst_std[i];
        off += in2d;
    }
    for (int i = 0; i < in2d; ++i) feedback[off + i] = tisr_std[i];
}

/* local_model for one region from the SPEEDY forecast grids
 * (tile_4d_and_logp_full_grid_to_local_res_vec, res_domain.f90:1000-1031, then
 * standardize_state_vec_res, :1248-1293; forecast q clipped >= 1e-6 by
 * run_model, mpires.f90:1616-1618, which callers apply to the grid). */
void orc_tile_local_model(int numregions, int region, const double *fc4d, const double *fc2d, const double *mean,
                          const double *std, double *local_model)
{
    orc_region_geom g;
    orc_region_geometry(numregions, region, 1, &g);
    int rx = g.resxchunk, ry = g.resychunk, natmo = 4 * rx * ry * ZGRID;
    for (int z = 0; z < ZGRID; ++z)
        for (int y = 0; y < ry; ++y)
            for (int x = 0; x < rx; ++x)
                for (int v = 0; v < 4; ++v) {
                    int l = v * ZGRID + z;
                    double t = fc4d[G4(v, g.res_xstart - 1 + x, g.res_ystart - 1 + y, z)] - mean[l];
                    local_model[v + 4 * (x + rx * (y + ry * z))] = t / std[l];
                }
    for (int y = 0; y < ry; ++y)
        for (int x = 0; x < rx; ++x) {
            double t = fc2d[G2(g.res_xstart - 1 + x, g.res_ystart - 1 + y)] - mean[32];
            local_model[natmo + x + rx * y] = t / std[32];
        }
}

/* ------------------------------------------------------------------------- */
/* SPEEDY dynamical core: one `step` (SURVEY.md section 8a, row "step").      */
/*   indyns  src/ini_indyns.f90:1-128      impint  src/ini_impint.f90:1-153   */
/*   ludcmp/lubksb/inv src/spe_matinv.f90  geop    src/dyn_geop.f90:1-33      */
/*   step/hordif/timint src/dyn_step.f90:1-190                                */
/*   grtend  src/dyn_grtend.f90:1-279      sptend  src/dyn_sptend.f90:1-67    */
/*   implic  src/dyn_implic.f90:1-68                                          */
/* Physics (phypar, dyn_grtend.f90:225) is an input: its grid-point tendencies */
/* (u, v, t, q) are added where phypar adds them, or zero when absent.        */
/* Pinned against the reference step compiled as-is (tests/golden/dyn_ref.npz, */
/* tests/golden/make_dyn_golden.py).                                          */
/* Arrays: Fortran order.  vor/div/t(mx,nx,kx,2) complex = double[2][KX][NX][2*MX], */
/* ps(mx,nx,2), tr(mx,nx,kx,2,1), phys [4][KX][IL][IX].                        */
/* ------------------------------------------------------------------------- */
#define KX 8
#define KXP 9
#define LMAX 61
#define SF (2 * MX * NX)
#define GF (IX * IL)
static const double d_rearth = 6.371e+6, d_omega = 7.292e-05, d_grav = 9.81, d_akap = 2. / 7.;
static const double d_gamma = 6.0, d_hscale = 7.5, d_hshum = 2.5, d_thd = 2.4, d_thdd = 2.4, d_thds = 12.0,
                    d_tdrs = 24.0 * 30.0;
#define d_rgas (d_akap * 1004.)
static double hsg[KXP], dhs[KX], fsg[KX], dhsr[KX], fsgr[KX], coriol[IL], xgeop1[KX], xgeop2[KX];
static double dmp[NX][MX], dmpd[NX][MX], dmps[NX][MX], dmp1[NX][MX], dmp1d[NX][MX], dmp1s[NX][MX];
static double tcorv[KX], qcorv[KX];
static double tref[KX], tref1[KX], tref2[KX], tref3[KX], dhsx[KX], elz[NX][MX];
/* column-major (k, k1) matrices stored m[k1][k] (xc, xd) and xj(k, k1, l) as xj[l][k1][k] */
static double xc_[KX][KX], xd_[KX][KX], xj_[LMAX][KX][KX];

/* indyns (ini_indyns.f90:21-127); needs orc_spectral_init(rearth) first */
void orc_dyn_init(void)
{
    static const double h8[KXP] = {0.000, 0.050, 0.140, 0.260, 0.420, 0.600, 0.770, 0.900, 1.000};
    for (int k = 0; k < KXP; ++k) hsg[k] = h8[k];
    for (int k = 1; k <= KX; ++k) {
        dhs[k - 1] = hsg[k] - hsg[k - 1];
        fsg[k - 1] = 0.5 * (hsg[k] + hsg[k - 1]);
    }
    for (int k = 0; k < KX; ++k) {
        dhsr[k] = 0.5 / dhs[k];
        fsgr[k] = d_akap / (2. * fsg[k]);
    }
    double gsin[IL];
    for (int j = 1; j <= IY; ++j) {
        int jj = IL + 1 - j;
        gsin[j - 1] = -sia[j - 1];
        gsin[jj - 1] = sia[j - 1];
    }
    for (int j = 0; j < IL; ++j) coriol[j] = 2. * d_omega * gsin[j];
    for (int k = 1; k <= KX; ++k) {
        xgeop1[k - 1] = d_rgas * log(hsg[k] / fsg[k - 1]);
        if (k != KX) xgeop2[k] = d_rgas * log(fsg[k] / hsg[k]);
    }
    double hdiff = 1. / (d_thd * 3600.), hdifd = 1. / (d_thdd * 3600.), hdifs = 1. / (d_thds * 3600.);
    double rlap = 1. / (double)(NTRUN * (NTRUN + 1));
    for (int j = 1; j <= NX; ++j)
        for (int k = 1; k <= MX; ++k) {
            double twn = (double)(k - 1 + j - 1);
            double elap = (twn * (twn + 1.) * rlap);
            double elapn = pow(elap, 4); /* elap**npowhd, integer power */
            dmp[j - 1][k - 1] = hdiff * elapn;
            dmpd[j - 1][k - 1] = hdifd * elapn;
            dmps[j - 1][k - 1] = hdifs * elap;
        }
    double rgam = d_rgas * d_gamma / (1000. * d_grav), qexp = d_hscale / d_hshum;
    tcorv[0] = 0.;
    qcorv[0] = 0.;
    qcorv[1] = 0.;
    for (int k = 2; k <= KX; ++k) {
        tcorv[k - 1] = pow(fsg[k - 1], rgam);
        if (k > 2) qcorv[k - 1] = pow(fsg[k - 1], qexp);
    }
}

/* ludcmp / lubksb / inv (spe_matinv.f90), a(i, j) -> a[j][i] */
static void orc_ludcmp(double a[KX][KX], int n, int *indx)
{
    double vv[KX];
    for (int i = 0; i < n; ++i) {
        double aamax = 0.;
        for (int j = 0; j < n; ++j)
            if (fabs(a[j][i]) > aamax) aamax = fabs(a[j][i]);
        vv[i] = 1. / aamax;
    }
    for (int j = 0; j < n; ++j) {
        for (int i = 1; i < j; ++i) {
            double sum = a[j][i];
            for (int k = 0; k < i; ++k) sum = sum - a[k][i] * a[j][k];
            a[j][i] = sum;
        }
        double aamax = 0.;
        int imax = j;
        for (int i = j; i < n; ++i) {
            double sum = a[j][i];
            if (j > 0) {
                for (int k = 0; k < j; ++k) sum = sum - a[k][i] * a[j][k];
                a[j][i] = sum;
            }
            double dum = vv[i] * fabs(sum);
            if (dum >= aamax) {
                imax = i;
                aamax = dum;
            }
        }
        if (j != imax) {
            for (int k = 0; k < n; ++k) {
                double dum = a[k][imax];
                a[k][imax] = a[k][j];
                a[k][j] = dum;
            }
            vv[imax] = vv[j];
        }
        indx[j] = imax;
        if (j != n - 1) {
            double dum = 1. / a[j][j];
            for (int i = j + 1; i < n; ++i) a[j][i] = a[j][i] * dum;
        }
    }
}

static void orc_lubksb(double a[KX][KX], int n, const int *indx, double *b)
{
    int ii = 0; /* 1-based as the reference, 0 = unset */
    for (int i = 1; i <= n; ++i) {
        int ll = indx[i - 1] + 1;
        double sum = b[ll - 1];
        b[ll - 1] = b[i - 1];
        if (ii != 0) {
            for (int j = ii; j <= i - 1; ++j) sum = sum - a[j - 1][i - 1] * b[j - 1];
        } else if (sum != 0) {
            ii = i;
        }
        b[i - 1] = sum;
    }
    for (int i = n; i >= 1; --i) {
        double sum = b[i - 1];
        for (int j = i + 1; j <= n; ++j) sum = sum - a[j - 1][i - 1] * b[j - 1];
        b[i - 1] = sum / a[i - 1][i - 1];
    }
}

/* impint(dt, alph) (ini_impint.f90:26-152) */
void orc_dyn_impint(double dt, double alph)
{
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) {
            dmp1[n][m] = 1. / (1. + dmp[n][m] * dt);
            dmp1d[n][m] = 1. / (1. + dmpd[n][m] * dt);
            dmp1s[n][m] = 1. / (1. + dmps[n][m] * dt);
        }
    double rgam = d_rgas * d_gamma / (1000. * d_grav);
    for (int k = 0; k < KX; ++k) {
        tref[k] = 288. * pow(fmax(0.2, fsg[k]), rgam);
        tref1[k] = d_rgas * tref[k];
        tref2[k] = d_akap * tref[k];
        tref3[k] = fsgr[k] * tref[k];
    }
    double xi = dt * alph, xxi = xi / (d_rearth * d_rearth);
    for (int k = 0; k < KX; ++k) dhsx[k] = xi * dhs[k];
    for (int n = 1; n <= NX; ++n)
        for (int m = 1; m <= MX; ++m) {
            int ll = m + n - 2;
            elz[n - 1][m - 1] = (double)ll * (double)(ll + 1) * xxi;
        }
    double xa[KX][KX], ya[KX][KX], xb[KX][KX], xe[KX][KX], dsum[KX];
    memset(xa, 0, sizeof xa);
    memset(xb, 0, sizeof xb);
    for (int k = 0; k < KX; ++k)
        for (int k1 = 0; k1 < KX; ++k1) ya[k1][k] = -d_akap * tref[k] * dhs[k1];
    for (int k = 1; k < KX; ++k) xa[k - 1][k] = 0.5 * (d_akap * tref[k] / fsg[k] - (tref[k] - tref[k - 1]) / dhs[k]);
    for (int k = 0; k < KX - 1; ++k) xa[k][k] = 0.5 * (d_akap * tref[k] / fsg[k] - (tref[k + 1] - tref[k]) / dhs[k]);
    dsum[0] = dhs[0];
    for (int k = 1; k < KX; ++k) dsum[k] = dsum[k - 1] + dhs[k];
    for (int k = 0; k < KX - 1; ++k)
        for (int k1 = 0; k1 < KX; ++k1) {
            xb[k1][k] = dhs[k1] * dsum[k];
            if (k1 <= k) xb[k1][k] = xb[k1][k] - dhs[k1];
        }
    for (int k = 0; k < KX; ++k)
        for (int k1 = 0; k1 < KX; ++k1) {
            xc_[k1][k] = ya[k1][k];
            for (int k2 = 0; k2 < KX - 1; ++k2) xc_[k1][k] = xc_[k1][k] + xa[k2][k] * xb[k1][k2];
        }
    memset(xd_, 0, sizeof xd_);
    for (int k = 0; k < KX; ++k)
        for (int k1 = k + 1; k1 < KX; ++k1) xd_[k1][k] = d_rgas * log(hsg[k1 + 1] / hsg[k1]);
    for (int k = 0; k < KX; ++k) xd_[k][k] = d_rgas * log(hsg[k + 1] / fsg[k]);
    for (int k = 0; k < KX; ++k)
        for (int k1 = 0; k1 < KX; ++k1) {
            xe[k1][k] = 0.;
            for (int k2 = 0; k2 < KX; ++k2) xe[k1][k] = xe[k1][k] + xd_[k2][k] * xc_[k1][k2];
        }
    for (int l = 1; l <= LMAX; ++l) {
        double xxx = ((double)l * (double)(l + 1)) / (d_rearth * d_rearth);
        double xf[KX][KX];
        int indx[KX];
        for (int k = 0; k < KX; ++k)
            for (int k1 = 0; k1 < KX; ++k1) xf[k1][k] = xi * xi * xxx * (d_rgas * tref[k] * dhs[k1] - xe[k1][k]);
        for (int k = 0; k < KX; ++k) xf[k][k] = xf[k][k] + 1.;
        double(*y)[KX] = xj_[l - 1];
        memset(y, 0, sizeof(double) * KX * KX);
        for (int i = 0; i < KX; ++i) y[i][i] = 1.;
        orc_ludcmp(xf, KX, indx);
        for (int i = 0; i < KX; ++i) orc_lubksb(xf, KX, indx, y[i]);
    }
    for (int k = 0; k < KX; ++k)
        for (int k1 = 0; k1 < KX; ++k1) xc_[k1][k] = xc_[k1][k] * xi;
}

#define SPX(a, lev, k) ((a) + ((size_t)(lev) * KX + (k)) * SF) /* field (.., k, lev) of a (mx,nx,kx,2) array */

/* geop(jj) (dyn_geop.f90:16-32) */
static void orc_geop(const double *t, const double *phis, int jj, double *phi)
{
    const double *tj = SPX(t, jj - 1, 0);
    for (int c = 0; c < SF; ++c) phi[(KX - 1) * SF + c] = phis[c] + xgeop1[KX - 1] * tj[(KX - 1) * SF + c];
    for (int k = KX - 2; k >= 0; --k)
        for (int c = 0; c < SF; ++c)
            phi[k * SF + c] = phi[(k + 1) * SF + c] + xgeop2[k + 1] * tj[(k + 1) * SF + c] + xgeop1[k] * tj[k * SF + c];
    for (int k = 2; k <= KX - 1; ++k) {
        double corf = xgeop1[k - 1] * 0.5 * log(hsg[k] / fsg[k - 1]) / log(fsg[k] / fsg[k - 2]);
        for (int n = 0; n < NX; ++n)
            for (int p = 0; p < 2; ++p)
                phi[(k - 1) * SF + C3(p, 0, n)] =
                    phi[(k - 1) * SF + C3(p, 0, n)] + corf * (tj[k * SF + C3(p, 0, n)] - tj[(k - 2) * SF + C3(p, 0, n)]);
    }
}

/* phypar's grid inputs of time level 1 (dyn_grtend.f90:223-226, phy_phypar.f90:54-66):
 * geop(1), then per level uvspec + grid(.,2) -> ug1, vg1; grid(t1), grid(q1),
 * grid(phi) -> tg1, qg1, phig1 [KX][GF]; grid(ps1) -> pslg1 [GF]. */
void orc_phys_inputs(const double *vor, const double *div, const double *t, const double *ps, const double *tr,
                     const double *phis, double *ug1, double *vg1, double *tg1, double *qg1, double *phig1,
                     double *pslg1)
{
    static double phi[KX * SF], uc[SF], vc[SF];
    orc_geop(t, phis, 1, phi);
    for (int k = 0; k < KX; ++k) {
        orc_uvspec(SPX(vor, 0, k), SPX(div, 0, k), uc, vc);
        orc_grid(uc, ug1 + (size_t)k * GF, 2);
        orc_grid(vc, vg1 + (size_t)k * GF, 2);
    }
    for (int k = 0; k < KX; ++k) {
        orc_grid(SPX(t, 0, k), tg1 + (size_t)k * GF, 1);
        orc_grid(SPX(tr, 0, k), qg1 + (size_t)k * GF, 1);
        orc_grid(phi + (size_t)k * SF, phig1 + (size_t)k * GF, 1);
    }
    orc_grid(ps, pslg1, 1);
}

/* grtend(vordt, divdt, tdt, psdt, trdt, 1, j2) (dyn_grtend.f90:61-278) */
static void orc_grtend(const double *vor, const double *div, const double *t, const double *ps, const double *tr,
                       const double *phys, int j2, double *vordt, double *divdt, double *tdt, double *psdt,
                       double *trdt)
{
    static double ug[KX][GF], vg[KX][GF], tg[KX][GF], vorg[KX][GF], divg[KX][GF], tgg[KX][GF], puv[KX][GF];
    static double trg[KX][GF], utend[KX][GF], vtend[KX][GF], ttend[KX][GF], trtend[KX][GF];
    static double sigdt[KXP][GF], sigm[KXP][GF], temp[KXP][GF];
    static double px[GF], py[GF], umean[GF], vmean[GF], dmean[GF], dumr[3][GF];
    static double dumc[3][SF];
    const int l2 = j2 - 1;
    for (int k = 0; k < KX; ++k) {
        orc_grid(SPX(vor, l2, k), vorg[k], 1);
        orc_grid(SPX(div, l2, k), divg[k], 1);
        orc_grid(SPX(t, l2, k), tg[k], 1);
        orc_grid(SPX(tr, l2, k), trg[k], 1);
        orc_uvspec(SPX(vor, l2, k), SPX(div, l2, k), dumc[0], dumc[1]);
        orc_grid(dumc[1], vg[k], 2);
        orc_grid(dumc[0], ug[k], 2);
        for (int j = 0; j < IL; ++j)
            for (int i = 0; i < IX; ++i) vorg[k][j * IX + i] = vorg[k][j * IX + i] + coriol[j];
    }
    for (int g = 0; g < GF; ++g) umean[g] = vmean[g] = dmean[g] = 0.0;
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g) {
            umean[g] = umean[g] + ug[k][g] * dhs[k];
            vmean[g] = vmean[g] + vg[k][g] * dhs[k];
            dmean[g] = dmean[g] + divg[k][g] * dhs[k];
        }
    orc_grad(ps + (size_t)l2 * SF, dumc[1], dumc[2]);
    orc_grid(dumc[1], px, 2);
    orc_grid(dumc[2], py, 2);
    for (int g = 0; g < GF; ++g) dumr[0][g] = -umean[g] * px[g] - vmean[g] * py[g];
    orc_spec(dumr[0], psdt);
    psdt[0] = psdt[1] = 0.0;
    for (int g = 0; g < GF; ++g) sigdt[0][g] = sigdt[KX][g] = sigm[0][g] = sigm[KX][g] = 0.0;
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g) puv[k][g] = (ug[k][g] - umean[g]) * px[g] + (vg[k][g] - vmean[g]) * py[g];
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g) {
            sigdt[k + 1][g] = sigdt[k][g] - dhs[k] * (puv[k][g] + divg[k][g] - dmean[g]);
            sigm[k + 1][g] = sigm[k][g] - dhs[k] * puv[k][g];
        }
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g) tgg[k][g] = tg[k][g] - tref[k];
    for (int g = 0; g < GF; ++g) {
        px[g] = d_rgas * px[g];
        py[g] = d_rgas * py[g];
    }
    for (int g = 0; g < GF; ++g) temp[0][g] = temp[KX][g] = 0.0;
    for (int k = 1; k < KX; ++k)
        for (int g = 0; g < GF; ++g) temp[k][g] = sigdt[k][g] * (ug[k][g] - ug[k - 1][g]);
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g)
            utend[k][g] = vg[k][g] * vorg[k][g] - tgg[k][g] * px[g] - (temp[k + 1][g] + temp[k][g]) * dhsr[k];
    for (int k = 1; k < KX; ++k)
        for (int g = 0; g < GF; ++g) temp[k][g] = sigdt[k][g] * (vg[k][g] - vg[k - 1][g]);
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g)
            vtend[k][g] = -ug[k][g] * vorg[k][g] - tgg[k][g] * py[g] - (temp[k + 1][g] + temp[k][g]) * dhsr[k];
    for (int k = 1; k < KX; ++k)
        for (int g = 0; g < GF; ++g)
            temp[k][g] = sigdt[k][g] * (tgg[k][g] - tgg[k - 1][g]) + sigm[k][g] * (tref[k] - tref[k - 1]);
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g)
            ttend[k][g] = tgg[k][g] * divg[k][g] - (temp[k + 1][g] + temp[k][g]) * dhsr[k] +
                          fsgr[k] * tgg[k][g] * (sigdt[k + 1][g] + sigdt[k][g]) +
                          tref3[k] * (sigm[k + 1][g] + sigm[k][g]) + d_akap * (tg[k][g] * puv[k][g] - tgg[k][g] * dmean[g]);
    for (int k = 1; k < KX; ++k)
        for (int g = 0; g < GF; ++g) temp[k][g] = sigdt[k][g] * (trg[k][g] - trg[k - 1][g]);
    for (int g = 0; g < GF; ++g) temp[1][g] = temp[2][g] = 0.;
    for (int k = 0; k < KX; ++k)
        for (int g = 0; g < GF; ++g) trtend[k][g] = trg[k][g] * divg[k][g] - (temp[k + 1][g] + temp[k][g]) * dhsr[k];
    if (phys) /* phypar's additions (dyn_grtend.f90:223-226) */
        for (int k = 0; k < KX; ++k)
            for (int g = 0; g < GF; ++g) {
                utend[k][g] = utend[k][g] + phys[(0 * KX + k) * GF + g];
                vtend[k][g] = vtend[k][g] + phys[(1 * KX + k) * GF + g];
                ttend[k][g] = ttend[k][g] + phys[(2 * KX + k) * GF + g];
                trtend[k][g] = trtend[k][g] + phys[(3 * KX + k) * GF + g];
            }
    for (int k = 0; k < KX; ++k) {
        orc_vdspec(utend[k], vtend[k], vordt + k * SF, divdt + k * SF, 2);
        for (int g = 0; g < GF; ++g) {
            dumr[0][g] = 0.5 * (ug[k][g] * ug[k][g] + vg[k][g] * vg[k][g]);
            dumr[1][g] = -ug[k][g] * tgg[k][g];
            dumr[2][g] = -vg[k][g] * tgg[k][g];
        }
        orc_spec(dumr[0], dumc[0]);
        orc_lap(dumc[0], dumc[1]);
        for (int c = 0; c < SF; ++c) divdt[k * SF + c] = divdt[k * SF + c] - dumc[1][c];
        orc_vdspec(dumr[1], dumr[2], dumc[0], tdt + k * SF, 2);
        orc_spec(ttend[k], dumc[1]);
        for (int c = 0; c < SF; ++c) tdt[k * SF + c] = tdt[k * SF + c] + dumc[1][c];
        for (int g = 0; g < GF; ++g) {
            dumr[1][g] = -ug[k][g] * trg[k][g];
            dumr[2][g] = -vg[k][g] * trg[k][g];
        }
        orc_spec(trtend[k], dumc[1]);
        orc_vdspec(dumr[1], dumr[2], dumc[0], trdt + k * SF, 2);
        for (int c = 0; c < SF; ++c) trdt[k * SF + c] = trdt[k * SF + c] + dumc[1][c];
    }
}

/* sptend(divdt, tdt, psdt, j4) (dyn_sptend.f90:29-66); writes phi = geop(j4) */
static void orc_sptend(const double *div, const double *t, const double *ps, const double *phis, int j4,
                       double *divdt, double *tdt, double *psdt, double *phi)
{
    static double dmeanc[SF], sigdtc[KXP][SF], dumk[KXP][SF], dumc[2][SF];
    for (int c = 0; c < SF; ++c) dmeanc[c] = 0.0;
    for (int k = 0; k < KX; ++k)
        for (int c = 0; c < SF; ++c) dmeanc[c] = dmeanc[c] + SPX(div, j4 - 1, k)[c] * dhs[k];
    for (int c = 0; c < SF; ++c) psdt[c] = psdt[c] - dmeanc[c];
    psdt[0] = psdt[1] = 0.0;
    for (int c = 0; c < SF; ++c) sigdtc[0][c] = sigdtc[KX][c] = 0.0;
    for (int k = 0; k < KX - 1; ++k)
        for (int c = 0; c < SF; ++c) sigdtc[k + 1][c] = sigdtc[k][c] - dhs[k] * (SPX(div, j4 - 1, k)[c] - dmeanc[c]);
    for (int c = 0; c < SF; ++c) dumk[0][c] = dumk[KX][c] = 0.0;
    for (int k = 1; k < KX; ++k)
        for (int c = 0; c < SF; ++c) dumk[k][c] = sigdtc[k][c] * (tref[k] - tref[k - 1]);
    for (int k = 0; k < KX; ++k)
        for (int c = 0; c < SF; ++c)
            tdt[k * SF + c] = tdt[k * SF + c] - (dumk[k + 1][c] + dumk[k][c]) * dhsr[k] +
                              tref3[k] * (sigdtc[k + 1][c] + sigdtc[k][c]) - tref2[k] * dmeanc[c];
    orc_geop(t, phis, j4, phi);
    for (int k = 0; k < KX; ++k) {
        for (int c = 0; c < SF; ++c) dumc[0][c] = phi[k * SF + c] + d_rgas * tref[k] * ps[(size_t)(j4 - 1) * SF + c];
        orc_lap(dumc[0], dumc[1]);
        for (int c = 0; c < SF; ++c) divdt[k * SF + c] = divdt[k * SF + c] - dumc[1][c];
    }
}

/* implic(divdt, tdt, psdt) (dyn_implic.f90:22-67) */
static void orc_implic(double *divdt, double *tdt, double *psdt)
{
    static double ye[KX][SF], yf[KX][SF];
    memset(ye, 0, sizeof ye);
    for (int k1 = 0; k1 < KX; ++k1)
        for (int k = 0; k < KX; ++k)
            for (int c = 0; c < SF; ++c) ye[k][c] = ye[k][c] + xd_[k1][k] * tdt[k1 * SF + c];
    for (int k = 0; k < KX; ++k)
        for (int c = 0; c < SF; ++c) ye[k][c] = ye[k][c] + tref1[k] * psdt[c];
    for (int k = 0; k < KX; ++k)
        for (int n = 0; n < NX; ++n)
            for (int m = 0; m < MX; ++m)
                for (int p = 0; p < 2; ++p)
                    yf[k][C3(p, m, n)] = divdt[k * SF + C3(p, m, n)] + elz[n][m] * ye[k][C3(p, m, n)];
    memset(divdt, 0, sizeof(double) * KX * SF);
    for (int n = 0; n < NX; ++n)
        for (int m = 0; m < MX; ++m) {
            int ll = m + n;
            if (ll == 0) continue;
            for (int k1 = 0; k1 < KX; ++k1)
                for (int k = 0; k < KX; ++k)
                    for (int p = 0; p < 2; ++p)
                        divdt[k * SF + C3(p, m, n)] =
                            divdt[k * SF + C3(p, m, n)] + xj_[ll - 1][k1][k] * yf[k1][C3(p, m, n)];
        }
    for (int k = 0; k < KX; ++k)
        for (int c = 0; c < SF; ++c) psdt[c] = psdt[c] - divdt[k * SF + c] * dhsx[k];
    for (int k = 0; k < KX; ++k)
        for (int k1 = 0; k1 < KX; ++k1)
            for (int c = 0; c < SF; ++c) tdt[k * SF + c] = tdt[k * SF + c] + xc_[k1][k] * divdt[k1 * SF + c];
}

/* hordif (dyn_step.f90:130-151) */
static void orc_hordif(int nlev, const double *field, double *fdt, double dm[NX][MX], double dm1[NX][MX])
{
    for (int k = 0; k < nlev; ++k)
        for (int n = 0; n < NX; ++n)
            for (int m = 0; m < MX; ++m)
                for (int p = 0; p < 2; ++p) {
                    int c = k * SF + C3(p, m, n);
                    fdt[c] = (fdt[c] - dm[n][m] * field[c]) * dm1[n][m];
                }
}

/* timint (dyn_step.f90:153-190) */
static void orc_timint(int j1, double dt, double eps, double wil, int nlev, double *field, double *fdt)
{
    for (int k = 0; k < nlev; ++k) orc_trunct(fdt + k * SF);
    for (int k = 0; k < nlev; ++k)
        for (int c = 0; c < SF; ++c) {
            double *f1 = field + (size_t)k * SF + c, *f2 = field + ((size_t)nlev + k) * SF + c;
            double *fj1 = (j1 == 1) ? f1 : f2;
            double fnew = *f1 + dt * fdt[k * SF + c];
            *f1 = *fj1 + wil * eps * (*f1 - 2 * *fj1 + fnew);
            *f2 = fnew - (1 - wil) * eps * (*f1 - 2 * *fj1 + fnew);
        }
}

/* step(j1, j2, dt, alph, rob, wil) (dyn_step.f90:1-128).  phys may be NULL.
 * phi (KX spectral fields) receives geop(j4); tend (optional, 4*KX+1 fields:
 * vordt|divdt|tdt|trdt|psdt) receives the final tendencies before timint. */
void orc_dyn_step(double *vor, double *div, double *t, double *ps, double *tr, const double *phis, const double *tcorh,
                  const double *qcorh, const double *phys, int j1, int j2, double dt, double alph, double rob,
                  double wil, double *phi, double *tend)
{
    static double vordt[KX * SF], divdt[KX * SF], tdt[KX * SF], trdt[KX * SF], psdt[SF], ctmp[KX * SF];
    static double phil[KX * SF];
    orc_grtend(vor, div, t, ps, tr, phys, j2, vordt, divdt, tdt, psdt, trdt);
    if (alph == 0.) {
        orc_sptend(div, t, ps, phis, j2, divdt, tdt, psdt, phil);
    } else {
        orc_sptend(div, t, ps, phis, 1, divdt, tdt, psdt, phil);
        orc_implic(divdt, tdt, psdt);
    }
    if (phi) memcpy(phi, phil, sizeof phil);
    orc_hordif(KX, vor, vordt, dmp, dmp1);
    orc_hordif(KX, div, divdt, dmpd, dmp1d);
    for (int k = 0; k < KX; ++k)
        for (int n = 0; n < NX; ++n)
            for (int m = 0; m < MX; ++m)
                for (int p = 0; p < 2; ++p)
                    ctmp[k * SF + C3(p, m, n)] = t[k * SF + C3(p, m, n)] + tcorh[C3(p, m, n)] * tcorv[k];
    orc_hordif(KX, ctmp, tdt, dmp, dmp1);
    double sdrag = 1. / (d_tdrs * 3600.);
    for (int n = 0; n < NX; ++n)
        for (int p = 0; p < 2; ++p) {
            vordt[C3(p, 0, n)] = vordt[C3(p, 0, n)] - sdrag * vor[C3(p, 0, n)];
            divdt[C3(p, 0, n)] = divdt[C3(p, 0, n)] - sdrag * div[C3(p, 0, n)];
        }
    orc_hordif(1, vor, vordt, dmps, dmp1s);
    orc_hordif(1, div, divdt, dmps, dmp1s);
    orc_hordif(1, ctmp, tdt, dmps, dmp1s);
    for (int k = 0; k < KX; ++k)
        for (int n = 0; n < NX; ++n)
            for (int m = 0; m < MX; ++m)
                for (int p = 0; p < 2; ++p)
                    ctmp[k * SF + C3(p, m, n)] = tr[k * SF + C3(p, m, n)] + qcorh[C3(p, m, n)] * qcorv[k];
    orc_hordif(KX, ctmp, trdt, dmpd, dmp1d);
    if (tend) {
        memcpy(tend, vordt, sizeof vordt);
        memcpy(tend + KX * SF, divdt, sizeof divdt);
        memcpy(tend + 2 * KX * SF, tdt, sizeof tdt);
        memcpy(tend + 3 * KX * SF, trdt, sizeof trdt);
        memcpy(tend + 4 * KX * SF, psdt, sizeof psdt);
    }
    if (dt <= 0.) return;
    double eps = (j1 == 1) ? 0. : rob;
    orc_timint(j1, dt, eps, wil, 1, ps, psdt);
    orc_timint(j1, dt, eps, wil, KX, vor, vordt);
    orc_timint(j1, dt, eps, wil, KX, div, divdt);
    orc_timint(j1, dt, eps, wil, KX, t, tdt);
    orc_timint(j1, dt, eps, wil, KX, tr, trdt);
}

/* ------------------------------------------------------------------------- */
/* SPEEDY window entry / exit: iogrid(30) / iogrid(31) (ppo_iogrid.f90:497-601) */
/* grid4d = variables3d(4, ix, il, kx) (var = T, u, v, q), logp(ix, il).       */
/* Pinning: ppo_iogrid.f90 needs mpires/mod_utilities (MPI) and is not built   */
/* here; these two routines are compositions of vdspec/spec/trunct/uvspec/grid, */
/* each pinned to the reference by the spectral fixtures.                     */
/* ------------------------------------------------------------------------- */
#define G4I(v, i, j, k) ((v) + 4 * ((i) + IX * ((j) + IL * (k))))

/* spectral state level 1 -> gridded T, u, v, q, logp (iogrid(31), :573-595) */
static void orc_state_to_grid(const double *vor, const double *div, const double *t, const double *ps,
                              const double *tr, double *ugr, double *vgr, double *tgr, double *qgr, double *psgr)
{
    static double ucos[SF], vcos[SF];
    for (int k = 0; k < KX; ++k) {
        orc_uvspec(vor + k * SF, div + k * SF, ucos, vcos);
        orc_grid(ucos, ugr + k * GF, 2);
        orc_grid(vcos, vgr + k * GF, 2);
    }
    for (int k = 0; k < KX; ++k) {
        orc_grid(t + k * SF, tgr + k * GF, 1);
        orc_grid(tr + k * SF, qgr + k * GF, 1);
    }
    orc_grid(ps, psgr, 1);
}

/* iogrid(30): writes level 1 of vor/div/t/tr/ps; minmax[8] = min/max of the
 * re-gridded u, v, t, q; returns is_safe_to_run_speedy (:556-571) */
int orc_iogrid30(const double *grid4d, const double *logp, double *vor, double *div, double *t, double *ps,
                 double *tr, double *minmax)
{
    static double ugr[KX * GF], vgr[KX * GF], tgr[KX * GF], qgr[KX * GF], psgr[GF];
    for (int k = 0; k < KX; ++k)
        for (int j = 0; j < IL; ++j)
            for (int i = 0; i < IX; ++i) {
                int g = k * GF + j * IX + i;
                /* real(4) copies (:503-511), q < 0 -> 0 on the real(4) copy (:516-518) */
                tgr[g] = (double)(float)grid4d[G4I(0, i, j, k)];
                ugr[g] = (double)(float)grid4d[G4I(1, i, j, k)];
                vgr[g] = (double)(float)grid4d[G4I(2, i, j, k)];
                float q4 = (float)grid4d[G4I(3, i, j, k)];
                if (q4 < 0.0f) q4 = 0.0f;
                qgr[g] = (double)q4;
            }
    for (int g = 0; g < GF; ++g) psgr[g] = (double)(float)logp[g];
    for (int k = 0; k < KX; ++k) {
        orc_vdspec(ugr + k * GF, vgr + k * GF, vor + k * SF, div + k * SF, 2);
        orc_spec(tgr + k * GF, t + k * SF);
        orc_spec(qgr + k * GF, tr + k * SF);
        orc_trunct(vor + k * SF);
        orc_trunct(div + k * SF);
        orc_trunct(t + k * SF);
        orc_trunct(tr + k * SF);
    }
    orc_spec(psgr, ps);
    orc_trunct(ps);
    orc_state_to_grid(vor, div, t, ps, tr, ugr, vgr, tgr, qgr, psgr);
    const double *f[4] = {ugr, vgr, tgr, qgr};
    for (int v = 0; v < 4; ++v) {
        double mn = f[v][0], mxv = f[v][0];
        for (int g = 1; g < KX * GF; ++g) {
            if (f[v][g] < mn) mn = f[v][g];
            if (f[v][g] > mxv) mxv = f[v][g];
        }
        minmax[2 * v] = mn;
        minmax[2 * v + 1] = mxv;
    }
    if (minmax[0] < -150.0 || minmax[1] > 150.0) return 0;
    if (minmax[2] < -120.0 || minmax[3] > 120.0) return 0;
    if (minmax[4] < 160.0 || minmax[5] > 330.0) return 0;
    if (minmax[6] < -6.0 || minmax[7] > 30.0) return 0;
    return 1;
}

/* iogrid(31): level 1 of the spectral state -> grid4d / logp (:573-595) */
void orc_iogrid31(const double *vor, const double *div, const double *t, const double *ps, const double *tr,
                  double *grid4d, double *logp)
{
    static double ugr[KX * GF], vgr[KX * GF], tgr[KX * GF], qgr[KX * GF];
    orc_state_to_grid(vor, div, t, ps, tr, ugr, vgr, tgr, qgr, logp);
    for (int k = 0; k < KX; ++k)
        for (int j = 0; j < IL; ++j)
            for (int i = 0; i < IX; ++i) {
                int g = k * GF + j * IX + i;
                grid4d[G4I(0, i, j, k)] = tgr[g];
                grid4d[G4I(1, i, j, k)] = ugr[g];
                grid4d[G4I(2, i, j, k)] = vgr[g];
                grid4d[G4I(3, i, j, k)] = qgr[g];
            }
}

/* ------------------------------------------------------------------------- */
/* W_out training (BASELINE configs[4])          */
/*   chunking_matmul  src/mod_reservoir.f90:1643-1699                         */
/*   fit_chunk_hybrid src/mod_reservoir.f90:1233-1332                         */
/*   mldivide -> LAPACK dgesv (src/mod_linalg.f90:109-151).  LAPACK is not    */
/*   vendored in the reference; dgesv's published algorithm (LU with partial */
/*   pivoting, dgetrf + dgetrs) is restated unblocked.  Parity is pinned on   */
/*   the reference's call sites only (no reference test covers training).    */
/* Layouts (column-major, as the reference): S = augmented_states(naug, m),   */
/* T = targetdata(nout, m), G = states_x_states_aug(naug, naug),              */
/* B = states_x_trainingdata_aug(nout, naug), wout(nout, naug).               */
/* ------------------------------------------------------------------------- */
void orc_train_accumulate(int naug, int nout, int m, const double *S, const double *T, double *G, double *B)
{
    /* temp = matmul(targetdata, transpose(augmented_states)); B += temp */
    for (int j = 0; j < naug; ++j)
        for (int o = 0; o < nout; ++o) {
            double s = 0.0;
            for (int t = 0; t < m; ++t) s += T[o + (size_t)nout * t] * S[j + (size_t)naug * t];
            B[o + (size_t)nout * j] += s;
        }
    /* DGEMM(augmented_states, transpose(augmented_states)); G += temp */
    for (int j = 0; j < naug; ++j)
        for (int i = 0; i < naug; ++i) {
            double s = 0.0;
            for (int t = 0; t < m; ++t) s += S[i + (size_t)naug * t] * S[j + (size_t)naug * t];
            G[i + (size_t)naug * j] += s;
        }
}

/* dgesv: A (n x n, column-major) overwritten by its LU factors, B (n x nrhs)
 * by the solution.  Returns info (0 = ok, k > 0: U(k,k) = 0). */
static int orc_dgesv(int n, int nrhs, double *A, double *B)
{
    int info = 0;
    int *ipiv = malloc(sizeof(int) * n);
    for (int j = 0; j < n; ++j) {
        int p = j;
        double amax = fabs(A[j + (size_t)n * j]);
        for (int i = j + 1; i < n; ++i)
            if (fabs(A[i + (size_t)n * j]) > amax) {
                amax = fabs(A[i + (size_t)n * j]);
                p = i;
            }
        ipiv[j] = p;
        if (A[p + (size_t)n * j] != 0.0) {
            if (p != j)
                for (int k = 0; k < n; ++k) {
                    double tmp = A[j + (size_t)n * k];
                    A[j + (size_t)n * k] = A[p + (size_t)n * k];
                    A[p + (size_t)n * k] = tmp;
                }
            double r = 1.0 / A[j + (size_t)n * j];
            for (int i = j + 1; i < n; ++i) A[i + (size_t)n * j] *= r;
        } else if (info == 0) {
            info = j + 1;
        }
        for (int k = j + 1; k < n; ++k) {
            double a = A[j + (size_t)n * k];
            if (a != 0.0)
                for (int i = j + 1; i < n; ++i) A[i + (size_t)n * k] -= A[i + (size_t)n * j] * a;
        }
    }
    if (info == 0)
        for (int c = 0; c < nrhs; ++c) {
            double *b = B + (size_t)n * c;
            for (int j = 0; j < n; ++j)
                if (ipiv[j] != j) {
                    double tmp = b[j];
                    b[j] = b[ipiv[j]];
                    b[ipiv[j]] = tmp;
                }
            for (int j = 0; j < n; ++j) /* L y = P b (unit lower) */
                for (int i = j + 1; i < n; ++i) b[i] -= b[j] * A[i + (size_t)n * j];
            for (int j = n - 1; j >= 0; --j) { /* U x = y */
                b[j] /= A[j + (size_t)n * j];
                for (int i = 0; i < j; ++i) b[i] -= b[j] * A[i + (size_t)n * j];
            }
        }
    free(ipiv);
    return info;
}

/* fit_chunk_hybrid (using_prior = 1) / the unsquared regularisation of the
 * no-prior branch, then mldivide(a_trans, b_trans), wout = transpose(b_trans).
 * G and B are consumed. Returns dgesv's info. */
int orc_train_solve(int naug, int nout, int ncs, double beta_res, double beta_model, int using_prior,
                    double prior_val, double *G, const double *B, double *wout)
{
    for (int i = 0; i < naug; ++i) {
        double add;
        if (using_prior)
            add = (i < ncs) ? pow(beta_model, 2.0) : pow(beta_res, 2.0);
        else
            add = (i < ncs) ? beta_model : beta_res;
        G[i + (size_t)naug * i] += add;
    }
    double *a_t = malloc(sizeof(double) * naug * naug), *b_t = malloc(sizeof(double) * naug * nout);
    for (int j = 0; j < naug; ++j)
        for (int i = 0; i < naug; ++i) a_t[i + (size_t)naug * j] = G[j + (size_t)naug * i];
    for (int o = 0; o < nout; ++o)
        for (int j = 0; j < naug; ++j) b_t[j + (size_t)naug * o] = B[o + (size_t)nout * j];
    if (using_prior) /* prior(i,i) = prior_val*beta_model**2, i <= chunk_size_speedy */
        for (int i = 0; i < ncs && i < nout; ++i) b_t[i + (size_t)naug * i] += prior_val * pow(beta_model, 2.0);
    int info = orc_dgesv(naug, nout, a_t, b_t);
    for (int o = 0; o < nout; ++o)
        for (int j = 0; j < naug; ++j) wout[o + (size_t)nout * j] = b_t[j + (size_t)naug * o];
    free(a_t);
    free(b_t);
    return info;
}

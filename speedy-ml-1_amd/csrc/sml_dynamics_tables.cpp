// sml_dynamics_tables.cpp -- restatement of SPEEDY's dynamics initialisation:
//   indyns  (src/ini_indyns.f90:1-128): sigma levels, Coriolis, hydrostatic and
//           horizontal-diffusion coefficients
//   impint  (src/ini_impint.f90:1-153): semi-implicit gravity-wave matrices for a
//           given (dt, alph), using ludcmp/lubksb/inv (src/spe_matinv.f90)
// Computed on the host once per (dt, alph) and uploaded by sml_dynamics.hip.
#include "sml_dynamics_tables.hpp"
#include "sml_physics.hpp"

#include <cmath>
#include <cstring>

namespace sml {

void build_dyn_indyns(const SpectralTables &sp, DynTables *d) {
    std::memset(d, 0, sizeof *d);
    const double hsg[kKXP] = {0.000, 0.050, 0.140, 0.260, 0.420, 0.600, 0.770, 0.900, 1.000};
    std::memcpy(d->hsg, hsg, sizeof hsg);
    for (int k = 0; k < kKX; ++k) {
        d->dhs[k] = d->hsg[k + 1] - d->hsg[k];
        d->fsg[k] = 0.5 * (d->hsg[k + 1] + d->hsg[k]);
    }
    for (int k = 0; k < kKX; ++k) {
        d->dhsr[k] = 0.5 / d->dhs[k];
        d->fsgr[k] = kAkap / (2. * d->fsg[k]);
    }
    for (int j = 0; j < kIY; ++j) {
        const int jj = kIL - 1 - j;
        const double rad1 = std::asin(sp.sia[j]);
        d->radang[j] = -rad1;
        d->radang[jj] = rad1;
        d->gsin[j] = -sp.sia[j];
        d->gsin[jj] = sp.sia[j];
    }
    for (int j = 0; j < kIL; ++j) d->coriol[j] = 2. * kOmega * d->gsin[j];
    for (int k = 0; k < kKX; ++k) {
        d->xgeop1[k] = kRgas * std::log(d->hsg[k + 1] / d->fsg[k]);
        if (k != kKX - 1) d->xgeop2[k + 1] = kRgas * std::log(d->fsg[k + 1] / d->hsg[k + 1]);
    }
    const double hdiff = 1. / (kThd * 3600.), hdifd = 1. / (kThdd * 3600.), hdifs = 1. / (kThds * 3600.);
    const double rlap = 1. / (double)(kNTRUN * (kNTRUN + 1));
    for (int n = 0; n < kNX; ++n)
        for (int m = 0; m < kMX; ++m) {
            const double twn = (double)(m + n);
            const double elap = (twn * (twn + 1.) * rlap);
            const double e2 = elap * elap, elapn = e2 * e2;  // elap**npowhd, npowhd = 4
            d->dmp[n][m] = hdiff * elapn;
            d->dmpd[n][m] = hdifd * elapn;
            d->dmps[n][m] = hdifs * elap;
        }
    const double rgam = kRgas * kGamma / (1000. * kGrav), qexp = kHscale / kHshum;
    d->tcorv[0] = d->qcorv[0] = d->qcorv[1] = 0.;
    for (int k = 1; k < kKX; ++k) {
        d->tcorv[k] = std::pow(d->fsg[k], rgam);
        if (k > 1) d->qcorv[k] = std::pow(d->fsg[k], qexp);
    }
    for (int k = 1; k < kKX - 1; ++k)
        d->corf[k] = d->xgeop1[k] * 0.5 * std::log(d->hsg[k + 1] / d->fsg[k]) /
                     std::log(d->fsg[k + 1] / d->fsg[k - 1]);
    std::memcpy(d->gradx, sp.gradx, sizeof d->gradx);
    std::memcpy(d->gradym, sp.gradym, sizeof d->gradym);
    std::memcpy(d->gradyp, sp.gradyp, sizeof d->gradyp);
    std::memcpy(d->uvdx, sp.uvdx, sizeof d->uvdx);
    std::memcpy(d->uvdym, sp.uvdym, sizeof d->uvdym);
    std::memcpy(d->uvdyp, sp.uvdyp, sizeof d->uvdyp);
    std::memcpy(d->vddym, sp.vddym, sizeof d->vddym);
    std::memcpy(d->vddyp, sp.vddyp, sizeof d->vddyp);
    std::memcpy(d->el2, sp.el2, sizeof d->el2);
    for (int n = 0; n < kNX; ++n)
        for (int m = 0; m < kMX; ++m) d->trfilt[n][m] = (m + n <= kNTRUN) ? 1.0 : 0.0;
}

// ludcmp / lubksb / inv (src/spe_matinv.f90), on a column-major n x n matrix a(i, j)
// stored [j][i].  `tiny` is declared integer in the reference, so it is 0.
static void ludcmp(double a[kKX][kKX], int n, int *indx) {
    double vv[kKX];
    for (int i = 0; i < n; ++i) {
        double aamax = 0.;
        for (int j = 0; j < n; ++j)
            if (std::fabs(a[j][i]) > aamax) aamax = std::fabs(a[j][i]);
        vv[i] = 1. / aamax;
    }
    for (int j = 0; j < n; ++j) {
        for (int i = 0; i < j; ++i) {
            double sum = a[j][i];
            if (i > 0) {
                for (int k = 0; k < i; ++k) sum = sum - a[k][i] * a[j][k];
                a[j][i] = sum;
            }
        }
        double aamax = 0.;
        int imax = j;
        for (int i = j; i < n; ++i) {
            double sum = a[j][i];
            if (j > 0) {
                for (int k = 0; k < j; ++k) sum = sum - a[k][i] * a[j][k];
                a[j][i] = sum;
            }
            const double dum = vv[i] * std::fabs(sum);
            if (dum >= aamax) {
                imax = i;
                aamax = dum;
            }
        }
        if (j != imax) {
            for (int k = 0; k < n; ++k) {
                const double dum = a[k][imax];
                a[k][imax] = a[k][j];
                a[k][j] = dum;
            }
            vv[imax] = vv[j];
        }
        indx[j] = imax;
        if (j != n - 1) {
            if (a[j][j] == 0.) a[j][j] = 0.;
            const double dum = 1. / a[j][j];
            for (int i = j + 1; i < n; ++i) a[j][i] = a[j][i] * dum;
        }
    }
}

static void lubksb(double a[kKX][kKX], int n, const int *indx, double *b) {
    int ii = -1;
    for (int i = 0; i < n; ++i) {
        const int ll = indx[i];
        double sum = b[ll];
        b[ll] = b[i];
        if (ii >= 0) {
            for (int j = ii; j < i; ++j) sum = sum - a[j][i] * b[j];
        } else if (sum != 0.) {
            ii = i;
        }
        b[i] = sum;
    }
    for (int i = n - 1; i >= 0; --i) {
        double sum = b[i];
        for (int j = i + 1; j < n; ++j) sum = sum - a[j][i] * b[j];
        b[i] = sum / a[i][i];
    }
}

static void inv(double a[kKX][kKX], double y[kKX][kKX], int n) {
    int indx[kKX];
    std::memset(y, 0, sizeof(double) * kKX * kKX);
    for (int i = 0; i < n; ++i) y[i][i] = 1.;
    ludcmp(a, n, indx);
    for (int i = 0; i < n; ++i) lubksb(a, n, indx, y[i]);
}

void build_dyn_impint(double dt, double alph, DynTables *d) {
    d->dt = dt;
    d->alph = alph;
    for (int n = 0; n < kNX; ++n)
        for (int m = 0; m < kMX; ++m) {
            d->dmp1[n][m] = 1. / (1. + d->dmp[n][m] * dt);
            d->dmp1d[n][m] = 1. / (1. + d->dmpd[n][m] * dt);
            d->dmp1s[n][m] = 1. / (1. + d->dmps[n][m] * dt);
        }
    const double rgam = kRgas * kGamma / (1000. * kGrav);
    for (int k = 0; k < kKX; ++k) {
        d->tref[k] = 288. * std::pow(std::fmax(0.2, d->fsg[k]), rgam);
        d->tref1[k] = kRgas * d->tref[k];
        d->tref2[k] = kAkap * d->tref[k];
        d->tref3[k] = d->fsgr[k] * d->tref[k];
    }
    const double xi = dt * alph, xxi = xi / (kRearth * kRearth);
    for (int k = 0; k < kKX; ++k) d->dhsx[k] = xi * d->dhs[k];
    for (int n = 0; n < kNX; ++n)
        for (int m = 0; m < kMX; ++m) {
            const int ll = m + n;
            d->elz[n][m] = (double)ll * (double)(ll + 1) * xxi;
        }
    // [col][row] storage of the reference's column-major (row, col) matrices
    double xa[kKX][kKX] = {}, ya[kKX][kKX], xb[kKX][kKX] = {}, xe[kKX][kKX], dsum[kKX];
    for (int k = 0; k < kKX; ++k)
        for (int k1 = 0; k1 < kKX; ++k1) ya[k1][k] = -kAkap * d->tref[k] * d->dhs[k1];
    for (int k = 1; k < kKX; ++k)
        xa[k - 1][k] = 0.5 * (kAkap * d->tref[k] / d->fsg[k] - (d->tref[k] - d->tref[k - 1]) / d->dhs[k]);
    for (int k = 0; k < kKX - 1; ++k)
        xa[k][k] = 0.5 * (kAkap * d->tref[k] / d->fsg[k] - (d->tref[k + 1] - d->tref[k]) / d->dhs[k]);
    dsum[0] = d->dhs[0];
    for (int k = 1; k < kKX; ++k) dsum[k] = dsum[k - 1] + d->dhs[k];
    for (int k = 0; k < kKX - 1; ++k)
        for (int k1 = 0; k1 < kKX; ++k1) {
            xb[k1][k] = d->dhs[k1] * dsum[k];
            if (k1 <= k) xb[k1][k] = xb[k1][k] - d->dhs[k1];
        }
    for (int k = 0; k < kKX; ++k)
        for (int k1 = 0; k1 < kKX; ++k1) {
            double s = ya[k1][k];
            for (int k2 = 0; k2 < kKX - 1; ++k2) s = s + xa[k2][k] * xb[k1][k2];
            d->xc[k1][k] = s;
        }
    std::memset(d->xd, 0, sizeof d->xd);
    for (int k = 0; k < kKX; ++k)
        for (int k1 = k + 1; k1 < kKX; ++k1) d->xd[k1][k] = kRgas * std::log(d->hsg[k1 + 1] / d->hsg[k1]);
    for (int k = 0; k < kKX; ++k) d->xd[k][k] = kRgas * std::log(d->hsg[k + 1] / d->fsg[k]);
    for (int k = 0; k < kKX; ++k)
        for (int k1 = 0; k1 < kKX; ++k1) {
            double s = 0.;
            for (int k2 = 0; k2 < kKX; ++k2) s = s + d->xd[k2][k] * d->xc[k1][k2];
            xe[k1][k] = s;
        }
    for (int l = 1; l <= kLMAX; ++l) {
        const double xxx = ((double)l * (double)(l + 1)) / (kRearth * kRearth);
        double xf[kKX][kKX];
        for (int k = 0; k < kKX; ++k)
            for (int k1 = 0; k1 < kKX; ++k1)
                xf[k1][k] = xi * xi * xxx * (kRgas * d->tref[k] * d->dhs[k1] - xe[k1][k]);
        for (int k = 0; k < kKX; ++k) xf[k][k] = xf[k][k] + 1.;
        inv(xf, d->xj[l - 1], kKX);
    }
    for (int k = 0; k < kKX; ++k)
        for (int k1 = 0; k1 < kKX; ++k1) d->xc[k1][k] = d->xc[k1][k] * xi;
}

// ---------------------------------------------------------------- physics
// inphys(hsg, ppl, radang) (src/ini_inphys.f90:22-50) and radset's longwave band
// fractions (src/phy_radiat.f90:659-688).
void build_phys_tables(const DynTables &dt, PhysTables *p) {
    std::memset(p, 0, sizeof *p);
    const double gg = phys::gg, p0 = phys::p0, cp = phys::cp;
    p->sigh[0] = dt.hsg[0];
    for (int k = 0; k < kKX; ++k) {
        p->sig[k] = 0.5 * (dt.hsg[k + 1] + dt.hsg[k]);
        p->sigl[k] = std::log(p->sig[k]);
        p->sigh[k + 1] = dt.hsg[k + 1];
        p->dsig[k] = dt.hsg[k + 1] - dt.hsg[k];
        p->grdsig[k] = gg / (p->dsig[k] * p0);
        p->grdscp[k] = p->grdsig[k] / cp;
    }
    // half-level interpolation weights; the last row extrapolates to sigma = 0.99
    for (int k = 0; k < kKX - 1; ++k) {
        p->wvi[k][0] = 1. / (p->sigl[k + 1] - p->sigl[k]);
        p->wvi[k][1] = (std::log(p->sigh[k + 1]) - p->sigl[k]) * p->wvi[k][0];
    }
    p->wvi[kKX - 1][0] = 0.;
    p->wvi[kKX - 1][1] = (std::log(0.99) - p->sigl[kKX - 1]) * p->wvi[kKX - 2][0];
    for (int j = 0; j < kIL; ++j) {
        p->slat[j] = std::sin(dt.radang[j]);
        p->clat[j] = std::cos(dt.radang[j]);
    }
    // fband(T, band): emission fraction of each of the 4 bands at temperature T
    const double eps1 = 1. - phys::epslw;
    for (int it = 200; it <= 320; ++it) {
        double *f = p->fband[it - 100];
        const double d1 = (double)((it - 247) * (it - 247)), d2 = (double)((it - 282) * (it - 282)),
                     d3 = (double)((it - 315) * (it - 315));
        f[1] = (0.148 - 3.0e-6 * d1) * eps1;
        f[2] = (0.356 - 5.2e-6 * d2) * eps1;
        f[3] = (0.314 + 1.0e-5 * d3) * eps1;
        f[0] = eps1 - (f[1] + f[2] + f[3]);
    }
    for (int b = 0; b < 4; ++b) {
        for (int it = 100; it < 200; ++it) p->fband[it - 100][b] = p->fband[200 - 100][b];
        for (int it = 321; it <= 400; ++it) p->fband[it - 100][b] = p->fband[320 - 100][b];
    }
}

// sol_oz + solar (src/phy_radiat.f90:1-121): zonal daily-mean insolation and
// ozone absorption, replicated along each latitude row.
void phys_sol_oz(const PhysTables &p, double tyear, double *out5) {
    double lat[5 * kIL];
    phys_sol_oz_lat(p, tyear, lat);
    for (int f = 0; f < 5; ++f)
        for (int j = 0; j < kIL; ++j)
            for (int i = 0; i < kIX; ++i) out5[(size_t)f * kNGP + j * kIX + i] = lat[f * kIL + j];
}

// newdate(0) (src/mod_date.f90:17-79, 365-day calendar, iseasc = 1) and the weights of
// forin5 (src/cpl_bcinterp.f90:25-56) and forint (:1-23) for imon = imont1, fmon = tmonth
void phys_fordate_weights(int imonth, int iday, ForDate *f) {
    static const int ncal365[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    int before = 0;  // ndaycal(imonth, 2)
    for (int m = 1; m < imonth; ++m) before += ncal365[m - 1];
    f->imont1 = imonth;
    f->tmonth = (iday - 0.5) / (double)ncal365[imonth - 1];
    f->tyear = (before + iday - 0.5) / (double)365;
    // forin5: non-linear, mean-conserving
    const double fmon = f->tmonth;
    int im2 = imonth - 2, im1 = imonth - 1, ip1 = imonth + 1, ip2 = imonth + 2;
    if (im2 < 1) im2 += 12;
    if (im1 < 1) im1 += 12;
    if (ip1 > 12) ip1 -= 12;
    if (ip2 > 12) ip2 -= 12;
    const double c0 = 1. / 12., t0 = c0 * fmon, t1 = c0 * (1. - fmon), t2 = 0.25 * fmon * (1 - fmon);
    f->w5[0] = -t1 + t2;
    f->w5[1] = -c0 + 8 * t1 - 6 * t2;
    f->w5[2] = 7 * c0 + 10 * t2;
    f->w5[3] = -c0 + 8 * t0 - 6 * t2;
    f->w5[4] = -t0 + t2;
    const int m5[5] = {im2, im1, imonth, ip1, ip2};
    for (int k = 0; k < 5; ++k) f->m5[k] = m5[k] - 1;
    // forint: linear between the month and its neighbour on the side of the date
    int imon2;
    if (fmon <= 0.5) {
        imon2 = imonth == 1 ? 12 : imonth - 1;
        f->wmon = 0.5 - fmon;
    } else {
        imon2 = imonth == 12 ? 1 : imonth + 1;
        f->wmon = fmon - 0.5;
    }
    f->mi[0] = imonth - 1;
    f->mi[1] = imon2 - 1;
}

void phys_sol_oz_lat(const PhysTables &p, double tyear, double *out5) {
    const double pi = 2. * std::asin(1.);
    // solar(tyear, 4 solc): declination and Earth-Sun distance (Hartmann 1994)
    const double a = 2. * pi * tyear;
    const double c1 = std::cos(a), s1 = std::sin(a);
    const double c2 = c1 * c1 - s1 * s1, s2 = 2. * s1 * c1;
    const double c3 = c1 * c2 - s1 * s2, s3 = s1 * c2 + s2 * c1;
    const double decl = 0.006918 - 0.399912 * c1 + 0.070257 * s1 - 0.006758 * c2 + 0.000907 * s2 - 0.002697 * c3 +
                        0.001480 * s3;
    const double fdis = 1.000110 + 0.034221 * c1 + 0.001280 * s1 + 0.000719 * c2 + 0.000077 * s2;
    const double cdecl = std::cos(decl), sdecl = std::sin(decl), tdecl = sdecl / cdecl;
    const double csolp = (4. * phys::solc) / pi;
    // sol_oz proper
    const double alpha = 4. * std::asin(1.) * (tyear + 10. / 365.), dalpha = 0.;
    const double coz1 = 1.0 * std::fmax(0., std::cos(alpha - dalpha)), coz2 = 1.8, azen = 1.0;
    const double rzen = -std::cos(alpha) * 23.45 * std::asin(1.) / 90.;
    const double czen = std::cos(rzen), szen = std::sin(rzen), fs0 = 6.;
    double *fsol = out5, *ozone = out5 + kIL, *ozupp = out5 + 2 * kIL, *zenit = out5 + 3 * kIL,
           *stratz = out5 + 4 * kIL;
    for (int j = 0; j < kIL; ++j) {
        const double ch0 = std::fmin(1., std::fmax(-1., -tdecl * p.slat[j] / p.clat[j]));
        const double h0 = std::acos(ch0), sh0 = std::sin(h0);
        const double top = csolp * fdis * (h0 * p.slat[j] * sdecl + sh0 * p.clat[j] * cdecl);
        const double flat2 = 1.5 * p.slat[j] * p.slat[j] - 0.5;
        double up = 0.5 * phys::epssw;
        double oz = 0.4 * phys::epssw * (1.0 + coz1 * p.slat[j] + coz2 * flat2);
        const double b = 1. - (p.clat[j] * czen + p.slat[j] * szen);
        const double zen = 1. + azen * (b * b);  // (..)**nzen, nzen = 2
        up = top * up * zen;
        oz = top * oz * zen;
        fsol[j] = top;
        ozone[j] = oz;
        ozupp[j] = up;
        zenit[j] = zen;
        stratz[j] = std::fmax(fs0 - top, 0.);
    }
}

// sflset (src/phy_suflux.f90:358-382): orographic drag factor
void phys_sflset(const double *phi0, double *forog) {
    const double rhdrag = 1. / (phys::gg * phys::hdrag);
    for (int j = 0; j < kNGP; ++j) forog[j] = 1. + phys::fhdrag * (1. - std::exp(-std::fmax(phi0[j], 0.) * rhdrag));
}

}  // namespace sml

// sml_dynamics_tables.hpp -- host-side constants of SPEEDY's dynamical core (T30L8).
#pragma once
#include "sml_spectral_tables.hpp"

namespace sml {

constexpr int kKX = 8, kKXP = 9, kLMAX = 61;  // mod_atparam.f90: kx, kxp, lmax = mxp+nx-2

// physical constants (mod_dyncon0.f90, mod_dyncon1.f90; -fdefault-real-8 literals)
constexpr double kRearth = 6.371e+6, kOmega = 7.292e-05, kGrav = 9.81;
constexpr double kAkap = 2. / 7., kRgas = (2. / 7.) * 1004.;
constexpr double kGamma = 6.0, kHscale = 7.5, kHshum = 2.5;
constexpr double kThd = 2.4, kThdd = 2.4, kThds = 12.0, kTdrs = 24.0 * 30.0;

// Arrays use the reference's Fortran index order flattened C-style with the
// FIRST Fortran index fastest: a(m, n) -> [n][m], xc(k, k1) -> [k1][k],
// xj(k, k1, l) -> [l][k1][k].
struct DynTables {
    // indyns (ini_indyns.f90:1-128)
    double hsg[kKXP], dhs[kKX], fsg[kKX], dhsr[kKX], fsgr[kKX];
    double radang[kIL], gsin[kIL], coriol[kIL];
    double xgeop1[kKX], xgeop2[kKX];
    double dmp[kNX][kMX], dmpd[kNX][kMX], dmps[kNX][kMX];
    double tcorv[kKX], qcorv[kKX];
    double corf[kKX];  // geop lapse-rate correction factors (dyn_geop.f90:27-31)
    // spectral-operator coefficients used inside the step (copied from parmtr)
    double gradx[kMX], gradym[kNX][kMX], gradyp[kNX][kMX];
    double uvdx[kNX][kMX], uvdym[kNX][kMX], uvdyp[kNX][kMX];
    double vddym[kNX][kMX], vddyp[kNX][kMX];
    double el2[kNX][kMX], trfilt[kNX][kMX];
    // impint (ini_impint.f90:1-153), depend on (dt, alph)
    double dt, alph;
    double dmp1[kNX][kMX], dmp1d[kNX][kMX], dmp1s[kNX][kMX];
    double tref[kKX], tref1[kKX], tref2[kKX], tref3[kKX];
    double xc[kKX][kKX], xd[kKX][kKX];
    double xj[kLMAX][kKX][kKX];
    double dhsx[kKX], elz[kNX][kMX];
};

// indyns constants (radius from the spectral tables)
void build_dyn_indyns(const SpectralTables &sp, DynTables *d);
// impint(dt, alph) constants
void build_dyn_impint(double dt, double alph, DynTables *d);

}  // namespace sml

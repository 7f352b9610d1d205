// sml_physics.hpp -- SPEEDY's column physics (phypar) as a device function.
//
// Reference: phypar (src/phy_phypar.f90:1-228) with the routines it calls:
//   shtorh  (src/phy_shtorh.f90)             saturation humidity
//   convmf  (src/phy_convmf.f90:22-238)      deep convection (mass flux)
//   lscond  (src/phy_lscond.f90:20-109)      large-scale condensation
//   cloud   (src/phy_radiat.f90:86-152)      cloud cover
//   radsw   (src/phy_radiat.f90:154-328)     shortwave + longwave transmissivities
//   radlw   (src/phy_radiat.f90:330-458)     longwave, downward (-1) and upward (1)
//   suflux  (src/phy_suflux.f90:1-355)       surface fluxes, land skin temperature
//   vdifsc  (src/phy_vdifsc.f90:17-124)      vertical diffusion, shallow convection
// Scope as the reference runs it in the hybrid path: icsea = 0, lrandf = .false.
// (nstrdf = 0, src/mod_tsteps.f90:72), sppt_on = .false. (:68); dmflux's flux
// accumulation (daily means for output) is not part of the tendencies.
//
// MI355X layout: the physics is column-local, so one thread owns one grid column
// (all 8 levels in registers; every level loop has a constant trip count so the
// per-level arrays stay in VGPRs -- runtime level bounds such as the cloud top or
// the convection top are predicates, not loop bounds).  Radiation state that the
// reference keeps in module variables between steps (tau2, stratc, tt_rsw, ssrd;
// refreshed when lradsw) lives in device buffers, field-major [..][ngp] so every
// access of a wave is coalesced.
#pragma once
#include "sml_dynamics_tables.hpp"
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#endif

namespace sml {

constexpr int kNGP = kIX * kIL;  // 4608 columns

// inphys (src/ini_inphys.f90:22-50) + radset (src/phy_radiat.f90:659-688), built on
// the host from indyns' hsg and radang.  Level index 0 = top (the reference's k = 1).
struct PhysTables {
    double sig[kKX], sigl[kKX], sigh[kKX + 1], dsig[kKX], grdsig[kKX], grdscp[kKX];
    double wvi[kKX][2];
    double slat[kIL], clat[kIL];
    double fband[301][4];  // fband(100:400, 4)
};

void build_phys_tables(const DynTables &dt, PhysTables *p);
// sol_oz(tyear) (src/phy_radiat.f90:1-121): fsol, ozone, ozupp, zenit, stratz [5][ngp]
void phys_sol_oz(const PhysTables &p, double tyear, double *out5);
// the same, one value per latitude row (sol_oz replicates it along the row): [5][il]
void phys_sol_oz_lat(const PhysTables &p, double tyear, double *out5);

// The forcing date of one window: newdate(0) with iseasc = 1 (src/mod_date.f90:17-79;
// agcm_init sets iyear / imonth / iday from run_model's calendar, ini_agcm_init.f90:
// 43-62) and the monthly interpolation weights the coupler applies at that date
// (forin5 / forint, src/cpl_bcinterp.f90:1-56).  Months 0-based.
struct ForDate {
    int imont1;             // 1..12 (imonth)
    double tmonth, tyear;   // (iday - 0.5) / ndays(imonth), (days before + iday - 0.5) / 365
    int m5[5];              // forin5: imon-2 .. imon+2, wrapped
    double w5[5];           // wm2, wm1, w0, wp1, wp2
    int mi[2];              // forint: imon, imon2
    double wmon;
};
void phys_fordate_weights(int imonth, int iday, ForDate *f);
// sflset (src/phy_suflux.f90:358-382): forog from phi0 [ngp]
void phys_sflset(const double *phi0, double *forog);

// boundary fields of phypar, each [ngp] (mod_surfcon, mod_var_land, mod_var_sea,
// mod_radcon, mod_sflcon); the order of sml_dyn_set_physics' bc argument
enum PhysBc {
    kBcFmask1 = 0, kBcPhis0, kBcStl, kBcSst, kBcSoilw, kBcAlbL, kBcAlbS, kBcAlbsfc, kBcSnowc,
    kBcFsol, kBcOzone, kBcOzupp, kBcZenit, kBcStratz, kBcForog, kNBc
};

// radiation state kept between steps, offsets in doubles into one buffer
constexpr size_t kRadTau2 = 0;                              // tau2 [4][kx][ngp]
constexpr size_t kRadStratc = kRadTau2 + 4 * kKX * kNGP;    // stratc [2][ngp]
constexpr size_t kRadTtRsw = kRadStratc + 2 * kNGP;         // tt_rsw [kx][ngp]
constexpr size_t kRadSsrd = kRadTtRsw + kKX * kNGP;         // ssrd [ngp]
constexpr size_t kRadSize = kRadSsrd + kNGP;

namespace phys {

// mod_physcon.f90
constexpr double p0 = 1.e+5, gg = 9.81, rd = 287., cp = 1004., alhc = 2501.0, sbc = 5.67e-8;
// mod_cnvcon.f90
constexpr double psmin = 0.8, trcnv = 6.0, rhbl = 0.9, rhil = 0.7, entmax = 0.5, smf = 0.8;
// mod_lsccon.f90
constexpr double trlsc = 4.0, rhlsc = 0.9, drhlsc = 0.1, rhblsc = 0.95;
// mod_vdicon.f90
constexpr double trshc = 6.0, trvdi = 24.0, trvds = 6.0, redshc = 0.5, rhgrad = 0.5, segrad = 0.1;
// mod_sflcon.f90 (fhum0 = 0: suflux's humidity-profile branch is inactive)
constexpr double fwind0 = 0.95, ftemp0 = 1.0, cdl = 2.4e-3, cds = 1.0e-3, chl = 1.2e-3, chs = 0.9e-3,
                 vgust = 5.0, ctday = 1.0e-2, dtheta = 3.0, fstab = 0.67, hdrag = 2000.0, fhdrag = 0.5,
                 clambda = 7.0, clambsn = 7.0;
// mod_radcon.f90
constexpr double solc = 342.0, rhcl1 = 0.30, rhcl2 = 1.00, qacl = 0.20, wpcl = 0.2, pmaxcl = 10.0,
                 clsmax = 0.60, clsminl = 0.15, gse_s0 = 0.25, gse_s1 = 0.40, albcl = 0.43, albcls = 0.50,
                 epssw = 0.020, epslw = 0.05, emisfc = 0.98, absdry = 0.033, absaer = 0.033, abswv1 = 0.022,
                 abswv2 = 15.000, abscl1 = 0.015, abscl2 = 0.15, ablwin = 0.3, ablco2 = 6.0, ablwv1 = 0.7,
                 ablwv2 = 50.0, ablcl1 = 12.0, ablcl2 = 0.6;

#ifdef __HIPCC__
// shtorh (src/phy_shtorh.f90): saturation specific humidity (g/kg) at pressure s*ps
__device__ inline double qsat_at(double ta, double ps, double s) {
    const double e0 = 6.108e-3, c1 = 17.269, c2 = 21.875, t0 = 273.16, t1 = 35.86, t2 = 7.66;
    const double q = (ta >= t0) ? e0 * exp(c1 * (ta - t0) / (ta - t1)) : e0 * exp(c2 * (ta - t0) / (ta - t2));
    return 622. * q / (s * ps - 0.378 * q);
}

// row fband(nint(t), 1:4) of the table fb[301][4] (global or an LDS copy); the
// index is clamped to the table (the reference reads outside it only for
// temperatures outside 100..400 K)
__device__ inline const double *fband_row(const double *fb, double t) {
    int it = (int)round(t);
    it = it < 100 ? 100 : (it > 400 ? 400 : it);
    return fb + (it - 100) * 4;
}

#endif  // __HIPCC__
}  // namespace phys

#ifdef __HIPCC__
// sub-phase stamps of the row kernel's physics, a profiling build only
// (-DSML_PSTAMPS, tools/probe_pst.py): lane 0 of each wave records wall_clock64 at
// slot s of its block (48 blocks x 32 slots); compiled out otherwise
#ifdef SML_PSTAMPS
static __device__ long long g_pst[kIL * 32];
#define SML_PST(s)                                                                          \
    do {                                                                                   \
        if ((threadIdx.x & 63) == 0) g_pst[blockIdx.x * 32 + (s)] = wall_clock64();         \
    } while (0)
// the same from one given thread (the quad row kernel's waves share roles)
#define SML_PST_T(s, t)                                                                     \
    do {                                                                                   \
        if (threadIdx.x == (t)) g_pst[blockIdx.x * 32 + (s)] = wall_clock64();              \
    } while (0)
#else
#define SML_PST(s) \
    do {           \
    } while (0)
#define SML_PST_T(s, t) \
    do {                \
    } while (0)
#endif

// phypar's pieces (phy_phypar.f90:79-196), composed by phys_column in the
// reference's order; k_st_gridspec also runs the moist / diffusion part and the
// longwave / surface part of a column on different waves (sml_dynamics.hip).
// 1.2 thermodynamic variables (phy_phypar.f90:79-94)
struct PhysThermo {
    double psg, rps;
    double qa[kKX], se[kKX], rh[kKX], qsat[kKX];
};

__device__ inline void phys_thermo(const double *ta, const double *qa_in, const double *phi, double psl,
                                   const PhysTables *P, PhysThermo &h) {
    using namespace phys;
    constexpr int NL = kKX;
    h.psg = exp(psl);
    h.rps = 1. / h.psg;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        h.qa[k] = fmax(qa_in[k], 0.);
        h.se[k] = cp * ta[k] + phi[k];
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        h.qsat[k] = qsat_at(ta[k], h.psg, P->sig[k]);
        h.rh[k] = h.qa[k] / h.qsat[k];
    }
}

// convmf's entrainment profile (phy_convmf.f90:52-60): entr(k), k = 2..nlev-1
// (1-based), normalised to entmax; a function of the sigma levels only
__device__ inline void phys_entr(const PhysTables *P, double (&entr)[kKX + 1]) {
    using namespace phys;
    constexpr int nl1 = kKX - 1;
#pragma unroll
    for (int k = 0; k <= kKX; ++k) entr[k] = 0.;
    double sentr = 0.;
#pragma unroll
    for (int k = 2; k <= nl1; ++k) {
        const double e = fmax(0., P->sig[k - 1] - 0.5);
        entr[k] = e * e;
        sentr = sentr + entr[k];
    }
    sentr = entmax / sentr;
#pragma unroll
    for (int k = 2; k <= nl1; ++k) entr[k] = entr[k] * sentr;
}

// convmf's trigger (phy_convmf.f90:62-118): the cloud top itop (nlev + 1: no
// convection), the humidity excess qdif; 1-based level indices as the reference
__device__ inline void phys_convmf_trigger(const PhysThermo &h, const PhysTables *P, int &itop_o, double &qdif_o) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1, nlev = NL, nlp = NL + 1;
    const double psg = h.psg;
    const double *qa = h.qa, *se = h.se, *qsat = h.qsat;
    double mss[NL + 1];
#pragma unroll
    for (int k = 2; k <= nlev; ++k) mss[k] = se[k - 1] + alhc * qsat[k - 1];
    const double rlhc = 1. / alhc;
    double qdif = 0., msthr = 0.;
    int itop = nlp;
    if (psg > psmin) {
        const double mse0 = se[nlev - 1] + alhc * qa[nlev - 1];
        double mse1 = se[nl1 - 1] + alhc * qa[nl1 - 1];
        mse1 = fmin(mse0, mse1);
        const double mss0 = fmax(mse0, mss[nlev]);
        int ktop1 = nlev, ktop2 = nlev;
#pragma unroll
        for (int k = nlev - 3; k >= 3; --k) {
            const double mss2 = mss[k] + P->wvi[k - 1][1] * (mss[k + 1] - mss[k]);
            if (mss0 > mss2) ktop1 = k;
            if (mse1 > mss2) {
                ktop2 = k;
                msthr = mss2;
            }
        }
        if (ktop1 < nlev) {
            const double qthr0 = rhbl * qsat[nlev - 1], qthr1 = rhbl * qsat[nl1 - 1];
            const bool lqthr = (qa[nlev - 1] > qthr0 && qa[nl1 - 1] > qthr1);
            if (ktop2 < nlev) {
                itop = ktop1;
                qdif = fmax(qa[nlev - 1] - qthr0, (mse0 - msthr) * rlhc);
            } else if (lqthr) {
                itop = ktop1;
                qdif = qa[nlev - 1] - qthr0;
            }
        }
    }
    itop_o = itop;
    qdif_o = qdif;
}

// 2.1 convmf (phy_convmf.f90:22-238), 1-based level indices as the reference: the
// unscaled fluxes dfse / dfqa of every level into tt_cnv / qt_cnv (level k at k - 1),
// the convective precipitation and the cloud top itop (nlev + 1: no convection)
__device__ inline void phys_convmf(const PhysThermo &h, const PhysTables *P, const double *entr, double *tt_cnv,
                                   double *qt_cnv, double &precnv_o, int &itop_o) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1;
    const double psg = h.psg;
    const double *qa = h.qa, *se = h.se, *qsat = h.qsat;
#pragma unroll
    for (int k = 0; k < NL; ++k) tt_cnv[k] = qt_cnv[k] = 0.;
    double cbmf = 0., precnv = 0.;
    int itop;
    {
        constexpr int nlev = NL, nlp = NL + 1;
        const double fqmax = 5., fm0 = p0 * P->dsig[nlev - 1] / (gg * trcnv * 3600), rdps = 2. / (1. - psmin);
        double qdif;
        phys_convmf_trigger(h, P, itop, qdif);
        if (itop != nlp) {  // itop is in 3 .. nlev-3 here
            double dfse[NL + 1], dfqa[NL + 1];
#pragma unroll
            for (int k = 0; k <= NL; ++k) dfse[k] = dfqa[k] = 0.;
            // boundary layer (cloud base), k = nlev
            const double qmax = fmax(1.01 * qa[nlev - 1], qsat[nlev - 1]);
            double sb = se[nl1 - 1] + P->wvi[nl1 - 1][1] * (se[nlev - 1] - se[nl1 - 1]);
            double qb = qa[nl1 - 1] + P->wvi[nl1 - 1][1] * (qa[nlev - 1] - qa[nl1 - 1]);
            qb = fmin(qb, qa[nlev - 1]);
            const double fpsa = psg * fmin(1., (psg - psmin) * rdps);
            double fmass = fm0 * fpsa * fmin(fqmax, qdif / (qmax - qb));
            cbmf = fmass;
            double fus = fmass * se[nlev - 1], fuq = fmass * qmax, fds = fmass * sb, fdq = fmass * qb;
            dfse[nlev] = fds - fus;
            dfqa[nlev] = fdq - fuq;
            // intermediate layers (entrainment), k = nlev-1 .. itop+1
#pragma unroll
            for (int k = nlev - 1; k >= 4; --k) {
                if (k < itop + 1) continue;
                const int k1 = k - 1;
                dfse[k] = fus - fds;
                dfqa[k] = fuq - fdq;
                const double enmass = entr[k] * psg * cbmf;
                fmass = fmass + enmass;
                fus = fus + enmass * se[k - 1];
                fuq = fuq + enmass * qa[k - 1];
                sb = se[k1 - 1] + P->wvi[k1 - 1][1] * (se[k - 1] - se[k1 - 1]);
                qb = qa[k1 - 1] + P->wvi[k1 - 1][1] * (qa[k - 1] - qa[k1 - 1]);
                fds = fmass * sb;
                fdq = fmass * qb;
                dfse[k] = dfse[k] + fds - fus;
                dfqa[k] = dfqa[k] + fdq - fuq;
                const double delq = rhil * qsat[k - 1] - qa[k - 1];
                if (delq > 0.0) {
                    const double fsq = smf * cbmf * delq;
                    dfqa[k] = dfqa[k] + fsq;
                    dfqa[nlev] = dfqa[nlev] - fsq;
                }
            }
            // top layer (condensation and detrainment), k = itop
#pragma unroll
            for (int k = 3; k <= nlev - 3; ++k) {
                if (k != itop) continue;
                const double qsatb = qsat[k - 1] + P->wvi[k - 1][1] * (qsat[k] - qsat[k - 1]);
                precnv = fmax(fuq - fmass * qsatb, 0.0);
                dfse[k] = fus - fds + alhc * precnv;
                dfqa[k] = fuq - fdq - precnv;
            }
#pragma unroll
            for (int k = 1; k <= nlev; ++k) {
                tt_cnv[k - 1] = dfse[k];
                qt_cnv[k - 1] = dfqa[k];
            }
        }
    }
    precnv_o = precnv;
    itop_o = itop;
}

// 2.1 convmf + 2.2 lscond: tt, qt = 0 + the convection + the condensation tendencies
// (phy_phypar.f90:96-119); precnv, precls and the cloud top (itop) for the
// shortwave, icnv for vdifsc
__device__ inline void phys_moist(const PhysThermo &h, const PhysTables *P, double *tt, double *qt, double &precnv_o,
                                  double &precls_o, int &itop_o, int &icnv_o) {
    using namespace phys;
    constexpr int NL = kKX;
    const double psg = h.psg, rps = h.rps;
    const double *qa = h.qa, *qsat = h.qsat;
    double entr[kKX + 1];
    phys_entr(P, entr);
    double tt_cnv[NL], qt_cnv[NL], precnv;
    int itop;
    phys_convmf(h, P, entr, tt_cnv, qt_cnv, precnv, itop);
#pragma unroll
    for (int k = 1; k < NL; ++k) {  // phy_phypar.f90:100-105, k = 2..nlev
        tt_cnv[k] = tt_cnv[k] * rps * P->grdscp[k];
        qt_cnv[k] = qt_cnv[k] * rps * P->grdsig[k];
    }
    const int icnv = NL - itop;  // :107-109

    // 2.2 lscond (phy_lscond.f90:20-109)
    double tt_lsc[NL], qt_lsc[NL];
    double precls = 0.;
    {
        const double qsmax = 10., rtlsc = 1. / (trlsc * 3600.), tfact = alhc / cp, prg = p0 / gg;
        const double psa2 = psg * psg;
        tt_lsc[0] = qt_lsc[0] = 0.;
#pragma unroll
        for (int k = 2; k <= NL; ++k) {
            const double sig2 = P->sig[k - 1] * P->sig[k - 1];
            double rhref = rhlsc + drhlsc * (sig2 - 1.);
            if (k == NL) rhref = fmax(rhref, rhblsc);
            const double dqmax = qsmax * sig2 * rtlsc;
            const double dqa = rhref * qsat[k - 1] - qa[k - 1];
            if (dqa < 0.0) {
                itop = (k < itop) ? k : itop;
                qt_lsc[k - 1] = dqa * rtlsc;
                tt_lsc[k - 1] = tfact * fmin(-qt_lsc[k - 1], dqmax * psa2);
            } else {
                qt_lsc[k - 1] = 0.;
                tt_lsc[k - 1] = 0.;
            }
        }
#pragma unroll
        for (int k = 2; k <= NL; ++k) precls = precls - (P->dsig[k - 1] * prg) * qt_lsc[k - 1];
        precls = precls * psg;
    }
    // :118-119 (input tendencies are zero here)
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        tt[k] = 0. + tt_cnv[k] + tt_lsc[k];
        qt[k] = 0. + qt_cnv[k] + qt_lsc[k];
    }
    precnv_o = precnv;
    precls_o = precls;
    itop_o = itop;
    icnv_o = icnv;
}

// column j's radiation state -- rad's tau2 (4 bands x kx), stratc (2), ssrd, tt_rsw
// (kx) -- in registers: on a shortwave step the longwave / surface chain takes what
// phys_sw computed straight from it instead of re-reading rad (a dependent memory
// round trip per field on the column's chain); otherwise rad_load reads it at once
struct RadCol {
    double tau[4][kKX];
    double strat[2], ssrd, ttrsw[kKX];
};

__device__ inline void rad_load(int j, const double *__restrict__ rad, RadCol &rc) {
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
#pragma unroll
        for (int k = 0; k < kKX; ++k) rc.tau[jb][k] = rad[kRadTau2 + ((size_t)jb * kKX + k) * kNGP + j];
    rc.strat[0] = rad[kRadStratc + j];
    rc.strat[1] = rad[kRadStratc + kNGP + j];
    rc.ssrd = rad[kRadSsrd + j];
#pragma unroll
    for (int k = 0; k < kKX; ++k) rc.ttrsw[k] = rad[kRadTtRsw + (size_t)k * kNGP + j];
}

// column j's boundary fields (bc[f][ngp], f < kNBc) in registers, loaded at once at
// the start of the column's chain: phys_sw and phys_lw_sfc read them in the middle of
// theirs, a dependent memory round trip each where the compiler left the load
__device__ inline void bc_load(int j, const double *__restrict__ bc, double (&bcv)[kNBc]) {
#pragma unroll
    for (int f = 0; f < kNBc; ++f) bcv[f] = bc[(size_t)f * kNGP + j];
}

// the fband rows of the column's levels (radlw's fband(nint(ta(k)), 1:4)), read once
// for both radlw passes as soon as ta is known
__device__ inline void fband_rows(const double *fbt, const double *ta, double (&fbk)[kKX][4]) {
#pragma unroll
    for (int k = 0; k < kKX; ++k) {
        const double *row = phys::fband_row(fbt, ta[k]);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) fbk[k][jb] = row[jb];
    }
}

// 3.1 shortwave radiation and longwave transmissivities (phy_phypar.f90:126-145),
// the lradsw steps only: the radiation state of column j into rc and rad
__device__ inline void phys_sw(int j, const PhysThermo &h, const double *phi, double precnv, double precls, int itop,
                               const double (&bcv)[kNBc], double *__restrict__ rad, const PhysTables *P,
                               RadCol &rc) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1;  // nl1: 1-based index of the level above the bottom
    (void)nl1;
    auto BC = [&](int f) { return bcv[f]; };
    auto TAU = [&](int jb, int k) -> double & { return rc.tau[jb][k]; };
    const double psg = h.psg, rps = h.rps;
    const double *qa = h.qa, *se = h.se, *rh = h.rh, *qsat = h.qsat;
    (void)psg; (void)rps; (void)qa; (void)se; (void)rh; (void)qsat;
        const double gse = (se[NL - 2] - se[NL - 1]) / (phi[NL - 2] - phi[NL - 1]);
        // cloud (phy_radiat.f90:123-152)
        constexpr int nlp = NL + 1;
        const double rrcl = 1. / (rhcl2 - rhcl1);
        double cloudc, clstr;
        int icltop;
        if (rh[nl1 - 1] > rhcl1) {
            cloudc = rh[nl1 - 1] - rhcl1;
            icltop = nl1;
        } else {
            cloudc = 0.;
            icltop = nlp;
        }
#pragma unroll
        for (int k = 3; k <= NL - 2; ++k) {
            const double drh = rh[k - 1] - rhcl1;
            if (drh > cloudc && qa[k - 1] > qacl) {
                cloudc = drh;
                icltop = k;
            }
        }
        const double cl1 = fmin(1., cloudc * rrcl);
        const double pr1 = fmin(pmaxcl, 86.4 * (precnv + precls));
        cloudc = fmin(1., wpcl * sqrt(pr1) + cl1 * cl1);
        icltop = (itop < icltop) ? itop : icltop;
        const double qcloud = qa[nl1 - 1];
        {
            const double clfact = 1.2, rgse = 1. / (gse_s1 - gse_s0);
            const double fst = fmax(0., fmin(1., rgse * (gse - gse_s0)));
            clstr = fst * fmax(clsmax - clfact * cloudc, 0.);
            const double clstrl = fmax(clstr, clsminl) * rh[NL - 1];
            clstr = clstr + BC(kBcFmask1) * (clstrl - clstr);
        }
        // radsw (phy_radiat.f90:154-328)
        const double fband2 = 0.05, fband1 = 1. - fband2;
        double t1[NL], t2[NL], t3[NL], dfabs[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            t1[k] = t2[k] = 0.0;
            t3[k] = (k + 1 == icltop) ? albcl * cloudc : 0.0;  // icltop <= nlev only
        }
        t3[NL - 1] = albcls * clstr;
        const double psaz = psg * BC(kBcZenit);
        const double acloud = cloudc * fmin(abscl1 * qcloud, abscl2);
        t1[0] = exp(-(psaz * P->dsig[0]) * absdry);
#pragma unroll
        for (int k = 2; k <= nl1; ++k) {
            const double abs1 = absdry + absaer * P->sig[k - 1] * P->sig[k - 1];
            const double deltap = psaz * P->dsig[k - 1];
            if (k >= icltop)
                t1[k - 1] = exp(-deltap * (abs1 + abswv1 * qa[k - 1] + acloud));
            else
                t1[k - 1] = exp(-deltap * (abs1 + abswv1 * qa[k - 1]));
        }
        {
            const double abs1 = absdry + absaer * P->sig[NL - 1] * P->sig[NL - 1];
            const double deltap = psaz * P->dsig[NL - 1];
            t1[NL - 1] = exp(-deltap * (abs1 + abswv1 * qa[NL - 1]));
        }
#pragma unroll
        for (int k = 2; k <= NL; ++k) t2[k - 1] = exp(-(psaz * P->dsig[k - 1]) * abswv2 * qa[k - 1]);
        const double fsol = BC(kBcFsol);
        double f1 = fsol * fband1, f2 = fsol * fband2;
        dfabs[0] = f1;
        f1 = t1[0] * (f1 - BC(kBcOzupp) * psg);
        dfabs[0] = dfabs[0] - f1;
        dfabs[1] = f1;
        f1 = t1[1] * (f1 - BC(kBcOzone) * psg);
        dfabs[1] = dfabs[1] - f1;
#pragma unroll
        for (int k = 3; k <= NL; ++k) {
            t3[k - 1] = f1 * t3[k - 1];
            f1 = f1 - t3[k - 1];
            dfabs[k - 1] = f1;
            f1 = t1[k - 1] * f1;
            dfabs[k - 1] = dfabs[k - 1] - f1;
        }
#pragma unroll
        for (int k = 2; k <= NL; ++k) {
            dfabs[k - 1] = dfabs[k - 1] + f2;
            f2 = t2[k - 1] * f2;
            dfabs[k - 1] = dfabs[k - 1] - f2;
        }
        const double fsfcd = f1 + f2;
        f1 = f1 * BC(kBcAlbsfc);
#pragma unroll
        for (int k = NL; k >= 1; --k) {
            dfabs[k - 1] = dfabs[k - 1] + f1;
            f1 = t1[k - 1] * f1;
            dfabs[k - 1] = dfabs[k - 1] - f1;
            f1 = f1 + t3[k - 1];
        }
        rc.ssrd = fsfcd;
        // longwave transmissivities (phy_radiat.f90:262-300)
        double deltap = psg * P->dsig[0];
        TAU(0, 0) = exp(-deltap * ablwin);
        TAU(1, 0) = exp(-deltap * ablco2);
        TAU(2, 0) = 1.;
        TAU(3, 0) = 1.;
#pragma unroll
        for (int k = 2; k <= NL; k += NL - 2) {
            deltap = psg * P->dsig[k - 1];
            TAU(0, k - 1) = exp(-deltap * ablwin);
            TAU(1, k - 1) = exp(-deltap * ablco2);
            TAU(2, k - 1) = exp(-deltap * ablwv1 * qa[k - 1]);
            TAU(3, k - 1) = exp(-deltap * ablwv2 * qa[k - 1]);
        }
        const double acl = cloudc * ablcl2;
#pragma unroll
        for (int k = 3; k <= nl1; ++k) {
            deltap = psg * P->dsig[k - 1];
            const double acloud1 = (k < icltop) ? acl : ablcl1 * cloudc;
            TAU(0, k - 1) = exp(-deltap * (ablwin + acloud1));
            TAU(1, k - 1) = exp(-deltap * ablco2);
            TAU(2, k - 1) = exp(-deltap * fmax(ablwv1 * qa[k - 1], acl));
            TAU(3, k - 1) = exp(-deltap * fmax(ablwv2 * qa[k - 1], acl));
        }
        const double eps1 = epslw / (P->dsig[0] + P->dsig[1]);
        rc.strat[0] = BC(kBcStratz) * psg;
        rc.strat[1] = eps1 * psg;
#pragma unroll
        for (int k = 0; k < NL; ++k) rc.ttrsw[k] = dfabs[k] * rps * P->grdscp[k];
        // the column's state for the steps until the next shortwave step
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int k = 0; k < NL; ++k) rad[kRadTau2 + ((size_t)jb * NL + k) * kNGP + j] = rc.tau[jb][k];
        rad[kRadStratc + j] = rc.strat[0];
        rad[kRadStratc + kNGP + j] = rc.strat[1];
        rad[kRadSsrd + j] = rc.ssrd;
#pragma unroll
        for (int k = 0; k < NL; ++k) rad[kRadTtRsw + (size_t)k * kNGP + j] = rc.ttrsw[k];
    }

// 3.2 radlw(-1), 3.3 suflux, 3.4 radlw(1) (phy_phypar.f90:147-179): the longwave
// temperature tendency tt_rlw and the surface fluxes of column j
__device__ inline void phys_lw_sfc(int j, const double *ua, const double *va, const double *ta, const double *qa,
                                   const double *phi, double psg, double rps, const double (&bcv)[kNBc],
                                   const RadCol &rc, const PhysTables *P, const double *fbt,
                                   const double (&fbk)[kKX][4], double *tt_rlw, double &ustr3_o, double &vstr3_o,
                                   double &shf3_o, double &evap3_o) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1;  // nl1: 1-based index of the level above the bottom
    (void)nl1;
    auto BC = [&](int f) { return bcv[f]; };
    auto TAU = [&](int jb, int k) { return rc.tau[jb][k]; };
    const int jlat = j / kIX;
    // 3.2 radlw(-1): downward longwave (phy_radiat.f90:330-413)
    double st4a1[NL], st4a2[NL], flux[4], dfabs[NL], fsfcd;
    // (fbk: fband(nint(ta(k)), 1:4), one table row per level for both radlw passes, fband_rows)
    {
#pragma unroll
        for (int k = 1; k <= nl1; ++k) st4a1[k - 1] = ta[k - 1] + P->wvi[k - 1][1] * (ta[k] - ta[k - 1]);
        st4a2[0] = 0.75 * ta[0] + 0.25 * st4a1[0];
        st4a2[1] = 0.50 * ta[1] + 0.25 * (st4a1[0] + st4a1[1]);
        const double anis = 1.0, anish = 0.5 * anis;
#pragma unroll
        for (int k = 3; k <= nl1; ++k) st4a2[k - 1] = anish * fmax(st4a1[k - 1] - st4a1[k - 2], 0.);
        st4a2[NL - 1] = anis * fmax(ta[NL - 1] - st4a1[nl1 - 1], 0.);
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const double x = st4a2[k];
            st4a1[k] = sbc * ((x * x) * (x * x));
            st4a2[k] = 0.;
        }
#pragma unroll
        for (int k = 3; k <= NL; ++k) {
            const double t = ta[k - 1];
            const double st3a = sbc * (t * t * t);
            st4a1[k - 1] = st3a * t;
            st4a2[k - 1] = 4. * st3a * st4a2[k - 1];
        }
        fsfcd = 0.0;
#pragma unroll
        for (int k = 0; k < NL; ++k) dfabs[k] = 0.0;
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            const double emis = 1. - TAU(jb, 0);
            const double brad = fbk[0][jb] * (st4a1[0] + emis * st4a2[0]);
            flux[jb] = emis * brad;
            dfabs[0] = dfabs[0] - flux[jb];
        }
        flux[2] = flux[3] = 0.0;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int k = 2; k <= NL; ++k) {
                const double tau = TAU(jb, k - 1);
                const double emis = 1. - tau;
                const double brad = fbk[k - 1][jb] * (st4a1[k - 1] + emis * st4a2[k - 1]);
                dfabs[k - 1] = dfabs[k - 1] + flux[jb];
                flux[jb] = tau * flux[jb] + emis * brad;
                dfabs[k - 1] = dfabs[k - 1] - flux[jb];
            }
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) fsfcd = fsfcd + emisfc * flux[jb];
        const double corlw = (epslw * emisfc) * st4a1[NL - 1];
        dfabs[NL - 1] = dfabs[NL - 1] - corlw;
        fsfcd = fsfcd + corlw;
    }
    const double slrd = fsfcd;
    SML_PST(2);

    // 3.3 suflux with lfluxland = .true. (phy_suflux.f90:1-355)
    double ustr3, vstr3, shf3, evap3, slru3, tsfc;
    {
        constexpr int nlev = NL;
        const double esbc = emisfc * sbc, esbc4 = 4. * esbc, dlambda = clambsn - clambda;
        const double u0 = fwind0 * ua[nlev - 1], v0 = fwind0 * va[nlev - 1];
        const double gtemp0 = 1. - ftemp0, rcp = 1. / cp, rdphi0 = -1. / (rd * 288. * P->sigl[nlev - 1]);
        const double phi0 = BC(kBcPhis0), fmask = BC(kBcFmask1), ssrdj = rc.ssrd;
        double t1[2], t2[2], denvvs[3], qsat0[2];
        const double dt1 = P->wvi[nlev - 1][1] * (ta[nlev - 1] - ta[nl1 - 1]);
        t1[0] = ta[nlev - 1] + dt1;
        t1[1] = t1[0] + phi0 * dt1 * rdphi0;
        t2[1] = ta[nlev - 1] + rcp * phi[nlev - 1];
        t2[0] = t2[1] - rcp * phi0;
        if (ta[nlev - 1] > ta[nl1 - 1]) {
            t1[0] = ftemp0 * t1[0] + gtemp0 * t2[0];
            t1[1] = ftemp0 * t1[1] + gtemp0 * t2[1];
        } else {
            t1[0] = ta[nlev - 1];
            t1[1] = ta[nlev - 1];
        }
        const double t0 = t1[1] + fmask * (t1[0] - t1[1]);
        const double prd = p0 / rd, vg2 = vgust * vgust;
        denvvs[0] = (prd * psg / t0) * sqrt(u0 * u0 + v0 * v0 + vg2);
        // land: skin temperature, fluxes, skin energy balance (lskineb)
        const double stl = BC(kBcStl), albl = BC(kBcAlbL);
        double tskin = stl + ctday * sqrt(P->clat[jlat]) * ssrdj * (1. - albl) * psg;
        const double rdth = fstab / dtheta, astab = 0.5;
        const double dthl = (tskin > t2[0]) ? fmin(dtheta, tskin - t2[0]) : fmax(-dtheta, astab * (tskin - t2[0]));
        denvvs[1] = denvvs[0] * (1. + dthl * rdth);
        const double cdldv = cdl * denvvs[0] * BC(kBcForog);
        const double ustr1 = -cdldv * ua[nlev - 1], vstr1 = -cdldv * va[nlev - 1];
        const double chlcp = chl * cp;
        double shf1 = chlcp * denvvs[1] * (tskin - t1[0]);
        const double q1l = qa[nlev - 1];  // fhum0 = 0
        qsat0[0] = qsat_at(tskin, psg, 1.);
        const double swav = BC(kBcSoilw);
        double evap1 = chl * denvvs[1] * fmax(0., swav * qsat0[0] - q1l);
        const double tsk3 = tskin * tskin * tskin;
        const double dslr = esbc4 * tsk3;
        double slru1 = esbc * tsk3 * tskin;
        double hfl1 = ssrdj * (1. - albl) + slrd - (slru1 + shf1 + alhc * evap1);
        const double clamb = clambda + BC(kBcSnowc) * dlambda;
        hfl1 = hfl1 - clamb * (tskin - stl);
        qsat0[1] = qsat_at(tskin + 1., psg, 1.);
        if (evap1 > 0)
            qsat0[1] = swav * (qsat0[1] - qsat0[0]);
        else
            qsat0[1] = 0.;
        const double dhfdt = clamb + dslr + chl * denvvs[1] * (cp + alhc * qsat0[1]);
        const double dtskin = hfl1 / dhfdt;
        tskin = tskin + dtskin;
        shf1 = shf1 + chlcp * denvvs[1] * dtskin;
        evap1 = evap1 + chl * denvvs[1] * qsat0[1] * dtskin;
        slru1 = slru1 + dslr * dtskin;
        // sea
        const double tsea = BC(kBcSst);
        const double dths = (tsea > t2[1]) ? fmin(dtheta, tsea - t2[1]) : fmax(-dtheta, astab * (tsea - t2[1]));
        denvvs[2] = denvvs[0] * (1. + dths * rdth);
        const double q1s = qa[nlev - 1];
        const double cdsdv = cds * denvvs[2];
        const double ustr2 = -cdsdv * ua[nlev - 1], vstr2 = -cdsdv * va[nlev - 1];
        const double chscp = chs * cp;
        const double shf2 = chscp * denvvs[2] * (tsea - t1[1]);
        const double qs = qsat_at(tsea, psg, 1.);
        const double evap2 = chs * denvvs[2] * (qs - q1s);
        const double ts2 = tsea * tsea;
        const double slru2 = esbc * (ts2 * ts2);
        // weighted averages with the land-sea mask
        ustr3 = ustr2 + fmask * (ustr1 - ustr2);
        vstr3 = vstr2 + fmask * (vstr1 - vstr2);
        shf3 = shf2 + fmask * (shf1 - shf2);
        evap3 = evap2 + fmask * (evap1 - evap2);
        slru3 = slru2 + fmask * (slru1 - slru2);
        tsfc = tsea + fmask * (stl - tsea);
    }

    SML_PST(3);
    // 3.4 radlw(1): upward longwave (phy_radiat.f90:414-458)
    {
        const double refsfc = 1. - emisfc, fsfcu = slru3;
        const double *fsr = fband_row(fbt, tsfc);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) flux[jb] = fsr[jb] * fsfcu + refsfc * flux[jb];
        dfabs[NL - 1] = dfabs[NL - 1] + epslw * fsfcu;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int k = NL; k >= 2; --k) {
                const double tau = TAU(jb, k - 1);
                const double emis = 1. - tau;
                const double brad = fbk[k - 1][jb] * (st4a1[k - 1] - emis * st4a2[k - 1]);
                dfabs[k - 1] = dfabs[k - 1] + flux[jb];
                flux[jb] = tau * flux[jb] + emis * brad;
                dfabs[k - 1] = dfabs[k - 1] - flux[jb];
            }
#pragma unroll
        for (int jb = 0; jb < 2; ++jb) {
            const double tau = TAU(jb, 0);
            const double emis = 1. - tau;
            const double brad = fbk[0][jb] * (st4a1[0] - emis * st4a2[0]);
            dfabs[0] = dfabs[0] + flux[jb];
            flux[jb] = tau * flux[jb] + emis * brad;
            dfabs[0] = dfabs[0] - flux[jb];
        }
        const double corlw1 = P->dsig[0] * rc.strat[1] * st4a1[0] + rc.strat[0];
        const double corlw2 = P->dsig[1] * rc.strat[1] * st4a1[1];
        dfabs[0] = dfabs[0] - corlw1;
        dfabs[1] = dfabs[1] - corlw2;
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) tt_rlw[k] = dfabs[k] * rps * P->grdscp[k];
    ustr3_o = ustr3;
    vstr3_o = vstr3;
    shf3_o = shf3;
    evap3_o = evap3;
}

// vdifsc's constants (phy_vdifsc.f90:36-57): functions of the sigma levels only
struct VdifK {
    double fshcq, fshcse, fvdiq, fvdise;
    double rsig[kKX], rsig1[kKX];  // rsig1(k), k = 1..nlev-1 (rsig1[kKX - 1] unused)
};
__device__ inline void phys_vdif_consts(const PhysTables *P, VdifK &v) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1, nlev = NL;
    const double cshc = P->dsig[nlev - 1] / 3600., cvdi = (P->sigh[nl1] - P->sigh[1]) / ((nl1 - 1) * 3600.);
    v.fshcq = cshc / trshc;
    v.fshcse = cshc / (trshc * cp);
    v.fvdiq = cvdi / trvdi;
    v.fvdise = cvdi / (trvds * cp);
#pragma unroll
    for (int k = 1; k <= nl1; ++k) {
        v.rsig[k - 1] = 1. / P->dsig[k - 1];
        v.rsig1[k - 1] = 1. / (1. - P->sigh[k]);
    }
    v.rsig[nlev - 1] = 1. / P->dsig[nlev - 1];
    v.rsig1[nlev - 1] = 0.;
}

// 4.1 vdifsc (phy_vdifsc.f90:17-124): ttv, qtv (utv = vtv = 0 here)
__device__ inline void phys_vdif(const PhysThermo &h, const double *phi, int icnv, const PhysTables *P, double *ttv,
                                 double *qtv) {
    using namespace phys;
    constexpr int NL = kKX, nl1 = kKX - 1;  // nl1: 1-based index of the level above the bottom
    (void)nl1;
    const double *qa = h.qa, *se = h.se, *rh = h.rh, *qsat = h.qsat;
    // 4.1 vdifsc (phy_vdifsc.f90:17-124)
#pragma unroll
    for (int k = 0; k < NL; ++k) ttv[k] = qtv[k] = 0.;
    {
        constexpr int nlev = NL;
        VdifK vk;
        phys_vdif_consts(P, vk);
        const double fshcq = vk.fshcq, fshcse = vk.fshcse, fvdiq = vk.fvdiq, fvdise = vk.fvdise;
        const double *rsig = vk.rsig, *rsig1 = vk.rsig1;
        double drh0 = rhgrad * (P->sig[nlev - 1] - P->sig[nl1 - 1]);
        double fvdiq2 = fvdiq * P->sigh[nl1];
        // shallow convection
        const double dmse = (se[nlev - 1] - se[nl1 - 1]) + alhc * (qa[nlev - 1] - qsat[nl1 - 1]);
        double drh = rh[nlev - 1] - rh[nl1 - 1];
        double fcnv = 1.;
        if (dmse >= 0.0) {
            if (icnv > 0) fcnv = redshc;
            const double fluxse = fcnv * fshcse * dmse;
            ttv[nl1 - 1] = fluxse * rsig[nl1 - 1];
            ttv[nlev - 1] = -fluxse * rsig[nlev - 1];
            if (drh >= 0.0) {
                const double fluxq = fcnv * fshcq * qsat[nlev - 1] * drh;
                qtv[nl1 - 1] = fluxq * rsig[nl1 - 1];
                qtv[nlev - 1] = -fluxq * rsig[nlev - 1];
            }
        } else if (drh >= drh0) {
            const double fluxq = fvdiq2 * qsat[nl1 - 1] * drh;
            qtv[nl1 - 1] = fluxq * rsig[nl1 - 1];
            qtv[nlev - 1] = -fluxq * rsig[nlev - 1];
        }
        // vertical diffusion of moisture above the PBL
#pragma unroll
        for (int k = 3; k <= nlev - 2; ++k)
            if (P->sigh[k] > 0.5) {
                drh0 = rhgrad * (P->sig[k] - P->sig[k - 1]);
                fvdiq2 = fvdiq * P->sigh[k];
                drh = rh[k] - rh[k - 1];
                if (drh >= drh0) {
                    const double fluxq = fvdiq2 * qsat[k - 1] * drh;
                    qtv[k - 1] = qtv[k - 1] + fluxq * rsig[k - 1];
                    qtv[k] = qtv[k] - fluxq * rsig[k];
                }
            }
        // dry static energy: damping of super-adiabatic lapse rate
#pragma unroll
        for (int k = 1; k <= nl1; ++k) {
            const double se0 = se[k] + segrad * (phi[k - 1] - phi[k]);
            if (se[k - 1] < se0) {
                const double fluxse = fvdise * (se0 - se[k - 1]);
                ttv[k - 1] = ttv[k - 1] + fluxse * rsig[k - 1];
#pragma unroll
                for (int k1 = k + 1; k1 <= nlev; ++k1) ttv[k1 - 1] = ttv[k1 - 1] - fluxse * rsig1[k - 1];
            }
        }
    }
}

// One column j of phypar's physics.  Inputs (registers): ua, va, ta, qa, phi [kx]
// (k = 0 top) and psl = the column's ug1, vg1, tg1, qg1, phig1, pslg1
// (phy_phypar.f90:53-66); bc = kNBc fields [ngp]; rad = radiation state (in/out,
// column j); fbt = P->fband or a copy of it in LDS.  Outputs: the u, v, t, q
// tendencies of the physics (phypar's additions to the dynamical tendencies).
__device__ inline void phys_column(int j, const double *ua, const double *va, const double *ta, const double *qa_in,
                                   const double *phi, double psl, const double *__restrict__ bc,
                                   double *__restrict__ rad, const PhysTables *P, const double *fbt, bool lradsw,
                                   double *ut_o, double *vt_o, double *tt_o, double *qt_o) {
    using namespace phys;
    constexpr int NL = kKX;
    PhysThermo h;
    phys_thermo(ta, qa_in, phi, psl, P, h);
    double tt[NL], qt[NL], precnv, precls;
    int itop, icnv;
    phys_moist(h, P, tt, qt, precnv, precls, itop, icnv);
    double bcv[kNBc], fbk[NL][4];
    bc_load(j, bc, bcv);
    fband_rows(fbt, ta, fbk);
    RadCol rc;
    if (lradsw)
        phys_sw(j, h, phi, precnv, precls, itop, bcv, rad, P, rc);
    else
        rad_load(j, rad, rc);
    double tt_rlw[NL], ustr3, vstr3, shf3, evap3;
    phys_lw_sfc(j, ua, va, ta, h.qa, phi, h.psg, h.rps, bcv, rc, P, fbt, fbk, tt_rlw, ustr3, vstr3, shf3, evap3);
    const double rps = h.rps;
#pragma unroll
    for (int k = 0; k < NL; ++k) tt[k] = tt[k] + rc.ttrsw[k] + tt_rlw[k];  // :174-179
    double utv[NL], vtv[NL], ttv[NL], qtv[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) utv[k] = vtv[k] = 0.;
    phys_vdif(h, phi, icnv, P, ttv, qtv);
    // 4.2 surface fluxes into the bottom layer (phy_phypar.f90:186-191), then sums (:193-196)
    utv[NL - 1] = utv[NL - 1] + ustr3 * rps * P->grdsig[NL - 1];
    vtv[NL - 1] = vtv[NL - 1] + vstr3 * rps * P->grdsig[NL - 1];
    ttv[NL - 1] = ttv[NL - 1] + shf3 * rps * P->grdscp[NL - 1];
    qtv[NL - 1] = qtv[NL - 1] + evap3 * rps * P->grdsig[NL - 1];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        ut_o[k] = 0. + utv[k];
        vt_o[k] = 0. + vtv[k];
        tt_o[k] = tt[k] + ttv[k];
        qt_o[k] = qt[k] + qtv[k];
    }
}

#endif  // __HIPCC__

}  // namespace sml

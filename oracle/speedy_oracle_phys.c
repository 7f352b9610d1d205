/*
 * oracle/speedy_oracle_phys.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of SPEEDY's column physics as phypar drives it
 * (src/phy_phypar.f90:1-228): shtorh (phy_shtorh.f90), convmf (phy_convmf.f90),
 * lscond (phy_lscond.f90), cloud / radsw / radlw / radset / sol_oz / solar
 * (phy_radiat.f90), suflux / sflset (phy_suflux.f90), vdifsc (phy_vdifsc.f90), the
 * physics constants of inphys (ini_inphys.f90) and the module constants of
 * mod_physcon / mod_cnvcon / mod_lsccon / mod_vdicon / mod_sflcon / mod_radcon.
 *
 * Scope: the tendencies phypar adds to the dynamical ones, with zero input
 * tendencies (so the result is the physics alone), icsea = 0, lrandf = .false.,
 * sppt_on = .false. (their defaults), without dmflux's flux accumulation (daily
 * means for output).  Radiation state that the reference keeps in module
 * variables between calls (tau2, stratc, tt_rsw, ssrd; refreshed when lradsw) is
 * explicit in/out state here.
 *
 * Pinned against the reference's own phypar (compiled as-is into
 * oracle/_ref/libspeedy_ref_dyn.so) by tests/golden/phys_ref.npz
 * (tests/golden/make_phys_golden.py).
 *
 * Layouts follow the reference's physics arrays: grid fields (ngp) with
 * ngp = 96*48 (x fastest, j = 0 southernmost), level fields (ngp, kx) as [k][ngp]
 * with k = 0 the top level.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define NLON 96
#define NLAT 48
#define NGP (NLON * NLAT)
#define NLEV 8

/* mod_physcon.f90 */
static const double p0 = 1.e+5, gg = 9.81, rd = 287., cp = 1004., alhc = 2501.0, sbc = 5.67e-8;
/* mod_cnvcon.f90 */
static const double psmin = 0.8, trcnv = 6.0, rhbl = 0.9, rhil = 0.7, entmax = 0.5, smf = 0.8;
/* mod_lsccon.f90 */
static const double trlsc = 4.0, rhlsc = 0.9, drhlsc = 0.1, rhblsc = 0.95;
/* mod_vdicon.f90 */
static const double trshc = 6.0, trvdi = 24.0, trvds = 6.0, redshc = 0.5, rhgrad = 0.5, segrad = 0.1;
/* mod_sflcon.f90 (fhum0 = 0: the humidity-profile branch of suflux is inactive) */
static const double fwind0 = 0.95, ftemp0 = 1.0, cdl = 2.4e-3, cds = 1.0e-3, chl = 1.2e-3,
                    chs = 0.9e-3, vgust = 5.0, ctday = 1.0e-2, dtheta = 3.0, fstab = 0.67, hdrag = 2000.0,
                    fhdrag = 0.5, clambda = 7.0, clambsn = 7.0;
/* mod_radcon.f90 */
static const double solc = 342.0, rhcl1 = 0.30, rhcl2 = 1.00, qacl = 0.20, wpcl = 0.2, pmaxcl = 10.0,
                    clsmax = 0.60, clsminl = 0.15, gse_s0 = 0.25, gse_s1 = 0.40, albcl = 0.43, albcls = 0.50,
                    epssw = 0.020, epslw = 0.05, emisfc = 0.98, absdry = 0.033, absaer = 0.033, abswv1 = 0.022,
                    abswv2 = 15.000, abscl1 = 0.015, abscl2 = 0.15, ablwin = 0.3, ablco2 = 6.0, ablwv1 = 0.7,
                    ablwv2 = 50.0, ablcl1 = 12.0, ablcl2 = 0.6;

/* inphys (ini_inphys.f90:13-41) */
static double sig[NLEV], sigl[NLEV], sigh[NLEV + 1], dsig[NLEV], grdsig[NLEV], grdscp[NLEV], wvi[NLEV][2];
static double slat[NLAT], clat[NLAT];
static double fband[301][4]; /* fband(100:400, 4) */

/* hsg(0:kx) (mod_dyncon1 hsg), rlat = radang (ini_indyns.f90:49-56) */
void orc_phys_init(const double *hsg, const double *rlat)
{
    sigh[0] = hsg[0];
    for (int k = 1; k <= NLEV; ++k) {
        sig[k - 1] = 0.5 * (hsg[k] + hsg[k - 1]);
        sigl[k - 1] = log(sig[k - 1]);
        sigh[k] = hsg[k];
        dsig[k - 1] = hsg[k] - hsg[k - 1];
        grdsig[k - 1] = gg / (dsig[k - 1] * p0);
        grdscp[k - 1] = grdsig[k - 1] / cp;
    }
    for (int k = 1; k <= NLEV - 1; ++k) {
        wvi[k - 1][0] = 1. / (sigl[k] - sigl[k - 1]);
        wvi[k - 1][1] = (log(sigh[k]) - sigl[k - 1]) * wvi[k - 1][0];
    }
    wvi[NLEV - 1][0] = 0.;
    wvi[NLEV - 1][1] = (log(0.99) - sigl[NLEV - 1]) * wvi[NLEV - 2][0];
    for (int j = 0; j < NLAT; ++j) {
        slat[j] = sin(rlat[j]);
        clat[j] = cos(rlat[j]);
    }
    /* radset (phy_radiat.f90:659-688) */
    double eps1 = 1. - epslw;
    for (int jt = 200; jt <= 320; ++jt) {
        double *f = fband[jt - 100];
        f[1] = (0.148 - 3.0e-6 * (double)((jt - 247) * (jt - 247))) * eps1;
        f[2] = (0.356 - 5.2e-6 * (double)((jt - 282) * (jt - 282))) * eps1;
        f[3] = (0.314 + 1.0e-5 * (double)((jt - 315) * (jt - 315))) * eps1;
        f[0] = eps1 - (f[1] + f[2] + f[3]);
    }
    for (int jb = 0; jb < 4; ++jb) {
        for (int jt = 100; jt <= 199; ++jt) fband[jt - 100][jb] = fband[100][jb];
        for (int jt = 321; jt <= 400; ++jt) fband[jt - 100][jb] = fband[220][jb];
    }
}

void orc_phys_tables(double *out_sig, double *out_wvi, double *out_fband)
{
    memcpy(out_sig, sig, sizeof sig);
    memcpy(out_wvi, wvi, sizeof wvi);
    memcpy(out_fband, fband, sizeof fband);
}

static double fb(double t, int jb) { return fband[(int)lround(t) - 100][jb]; } /* fband(nint(t), jb) */

/* solar + sol_oz (phy_radiat.f90:1-84): fsol, ozone, ozupp, zenit, stratz (ngp each) */
void orc_sol_oz(double tyear, double *fsol, double *ozone, double *ozupp, double *zenit, double *stratz)
{
    double pigr = 2. * asin(1.), alpha = 2. * pigr * tyear;
    double ca1 = cos(alpha), sa1 = sin(alpha);
    double ca2 = ca1 * ca1 - sa1 * sa1, sa2 = 2. * sa1 * ca1;
    double ca3 = ca1 * ca2 - sa1 * sa2, sa3 = sa1 * ca2 + sa2 * ca1;
    double decl = 0.006918 - 0.399912 * ca1 + 0.070257 * sa1 - 0.006758 * ca2 + 0.000907 * sa2 - 0.002697 * ca3 +
                  0.001480 * sa3;
    double fdis = 1.000110 + 0.034221 * ca1 + 0.001280 * sa1 + 0.000719 * ca2 + 0.000077 * sa2;
    double cdecl = cos(decl), sdecl = sin(decl), tdecl = sdecl / cdecl;
    double csolp = (4. * solc) / pigr;
    double topsr[NLAT];
    for (int j = 0; j < NLAT; ++j) {
        double ch0 = fmin(1., fmax(-1., -tdecl * slat[j] / clat[j]));
        double h0 = acos(ch0), sh0 = sin(h0);
        topsr[j] = csolp * fdis * (h0 * slat[j] * sdecl + sh0 * clat[j] * cdecl);
    }
    double alp = 4. * asin(1.) * (tyear + 10. / 365.), dalpha = 0.;
    double coz1 = 1.0 * fmax(0., cos(alp - dalpha)), coz2 = 1.8, azen = 1.0;
    double rzen = -cos(alp) * 23.45 * asin(1.) / 90.;
    double czen = cos(rzen), szen = sin(rzen), fs0 = 6.;
    for (int j = 0; j < NLAT; ++j) {
        double flat2 = 1.5 * slat[j] * slat[j] - 0.5;
        double fs = topsr[j];
        double ozu = 0.5 * epssw, oz = 0.4 * epssw * (1.0 + coz1 * slat[j] + coz2 * flat2);
        double b = 1. - (clat[j] * czen + slat[j] * szen);
        double zen = 1. + azen * (b * b); /* (..)**nzen with nzen = 2 (a real variable) */
        ozu = fs * ozu * zen;
        oz = fs * oz * zen;
        double st = fmax(fs0 - fs, 0.);
        for (int i = 0; i < NLON; ++i) {
            int g = j * NLON + i;
            fsol[g] = fs;
            ozone[g] = oz;
            ozupp[g] = ozu;
            zenit[g] = zen;
            stratz[g] = st;
        }
    }
}

/* sflset (phy_suflux.f90:358-382) */
void orc_sflset(const double *phi0, double *forog)
{
    double rhdrag = 1. / (gg * hdrag);
    for (int j = 0; j < NGP; ++j) forog[j] = 1. + fhdrag * (1. - exp(-fmax(phi0[j], 0.) * rhdrag));
}

/* shtorh for one point (phy_shtorh.f90); sig <= 0 selects ps(1) as the pressure */
static double qsat_of(double ta, double ps, double s)
{
    const double e0 = 6.108e-3, c1 = 17.269, c2 = 21.875, t0 = 273.16, t1 = 35.86, t2 = 7.66;
    double q = (ta >= t0) ? e0 * exp(c1 * (ta - t0) / (ta - t1)) : e0 * exp(c2 * (ta - t0) / (ta - t2));
    return 622. * q / (s * ps - 0.378 * q);
}

/* Boundary fields of one call (all ngp arrays; mod_surfcon / mod_var_land /
 * mod_var_sea / mod_radcon / mod_sflcon). */
typedef struct {
    const double *fmask1, *phis0, *stl_am, *sst_am, *soilw_am, *alb_l, *alb_s, *albsfc, *snowc;
    const double *fsol, *ozone, *ozupp, *zenit, *stratz, *forog;
} orc_phys_bc;

/* Radiation state kept between calls by the reference's modules. */
typedef struct {
    double *tau2;   /* [4][NLEV][NGP]: tau2(ngp, kx, 4) */
    double *stratc; /* [2][NGP] */
    double *tt_rsw; /* [NLEV][NGP] */
    double *ssrd;   /* [NGP] */
} orc_phys_state;

#define LV(a, k, j) ((a)[(size_t)(k) * NGP + (j)])
#define TAU(s, jb, k, j) ((s)->tau2[((size_t)(jb) * NLEV + (k)) * NGP + (j)])

/* One column of phypar's physics.  Inputs: grid-point ug1, vg1, tg1, qg1, phig1
 * [NLEV][NGP] and pslg1 [NGP] (phy_phypar.f90:53-66).  Outputs: tend[4][NLEV][NGP]
 * (u, v, t, q tendencies of the physics).  j = column. */
static void orc_phys_column(int j, const double *ug1, const double *vg1, const double *tg1, const double *qg1_in,
                            const double *phig1, const double *pslg1, const orc_phys_bc *bc, orc_phys_state *st,
                            int lradsw, double *tend)
{
    const int nl1 = NLEV - 1; /* 1-based index of the level above the bottom */
    double ua[NLEV], va[NLEV], ta[NLEV], qa[NLEV], phi[NLEV], se[NLEV], rh[NLEV], qsat[NLEV];
    for (int k = 0; k < NLEV; ++k) {
        ua[k] = LV(ug1, k, j);
        va[k] = LV(vg1, k, j);
        ta[k] = LV(tg1, k, j);
        qa[k] = LV(qg1_in, k, j);
        phi[k] = LV(phig1, k, j);
    }
    /* 1.2 thermodynamic variables (:73-92) */
    double psg = exp(pslg1[j]);
    double rps = 1. / psg;
    for (int k = 0; k < NLEV; ++k) {
        qa[k] = fmax(qa[k], 0.);
        se[k] = cp * ta[k] + phi[k];
    }
    for (int k = 0; k < NLEV; ++k) {
        qsat[k] = qsat_of(ta[k], psg, sig[k]);
        rh[k] = qa[k] / qsat[k];
    }
    /* 2.1 convmf (phy_convmf.f90:22-238) */
    double tt_cnv[NLEV] = {0}, qt_cnv[NLEV] = {0}, cbmf = 0., precnv = 0.;
    int itop;
    {
        const int nlev = NLEV, nlp = NLEV + 1;
        double fqmax = 5., fm0 = p0 * dsig[nlev - 1] / (gg * trcnv * 3600), rdps = 2. / (1. - psmin);
        double mss[NLEV + 1], entr[NLEV + 1], sentr = 0.;
        for (int k = 2; k <= nlev; ++k) mss[k] = se[k - 1] + alhc * qsat[k - 1];
        for (int k = 2; k <= nl1; ++k) {
            double e = fmax(0., sig[k - 1] - 0.5);
            entr[k] = e * e;
            sentr = sentr + entr[k];
        }
        sentr = entmax / sentr;
        for (int k = 2; k <= nl1; ++k) entr[k] = entr[k] * sentr;
        double rlhc = 1. / alhc, qdif = 0., msthr = 0.;
        itop = nlp;
        if (psg > psmin) {
            double mse0 = se[nlev - 1] + alhc * qa[nlev - 1];
            double mse1 = se[nl1 - 1] + alhc * qa[nl1 - 1];
            mse1 = fmin(mse0, mse1);
            double mss0 = fmax(mse0, mss[nlev]);
            int ktop1 = nlev, ktop2 = nlev;
            for (int k = nlev - 3; k >= 3; --k) {
                double mss2 = mss[k] + wvi[k - 1][1] * (mss[k + 1] - mss[k]);
                if (mss0 > mss2) ktop1 = k;
                if (mse1 > mss2) {
                    ktop2 = k;
                    msthr = mss2;
                }
            }
            if (ktop1 < nlev) {
                double qthr0 = rhbl * qsat[nlev - 1], qthr1 = rhbl * qsat[nl1 - 1];
                int lqthr = (qa[nlev - 1] > qthr0 && qa[nl1 - 1] > qthr1);
                if (ktop2 < nlev) {
                    itop = ktop1;
                    qdif = fmax(qa[nlev - 1] - qthr0, (mse0 - msthr) * rlhc);
                } else if (lqthr) {
                    itop = ktop1;
                    qdif = qa[nlev - 1] - qthr0;
                }
            }
        }
        if (itop != nlp) {
            double dfse[NLEV + 1] = {0}, dfqa[NLEV + 1] = {0};
            int k = nlev, k1 = k - 1;
            double qmax = fmax(1.01 * qa[k - 1], qsat[k - 1]);
            double sb = se[k1 - 1] + wvi[k1 - 1][1] * (se[k - 1] - se[k1 - 1]);
            double qb = qa[k1 - 1] + wvi[k1 - 1][1] * (qa[k - 1] - qa[k1 - 1]);
            qb = fmin(qb, qa[k - 1]);
            double fpsa = psg * fmin(1., (psg - psmin) * rdps);
            double fmass = fm0 * fpsa * fmin(fqmax, qdif / (qmax - qb));
            cbmf = fmass;
            double fus = fmass * se[k - 1], fuq = fmass * qmax, fds = fmass * sb, fdq = fmass * qb;
            dfse[k] = fds - fus;
            dfqa[k] = fdq - fuq;
            for (k = nlev - 1; k >= itop + 1; --k) {
                k1 = k - 1;
                dfse[k] = fus - fds;
                dfqa[k] = fuq - fdq;
                double enmass = entr[k] * psg * cbmf;
                fmass = fmass + enmass;
                fus = fus + enmass * se[k - 1];
                fuq = fuq + enmass * qa[k - 1];
                sb = se[k1 - 1] + wvi[k1 - 1][1] * (se[k - 1] - se[k1 - 1]);
                qb = qa[k1 - 1] + wvi[k1 - 1][1] * (qa[k - 1] - qa[k1 - 1]);
                fds = fmass * sb;
                fdq = fmass * qb;
                dfse[k] = dfse[k] + fds - fus;
                dfqa[k] = dfqa[k] + fdq - fuq;
                double delq = rhil * qsat[k - 1] - qa[k - 1];
                if (delq > 0.0) {
                    double fsq = smf * cbmf * delq;
                    dfqa[k] = dfqa[k] + fsq;
                    dfqa[nlev] = dfqa[nlev] - fsq;
                }
            }
            k = itop;
            double qsatb = qsat[k - 1] + wvi[k - 1][1] * (qsat[k] - qsat[k - 1]);
            precnv = fmax(fuq - fmass * qsatb, 0.0);
            dfse[k] = fus - fds + alhc * precnv;
            dfqa[k] = fuq - fdq - precnv;
            for (int kk = 1; kk <= nlev; ++kk) {
                tt_cnv[kk - 1] = dfse[kk];
                qt_cnv[kk - 1] = dfqa[kk];
            }
        }
    }
    for (int k = 1; k < NLEV; ++k) { /* phypar :95-100, k = 2..nlev */
        tt_cnv[k] = tt_cnv[k] * rps * grdscp[k];
        qt_cnv[k] = qt_cnv[k] * rps * grdsig[k];
    }
    int icnv = NLEV - itop;
    /* 2.2 lscond (phy_lscond.f90:20-109) */
    double tt_lsc[NLEV] = {0}, qt_lsc[NLEV] = {0}, precls = 0.;
    {
        double qsmax = 10., rtlsc = 1. / (trlsc * 3600.), tfact = alhc / cp, prg = p0 / gg;
        double psa2 = psg * psg;
        for (int k = 2; k <= NLEV; ++k) {
            double sig2 = sig[k - 1] * sig[k - 1];
            double rhref = rhlsc + drhlsc * (sig2 - 1.);
            if (k == NLEV) rhref = fmax(rhref, rhblsc);
            double dqmax = qsmax * sig2 * rtlsc;
            double dqa = rhref * qsat[k - 1] - qa[k - 1];
            if (dqa < 0.0) {
                itop = (k < itop) ? k : itop;
                qt_lsc[k - 1] = dqa * rtlsc;
                tt_lsc[k - 1] = tfact * fmin(-qt_lsc[k - 1], dqmax * psa2);
            } else {
                qt_lsc[k - 1] = 0.;
                tt_lsc[k - 1] = 0.;
            }
        }
        for (int k = 2; k <= NLEV; ++k) {
            double pfact = dsig[k - 1] * prg;
            precls = precls - pfact * qt_lsc[k - 1];
        }
        precls = precls * psg;
    }
    double ut[NLEV], vt[NLEV], tt[NLEV], qt[NLEV];
    for (int k = 0; k < NLEV; ++k) {
        ut[k] = 0.;
        vt[k] = 0.;
        tt[k] = 0. + tt_cnv[k] + tt_lsc[k];
        qt[k] = 0. + qt_cnv[k] + qt_lsc[k];
    }
    const int jlat = j / NLON;
    /* 3.1 shortwave (phypar :125-147): cloud + radsw */
    if (lradsw) {
        double gse = (se[NLEV - 2] - se[NLEV - 1]) / (phi[NLEV - 2] - phi[NLEV - 1]);
        /* cloud (phy_radiat.f90:86-152) */
        const int nlp = NLEV + 1;
        double rrcl = 1. / (rhcl2 - rhcl1), cloudc, clstr;
        int icltop;
        if (rh[nl1 - 1] > rhcl1) {
            cloudc = rh[nl1 - 1] - rhcl1;
            icltop = nl1;
        } else {
            cloudc = 0.;
            icltop = nlp;
        }
        for (int k = 3; k <= NLEV - 2; ++k) {
            double drh = rh[k - 1] - rhcl1;
            if (drh > cloudc && qa[k - 1] > qacl) {
                cloudc = drh;
                icltop = k;
            }
        }
        double cl1 = fmin(1., cloudc * rrcl);
        double pr1 = fmin(pmaxcl, 86.4 * (precnv + precls));
        cloudc = fmin(1., wpcl * sqrt(pr1) + cl1 * cl1);
        icltop = (itop < icltop) ? itop : icltop;
        double qcloud = qa[nl1 - 1];
        {
            double clfact = 1.2, rgse = 1. / (gse_s1 - gse_s0);
            double fst = fmax(0., fmin(1., rgse * (gse - gse_s0)));
            clstr = fst * fmax(clsmax - clfact * cloudc, 0.);
            double clstrl = fmax(clstr, clsminl) * rh[NLEV - 1];
            clstr = clstr + bc->fmask1[j] * (clstrl - clstr);
        }
        /* radsw (phy_radiat.f90:154-328) */
        double fband2 = 0.05, fband1 = 1. - fband2;
        double t1[NLEV], t2[NLEV], t3[NLEV], dfabs[NLEV];
        for (int k = 0; k < NLEV; ++k) t1[k] = t2[k] = t3[k] = 0.0;
        if (icltop <= NLEV) t3[icltop - 1] = albcl * cloudc;
        t3[NLEV - 1] = albcls * clstr;
        double psaz = psg * bc->zenit[j];
        double acloud = cloudc * fmin(abscl1 * qcloud, abscl2);
        t1[0] = exp(-(psaz * dsig[0]) * absdry);
        for (int k = 2; k <= nl1; ++k) {
            double abs1 = absdry + absaer * sig[k - 1] * sig[k - 1];
            double deltap = psaz * dsig[k - 1];
            if (k >= icltop)
                t1[k - 1] = exp(-deltap * (abs1 + abswv1 * qa[k - 1] + acloud));
            else
                t1[k - 1] = exp(-deltap * (abs1 + abswv1 * qa[k - 1]));
        }
        {
            double abs1 = absdry + absaer * sig[NLEV - 1] * sig[NLEV - 1];
            double deltap = psaz * dsig[NLEV - 1];
            t1[NLEV - 1] = exp(-deltap * (abs1 + abswv1 * qa[NLEV - 1]));
        }
        for (int k = 2; k <= NLEV; ++k) t2[k - 1] = exp(-(psaz * dsig[k - 1]) * abswv2 * qa[k - 1]);
        double ftop = bc->fsol[j];
        double f1 = bc->fsol[j] * fband1, f2 = bc->fsol[j] * fband2;
        dfabs[0] = f1;
        f1 = t1[0] * (f1 - bc->ozupp[j] * psg);
        dfabs[0] = dfabs[0] - f1;
        dfabs[1] = f1;
        f1 = t1[1] * (f1 - bc->ozone[j] * psg);
        dfabs[1] = dfabs[1] - f1;
        for (int k = 3; k <= NLEV; ++k) {
            t3[k - 1] = f1 * t3[k - 1];
            f1 = f1 - t3[k - 1];
            dfabs[k - 1] = f1;
            f1 = t1[k - 1] * f1;
            dfabs[k - 1] = dfabs[k - 1] - f1;
        }
        for (int k = 2; k <= NLEV; ++k) {
            dfabs[k - 1] = dfabs[k - 1] + f2;
            f2 = t2[k - 1] * f2;
            dfabs[k - 1] = dfabs[k - 1] - f2;
        }
        double fsfcd = f1 + f2;
        f1 = f1 * bc->albsfc[j];
        (void)ftop;
        for (int k = NLEV; k >= 1; --k) {
            dfabs[k - 1] = dfabs[k - 1] + f1;
            f1 = t1[k - 1] * f1;
            dfabs[k - 1] = dfabs[k - 1] - f1;
            f1 = f1 + t3[k - 1];
        }
        st->ssrd[j] = fsfcd;
        /* longwave transmissivities (:262-300) */
        double deltap = psg * dsig[0];
        TAU(st, 0, 0, j) = exp(-deltap * ablwin);
        TAU(st, 1, 0, j) = exp(-deltap * ablco2);
        TAU(st, 2, 0, j) = 1.;
        TAU(st, 3, 0, j) = 1.;
        for (int k = 2; k <= NLEV; k += NLEV - 2) {
            deltap = psg * dsig[k - 1];
            TAU(st, 0, k - 1, j) = exp(-deltap * ablwin);
            TAU(st, 1, k - 1, j) = exp(-deltap * ablco2);
            TAU(st, 2, k - 1, j) = exp(-deltap * ablwv1 * qa[k - 1]);
            TAU(st, 3, k - 1, j) = exp(-deltap * ablwv2 * qa[k - 1]);
        }
        double acl = cloudc * ablcl2;
        for (int k = 3; k <= nl1; ++k) {
            deltap = psg * dsig[k - 1];
            double acloud1 = (k < icltop) ? acl : ablcl1 * cloudc;
            TAU(st, 0, k - 1, j) = exp(-deltap * (ablwin + acloud1));
            TAU(st, 1, k - 1, j) = exp(-deltap * ablco2);
            TAU(st, 2, k - 1, j) = exp(-deltap * fmax(ablwv1 * qa[k - 1], acl));
            TAU(st, 3, k - 1, j) = exp(-deltap * fmax(ablwv2 * qa[k - 1], acl));
        }
        double eps1 = epslw / (dsig[0] + dsig[1]);
        st->stratc[j] = bc->stratz[j] * psg;
        st->stratc[NGP + j] = eps1 * psg;
        for (int k = 0; k < NLEV; ++k) LV(st->tt_rsw, k, j) = dfabs[k] * rps * grdscp[k];
    }
    /* 3.2 radlw(-1) (phy_radiat.f90:330-413) */
    double st4a1[NLEV], st4a2[NLEV], flux[4], dfabs[NLEV], fsfcd;
    {
        for (int k = 1; k <= nl1; ++k) st4a1[k - 1] = ta[k - 1] + wvi[k - 1][1] * (ta[k] - ta[k - 1]);
        st4a2[0] = 0.75 * ta[0] + 0.25 * st4a1[0];
        st4a2[1] = 0.50 * ta[1] + 0.25 * (st4a1[0] + st4a1[1]);
        double anis = 1.0, anish = 0.5 * anis;
        for (int k = 3; k <= nl1; ++k) st4a2[k - 1] = anish * fmax(st4a1[k - 1] - st4a1[k - 2], 0.);
        st4a2[NLEV - 1] = anis * fmax(ta[NLEV - 1] - st4a1[nl1 - 1], 0.);
        for (int k = 0; k < 2; ++k) {
            double x = st4a2[k];
            st4a1[k] = sbc * ((x * x) * (x * x));
            st4a2[k] = 0.;
        }
        for (int k = 3; k <= NLEV; ++k) {
            double t = ta[k - 1];
            double st3a = sbc * (t * t * t);
            st4a1[k - 1] = st3a * t;
            st4a2[k - 1] = 4. * st3a * st4a2[k - 1];
        }
        fsfcd = 0.0;
        for (int k = 0; k < NLEV; ++k) dfabs[k] = 0.0;
        for (int jb = 0; jb < 2; ++jb) {
            double emis = 1. - TAU(st, jb, 0, j);
            double brad = fb(ta[0], jb) * (st4a1[0] + emis * st4a2[0]);
            flux[jb] = emis * brad;
            dfabs[0] = dfabs[0] - flux[jb];
        }
        flux[2] = flux[3] = 0.0;
        for (int jb = 0; jb < 4; ++jb)
            for (int k = 2; k <= NLEV; ++k) {
                double emis = 1. - TAU(st, jb, k - 1, j);
                double brad = fb(ta[k - 1], jb) * (st4a1[k - 1] + emis * st4a2[k - 1]);
                dfabs[k - 1] = dfabs[k - 1] + flux[jb];
                flux[jb] = TAU(st, jb, k - 1, j) * flux[jb] + emis * brad;
                dfabs[k - 1] = dfabs[k - 1] - flux[jb];
            }
        for (int jb = 0; jb < 4; ++jb) fsfcd = fsfcd + emisfc * flux[jb];
        double eps1 = epslw * emisfc;
        double corlw = eps1 * st4a1[NLEV - 1];
        dfabs[NLEV - 1] = dfabs[NLEV - 1] - corlw;
        fsfcd = fsfcd + corlw;
    }
    double slrd = fsfcd;
    /* 3.3 suflux (phy_suflux.f90:1-355), lfluxland = .true. */
    double ustr3, vstr3, shf3, evap3, slru3, tsfc;
    {
        const int nlev = NLEV;
        double esbc = emisfc * sbc, esbc4 = 4. * esbc, dlambda = clambsn - clambda;
        double u0 = fwind0 * ua[nlev - 1], v0 = fwind0 * va[nlev - 1];
        double gtemp0 = 1. - ftemp0, rcp = 1. / cp, rdphi0 = -1. / (rd * 288. * sigl[nlev - 1]);
        double phi0 = bc->phis0[j], fmask = bc->fmask1[j];
        double t1[2], t2[2], q1[2], denvvs[3], qsat0[2];
        double dt1 = wvi[nlev - 1][1] * (ta[nlev - 1] - ta[nl1 - 1]);
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
        double t0 = t1[1] + fmask * (t1[0] - t1[1]);
        double prd = p0 / rd, vg2 = vgust * vgust;
        denvvs[0] = (prd * psg / t0) * sqrt(u0 * u0 + v0 * v0 + vg2);
        double sqclat = sqrt(clat[jlat]);
        double tskin = bc->stl_am[j] + ctday * sqclat * st->ssrd[j] * (1. - bc->alb_l[j]) * psg;
        double rdth = fstab / dtheta, astab = 0.5;
        double dthl = (tskin > t2[0]) ? fmin(dtheta, tskin - t2[0]) : fmax(-dtheta, astab * (tskin - t2[0]));
        denvvs[1] = denvvs[0] * (1. + dthl * rdth);
        double cdldv = cdl * denvvs[0] * bc->forog[j];
        double ustr1 = -cdldv * ua[nlev - 1], vstr1 = -cdldv * va[nlev - 1];
        double chlcp = chl * cp;
        double shf1 = chlcp * denvvs[1] * (tskin - t1[0]);
        q1[0] = qa[nlev - 1]; /* fhum0 = 0 */
        qsat0[0] = qsat_of(tskin, psg, 1.);
        double swav = bc->soilw_am[j];
        double evap1 = chl * denvvs[1] * fmax(0., swav * qsat0[0] - q1[0]);
        double tsk3 = tskin * tskin * tskin;
        double dslr = esbc4 * tsk3;
        double slru1 = esbc * tsk3 * tskin;
        double hfl1 = st->ssrd[j] * (1. - bc->alb_l[j]) + slrd - (slru1 + shf1 + alhc * evap1);
        /* lskineb */
        double clamb = clambda + bc->snowc[j] * dlambda;
        hfl1 = hfl1 - clamb * (tskin - bc->stl_am[j]);
        double dtskin = tskin + 1.;
        qsat0[1] = qsat_of(dtskin, psg, 1.);
        if (evap1 > 0)
            qsat0[1] = swav * (qsat0[1] - qsat0[0]);
        else
            qsat0[1] = 0.;
        double dhfdt = clamb + dslr + chl * denvvs[1] * (cp + alhc * qsat0[1]);
        dtskin = hfl1 / dhfdt;
        tskin = tskin + dtskin;
        shf1 = shf1 + chlcp * denvvs[1] * dtskin;
        evap1 = evap1 + chl * denvvs[1] * qsat0[1] * dtskin;
        slru1 = slru1 + dslr * dtskin;
        /* sea */
        double tsea = bc->sst_am[j];
        double dths = (tsea > t2[1]) ? fmin(dtheta, tsea - t2[1]) : fmax(-dtheta, astab * (tsea - t2[1]));
        denvvs[2] = denvvs[0] * (1. + dths * rdth);
        q1[1] = qa[nlev - 1];
        double cdsdv = cds * denvvs[2];
        double ustr2 = -cdsdv * ua[nlev - 1], vstr2 = -cdsdv * va[nlev - 1];
        double chscp = chs * cp;
        double shf2 = chscp * denvvs[2] * (tsea - t1[1]);
        double qs = qsat_of(tsea, psg, 1.);
        double evap2 = chs * denvvs[2] * (qs - q1[1]);
        double ts2 = tsea * tsea;
        double slru2 = esbc * (ts2 * ts2);
        ustr3 = ustr2 + fmask * (ustr1 - ustr2);
        vstr3 = vstr2 + fmask * (vstr1 - vstr2);
        shf3 = shf2 + fmask * (shf1 - shf2);
        evap3 = evap2 + fmask * (evap1 - evap2);
        slru3 = slru2 + fmask * (slru1 - slru2);
        tsfc = tsea + fmask * (bc->stl_am[j] - tsea);
    }
    /* 3.4 radlw(1) (phy_radiat.f90:414-458) */
    {
        double refsfc = 1. - emisfc, fsfcu = slru3, ts = tsfc;
        for (int jb = 0; jb < 4; ++jb) flux[jb] = fb(ts, jb) * fsfcu + refsfc * flux[jb];
        dfabs[NLEV - 1] = dfabs[NLEV - 1] + epslw * fsfcu;
        for (int jb = 0; jb < 4; ++jb)
            for (int k = NLEV; k >= 2; --k) {
                double emis = 1. - TAU(st, jb, k - 1, j);
                double brad = fb(ta[k - 1], jb) * (st4a1[k - 1] - emis * st4a2[k - 1]);
                dfabs[k - 1] = dfabs[k - 1] + flux[jb];
                flux[jb] = TAU(st, jb, k - 1, j) * flux[jb] + emis * brad;
                dfabs[k - 1] = dfabs[k - 1] - flux[jb];
            }
        for (int jb = 0; jb < 2; ++jb) {
            double emis = 1. - TAU(st, jb, 0, j);
            double brad = fb(ta[0], jb) * (st4a1[0] - emis * st4a2[0]);
            dfabs[0] = dfabs[0] + flux[jb];
            flux[jb] = TAU(st, jb, 0, j) * flux[jb] + emis * brad;
            dfabs[0] = dfabs[0] - flux[jb];
        }
        double corlw1 = dsig[0] * st->stratc[NGP + j] * st4a1[0] + st->stratc[j];
        double corlw2 = dsig[1] * st->stratc[NGP + j] * st4a1[1];
        dfabs[0] = dfabs[0] - corlw1;
        dfabs[1] = dfabs[1] - corlw2;
    }
    for (int k = 0; k < NLEV; ++k) {
        double tt_rlw = dfabs[k] * rps * grdscp[k];
        tt[k] = tt[k] + LV(st->tt_rsw, k, j) + tt_rlw;
    }
    /* 4.1 vdifsc (phy_vdifsc.f90:17-124) */
    double utv[NLEV] = {0}, vtv[NLEV] = {0}, ttv[NLEV] = {0}, qtv[NLEV] = {0};
    {
        const int nlev = NLEV;
        double cshc = dsig[nlev - 1] / 3600., cvdi = (sigh[nl1] - sigh[1]) / ((nl1 - 1) * 3600.);
        double fshcq = cshc / trshc, fshcse = cshc / (trshc * cp);
        double fvdiq = cvdi / trvdi, fvdise = cvdi / (trvds * cp);
        double rsig[NLEV], rsig1[NLEV];
        for (int k = 1; k <= nl1; ++k) {
            rsig[k - 1] = 1. / dsig[k - 1];
            rsig1[k - 1] = 1. / (1. - sigh[k]);
        }
        rsig[nlev - 1] = 1. / dsig[nlev - 1];
        double drh0 = rhgrad * (sig[nlev - 1] - sig[nl1 - 1]);
        double fvdiq2 = fvdiq * sigh[nl1];
        double dmse = (se[nlev - 1] - se[nl1 - 1]) + alhc * (qa[nlev - 1] - qsat[nl1 - 1]);
        double drh = rh[nlev - 1] - rh[nl1 - 1];
        double fcnv = 1.;
        if (dmse >= 0.0) {
            if (icnv > 0) fcnv = redshc;
            double fluxse = fcnv * fshcse * dmse;
            ttv[nl1 - 1] = fluxse * rsig[nl1 - 1];
            ttv[nlev - 1] = -fluxse * rsig[nlev - 1];
            if (drh >= 0.0) {
                double fluxq = fcnv * fshcq * qsat[nlev - 1] * drh;
                qtv[nl1 - 1] = fluxq * rsig[nl1 - 1];
                qtv[nlev - 1] = -fluxq * rsig[nlev - 1];
            }
        } else if (drh >= drh0) {
            double fluxq = fvdiq2 * qsat[nl1 - 1] * drh;
            qtv[nl1 - 1] = fluxq * rsig[nl1 - 1];
            qtv[nlev - 1] = -fluxq * rsig[nlev - 1];
        }
        for (int k = 3; k <= nlev - 2; ++k)
            if (sigh[k] > 0.5) {
                drh0 = rhgrad * (sig[k] - sig[k - 1]);
                fvdiq2 = fvdiq * sigh[k];
                drh = rh[k] - rh[k - 1];
                if (drh >= drh0) {
                    double fluxq = fvdiq2 * qsat[k - 1] * drh;
                    qtv[k - 1] = qtv[k - 1] + fluxq * rsig[k - 1];
                    qtv[k] = qtv[k] - fluxq * rsig[k];
                }
            }
        for (int k = 1; k <= nl1; ++k) {
            double se0 = se[k] + segrad * (phi[k - 1] - phi[k]);
            if (se[k - 1] < se0) {
                double fluxse = fvdise * (se0 - se[k - 1]);
                ttv[k - 1] = ttv[k - 1] + fluxse * rsig[k - 1];
                for (int k1 = k + 1; k1 <= nlev; ++k1) ttv[k1 - 1] = ttv[k1 - 1] - fluxse * rsig1[k - 1];
            }
        }
    }
    /* 4.2 surface fluxes into the bottom layer (phypar :192-200) */
    utv[NLEV - 1] = utv[NLEV - 1] + ustr3 * rps * grdsig[NLEV - 1];
    vtv[NLEV - 1] = vtv[NLEV - 1] + vstr3 * rps * grdsig[NLEV - 1];
    ttv[NLEV - 1] = ttv[NLEV - 1] + shf3 * rps * grdscp[NLEV - 1];
    qtv[NLEV - 1] = qtv[NLEV - 1] + evap3 * rps * grdsig[NLEV - 1];
    for (int k = 0; k < NLEV; ++k) {
        LV(tend, k, j) = ut[k] + utv[k];
        LV(tend + (size_t)NLEV * NGP, k, j) = vt[k] + vtv[k];
        LV(tend + (size_t)2 * NLEV * NGP, k, j) = tt[k] + ttv[k];
        LV(tend + (size_t)3 * NLEV * NGP, k, j) = qt[k] + qtv[k];
    }
}

/* phypar's physics for the whole grid from grid-point inputs (see above).
 * bc_fields: 15 ngp arrays in the orc_phys_bc order; state: tau2 [4][kx][ngp],
 * stratc [2][ngp], tt_rsw [kx][ngp], ssrd [ngp] (in/out); tend [4][kx][ngp]. */
void orc_phypar_grid(const double *ug1, const double *vg1, const double *tg1, const double *qg1, const double *phig1,
                     const double *pslg1, const double *bc_fields, double *tau2, double *stratc, double *tt_rsw,
                     double *ssrd, int lradsw, double *tend)
{
    orc_phys_bc bc;
    const double **f = (const double **)&bc;
    for (int i = 0; i < 15; ++i) f[i] = bc_fields + (size_t)i * NGP;
    orc_phys_state st = {tau2, stratc, tt_rsw, ssrd};
    for (int j = 0; j < NGP; ++j) orc_phys_column(j, ug1, vg1, tg1, qg1, phig1, pslg1, &bc, &st, lradsw, tend);
}

/* ------------------------------------------------------------ per-window forcing
 * What agcm_init rebuilds before every window from run_model's date
 * (ini_agcm_init.f90:57-89; run_model passes the calendar date, mpires.f90:1545,
 * 1595-1598), with the coupler flags of mod_cpl_flags.f90 (icland 1, icsea 0,
 * icice 1, isstan 0) at jday 0.  Pinned by tests/golden/fordate_ref.npz
 * (tests/golden/make_fordate_golden.py: newdate, forin5, forint, ini_land and fordate
 * of the reference compiled as-is).  atm2sea / sea2atm live in cpl_sea.f90, which
 * also holds ini_sea's `use mpires` and does not build here: their sea-ice adjustment
 * (cpl_sea.f90:96-117, 190-197) is restated below, parity unpinned for those lines. */

/* newdate(0) with iseasc = 1 (mod_date.f90:17-79): tmonth, tyear of (imonth, iday) */
void orc_newdate(int imonth, int iday, double *tmonth, double *tyear)
{
    static const int ncal365[12] = {31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    int before = 0;
    for (int m = 1; m < imonth; ++m) before += ncal365[m - 1];
    *tmonth = (iday - 0.5) / (double)ncal365[imonth - 1];
    *tyear = (before + iday - 0.5) / (double)365;
}

/* forint (cpl_bcinterp.f90:1-23): for12 [12][NGP] (month 1 first) */
void orc_forint(int imon, double fmon, const double *for12, double *for1)
{
    int imon2;
    double wmon;
    if (fmon <= 0.5) {
        imon2 = imon - 1;
        if (imon == 1) imon2 = 12;
        wmon = 0.5 - fmon;
    } else {
        imon2 = imon + 1;
        if (imon == 12) imon2 = 1;
        wmon = fmon - 0.5;
    }
    const double *a = for12 + (size_t)(imon - 1) * NGP, *b = for12 + (size_t)(imon2 - 1) * NGP;
    for (int j = 0; j < NGP; ++j) for1[j] = a[j] + wmon * (b[j] - a[j]);
}

/* forin5 (cpl_bcinterp.f90:25-56): non-linear, mean-conserving */
void orc_forin5(int imon, double fmon, const double *for12, double *for1)
{
    int im2 = imon - 2, im1 = imon - 1, ip1 = imon + 1, ip2 = imon + 2;
    if (im2 < 1) im2 = im2 + 12;
    if (im1 < 1) im1 = im1 + 12;
    if (ip1 > 12) ip1 = ip1 - 12;
    if (ip2 > 12) ip2 = ip2 - 12;
    double c0 = 1. / 12., t0 = c0 * fmon, t1 = c0 * (1. - fmon), t2 = 0.25 * fmon * (1 - fmon);
    double wm2 = -t1 + t2, wm1 = -c0 + 8 * t1 - 6 * t2, w0 = 7 * c0 + 10 * t2, wp1 = -c0 + 8 * t0 - 6 * t2,
           wp2 = -t0 + t2;
    const double *f[5];
    const int mm[5] = {im2, im1, imon, ip1, ip2};
    for (int k = 0; k < 5; ++k) f[k] = for12 + (size_t)(mm[k] - 1) * NGP;
    for (int j = 0; j < NGP; ++j)
        for1[j] = wm2 * f[0][j] + wm1 * f[1][j] + w0 * f[2][j] + wp1 * f[3][j] + wp2 * f[4][j];
}

/* ini_coupler(2) at (imonth, iday): clim [5][12][NGP] = stl12, snowd12, soilw12, sst12,
 * sice12.  Land: atm2land(0), stl_lm = stlcl_ob, land2atm(0) (cpl_land.f90:1-95).
 * Sea: atm2sea(0) with the adjustment over sea ice, ini_sea's start from the
 * climatology, sea2atm(0) (cpl_sea.f90:1-37, 50-117, 138-199): sst_am ice-blended. */
void orc_coupler(int imonth, int iday, const double *clim, double *stl_am, double *snowd_am, double *soilw_am,
                 double *sst_am, double *sice_am, double *tice_am)
{
    double tmonth, tyear;
    orc_newdate(imonth, iday, &tmonth, &tyear);
    const size_t F = (size_t)12 * NGP;
    orc_forin5(imonth, tmonth, clim, stl_am);
    orc_forint(imonth, tmonth, clim + F, snowd_am);
    orc_forint(imonth, tmonth, clim + 2 * F, soilw_am);
    double *sstcl = malloc(NGP * sizeof(double)), *sicecl = malloc(NGP * sizeof(double));
    orc_forin5(imonth, tmonth, clim + 3 * F, sstcl);
    orc_forint(imonth, tmonth, clim + 4 * F, sicecl);
    const double sstfr = 273.2 - 1.8;
    for (int j = 0; j < NGP; ++j) {
        double ticecl;
        if (sstcl[j] > sstfr) {
            sicecl[j] = fmin(0.5, sicecl[j]);
            ticecl = sstfr;
            if (sicecl[j] > 0.) sstcl[j] = sstfr + (sstcl[j] - sstfr) / (1. - sicecl[j]);
        } else {
            sicecl[j] = fmax(0.5, sicecl[j]);
            ticecl = sstfr + (sstcl[j] - sstfr) / sicecl[j];
            sstcl[j] = sstfr;
        }
        /* sst_om = sstcl_ob, tice_om = ticecl_ob, sice_om = sicecl_ob (ini_sea);
         * sea2atm(0): sst_am = sstcl_ob + 0, sice_am = sice_om, tice_am = tice_om */
        double s = sstcl[j] + 0.0;
        sice_am[j] = sicecl[j];
        tice_am[j] = ticecl;
        sst_am[j] = s + sicecl[j] * (ticecl - s);
    }
    free(sstcl);
    free(sicecl);
}

void orc_spec(const double *vorg, double *vorm);

/* fordate(0) (ini_fordate.f90:1-115; lco2 .false.): sol_oz(tyear) into sol5
 * [5][NGP]; the surface albedo; tcorh, qcorh (spectral (mx2, nx)).  snowd_am NULL:
 * snowc is an input (the coupler's snow cover as the host gave it). */
void orc_fordate(double tyear, const double *fmask_l, const double *fmask_s, const double *alb0,
                 const double *phis0, const double *stl_am, const double *sst_am, const double *snowd_am,
                 const double *sice_am, double *snowc, double *alb_l, double *alb_s, double *albsfc, double *sol5,
                 double *tcorh, double *qcorh)
{
    orc_sol_oz(tyear, sol5, sol5 + NGP, sol5 + 2 * NGP, sol5 + 3 * NGP, sol5 + 4 * NGP);
    const double albsn = 0.60, albsea = 0.07, albice = 0.60, sd2sc = 60.0;
    for (int j = 0; j < NGP; ++j) {
        if (snowd_am) snowc[j] = fmin(1., snowd_am[j] / sd2sc);
        alb_l[j] = alb0[j] + snowc[j] * (albsn - alb0[j]);
        alb_s[j] = albsea + sice_am[j] * (albice - albsea);
        albsfc[j] = alb_s[j] + fmask_l[j] * (alb_l[j] - alb_s[j]);
    }
    /* setgam: gamlat(j) = gamma / (1000 g) on every latitude (mod_dyncon0 gamma = 6) */
    const double gamlat = 6.0 / (1000. * gg), refrh1 = 0.7;
    double *corh = malloc(NGP * sizeof(double)), *corq = malloc(NGP * sizeof(double));
    for (int j = 0; j < NGP; ++j) corh[j] = gamlat * phis0[j];
    orc_spec(corh, tcorh);
    const double pexp = 1. / (rd * gamlat);
    for (int j = 0; j < NGP; ++j) {
        double tsfc = fmask_l[j] * stl_am[j] + fmask_s[j] * sst_am[j];
        double tref = tsfc + corh[j];
        double psfc = pow(tsfc / tref, pexp);
        double qref = qsat_of(tref, 1.0, 1.0); /* shtorh(0, .., tref, psfc_dummy = 1, -1.) */
        double qsfc = qsat_of(tsfc, psfc, 1.0); /* shtorh(0, .., tsfc, psfc, 1.) */
        corq[j] = refrh1 * (qref - qsfc);
    }
    orc_spec(corq, qcorh);
    free(corh);
    free(corq);
}

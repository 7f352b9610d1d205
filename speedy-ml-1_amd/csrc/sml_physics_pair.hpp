// sml_physics_pair.hpp -- phypar's longwave / surface side (and, on a shortwave step, its
// shortwave) on two lanes per column: the row kernel whose three roles each have waves
// of their own (k_st_gridspec_p, sml_dynamics.hip).
//
// Reference: phypar (src/phy_phypar.f90:121-179) -- radsw (phy_radiat.f90:154-328), radlw
// (:330-458), suflux (phy_suflux.f90:1-355) -- with the expressions of sml_physics.hpp.
//
// Layout.  Lanes 2i and 2i + 1 own column i; lane h owns the levels 4h .. 4h + 3 (the
// shortwave transmissivities t1 / t2, the heating rates' scaling, the flux divergences)
// and the longwave bands 2h, 2h + 1 (their eight transmissivities, fband rows and flux
// recurrences down and up).  The column-wide chains (on a shortwave step the moist part,
// cloud and radsw's flux chains; suflux) run on both lanes alike.  The partners trade
// values by DPP (one row permutation per double, no LDS), so every level's divergence
// adds the four bands' fluxes in radlw's order: bitwise the one-lane form.
#pragma once
#include "sml_physics.hpp"

namespace sml {
#ifdef __HIPCC__

// a longwave-only step's radiation state for lane h: bands 2h, 2h + 1 and its four levels of tt_rsw
struct PairPre {
    double tau[2][kKX];
    double strat0, strat1, ssrd, ttrsw[4];
};

// lane h's share of phys_column's results: its four levels, the surface fluxes
struct PairOut {
    double rsw[4], rlw[4];
    double ust, vst, shf, evp, rps;
};

// radlw(1)'s surface emission row fband(nint(tsfc), jb) of column pt (suflux's tsfc =
// sst + fmask (stl - sst), phy_suflux.f90, from the boundary fields alone): the row
// kernel stages it during gridx, off the physics' chain of dependent loads
__device__ __forceinline__ double sfc_fband(const double *__restrict__ bc, const double *__restrict__ fbt, int pt,
                                            int jb) {
    const double tsea = bc[(size_t)kBcSst * kNGP + pt], fmask = bc[(size_t)kBcFmask1 * kNGP + pt];
    const double stl = bc[(size_t)kBcStl * kNGP + pt];
    const double tsfc = tsea + fmask * (stl - tsea);
    return phys::fband_row(fbt, tsfc)[jb];
}

namespace pairx {

// the partner's value (lanes ^ 1: DPP quad permutation 1 0 3 2)
__device__ __forceinline__ double swap(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)(b >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// level 4 h + j of a whole-column array (h a lane value, j compile-time)
__device__ __forceinline__ double own(const double (&a)[kKX], int h, int j) { return h ? a[4 + j] : a[j]; }
// level 4 (1 - h) + j (the partner's levels)
__device__ __forceinline__ double oth(const double (&a)[kKX], int h, int j) { return h ? a[j] : a[4 + j]; }

}  // namespace pairx

// The longwave / surface chain of column pt on pair lane h (and the shortwave before it
// on a lradsw step).  Ai: the column's row in A (t, q, phi at kOT / kOQ / kOPhi + k,
// log ps at kOPs); u7 / v7: the bottom level's wind (x cosgr); fsr: fband(nint(tsfc),
// 2h + b) for b = 0, 1; P: PhysTables (LDS copy); fbt: fband (global); mh: on a
// shortwave step the moist side's precnv, precls, itop and rh of the column (LDS).
template <int kOT, int kOQ, int kOPhi, int kOPs>
__device__ __forceinline__ void phys_pair(int h, int pt, int jlat, const double *Ai, double u7, double v7,
                                          const PairPre &pre, const double *__restrict__ bc, double *__restrict__ rad,
                                          const PhysTables *P, const double *__restrict__ fbt, const double (&fsr)[2],
                                          const double *mh, bool lradsw, PairOut &o) {
    using namespace phys;
    using pairx::oth;
    using pairx::own;
    using pairx::swap;
    constexpr int NL = kKX, nl1 = kKX - 1;  // nl1: 1-based index of the level above the bottom
    auto BC = [&](int f) { return bc[(size_t)f * kNGP + pt]; };

    double ta[NL], qa[NL], ph[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        ta[k] = Ai[kOT + k];
        qa[k] = Ai[kOQ + k];
        ph[k] = Ai[kOPhi + k];
    }
    const double ps1 = Ai[kOPs];
    // bands 2h, 2h + 1's fband rows (radlw, both passes): issued as soon as ta is known on a
    // longwave-only step, after the shortwave on a shortwave step (registers)
    double fbq[2][NL];
    auto load_fbq = [&]() {
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int k = 0; k < NL; ++k) fbq[b][k] = fband_row(fbt, ta[k])[2 * h + b];
    };
    if (!lradsw) load_fbq();

    double psg, rps, qc[NL];
    double tq[2][NL], strat0, strat1, ssrd, rsw[4];
    if (lradsw) {
        // the moist part's results from the moist side (mh: precnv, precls, itop, rh(1..8),
        // phys_moist / phys_thermo's values, handed over at the block barrier of a
        // shortwave step), then cloud and radsw (phys_sw) level- and band-split
        psg = exp(ps1);
        rps = 1. / psg;
#pragma unroll
        for (int k = 0; k < NL; ++k) qc[k] = fmax(qa[k], 0.);
        const double precnv = mh[0], precls = mh[1];
        const int itop = (int)mh[2];
        double rh[NL], se[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            rh[k] = mh[3 + k];
            se[k] = cp * ta[k] + ph[k];
        }
        const double *qa_ = qc;
        const double gse = (se[NL - 2] - se[NL - 1]) / (ph[NL - 2] - ph[NL - 1]);
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
            if (drh > cloudc && qa_[k - 1] > qacl) {
                cloudc = drh;
                icltop = k;
            }
        }
        const double cl1 = fmin(1., cloudc * rrcl);
        const double pr1 = fmin(pmaxcl, 86.4 * (precnv + precls));
        cloudc = fmin(1., wpcl * sqrt(pr1) + cl1 * cl1);
        icltop = (itop < icltop) ? itop : icltop;
        const double qcloud = qa_[nl1 - 1];
        {
            const double clfact = 1.2, rgse = 1. / (gse_s1 - gse_s0);
            const double fst = fmax(0., fmin(1., rgse * (gse - gse_s0)));
            clstr = fst * fmax(clsmax - clfact * cloudc, 0.);
            const double clstrl = fmax(clstr, clsminl) * rh[NL - 1];
            clstr = clstr + BC(kBcFmask1) * (clstrl - clstr);
        }
        // radsw's t1, t2 of the lane's levels (phy_radiat.f90:190-214), then the column's
        const double fband2 = 0.05, fband1 = 1. - fband2;
        const double psaz = psg * BC(kBcZenit);
        const double acloud = cloudc * fmin(abscl1 * qcloud, abscl2);
        double t1[NL], t2[NL], t3[NL], dfabs[NL];
        {
            double o1[4], o2[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int L = 4 * h + j, k = L + 1;
                const double qk = own(qc, h, j);
                const double abs1 = absdry + absaer * P->sig[k - 1] * P->sig[k - 1];
                const double deltap = psaz * P->dsig[k - 1];
                const double a0 = -(psaz * P->dsig[k - 1]) * absdry;
                const double ax = -deltap * (abs1 + abswv1 * qk + acloud);
                const double ay = -deltap * (abs1 + abswv1 * qk);
                o1[j] = exp(L == 0 ? a0 : (L < NL - 1 && k >= icltop) ? ax : ay);
                const double e2 = exp(-(psaz * P->dsig[k - 1]) * abswv2 * qk);
                o2[j] = L >= 1 ? e2 : 0.0;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const double w1 = swap(o1[j]), w2 = swap(o2[j]);
                t1[j] = h ? w1 : o1[j];
                t1[4 + j] = h ? o1[j] : w1;
                t2[j] = h ? w2 : o2[j];
                t2[4 + j] = h ? o2[j] : w2;
            }
        }
#pragma unroll
        for (int k = 0; k < NL; ++k) t3[k] = (k + 1 == icltop) ? albcl * cloudc : 0.0;  // icltop <= nlev only
        t3[NL - 1] = albcls * clstr;
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
        ssrd = fsfcd;
        // longwave transmissivities of bands 2h, 2h + 1 (phy_radiat.f90:262-300)
        const double acl = cloudc * ablcl2;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            const int jb = 2 * h + b;
#pragma unroll
            for (int k = 1; k <= NL; ++k) {
                const double deltap = psg * P->dsig[k - 1];
                const double qk = qc[k - 1];
                const bool mid = k >= 3 && k <= nl1;
                double e;
                if (b == 0) {  // band 0 (h = 0) or 2 (h = 1)
                    const double acloud1 = (k < icltop) ? acl : ablcl1 * cloudc;
                    const double a0 = mid ? -deltap * (ablwin + acloud1) : -deltap * ablwin;
                    const double a2 = mid ? -deltap * fmax(ablwv1 * qk, acl) : -deltap * ablwv1 * qk;
                    e = exp(h ? a2 : a0);
                } else {  // band 1 (h = 0) or 3 (h = 1)
                    const double a1 = -deltap * ablco2;
                    const double a3 = mid ? -deltap * fmax(ablwv2 * qk, acl) : -deltap * ablwv2 * qk;
                    e = exp(h ? a3 : a1);
                }
                tq[b][k - 1] = (k == 1 && jb >= 2) ? 1. : e;
            }
        }
        const double eps1 = epslw / (P->dsig[0] + P->dsig[1]);
        strat0 = BC(kBcStratz) * psg;
        strat1 = eps1 * psg;
#pragma unroll
        for (int j = 0; j < 4; ++j) rsw[j] = own(dfabs, h, j) * rps * P->grdscp[4 * h + j];
        // the column's state for the steps until the next shortwave step
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int k = 0; k < NL; ++k) rad[kRadTau2 + ((size_t)(2 * h + b) * NL + k) * kNGP + pt] = tq[b][k];
        if (h == 0) {
            rad[kRadStratc + pt] = strat0;
            rad[kRadStratc + kNGP + pt] = strat1;
            rad[kRadSsrd + pt] = fsfcd;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) rad[kRadTtRsw + (size_t)(4 * h + j) * kNGP + pt] = rsw[j];
    } else {  // phys_thermo's psg, rps and clipped q; rad's state
        psg = exp(ps1);
        rps = 1. / psg;
#pragma unroll
        for (int k = 0; k < NL; ++k) qc[k] = fmax(qa[k], 0.);
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int k = 0; k < NL; ++k) tq[b][k] = pre.tau[b][k];
        strat0 = pre.strat0;
        strat1 = pre.strat1;
        ssrd = pre.ssrd;
#pragma unroll
        for (int j = 0; j < 4; ++j) rsw[j] = pre.ttrsw[j];
    }

    SML_PST_T(15, 256);
    if (lradsw) load_fbq();
    // 3.2 radlw(-1) (phy_radiat.f90:330-413): the blackbody terms on both lanes, bands
    // 2h, 2h + 1's downward fluxes after each level
    double st4a1[NL], st4a2[NL];
#pragma unroll
    for (int k = 1; k <= nl1; ++k) st4a1[k - 1] = ta[k - 1] + P->wvi[k - 1][1] * (ta[k] - ta[k - 1]);
    st4a2[0] = 0.75 * ta[0] + 0.25 * st4a1[0];
    st4a2[1] = 0.50 * ta[1] + 0.25 * (st4a1[0] + st4a1[1]);
    {
        const double anis = 1.0, anish = 0.5 * anis;
#pragma unroll
        for (int k = 3; k <= nl1; ++k) st4a2[k - 1] = anish * fmax(st4a1[k - 1] - st4a1[k - 2], 0.);
        st4a2[NL - 1] = anis * fmax(ta[NL - 1] - st4a1[nl1 - 1], 0.);
    }
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
    double fo[2][NL];  // band 2h + b's flux after level k
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const double emis = 1. - tq[b][0];
        const double brad = fbq[b][0] * (st4a1[0] + emis * st4a2[0]);
        const double f0 = emis * brad;
        double fl = h == 0 ? f0 : 0.0;  // (bands 3, 4 start at the second level)
        fo[b][0] = fl;
#pragma unroll
        for (int k = 2; k <= NL; ++k) {
            const double tau = tq[b][k - 1];
            const double e = 1. - tau;
            const double br = fbq[b][k - 1] * (st4a1[k - 1] + e * st4a2[k - 1]);
            fl = tau * fl + e * br;
            fo[b][k - 1] = fl;
        }
    }
    // the partner's bands at this lane's levels (and at level 3, and the surface)
    double pr[2][4], pm[2], p7[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) pr[b][j] = swap(oth(fo[b], h, j));
        pm[b] = swap(h == 0 ? fo[b][3] : 0.0);
        p7[b] = swap(fo[b][NL - 1]);
    }
    // band jb's flux after level 4h + j (j = -1: level 4h - 1), from this lane or the partner
    auto fdn = [&](int jb, int j) -> double {
        const int b = jb & 1;
        const bool mine = (jb >> 1) == h;
        const double m = j < 0 ? (h ? fo[b][3] : 0.0) : own(fo[b], h, j);
        const double p = j < 0 ? pm[b] : pr[b][j];
        return mine ? m : p;
    };
    double fsfcd = 0.0;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb) fsfcd = fsfcd + emisfc * (((jb >> 1) == h) ? fo[jb & 1][NL - 1] : p7[jb & 1]);
    const double corlw = (epslw * emisfc) * st4a1[NL - 1];
    fsfcd = fsfcd + corlw;
    double dl[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int L = 4 * h + j;
        double dg = 0.0;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
            dg = dg + fdn(jb, j - 1);
            dg = dg - fdn(jb, j);
        }
        double d0 = 0.0;
        d0 = d0 - fo[0][0];
        d0 = d0 - fo[1][0];
        double d = L == 0 ? d0 : dg;
        const double dc = d - corlw;
        dl[j] = L == NL - 1 ? dc : d;
    }
    const double slrd = fsfcd;
    SML_PST_T(16, 256);

    // 3.3 suflux with lfluxland = .true. (phy_suflux.f90:1-355), both lanes
    double ustr3, vstr3, shf3, evap3, slru3;
    {
        constexpr int nlev = NL;
        const double esbc = emisfc * sbc, esbc4 = 4. * esbc, dlambda = clambsn - clambda;
        const double u0 = fwind0 * u7, v0 = fwind0 * v7;
        const double gtemp0 = 1. - ftemp0, rcp = 1. / cp, rdphi0 = -1. / (rd * 288. * P->sigl[nlev - 1]);
        const double phi0 = BC(kBcPhis0), fmask = BC(kBcFmask1), ssrdj = ssrd;
        double t1[2], t2[2], denvvs[3], qsat0[2];
        const double dt1 = P->wvi[nlev - 1][1] * (ta[nlev - 1] - ta[nl1 - 1]);
        t1[0] = ta[nlev - 1] + dt1;
        t1[1] = t1[0] + phi0 * dt1 * rdphi0;
        t2[1] = ta[nlev - 1] + rcp * ph[nlev - 1];
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
        const double stl = BC(kBcStl), albl = BC(kBcAlbL);
        double tskin = stl + ctday * sqrt(P->clat[jlat]) * ssrdj * (1. - albl) * psg;
        const double rdth = fstab / dtheta, astab = 0.5;
        const double dthl = (tskin > t2[0]) ? fmin(dtheta, tskin - t2[0]) : fmax(-dtheta, astab * (tskin - t2[0]));
        denvvs[1] = denvvs[0] * (1. + dthl * rdth);
        const double cdldv = cdl * denvvs[0] * BC(kBcForog);
        const double ustr1 = -cdldv * u7, vstr1 = -cdldv * v7;
        const double chlcp = chl * cp;
        double shf1 = chlcp * denvvs[1] * (tskin - t1[0]);
        const double q1l = qc[nlev - 1];  // fhum0 = 0
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
        const double tsea = BC(kBcSst);
        const double dths = (tsea > t2[1]) ? fmin(dtheta, tsea - t2[1]) : fmax(-dtheta, astab * (tsea - t2[1]));
        denvvs[2] = denvvs[0] * (1. + dths * rdth);
        const double q1s = qc[nlev - 1];
        const double cdsdv = cds * denvvs[2];
        const double ustr2 = -cdsdv * u7, vstr2 = -cdsdv * v7;
        const double chscp = chs * cp;
        const double shf2 = chscp * denvvs[2] * (tsea - t1[1]);
        const double qs = qsat_at(tsea, psg, 1.);
        const double evap2 = chs * denvvs[2] * (qs - q1s);
        const double ts2 = tsea * tsea;
        const double slru2 = esbc * (ts2 * ts2);
        ustr3 = ustr2 + fmask * (ustr1 - ustr2);
        vstr3 = vstr2 + fmask * (vstr1 - vstr2);
        shf3 = shf2 + fmask * (shf1 - shf2);
        evap3 = evap2 + fmask * (evap1 - evap2);
        slru3 = slru2 + fmask * (slru1 - slru2);
    }

    SML_PST_T(17, 256);
    // 3.4 radlw(1) (phy_radiat.f90:414-458): bands 2h, 2h + 1 upward
    const double refsfc = 1. - emisfc, fsfcu = slru3;
    double fu[2][NL], fs0[2];  // band 2h + b's flux after level k going up; its surface start
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        double fl = fsr[b] * fsfcu + refsfc * fo[b][NL - 1];
        fs0[b] = fl;
#pragma unroll
        for (int k = NL; k >= 2; --k) {
            const double tau = tq[b][k - 1];
            const double e = 1. - tau;
            const double br = fbq[b][k - 1] * (st4a1[k - 1] - e * st4a2[k - 1]);
            fl = tau * fl + e * br;
            fu[b][k - 1] = fl;
        }
        const double tau = tq[b][0];
        const double e = 1. - tau;
        const double br = fbq[b][0] * (st4a1[0] - e * st4a2[0]);
        fu[b][0] = tau * fl + e * br;  // (bands 3, 4: unused)
    }
    // the partner's bands at this lane's levels, and at the level above its top one (4h + 4:
    // level 4, or the surface start for level 7)
    double qr[2][4], qp[2];
#pragma unroll
    for (int b = 0; b < 2; ++b) {
#pragma unroll
        for (int j = 0; j < 4; ++j) qr[b][j] = swap(oth(fu[b], h, j));
        qp[b] = swap(h == 1 ? fu[b][4] : fs0[b]);
    }
    // band jb's upward flux after level 4h + j (j = 4: level 4h + 4, the surface start at 8)
    auto fup = [&](int jb, int j) -> double {
        const int b = jb & 1;
        const bool mine = (jb >> 1) == h;
        const double m = j > 3 ? (h ? fs0[b] : fu[b][4]) : own(fu[b], h, j);
        const double p = j > 3 ? qp[b] : qr[b][j];
        return mine ? m : p;
    };
    const double corlw1 = P->dsig[0] * strat1 * st4a1[0] + strat0;
    const double corlw2 = P->dsig[1] * strat1 * st4a1[1];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int L = 4 * h + j;
        double d = dl[j];
        const double ds = d + epslw * fsfcu;
        d = L == NL - 1 ? ds : d;
        double dg = d;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) {
            dg = dg + fup(jb, j + 1);
            dg = dg - fup(jb, j);
        }
        double d0 = d;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            d0 = d0 + fu[b][1];
            d0 = d0 - fu[b][0];
        }
        d = L == 0 ? d0 : dg;
        const double c1 = d - corlw1, c2 = d - corlw2;
        d = L == 0 ? c1 : L == 1 ? c2 : d;
        o.rlw[j] = d * rps * P->grdscp[L];
        o.rsw[j] = rsw[j];
    }
    o.ust = ustr3;
    o.vst = vstr3;
    o.shf = shf3;
    o.evp = evap3;
    o.rps = rps;
}

#endif  // __HIPCC__
}  // namespace sml

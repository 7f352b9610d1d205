// sml_physics_quad.hpp -- phypar on four lanes per grid column (the row kernel's form).
//
// Reference: phypar (src/phy_phypar.f90:53-196) and the routines sml_physics.hpp
// restates: convmf (phy_convmf.f90:22-238), lscond (phy_lscond.f90:20-109), cloud +
// radsw (phy_radiat.f90:86-328), radlw (:330-458), suflux (phy_suflux.f90:1-355),
// vdifsc (phy_vdifsc.f90:17-124).
//
// Layout.  A quad of four neighbouring lanes owns one column; lane q owns the levels
// 2q and 2q + 1 (0 = top).  Work that is independent per level -- the saturation
// humidity, lscond, the shortwave transmissivities t1 / t2, the tendencies' scaling,
// vdifsc's per-level sums -- runs on the owning lane; the longwave's four spectral
// bands run one per lane (band q: its eight transmissivities, fband rows and flux
// recurrence down and up); the column-wide recurrences the reference evaluates in one
// order (convmf's trigger and mass-flux chain, cloud, radsw's flux chains, suflux) run
// on all four lanes alike on the whole column.  The lanes meet through a few LDS
// slots of their column (the row kernel's spare columns): a quad lies inside one wave,
// whose LDS operations complete in issue order, so a compiler barrier orders a slot's
// writes before the other lanes' reads.
//
// Every expression is sml_physics.hpp's, and every sum keeps the reference's order
// (the band contributions to a level's flux divergence are added band by band,
// incoming before outgoing, as radlw's band-outer loop adds them), so the quad form
// is bitwise the one-lane-per-column form (tests/test_physics_gpu.py).
#pragma once
#include "sml_physics.hpp"

namespace sml {
#ifdef __HIPCC__

// per-block constants, computed once from PhysTables (the same helpers phys_moist and
// phys_vdif call, so the same values)
struct QuadK {
    double entr[kKX + 1];
    VdifK vk;
};

// a longwave-only step's radiation state of the column, loaded as the physics starts
// (band q's transmissivities, the lane's two levels of tt_rsw)
struct QuadPre {
    double tau[kKX];
    double strat0, strat1, ssrd, ttrsw[2];
};

// the quad lane's share of phys_column's results, for the sums of phy_phypar.f90:174-196
struct QuadOut {
    double ttm[2], rsw[2], rlw[2], ttv[2], qtk[2];  // own levels 2q + s
    double utv7, vtv7;                              // the surface stress (bottom level)
};

namespace quad {

// orders a quad's slot writes before its lanes' reads (see above): a wavefront-scope
// fence is a compiler barrier for memory operations and emits no wait (an inline-asm
// memory clobber made the compiler wait for every global load in flight, vmcnt(0):
// 2-3 us per step of the loads issued ahead)
__device__ __forceinline__ void qsync() {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// min over the four lanes of the quad (DPP quad permutations)
__device__ __forceinline__ int qmin(int v) {
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false));  // lanes ^ 1
    v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false));  // lanes ^ 2
    return v;
}

// a[2 q + s] for a lane value q (s compile-time): selects, no indexed register access
__device__ __forceinline__ double pk(const double (&a)[kKX], int q, int s) {
    const double v0 = a[s], v1 = a[2 + s], v2 = a[4 + s], v3 = a[6 + s];
    return q == 0 ? v0 : q == 1 ? v1 : q == 2 ? v2 : v3;
}

// radlw's per-band flux slots in the A row: band b's eight levels, then the upward
// pass's four start values (the physics-only columns t1 q1 phi1 ps1 | ucos1 vcos1 and
// A's unused tail, free once the quad has read its inputs)
__device__ __forceinline__ int lw_slot(int b) { return b < 3 ? 32 + 8 * b : 75; }
__device__ __forceinline__ int lw_up0(int b) { return 83 + b; }

}  // namespace quad

// radlw(1)'s surface emission row fband(nint(tsfc), jb) of column pt (suflux's tsfc =
// sst + fmask (stl - sst), phy_suflux.f90, from the boundary fields alone): the row
// kernel stages it during gridx, off the physics' chain of dependent loads
__device__ __forceinline__ double quad_fsr(const double *__restrict__ bc, const double *__restrict__ fbt, int pt,
                                           int jb) {
    const double tsea = bc[(size_t)kBcSst * kNGP + pt], fmask = bc[(size_t)kBcFmask1 * kNGP + pt];
    const double stl = bc[(size_t)kBcStl * kNGP + pt];
    const double tsfc = tsea + fmask * (stl - tsea);
    return phys::fband_row(fbt, tsfc)[jb];
}

// phypar of column pt on quad lane q.  Ai: the column's row in A (the transformed
// level-1 fields t, q, phi at kOT / kOQ / kOPhi + k, log ps at kOPs; the LW slots); Sb: 24 spare
// slots of the column in B; u7 / v7: the bottom level's wind (x cosgr);
// P: PhysTables (LDS copy); fbt: fband (global); fsrq: fband(nint(tsfc), q + 1) of
// the upward pass's surface term (quad_fsr, staged ahead); rad: radiation state
// (written on a shortwave step).
template <int kOT, int kOQ, int kOPhi, int kOPs>
__device__ __forceinline__ void phys_quad(int q, int pt, int jlat, double *Ai, double *Sb, double u7, double v7,
                                          const QuadPre &pre, const double *__restrict__ bc, double *__restrict__ rad, const PhysTables *P,
                                          const QuadK *K, const double *__restrict__ fbt, double fsrq, bool lradsw,
                                          QuadOut &o) {
    using namespace phys;
    using quad::pk;
    constexpr int NL = kKX, nl1 = kKX - 1;  // nl1: 1-based index of the level above the bottom
    auto BC = [&](int f) { return bc[(size_t)f * kNGP + pt]; };  // (read where used)

    // the column's inputs, on every lane of the quad
    double ta[NL], qa[NL], ph[NL], se[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        ta[k] = Ai[kOT + k];
        qa[k] = Ai[kOQ + k];
        ph[k] = Ai[kOPhi + k];
    }
    const double ps1 = Ai[kOPs];
    quad::qsync();  // (the inputs' columns become the longwave's slots)
    SML_PST_T(30, 128);
    // band q's fband rows (radlw, both passes), issued as soon as their indices are known
    double fbq[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) fbq[k] = fband_row(fbt, ta[k])[q];
    // 1.2 thermodynamic variables (phys_thermo): qsat, rh on the owning lane
    const double psg = exp(ps1), rps = 1. / psg;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        qa[k] = fmax(qa[k], 0.);
        se[k] = cp * ta[k] + ph[k];
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const int L = 2 * q + s;
        const double qs = qsat_at(pk(ta, q, s), psg, P->sig[L]);
        Sb[L] = qs;
        Sb[8 + L] = pk(qa, q, s) / qs;
    }
    quad::qsync();
    double qsat[NL], rh[NL];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        qsat[k] = Sb[k];
        rh[k] = Sb[8 + k];
    }
    SML_PST_T(22, 128);

    // 2.1 convmf on the whole column (every lane)
    PhysThermo h;
    h.psg = psg;
    h.rps = rps;
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        h.qa[k] = qa[k];
        h.se[k] = se[k];
        h.rh[k] = rh[k];
        h.qsat[k] = qsat[k];
    }
    double dfs[NL], dfq[NL], precnv;
    int itop;
    phys_convmf(h, P, K->entr, dfs, dfq, precnv, itop);
    const int icnv = NL - itop;  // phy_phypar.f90:107-109
    SML_PST_T(23, 128);

    // 2.2 lscond on the owning lane; itop = min(itop, the condensing levels), precls
    // summed in level order from the lanes' slots
    double ttl[2], qtl[2], qtm[2];
    {
        const double qsmax = 10., rtlsc = 1. / (trlsc * 3600.), tfact = alhc / cp, prg = p0 / gg;
        const double psa2 = psg * psg;
        int itl = itop;
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int L = 2 * q + s, k = L + 1;
            const double sig2 = P->sig[L] * P->sig[L];
            double rhref = rhlsc + drhlsc * (sig2 - 1.);
            if (k == NL) rhref = fmax(rhref, rhblsc);
            const double dqmax = qsmax * sig2 * rtlsc;
            const double dqa = rhref * pk(qsat, q, s) - pk(qa, q, s);
            const bool hit = L >= 1 && dqa < 0.0;
            const double qv = dqa * rtlsc;
            qtl[s] = hit ? qv : 0.;
            ttl[s] = hit ? tfact * fmin(-qv, dqmax * psa2) : 0.;
            itl = (hit && k < itl) ? k : itl;
            Sb[16 + L] = qtl[s];
        }
        itop = quad::qmin(itl);
        SML_PST_T(31, 128);
        quad::qsync();
        double precls = 0.;
#pragma unroll
        for (int k = 2; k <= NL; ++k) precls = precls - (P->dsig[k - 1] * prg) * Sb[16 + k - 1];
        precls = precls * psg;
        // convection scaled (phy_phypar.f90:100-105) + condensation, own levels (:118-119)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int L = 2 * q + s;
            double ttc = pk(dfs, q, s), qtc = pk(dfq, q, s);
            const double tts = ttc * rps * P->grdscp[L], qts = qtc * rps * P->grdsig[L];
            ttc = L >= 1 ? tts : ttc;
            qtc = L >= 1 ? qts : qtc;
            o.ttm[s] = 0. + ttc + ttl[s];
            qtm[s] = 0. + qtc + qtl[s];
        }

        double tq[NL], strat0, strat1, ssrd;  // band q's transmissivities, rad's stratc / ssrd
        // 4.1 vdifsc (phys_vdif; it needs nothing from the radiation, so it runs here and
        // the column's arrays it reads die before the longwave): the interface fluxes on
        // every lane, each level's sums in the reference's order on the owning lane
        double qvd[2];
        {
            constexpr int nlev = NL;
            const VdifK &vk = K->vk;
            const double drh0 = rhgrad * (P->sig[nlev - 1] - P->sig[nl1 - 1]);
            const double fvdiq2 = vk.fvdiq * P->sigh[nl1];
            // shallow convection: the two bottom levels
            const double dmse = (se[nlev - 1] - se[nl1 - 1]) + alhc * (qa[nlev - 1] - qsat[nl1 - 1]);
            const double drh = rh[nlev - 1] - rh[nl1 - 1];
            double fcnv = 1.;
            double tv6 = 0., tv7 = 0., qv6 = 0., qv7 = 0.;
            if (dmse >= 0.0) {
                if (icnv > 0) fcnv = redshc;
                const double fluxse = fcnv * vk.fshcse * dmse;
                tv6 = fluxse * vk.rsig[nl1 - 1];
                tv7 = -fluxse * vk.rsig[nlev - 1];
                if (drh >= 0.0) {
                    const double fluxq = fcnv * vk.fshcq * qsat[nlev - 1] * drh;
                    qv6 = fluxq * vk.rsig[nl1 - 1];
                    qv7 = -fluxq * vk.rsig[nlev - 1];
                }
            } else if (drh >= drh0) {
                const double fluxq = fvdiq2 * qsat[nl1 - 1] * drh;
                qv6 = fluxq * vk.rsig[nl1 - 1];
                qv7 = -fluxq * vk.rsig[nlev - 1];
            }
            // moisture above the PBL (k = 3 .. nlev-2) and the super-adiabatic damping
            // (k = 1 .. nlev-1): each interface's flux
            double fq[NL + 1], fs[NL + 1];
            bool cq[NL + 1], cs[NL + 1];
#pragma unroll
            for (int k = 0; k <= NL; ++k) {
                fq[k] = fs[k] = 0.;
                cq[k] = cs[k] = false;
            }
#pragma unroll
            for (int k = 3; k <= nlev - 2; ++k)
                if (P->sigh[k] > 0.5) {
                    const double drh0k = rhgrad * (P->sig[k] - P->sig[k - 1]);
                    const double fvdiq2k = vk.fvdiq * P->sigh[k];
                    const double drhk = rh[k] - rh[k - 1];
                    cq[k] = drhk >= drh0k;
                    fq[k] = fvdiq2k * qsat[k - 1] * drhk;
                }
#pragma unroll
            for (int k = 1; k <= nl1; ++k) {
                const double se0 = se[k] + segrad * (ph[k - 1] - ph[k]);
                cs[k] = se[k - 1] < se0;
                fs[k] = vk.fvdise * (se0 - se[k - 1]);
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int L = 2 * q + s;
                double tv = L == nl1 - 1 ? tv6 : L == nlev - 1 ? tv7 : 0.;
                double qv = L == nl1 - 1 ? qv6 : L == nlev - 1 ? qv7 : 0.;
                const double rsL = L == 0 ? vk.rsig[0] : L == 1 ? vk.rsig[1] : L == 2 ? vk.rsig[2] : L == 3 ? vk.rsig[3]
                                 : L == 4 ? vk.rsig[4] : L == 5 ? vk.rsig[5] : L == 6 ? vk.rsig[6] : vk.rsig[7];
                // qtv[k-1] += fluxq rsig[k-1]; qtv[k] -= fluxq rsig[k]: level L takes k = L first
#pragma unroll
                for (int k = 3; k <= nlev - 2; ++k) {
                    const double qm = qv - fq[k] * rsL, qp = qv + fq[k] * rsL;
                    qv = (k == L && cq[k]) ? qm : qv;
                    qv = (k == L + 1 && cq[k]) ? qp : qv;
                }
                // ttv[k-1] += fluxse rsig[k-1]; ttv[k1-1] -= fluxse rsig1[k-1], k1 > k
#pragma unroll
                for (int k = 1; k <= nl1; ++k) {
                    const double tm = tv - fs[k] * vk.rsig1[k - 1], tp = tv + fs[k] * rsL;
                    tv = (k <= L && cs[k]) ? tm : tv;
                    tv = (k == L + 1 && cs[k]) ? tp : tv;
                }
                o.ttv[s] = tv;
                qvd[s] = qv;
            }
        }
        SML_PST_T(24, 128);
        // 3.1 shortwave (phys_sw), on lradsw steps; otherwise the state kept in rad
        if (lradsw) {
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
            // radsw: t1, t2 of the owning lane's levels (phy_radiat.f90:190-214)
            const double fband2 = 0.05, fband1 = 1. - fband2;
            const double psaz = psg * BC(kBcZenit);
            const double acloud = cloudc * fmin(abscl1 * qcloud, abscl2);
            quad::qsync();  // (qsat / rh's slots are read: t1 / t2 reuse them)
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int L = 2 * q + s, k = L + 1;
                const double qk = pk(qa, q, s);
                const double abs1 = absdry + absaer * P->sig[k - 1] * P->sig[k - 1];
                const double deltap = psaz * P->dsig[k - 1];
                const double a0 = -(psaz * P->dsig[k - 1]) * absdry;
                const double ax = -deltap * (abs1 + abswv1 * qk + acloud);
                const double ay = -deltap * (abs1 + abswv1 * qk);
                const double a1 = L == 0 ? a0 : (L < NL - 1 && k >= icltop) ? ax : ay;
                Sb[L] = exp(a1);
                const double e2 = exp(-(psaz * P->dsig[k - 1]) * abswv2 * qk);
                Sb[8 + L] = L >= 1 ? e2 : 0.0;
            }
            quad::qsync();
            double t1[NL], t2[NL], t3[NL], dfabs[NL];
#pragma unroll
            for (int k = 0; k < NL; ++k) {
                t1[k] = Sb[k];
                t2[k] = Sb[8 + k];
                t3[k] = (k + 1 == icltop) ? albcl * cloudc : 0.0;  // icltop <= nlev only
            }
            t3[NL - 1] = albcls * clstr;
            // the flux chains on the whole column (phy_radiat.f90:216-258)
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
            // longwave transmissivities of band q (phy_radiat.f90:262-300)
            const double acl = cloudc * ablcl2;
#pragma unroll
            for (int k = 1; k <= NL; ++k) {
                const double deltap = psg * P->dsig[k - 1];
                const double qk = qa[k - 1];
                const bool mid = k >= 3 && k <= nl1;
                const double acloud1 = (k < icltop) ? acl : ablcl1 * cloudc;
                const double a0 = mid ? -deltap * (ablwin + acloud1) : -deltap * ablwin;
                const double a1 = -deltap * ablco2;
                const double c23 = q == 2 ? ablwv1 : ablwv2;
                const double a23 = mid ? -deltap * fmax(c23 * qk, acl) : -deltap * c23 * qk;
                const double e = exp(q == 0 ? a0 : q == 1 ? a1 : a23);
                tq[k - 1] = (k == 1 && q >= 2) ? 1. : e;
            }
            const double eps1 = epslw / (P->dsig[0] + P->dsig[1]);
            strat0 = BC(kBcStratz) * psg;
            strat1 = eps1 * psg;
            ssrd = fsfcd;
            double rsw[2];
#pragma unroll
            for (int s = 0; s < 2; ++s) rsw[s] = pk(dfabs, q, s) * rps * P->grdscp[2 * q + s];
            // the column's state for the steps until the next shortwave step
#pragma unroll
            for (int k = 0; k < NL; ++k) rad[kRadTau2 + ((size_t)q * NL + k) * kNGP + pt] = tq[k];
            if (q == 0) {
                rad[kRadStratc + pt] = strat0;
                rad[kRadStratc + kNGP + pt] = strat1;
                rad[kRadSsrd + pt] = fsfcd;
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) rad[kRadTtRsw + (size_t)(2 * q + s) * kNGP + pt] = rsw[s];
            o.rsw[0] = rsw[0];
            o.rsw[1] = rsw[1];
        } else {
#pragma unroll
            for (int k = 0; k < NL; ++k) tq[k] = pre.tau[k];
            strat0 = pre.strat0;
            strat1 = pre.strat1;
            ssrd = pre.ssrd;
            o.rsw[0] = pre.ttrsw[0];
            o.rsw[1] = pre.ttrsw[1];
        }

        SML_PST_T(25, 128);
        // 3.2 radlw(-1) (phy_radiat.f90:330-413): the column's blackbody terms on every
        // lane, band q's downward flux on lane q; each flux after each level into the
        // band's slots
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
        const int sq = quad::lw_slot(q);
        double fl;
        {
            const double emis = 1. - tq[0];
            const double brad = fbq[0] * (st4a1[0] + emis * st4a2[0]);
            const double f0 = emis * brad;
            fl = q < 2 ? f0 : 0.0;  // (bands 3, 4 start at the second level)
        }
        Ai[sq] = fl;
#pragma unroll
        for (int k = 2; k <= NL; ++k) {
            const double tau = tq[k - 1];
            const double emis = 1. - tau;
            const double brad = fbq[k - 1] * (st4a1[k - 1] + emis * st4a2[k - 1]);
            fl = tau * fl + emis * brad;
            Ai[sq + k - 1] = fl;
        }
        quad::qsync();
        // the surface's downward longwave; the owning lane's flux divergence, band by band
        double fsfcd = 0.0;
#pragma unroll
        for (int jb = 0; jb < 4; ++jb) fsfcd = fsfcd + emisfc * Ai[quad::lw_slot(jb) + NL - 1];
        const double corlw = (epslw * emisfc) * st4a1[NL - 1];
        fsfcd = fsfcd + corlw;
        double dl[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int L = 2 * q + s, Lm = L > 0 ? L - 1 : 0;
            double dg = 0.0;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                dg = dg + Ai[quad::lw_slot(jb) + Lm];
                dg = dg - Ai[quad::lw_slot(jb) + L];
            }
            double d0 = 0.0;
            d0 = d0 - Ai[quad::lw_slot(0)];
            d0 = d0 - Ai[quad::lw_slot(1)];
            double d = L == 0 ? d0 : dg;
            const double dc = d - corlw;
            dl[s] = L == NL - 1 ? dc : d;
        }
        const double slrd = fsfcd;
        SML_PST_T(26, 128);

        // 3.3 suflux with lfluxland = .true. (phy_suflux.f90:1-355), every lane
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
            // land: skin temperature, fluxes, skin energy balance (lskineb)
            const double stl = BC(kBcStl), albl = BC(kBcAlbL);
            double tskin = stl + ctday * sqrt(P->clat[jlat]) * ssrdj * (1. - albl) * psg;
            const double rdth = fstab / dtheta, astab = 0.5;
            const double dthl = (tskin > t2[0]) ? fmin(dtheta, tskin - t2[0]) : fmax(-dtheta, astab * (tskin - t2[0]));
            denvvs[1] = denvvs[0] * (1. + dthl * rdth);
            const double cdldv = cdl * denvvs[0] * BC(kBcForog);
            const double ustr1 = -cdldv * u7, vstr1 = -cdldv * v7;
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
            const double ustr2 = -cdsdv * u7, vstr2 = -cdsdv * v7;
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
        }

        SML_PST_T(27, 128);
        // 3.4 radlw(1) (phy_radiat.f90:414-458): band q's upward flux on lane q into the
        // slots (the downward pass's are read), then the owning lane's divergence
        const double refsfc = 1. - emisfc, fsfcu = slru3;
        fl = fsrq * fsfcu + refsfc * fl;
        quad::qsync();
        Ai[quad::lw_up0(q)] = fl;
#pragma unroll
        for (int k = NL; k >= 2; --k) {
            const double tau = tq[k - 1];
            const double emis = 1. - tau;
            const double brad = fbq[k - 1] * (st4a1[k - 1] - emis * st4a2[k - 1]);
            fl = tau * fl + emis * brad;
            Ai[sq + k - 1] = fl;
        }
        {
            const double tau = tq[0];
            const double emis = 1. - tau;
            const double brad = fbq[0] * (st4a1[0] - emis * st4a2[0]);
            fl = tau * fl + emis * brad;
            Ai[sq] = fl;  // (bands 3, 4: unused)
        }
        quad::qsync();
        const double corlw1 = P->dsig[0] * strat1 * st4a1[0] + strat0;
        const double corlw2 = P->dsig[1] * strat1 * st4a1[1];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            const int L = 2 * q + s, Lp = L < NL - 1 ? L + 1 : L;
            double d = dl[s];
            const double ds = d + epslw * fsfcu;
            d = L == NL - 1 ? ds : d;
            double dg = d;
#pragma unroll
            for (int jb = 0; jb < 4; ++jb) {
                const double in = L == NL - 1 ? Ai[quad::lw_up0(jb)] : Ai[quad::lw_slot(jb) + Lp];
                dg = dg + in;
                dg = dg - Ai[quad::lw_slot(jb) + L];
            }
            double d0 = d;
#pragma unroll
            for (int jb = 0; jb < 2; ++jb) {
                d0 = d0 + Ai[quad::lw_slot(jb) + 1];
                d0 = d0 - Ai[quad::lw_slot(jb)];
            }
            d = L == 0 ? d0 : dg;
            const double c1 = d - corlw1, c2 = d - corlw2;
            d = L == 0 ? c1 : L == 1 ? c2 : d;
            o.rlw[s] = d * rps * P->grdscp[L];
        }

        SML_PST_T(28, 128);
        // 4.2 the surface fluxes into the bottom layer (phy_phypar.f90:186-191)
        {
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const int L = 2 * q + s;
                const double tvs = o.ttv[s] + shf3 * rps * P->grdscp[NL - 1];
                const double qvs = qvd[s] + evap3 * rps * P->grdsig[NL - 1];
                o.ttv[s] = L == NL - 1 ? tvs : o.ttv[s];
                const double qv = L == NL - 1 ? qvs : qvd[s];
                o.qtk[s] = qtm[s] + qv;
            }
            double utv = 0., vtv = 0.;
            utv = utv + ustr3 * rps * P->grdsig[NL - 1];
            vtv = vtv + vstr3 * rps * P->grdsig[NL - 1];
            o.utv7 = utv;
            o.vtv7 = vtv;
        }
    }
}

#endif  // __HIPCC__
}  // namespace sml

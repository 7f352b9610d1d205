"""Generate tests/golden/phys_ref.npz from the reference's own phypar.

Run in the survey/build container after `make -C oracle ref`:

    python tests/golden/make_phys_golden.py

Drives oracle/_ref/libspeedy_ref_dyn.so (the reference's dyn_*, phy_*, ini_*
sources compiled as-is) like make_dyn_golden.py does, with:
  * reference initialisation (inifft, indyns, inphys, radset), sol_oz(tyear)
    for the radiation forcing, sflset(phis0);
  * a seeded synthetic atmosphere (moist lower levels so that convection, large
    scale condensation, clouds and the shallow-convection branches all fire) and
    synthetic surface fields (land-sea mask, SST, land temperature, soil water,
    albedos);
  * case "rad": lradsw = .true. -> geop(1), phypar with zero input tendencies
    (the physics alone, dyn_grtend.f90:223-226);
  * case "norad": another state, lradsw = .false. (radiation state kept from
    "rad", as the reference keeps it between its nstrad steps).
Physics is column-local, so each case stores the grid inputs phypar computed
(mod_physvar ug1..pslg1) and its tendencies at every 4th longitude only (all
latitudes), plus the radiation state after "rad" at the same columns.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_dyn_golden import IL, IX, KX, MX, NX, Ref, _int, _p, spectral_field  # noqa: E402

SEED = 20250302
TYEAR = 0.3
NGP = IX * IL
SEL = np.arange(NGP)[np.arange(NGP) % 4 == 0]  # every 4th longitude


def main():
    R = Ref()
    L = R.L
    rng = np.random.default_rng(SEED)
    L.inifft_()
    L.indyns_()
    hsg = R.var("mod_dyncon1", "hsg", (KX + 1,))
    fsg = R.var("mod_dyncon1", "fsg", (KX,))
    radang = R.var("mod_dyncon1", "radang", (IL,))
    ppl = np.ascontiguousarray(fsg.copy())
    L.inphys_(_p(hsg), _p(ppl), _p(radang))
    L.radset_()
    ty = ctypes.c_double(TYEAR)
    L.sol_oz_(ctypes.byref(ty))

    rgam = (2.0 / 7.0) * 1004.0 * 6.0 / (1000.0 * 9.81)
    tref = 288.0 * np.maximum(0.2, fsg) ** rgam
    vor = R.var("mod_dynvar", "vor", (MX, NX, KX, 2), np.complex128)
    div = R.var("mod_dynvar", "div", (MX, NX, KX, 2), np.complex128)
    t = R.var("mod_dynvar", "t", (MX, NX, KX, 2), np.complex128)
    ps = R.var("mod_dynvar", "ps", (MX, NX, 2), np.complex128)
    tr = R.var("mod_dynvar", "tr", (MX, NX, KX, 2, 1), np.complex128)
    phi = R.var("mod_dynvar", "phi", (MX, NX, KX), np.complex128)
    phis = R.var("mod_dynvar", "phis", (MX, NX), np.complex128)

    lat = np.repeat(radang, IX)
    lon = np.tile(np.arange(IX) * 2 * np.pi / IX, IL)
    bc = {
        "fmask1": np.clip(0.5 + 0.6 * np.sin(2 * lon) * np.cos(3 * lat), 0.0, 1.0),
        "sst_am": 271.0 + 30.0 * np.cos(lat) ** 2 + 0.5 * rng.standard_normal(NGP),
        "stl_am": 265.0 + 30.0 * np.cos(lat) ** 2 + 1.0 * rng.standard_normal(NGP),
        "soilw_am": np.clip(0.4 + 0.3 * rng.standard_normal(NGP), 0.0, 1.0),
        "alb_l": 0.2 + 0.1 * rng.random(NGP),
        "alb_s": 0.07 + 0.05 * rng.random(NGP),
        "snowc": np.clip(rng.random(NGP) - 0.7, 0.0, 1.0),
    }
    bc["albsfc"] = bc["alb_s"] + bc["fmask1"] * (bc["alb_l"] - bc["alb_s"])
    phis[...] = spectral_field(rng, 2000.0, 1.5, mean=3000.0)
    g = np.zeros((IL, IX))
    L.grid_(_p(np.ascontiguousarray(phis.T).view(np.float64)), _p(g), _int(1))
    bc["phis0"] = g.ravel().copy()
    for name, mod in (("fmask1", "mod_surfcon"), ("phis0", "mod_surfcon")):
        R.var(mod, name, (IX, IL))[...] = bc[name].reshape(IL, IX).T
    for name, mod in (("sst_am", "mod_var_sea"), ("stl_am", "mod_var_land"), ("soilw_am", "mod_var_land"),
                      ("alb_l", "mod_radcon"), ("alb_s", "mod_radcon"), ("snowc", "mod_radcon"),
                      ("albsfc", "mod_radcon")):
        R.var(mod, name, (NGP,))[...] = bc[name]
    R.var("mod_var_sea", "ssti_om", (NGP,))[...] = bc["sst_am"]
    L.sflset_(_p(np.ascontiguousarray(bc["phis0"])))
    forog = R.var("mod_sflcon", "forog", (NGP,)).copy()
    solar = {k: R.var("mod_radcon", k, (NGP,)).copy() for k in ("fsol", "ozone", "ozupp", "zenit", "stratz")}

    def set_state(seed):
        r = np.random.default_rng(seed)
        for k in range(KX):
            vor[:, :, k, 0] = spectral_field(r, 6e-6, 1.5)
            div[:, :, k, 0] = spectral_field(r, 6e-7, 1.5)
            t[:, :, k, 0] = spectral_field(r, 3.0, 1.2, mean=tref[k])
            qm = 14.0 * fsg[k] ** 3
            tr[:, :, k, 0, 0] = spectral_field(r, 0.3 * qm, 1.2, mean=qm)
        ps[:, :, 0] = spectral_field(r, 0.03, 1.5, mean=-0.02)

    def physics(lradsw):
        R.scalar_logical("mod_lflags", "lradsw", lradsw)
        L.geop_(_int(1))
        tend = [np.zeros((KX, IL, IX)) for _ in range(4)]
        L.phypar_(_p(vor), _p(div), _p(t), _p(tr), _p(phi), _p(ps), *[_p(x) for x in tend])
        ins = {k: R.var("mod_physvar", k, (NGP, KX)).T.copy() for k in ("ug1", "vg1", "tg1", "qg1", "phig1")}
        ins["pslg1"] = R.var("mod_physvar", "pslg1", (NGP,)).copy()
        return ins, np.stack([x.reshape(KX, NGP) for x in tend])

    out = {"tyear": np.float64(TYEAR), "sel": SEL, "radang": radang.copy(), "forog": forog}
    out.update({f"bc_{k}": v for k, v in bc.items()})
    out.update({f"sol_{k}": v.reshape(IL, IX)[:, 0].copy() for k, v in solar.items()})
    for case, seed, lradsw in (("rad", 11, True), ("norad", 12, False)):
        set_state(seed)
        ins, tend = physics(lradsw)
        assert np.all(np.isfinite(tend)), case
        for k, v in ins.items():
            out[f"{case}_{k}"] = v[..., SEL]
        out[f"{case}_tend"] = tend[..., SEL]
        if case == "rad":
            tau2 = R.var("mod_radcon", "tau2", (NGP, KX, 4)).transpose(2, 1, 0)
            out["rad_tau2"] = tau2[..., SEL].copy()
            out["rad_stratc"] = R.var("mod_radcon", "stratc", (NGP, 2)).T[:, SEL].copy()
            out["rad_tt_rsw"] = R.var("mod_physvar", "tt_rsw", (NGP, KX)).T[:, SEL].copy()
            out["rad_ssrd"] = R.var("mod_physvar", "ssrd", (NGP,))[SEL].copy()
        # branch coverage evidence
        cb = R.var("mod_physvar", "cbmf", (NGP,))
        pl = R.var("mod_physvar", "precls", (NGP,))
        print(case, "convective columns", int((cb > 0).sum()), "lsc columns", int((pl > 0).sum()),
              "max |tend|", [float(np.abs(x).max()) for x in tend])
    path = os.path.join(HERE, "phys_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

"""Generate tests/golden/fordate_ref.npz from the reference's own per-window forcing.

Run in the survey/build container after `make -C oracle ref`:

    python tests/golden/make_fordate_golden.py

Drives oracle/_ref/libspeedy_ref_dyn.so (the reference's sources compiled as-is;
oracle/Makefile) through its module state, as agcm_init does before every window
(ini_agcm_init.f90:57-89):
  * inifft, indyns, inphys(hsg, ppl, radang) (ini_iniatm.f90:19-33), radset, and the
    surface fields inbcon would have read: fmask_l (mod_cli_land), fmask_s (mod_cli_sea),
    alb0, phis0 (mod_surfcon) and the monthly climatologies stl12, snowd12, soilw12
    (mod_cli_land), sst12, sice12 (mod_cli_sea) -- all synthetic,
    speedy_ml_amd.synthetic.surface_climatology(fmask, seed) with the fmask and phis of
    synthetic.phys_boundary's construction below;
  * per date: mod_date iyear / imonth / iday and mod_tsteps imont0, then newdate(0)
    (tmonth, tyear, imont1); ini_land(2) -> stl_am, snowd_am, soilw_am (cpl_land.f90:
    1-95: atm2land(0), stl_lm = stlcl_ob, land2atm(0) with icland = 1); forin5(sst12),
    forint(sice12) (cpl_bcinterp.f90) -- the sea side's interpolation (atm2sea itself
    lives in cpl_sea.f90, which does not build here);
  * per (date, sst case): sst_am and sice_am (mod_var_sea) set, then fordate(0) ->
    tcorh, qcorh (mod_hdifcon), fsol, ozone, ozupp, zenit, stratz, snowc, alb_l,
    alb_s, albsfc (mod_radcon).
Dates: 1982-01-15 (tmonth <= 0.5, forint wraps to December), 1982-07-03, 1982-12-20
(tmonth > 0.5, wraps to January).  sst cases: the ice-free climatology of the date's
month, and the same + a smooth anomaly (a hybrid SST).  Grid outputs are stored at
every 4th grid point; tcorh / qcorh whole.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from make_dyn_golden import IL, IX, KX, MX, NX, Ref, _int, _p, spectral_field  # noqa: E402

from speedy_ml_amd.synthetic import surface_climatology  # noqa: E402

NGP = IX * IL
SEED = 20251018
SEL = np.arange(0, NGP, 4)
DATES = ((1982, 1, 15), (1982, 7, 3), (1982, 12, 20))
SOL = ("fsol", "ozone", "ozupp", "zenit", "stratz")
ALB = ("snowc", "alb_l", "alb_s", "albsfc")


def inputs():
    """The synthetic fields (seeded): land fraction, spectral orography, surface fields,
    climatologies, the two sst cases' anomaly and a sea-ice field for fordate."""
    rng = np.random.default_rng(SEED)
    lat = np.repeat(np.arcsin(np.polynomial.legendre.leggauss(IL)[0]), IX)
    lon = np.tile(np.arange(IX) * 2 * np.pi / IX, IL)
    fmask = np.clip(0.5 + 0.6 * np.sin(2 * lon) * np.cos(3 * lat), 0.0, 1.0)
    phis = spectral_field(rng, 2000.0, 1.5, mean=3000.0)  # (MX, NX) complex
    surf, clim = surface_climatology(fmask, seed=SEED % 1000)
    anom = 1.5 * np.sin(lon) * np.cos(lat) ** 2 + 0.2 * rng.standard_normal(NGP)
    sice = np.clip(rng.random(NGP) - 0.6, 0.0, 1.0)
    return fmask, phis, surf, clim, anom, sice


def main():
    R = Ref()
    L = R.L
    fmask, phis_c, surf, clim, anom, sice = inputs()
    L.inifft_()
    L.indyns_()
    hsg = R.var("mod_dyncon1", "hsg", (KX + 1,))
    fsg = R.var("mod_dyncon1", "fsg", (KX,))
    radang = R.var("mod_dyncon1", "radang", (IL,))
    L.inphys_(_p(hsg), _p(np.ascontiguousarray(fsg.copy())), _p(radang))
    L.radset_()
    phis = R.var("mod_dynvar", "phis", (MX, NX), np.complex128)
    phis[...] = phis_c
    g = np.zeros((IL, IX))
    L.grid_(_p(np.ascontiguousarray(phis.T).view(np.float64)), _p(g), _int(1))
    phis0 = g.ravel().copy()
    R.var("mod_surfcon", "phis0", (IX, IL))[...] = phis0.reshape(IL, IX).T
    R.var("mod_surfcon", "alb0", (IX, IL))[...] = surf["alb0"].reshape(IL, IX).T
    R.var("mod_cli_land", "fmask_l", (IX, IL))[...] = surf["fmask_l"].reshape(IL, IX).T
    R.var("mod_cli_sea", "fmask_s", (IX, IL))[...] = surf["fmask_s"].reshape(IL, IX).T
    for name, mod in (("stl12", "mod_cli_land"), ("snowd12", "mod_cli_land"), ("soilw12", "mod_cli_land"),
                      ("sst12", "mod_cli_sea"), ("sice12", "mod_cli_sea")):
        R.var(mod, name, (IX, IL, 12))[...] = clim[name].reshape(12, IL, IX).transpose(2, 1, 0)
    sst12 = np.asfortranarray(clim["sst12"].T)   # (ngp, 12) for forin5 / forint
    sice12 = np.asfortranarray(clim["sice12"].T)

    out = {"seed": np.int64(SEED), "sel": SEL, "dates": np.array(DATES), "phis0": phis0}
    ci = lambda mod, name: ctypes.c_int32.in_dll(L, f"_QM{mod}E{name}")  # noqa: E731
    cd = lambda mod, name: ctypes.c_double.in_dll(L, f"_QM{mod}E{name}")  # noqa: E731
    newdate = getattr(L, "_QMmod_datePnewdate")
    for di, (y, mo, dd) in enumerate(DATES):
        ci("mod_tsteps", "iyear0").value = y
        ci("mod_tsteps", "imont0").value = mo
        ci("mod_date", "iyear").value = y
        ci("mod_date", "imonth").value = mo
        ci("mod_date", "iday").value = dd
        newdate(_int(0))
        tmonth, tyear, imont1 = cd("mod_date", "tmonth").value, cd("mod_date", "tyear").value, \
            ci("mod_date", "imont1").value
        L.ini_land_(_int(2))
        land = {k: R.var("mod_var_land", k, (NGP,)).copy() for k in ("stl_am", "snowd_am", "soilw_am")}
        sstcl, sicecl = np.zeros(NGP), np.zeros(NGP)
        L.forin5_(_int(NGP), _int(imont1), ctypes.byref(ctypes.c_double(tmonth)), _p(sst12), _p(sstcl))
        L.forint_(_int(NGP), _int(imont1), ctypes.byref(ctypes.c_double(tmonth)), _p(sice12), _p(sicecl))
        out[f"d{di}_tmonth"], out[f"d{di}_tyear"], out[f"d{di}_imont1"] = tmonth, tyear, imont1
        for k, v in land.items():
            out[f"d{di}_{k}"] = v[SEL]
        out[f"d{di}_sstcl_interp"], out[f"d{di}_sicecl_interp"] = sstcl[SEL], sicecl[SEL]
        base = np.maximum(clim["sst12"][mo - 1], 271.5)
        for si, sst in enumerate((base, base + anom)):
            R.var("mod_var_sea", "sst_am", (NGP,))[...] = sst
            R.var("mod_var_sea", "sice_am", (NGP,))[...] = sice
            L.fordate_(_int(0))
            case = f"d{di}s{si}"
            out[f"{case}_tcorh"] = R.var("mod_hdifcon", "tcorh", (MX, NX), np.complex128).T.copy()
            out[f"{case}_qcorh"] = R.var("mod_hdifcon", "qcorh", (MX, NX), np.complex128).T.copy()
            for k in SOL:
                out[f"{case}_{k}"] = R.var("mod_radcon", k, (NGP,)).reshape(IL, IX)[:, 0].copy()
            for k in ALB:
                out[f"{case}_{k}"] = R.var("mod_radcon", k, (NGP,))[SEL].copy()
            print(case, "tyear", tyear, "|qcorh|", float(np.abs(out[f"{case}_qcorh"]).max()),
                  "|tcorh|", float(np.abs(out[f"{case}_tcorh"]).max()))
    path = os.path.join(HERE, "fordate_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

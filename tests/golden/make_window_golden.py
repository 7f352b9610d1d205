"""Generate tests/golden/window_ref.npz: one whole SPEEDY window from the reference's
own dynamical core and physics, as run_model's agcm_main integrates it.

Run in the build container after `make -C oracle ref`:

    python tests/golden/make_window_golden.py

Drives oracle/_ref/libspeedy_ref_dyn.so (the reference's dyn_*, ini_*, phy_*
sources compiled as-is) through its module state, like make_dyn_golden.py:

 1. initialisation as ini_atm (ini_iniatm.f90:19-33): inifft, indyns, inphys,
    radset; sol_oz(tyear) and sflset(phis0) as fordate does (ini_fordate.f90:44-45);
 2. a seeded synthetic atmosphere (both leapfrog levels) and surface / boundary
    fields written into the reference's module variables (mod_surfcon,
    mod_var_sea, mod_var_land, mod_radcon);
 3. the window: stepone (ini_stepone.f90:19-34: impint(delt/2), step(1,1,delt/2),
    impint(delt), step(1,2,delt), impint(2 delt)) with lradsw = .true. (the
    mod_lflags default), then stloop's first 6-h block (dyn_stloop.f90:26-60 with
    window_size = 24/6 = 4 -> nsteps/4 = 24 steps): for istep = 1..24,
    lradsw = (mod(istep, nstrad = 3) == 1), step(2,2,2 delt).  The radiation state
    (tau2, stratc, tt_rsw, ssrd) starts at zero and persists between steps.

Stores the input state, the boundary fields in the order of sml_dyn_set_physics
(speedy_ml_amd.dynamics.PHYS_BC), the state after stepone and after the 24
leapfrog steps (both time levels).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_dyn_golden import DELT, IL, IX, KX, MX, NX, ROB, WIL, Ref, _dbl, _int, _p, spectral_field  # noqa: E402

SEED = 20250401
TYEAR = 0.2
NGP = IX * IL
NSTRAD = 3
ALPH = 0.5
PHYS_BC = ("fmask1", "phis0", "stl_am", "sst_am", "soilw_am", "alb_l", "alb_s", "albsfc", "snowc",
           "fsol", "ozone", "ozupp", "zenit", "stratz", "forog")


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

    vor = R.var("mod_dynvar", "vor", (MX, NX, KX, 2), np.complex128)
    div = R.var("mod_dynvar", "div", (MX, NX, KX, 2), np.complex128)
    t = R.var("mod_dynvar", "t", (MX, NX, KX, 2), np.complex128)
    ps = R.var("mod_dynvar", "ps", (MX, NX, 2), np.complex128)
    tr = R.var("mod_dynvar", "tr", (MX, NX, KX, 2, 1), np.complex128)
    phis = R.var("mod_dynvar", "phis", (MX, NX), np.complex128)
    tcorh = R.var("mod_hdifcon", "tcorh", (MX, NX), np.complex128)
    qcorh = R.var("mod_hdifcon", "qcorh", (MX, NX), np.complex128)

    # --- atmosphere: both levels (a leapfrog pair), moist lower levels
    rgam = (2.0 / 7.0) * 1004.0 * 6.0 / (1000.0 * 9.81)
    tref = 288.0 * np.maximum(0.2, fsg) ** rgam
    for k in range(KX):
        vor[:, :, k, 0] = spectral_field(rng, 6e-6, 1.5)
        div[:, :, k, 0] = spectral_field(rng, 6e-7, 1.5)
        t[:, :, k, 0] = spectral_field(rng, 2.0, 1.0, mean=tref[k])
        qm = 12.0 * fsg[k] ** 3
        tr[:, :, k, 0, 0] = spectral_field(rng, 0.2 * qm, 1.5, mean=qm)
    ps[:, :, 0] = spectral_field(rng, 0.02, 1.5)
    for arr, amp in ((vor, 2e-8), (div, 2e-9), (t, 2e-3)):
        for k in range(KX):
            arr[:, :, k, 1] = arr[:, :, k, 0] + spectral_field(rng, amp, 1.0)
    for k in range(KX):
        tr[:, :, k, 1, 0] = tr[:, :, k, 0, 0] + spectral_field(rng, 2e-4, 1.0)
    ps[:, :, 1] = ps[:, :, 0] + spectral_field(rng, 2e-5, 1.5)
    phis[...] = spectral_field(rng, 2000.0, 1.5, mean=3000.0)
    tcorh[...] = spectral_field(rng, 1.0, 1.5)
    qcorh[...] = spectral_field(rng, 0.1, 1.5)

    # --- surface / boundary fields
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
    bc["forog"] = R.var("mod_sflcon", "forog", (NGP,)).copy()
    for k in ("fsol", "ozone", "ozupp", "zenit", "stratz"):
        bc[k] = R.var("mod_radcon", k, (NGP,)).copy()

    def snap():
        return {"vor": vor.transpose(3, 2, 1, 0).copy(), "div": div.transpose(3, 2, 1, 0).copy(),
                "t": t.transpose(3, 2, 1, 0).copy(), "tr": tr[..., 0].transpose(3, 2, 1, 0).copy(),
                "ps": ps.transpose(2, 1, 0).copy()}

    out = {f"in_{k}": v for k, v in snap().items()}
    out.update(phis=phis.T.copy(), tcorh=tcorh.T.copy(), qcorh=qcorh.T.copy(),
               bc=np.stack([np.asarray(bc[k], dtype=np.float64).ravel() for k in PHYS_BC]),
               tyear=np.float64(TYEAR), delt=np.float64(DELT), alph=np.float64(ALPH))
    # --- stepone (ini_stepone.f90:19-34), lradsw as mod_lflags initialises it
    R.scalar_logical("mod_lflags", "lradsw", True)
    L.impint_(_dbl(0.5 * DELT), _dbl(ALPH))
    L.step_(_int(1), _int(1), _dbl(0.5 * DELT), _dbl(ALPH), _dbl(ROB), _dbl(WIL))
    L.impint_(_dbl(DELT), _dbl(ALPH))
    L.step_(_int(1), _int(2), _dbl(DELT), _dbl(ALPH), _dbl(ROB), _dbl(WIL))
    L.impint_(_dbl(2 * DELT), _dbl(ALPH))
    out.update({f"stepone_{k}": v for k, v in snap().items()})
    # --- stloop's 6-h block (dyn_stloop.f90:26-60): istep = 1..24
    for istep in range(1, 25):
        R.scalar_logical("mod_lflags", "lradsw", istep % NSTRAD == 1)
        L.step_(_int(2), _int(2), _dbl(2 * DELT), _dbl(ALPH), _dbl(ROB), _dbl(WIL))
    out.update({f"window_{k}": v for k, v in snap().items()})
    for k in ("vor", "div", "t", "tr", "ps"):
        assert np.all(np.isfinite(out[f"window_{k}"])), k
    tg = R.var("mod_dynvar", "t", (MX, NX, KX, 2), np.complex128)
    print("window done: T(0,0) levels", np.real(tg[0, 0, :, 0]) / np.sqrt(2.0))
    path = os.path.join(HERE, "window_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

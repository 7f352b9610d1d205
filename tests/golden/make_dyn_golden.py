"""Generate tests/golden/dyn_ref.npz from the reference's own dynamical core.

Run in the survey/build container (needs /root/reference and flang):

    make -C oracle ref          # builds oracle/_ref/libspeedy_ref_dyn.so
    python tests/golden/make_dyn_golden.py

The library is the reference's dyn_step/grtend/sptend/implic/geop, indyns/impint,
phypar and its physics, compiled as-is (oracle/Makefile).  This script drives it
through its own module state (flang symbols `_QM<module>E<name>`):

 1. initialisation as ini_atm does it (ini_iniatm.f90:19-33): inifft, indyns,
    inphys(hsg, ppl, radang), radset, sflset(phis0) (ini_fordate.f90:44-45);
 2. a seeded synthetic atmosphere: smooth random spectral vor/div/t/ps/q on the
    T30 triangle around the reference temperature profile, synthetic orography
    phis (+ phis0 = its grid image) and synthetic surface forcing (sst_am, stl_am,
    soilw_am, fmask1, albedos).  Shortwave radiation is off (lradsw = .false.), so
    the physics depends only on the state;
 3. the physics tendencies of that state: geop(1) then phypar with zero input
    tendencies (dyn_grtend.f90:223-226) -> P = (utend, vtend, ttend, qtend) on the
    grid.  grtend always evaluates the physics on time level 1 (dyn_step.f90:45),
    so P is the same for every step case below;
 4. reference `step` for the cases of stepone/stloop (ini_stepone.f90:19-34,
    dyn_stloop.f90:43), each from the same input state after impint(dt, alph):
        fwd    step(1,1, delt/2, 0.5)    forward half step
        lf0    step(1,2, delt,   0.5)    first leapfrog
        lf     step(2,2, 2 delt, 0.5)    leapfrog + Robert-Williams filter
        expl   step(1,1, delt/2, 0.0)    explicit gravity waves (sptend on j2)
    and records the updated prognostic fields (and phi = geop(j4) for lf).

The step's own physics call adds the same terms one by one to the dynamical
tendencies; the build adds P once, so parity with these outputs is to rounding
(tolerance stated in the tests), not bit-exact.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DYN = os.path.join(REPO, "oracle", "_ref", "libspeedy_ref_dyn.so")
SEED = 20250301
MX, NX, KX, IX, IL = 31, 32, 8, 96, 48
DELT = 86400.0 / 96  # mod_tsteps.f90: nsteps = 96
ROB, WIL = 0.05, 0.53


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _dbl(v):
    return ctypes.byref(ctypes.c_double(v))


def _int(v):
    return ctypes.byref(ctypes.c_int(v))


class Ref:
    def __init__(self):
        if not os.path.exists(REF_DYN):
            raise SystemExit("build the reference first: make -C oracle ref")
        self.L = ctypes.CDLL(REF_DYN)

    def var(self, module, name, shape, dtype=np.float64):
        """numpy view on a module array (Fortran order, as declared)."""
        addr = ctypes.addressof(ctypes.c_char.in_dll(self.L, f"_QM{module}E{name}"))
        count = int(np.prod(shape))
        buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(addr)
        return np.frombuffer(buf, dtype=dtype).reshape(shape, order="F")

    def scalar_logical(self, module, name, value):
        ctypes.c_int32.in_dll(self.L, f"_QM{module}E{name}").value = int(value)


def spectral_field(rng, amp, power, mean=0.0):
    """complex (mx, nx) coefficients on the T30 triangle (m + n <= 30), decaying
    as (1 + m + n)^-power; m = 0 imaginary parts zero (a real grid field)."""
    c = np.zeros((MX, NX), np.complex128)
    m = np.arange(MX)[:, None]
    n = np.arange(NX)[None, :]
    ll = m + n
    mask = ll <= 30
    a = amp * (1.0 + ll) ** (-power)
    c[mask] = (rng.standard_normal(mask.sum()) + 1j * rng.standard_normal(mask.sum())) * a[mask]
    c[0, :] = c[0, :].real
    c[0, 0] = mean * np.sqrt(2.0)  # P_00 = sqrt(1/2)
    return c


def main():
    R = Ref()
    L = R.L
    rng = np.random.default_rng(SEED)
    # 1. initialisation
    L.inifft_()
    L.indyns_()
    hsg = R.var("mod_dyncon1", "hsg", (KX + 1,))
    fsg = R.var("mod_dyncon1", "fsg", (KX,))
    radang = R.var("mod_dyncon1", "radang", (IL,))
    ppl = np.ascontiguousarray(fsg.copy())
    L.inphys_(_p(hsg), _p(ppl), _p(radang))
    L.radset_()
    R.scalar_logical("mod_lflags", "lradsw", False)

    # 2. synthetic atmosphere + forcing
    rgas = (2.0 / 7.0) * 1004.0
    rgam = rgas * 6.0 / (1000.0 * 9.81)
    tref = 288.0 * np.maximum(0.2, fsg) ** rgam
    vor = R.var("mod_dynvar", "vor", (MX, NX, KX, 2), np.complex128)
    div = R.var("mod_dynvar", "div", (MX, NX, KX, 2), np.complex128)
    t = R.var("mod_dynvar", "t", (MX, NX, KX, 2), np.complex128)
    ps = R.var("mod_dynvar", "ps", (MX, NX, 2), np.complex128)
    tr = R.var("mod_dynvar", "tr", (MX, NX, KX, 2, 1), np.complex128)
    phi = R.var("mod_dynvar", "phi", (MX, NX, KX), np.complex128)
    phis = R.var("mod_dynvar", "phis", (MX, NX), np.complex128)
    tcorh = R.var("mod_hdifcon", "tcorh", (MX, NX), np.complex128)
    qcorh = R.var("mod_hdifcon", "qcorh", (MX, NX), np.complex128)
    s_vor = np.zeros((2, KX, NX, MX), np.complex128)
    s_div = np.zeros_like(s_vor)
    s_t = np.zeros_like(s_vor)
    s_tr = np.zeros_like(s_vor)
    s_ps = np.zeros((2, NX, MX), np.complex128)
    for k in range(KX):
        s_vor[0, k] = spectral_field(rng, 2e-5, 1.0).T
        s_div[0, k] = spectral_field(rng, 2e-6, 1.0).T
        s_t[0, k] = spectral_field(rng, 2.0, 1.0, mean=tref[k]).T
        qm = 12.0 * fsg[k] ** 3
        s_tr[0, k] = spectral_field(rng, 0.2 * qm, 1.5, mean=qm).T
    s_ps[0] = spectral_field(rng, 0.02, 1.5).T
    # level 2 = level 1 + a small perturbation (a leapfrog pair)
    for arr, amp in ((s_vor, 2e-8), (s_div, 2e-9), (s_t, 2e-3), (s_tr, 2e-4)):
        for k in range(KX):
            arr[1, k] = arr[0, k] + spectral_field(rng, amp, 1.0).T
    s_ps[1] = s_ps[0] + spectral_field(rng, 2e-5, 1.5).T
    f_phis = spectral_field(rng, 2000.0, 1.5, mean=3000.0).T
    f_tcorh = spectral_field(rng, 1.0, 1.5).T
    f_qcorh = spectral_field(rng, 0.1, 1.5).T

    ngp = IX * IL
    lat = np.repeat(radang, IX)
    lon = np.tile(np.arange(IX) * 2 * np.pi / IX, IL)
    sst = 271.0 + 30.0 * np.cos(lat) ** 2 + 0.5 * rng.standard_normal(ngp)
    stl = 265.0 + 30.0 * np.cos(lat) ** 2 + 1.0 * rng.standard_normal(ngp)
    fmask1 = np.clip(0.5 + 0.6 * np.sin(2 * lon) * np.cos(3 * lat), 0.0, 1.0)
    surf = dict(sst=sst, stl=stl, fmask1=fmask1)

    def load_state():
        vor[...] = s_vor.transpose(3, 2, 1, 0)
        div[...] = s_div.transpose(3, 2, 1, 0)
        t[...] = s_t.transpose(3, 2, 1, 0)
        tr[..., 0] = s_tr.transpose(3, 2, 1, 0)
        ps[...] = s_ps.transpose(2, 1, 0)
        phis[...] = f_phis.T
        tcorh[...] = f_tcorh.T
        qcorh[...] = f_qcorh.T

    load_state()
    # phis0 = grid image of phis (ini_inbcon.f90:38-44 builds phis from phi0 likewise)
    phis0 = R.var("mod_surfcon", "phis0", (IX, IL))
    g = np.zeros((IL, IX))
    L.grid_(_p(np.ascontiguousarray(f_phis).view(np.float64)), _p(g), _int(1))
    phis0[...] = g.T
    R.var("mod_surfcon", "fmask1", (IX, IL))[...] = fmask1.reshape(IL, IX).T
    L.sflset_(_p(np.ascontiguousarray(g)))
    R.var("mod_var_sea", "sst_am", (ngp,))[...] = sst
    R.var("mod_var_sea", "ssti_om", (ngp,))[...] = sst
    R.var("mod_var_land", "stl_am", (ngp,))[...] = stl
    R.var("mod_var_land", "soilw_am", (ngp,))[...] = 0.4
    R.var("mod_radcon", "alb_l", (ngp,))[...] = 0.25
    R.var("mod_radcon", "alb_s", (ngp,))[...] = 0.07
    R.var("mod_radcon", "snowc", (ngp,))[...] = 0.0

    # 3. physics tendencies of level 1 (twice: the second must repeat the first)
    def physics():
        load_state()
        L.geop_(_int(1))
        tend = [np.zeros((KX, IL, IX)) for _ in range(4)]
        L.phypar_(_p(vor), _p(div), _p(t), _p(tr), _p(phi), _p(ps), *[_p(x) for x in tend])
        return np.stack(tend)

    phys = physics()
    phys2 = physics()
    assert np.array_equal(phys, phys2), "reference physics is not repeatable"
    assert np.all(np.isfinite(phys))

    out = dict(vor=s_vor, div=s_div, t=s_t, tr=s_tr, ps=s_ps, phis=f_phis, tcorh=f_tcorh, qcorh=f_qcorh,
               phys=phys, delt=np.float64(DELT), rob=np.float64(ROB), wil=np.float64(WIL), **surf)
    cases = {"fwd": (1, 1, 0.5 * DELT, 0.5), "lf0": (1, 2, DELT, 0.5), "lf": (2, 2, 2 * DELT, 0.5),
             "expl": (1, 1, 0.5 * DELT, 0.0)}
    for name, (j1, j2, dt, alph) in cases.items():
        load_state()
        L.impint_(_dbl(dt), _dbl(alph))
        L.step_(_int(j1), _int(j2), _dbl(dt), _dbl(alph), _dbl(ROB), _dbl(WIL))
        res = {
            "vor": vor.transpose(3, 2, 1, 0).copy(),
            "div": div.transpose(3, 2, 1, 0).copy(),
            "t": t.transpose(3, 2, 1, 0).copy(),
            "tr": tr[..., 0].transpose(3, 2, 1, 0).copy(),
            "ps": ps.transpose(2, 1, 0).copy(),
        }
        # eps = 0 when j1 = 1: level 1 is returned unchanged, store only level 2
        levels = (0, 1) if j1 == 2 else (1,)
        if j1 == 1:
            for f in ("vor", "div", "t", "tr", "ps"):
                src = {"vor": s_vor, "div": s_div, "t": s_t, "tr": s_tr, "ps": s_ps}[f]
                assert np.array_equal(res[f][0], src[0]), f"{name}: level 1 of {f} changed"
        for f, a in res.items():
            out[f"{name}_{f}"] = a[list(levels)]
        out[f"{name}_case"] = np.array([j1, j2, dt, alph])
        if name == "lf":
            out["lf_phi"] = phi.transpose(2, 1, 0).copy()
    path = os.path.join(HERE, "dyn_ref.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()

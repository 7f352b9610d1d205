"""SPEEDY's spectral dynamical core on the GPU (libspeedyml sml_dyn_*).

Mirrors the reference's time-stepping interface: `impint(dt, alph)`
(src/ini_impint.f90:1-153) and `step(j1, j2, dt, alph, rob, wil)`
(src/dyn_step.f90:1-128) acting on the prognostic state of mod_dynvar
(vor, div, t, ps, tr; src/mod_dynvar.f90:15-27), with `stepone`'s start-up
sequence (src/ini_stepone.f90:19-34) and the leapfrog loop (src/dyn_stloop.f90:43)
as conveniences.  Physics (phypar, src/phy_phypar.f90) runs on the GPU once the
boundary fields are given (`set_physics`); otherwise its grid-point tendencies
(u, v, t, q) can be handed to each step, or are zero.

State arrays (numpy complex128, C order == the reference's Fortran layout):
vor/div/t/tr (2, kx=8, nx=32, mx=31), ps (2, 32, 31); forcing phis/tcorh/qcorh
(32, 31).  Physics tendencies: float64 (4, 8, 48, 96).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr, stream_ptr

EARTH_RADIUS = 6.371e6  # mod_dyncon1.f90 rearth
KX, NX, MX = 8, 32, 31
FIELDS = ("vor", "div", "t", "tr", "ps")
NSTEPS = 96  # mod_tsteps.f90: nsteps per day
NGP = 96 * 48
# phypar's boundary fields, in the order of sml_dyn_set_physics (include/speedy_ml.h)
PHYS_BC = ("fmask1", "phis0", "stl_am", "sst_am", "soilw_am", "alb_l", "alb_s", "albsfc", "snowc",
           "fsol", "ozone", "ozupp", "zenit", "stratz", "forog")
# fordate's surface fields and the coupler's monthly climatologies (sml_dyn_set_surface,
# sml_dyn_set_climatology)
SURFACE = ("fmask_l", "fmask_s", "alb0")
CLIMATOLOGY = ("stl12", "snowd12", "soilw12", "sst12", "sice12")
RAD_SIZE = (4 * KX + 2 + KX + 1) * NGP
DELT = 86400.0 / NSTEPS
ROB, WIL, ALPH = 0.05, 0.53, 0.5  # mod_tsteps.f90:90,93; ini_indyns.f90 alph


def _c128(a, shape):
    a = np.ascontiguousarray(a, dtype=np.complex128)
    if a.shape != shape:
        raise ValueError(f"expected shape {shape}, got {a.shape}")
    return a


class Dynamics:
    def __init__(self, radius: float = EARTH_RADIUS):
        h = ctypes.c_void_p()
        check(lib().sml_dyn_create(radius, ctypes.byref(h)))
        self._h = h
        self._dtal = None

    def close(self):
        if self._h:
            lib().sml_dyn_destroy(self._h)
            self._h = None

    __del__ = close

    def set_fused(self, fused: bool):
        """The fused step (default; FMA-contracted transforms, 2 launches per step) or
        the unfused 8/9-launch step with FFTPACK-exact transforms (sml_dyn_set_fused)."""
        check(lib().sml_dyn_set_fused(self._h, int(bool(fused))))

    def impint(self, dt: float, alph: float = ALPH):
        check(lib().sml_dyn_impint(self._h, dt, alph))
        self._dtal = (dt, alph)

    def set_forcing(self, phis=None, tcorh=None, qcorh=None):
        args = [None if a is None else _c128(a, (NX, MX)) for a in (phis, tcorh, qcorh)]
        check(lib().sml_dyn_set_forcing(self._h, *[ptr(a) for a in args]))

    def set_state(self, state):
        a = {f: _c128(state[f], (2, KX, NX, MX) if f != "ps" else (2, NX, MX)) for f in FIELDS}
        check(lib().sml_dyn_set_state(self._h, ptr(a["vor"]), ptr(a["div"]), ptr(a["t"]), ptr(a["ps"]),
                                      ptr(a["tr"])))

    def get_state(self):
        out = {f: np.zeros((2, KX, NX, MX) if f != "ps" else (2, NX, MX), np.complex128) for f in FIELDS}
        check(lib().sml_dyn_get_state(self._h, ptr(out["vor"]), ptr(out["div"]), ptr(out["t"]), ptr(out["ps"]),
                                      ptr(out["tr"])))
        return out

    def get_phi(self):
        phi = np.zeros((KX, NX, MX), np.complex128)
        check(lib().sml_dyn_get_phi(self._h, ptr(phi)))
        return phi

    def get_tendencies(self):
        tend = np.zeros((4 * KX + 1, NX, MX), np.complex128)
        check(lib().sml_dyn_get_tendencies(self._h, ptr(tend)))
        return tend

    def device_buffers(self):
        """(state, phys) device addresses: [vor|div|t|tr|ps] and a phys scratch buffer."""
        s, p = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().sml_dyn_state_device(self._h, ctypes.byref(s), ctypes.byref(p)))
        return s.value, p.value

    # ------------------------------------------------------------- physics
    def set_physics(self, bc):
        """Boundary fields of phypar (dict of PHYS_BC arrays of 96*48 values, or a
        (15, 4608) array in that order); None switches the GPU physics off."""
        if bc is None:
            check(lib().sml_dyn_set_physics(self._h, None))
            return
        if isinstance(bc, dict):
            bc = np.stack([np.asarray(bc[k], dtype=np.float64).ravel() for k in PHYS_BC])
        a = np.ascontiguousarray(bc, dtype=np.float64)
        if a.size != len(PHYS_BC) * NGP:
            raise ValueError("bc must hold 15 x 4608 values")
        check(lib().sml_dyn_set_physics(self._h, ptr(a)))

    def set_clock(self, istep: int, lradsw: bool):
        check(lib().sml_dyn_set_clock(self._h, int(istep), int(bool(lradsw))))

    def get_clock(self):
        i, r = ctypes.c_int(), ctypes.c_int()
        check(lib().sml_dyn_get_clock(self._h, ctypes.byref(i), ctypes.byref(r)))
        return i.value, bool(r.value)

    def set_rad_state(self, rad=None):
        """Radiation state (tau2 (4, kx, ngp), stratc (2, ngp), tt_rsw (kx, ngp), ssrd
        (ngp,)) as a dict, or None = zero."""
        if rad is None:
            check(lib().sml_dyn_set_rad_state(self._h, None))
            return
        a = np.concatenate([np.asarray(rad[k], dtype=np.float64).ravel()
                            for k in ("tau2", "stratc", "tt_rsw", "ssrd")])
        assert a.size == RAD_SIZE
        check(lib().sml_dyn_set_rad_state(self._h, ptr(a)))

    def get_rad_state(self):
        a = np.zeros(RAD_SIZE)
        check(lib().sml_dyn_get_rad_state(self._h, ptr(a)))
        o = np.cumsum([0, 4 * KX * NGP, 2 * NGP, KX * NGP, NGP])
        return {"tau2": a[o[0]:o[1]].reshape(4, KX, NGP), "stratc": a[o[1]:o[2]].reshape(2, NGP),
                "tt_rsw": a[o[2]:o[3]].reshape(KX, NGP), "ssrd": a[o[3]:o[4]]}

    def phypar(self, ug1, vg1, tg1, qg1, phig1, pslg1, lradsw):
        """phypar alone on host grid inputs (kx, ngp) / (ngp,): returns the physics
        tendencies (4, kx, ngp) = u, v, t, q; updates the radiation state."""
        f = [np.ascontiguousarray(x, dtype=np.float64) for x in (ug1, vg1, tg1, qg1, phig1, pslg1)]
        for x in f[:5]:
            assert x.size == KX * NGP
        assert f[5].size == NGP
        tend = np.zeros((4, KX, NGP))
        check(lib().sml_dyn_phypar_host(self._h, *[ptr(x) for x in f], int(bool(lradsw)), ptr(tend)))
        return tend

    # ---------------------------------------------------- date-driven forcing
    def set_surface(self, surf):
        """fordate's surface fields: dict fmask_l, fmask_s, alb0 (or a (3, 4608) array
        in that order), as inbcon leaves them (ini_inbcon.f90:38-70, 140-156)."""
        if isinstance(surf, dict):
            surf = np.stack([np.asarray(surf[k], dtype=np.float64).ravel() for k in SURFACE])
        a = np.ascontiguousarray(surf, dtype=np.float64)
        if a.size != len(SURFACE) * NGP:
            raise ValueError("surface must hold 3 x 4608 values")
        check(lib().sml_dyn_set_surface(self._h, ptr(a)))

    def set_climatology(self, clim):
        """Monthly climatologies: dict of CLIMATOLOGY arrays (12, 4608) (January
        first), or a (5, 12, 4608) array; None keeps the coupler fields as set."""
        if clim is None:
            check(lib().sml_dyn_set_climatology(self._h, None))
            return
        if isinstance(clim, dict):
            clim = np.stack([np.asarray(clim[k], dtype=np.float64).reshape(12, NGP) for k in CLIMATOLOGY])
        a = np.ascontiguousarray(clim, dtype=np.float64)
        if a.size != len(CLIMATOLOGY) * 12 * NGP:
            raise ValueError("climatology must hold 5 x 12 x 4608 values")
        check(lib().sml_dyn_set_climatology(self._h, ptr(a)))

    def fordate(self, iyear: int, imonth: int, iday: int, force: bool = False, stream=None):
        """agcm_init's forcing of a window at that date (coupler, hybrid SST, fordate;
        ini_agcm_init.f90:57-89), asynchronous on `stream`; skipped when nothing changed."""
        check(lib().sml_dyn_fordate_ex(self._h, int(iyear), int(imonth), int(iday), int(bool(force)),
                                       stream_ptr(stream)))

    def fordate_count(self) -> int:
        c = ctypes.c_int()
        check(lib().sml_dyn_fordate_count(self._h, ctypes.byref(c)))
        return c.value

    def get_physics(self):
        """The boundary fields phypar reads, dict of PHYS_BC arrays (4608,)."""
        a = np.zeros((len(PHYS_BC), NGP))
        check(lib().sml_dyn_get_physics(self._h, ptr(a)))
        return dict(zip(PHYS_BC, a))

    def get_forcing(self):
        """(phis, tcorh, qcorh) complex (32, 31) as the next window reads them."""
        out = [np.zeros((NX, MX), np.complex128) for _ in range(3)]
        check(lib().sml_dyn_get_forcing(self._h, *[ptr(o) for o in out]))
        return dict(zip(("phis", "tcorh", "qcorh"), out))

    def get_sea_ice(self):
        sice, tice = np.zeros(NGP), np.zeros(NGP)
        check(lib().sml_dyn_get_sea_ice(self._h, ptr(sice), ptr(tice)))
        return sice, tice

    def sol_oz(self, tyear: float):
        """sol_oz(tyear): dict fsol, ozone, ozupp, zenit, stratz (ngp,)."""
        out = np.zeros((5, NGP))
        check(lib().sml_dyn_sol_oz(self._h, float(tyear), ptr(out)))
        return dict(zip(("fsol", "ozone", "ozupp", "zenit", "stratz"), out))

    @staticmethod
    def sflset(phi0):
        phi0 = np.ascontiguousarray(phi0, dtype=np.float64).ravel()
        assert phi0.size == NGP
        forog = np.zeros(NGP)
        check(lib().sml_phys_sflset(ptr(phi0), ptr(forog)))
        return forog

    def step(self, j1, j2, dt, alph=ALPH, rob=ROB, wil=WIL, phys=None, stream=None):
        """step(j1, j2, dt, alph, rob, wil).  `phys`: host numpy (4, 8, 48, 96)
        (synchronous), a float64 CUDA tensor of that shape or None (asynchronous on
        `stream`).  impint(dt, alph) is selected when (dt, alph) differs from the
        last call (the reference calls it explicitly, ini_stepone.f90:21-34); the
        library caches the tables of up to 4 (dt, alph) pairs on the device."""
        if self._dtal != (dt, alph):
            self.impint(dt, alph)
        if isinstance(phys, np.ndarray):  # host tendencies: synchronous H2D + step
            ph = np.ascontiguousarray(phys, dtype=np.float64)
            if ph.shape != (4, KX, 48, 96):
                raise ValueError("phys must be (4, 8, 48, 96)")
            check(lib().sml_dyn_step_host(self._h, j1, j2, dt, alph, rob, wil, ptr(ph)))
            return
        if phys is not None and not (phys.is_cuda and phys.is_contiguous() and phys.numel() == 4 * KX * 4608):
            raise ValueError("phys must be a contiguous float64 CUDA tensor (4, 8, 48, 96)")
        check(lib().sml_dyn_step(self._h, j1, j2, dt, alph, rob, wil, ptr(phys), stream_ptr(stream)))

    def from_grid(self, grid4d, logp, stream=None):
        """iogrid(30) (ppo_iogrid.f90:497-571): window entry from variables3d
        (4, 96, 48, 8) Fortran order == C (8, 48, 96, 4), and logp (48, 96).
        Host numpy -> synchronous, returns (minmax[8], is_safe); device tensors ->
        asynchronous, returns None (min/max left on the device)."""
        if isinstance(grid4d, np.ndarray):
            g = np.ascontiguousarray(grid4d, dtype=np.float64)
            lp = np.ascontiguousarray(logp, dtype=np.float64)
            if g.size != 4 * KX * 4608 or lp.size != 4608:
                raise ValueError("grid4d must hold 4*96*48*8 values and logp 96*48")
            mm = np.zeros(8)
            safe = ctypes.c_int(0)
            check(lib().sml_dyn_from_grid_host(self._h, ptr(g), ptr(lp), ptr(mm), ctypes.byref(safe)))
            return mm, bool(safe.value)
        check(lib().sml_dyn_from_grid(self._h, ptr(grid4d), ptr(logp), None, stream_ptr(stream)))
        return None

    def to_grid(self, grid4d=None, logp=None, stream=None):
        """iogrid(31) (ppo_iogrid.f90:573-595): level 1 -> (grid4d, logp).  With
        device tensors given, fills them asynchronously; else returns host arrays."""
        if grid4d is not None:
            check(lib().sml_dyn_to_grid(self._h, ptr(grid4d), ptr(logp), stream_ptr(stream)))
            return grid4d, logp
        g = np.zeros((KX, 48, 96, 4))
        lp = np.zeros((48, 96))
        check(lib().sml_dyn_to_grid_host(self._h, ptr(g), ptr(lp)))
        return g, lp

    def run_model(self, grid4d, logp, fc4d, fc2d, nleap: int = 24, delt: float = DELT, alph: float = ALPH,
                  stream=None):
        """run_model (mpires.f90:1516-1628) on device tensors, asynchronous: iogrid(30)
        + safety check, the window, iogrid(31) into (fc4d, fc2d), q floored at 1e-6;
        an unsafe entry state returns the input grid (q floored) as agcm_main skips
        the integration.  `last_safe()` gives the check's outcome."""
        check(lib().sml_dyn_run_model(self._h, ptr(grid4d), ptr(logp), nleap, delt, alph, ROB, WIL, ptr(fc4d),
                                      ptr(fc2d), stream_ptr(stream)))
        self._dtal = (2 * delt, alph)

    def last_safe(self):
        """(is_safe_to_run_speedy, minmax[8]) of the last from_grid / run_model."""
        safe = ctypes.c_int()
        mm = np.zeros(8)
        check(lib().sml_dyn_last_safe(self._h, ctypes.byref(safe), ptr(mm)))
        return bool(safe.value), mm

    def stepone(self, delt: float = DELT, alph: float = ALPH, phys=None, stream=None):
        """ini_stepone.f90:19-34 for istart = 0 / 2: forward half step, first leapfrog."""
        self.step(1, 1, 0.5 * delt, alph, phys=phys, stream=stream)
        self.step(1, 2, delt, alph, phys=phys, stream=stream)
        self.impint(2 * delt, alph)

    def window(self, nleap: int = 24, delt: float = DELT, alph: float = ALPH, stream=None, graph: bool = True):
        """One 6-h SPEEDY window after iogrid(30): stepone + nleap x step(2, 2)
        (dyn_stloop.f90:37-59 with window_size 4), asynchronous.  With the GPU
        physics on, stepone uses the lradsw the previous window left (the module
        flag persists) and stloop restarts at istep = 1 (at_gcm.f90:81, jday = 1)."""
        if graph:  # the whole window as one captured hipGraph (sml_dyn_window)
            check(lib().sml_dyn_window(self._h, nleap, delt, alph, ROB, WIL, stream_ptr(stream)))
            self._dtal = (2 * delt, alph)
            return
        self.stepone(delt, alph, stream=stream)
        _, lradsw = self.get_clock()
        self.set_clock(1, lradsw)
        self.leapfrog(nleap, delt, alph, stream=stream, graph=False)

    def leapfrog(self, nsteps: int, delt: float = DELT, alph: float = ALPH, phys=None, stream=None,
                 graph: bool = True):
        """dyn_stloop.f90:43: nsteps x step(2, 2, 2 delt), asynchronous on `stream`.
        graph=True replays one captured hipGraph per step (sml_dyn_leapfrog);
        phys: None or a device tensor held fixed over the steps."""
        if self._dtal != (2 * delt, alph):
            self.impint(2 * delt, alph)
        if graph:
            check(lib().sml_dyn_leapfrog(self._h, nsteps, 2 * delt, alph, ROB, WIL, ptr(phys), stream_ptr(stream)))
            return
        for _ in range(nsteps):  # stloop's clock, launched step by step
            istep, _ = self.get_clock()
            self.set_clock(istep, istep % 3 == 1)
            check(lib().sml_dyn_step(self._h, 2, 2, 2 * delt, alph, ROB, WIL, ptr(phys), stream_ptr(stream)))
            self.set_clock(istep + 1, istep % 3 == 1)

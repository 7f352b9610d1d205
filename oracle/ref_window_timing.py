"""TEST / BASELINE INFRASTRUCTURE ONLY: the reference's own SPEEDY window on one host
core, timed -- the window leg of bench.py's cpu_baseline.

Runs oracle/_ref/libspeedy_ref_dyn.so (the reference's dyn_* / ini_* / phy_* /
spe_* sources compiled as-is by `make -C oracle ref`, built in the build container;
the library travels to the GPU box like the product's own .so files) through the
window run_model integrates (src/mpires.f90:1516-1628):

  iogrid(30)  (src/ppo_iogrid.f90:497-577): real(4) copies, q < 0 -> 0, vdspec /
              spec / trunct per level, the re-grid uvspec / grid of the check and
              its min / max -- the reference's own grid_ / spec_ / vdspec_ /
              uvspec_ / trunct_ called in ppo_iogrid's order (ppo_iogrid.f90 itself
              needs mpires / MPI and is not built);
  stepone     (src/ini_stepone.f90:19-34): impint + step(1,1,delt/2), impint +
              step(1,2,delt), impint(2 delt);
  stloop      (src/dyn_stloop.f90:26-60): 24 x step(2,2,2 delt), lradsw =
              mod(istep, 3) == 1;
  iogrid(31)  (:579-601): uvspec / grid of level 1.

State, forcing and boundary fields are seeded synthetic ones (as
tests/golden/make_window_golden.py builds them).  The reference prints from
phypar every step; that output goes to /dev/null but its cost stays in the time,
as in the reference.

    python oracle/ref_window_timing.py [windows]   -> one JSON line on stdout
"""
from __future__ import annotations

import ctypes
import json
import os
import resource
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DYN = os.path.join(HERE, "_ref", "libspeedy_ref_dyn.so")
MX, NX, KX, IX, IL = 31, 32, 8, 96, 48
NGP = IX * IL
DELT = 86400.0 / 96
ROB, WIL, ALPH = 0.05, 0.53, 0.5


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _d(v):
    return ctypes.byref(ctypes.c_double(v))


def _i(v):
    return ctypes.byref(ctypes.c_int(v))


def field(rng, amp, power, mean=0.0):
    c = np.zeros((MX, NX), np.complex128)
    m = np.arange(MX)[:, None]
    n = np.arange(NX)[None, :]
    ll = m + n
    mask = ll <= 30
    a = amp * (1.0 + ll) ** (-power)
    c[mask] = (rng.standard_normal(mask.sum()) + 1j * rng.standard_normal(mask.sum())) * a[mask]
    c[0, :] = c[0, :].real
    c[0, 0] = mean * np.sqrt(2.0)
    return c


def main():
    nwin = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    soft, hard = resource.getrlimit(resource.RLIMIT_STACK)
    resource.setrlimit(resource.RLIMIT_STACK, (hard, hard))  # the reference's automatic arrays
    L = ctypes.CDLL(REF_DYN)

    def var(module, name, shape, dtype=np.float64):
        addr = ctypes.addressof(ctypes.c_char.in_dll(L, f"_QM{module}E{name}"))
        buf = (ctypes.c_char * (int(np.prod(shape)) * np.dtype(dtype).itemsize)).from_address(addr)
        return np.frombuffer(buf, dtype=dtype).reshape(shape, order="F")

    def logical(module, name, value):
        ctypes.c_int32.in_dll(L, f"_QM{module}E{name}").value = int(value)

    # silence the reference's per-step prints (fd 1 -> /dev/null for the timed part)
    devnull = os.open(os.devnull, os.O_WRONLY)
    saved = os.dup(1)
    os.dup2(devnull, 1)
    rng = np.random.default_rng(20250501)
    L.inifft_()
    L.indyns_()
    hsg = var("mod_dyncon1", "hsg", (KX + 1,))
    fsg = var("mod_dyncon1", "fsg", (KX,))
    radang = var("mod_dyncon1", "radang", (IL,))
    ppl = np.ascontiguousarray(fsg.copy())
    L.inphys_(_p(hsg), _p(ppl), _p(radang))
    L.radset_()
    L.sol_oz_(_d(0.2))
    vor = var("mod_dynvar", "vor", (MX, NX, KX, 2), np.complex128)
    div = var("mod_dynvar", "div", (MX, NX, KX, 2), np.complex128)
    t = var("mod_dynvar", "t", (MX, NX, KX, 2), np.complex128)
    ps = var("mod_dynvar", "ps", (MX, NX, 2), np.complex128)
    tr = var("mod_dynvar", "tr", (MX, NX, KX, 2, 1), np.complex128)
    phi = var("mod_dynvar", "phi", (MX, NX, KX), np.complex128)
    phis = var("mod_dynvar", "phis", (MX, NX), np.complex128)
    rgam = (2.0 / 7.0) * 1004.0 * 6.0 / (1000.0 * 9.81)
    tref = 288.0 * np.maximum(0.2, fsg) ** rgam
    for k in range(KX):
        vor[:, :, k, 0] = field(rng, 6e-6, 1.5)
        div[:, :, k, 0] = field(rng, 6e-7, 1.5)
        t[:, :, k, 0] = field(rng, 2.0, 1.0, mean=tref[k])
        tr[:, :, k, 0, 0] = field(rng, 2.4 * fsg[k] ** 3, 1.5, mean=12.0 * fsg[k] ** 3)
    ps[:, :, 0] = field(rng, 0.02, 1.5)
    phis[...] = field(rng, 2000.0, 1.5, mean=3000.0)
    lat = np.repeat(radang, IX)
    lon = np.tile(np.arange(IX) * 2 * np.pi / IX, IL)
    fmask = np.clip(0.5 + 0.6 * np.sin(2 * lon) * np.cos(3 * lat), 0.0, 1.0)
    g = np.zeros((IL, IX))
    L.grid_(_p(np.ascontiguousarray(phis.T).view(np.float64)), _p(g), _i(1))
    var("mod_surfcon", "phis0", (IX, IL))[...] = g.T
    var("mod_surfcon", "fmask1", (IX, IL))[...] = fmask.reshape(IL, IX).T
    var("mod_var_sea", "sst_am", (NGP,))[...] = 271.0 + 30.0 * np.cos(lat) ** 2
    var("mod_var_sea", "ssti_om", (NGP,))[...] = 271.0 + 30.0 * np.cos(lat) ** 2
    var("mod_var_land", "stl_am", (NGP,))[...] = 265.0 + 30.0 * np.cos(lat) ** 2
    var("mod_var_land", "soilw_am", (NGP,))[...] = 0.4
    var("mod_radcon", "alb_l", (NGP,))[...] = 0.25
    var("mod_radcon", "alb_s", (NGP,))[...] = 0.07
    var("mod_radcon", "albsfc", (NGP,))[...] = 0.07 + fmask * 0.18
    var("mod_radcon", "snowc", (NGP,))[...] = 0.0
    L.sflset_(_p(np.ascontiguousarray(g)))

    # the window's input grid: iogrid(31) of the seeded state
    ug = np.zeros((KX, IL, IX))
    vg = np.zeros((KX, IL, IX))
    tg = np.zeros((KX, IL, IX))
    qg = np.zeros((KX, IL, IX))
    pg = np.zeros((IL, IX))
    uc = np.zeros((NX, MX), np.complex128)
    vc = np.zeros((NX, MX), np.complex128)

    def iogrid31():
        for k in range(KX):
            L.uvspec_(_p(vor[:, :, k, 0].T.copy()), _p(div[:, :, k, 0].T.copy()), _p(uc), _p(vc))
            L.grid_(_p(uc), _p(ug[k]), _i(2))
            L.grid_(_p(vc), _p(vg[k]), _i(2))
        for k in range(KX):
            L.grid_(_p(t[:, :, k, 0].T.copy()), _p(tg[k]), _i(1))
            L.grid_(_p(tr[:, :, k, 0, 0].T.copy()), _p(qg[k]), _i(1))
            L.grid_(_p(phi[:, :, k].T.copy()), _p(np.zeros((IL, IX))), _i(1))
        L.grid_(_p(ps[:, :, 0].T.copy()), _p(pg), _i(1))

    iogrid31()
    g4 = [a.copy() for a in (tg, ug, vg, qg)]
    g2 = pg.copy()
    sp = np.zeros((NX, MX), np.complex128)
    sp2 = np.zeros((NX, MX), np.complex128)

    def iogrid30():
        t4, u4, v4, q4 = (a.astype(np.float32).astype(np.float64) for a in g4)
        q4[q4 < 0.0] = 0.0
        p4 = g2.astype(np.float32).astype(np.float64)
        for k in range(KX):
            L.vdspec_(_p(u4[k]), _p(v4[k]), _p(sp), _p(sp2), _i(2))
            vor[:, :, k, 0] = sp.T
            div[:, :, k, 0] = sp2.T
            L.spec_(_p(t4[k]), _p(sp))
            t[:, :, k, 0] = sp.T
            L.spec_(_p(q4[k]), _p(sp))
            tr[:, :, k, 0, 0] = sp.T
            for a in (vor[:, :, k, 0], div[:, :, k, 0], t[:, :, k, 0], tr[:, :, k, 0, 0]):
                c = a.T.copy()
                L.trunct_(_p(c))
                a[...] = c.T
        L.spec_(_p(p4), _p(sp))
        L.trunct_(_p(sp))
        ps[:, :, 0] = sp.T
        iogrid31()  # the safety check's re-grid (:541-554) and its min / max
        return min(ug.min(), vg.min()), max(tg.max(), qg.max())

    times = []
    lradsw = True
    for _ in range(nwin):
        t0 = time.perf_counter()
        iogrid30()
        logical("mod_lflags", "lradsw", lradsw)
        L.impint_(_d(0.5 * DELT), _d(ALPH))
        L.step_(_i(1), _i(1), _d(0.5 * DELT), _d(ALPH), _d(ROB), _d(WIL))
        L.impint_(_d(DELT), _d(ALPH))
        L.step_(_i(1), _i(2), _d(DELT), _d(ALPH), _d(ROB), _d(WIL))
        L.impint_(_d(2 * DELT), _d(ALPH))
        for istep in range(1, 25):
            lradsw = istep % 3 == 1
            logical("mod_lflags", "lradsw", lradsw)
            L.step_(_i(2), _i(2), _d(2 * DELT), _d(ALPH), _d(ROB), _d(WIL))
        iogrid31()
        times.append(time.perf_counter() - t0)
    finite = bool(np.isfinite(tg).all())
    # fd 1 stays on /dev/null: the Fortran runtime flushes its buffered prints at exit
    line = json.dumps({"window_s": float(np.median(times)), "windows": nwin, "finite": finite,
                       "all_s": [round(x, 4) for x in times]})
    os.write(saved, (line + "\n").encode())


if __name__ == "__main__":
    main()

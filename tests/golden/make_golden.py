"""Generate the committed golden fixtures from the reference itself.

Run in the survey/build container (needs /root/reference and flang):

    make -C oracle ref          # builds oracle/_ref/libspeedy_ref_spectral.so
    python tests/golden/make_golden.py

Outputs (all data, no reference source):
  tests/golden/spectral_ref.npz   seeded inputs + outputs of the reference's own
                                  spectral routines (spe_spectral.f90 /
                                  spe_subfft_fftpack.f90 compiled as-is with
                                  flang -fdefault-real-8), plus its tables
                                  (mod_spectral: sia, wt, cpol, nsh2, via parmtr).
  speedy-ml-1_amd/data/region_sst_mask.txt
                                  1152 flags: region has an sst input <=> any point
                                  of its overlap tile has sea fraction >= 0.1 in the
                                  reference's boundary file bin/fort.20 (record 1 =
                                  land fraction; layout per ini_inbcon.f90:463-495).
                                  Used to choose the synthetic sst/no-sst shape classes.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle  # noqa: E402

SEED = 20250213


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def spectral_fixture():
    R = oracle.ref_spectral()
    if R is None:
        raise SystemExit("build the reference first: make -C oracle ref")
    a = ctypes.c_double(oracle.EARTH_RADIUS)
    R.parmtr_(ctypes.byref(a))
    R.inifft_()
    rng = np.random.default_rng(SEED)
    nf = 3
    out = {}

    def ci(v):
        return ctypes.byref(ctypes.c_int(v))

    # spectral-space inputs: white coefficients on the triangular T30 mask (the
    # entries gridy reads), grid-space inputs: smooth + noise fields.
    spec_in = rng.standard_normal((nf, 32, 62))
    grid_in = rng.standard_normal((nf, 48, 96)) + 5.0 * np.cos(np.linspace(0, 6.28, 96))[None, None, :]
    grid_in2 = rng.standard_normal((nf, 48, 96))
    out["spec_in"] = spec_in
    out["grid_in"] = grid_in
    out["grid_in2"] = grid_in2
    for kcos in (1, 2):
        g = np.zeros((nf, 48, 96))
        for f in range(nf):
            v = spec_in[f].copy()
            R.grid_(_p(v), _p(g[f]), ci(kcos))
        out[f"grid_k{kcos}"] = g
    s = np.zeros((nf, 32, 62))
    for f in range(nf):
        gg = grid_in[f].copy()
        R.spec_(_p(gg), _p(s[f]))
    out["spec"] = s
    gy = np.zeros((nf, 48, 62))
    sy = np.zeros((nf, 32, 62))
    sx = np.zeros((nf, 48, 62))
    for f in range(nf):
        v = spec_in[f].copy()
        R.gridy_(_p(v), _p(gy[f]))
        R.specy_(_p(gy[f].copy()), _p(sy[f]))
        R.specx_(_p(grid_in[f].copy()), _p(sx[f]))
    out["gridy"] = gy
    out["specy_of_gridy"] = sy
    out["specx"] = sx
    for kcos in (1, 2):
        vo = np.zeros((nf, 32, 62))
        dv = np.zeros((nf, 32, 62))
        for f in range(nf):
            R.vdspec_(_p(grid_in[f].copy()), _p(grid_in2[f].copy()), _p(vo[f]), _p(dv[f]), ci(kcos))
        out[f"vdspec_k{kcos}_vor"] = vo
        out[f"vdspec_k{kcos}_div"] = dv
    uu = np.zeros((nf, 32, 62))
    vv = np.zeros((nf, 32, 62))
    dx = np.zeros((nf, 32, 62))
    dy = np.zeros((nf, 32, 62))
    lp = np.zeros((nf, 32, 62))
    il = np.zeros((nf, 32, 62))
    tr = np.zeros((nf, 32, 62))
    for f in range(nf):
        R.uvspec_(_p(spec_in[f].copy()), _p(spec_in[(f + 1) % nf].copy()), _p(uu[f]), _p(vv[f]))
        R.grad_(_p(spec_in[f].copy()), _p(dx[f]), _p(dy[f]))
        R.lap_(_p(spec_in[f].copy()), _p(lp[f]))
        R.invlap_(_p(spec_in[f].copy()), _p(il[f]))
        t = spec_in[f].copy()
        R.trunct_(_p(t))
        tr[f] = t
    out.update(uvspec_u=uu, uvspec_v=vv, grad_x=dx, grad_y=dy, lap=lp, invlap=il, trunct=tr)
    # tables from the reference module globals are not exported by symbol name in a
    # portable way; recover sia/wt/cpol through the routines instead: gridy of a unit
    # coefficient e_(m,n) returns cpol(m,n,j) on the southern rows (varm(m,j) =
    # vm1 - vm2) -- store the full gridy response of the identity basis for m = 0,1.
    basis = np.zeros((32, 48, 62))
    for n in range(32):
        v = np.zeros((32, 62))
        v[n, 0] = 1.0
        v[n, 1] = 1.0
        R.gridy_(_p(v), _p(basis[n]))
    out["gridy_basis_m0"] = basis[:, :, :2]
    np.savez_compressed(os.path.join(HERE, "spectral_ref.npz"), **out)
    print("wrote spectral_ref.npz", {k: v.shape for k, v in out.items()})


def sst_mask():
    path = "/root/reference/bin/fort.20"
    d = np.fromfile(path, dtype="<f4").reshape(-1, 96)
    lf = np.zeros((48, 96), dtype=np.float32)
    for i in range(1, 49):  # read(iunit, rec=offset*nlat+i) inp(:, nlat+1-i), offset 1
        lf[48 - i, :] = d[1 * 48 + i - 1]
    lf[lf <= -999] = 0.0
    sea = (1.0 - lf) >= 0.1
    flags = []
    for r in range(1152):
        g = oracle.region_geometry(r)
        xs = [((g["input_xstart"] - 1 + dx) % 96) for dx in range(g["inputxchunk"])]
        ys = list(range(g["input_ystart"] - 1, g["input_yend"]))
        flags.append(int(sea[np.ix_(ys, xs)].any()))
    out = os.path.join(REPO, "speedy-ml-1_amd", "data", "region_sst_mask.txt")
    with open(out, "w") as f:
        f.write("# region sst-input flag (1 = has sst input); derived from reference bin/fort.20 by\n")
        f.write("# tests/golden/make_golden.py (sea fraction >= 0.1 anywhere in the overlap tile)\n")
        for i in range(0, 1152, 48):
            f.write(" ".join(str(v) for v in flags[i:i + 48]) + "\n")
    print("wrote", out, "sst regions:", sum(flags))


if __name__ == "__main__":
    spectral_fixture()
    sst_mask()

"""Synthetic reservoir weights laid out exactly like the trained NetCDF files.

No trained weights are available offline (Zenodo fetch, scripts/get_trained_coupled_data.sh),
so benches and tests use weights drawn per region from a seeded generator, with the
structure the reference's training produces:

  A      k = int(0.001 n^2) COO entries; rows and cols are independent per-n-block
         random permutations as makesparse builds them (mod_linalg.f90:180-218), so
         duplicate (row, col) pairs occur; vals U(0,1) * radius / 3 (a degree-6 U(0,1)
         matrix has spectral radius ~3; gen_res rescales to `radius`, :180-205).
  W_in   block diagonal, q = n/ninp rows per input, sigma * U(-1,1), sigma = 0.5
         (train_reservoir, mod_reservoir.f90:260-278).
  W_out  U(-0.01, 0.01), shape (nout, ncs + n).
  mean   U(0,1); std 0.5 + U(0,1); std(36) = 0 where the region has no sst input
         (so sst_bool_input <=> std(36) > 0.2, mod_reservoir.f90:1837-1845).

Every array is rounded to float32 (the NF90_REAL file precision, mod_io.f90:1282).
Arrays use the reference layouts: win (ninp, n) C-order == Fortran win(n, ninp);
wout (ncs+n, nout) C-order == Fortran wout(nout, ncs+n).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .domain import CHUNK_PRED, CHUNK_SPEEDY, radius_by_region, reservoir_sizes


@dataclass
class RegionWeights:
    region: int
    sst: bool
    n: int
    ninp: int
    k: int
    rows: np.ndarray   # int32 (k,), 1-based
    cols: np.ndarray   # int32 (k,), 1-based
    vals: np.ndarray   # float32 (k,)
    win: np.ndarray    # float32 (ninp, n)
    wout: np.ndarray   # float32 (ncs+n, nout)
    mean: np.ndarray   # float64 (36,) (file values are float32, widened exactly)
    std: np.ndarray    # float64 (36,)

    def win_compressed(self):
        """(col, val) of the single nonzero per row of W_in."""
        nz = self.win != 0
        col = np.argmax(nz, axis=0).astype(np.int32)
        val = self.win[col, np.arange(self.n)]
        return col, val


def climatology_mean_std():
    """Physically scaled standardisation constants (36 = 4 vars x 8 levels, logp,
    tisr, precip, sst; index map of unstandardize_state_vec_res,
    res_domain.f90:1424-1434, mod_reservoir.f90:1821-1846), so that unstandardized
    synthetic outputs look like a T30L8 state (level 1 = top)."""
    z = np.arange(8) / 7.0
    mean = np.zeros(36)
    std = np.ones(36)
    mean[0:8], std[0:8] = 210.0 + 75.0 * z, 8.0          # T [K]
    mean[8:16], std[8:16] = 10.0 - 5.0 * z, 10.0         # u [m/s]
    mean[16:24], std[16:24] = 0.0, 6.0                   # v [m/s]
    mean[24:32], std[24:32] = 0.01 + 8.0 * z ** 3, 0.5 + 3.0 * z ** 2  # q [g/kg]
    mean[32], std[32] = -0.02, 0.05                      # logp
    mean[33], std[33] = 300.0, 150.0                     # tisr
    mean[34], std[34] = 1e-3, 2e-3                       # precip
    mean[35], std[35] = 285.0, 10.0                      # sst
    return mean.astype(np.float32).astype(np.float64), std.astype(np.float32).astype(np.float64)


def region_weights(region: int, sst: bool, seed: int = 1234, chunk_speedy: int = CHUNK_SPEEDY,
                   nout: int = CHUNK_PRED, n_override: int | None = None,
                   climatology: bool = False) -> RegionWeights:
    sz = reservoir_sizes(region, sst)
    n, ninp, k, q = sz.n, sz.ninp, sz.k, sz.q
    if n_override is not None:  # reduced sizes for fast CPU tests (same structure)
        q = max(1, n_override // ninp)
        n = q * ninp
        k = int((6.0 / 6000.0) * n * n) if n_override >= 1000 else 6 * n
    rng = np.random.default_rng([seed, region])
    # A: per-block permutations (makesparse)
    rows = np.empty(k, dtype=np.int32)
    cols = np.empty(k, dtype=np.int32)
    full, left = divmod(k, n)
    for b in range(full):
        rows[b * n:(b + 1) * n] = rng.permutation(n)[:n] + 1
        cols[b * n:(b + 1) * n] = rng.permutation(n)[:n] + 1
    if left:
        rows[full * n:] = rng.permutation(n)[:left] + 1
        cols[full * n:] = rng.permutation(n)[:left] + 1
    radius = radius_by_region(region)
    vals = (rng.random(k) * (radius / 3.0)).astype(np.float32)
    # W_in: block diagonal
    win = np.zeros((ninp, n), dtype=np.float32)
    blk = (0.5 * (2.0 * rng.random((ninp, q)) - 1.0)).astype(np.float32)
    idx = np.arange(ninp)
    for j in range(q):
        win[idx, idx * q + j] = blk[:, j]
    wout = ((rng.random((chunk_speedy + n, nout), dtype=np.float32) * 2.0 - 1.0) * 0.01).astype(np.float32)
    mean = rng.random(36).astype(np.float32).astype(np.float64)
    std = (0.5 + rng.random(36)).astype(np.float32).astype(np.float64)
    if climatology:
        mean, std = climatology_mean_std()
    if not sst:
        std[35] = 0.0
    return RegionWeights(region, sst, n, ninp, k, rows, cols, vals, win, wout, mean, std)


def slab_weights(region: int, seed: int = 4321, n_override: int | None = None) -> RegionWeights:
    """A slab-ocean reservoir (initialize_slab_ocean_model, mod_slab_ocean_reservoir.f90:
    9-134): m = 4000 nodes, degree 6 (density 6/4000), 7 * in2d inputs (the atmo
    feedback's lowest level's 4 variables, logp, sst, tisr: :1532-1563), the sst of the
    region's resolved points out (ML only: chunk_speedy 0).  n = NINT(4000/ninp) *
    ninp, k = int(density n^2); W_in block diagonal, W_out U(-0.01, 0.01), the sst
    mean / std (slot 36) of the climatology, the rest U(0,1) / 0.5 + U(0,1)."""
    from .domain import region_geometry

    geo = region_geometry(region)
    in2d = geo.inx * geo.iny
    ninp = 7 * in2d
    q = int(np.floor(4000.0 / ninp + 0.5))
    if n_override is not None:
        q = max(1, n_override // ninp)
    n = q * ninp
    k = int((6.0 / 4000.0) * n * n)
    rng = np.random.default_rng([seed, region, 5])
    rows = np.empty(k, dtype=np.int32)
    cols = np.empty(k, dtype=np.int32)
    full, left = divmod(k, n)
    for b in range(full):
        rows[b * n:(b + 1) * n] = rng.permutation(n) + 1
        cols[b * n:(b + 1) * n] = rng.permutation(n) + 1
    if left:
        rows[full * n:] = rng.permutation(n)[:left] + 1
        cols[full * n:] = rng.permutation(n)[:left] + 1
    vals = (rng.random(k) * (0.9 / 3.0)).astype(np.float32)  # radius 0.9 (:31)
    win = np.zeros((ninp, n), dtype=np.float32)
    blk = (0.6 * (2.0 * rng.random((ninp, q)) - 1.0)).astype(np.float32)  # sigma 0.6 (:34)
    idx = np.arange(ninp)
    for j in range(q):
        win[idx, idx * q + j] = blk[:, j]
    nout = geo.resx * geo.resy
    wout = ((rng.random((n, nout), dtype=np.float32) * 2.0 - 1.0) * 0.01).astype(np.float32)
    mean = rng.random(36).astype(np.float32).astype(np.float64)
    std = (0.5 + rng.random(36)).astype(np.float32).astype(np.float64)
    cm, cs = climatology_mean_std()
    mean[35], std[35] = cm[35], cs[35]
    return RegionWeights(region, True, n, ninp, k, rows, cols, vals, win, wout, mean, std)


def slab_fields(seed: int = 77):
    """Synthetic sea-surface fields on the T30 grid ((48, 96) == Fortran (96, 48)):
    base_sst_grid (the year's first SST hour, floored at 272 K; mod_reservoir.f90:
    855-867), sea_mask (1 = land / permanent ice: every hour < 273.1 K, :874-883), and
    the coupler's sea-ice fraction and temperature (sice_am, tice_am) [ngp]."""
    rng = np.random.default_rng(seed)
    lat = np.linspace(-87.16, 87.16, 48)[:, None] * np.pi / 180.0
    lon = np.arange(96)[None, :] * 2 * np.pi / 96
    base = 271.0 + 31.0 * np.cos(lat) ** 2 + 0.8 * rng.standard_normal((48, 96))
    base = np.where(base < 272.0, 272.0, base)
    mask = ((np.sin(2 * lon) * np.cos(3 * lat) > 0.35) | (np.abs(lat) > 1.35)).astype(np.float64)
    sice = np.clip((np.abs(lat) - 1.2) * 2.0, 0.0, 1.0) * np.ones((48, 96))
    tice = 255.0 + 10.0 * rng.random((48, 96))
    return base, mask, sice.ravel(), tice.ravel()


def slab_start_outvec(region: int, seed: int = 88) -> np.ndarray:
    """start_prediction_slab's outvec of one region: the sst of its 4 points (K)."""
    rng = np.random.default_rng([seed, region])
    return 285.0 + 8.0 * rng.standard_normal(4)


def initial_state(region: int, n: int, seed: int = 99) -> np.ndarray:
    rng = np.random.default_rng([seed, region, 1])
    return 0.1 * (2.0 * rng.random(n) - 1.0)


def feedback_vector(region: int, ninp: int, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng([seed, region, 2])
    return rng.standard_normal(ninp)


def local_model_vector(region: int, ncs: int = CHUNK_SPEEDY, seed: int = 7) -> np.ndarray:
    rng = np.random.default_rng([seed, region, 3])
    return 2.0 * rng.random(ncs) - 1.0


def synthetic_grids(seed: int = 5):
    """A plausible T30L8 state in the sendrecievegrid layout: grid4d (z, y, x, var)
    C-order == Fortran (4, 96, 48, 8); grid2d / precip (48, 96) == (96, 48).
    T ~ 220-300 K, u/v ~ +-20 m/s, q ~ 0-15 g/kg, logp ~ 0 +- 0.1, precip >= 0."""
    rng = np.random.default_rng(seed)
    g4 = np.empty((8, 48, 96, 4))
    g4[..., 0] = 250.0 + 30.0 * rng.random((8, 48, 96))
    g4[..., 1] = 20.0 * rng.standard_normal((8, 48, 96))
    g4[..., 2] = 20.0 * rng.standard_normal((8, 48, 96))
    g4[..., 3] = 15.0 * rng.random((8, 48, 96))
    g2 = 0.1 * rng.standard_normal((48, 96))
    pr = np.abs(rng.standard_normal((48, 96)))
    return g4, g2, pr


# ---------------------------------------------------------------- SPEEDY state
def _spectral_field(rng, amp, power, mean=0.0):
    """complex (nx=32, mx=31) coefficients on the T30 triangle (m + n <= 30)
    decaying as (1 + m + n)^-power, m = 0 imaginary parts zero; mean sets the
    global mean (P_00 = sqrt(1/2))."""
    m = np.arange(31)[None, :]
    n = np.arange(32)[:, None]
    ll = m + n
    mask = ll <= 30
    c = np.zeros((32, 31), np.complex128)
    a = amp * (1.0 + ll) ** (-power)
    c[mask] = (rng.standard_normal(mask.sum()) + 1j * rng.standard_normal(mask.sum())) * a[mask]
    c[:, 0] = c[:, 0].real
    c[0, 0] = mean * np.sqrt(2.0)
    return c


def dyn_state(seed: int = 2025):
    """Seeded T30L8 spectral state (mod_dynvar layout, both time levels) around the
    reference temperature profile tref (ini_impint.f90:43-49), plus forcing
    (phis, tcorh, qcorh).  Same construction as tests/golden/make_dyn_golden.py with
    weaker, redder vorticity and divergence (winds within the iogrid(30) limits)."""
    rng = np.random.default_rng(seed)
    hsg = np.array([0.000, 0.050, 0.140, 0.260, 0.420, 0.600, 0.770, 0.900, 1.000])
    fsg = 0.5 * (hsg[1:] + hsg[:-1])
    rgam = (2.0 / 7.0) * 1004.0 * 6.0 / (1000.0 * 9.81)
    tref = 288.0 * np.maximum(0.2, fsg) ** rgam
    st = {f: np.zeros((2, 8, 32, 31), np.complex128) for f in ("vor", "div", "t", "tr")}
    st["ps"] = np.zeros((2, 32, 31), np.complex128)
    for k in range(8):
        st["vor"][0, k] = _spectral_field(rng, 6e-6, 1.5)
        st["div"][0, k] = _spectral_field(rng, 6e-7, 1.5)
        st["t"][0, k] = _spectral_field(rng, 2.0, 1.0, mean=tref[k])
        qm = 12.0 * fsg[k] ** 3
        st["tr"][0, k] = _spectral_field(rng, 0.2 * qm, 1.5, mean=qm)
    st["ps"][0] = _spectral_field(rng, 0.02, 1.5)
    for f, amp in (("vor", 2e-8), ("div", 2e-9), ("t", 2e-3), ("tr", 2e-4)):
        for k in range(8):
            st[f][1, k] = st[f][0, k] + _spectral_field(rng, amp, 1.0)
    st["ps"][1] = st["ps"][0] + _spectral_field(rng, 2e-5, 1.5)
    forcing = {"phis": _spectral_field(rng, 2000.0, 1.5, mean=3000.0),
               "tcorh": _spectral_field(rng, 1.0, 1.5), "qcorh": _spectral_field(rng, 0.1, 1.5)}
    return st, forcing


def phys_boundary(dyn, phis, tyear: float = 0.25, seed: int = 41):
    """Synthetic boundary fields for phypar (sml_dyn_set_physics order, see
    dynamics.PHYS_BC) on the T30 grid: a smooth land-sea mask, SST / land
    temperature falling off with latitude, soil water, albedos, a little snow;
    phis0 = grid image of the spectral orography `phis` (as inbcon builds it,
    ini_inbcon.f90:38-44), forog = sflset(phis0), and the radiation forcing of
    sol_oz(tyear).  Shaped like the reference's boundary files, not read from them."""
    from .spectral import Spectral

    rng = np.random.default_rng(seed)
    ngp = 96 * 48
    sp = Spectral()
    sia = sp.tables()["sia"]
    lat_s = -np.arcsin(sia)
    radang = np.concatenate([lat_s, lat_s[::-1] * -1.0])  # south -> north (indyns)
    lat = np.repeat(radang, 96)
    lon = np.tile(np.arange(96) * 2 * np.pi / 96, 48)
    bc = {
        "fmask1": np.clip(0.5 + 0.6 * np.sin(2 * lon) * np.cos(3 * lat), 0.0, 1.0),
        "sst_am": 271.0 + 30.0 * np.cos(lat) ** 2 + 0.5 * rng.standard_normal(ngp),
        "stl_am": 265.0 + 30.0 * np.cos(lat) ** 2 + 1.0 * rng.standard_normal(ngp),
        "soilw_am": np.clip(0.4 + 0.3 * rng.standard_normal(ngp), 0.0, 1.0),
        "alb_l": 0.2 + 0.1 * rng.random(ngp),
        "alb_s": 0.07 + 0.05 * rng.random(ngp),
        "snowc": np.clip(rng.random(ngp) - 0.7, 0.0, 1.0),
    }
    bc["albsfc"] = bc["alb_s"] + bc["fmask1"] * (bc["alb_l"] - bc["alb_s"])
    ph = np.ascontiguousarray(np.asarray(phis, dtype=np.complex128)).view(np.float64).reshape(1, 32, 62)
    bc["phis0"] = np.asarray(sp.grid_host(ph, kcos=1)).ravel()
    bc["forog"] = dyn.sflset(bc["phis0"])
    bc.update(dyn.sol_oz(tyear))
    return bc


def _mask_threshold(frac, thrsh=0.1):
    """inbcon's fractional masks (ini_inbcon.f90:49-63, 146-156): below thrsh -> 0,
    above 1 - thrsh -> 1."""
    f = np.where(frac >= thrsh, frac, 0.0)
    return np.where(frac > 1.0 - thrsh, 1.0, f)


def surface_climatology(fmask, seed: int = 43):
    """Synthetic inputs of the window's date-driven forcing on the T30 grid, shaped
    like inbcon's (ini_inbcon.f90): the surface fields of sml_dyn_set_surface
    {fmask_l, fmask_s, alb0} from a land fraction `fmask` (ngp,), and the monthly
    climatologies of sml_dyn_set_climatology {stl12, snowd12, soilw12, sst12, sice12}
    (12, ngp) with a seasonal cycle of opposite phase in the two hemispheres: polar
    SSTs below freezing in winter with sea ice (the coupler's ice branch), snow depths
    past sd2sc at high latitudes (snowc clipped at 1).  Not read from the reference's
    boundary files."""
    rng = np.random.default_rng(seed)
    ngp = 96 * 48
    lat = np.repeat(np.arcsin(np.polynomial.legendre.leggauss(48)[0]), 96)  # Gaussian, south -> north
    fmask = np.asarray(fmask, dtype=np.float64).ravel()
    surf = {"fmask_l": _mask_threshold(fmask), "fmask_s": _mask_threshold(1.0 - fmask),
            "alb0": 0.1 + 0.25 * rng.random(ngp)}
    m = np.arange(12)[:, None]
    season = np.cos(2 * np.pi * (m - 6.5) / 12) * np.sign(lat)[None, :]  # > 0: summer
    c2 = np.cos(lat)[None, :] ** 2
    clim = {
        "stl12": 262.0 + 30.0 * c2 + 14.0 * season * (1 - c2) + rng.standard_normal((12, ngp)),
        "sst12": 270.5 + 31.0 * c2 + 3.5 * season * (1 - c2) + 0.3 * rng.standard_normal((12, ngp)),
        "soilw12": np.clip(0.35 + 0.25 * season * c2 + 0.1 * rng.standard_normal((12, ngp)), 0.0, 1.0),
    }
    cold = np.clip(-season * (1 - c2) - 0.2, 0.0, None)
    clim["snowd12"] = 150.0 * cold * rng.random((12, ngp))
    clim["sice12"] = np.clip(1.6 * cold + 0.05 * rng.standard_normal((12, ngp)), 0.0, 1.0)
    return surf, clim

"""Host-side decomposition logic (no compute): which regions a rank owns, region
geometry and reservoir sizes.

Mirrors the reference's res_domain / mod_reservoir bookkeeping:
  processor_decomposition      src/res_domain.f90:31-62
  getxyresextent / overlap     src/res_domain.f90:123-204, 258-292
  allocate_res_new sizes       src/mod_reservoir.f90:78-178
  trained_reservoir_prediction src/mod_reservoir.f90:1781-1884 (sst input <=> std(36) > 0.2)
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

XGRID, YGRID, ZGRID, NVARS = 96, 48, 8, 4
NUM_REGIONS = 1152
CHUNK_PRED = 136      # chunk_size_prediction: atmo 128 + logp 4 + precip 4
CHUNK_SPEEDY = 132    # chunk_size_speedy: atmo 128 + logp 4
M_NODES = 6000        # reservoir%m (mod_reservoir.f90:89)
DATA_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "data")


def processor_decomposition(numregions: int, numprocs: int, irank: int) -> list[int]:
    """Regions owned by rank `irank` (res_domain.f90:31-62)."""
    per = numregions // numprocs
    left = numregions % numprocs
    if irank >= left + 1 and irank > 0:
        return [per * irank + i for i in range(per)]
    if irank == 0:
        return list(range(per))
    return [per * irank + i for i in range(per)] + [numregions - left + irank - 1]


def _decompose(numregions: int):
    n = XGRID * YGRID // numregions
    fmax = int(np.floor(np.sqrt(float(n))))
    for i in range(fmax, 0, -1):
        if YGRID % i == 0:
            fy = i
            if n % fy == 0:
                fx = n // fy
                if XGRID % fx == 0:
                    return fx, fy
    raise ValueError(f"{numregions} regions do not tile the {XGRID}x{YGRID} grid")


@dataclass(frozen=True)
class RegionGeom:
    res_xstart: int
    res_xend: int
    res_ystart: int
    res_yend: int
    resx: int
    resy: int
    in_xstart: int
    in_xend: int
    in_ystart: int
    in_yend: int
    inx: int
    iny: int
    pole: bool
    periodic: bool

    def input_x(self, lx: int) -> int:
        """1-based global x of 1-based local input column lx (tileoverlapgrid4d wrap)."""
        if self.periodic and (self.res_xend > self.in_xend or self.in_xstart > self.res_xstart):
            nfirst = XGRID - (self.in_xstart - 1)
            return self.in_xstart + lx - 1 if lx <= nfirst else lx - nfirst
        return self.in_xstart + lx - 1


def region_geometry(region: int, numregions: int = NUM_REGIONS, overlap: int = 1) -> RegionGeom:
    fx, fy = _decompose(numregions)
    col = region % (YGRID // fy)
    row = region // (YGRID // fy)
    xs, xe, ys, ye = row * fx + 1, (row + 1) * fx, col * fy + 1, (col + 1) * fy
    inx, iny = fx + 2 * overlap, fy + 2 * overlap
    periodic = pole = False
    if xs - overlap < 1:
        ixs, periodic = XGRID - overlap + 1, True
    else:
        ixs = xs - overlap
    if xe + overlap > XGRID:
        ixe, periodic = overlap, True
    else:
        ixe = xe + overlap
    if ys - overlap < 1:
        iys, iny, pole = 1, fy + overlap + (ys - 1), True
    else:
        iys = ys - overlap
    if ye + overlap > YGRID:
        iye, iny, pole = YGRID, fy + overlap + (YGRID - ye), True
    else:
        iye = ye + overlap
    return RegionGeom(xs, xe, ys, ye, fx, fy, ixs, ixe, iys, iye, inx, iny, pole, periodic)


@dataclass(frozen=True)
class ReservoirSizes:
    ninp: int
    n: int
    k: int
    q: int  # nodes per input (W_in block height)


def reservoir_sizes(region: int, sst: bool, numregions: int = NUM_REGIONS, m_nodes: int = M_NODES) -> ReservoirSizes:
    """n, k, ninp of a bottom-level reservoir (allocate_res_new, mod_reservoir.f90:104-170)."""
    g = region_geometry(region, numregions)
    in2d, res2d = g.inx * g.iny, g.resx * g.resy
    chunk = res2d * NVARS * ZGRID + 2 * res2d
    locality = in2d * ZGRID * NVARS + 3 * in2d + (in2d if sst else 0) - chunk
    ninp = chunk + locality
    q = int(np.floor(m_nodes / ninp + 0.5))  # NINT of a positive value
    n = q * ninp
    k = int((6.0 / float(m_nodes)) * n * n)  # density*n*n, truncated (:99, :170)
    return ReservoirSizes(ninp=ninp, n=n, k=k, q=q)


def load_sst_mask() -> np.ndarray:
    """1152 sst-input flags derived from the reference's bin/fort.20 land mask
    (tests/golden/make_golden.py)."""
    path = os.path.join(DATA_DIR, "region_sst_mask.txt")
    vals = []
    with open(path) as f:
        for line in f:
            if line.startswith("#"):
                continue
            vals.extend(int(v) for v in line.split())
    arr = np.asarray(vals, dtype=np.uint8)
    assert arr.size == NUM_REGIONS
    return arr


def radius_by_region(region: int, numregions: int = NUM_REGIONS) -> float:
    """get_radius_by_lat (res_domain.f90:1601-1638) at the region's latitudes."""
    lat = SPEEDY_LAT
    g = region_geometry(region, numregions)
    start, end = lat[g.res_ystart - 1], lat[g.res_yend - 1]
    smallest = abs(min(start, end))
    if smallest >= 45.0:
        return 0.7
    return (0.7 - 0.3) / 45.0 + 0.3


SPEEDY_LAT = (-87.159, -83.479, -79.777, -76.070, -72.362, -68.652, -64.942, -61.232, -57.521, -53.810,
              -50.099, -46.389, -42.678, -38.967, -35.256, -31.545, -27.833, -24.122, -20.411, -16.700,
              -12.989, -9.278, -5.567, -1.856, 1.856, 5.567, 9.278, 12.989, 16.700, 20.411,
              24.122, 27.833, 31.545, 35.256, 38.967, 42.678, 46.389, 50.099, 53.810, 57.521,
              61.232, 64.942, 68.652, 72.362, 76.070, 79.777, 83.479, 87.159)

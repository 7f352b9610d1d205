"""Diagnostic: where the row kernel's physics phase goes, from the profiling build's
sub-phase stamps (-DSML_PSTAMPS: tools/build_variant.sh pst ...).  Runs chained windows
ending on a longwave-only step (nleap 24) and on a shortwave step (nleap 22) and prints
the median over the 48 row blocks of each stamped interval (us), per wave role.
    SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_pst.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd._lib import lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary  # noqa: E402

L = lib()
L.sml_dbg_pst.argtypes = [ctypes.c_void_p]
st, forcing = dyn_state()
d = Dynamics()
d.set_forcing(**forcing)
d.set_state(st)
d.set_physics(phys_boundary(d, forcing["phis"]))
MOIST = [(8, 9, "dynamics"), (9, 10, "thermo"), (10, 11, "convmf+lscond"), (11, 12, "vdifsc"), (12, 13, "hand-over")]
LW = [(0, 1, "loads/thermo"), (1, 2, "radlw down"), (2, 3, "suflux"), (3, 4, "radlw up"), (4, 5, "products")]
SW = [(0, 16, "loads+thermo"), (16, 17, "moist"), (17, 18, "sw (cloud+radsw)"), (18, 1, "->lw")]
for nleap, name in ((24, "longwave-only step"), (22, "shortwave step")):
    for rep in range(3):
        d.set_clock(1, True)
        d.window(nleap)
    torch.cuda.synchronize()
    buf = np.zeros((48, 32), dtype=np.int64)
    assert L.sml_dbg_pst(buf.ctypes.data) == 0
    b = buf.astype(np.float64) / 100.0  # wall_clock64 at 100 MHz -> us
    t0 = np.minimum(b[:, 8], b[:, 0])
    print(f"== {name} (nleap {nleap}); from the physics phase start, median over blocks (us):")
    for title, rows in (("moist side (wave 0)", MOIST), ("longwave side (wave 2)", LW + ([] if nleap == 24 else SW))):
        parts = [f"{lab} {np.median(b[:, e] - b[:, s]):.2f}" for s, e, lab in rows if b[:, e].max() > 0 and b[:, s].max() > 0]
        print(f"  {title}: " + " | ".join(parts))
    print(f"  moist side done at {np.median(b[:, 13] - t0):.2f}, longwave side done at {np.median(b[:, 5] - t0):.2f}, "
          f"barrier passed at {np.median(b[:, 20] - t0):.2f} (max {np.max(b[:, 20] - t0):.2f})")
d.close()

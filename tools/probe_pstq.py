"""Diagnostic: the quad row kernel's physics sub-phases from the profiling build's stamps
(-DSML_PSTAMPS: tools/build_variant.sh pst ...), wave 2's first quad and wave 0's
grid-point dynamics, median over the 48 row blocks (us) from the physics phase start,
for a window ending on a longwave-only step (nleap 24) and on a shortwave step (22).
    SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_pstq.py"""
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
Q = [(21, 30, "inputs"), (30, 22, "thermo"), (22, 23, "convmf"), (23, 31, "lscond"), (31, 24, "precls+vdif"), (24, 25, "sw"), (25, 26, "lw down"),
     (26, 27, "suflux"), (27, 28, "lw up"), (28, 29, "tail"), (29, 20, "barrier")]
for nleap, name in ((24, "longwave-only step"), (22, "shortwave step")):
    for rep in range(3):
        d.set_clock(1, True)
        d.window(nleap)
    torch.cuda.synchronize()
    buf = np.zeros((48, 32), dtype=np.int64)
    assert L.sml_dbg_pst(buf.ctypes.data) == 0
    b = buf.astype(np.float64) / 100.0  # wall_clock64 at 100 MHz -> us
    t0 = b[:, 21]
    print(f"== {name} (nleap {nleap}); median over blocks (us):")
    print("  quad (wave 2): " + " | ".join(f"{lab} {np.median(b[:, e] - b[:, s]):.2f}" for s, e, lab in Q))
    print(f"  quad done at {np.median(b[:, 29] - t0):.2f}, dynamics (wave 0) {np.median(b[:, 9] - b[:, 8]):.2f}, "
          f"barrier passed at {np.median(b[:, 20] - t0):.2f} (max {np.max(b[:, 20] - t0):.2f})")
d.close()

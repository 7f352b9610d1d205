"""Diagnostic: the pair row kernel's roles (k_st_gridspec_p) from the profiling build's
stamps (-DSML_PSTAMPS: tools/build_variant.sh pst ...), median over the 48 row blocks (us
from the physics phase start), for a window ending on a longwave-only step (nleap 24) and
on a shortwave step (nleap 22).
    SML_LIB=abx/pst/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_pstp.py"""
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
for nleap, name in ((24, "longwave-only step"), (22, "shortwave step")):
    for rep in range(3):
        d.set_clock(1, True)
        d.window(nleap)
    torch.cuda.synchronize()
    buf = np.zeros((48, 32), dtype=np.int64)
    assert L.sml_dbg_pst(buf.ctypes.data) == 0
    b = buf.astype(np.float64) / 100.0  # wall_clock64 at 100 MHz -> us
    t0 = b[:, 8]
    m = lambda s: np.median(b[:, s] - t0)  # noqa: E731
    print(f"== {name} (nleap {nleap}); median over blocks, us from the physics phase start:")
    print(f"  dynamics (wave 0) done {m(9):.2f}")
    print(f"  moist (wave 2): thermo {m(11):.2f} | moist {m(12):.2f} | vdifsc + hand-over {m(13):.2f}")
    print(f"  pairs (wave 4): sw/prefetch {m(15):.2f} | lw down {m(16):.2f} | suflux {m(17):.2f} | done {m(18):.2f}"
          f" (wave 6 done {m(19):.2f})")
    print(f"  barrier passed {m(20):.2f} (max {np.max(b[:, 20] - t0):.2f})")
d.close()

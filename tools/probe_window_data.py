"""Diagnostic: the window's per-phase stamps (SML_DYN_STAMPS, the last row kernel and
the per-m kernel before it) for a free-running window and for a window entered from a
synthetic grid (from_grid + window, what run_model integrates), to locate the phases
a fresh entry state slows.
    python tools/probe_window_data.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd._lib import lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids  # noqa: E402

dev = torch.device("cuda", 0)
os.environ["SML_DYN_STAMPS"] = "1"
d = Dynamics()
del os.environ["SML_DYN_STAMPS"]
st0, forcing = dyn_state()
d.set_forcing(**forcing)
d.set_state(st0)
d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_rad_state(None)
d.set_clock(1, True)
g4h, g2h, _ = synthetic_grids(11)
g4, g2 = torch.from_numpy(g4h).to(dev), torch.from_numpy(g2h).to(dev)
L = lib()
L.sml_dbg_dyn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def stamps():
    torch.cuda.synchronize()
    buf = np.zeros((4, 96, 8), dtype=np.int64)
    assert L.sml_dbg_dyn_stamps(d._h, buf.ctypes.data) == 0
    return buf


def phases(buf, kern, names):
    nb = int((buf[kern, :, 0] > 0).sum())
    b = buf[kern, :nb].astype(np.float64) / 100.0
    ph = {n: round(float(np.median(b[:, i + 1] - b[:, i])), 2) for i, n in enumerate(names)}
    mx = {n: round(float(np.max(b[:, i + 1] - b[:, i])), 2) for i, n in enumerate(names)}
    span = float(b[:, len(names)].max() - b[:, 0].min())
    return ph, mx, round(span, 2)


for name, fn in (("free run", lambda: d.window(24)), ("from_grid + window", lambda: (d.from_grid(g4, g2), d.window(24))),
                 ("free run", lambda: d.window(24))):
    res = []
    for _ in range(10):
        fn()
        res.append(stamps())
    for kern, names in ((0, ["gridx", "gridpoint_and_phypar", "specx"]),
                        (1, ["load", "specy", "combine", "tail", "inv_inputs", "gridy"])):
        ph = [phases(b, kern, names) for b in res[3:]]
        med = {n: round(float(np.median([p[0][n] for p in ph])), 2) for n in names}
        mxx = {n: round(float(np.median([p[1][n] for p in ph])), 2) for n in names}
        span = round(float(np.median([p[2] for p in ph])), 2)
        print(f"{name:20s} kernel {kern}: span {span:6.2f} median phases {med}  max-block phases {mxx}")
d.close()

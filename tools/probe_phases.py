"""Diagnostic: per-phase durations inside the fused SPEEDY step kernels
(SML_DYN_STAMPS=1), from a chained window.  python tools/probe_phases.py [phys=1]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
os.environ["SML_DYN_STAMPS"] = "1"
from speedy_ml_amd._lib import lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary  # noqa: E402

phys = (sys.argv[1] if len(sys.argv) > 1 else "1") == "1"
st, forcing = dyn_state()
d = Dynamics()
d.set_forcing(**forcing)
d.set_state(st)
if phys:
    d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_clock(1, True)
d.window(24)
torch.cuda.synchronize()
K = {0: ("grid" if phys else "rows", ["gridx", "gridpoint/physics", "specx"] if phys else ["load", "gridx", "gridpoint", "specx"]),
     1: ("spec (chained)", ["load", "specy", "combine", "tail", "inv_inputs", "gridy"]),
     2: ("specx", ["load", "fft+store"]),
     3: ("spec (last)", ["load", "specy", "combine", "tail"])}
L = lib()
L.sml_dbg_dyn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
for rep in range(2):
    d.window(24)
    torch.cuda.synchronize()
    buf = np.zeros((4, 96, 8), dtype=np.int64)
    assert L.sml_dbg_dyn_stamps(d._h, buf.ctypes.data) == 0
    for kern, (name, phases) in K.items():
        nb = int((buf[kern, :, 0] > 0).sum())
        if nb == 0:
            continue
        b = buf[kern, :nb].astype(np.float64)
        t0 = b[:, 0].min()
        line = [f"{name} ({nb} blocks)"]
        for i, ph in enumerate(phases):
            if b[:, i + 1].max() == 0:
                continue
            dt = (b[:, i + 1] - b[:, i]) / 100.0
            line.append(f"{ph} med {np.median(dt):.2f} max {dt.max():.2f}")
        last = max(i for i in range(8) if b[:, i].max() > 0)
        line.append(f"span {(b[:, last].max() - t0) / 100:.2f}us")
        print(" | ".join(line))
    # launch-to-launch gaps along one step: spec(chained, previous step) -> grid -> specx -> spec(last)
    se = {}
    for kern in (1, 0, 2, 3):
        nb = int((buf[kern, :, 0] > 0).sum())
        if nb:
            b = buf[kern, :nb]
            last = max(i for i in range(8) if b[:, i].max() > 0)
            se[kern] = (b[:, 0].min(), b[:, 0].max(), b[:, last].max())
    seq = [k for k in (1, 0, 2, 3) if k in se]
    print("gaps (last stamp of one kernel -> first / last block start of the next):",
          ", ".join(f"{K[a][0]}->{K[b][0]} {(se[b][0] - se[a][2]) / 100:.2f}/{(se[b][1] - se[a][2]) / 100:.2f}us"
                    for a, b in zip(seq, seq[1:])))
    print()

"""Diagnostic: where a chained SPEEDY window's time goes between its kernels.  Runs two
windows with the in-kernel wall_clock64 stamps on (SML_DYN_STAMPS, the same capture
as bench.py's speedy_roofline) and prints, for the last launch of each stamped kernel
kind, when its blocks started and ended relative to the earliest stamp -- so the gap
from one kernel's last block to the next kernel's first block (the kernel boundary)
and the blocks' start / end skew are visible.
    python tools/probe_window_gaps.py"""
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

NAMES = {0: "k_st_gridspec (last step)", 1: "k_st_spec (step before last)", 2: "kind 2", 3: "k_st_spec (last)"}
st, forcing = dyn_state()
os.environ["SML_DYN_STAMPS"] = "1"
d = Dynamics()
del os.environ["SML_DYN_STAMPS"]
d.set_forcing(**forcing)
d.set_state(st)
d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_rad_state(None)
d.set_clock(1, True)
for _ in range(3):
    d.window(24)
torch.cuda.synchronize()
buf = np.zeros((4, 96, 8), dtype=np.int64)
L = lib()
L.sml_dbg_dyn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
assert L.sml_dbg_dyn_stamps(d._h, buf.ctypes.data) == 0
d.close()
t0 = buf[buf > 0].min()
rows = []
for k in range(4):
    nb = int((buf[k, :, 0] > 0).sum())
    if nb == 0:
        continue
    b = buf[k, :nb]
    ns = int((b[0] > 0).sum())  # stamps per block
    s = (b[:, 0] - t0) / 100.0
    e = (b[:, ns - 1] - t0) / 100.0
    rows.append((s.min(), k, nb, ns, s.min(), s.max(), e.min(), e.max(), np.median(np.diff(b[:, :ns], axis=1), 0) / 100, e))
rows.sort()
prev_end = None
for _, k, nb, ns, s0, s1, e0, e1, ph, e in rows:
    gap = "" if prev_end is None else f"  boundary from previous last block: {s0 - prev_end:6.2f} us"
    print(f"{NAMES.get(k, k):30s} blocks {nb:3d}  start {s0:8.2f}..{s1:8.2f}  end {e0:8.2f}..{e1:8.2f}{gap}")
    print(f"{'':30s} median phases (us): {np.round(ph, 2).tolist()}")
    b = buf[k, :nb]
    late = np.argsort(e)[::-1][:8]
    print(f"{'':30s} latest blocks: " + ", ".join(
        f"{i}: end {e[i]:.2f} phases {np.round(np.diff(b[i, :ns]) / 100, 2).tolist()}" for i in late[:4]))
    print(f"{'':30s} end by block: {np.round(e - e.min(), 2).tolist()}")
    prev_end = e1

"""Diagnostic (timeline build): the same 26-step window in its three forms, nothing
beside it -- dyn.window (free run: k_state_to_m + k_st_inv + the window graph),
from_grid + window (iogrid(30) of a fixed grid, then the plain window graph), and
run_model (k_io_entry + the prepared window graph with the exit captured) -- to tell
whether run_model's window is slower for its data or for its form.
    SML_LIB=abx/tl/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_window_forms.py"""
import os
import statistics
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from probe_step_accounting import Timeline, launches, window_pieces  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids  # noqa: E402

dev = torch.device("cuda", 0)
tl = Timeline()
st0, forcing = dyn_state()
d = Dynamics()
d.set_forcing(**forcing)
d.set_state(st0)
d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_rad_state(None)
d.set_clock(1, True)
g4h, g2h, _ = synthetic_grids(11)
g4, g2 = torch.from_numpy(g4h).to(dev), torch.from_numpy(g2h).to(dev)
f4, f2 = torch.zeros_like(g4), torch.zeros_like(g2)
s = torch.cuda.Stream()


def measure(name, fn, n=30):
    tl.reset()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    rd = tl.read()
    r, p = launches(rd, "row"), launches(rd, "spec")
    w = [window_pieces(r[26 * i:26 * i + 26], p[26 * i:26 * i + 26]) for i in range(5, len(r) // 26)]
    m = {k: statistics.median([x[k] for x in w]) for k in w[0]}
    print(f"{name:34s} span {m['span']:7.1f}  row {m['row_kernels']:7.1f}  per-m {m['per_m_kernels']:7.1f}  "
          f"boundaries {m['boundaries']:6.1f}  (us, {len(w)} windows)")


with torch.cuda.stream(s):
    measure("window (free run)", lambda: d.window(24, stream=s))
    measure("from_grid + window", lambda: (d.from_grid(g4, g2, stream=s), d.window(24, stream=s)))
    measure("run_model", lambda: d.run_model(g4, g2, f4, f2, stream=s))
    measure("window (free run) again", lambda: d.window(24, stream=s))
d.close()

"""Diagnostic: host-side time of each call of the hybrid loop (predict / exchange /
advance), to see whether the host blocks while the GPU runs.  Small reservoirs
(n = 600) on all 1152 regions, the full SPEEDY window.
    python tools/probe_host_loop.py"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd import domain  # noqa: E402
from speedy_ml_amd._lib import check, lib, ptr  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.exchange import OutvecExchange  # noqa: E402
from speedy_ml_amd.hybrid import HybridLoop  # noqa: E402
from speedy_ml_amd.reservoir import Reservoirs  # noqa: E402
from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights,  # noqa: E402
                                     synthetic_grids)

mask = domain.load_sst_mask()
ws = [region_weights(r, bool(mask[r]), n_override=600, seed=5, climatology=True) for r in range(1152)]
res = Reservoirs(list(range(1152)), mask, [w.n for w in ws], [w.k for w in ws])
for r, w in enumerate(ws):
    res.load_region_weights(r, w)
    res.set_state(r, initial_state(r, w.n))
st0, forcing = dyn_state()
dyn = Dynamics()
dyn.set_forcing(**forcing)
dyn.set_state(st0)
dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
cuda = torch.device("cuda", 0)
loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=cuda), cuda)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
g4, g2, pr = synthetic_grids(11)
f4, f2, _ = synthetic_grids(12)
loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
for _ in range(5):
    loop.step()
loop.sync()
torch.cuda.synchronize()
rows = []
T0 = time.perf_counter()
for s in range(12):
    a = time.perf_counter()
    check(lib().sml_hybrid_predict(loop._h))
    b = time.perf_counter()
    with torch.cuda.stream(loop.main):
        glob = loop.exchange(loop.ov)
    c = time.perf_counter()
    check(lib().sml_hybrid_advance(loop._h, ptr(glob)))
    d = time.perf_counter()
    rows.append(((a - T0) * 1e3, (b - a) * 1e3, (c - b) * 1e3, (d - c) * 1e3))
loop.sync()
torch.cuda.synchronize()
tot = (time.perf_counter() - T0) * 1e3
for r in rows:
    print("t=%8.3f ms  predict %7.3f  exchange %7.3f  advance %7.3f" % r)
print(f"total {tot:.2f} ms for 12 steps = {tot / 12:.3f} ms/step")

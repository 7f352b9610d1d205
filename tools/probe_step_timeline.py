"""Diagnostic: an untraced timeline of the overlapped hybrid step.  It records HIP
events between the calls of sml_hybrid_predict / sml_hybrid_advance, issued one by
one from Python on the HybridLoop's own streams.  The reservoirs are full size, with
SPEEDY on CUs [0, 64) and the reservoir on the rest, as in bench.py.
    python tools/probe_step_timeline.py"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd import domain  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.hybrid import HybridLoop  # noqa: E402
from speedy_ml_amd.reservoir import Reservoirs  # noqa: E402
from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights,  # noqa: E402
                                     synthetic_grids)

dev = torch.device("cuda", 0)
nreg = 1152
mask = domain.load_sst_mask()
regions = list(range(nreg))
sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in regions]
res = Reservoirs(regions, [mask[r] for r in regions], [s.n for s in sizes], [s.k for s in sizes])
for i, r in enumerate(regions):
    w = region_weights(r, bool(mask[r]), climatology=True)
    res.load_region_weights(i, w)
    res.set_state(i, initial_state(r, w.n))
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
g4h, g2h, prh = synthetic_grids(11)
f4h, f2h, _ = synthetic_grids(12)
tisr = t(np.random.default_rng(13).standard_normal((nreg, 16)))
st0, forcing = dyn_state()
dyn = Dynamics()
dyn.set_forcing(**forcing)
dyn.set_state(st0)
dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
loop = HybridLoop(res, dyn, lambda ov: ov, dev, tisr=tisr, overlap=True)
loop.start(t(g4h), t(g2h), t(prh), t(f4h), t(f2h))
for _ in range(5):
    loop.step()
loop.sync()
torch.cuda.synchronize()
main, side = loop.main, loop.side
fb, lm, ov, g4, g2, pr, f4, f2 = loop.fb, loop.lm, loop.ov, loop.g4, loop.g2, loop.pr, loop.f4, loop.f2
ev_lm, ev_grid = torch.cuda.Event(), torch.cuda.Event()
ev_lm.record(main)


def ev(stream):
    e = torch.cuda.Event(enable_timing=True)
    e.record(stream)
    return e


NS = 24
rows = []
for step in range(NS):
    marks = {"main0": ev(main)}
    res.predict_begin(fb, stream=main)
    marks["begin_done"] = ev(main)
    main.wait_event(ev_lm)
    marks["lm_ready"] = ev(main)
    res.predict_finish_grid(f4, f2, lm, ov, stream=main)
    marks["finish_done"] = ev(main)
    res.assemble(ov, g4, g2, pr, stream=main)  # one rank: the exchange is the identity
    marks["assembled"] = ev(main)
    ev_grid.record(main)
    res.tile_feedback(g4, g2, pr, tisr, fb, stream=main)
    marks["tiled"] = ev(main)
    side.wait_event(ev_grid)
    marks["side_start"] = ev(side)
    dyn.run_model(g4, g2, f4, f2, stream=side)
    marks["window_done"] = ev(side)
    ev_lm.record(side)
    rows.append(marks)
torch.cuda.synchronize()
keys = ["begin_done", "lm_ready", "finish_done", "assembled", "tiled", "side_start", "window_done"]
sel = range(6, NS - 1)
print("ms from the step's first main-stream event (median over steady steps):")
tab = np.array([[rows[i]["main0"].elapsed_time(rows[i][k]) for k in keys] for i in sel])
for k, v in zip(keys, np.median(tab, axis=0)):
    print(f"  {k:12s} {v:8.4f}")
period = np.median([rows[i]["main0"].elapsed_time(rows[i + 1]["main0"]) for i in sel])
print(f"  step period  {period:8.4f} ms  ({1e3 / period:.1f} steps/s)")
med = lambda a, b, off=0: np.median([rows[i - off][a].elapsed_time(rows[i][b]) for i in sel]) * 1e3  # noqa: E731
print("segments (us):")
print(f"  prev window_done -> lm_ready       {med('window_done', 'lm_ready', 1):8.1f}")
print(f"  lm_ready -> finish_done            {med('lm_ready', 'finish_done'):8.1f}")
print(f"  finish_done -> assembled           {med('finish_done', 'assembled'):8.1f}")
print(f"  assembled -> side_start            {med('assembled', 'side_start'):8.1f}")
print(f"  side_start -> window_done          {med('side_start', 'window_done'):8.1f}")
print(f"  assembled -> tiled                 {med('assembled', 'tiled'):8.1f}")
print(f"  main0 -> begin_done                {med('main0', 'begin_done'):8.1f}")
print(f"  critical: window_done -> window_done {med('window_done', 'window_done', 1):8.1f}")
loop.close()

"""Diagnostic: host time spent in each call of HybridLoop.step (which call blocks
the issuing thread).  python tools/probe_host_block.py"""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd import domain  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.exchange import OutvecExchange  # noqa: E402
from speedy_ml_amd.hybrid import HybridLoop  # noqa: E402
from speedy_ml_amd.reservoir import Reservoirs  # noqa: E402
from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights,  # noqa: E402
                                     synthetic_grids)

dev = torch.device("cuda:0")
mask = domain.load_sst_mask()
n_over = int(os.environ.get("PROBE_N", "0")) or None
ws = [region_weights(r, bool(mask[r]), n_override=n_over, climatology=True) for r in range(1152)]
res = Reservoirs(list(range(1152)), mask, [w.n for w in ws], [w.k for w in ws])
for i, w in enumerate(ws):
    res.load_region_weights(i, w)
    res.set_state(i, initial_state(w.region, w.n))
st0, forcing = dyn_state()
dyn = Dynamics()
dyn.set_forcing(**forcing)
dyn.set_state(st0)
dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=dev), dev,
                  tisr=t(np.random.default_rng(13).standard_normal((1152, 16))),
                  side_priority=int(os.environ.get("PROBE_PRIO", "-1")))
g4, g2, pr = synthetic_grids(11)
f4, f2, _ = synthetic_grids(12)
loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
for _ in range(3):
    loop.step()
loop.sync()
m, s = loop.main, loop.side


def cu_stream(cus):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    mask = (ctypes.c_uint32 * 8)()
    for c in cus:
        mask[c // 32] |= 1 << (c % 32)
    h = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, mask)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(h.value)


split = os.environ.get("PROBE_SPLIT")
if split:
    kind, n = split.split(":")
    n = int(n)
    if kind == "hi":
        side_cus = list(range(256 - n, 256))
    else:
        side_cus = list(range(0, 256, 256 // n))
    main_cus = [c for c in range(256) if c not in side_cus]
    m, s = cu_stream(main_cus), cu_stream(side_cus)
    loop.main, loop.side = m, s
    print("split", split)


def variant(graph=True, events=True, speedy=True, res_=True):
    for _ in range(2):
        one(graph, events, speedy, res_)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        one(graph, events, speedy, res_)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 10 * 1e3


def one(graph, events, speedy, res_):
    if res_:
        loop.res.predict_begin(loop.fb, stream=m)
        if events:
            m.wait_event(loop.ev_lm)
        loop.res.predict_finish(loop.lm, loop.ov, stream=m)
        loop.res.assemble(loop.ov, loop.g4, loop.g2, loop.pr, stream=m)
        if events:
            loop.ev_grid.record(m)
        loop.res.tile_feedback(loop.g4, loop.g2, loop.pr, loop.tisr, loop.fb, stream=m)
    if speedy:
        if events:
            s.wait_event(loop.ev_grid)
        loop.dyn.from_grid(loop.g4, loop.g2, stream=s)
        loop.dyn.window(24, stream=s, graph=graph)
        loop.dyn.to_grid(loop.f4, loop.f2, stream=s)
        loop.res.tile_local_model(loop.f4, loop.f2, loop.lm, stream=s)
        if events:
            loop.ev_lm.record(s)


for kw in ({}, {"events": False}, {"speedy": False}, {"res_": False}):
    print(kw, f"{variant(**kw):.3f} ms/step", flush=True)

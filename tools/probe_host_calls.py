"""Diagnostic: host time of each call inside HybridLoop.step in steady state (does
any call block the issuing thread?).  python tools/probe_host_calls.py"""
import os
import sys
import time
from collections import defaultdict

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
ws = [region_weights(r, bool(mask[r]), climatology=True) for r in range(1152)]
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
                  tisr=t(np.random.default_rng(13).standard_normal((1152, 16))))
g4, g2, pr = synthetic_grids(11)
f4, f2, _ = synthetic_grids(12)
loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
for _ in range(5):
    loop.step()
loop.sync()

acc = defaultdict(float)


def wrap(obj, name):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[name] += time.perf_counter() - t0
        return r
    setattr(obj, name, g)


for n in ("predict_begin", "predict_finish", "assemble", "tile_feedback", "tile_local_model"):
    wrap(loop.res, n)
for n in ("from_grid", "window", "to_grid"):
    wrap(loop.dyn, n)
N = 30
stamps = []
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(N):
    loop.step()
    stamps.append(time.perf_counter() - t0)
t_issue = time.perf_counter() - t0
loop.sync()
t_all = time.perf_counter() - t0
print(f"steps {N}: issue {t_issue / N * 1e3:.3f} ms/step, total {t_all / N * 1e3:.3f} ms/step")
for k, v in sorted(acc.items(), key=lambda x: -x[1]):
    print(f"  {k:18s} {v / N * 1e3:8.3f} ms/step host")
print("issue stamps (ms):", " ".join(f"{s * 1e3:.2f}" for s in stamps[:12]))

# untraced timeline of one steady-state step from timing events on both streams
E = lambda: torch.cuda.Event(enable_timing=True)  # noqa: E731
m, s = loop.main, loop.side
prio = os.environ.get("PROBE_PRIO")
for rep in range(2):
    evs = {}
    base = E()
    base.record(m)
    for k in range(4):
        evs[f"{k} m.begin_start"] = E(); evs[f"{k} m.begin_start"].record(m)
        loop.res.predict_begin(loop.fb, stream=m)
        evs[f"{k} m.begin_end"] = E(); evs[f"{k} m.begin_end"].record(m)
        m.wait_event(loop.ev_lm)
        evs[f"{k} m.finish_start"] = E(); evs[f"{k} m.finish_start"].record(m)
        loop.res.predict_finish(loop.lm, loop.ov, stream=m)
        loop.res.assemble(loop.ov, loop.g4, loop.g2, loop.pr, stream=m)
        loop.ev_grid.record(m)
        loop.res.tile_feedback(loop.g4, loop.g2, loop.pr, loop.tisr, loop.fb, stream=m)
        evs[f"{k} m.tile_end"] = E(); evs[f"{k} m.tile_end"].record(m)
        s.wait_event(loop.ev_grid)
        evs[f"{k} s.from_start"] = E(); evs[f"{k} s.from_start"].record(s)
        loop.dyn.from_grid(loop.g4, loop.g2, stream=s)
        evs[f"{k} s.win_start"] = E(); evs[f"{k} s.win_start"].record(s)
        loop.dyn.window(24, stream=s)
        evs[f"{k} s.win_end"] = E(); evs[f"{k} s.win_end"].record(s)
        loop.dyn.to_grid(loop.f4, loop.f2, stream=s)
        loop.res.tile_local_model(loop.f4, loop.f2, loop.lm, stream=s)
        loop.ev_lm.record(s)
        evs[f"{k} s.lm_end"] = E(); evs[f"{k} s.lm_end"].record(s)
    torch.cuda.synchronize()
    if rep:
        for k, e in sorted(evs.items(), key=lambda kv: base.elapsed_time(kv[1])):
            print(f"{base.elapsed_time(e) * 1e3:9.1f} us  {k}")

if os.environ.get("PROBE_SPLITS"):  # each variant creates 2 more HW queues: run alone
    # CU split: SPEEDY's stream on its own CUs, the reservoir stream on the rest
    import ctypes  # noqa: E402
    hip = ctypes.CDLL("libamdhip64.so")


    def cu_stream(cus, prio=0):
        mask = (ctypes.c_uint32 * 8)()
        for c in cus:
            mask[c // 32] |= 1 << (c % 32)
        h = ctypes.c_void_p()
        assert hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), 8, mask) == 0
        return torch.cuda.ExternalStream(h.value)


    def timed_steps(n=30):
        for _ in range(5):
            loop.step()
        loop.sync()
        t0 = time.perf_counter()
        for _ in range(n):
            loop.step()
        loop.sync()
        return (time.perf_counter() - t0) / n * 1e3


    m0, s0 = loop.main, loop.side
    print(f"split none: {timed_steps():.3f} ms/step")
    for kind, n in [(k, n) for n in (32, 48, 64, 80, 96, 128) for k in ("lo", "hi")] + [("lo", 64), ("hi", 64)]:
        side_cus = list(range(n)) if kind == "lo" else list(range(256 - n, 256))
        main_cus = [c for c in range(256) if c not in side_cus]
        loop.main, loop.side = cu_stream(main_cus), cu_stream(side_cus)
        a = timed_steps()
        loop.main, loop.side = m0, s0
        c = timed_steps()
        print(f"split {kind}:{n}: both masked {a:.3f}, none {c:.3f} ms/step")

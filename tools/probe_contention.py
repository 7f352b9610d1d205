"""Diagnostic: the SPEEDY window's time beside other work on the reservoir's CUs.
Full-size reservoirs (1152 regions), SPEEDY on CUs [0, 64), the partner on [64, 224) as
in the hybrid loop:
alone, beside predict_begin (update + v_ml readout), beside a plain HBM copy and
beside a plain HBM read of about the readout's byte count.
    python tools/probe_contention.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd import domain  # noqa: E402
from speedy_ml_amd._lib import check, lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.reservoir import Reservoirs  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, initial_state, phys_boundary, region_weights  # noqa: E402

dev = torch.device("cuda", 0)
mask = domain.load_sst_mask()
sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in range(1152)]
res = Reservoirs(list(range(1152)), mask, [s.n for s in sizes], [s.k for s in sizes])
for r in range(1152):
    w = region_weights(r, bool(mask[r]), climatology=True)
    res.load_region_weights(r, w)
    res.set_state(r, initial_state(r, w.n))
res.set_read_waves(0)
fb, lm, ov = res.alloc_io(dev)
st0, forcing = dyn_state()
dyn = Dynamics()
dyn.set_forcing(**forcing)
dyn.set_state(st0)
dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
L = lib()
s_side, s_main = ctypes.c_void_p(), ctypes.c_void_p()
check(L.sml_stream_create_cu_range(0, 64, ctypes.byref(s_side)))
check(L.sml_stream_create_cu_range(64, int(os.environ.get("PARTNER_CUS", "192")), ctypes.byref(s_main)))
side = torch.cuda.ExternalStream(s_side.value, device=dev)
main = torch.cuda.ExternalStream(s_main.value, device=dev)
nbytes = 3_700_000_000
src = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
dst = torch.empty_like(src)
src.uniform_()


def window_ms(partner, reps=8, window=True):
    ts = []
    for _ in range(reps + 2):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(main):
            p0.record()
            if partner:
                partner()
            p1.record()
        with torch.cuda.stream(side):
            e0.record()
            if window:
                dyn.window(24, stream=side)
            e1.record()
        torch.cuda.synchronize()
        ts.append((e0.elapsed_time(e1), p0.elapsed_time(p1)))
    ts = np.array(ts[2:])
    return np.median(ts[:, 0]), np.median(ts[:, 1])


def begin():
    res.predict_begin(fb, stream=main)
    res.predict_finish(lm, ov, stream=main)  # (small) closes the split step


def copy():
    dst.copy_(src, non_blocking=True)


def read_only():
    torch.sum(src)


w, p = window_ms(begin, window=False)
print(f"predict_begin alone on the partner CUs: {p:.3f} ms")
for name, fn in (("alone", None), ("beside predict_begin", begin), ("beside a 3.7 GB copy (7.4 GB traffic)", copy),
                 ("beside a 3.7 GB read (sum)", read_only), ("alone again", None)):
    w, p = window_ms(fn)
    print(f"window {w:.3f} ms  {name}  (partner {p:.3f} ms)")

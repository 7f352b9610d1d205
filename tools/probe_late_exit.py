"""Diagnostic: does a sleep kernel on the safety check's stream make run_model's exit
give up (zero check timeout)?  Prints the timings and the outcome."""
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "speedy-ml-1_amd"))
from speedy_ml_amd._lib import check, lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids  # noqa: E402

cuda = torch.device("cuda:0")
st0, forcing = dyn_state()
d = Dynamics()
d.set_forcing(**forcing)
d.set_state(st0)
d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_rad_state(None)
d.set_clock(1, True)
check(lib().sml_dyn_set_check_cus(d._h, 192, 64))
g4, g2, _ = synthetic_grids(5)
g4[:2, ..., 3] = 0.0
dg4, dg2 = torch.from_numpy(g4).to(cuda), torch.from_numpy(g2).to(cuda)
f4, f2 = torch.zeros_like(dg4), torch.zeros_like(dg2)
win = torch.cuda.Stream()
mode = sys.argv[1] if len(sys.argv) > 1 else "torch_stream"
ws = win if mode == "torch_stream" else None
d.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)
print("first safe", d.last_safe()[0])
s = ctypes.c_void_p()
check(lib().sml_dyn_check_stream(d._h, ctypes.byref(s)))
chk = torch.cuda.ExternalStream(s.value, device=cuda)
print("check stream", hex(s.value), "window stream", ws.cuda_stream if ws is not None else None)
torch.cuda.synchronize()
t0 = time.perf_counter()
with torch.cuda.stream(chk):
    torch.cuda._sleep(200_000_000)
chk.synchronize()
print(f"sleep alone {1e3 * (time.perf_counter() - t0):.1f} ms")
check(lib().sml_dyn_set_check_timeout(d._h, 0))
with torch.cuda.stream(chk):
    torch.cuda._sleep(200_000_000)
t0 = time.perf_counter()
d.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)
(ws or torch.cuda.current_stream()).synchronize()
t1 = time.perf_counter()
safe_late, mm = d.last_safe()
t2 = time.perf_counter()
want = g4.copy()
want[..., 3] = np.where(g4[..., 3] < 1e-6, 1e-6, g4[..., 3])
print(f"window stream done after {1e3 * (t1 - t0):.1f} ms, check after {1e3 * (t2 - t0):.1f} ms; safe {safe_late}; "
      f"forecast is the pass-through: {np.array_equal(f4.cpu().numpy(), want)}")
check(lib().sml_dyn_set_check_timeout(d._h, 1_000_000))
d.run_model(dg4, dg2, f4, f2, nleap=3, stream=ws)
print("next safe", d.last_safe()[0])
d.close()

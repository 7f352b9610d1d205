"""Diagnostic: which phases of the fused SPEEDY step grow beside an HBM stream.
In-kernel stamps (SML_DYN_STAMPS=1) of the window's last step, SPEEDY on CUs
[0, 64), alone and beside a partner on CUs [64, 256) that outlasts the window
(a plain read of 3.7 GB, twice; or predict_begin, PARTNER=begin).
    python tools/probe_phase_contention.py"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
os.environ["SML_DYN_STAMPS"] = "1"
from speedy_ml_amd._lib import check, lib  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.synthetic import dyn_state, phys_boundary  # noqa: E402

dev = torch.device("cuda", 0)
st, forcing = dyn_state()
d = Dynamics()
d.set_forcing(**forcing)
d.set_state(st)
d.set_physics(phys_boundary(d, forcing["phis"]))
d.set_clock(1, True)
L = lib()
L.sml_dbg_dyn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
s_side, s_main = ctypes.c_void_p(), ctypes.c_void_p()
check(L.sml_stream_create_cu_range(0, 64, ctypes.byref(s_side)))
check(L.sml_stream_create_cu_range(64, 192, ctypes.byref(s_main)))
side = torch.cuda.ExternalStream(s_side.value, device=dev)
main = torch.cuda.ExternalStream(s_main.value, device=dev)
NB = 3_700_000_000
MEM = os.environ.get("PARTNER_MEM", "default")  # default | uncached | finegrained: the partner's buffer
if MEM == "default":
    src = torch.empty(NB // 8, dtype=torch.float64, device=dev)
else:
    hip = ctypes.CDLL("libamdhip64.so")
    ptr = ctypes.c_void_p()
    assert hip.hipExtMallocWithFlags(ctypes.byref(ptr), ctypes.c_size_t(NB), {"uncached": 3, "finegrained": 1}[MEM]) == 0

    class _Buf:  # a torch view of the hipExtMallocWithFlags buffer
        __cuda_array_interface__ = {"shape": (NB // 8,), "typestr": "<f8", "data": (ptr.value, False), "version": 2}

    src = torch.as_tensor(_Buf(), device=dev)
src.uniform_()
# PARTNER_KIND: sum (torch.sum, the default) | nt | plain (tools/libstream_partner.so)
KIND = os.environ.get("PARTNER_KIND", "sum")
# NLEAP: leapfrog steps of the window (24, the hybrid's; 22 ends on a shortwave step)
NLEAP = int(os.environ.get("NLEAP", "24"))
if KIND != "sum":
    SP = ctypes.CDLL(os.path.join(REPO, "tools", "libstream_partner.so"))
    SP.sp_read.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    sink = torch.zeros(8, dtype=torch.float64, device=dev)
print("partner buffer:", MEM, "partner:", KIND)
K = {0: ("grid", ["gridx", "physics+sums", "specx"]),
     1: ("spec", ["load", "specy", "combine", "tail", "inv_inputs", "gridy"]),
     3: ("spec_last", ["load", "specy", "combine", "tail"])}


def run(partner, reps=6):
    rows, wins = [], []
    for _ in range(reps + 1):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if partner:
            with torch.cuda.stream(main):
                if KIND == "sum":
                    torch.sum(src)
                    torch.sum(src)
                else:  # tools/libstream_partner.so: nt or plain 16-B loads, 8 blocks per partner CU
                    for _ in range(2):
                        assert SP.sp_read(ctypes.c_void_p(src.data_ptr()), ctypes.c_size_t(NB), ctypes.c_void_p(sink.data_ptr()),
                                          1 if KIND == "nt" else 0, 192 * 8, s_main) == 0
        with torch.cuda.stream(side):
            e0.record()
            d.window(NLEAP, stream=side)
            e1.record()
        torch.cuda.synchronize()
        wins.append(e0.elapsed_time(e1))
        buf = np.zeros((4, 96, 8), dtype=np.int64)
        assert L.sml_dbg_dyn_stamps(d._h, buf.ctypes.data) == 0
        rec = {}
        ends = {}
        for kern, (name, phases) in K.items():
            nb = int((buf[kern, :, 0] > 0).sum())
            b = buf[kern, :nb].astype(np.float64)
            last = max(i for i in range(8) if b[:, i].max() > 0)
            for i, ph in enumerate(phases):
                if i + 1 <= last:
                    rec[f"{name}.{ph}"] = np.median((b[:, i + 1] - b[:, i]) / 100.0)
            rec[f"{name}.span"] = (b[:, last].max() - b[:, 0].min()) / 100.0
            ends[kern] = (b[:, 0].min(), b[:, last].max())
        rec["gap spec->grid"] = (ends[0][0] - ends[1][1]) / 100.0
        rec["gap grid->spec_last"] = (ends[3][0] - ends[0][1]) / 100.0
        rows.append(rec)
    keys = rows[0].keys()
    med = {k: float(np.median([r[k] for r in rows[1:]])) for k in keys}
    return float(np.median(wins[1:])), med


a_w, a = run(False)
b_w, b = run(True)
print(f"window alone {a_w:.3f} ms, beside the read stream {b_w:.3f} ms (+{(b_w - a_w) * 1e3 / 26:.2f} us per step)")
for k in a:
    print(f"{k:28s} alone {a[k]:6.2f} us  beside {b[k]:6.2f} us  (+{b[k] - a[k]:.2f})")

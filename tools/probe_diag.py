"""Diagnostic: the blocked diagonal factor's phases (k_chol_diag_b) from the profiling
build's stamps (-DSML_DSTAMPS: tools/build_variant.sh dst 'FLAGS_sml_train=-DSML_DSTAMPS'),
region 0's launch for block column K of a 4-region solve at naug 6000.
    SML_LIB=abx/dst/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_diag.py [K]"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd._lib import lib  # noqa: E402
from speedy_ml_amd.training import Trainer  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
L = lib()
L.sml_dbg_diag_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p]
naug, m = [6000] * 4, 400
g = torch.Generator(device="cuda").manual_seed(3)
S = torch.tanh(torch.randn(sum(naug) * m, dtype=torch.float64, device="cuda", generator=g))
T = torch.randn(len(naug) * m * 136, dtype=torch.float64, device="cuda", generator=g)
names = ["load"] + sum([[f"P{p} factor", f"P{p} panel", f"P{p} update", f"P{p} ->"] for p in range(4)], [])
for rep in range(3):
    assert L.sml_dbg_diag_stamps(K, None) == 0
    tr = Trainer(naug)
    tr.accumulate(S, T, m)
    tr.solve()
    torch.cuda.synchronize()
    buf = np.zeros(32, dtype=np.int64)
    assert L.sml_dbg_diag_stamps(K, buf.ctypes.data) == 0
    tr.close()
b = buf.astype(np.float64) / 100.0  # us
seq = [0, 1, 2, 3, 5, 6, 7, 9, 10, 11, 13, 17, 18, 19]
lab = {0: "start", 1: "loaded", 2: "P0 factor", 3: "P0 panel", 5: "P0 update", 6: "P1 factor", 7: "P1 panel",
       9: "P1 update", 10: "P2 factor", 11: "P2 panel", 13: "P2 update", 17: "P3 factor", 18: "inverse", 19: "stored"}
print(f"k_chol_diag_b, block column {K}, region 0 (us from start):")
print("  " + " | ".join(f"{lab[s]} {b[s] - b[0]:.1f}" for s in seq if b[s] > 0))

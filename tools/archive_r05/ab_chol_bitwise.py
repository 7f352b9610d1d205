"""Diagnostic: the training solve's W_out under two Cholesky configurations must be
bitwise equal (the variants reorder no arithmetic).  Env knobs are read at Trainer
creation (one argument per configuration, knobs space-separated):
    python tools/ab_chol_bitwise.py SML_SOLVE_SPLIT=0 'SML_SOLVE_SPLIT=1 SML_CHOL_TALL=1'
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd.training import Trainer  # noqa: E402

naug = [1000, 1290, 700, 1537]
m = 1800
g = torch.Generator(device="cuda").manual_seed(5)
S = torch.tanh(torch.randn(sum(naug) * m, dtype=torch.float64, device="cuda", generator=g))
T = torch.randn(len(naug) * m * 136, dtype=torch.float64, device="cuda", generator=g)
outs = []
for cfg in sys.argv[1:]:
    for kv in cfg.split():
        k, v = kv.split("=")
        os.environ[k] = v
    tr = Trainer(naug)
    tr.accumulate(S, T, m)
    w, info = tr.solve()
    torch.cuda.synchronize()
    outs.append((cfg, w.clone(), info.copy() if hasattr(info, "copy") else info))
    tr.close()
ref = outs[0][1]
for cfg, w, info in outs:
    d = (w - ref).abs().max().item()
    print(f"{cfg}: info {list(info)} max|dW| vs {outs[0][0]} = {d:.3e} bitwise {bool(torch.equal(w, ref))}")

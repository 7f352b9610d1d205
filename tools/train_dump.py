"""Diagnostic: W_out of a small training batch (the same seeded inputs as
tools/ab_chol_bitwise.py) saved to a .npy file, so two library builds can be compared
bit for bit:  SML_LIB=<other .so> python tools/train_dump.py a.npy; python tools/train_dump.py b.npy"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd.training import Trainer  # noqa: E402

naug = [1000, 1290, 700, 1537]
m = 1800
g = torch.Generator(device="cuda").manual_seed(5)
S = torch.tanh(torch.randn(sum(naug) * m, dtype=torch.float64, device="cuda", generator=g))
T = torch.randn(len(naug) * m * 136, dtype=torch.float64, device="cuda", generator=g)
tr = Trainer(naug)
tr.accumulate(S, T, m)
tr.accumulate(S, T, m)
w, info = tr.solve()
torch.cuda.synchronize()
np.save(sys.argv[1], w.cpu().numpy())
print("info", list(info))
tr.close()

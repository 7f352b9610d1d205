"""Child process of tests/test_hybrid_gpu.py::test_serialised_dispatch_takes_event_hops:
runs the small 1152-region loop of that file for 3 steps in a fresh process (whose
environment the parent sets, e.g. AMD_SERIALIZE_KERNEL=3) and saves the snapshots and
the hop mode in effect to argv[1] (.npz)."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "speedy-ml-1_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "oracle"))


def main(out):
    import torch

    from test_hybrid_gpu import _loop, _snapshot

    cuda = torch.device("cuda:0")
    loop, _ = _loop(cuda, True)
    requested, effective = loop.hop_mode()
    snaps = {}
    for s in range(3):
        loop.step()
        loop.sync()
        for k, v in _snapshot(loop).items():
            snaps[f"{k}{s}"] = v
    loop.close()
    np.savez(out, requested=requested, effective=effective, **snaps)
    print("hop child done", requested, effective, flush=True)


if __name__ == "__main__":
    main(sys.argv[1])

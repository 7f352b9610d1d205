"""Diagnostic: the hybrid loop's hop mode in effect in this process's environment
(sml_hybrid_hop_mode), e.g. under `rocprofv3 --pmc ...` (ROCPROF_COUNTER_COLLECTION)
or AMD_SERIALIZE_KERNEL.  Prints the requested / effective mode; steps a small loop
twice only when the effective mode is event hops (the mode that cannot stall under
serialised dispatch), so it never issues a wait-value hop under a serialiser.
    python tools/hop_mode_check.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))


def main():
    import torch

    from speedy_ml_amd._lib import SML_HOP_EVENTS
    from test_hybrid_gpu import _loop

    loop, _ = _loop(torch.device("cuda:0"), True)
    req, eff = loop.hop_mode()
    names = {0: "auto", 1: "wait-value", 2: "events"}
    env = {k: os.environ.get(k) for k in ("ROCPROF_COUNTER_COLLECTION", "AMD_SERIALIZE_KERNEL", "SML_HYBRID_EVENTS")}
    print(f"hop mode: requested {names[req]}, effective {names[eff]}; env {env}", flush=True)
    if eff == SML_HOP_EVENTS:
        for _ in range(2):
            loop.step()
        loop.sync()
        print("stepped 2 hybrid steps with event hops", flush=True)
    loop.close()


if __name__ == "__main__":
    main()

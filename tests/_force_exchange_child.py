"""Child of tests/test_force_exchange_gpu.py: the one-rank loop through the real RCCL
transport.  torch.distributed's NCCL group is initialised as bench.py does at world >
1 (MASTER_ADDR 127.0.0.1, device_id), the library's own communicator joins it
(NativeComm(1, 0): ncclCommInitRank), and sml_hybrid_set_force_exchange makes
sml_hybrid_step take its world > 1 branch: outvecs -> ncclAllGather on the main
stream -> sml_hybrid_advance_slabs -> separate assembly.  The same loop without a
communicator (identity exchange, assembly fused into the finish) runs after it; both
with the slab ocean (140-wide rows, a slab step at step 4) and the pipelined loop.
Writes argv[1] (npz) with every step's buffers of both loops and the allgather count."""
import os
import socket
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))

STEPS = 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run(cuda, comm):
    import torch

    from speedy_ml_amd import domain
    from speedy_ml_amd._lib import check, lib, ptr
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights, slab_fields,
                                         slab_start_outvec, slab_weights, synthetic_grids)

    mask = domain.load_sst_mask()
    ws = [region_weights(r, bool(mask[r]), n_override=96, seed=5, climatology=True) for r in range(1152)]
    res = Reservoirs(list(range(1152)), mask, [w.n for w in ws], [w.k for w in ws])
    for i, w in enumerate(ws):
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(w.region, w.n))
    sids = [r for r in range(1152) if mask[r]]
    sws = [slab_weights(r, n_override=200) for r in sids]
    slab = Reservoirs(sids, [0] * len(sids), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0, nout=4,
                      ninp=[w.ninp for w in sws], out_index=[35] * 4)
    for j, w in enumerate(sws):
        slab.load_region_weights(j, w)
        slab.set_state(j, initial_state(sids[j], w.n, seed=17))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    base, smask, sice, tice = slab_fields()
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.ascontiguousarray(tice))))
    tisr = t(np.random.default_rng(13).standard_normal((1152, 16)))
    so = SlabOcean(slab, t(base), t(smask), timestep=6, timestep_slab=24)
    ex = OutvecExchange(1152, 1, 0, device=cuda) if comm is None else None
    loop = HybridLoop(res, dyn, ex, cuda, tisr=tisr, nleap=4, comm=comm, slab=so)
    if comm is not None:
        loop.set_force_exchange(True)
    loop.set_pipelined(True)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.start_slab(t(np.stack([slab_start_outvec(r) for r in sids])))
    loop.sync()
    out = {}
    for s in range(STEPS):
        loop.step()
        loop.sync()
        torch.cuda.synchronize()
        for k in ("ov", "fb", "lm", "g4", "g2", "pr", "f4", "f2"):
            out[f"{k}{s}"] = getattr(loop, k).cpu().numpy().copy()
        out[f"sst{s}"] = loop.slab_state()["sst"]
        out[f"run{s}"] = np.array(loop.run_speedy())
    n = loop.exchanges()
    loop.close()
    dyn.close()
    res.close()
    slab.close()
    return out, n


def main():
    import torch
    import torch.distributed as dist

    from speedy_ml_amd.comm import NativeComm

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
                      LOCAL_RANK="0")
    cuda = torch.device("cuda", 0)
    torch.cuda.set_device(cuda)
    dist.init_process_group("nccl", device_id=cuda)
    comm = NativeComm(1, 0)
    forced, n_forced = run(cuda, comm)
    ident, n_ident = run(cuda, None)
    comm.close()
    dist.destroy_process_group()
    save = {"n_forced": np.array(n_forced), "n_ident": np.array(n_ident)}
    save.update({"forced_" + k: v for k, v in forced.items()})
    save.update({"ident_" + k: v for k, v in ident.items()})
    np.savez(sys.argv[1], **save)
    print("force-exchange child done", n_forced, n_ident, flush=True)


if __name__ == "__main__":
    main()

"""The sharded path on CPU: world_size 2 (and 3, uneven shares) over gloo.

Each rank owns the regions processor_decomposition gives it (res_domain.f90:31-62),
computes its regions' outvecs (oracle predict), exchanges them with the bench's
OutvecExchange all-gather, assembles the global grid and re-tiles its own regions'
feedback -- and must get exactly what a single process gets for those regions."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

NREG = 1152


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _outvecs_for(regions):
    rng = np.random.default_rng(0)
    allv = rng.standard_normal((NREG, 136))
    return allv[regions]


def _worker(rank, world, port, out_dir):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "speedy-ml-1_amd"))
    sys.path.insert(0, os.path.join(repo, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle
    from speedy_ml_amd.exchange import OutvecExchange

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ex = OutvecExchange(NREG, world, rank)
    local = torch.from_numpy(_outvecs_for(ex.regions))
    glob = ex(local).numpy()
    g4, g2, pr = oracle.assemble(glob)
    mean, std = np.zeros(36), np.ones(36)
    fbs = [oracle.tile_feedback(r, g4, g2, pr, mean, std, np.zeros(16)) for r in ex.regions[:40]]
    np.save(os.path.join(out_dir, f"rank{rank}_glob.npy"), glob)
    np.save(os.path.join(out_dir, f"rank{rank}_fb.npy"), np.concatenate(fbs))
    np.save(os.path.join(out_dir, f"rank{rank}_regions.npy"), np.array(ex.regions))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_exchange_matches_single_process(tmp_path, world):
    import oracle

    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ref = _outvecs_for(np.arange(NREG))
    g4, g2, pr = oracle.assemble(ref)
    seen = []
    for rank in range(world):
        glob = np.load(tmp_path / f"rank{rank}_glob.npy")
        np.testing.assert_array_equal(glob, ref)  # every rank holds all outvecs in region order
        regions = np.load(tmp_path / f"rank{rank}_regions.npy")
        seen += list(regions)
        fb = np.load(tmp_path / f"rank{rank}_fb.npy")
        want = np.concatenate([oracle.tile_feedback(int(r), g4, g2, pr, np.zeros(36), np.ones(36), np.zeros(16))
                               for r in regions[:40]])
        np.testing.assert_array_equal(fb, want)
    assert sorted(seen) == list(range(NREG))

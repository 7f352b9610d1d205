"""The all-gather's layout of the native sharded step (sml_exchange_plan, the host half
of sml_hybrid_step / sml_hybrid_advance_slabs at world > 1), on CPU.

processor_decomposition (res_domain.f90:31-62) gives rank q of N the regions
q*per .. q*per+per-1 and, for q in 1..left, one of the `left` leftover regions at the
end.  The native step sends every rank's outvecs zero-padded to the largest share
(maxc), receives [N][maxc][nout] and, when the shares are uneven, permutes the slab
rows into global region order with perm (k_gather_rows).  Checked here:

* perm / maxc / contiguous against an independent construction from
  speedy_ml_amd.domain.processor_decomposition and against the Python exchange's
  own permutation (speedy_ml_amd.exchange.OutvecExchange), N = 1, 2, 3, 5, 7, 8;
* the permutation applied to padded slabs gives back the global outvec array
  (what k_gather_rows computes on the device);
* the whole native recipe -- pad, all_gather_into_tensor, permute with the library's
  perm -- across 5 gloo ranks (uneven shares) equals the single-process array."""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from speedy_ml_amd import domain

NREG = 1152
NOUT = 136


def _plan(world, numregions=NREG):
    from speedy_ml_amd._lib import check, lib, ptr

    maxc, contig = ctypes.c_int(), ctypes.c_int()
    perm = np.full(numregions, -7, dtype=np.int32)
    check(lib().sml_exchange_plan(numregions, world, ctypes.byref(maxc), ctypes.byref(contig), ptr(perm)))
    return maxc.value, bool(contig.value), perm


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8])
def test_plan_matches_processor_decomposition(world):
    maxc, contig, perm = _plan(world)
    shares = [domain.processor_decomposition(NREG, world, q) for q in range(world)]
    assert maxc == max(len(s) for s in shares)
    want = np.full(NREG, -1)
    for q, s in enumerate(shares):
        for i, r in enumerate(s):
            assert want[r] == -1, "region owned twice"
            want[r] = q * maxc + i
    assert (want >= 0).all()
    np.testing.assert_array_equal(perm, want)
    assert contig == (NREG % world == 0)
    if contig:
        np.testing.assert_array_equal(perm, np.arange(NREG))
    if world > 1:
        from speedy_ml_amd.exchange import OutvecExchange

        ex = OutvecExchange(NREG, world, 0)
        assert ex.maxc == maxc and ex.contiguous == contig
        np.testing.assert_array_equal(ex.perm.numpy(), perm)


@pytest.mark.parametrize("world", [3, 5, 7])
def test_permuting_padded_slabs_gives_region_order(world):
    maxc, _, perm = _plan(world)
    rng = np.random.default_rng(world)
    glob = rng.standard_normal((NREG, NOUT))
    slabs = np.zeros((world, maxc, NOUT))
    for q in range(world):
        s = domain.processor_decomposition(NREG, world, q)
        slabs[q, :len(s)] = glob[s]
    np.testing.assert_array_equal(slabs.reshape(world * maxc, NOUT)[perm], glob)


def test_plan_rejects_bad_arguments():
    from speedy_ml_amd._lib import lib

    m, c = ctypes.c_int(), ctypes.c_int()
    assert lib().sml_exchange_plan(NREG, 0, ctypes.byref(m), ctypes.byref(c), None) == -1
    assert lib().sml_exchange_plan(4, 5, ctypes.byref(m), ctypes.byref(c), None) == -1
    assert lib().sml_exchange_plan(NREG, 2, None, ctypes.byref(c), None) == -1


def test_local_rank_descriptor_has_no_transport():
    """sml_comm_create_local: world / rank only; the all-gather refuses it."""
    from speedy_ml_amd._lib import SML_OK, lib

    h = ctypes.c_void_p()
    assert lib().sml_comm_create_local(8, 3, ctypes.byref(h)) == SML_OK
    w, r = ctypes.c_int(), ctypes.c_int()
    assert lib().sml_comm_rank(h, ctypes.byref(w), ctypes.byref(r)) == SML_OK
    assert (w.value, r.value) == (8, 3)
    buf = (ctypes.c_double * 4)()
    assert lib().sml_comm_allgather(h, buf, buf, 4, None) == -4  # SML_ERR_STATE
    assert b"without a transport" in lib().sml_last_error()
    assert lib().sml_comm_destroy(h) == SML_OK
    assert lib().sml_comm_create_local(2, 2, ctypes.byref(h)) == -1


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(repo, "speedy-ml-1_amd"))
    import torch
    import torch.distributed as dist

    from speedy_ml_amd import domain as dom

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    maxc, _, perm = _plan(world)
    glob = np.random.default_rng(0).standard_normal((NREG, NOUT))
    mine = dom.processor_decomposition(NREG, world, rank)
    send = torch.zeros((maxc, NOUT), dtype=torch.float64)  # sml_hybrid_step's d_send, zero padding
    send[:len(mine)] = torch.from_numpy(glob[mine])
    recv = torch.zeros((world * maxc, NOUT), dtype=torch.float64)  # d_recv [world][maxc][nout]
    dist.all_gather_into_tensor(recv, send)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), recv.numpy()[perm])  # k_gather_rows
    dist.barrier()
    dist.destroy_process_group()


def test_native_recipe_over_gloo_uneven_shares(tmp_path):
    world = 5
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    want = np.random.default_rng(0).standard_normal((NREG, NOUT))
    for rank in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"rank{rank}.npy"), want)

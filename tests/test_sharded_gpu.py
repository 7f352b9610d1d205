"""configs[3]'s sharded per-rank path, every rank on the one GPU.

BASELINE configs[3] runs the hybrid step with res_domain's processor_decomposition
over N ranks (res_domain.f90:31-62; rank q of 8 owns regions 144q .. 144q+143) and
one outvec all-gather per step (replacing sendrecievegrid's gather/scatter,
mpires.f90:338-716).  Here all N ranks' native loops (sml_hybrid_*, a
transport-less rank descriptor each, sml_comm_create_local) run on cuda:0 with their
full-size shares; the all-gather is stood in for by a device [N][maxc][136] slab
buffer filled from every rank's `ov` (zero-padded to maxc, exactly what
ncclAllGather delivers in sml_hybrid_step), and each rank advances with
sml_hybrid_advance_slabs -- the world > 1 code of the native step, including the
uneven-share permutation (k_gather_rows) at N = 7.

Done when, over 3 hybrid steps, every rank's outvecs, feedback and local-model
vectors, reservoir states, assembled and forecast grids and run_speedy are
bitwise those of the one-rank HybridLoop over all 1152 regions (the window is
deterministic, so every rank's redundant SPEEDY forecast is the same).  The RCCL
transport itself is the only piece not exercised (it needs N GPUs)."""
import numpy as np
import pytest

from speedy_ml_amd import domain
from speedy_ml_amd.synthetic import initial_state, region_weights

pytestmark = pytest.mark.gpu

NREG = 1152
STEPS = 3
SAMPLE_X = (0, 143, 144, 575, 1000, 1151)


def _weights(r, mask):
    return region_weights(r, bool(mask[r]), climatology=True)


def _setup(cuda, regions, mask, comm):
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary, synthetic_grids

    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in regions]
    res = Reservoirs(list(regions), mask[regions], [s.n for s in sizes], [s.k for s in sizes])
    for i, r in enumerate(regions):
        res.load_region_weights(i, _weights(r, mask))
        res.set_state(i, initial_state(r, sizes[i].n))
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    dyn.set_physics(phys_boundary(dyn, forcing["phis"]))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)  # noqa: E731
    tisr = np.random.default_rng(13).standard_normal((NREG, 16))[regions]
    ex = OutvecExchange(NREG, 1, 0, device=cuda) if comm is None else None
    loop = HybridLoop(res, dyn, ex, cuda, tisr=t(tisr), comm=comm)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.sync()
    return loop


def _want_res_cus(nlocal, ncu, speedy_cus=64):
    """sml_hybrid_create's CU split: one reservoir CU per 6 of the rank's regions, a
    multiple of 8, at least 64, at most every CU SPEEDY leaves."""
    c = -(-nlocal // 6)
    return min(ncu - speedy_cus, max(64, -(-c // 8) * 8))


def _close(loop):
    loop.close()
    loop.dyn.close()
    loop.res.close()


def _snap(loop):
    import torch

    torch.cuda.synchronize()
    return {k: getattr(loop, k).cpu().numpy().copy() for k in ("ov", "fb", "lm", "g4", "g2", "pr", "f4", "f2")}


@pytest.fixture(scope="module")
def one_rank(cuda):
    """The single-rank HybridLoop over all 1152 full-size regions: 3 steps."""
    mask = domain.load_sst_mask()
    loop = _setup(cuda, np.arange(NREG), mask, None)
    import torch

    ncu = torch.cuda.get_device_properties(cuda).multi_processor_count
    assert (loop.speedy_cus, loop.res_cus) == (64, _want_res_cus(NREG, ncu))  # 192 of 256
    snaps, runs = [], []
    for _ in range(STEPS):
        loop.step()
        loop.sync()
        snaps.append(_snap(loop))
        runs.append(loop.run_speedy())
    states = {r: loop.res.get_state(r) for r in SAMPLE_X}
    offs = loop.res.fb_offsets.copy()
    _close(loop)
    return snaps, runs, states, offs


@pytest.mark.parametrize("world", [8, 7])
def test_every_rank_of_the_sharded_step_is_bitwise_the_one_rank_loop(cuda, one_rank, world):
    import torch

    from speedy_ml_amd.comm import LocalRank, exchange_plan

    snaps1, runs1, states1, offs1 = one_rank
    mask = domain.load_sst_mask()
    maxc, contiguous, perm = exchange_plan(NREG, world)
    assert contiguous == (NREG % world == 0)
    shares = [np.array(domain.processor_decomposition(NREG, world, q)) for q in range(world)]
    comms = [LocalRank(world, q) for q in range(world)]
    loops = [_setup(cuda, shares[q], mask, comms[q]) for q in range(world)]
    ncu = torch.cuda.get_device_properties(cuda).multi_processor_count
    for q, lp in enumerate(loops):  # a share's reservoir stream: 64 CUs (144 / 165 regions)
        assert (lp.speedy_cus, lp.res_cus) == (64, _want_res_cus(len(shares[q]), ncu)), q
    recv = torch.zeros((world * maxc, 136), dtype=torch.float64, device=cuda)
    for step in range(STEPS):
        for lp in loops:
            lp.predict()
        for lp in loops:
            lp.xstream.synchronize()
        recv.zero_()  # the padding rows of a short share
        for q, lp in enumerate(loops):
            recv[q * maxc:q * maxc + len(shares[q])] = lp.ov  # ncclAllGather's [rank][maxc] slabs
        torch.cuda.synchronize()
        for lp in loops:
            lp.advance_slabs(recv)
        for lp in loops:
            lp.sync()
        want = snaps1[step]
        for q, lp in enumerate(loops):
            got = _snap(lp)
            s = shares[q]
            tag = f"world {world} rank {q} step {step + 1}"
            np.testing.assert_array_equal(got["ov"], want["ov"][s], err_msg=tag + " ov")
            np.testing.assert_array_equal(got["lm"], want["lm"][s], err_msg=tag + " lm")
            fb1 = np.concatenate([want["fb"][offs1[r]:offs1[r + 1]] for r in s])
            np.testing.assert_array_equal(got["fb"], fb1, err_msg=tag + " fb")
            for k in ("g4", "g2", "pr", "f4", "f2"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"{tag} {k}")
            assert lp.run_speedy() == runs1[step], tag
    for q, lp in enumerate(loops):
        for r in SAMPLE_X:
            hit = np.nonzero(shares[q] == r)[0]
            if len(hit):
                np.testing.assert_array_equal(lp.res.get_state(int(hit[0])), states1[r], err_msg=f"x region {r}")
    for lp in loops:
        _close(lp)
    for c in comms:
        c.close()


def test_transportless_rank_refuses_the_native_step(cuda):
    """sml_hybrid_step needs a transport at world > 1: a LocalRank loop says so."""
    from speedy_ml_amd._lib import SmlError
    from speedy_ml_amd.comm import LocalRank

    mask = domain.load_sst_mask()
    comm = LocalRank(8, 1)
    share = np.array(domain.processor_decomposition(NREG, 8, 1))
    loop = _setup(cuda, share, mask, comm)
    with pytest.raises(SmlError, match="no transport"):
        loop.step()
    _close(loop)
    comm.close()


# ---------------------------------------------------------------------------
# configs[3] as bench.py runs it: the slab ocean on (exchange rows of 140: each
# region's 136-value outvec and its slab sst, sendrecievegrid's SST half,
# mpires.f90:358-383 workers -> root, :458-472 wholegrid_sst, :575-581 / :733-736 the
# SST back into every rank's feedback) and the pipelined loop.  One rank owns no sst
# region at all (rank 1 of 8: its regions' sst flags are cleared in the mask the
# one-rank loop uses too), so on a slab step it predicts no slab yet must rebuild
# wholegrid_sst from the other ranks' rows.
SLAB_STEPS = 4          # timestep_slab 24 h: the 4th hybrid step is a slab step
SLAB_HOURS = 24


def _slab_mask():
    m = domain.load_sst_mask().copy()
    m[domain.processor_decomposition(NREG, 8, 1)] = 0
    return m


def _slab_setup(cuda, regions, mask, comm):
    import torch

    from speedy_ml_amd._lib import check, lib, ptr
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import (dyn_state, phys_boundary, slab_fields, slab_start_outvec, slab_weights,
                                         synthetic_grids)

    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in regions]
    res = Reservoirs(list(regions), mask[regions], [s.n for s in sizes], [s.k for s in sizes])
    for i, r in enumerate(regions):
        res.load_region_weights(i, _weights(r, mask))
        res.set_state(i, initial_state(r, sizes[i].n))
    sids = [int(r) for r in regions if mask[r]]
    sws = [slab_weights(r) for r in sids]
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
    tisr = np.random.default_rng(13).standard_normal((NREG, 16))[regions]
    ex = OutvecExchange(NREG, 1, 0, device=cuda) if comm is None else None
    so = SlabOcean(slab, t(base), t(smask), timestep=6, timestep_slab=SLAB_HOURS)
    loop = HybridLoop(res, dyn, ex, cuda, tisr=t(tisr), comm=comm, slab=so)
    assert loop.exchange_width == 140
    loop.set_pipelined(True)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.start_slab(t(np.stack([slab_start_outvec(r) for r in sids]) if sids else np.zeros((0, 4))))
    loop.sync()
    loop._keep = (slab, so)
    return loop, sids


def _slab_snap(loop):
    s = _snap(loop)
    st = loop.slab_state()
    s["sst"], s["sov"] = st["sst"], st["outvec"]
    return s


@pytest.fixture(scope="module")
def one_rank_slab(cuda):
    """The one-rank slab + pipelined loop over all 1152 full-size regions, SLAB_STEPS steps."""
    mask = _slab_mask()
    loop, sids = _slab_setup(cuda, np.arange(NREG), mask, None)
    snaps, runs = [], []
    for _ in range(SLAB_STEPS):
        loop.step()
        loop.sync()
        snaps.append(_slab_snap(loop))
        runs.append(loop.run_speedy())
    offs = loop.res.fb_offsets.copy()
    _close(loop)
    loop._keep[0].close()
    return snaps, runs, offs, sids


@pytest.mark.parametrize("world", [8, 7])
def test_sharded_slab_pipelined_step_is_bitwise_the_one_rank_loop(cuda, one_rank_slab, world):
    import torch

    from speedy_ml_amd.comm import LocalRank, exchange_plan

    snaps1, runs1, offs1, sids1 = one_rank_slab
    mask = _slab_mask()
    maxc, contiguous, perm = exchange_plan(NREG, world)
    shares = [np.array(domain.processor_decomposition(NREG, world, q)) for q in range(world)]
    comms = [LocalRank(world, q) for q in range(world)]
    built = [_slab_setup(cuda, shares[q], mask, comms[q]) for q in range(world)]
    loops = [b[0] for b in built]
    # odd ranks run the chain on SPEEDY's stream (sml_hybrid_set_chain): the same bits
    from speedy_ml_amd._lib import SML_CHAIN_SPEEDY

    for q in range(1, world, 2):
        loops[q].set_chain(SML_CHAIN_SPEEDY)
    if world == 8:
        assert built[1][1] == [], "rank 1 of 8 must own no sst region"
    recv = torch.zeros((world * maxc, 140), dtype=torch.float64, device=cuda)
    slab_step_seen = False
    for step in range(SLAB_STEPS):
        for lp in loops:
            lp.predict()
        for lp in loops:
            lp.xstream.synchronize()
        recv.zero_()
        for q, lp in enumerate(loops):
            recv[q * maxc:q * maxc + len(shares[q])] = lp.ov  # ncclAllGather's [rank][maxc] slabs
        torch.cuda.synchronize()
        for lp in loops:
            lp.advance_slabs(recv)
        for lp in loops:
            lp.sync()
        want = snaps1[step]
        slab_step_seen |= ((step + 1) * 6) % SLAB_HOURS == 0
        for q, lp in enumerate(loops):
            got = _slab_snap(lp)
            s = shares[q]
            tag = f"world {world} rank {q} step {step + 1}"
            np.testing.assert_array_equal(got["ov"], want["ov"][s], err_msg=tag + " ov (outvec + slab sst)")
            np.testing.assert_array_equal(got["lm"], want["lm"][s], err_msg=tag + " lm")
            fb1 = np.concatenate([want["fb"][offs1[r]:offs1[r + 1]] for r in s])
            np.testing.assert_array_equal(got["fb"], fb1, err_msg=tag + " fb")
            for k in ("g4", "g2", "pr", "f4", "f2", "sst"):
                np.testing.assert_array_equal(got[k], want[k], err_msg=f"{tag} {k}")
            mine = [sids1.index(r) for r in built[q][1]]
            np.testing.assert_array_equal(got["sov"], want["sov"][mine], err_msg=tag + " slab outvec")
            assert lp.run_speedy() == runs1[step], tag
    assert slab_step_seen
    # the slab step changed the sst the window sees (else the test would not cover it)
    assert not np.array_equal(snaps1[SLAB_STEPS - 1]["sst"], snaps1[0]["sst"])
    for lp in loops:
        _close(lp)
        lp._keep[0].close()
    for c in comms:
        c.close()

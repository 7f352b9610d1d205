#!/usr/bin/env python3
"""bench.py -- SPEEDY-ML hybrid hot path on MI355X (one process per GPU).

One "step" = one hybrid timestep (BASELINE.json
configs[2] on one GPU, configs[3] sharded over N):

  1. predict for every local region: A x + W_in u -> tanh -> W_out [model; x~],
     unstandardize                       (mod_reservoir.f90:1416-1487, 2 kernels)
  2. exchange: all-gather of every rank's outvecs over RCCL (N > 1)
                                         (replaces mpires.f90:338-716 MPI p2p)
  3. assemble the global T30L8 grid + clips (mpires.f90:300-478)
  4. the SPEEDY 6-h window on the assembled grid (run_model -> agcm_main,
     mpires.f90:1516-1628): iogrid(30) entry transforms + safety check, stepone +
     24 leapfrog steps of dyn_step WITH phypar's physics (dyn_stloop.f90:26-92),
     iogrid(31) exit transforms -- every transform, the dynamics and the column
     physics on the GPU, replicated on every rank
  5. re-tile every local region's next feedback (overlap tiles, standardized) and
     its standardized SPEEDY local vector (mpires.f90:558-751)

Data are synthetic: weights random with the trained structure, 6000-node-class
reservoirs (n = 5760/6160/6048/5880), a seeded T30L8 analysis state, synthetic
boundary fields for the physics.  fp64 arithmetic throughout; reservoir weights
held at their fp32 file precision (exact).  The reservoir side alone (configs[1])
is reported beside the headline as `reservoir_only`.

Usage: python bench.py [--gpus N --steps K --warmup W]
       python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

`python bench.py --gpus N` (N > 1, WORLD_SIZE unset) launches its N ranks itself:
the parent starts N fresh child processes of this script, one per GPU, with RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set -- the role
startmpi plays under mpirun in the reference (src/mpires.f90:21-37) -- before it
touches the GPU itself (it never does), relays rank 0's JSON line and exits non-zero
when any rank fails or the launch times out.  Under torch.distributed.run (WORLD_SIZE
set) every process is already one rank and runs directly.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import signal
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # a hybrid step is ~1.2 ms: 300 timed steps (0.35 s) after 20 warmup steps give
    # the steady state (30 steps after 5 read ~2 % low: clocks and queues still ramping)
    p.add_argument("--steps", type=int, default=300)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--regions", type=int, default=1152)
    p.add_argument("--weights", choices=("f32", "f64"), default="f32")
    p.add_argument("--cpu-threads", type=int,
                   default=len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count(),
                   help="OpenMP threads of the CPU baseline's predict leg (0 = skip the CPU baseline; default: "
                        "every core of this process's affinity mask; 1 thread and OMP_NUM_THREADS, the box's "
                        "CPU share, are timed beside it)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--overlap", action=argparse.BooleanOptionalAction, default=True,
                   help="issue the reservoir update + v_ml readout beside SPEEDY's window on two streams "
                        "(speedy_ml_amd/hybrid.py; default, +2.7 %% at 1 GPU, profiles/r01o); --no-overlap: one "
                        "stream, one-pass readout")
    p.add_argument("--speedy-cus", type=int, default=64,
                   help="with --overlap: CUs [0, N) for SPEEDY's stream, the rest for the reservoir's "
                        "(speedy_ml_amd/hybrid.py; 0 = no split)")
    p.add_argument("--train-regions", type=int, default=144,
                   help="regions per rank in the supplementary W_out-training leg, one batch resident in HBM "
                        "(144 x 8 ranks = all 1152; 0 = skip)")
    p.add_argument("--train-steps", type=int, default=4096, help="training time steps per region in that leg")
    p.add_argument("--train-batches", type=int, default=4,
                   help="chunking_matmul batches the training steps are accumulated in (one Gram launch each)")
    p.add_argument("--train-panel", type=int, default=8,
                   help="block columns per Cholesky panel in that leg (sml_train_set_panel)")
    p.add_argument("--reservoir-steps", type=int, default=50,
                   help="steps timed in the supplementary reservoir-only (configs[1]) leg (0 = skip)")
    p.add_argument("--exchange", choices=("native", "torch"), default="native",
                   help="N > 1: the outvec all-gather as the library's own ncclAllGather on the loop's main "
                        "stream (speedy_ml_amd.comm, sml_hybrid_step; default) or torch.distributed's "
                        "all_gather between predict and advance (its NCCL stream, two event hops)")
    p.add_argument("--sim-ranks", type=int, default=1,
                   help="diagnostic: run rank 0's share of an N-rank decomposition on this one GPU, the "
                        "all-gather replaced by a local copy (other ranks' outvecs stale); never the headline")
    p.add_argument("--pipelined", action=argparse.BooleanOptionalAction, default=True,
                   help="each step also issues the next step's reservoir begin (sml_hybrid_set_pipelined): "
                        "the loop a long run is in, also for the first timed step after the warmup's sync")
    p.add_argument("--chain", choices=("auto", "two-streams", "speedy"), default="auto",
                   help="where the step's serial chain (v_p finish, exchange, assembly) runs (sml_hybrid_set_chain): "
                        "auto = the reservoir's stream between two hops (measured faster at N = 1 and 8-rank shares), "
                        "speedy = SPEEDY's stream right behind the window")
    p.add_argument("--slab", action=argparse.BooleanOptionalAction, default=True,
                   help="the slab ocean in the loop, as the reference runs by default (mod_reservoir.f90:41): a "
                        "slab reservoir per sst region, predict_slab_ml every 168 h (28 steps), its sst in the "
                        "window (sml_hybrid_set_slab)")
    p.add_argument("--date-forcing", action=argparse.BooleanOptionalAction, default=True,
                   help="run_model's calendar drives each window's forcing (agcm_init: the coupler's monthly "
                        "climatologies at the date, the hybrid SST, fordate; sml_hybrid_set_calendar), from "
                        "1982-01-01 00 h as the loop's first hour; --no-date-forcing holds the start's forcing")
    p.add_argument("--speedy-steps", type=int, default=48,
                   help="leapfrog steps timed in the supplementary SPEEDY-step leg (0 = skip)")
    p.add_argument("--poll-run-speedy", action=argparse.BooleanOptionalAction, default=True,
                   help="after every timed step the host reads run_speedy and ends the loop when it is false, "
                        "as parallelmain.f90:268-270 does (sml_hybrid_run_speedy waits for that step's safety "
                        "check); --no-poll-run-speedy times the enqueued chain alone")
    p.add_argument("--launch-timeout", type=float, default=1500.0,
                   help="--gpus N > 1 without WORLD_SIZE: seconds before the launcher ends its ranks")
    p.add_argument("--dry-run", choices=("env", "gloo", "fail"), default=None,
                   help=argparse.SUPPRESS)  # launcher self-test (tests/test_bench_launch.py): no GPU, no torch.cuda
    return p.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args) -> int:
    """One fresh process per GPU (startmpi's role, mpires.f90:21-37): rank r gets
    RANK = LOCAL_RANK = r, WORLD_SIZE = N and a 127.0.0.1 rendezvous.  Runs before
    anything touches the GPU and never execs; rank 0's stdout (the JSON line) is
    this process's stdout, the other ranks' goes to stderr.  Returns the exit code:
    0 when every rank succeeded, else the first failure's (or 124 on a timeout), after
    ending the ranks still running."""
    n = args.gpus
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # the box's driver supports dmabuf IPC only
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr, start_new_session=False))
    print(f"[bench] launched {n} ranks (pids {[p.pid for p in procs]}), rendezvous 127.0.0.1:{port}",
          file=sys.stderr, flush=True)

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_signal(signum, _frame):
        stop_all(signum)

    old = {s: signal.signal(s, on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    t0, rc = time.time(), 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, c = bad[0]
                print(f"[bench] rank {r} exited with {c}: ending the other ranks", file=sys.stderr, flush=True)
                rc = c if c > 0 else 128 - c
                break
            if all(c == 0 for c in codes):
                break
            if time.time() - t0 > args.launch_timeout:
                print(f"[bench] launch timed out after {args.launch_timeout:.0f} s", file=sys.stderr, flush=True)
                rc = 124
                break
            time.sleep(0.2)
    finally:
        if rc:
            stop_all()
            t1 = time.time()
            while any(p.poll() is None for p in procs) and time.time() - t1 < 15:
                time.sleep(0.2)
            stop_all(signal.SIGKILL)
        for p in procs:
            p.wait()
        for s_, h in old.items():
            signal.signal(s_, h)
    return rc


def dry_run(args) -> None:
    """Launcher self-test: report this rank's environment (env), or join a gloo group
    over the launcher's rendezvous and gather every rank's (gloo); `fail`: rank 1
    exits with 3 while rank 0 waits, so the launcher must end rank 0 and fail."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    me = {k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    me["pid"] = os.getpid()
    if args.dry_run == "fail":
        if rank == 1:
            sys.exit(3)
        time.sleep(120)
        return
    if args.dry_run == "gloo":
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        allv = [None] * world
        dist.all_gather_object(allv, me)
        dist.barrier()
        dist.destroy_process_group()
        if rank == 0:
            print(json.dumps({"dry_run": "gloo", "n_gpus": world, "ranks": allv}), flush=True)
        return
    # one write per line (print's text and newline are two): the ranks share the stderr pipe
    sys.stdout.write(json.dumps({"dry_run": "env", "n_gpus": world, "rank": me}) + "\n")
    sys.stdout.flush()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    if args.dry_run:
        dry_run(args)
        return
    import torch
    import torch.distributed as dist

    from speedy_ml_amd import domain
    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.hybrid import HybridLoop, SlabOcean
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights, slab_fields,
                                         slab_start_outvec, slab_weights, synthetic_grids)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)

    nreg = args.regions
    mask = domain.load_sst_mask()
    sim = args.sim_ranks if world == 1 and args.sim_ranks > 1 else 1
    regions = domain.processor_decomposition(nreg, world * sim, rank)

    # ---- setup: synthetic weights with the trained structure, loaded per region
    t_setup = time.time()
    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in regions]
    res = Reservoirs(regions, [mask[r] for r in regions], [s.n for s in sizes], [s.k for s in sizes],
                     weight_dtype=args.weights)
    for i, r in enumerate(regions):
        w = region_weights(r, bool(mask[r]), climatology=True)
        if args.weights == "f64":
            res.load_region(i, w.rows, w.cols, w.vals.astype(np.float64), w.win.astype(np.float64),
                            w.wout.astype(np.float64), w.mean, w.std)
        else:
            res.load_region_weights(i, w)
        res.set_state(i, initial_state(r, w.n))
        if i % 144 == 0:
            log(rank, f"loaded {i}/{len(regions)} regions ({time.time() - t_setup:.1f}s)")
    slab_ocean, slab_ids = None, []
    if args.slab:  # the slab-ocean reservoirs of this rank's sst regions (synthetic, n = 4032)
        slab_ids = [r for r in regions if mask[r]]
        sws = [slab_weights(r) for r in slab_ids]
        slab_res = Reservoirs(slab_ids, [0] * len(slab_ids), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0,
                              nout=4, ninp=[w.ninp for w in sws], out_index=[35] * 4)
        for j, w in enumerate(sws):
            slab_res.load_region_weights(j, w)
            slab_res.set_state(j, initial_state(slab_ids[j], w.n, seed=17))
        del sws
        base_h, smask_h, sice_h, tice_h = slab_fields()
        slab_ocean = SlabOcean(slab_res, torch.from_numpy(base_h).to(dev), torch.from_numpy(smask_h).to(dev))
        log(rank, f"slab ocean: {len(slab_ids)} slab reservoirs ({time.time() - t_setup:.1f}s)")
    exchange = OutvecExchange(nreg, world, rank, device=dev, nout=136 + (4 if args.slab else 0))
    if sim > 1:  # rank 0 of `sim` ranks: its outvecs into a global array, the others stale
        glob_sim = torch.zeros((nreg, 136 + (4 if args.slab else 0)), dtype=torch.float64, device=dev)
        sim_filled = []

        def exchange(ov_local):
            if not sim_filled:
                # the other ranks' rows once, from this rank's first outvecs repeated (every
                # region's row has the same variable layout): the assembled state stays in
                # iogrid's safe range, so the window's entry check passes and run_model's
                # exit takes the integrated path, as on a real rank
                nl = len(regions)
                idx = torch.arange(nreg, device=dev) % nl
                glob_sim.copy_(ov_local[idx])
                sim_filled.append(True)
            glob_sim[:len(regions)].copy_(ov_local)
            return glob_sim
    g4h, g2h, prh = synthetic_grids(11)
    f4h, f2h, _ = synthetic_grids(12)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    tisr = t(np.random.default_rng(13).standard_normal((len(regions), 16)))
    # SPEEDY on the GPU: dynamical core + physics, forcing and boundary fields
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    phys_bc = phys_boundary(dyn, forcing["phis"])
    if args.date_forcing:  # inbcon's surface fields and monthly climatologies (synthetic)
        from speedy_ml_amd.synthetic import surface_climatology

        surf_h, clim_h = surface_climatology(phys_bc["fmask1"])
        phys_bc["fmask1"] = surf_h["fmask_l"]
    dyn.set_physics(phys_bc)
    if args.date_forcing:
        dyn.set_surface(surf_h)
        dyn.set_climatology(clim_h)
    if slab_ocean is not None:
        from speedy_ml_amd._lib import check as _check, lib as _lib, ptr as _ptr

        _check(_lib().sml_dyn_set_sea_ice(dyn._h, _ptr(np.ascontiguousarray(sice_h)),
                                          _ptr(np.ascontiguousarray(tice_h))))
    # the hybrid loop (speedy_ml_amd/hybrid.py); --overlap puts SPEEDY's window on a
    # second stream beside the reservoir update + v_ml readout
    ncu = torch.cuda.get_device_properties(dev).multi_processor_count
    comm = None
    if world > 1 and sim == 1 and args.exchange == "native":
        from speedy_ml_amd.comm import NativeComm

        comm = NativeComm(world, rank)
    loop = HybridLoop(res, dyn, exchange, dev, tisr=tisr, overlap=args.overlap, speedy_cus=args.speedy_cus,
                      comm=comm, slab=slab_ocean)
    if args.date_forcing:  # the hours before the first step: traininglength + marker + synclength in the reference
        loop.set_calendar(1981, 24 * 365, 6)
    if args.pipelined:
        loop.set_pipelined(True)
    from speedy_ml_amd._lib import SML_CHAIN_SPEEDY, SML_CHAIN_TWO_STREAMS

    if args.chain != "auto":
        loop.set_chain(SML_CHAIN_TWO_STREAMS if args.chain == "two-streams" else SML_CHAIN_SPEEDY)
    chain_eff = loop.chain()[1]
    # initial inputs from the synthetic analysis state (start_prediction analogue)
    loop.start(t(g4h), t(g2h), t(prh), t(f4h), t(f2h))
    if slab_ocean is not None:
        loop.start_slab(t(np.stack([slab_start_outvec(r) for r in slab_ids]) if slab_ids else np.zeros((0, 4))))
    fb, lm, ov, g4, g2, pr, f4, f2 = loop.fb, loop.lm, loop.ov, loop.g4, loop.g2, loop.pr, loop.f4, loop.f2
    torch.cuda.synchronize()
    log(rank, f"setup {time.time() - t_setup:.1f}s, {len(regions)} regions on rank 0")

    ended = []  # the step after which run_speedy was false (the reference's loop exit)
    ran = [0]   # steps the last timed region ran

    def step():
        loop.step()

    def step_polled():
        """parallelmain.f90:268-270: after every step the host reads run_speedy (rank 0
        decides in the reference and broadcasts it, mpires.f90:721; here every rank's
        redundant window gives the same flag) and ends the prediction when it is false."""
        loop.step()
        if not loop.run_speedy():
            ended.append(True)
            return False
        return True

    def timed(fn, nsteps, timing=False):
        if timing:
            res.enable_timing(nsteps)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        host = []
        ran[0] = 0
        for _ in range(nsteps):
            h0 = time.perf_counter()
            go = fn()
            host.append(time.perf_counter() - h0)
            ran[0] += 1
            if go is False:  # run_speedy false: the reference's loop ends here
                break
        th = time.perf_counter() - t0
        loop.sync()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        if os.environ.get("SML_BENCH_HOST"):  # diagnostic: does the host keep ahead of the GPU?
            log(rank, f"host: enqueue {th * 1e3 / nsteps:.3f} ms/step of {dt * 1e3 / nsteps:.3f}; per call median "
                      f"{np.median(host) * 1e3:.3f} max {max(host) * 1e3:.3f} ms")
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        return dt

    for _ in range(args.warmup):
        step()
    loop.sync()
    poll = args.poll_run_speedy
    n_ford0 = dyn.fordate_count()
    dt = timed(step_polled if poll else step, args.steps, timing=True)
    upd_ms, rd_ms = res.kernel_times()
    steps_done = ran[0]
    n_ford = dyn.fordate_count() - n_ford0
    # the poll's cost: the same K steps again without the host waiting on run_speedy
    dt_nopoll = timed(step, args.steps) if poll and not ended else None
    if args.pipelined and args.overlap:  # the next step's begin is in flight: close it (untimed)
        res.predict_finish(lm, ov, stream=loop.main)
        torch.cuda.synchronize()
    _, safe = dyn.from_grid(g4.cpu().numpy(), g2.cpu().numpy())
    finite = bool(torch.isfinite(f4).all().item()) and bool(torch.isfinite(ov).all().item())

    # ---- roofline of the dominant kernel (readout: streams W_out)
    wb = 4 if args.weights == "f32" else 8
    # the timed readout launch: one pass over W_out [local_model; x~] + unstandardize
    # (columns 132 + n, x_aug in, outvec + mean/std), or with --overlap the v_ml half
    # (W_out(:, ncs+1:) x~: n columns, x~ in, 136 partial sums out), per region
    if args.overlap:
        rd_cost = lambda s, b: b * 136 * s.n + 8 * s.n + 8 * 136  # noqa: E731
    else:
        rd_cost = lambda s, b: b * 136 * (132 + s.n) + 8 * (132 + s.n) + 8 * 136 + 2 * 36 * 8  # noqa: E731
    rd_bytes = sum(rd_cost(s, wb) for s in sizes)
    rd_bytes_f64 = sum(rd_cost(s, 8) for s in sizes)
    rd_avg_s = float(np.mean(rd_ms)) * 1e-3
    upd_avg_s = float(np.mean(upd_ms)) * 1e-3
    achieved = rd_bytes / rd_avg_s / 1e9
    # the update's algorithmic bytes: A's k entries (column + value), W_in's n values (its
    # block-diagonal column i / q is computed, not read: mod_reservoir.f90:260-278), the
    # state in and out, the feedback (r04b; before, A was counted as 8 ELL slots per row
    # and W_in's column as read: 48 n + 6 n instead of (2 + wb) k + wb n)
    upd_bytes = sum((2 + wb) * s.k + wb * s.n + 2 * 8 * s.n + 8 * s.ninp for s in sizes)
    _, algo_step = res.footprint()
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", "readout_pmc.json")
    if os.path.exists(pmc_path) and world == 1 and nreg == 1152 and args.weights == "f32":
        try:
            pmc = json.load(open(pmc_path))
            # the PMC pass must have profiled the same readout form as this run
            if pmc.get("kernel", "").startswith("k_res_readout_ml" if args.overlap else "k_res_readout_full"):
                traffic = pmc.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    # supplementary: the reservoir side alone (configs[1]), SPEEDY's step alone
    reservoir_only = None
    if args.reservoir_steps > 0:
        res.set_update_cus(0)  # this leg runs on the whole device: one balanced-update block per CU of all 256

        def rstep():
            res.predict(fb, lm, ov)
            glob = exchange(ov)
            res.assemble(glob, g4, g2, pr)
            res.tile_inputs(g4, g2, pr, f4, f2, tisr, fb, lm)

        for _ in range(3):
            rstep()
        rdt = timed(rstep, args.reservoir_steps, timing=True)
        u_upd, u_rd = res.kernel_times()
        full_cost = lambda s, b: b * 136 * (132 + s.n) + 8 * (132 + s.n) + 8 * 136 + 2 * 36 * 8  # noqa: E731
        full_bytes = sum(full_cost(s, wb) for s in sizes)
        u_rd_s = float(np.mean(u_rd)) * 1e-3
        unpaced = {"kernel": "k_res_readout<full> (one pass, on the critical path of the reservoir-only step)",
                   "achieved": round(full_bytes / u_rd_s / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(full_bytes / u_rd_s / 1e9 / HBM_PEAK_GBS, 4),
                   "algorithmic_bytes_per_launch": full_bytes, "readout_avg_ms": round(u_rd_s * 1e3, 4),
                   "update_avg_ms": round(float(np.mean(u_upd)), 4),
                   "update_achieved_GBps": round(upd_bytes / (float(np.mean(u_upd)) * 1e-3) / 1e9, 1),
                   "update_frac": round(upd_bytes / (float(np.mean(u_upd)) * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        reservoir_only = {
            "workload": "configs[1]: predict for all 1152 subdomains + outvec exchange + assemble + re-tile "
                        "(SPEEDY forecast grids held fixed)",
            "value": round(args.reservoir_steps / rdt, 3), "unit": "hybrid timesteps/s",
            "ms_per_step": round(rdt / args.reservoir_steps * 1e3, 4), "steps": args.reservoir_steps,
            "roofline_unpaced": unpaced}
    date_forcing = {"on": False}
    if args.date_forcing:
        # the forcing's own cost: forced recomputations (the coupler at a date + hybrid SST
        # + fordate: one grid-point kernel and spec of tcorh / qcorh), on one stream
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for i in range(3):
            dyn.fordate(1982, 1 + i % 12, 1 + i % 28, force=True)
        ev0.record()
        nrep = 50
        for i in range(nrep):
            dyn.fordate(1982, 1 + i % 12, 1 + i % 28, force=True)
        ev1.record()
        torch.cuda.synchronize()
        f_ms = ev0.elapsed_time(ev1) / nrep
        date_forcing = {
            "on": True,
            "calendar": "startyear 1981, hours_base 8760 (1982-01-01), 6 h per step: each window's date as "
                        "run_model's get_current_time_delta_hour gives it (mpires.f90:1545)",
            "recomputed_windows": n_ford, "timed_windows": steps_done,
            "note": "recomputed when the date (once a day: every 4th step) or the slab's hybrid SST changed; "
                    "on SPEEDY's stream behind the previous window (beside the finish and assembly), or, on a "
                    "step with a new hybrid SST, behind that SST on the reservoir stream before the grid hop",
            "recompute_ms": round(f_ms, 4),
            "per_step_ms": round(f_ms * n_ford / max(steps_done, 1), 4)}
    dyn.close()
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_threads > 0:
        cpu = cpu_baseline(nreg, mask, args.cpu_threads)
    speedy = speedy_leg(dev, world, rank, args) if args.speedy_steps > 0 else None
    training = training_leg(dev, mask, args, world, rank) if args.train_regions > 0 else None

    if rank == 0:
        steps_per_s = steps_done / dt
        line = {
            "metric": "hybrid timesteps/sec, T30L8 + 1152x6k-node reservoirs; 1/2/4/8-GPU scaling",
            "value": round(steps_per_s, 3),
            "unit": "hybrid timesteps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / steps_done * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded T30L8 state and boundary fields, random weights with the trained structure)",
            "config": {
                "workload": f"configs[{2 if world == 1 else 3}]: full hybrid timestep -- reservoir predict for all "
                            "1152 subdomains, "
                            + ("outvec exchange (identity on one GPU)" if world == 1 else
                               f"outvec all-gather over RCCL ({world} ranks, "
                               + ("the library's ncclAllGather on the loop's main stream)" if comm is not None
                                  else "torch.distributed)"))
                            + ", assemble, SPEEDY 6-h window (iogrid(30), stepone + 24 leapfrog dyn_steps with "
                              "phypar physics, iogrid(31)) on the GPU, re-tile"
                            + (f"; slab ocean ON ({len(slab_ids)} slab reservoirs of n = 4032 on this rank, "
                               "predict_slab_ml every 28th step, its sst in the window and the feedback)"
                               if args.slab else "; slab ocean OFF"),
                "slab_ocean": bool(args.slab),
                "regions": nreg,
                "regions_per_gpu": len(regions),
                "reservoir_nodes": "5760/6160/6048/5880 (NINT(6000/ninp)*ninp)",
                "weights": f"{args.weights} storage ({'exact file precision' if args.weights == 'f32' else 'fp64'}), "
                           "fp64 arithmetic",
                "parallelism": f"res_domain sharded over {world} GPU(s); SPEEDY window replicated per GPU"
                               + (f" [DIAGNOSTIC: rank 0 of {sim} simulated ranks, exchange local]" if sim > 1 else ""),
                "speedy": "T30L8, 26 dyn_steps per window (nsteps 96/day, delt 900 s), physics on, "
                          "shortwave every 3rd step",
                "loop": ("pipelined: each step issues the next step's reservoir begin beside its window, so the "
                         "timed steps run begins 2..K+1 and windows 1..K -- K of each, none skipped"
                         if args.pipelined and args.overlap else "each step issues its own begin"),
                "chain": ("the step's serial chain (v_p finish, exchange, assembly, tiling) on SPEEDY's stream behind "
                      "the window" if chain_eff == SML_CHAIN_SPEEDY else
                      "the step's serial chain on the reservoir's stream, two cross-stream hops per step"),
            "streams": (f"overlapped: SPEEDY on CUs [0, {loop.speedy_cus}), reservoir on CUs [{loop.speedy_cus}, "
                            f"{loop.speedy_cus + loop.res_cus}) (one CU per 6 of the rank's {res.nlocal} regions, "
                            f"at least 64), the safety check on the rest"
                            if loop.res_cus > 0 else
                            "overlapped, no CU split" if args.overlap else "one stream"),
            },
            "run_speedy_poll": ({"per_step": True, "ended_after_step": steps_done if ended else None,
                                 "note": "the host reads run_speedy after every timed step and would end the loop "
                                         "on false (parallelmain.f90:268-270); the same K steps without the poll",
                                 "value_without_poll": round(args.steps / dt_nopoll, 3) if dt_nopoll else None,
                                 "cost_pct": round((dt - dt_nopoll) / dt_nopoll * 100, 2) if dt_nopoll else None}
                                if poll else {"per_step": False}),
            "date_forcing": date_forcing,
            "last_window_safe": bool(safe),
            "finite": finite,
            "roofline": {
                "kernel": (("k_res_readout<ml> (v_ml = W_out(:, ncs+1:) x~, GEMV, 17 rows per wave, 128-B-aligned rows; beside "
                            + (f"SPEEDY's window on {loop.res_cus} of the {ncu - loop.speedy_cus} CUs SPEEDY does "
                               "not use, unpaced"
                               if loop.res_cus > 0 else "SPEEDY's window on shared CUs, paced at 2048 waves")
                            + "; the one-pass form on all CUs: reservoir_only.roofline_unpaced)")
                           if args.overlap else
                           "k_res_readout<full> (W_out [local_model; x~] + unstandardize, GEMV, 17 waves x 8 rows "
                           "per region)"),
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": rd_bytes,
                "fp64_weight_equivalent_GBps": round(rd_bytes_f64 / rd_avg_s / 1e9, 1),
                "readout_avg_ms": round(rd_avg_s * 1e3, 4),
                "update_avg_ms": round(upd_avg_s * 1e3, 4),
                # the state update beside the window (k_res_update_bal, 192 CUs): A as ELL rows of 8
                # slots (u16 column + weight), W_in's one entry per row, x read once (LDS staging),
                # x and x~ written, the feedback read
                "update_algorithmic_bytes": upd_bytes,
                "update_achieved_GBps": round(upd_bytes / upd_avg_s / 1e9, 1),
                "update_frac": round(upd_bytes / upd_avg_s / 1e9 / HBM_PEAK_GBS, 4),
                "step_algorithmic_bytes": algo_step,
            },
            "cpu_baseline": cpu,
            "reservoir_only": reservoir_only,
            "speedy_step": speedy,
            "training": training,
        }
        print(json.dumps(line), flush=True)
    loop.close()  # before the communicators go: the loop's streams are drained first
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


F64_VALU_PEAK_TF = 78.6  # MI355X fp64 vector (256 CUs x 4 SIMDs x 64 lanes x 2 flop / 4 clk x 2.4 GHz)
F64_MFMA_PEAK_TF = 78.6  # v_mfma_f64_16x16x4: 2048 flop in 64 clk per SIMD (SQ_VALU_MFMA_BUSY_CYCLES / MFMAs = 64)


def speedy_roofline(st, forcing, bc):
    """The fused SPEEDY step's two kernels, measured live: per-phase durations from
    the kernels' own wall_clock64 stamps (SML_DYN_STAMPS, a chained 26-step window,
    median over blocks) and the work per dispatch from the committed counter pass
    (profiles/speedy_pmc.json, tools/speedy_pmc.py: SQ_INSTS_VALU_*_F64 and
    SQ_INSTS_VALU_MFMA_MOPS_F64; deterministic per dispatch).  Both kernels are
    latency-bound (dependent f64 chains of one lane, one wave per SIMD; barriers
    between phases), so `frac` is far below 1 by construction: the numbers say how
    much of the occupied CUs' f64 issue / MFMA the step keeps busy."""
    import ctypes

    import numpy as np
    import torch

    from speedy_ml_amd._lib import lib
    from speedy_ml_amd.dynamics import Dynamics

    pmc_path = os.path.join(REPO, "profiles", "speedy_pmc.json")
    pmc = json.load(open(pmc_path))["kernels"] if os.path.exists(pmc_path) else {}
    os.environ["SML_DYN_STAMPS"] = "1"
    try:
        d = Dynamics()
    finally:
        del os.environ["SML_DYN_STAMPS"]
    d.set_forcing(**forcing)
    d.set_state(st)
    d.set_physics(bc)
    d.set_rad_state(None)
    d.set_clock(1, True)
    d.window(24)
    d.window(24)
    torch.cuda.synchronize()
    buf = np.zeros((4, 96, 8), dtype=np.int64)
    L = lib()
    L.sml_dbg_dyn_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    rc = L.sml_dbg_dyn_stamps(d._h, buf.ctypes.data)
    d.close()
    if rc != 0:
        return None

    def phases(kern, names):
        nb = int((buf[kern, :, 0] > 0).sum())
        b = buf[kern, :nb].astype(np.float64) / 100.0  # wall_clock64 ticks at 100 MHz -> us
        ph = {n: round(float(np.median(b[:, i + 1] - b[:, i])), 2) for i, n in enumerate(names)}
        span = float(b[:, len(names)].max() - b[:, 0].min())
        return nb, ph, round(span, 2)

    nb_g, ph_g, span_g = phases(0, ["gridx", "gridpoint_and_phypar", "specx"])
    nb_s, ph_s, span_s = phases(1, ["load", "specy", "combine", "tail", "inv_inputs", "gridy"])
    g = pmc.get("k_st_gridspec", {})
    spec_last, inv = pmc.get("k_st_spec", {}), pmc.get("k_st_inv", {})
    valu_g = g.get("valu_f64_flops_per_dispatch")
    # specy (the launched-mode k_st_spec has no gridy); each of its kSpecSplit blocks per
    # m repeats the m's specy (csrc/sml_dynamics.hip), so the algorithmic flops are the
    # counted ones / kSpecSplit and the kernel occupies kSpecSplit CUs per m
    spec_split = 2
    specy_fl = spec_last.get("mfma_f64_flops_per_dispatch")
    if specy_fl:
        specy_fl = specy_fl / spec_split
    gridy_fl = inv.get("mfma_f64_flops_per_dispatch")        # gridy (k_st_inv)
    out = {"source": "phase stamps (live, chained window) + profiles/speedy_pmc.json (work per dispatch)",
           "peak_f64_valu_tflops": F64_VALU_PEAK_TF, "peak_f64_mfma_tflops": F64_MFMA_PEAK_TF}
    e = {"blocks": nb_g, "span_us": span_g, "phases_us": ph_g, "bound": "latency (per-lane f64 chains: FFTPACK "
         "passes, phypar; one wave per SIMD)"}
    if valu_g:
        tf = valu_g / (span_g * 1e-6) / 1e12
        occ = F64_VALU_PEAK_TF * nb_g / 256
        e.update({"valu_f64_flops": valu_g, "achieved_tflops": round(tf, 3),
                  "frac_of_occupied_cus": round(tf / occ, 4), "frac_of_chip": round(tf / F64_VALU_PEAK_TF, 5)})
    out["k_st_gridspec"] = e
    e = {"blocks": nb_s, "span_us": span_s, "phases_us": ph_s, "bound": "latency (phase chain with barriers)"}
    # algorithmic Legendre work: the reference sums only
    # m <= nsh2(n) (spe_spectral.f90:476-493 gridy, :513-535 specy): 50.6 kflop per
    # inverse field (24 latitude pairs x 1054 FMA) and 50.5 kflop per forward field;
    # a fused step runs 73 forward (specx -> specy) and 91 inverse (gridy -> gridx) fields
    specy_algo, gridy_algo = 73 * 50.5e3, 91 * 50.6e3
    occ = F64_MFMA_PEAK_TF * nb_s * spec_split / 256
    sy = specy_algo / (ph_s["specy"] * 1e-6) / 1e12
    gy = gridy_algo / (ph_s["gridy"] * 1e-6) / 1e12
    leg_algo = specy_algo + gridy_algo
    e.update({
        "blocks": nb_s * spec_split,
        "legendre_algorithmic_flops": leg_algo,
        "achieved_tflops_kernel": round(leg_algo / (span_s * 1e-6) / 1e12, 3),
        "legendre_mfma_utilisation": {
            "basis": "algorithmic flops (the triangle m <= nsh2(n) the reference sums) / phase time",
            "specy_tflops": round(sy, 3), "gridy_tflops": round(gy, 3),
            "specy_frac_of_occupied_cus": round(sy / occ, 4), "gridy_frac_of_occupied_cus": round(gy / occ, 4),
            "specy_frac_of_chip": round(sy / F64_MFMA_PEAK_TF, 5),
            "gridy_frac_of_chip": round(gy / F64_MFMA_PEAK_TF, 5),
            "step_frac_of_chip": round(leg_algo / (span_s * 1e-6) / 1e12 / F64_MFMA_PEAK_TF, 5),
        }})
    if specy_fl and gridy_fl:  # what the MFMAs issued (PMC), padding and the zero triangle included
        leg = specy_fl + gridy_fl
        e["legendre_issued"] = {
            "source": "SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 per dispatch (profiles/speedy_pmc.json)",
            "flops": leg, "specy_flops": specy_fl, "gridy_flops": gridy_fl,
            "issued_over_algorithmic": round(leg / leg_algo, 3),
            "specy_tflops": round(specy_fl / (ph_s["specy"] * 1e-6) / 1e12, 3),
            "gridy_tflops": round(gridy_fl / (ph_s["gridy"] * 1e-6) / 1e12, 3)}
    out["k_st_spec"] = e
    return out


def speedy_leg(dev, world, rank, args):
    """Supplementary measurement: one SPEEDY dyn_step on the GPU without and with
    the physics (leapfrog step(2,2), HIP events, launched step by step and replayed
    from hipGraphs), plus the oracle's step with physics on one host core."""
    import torch

    from speedy_ml_amd.dynamics import DELT, Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    st, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    bc = phys_boundary(dyn, forcing["phis"])
    out = {}
    for phys in (False, True):
        dyn.set_physics(bc if phys else None)
        for mode, graph in (("launch", False), ("graph", True)):
            dyn.set_state(st)
            dyn.set_rad_state(None)
            dyn.set_clock(1, True)
            dyn.stepone()
            dyn.leapfrog(6, DELT, graph=graph)  # warm-up (and graph capture for both lradsw values)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            dyn.leapfrog(args.speedy_steps, DELT, graph=graph)
            e1.record()
            torch.cuda.synchronize()
            out[f"step_ms_{mode}{'_physics' if phys else ''}"] = round(e0.elapsed_time(e1) / args.speedy_steps, 4)
    # the whole window as the hybrid step runs it: stepone + 24 leapfrog steps, one
    # hipGraph, consecutive fused steps chained (sml_dyn_window)
    dyn.set_physics(bc)
    dyn.set_state(st)
    dyn.set_rad_state(None)
    dyn.set_clock(1, True)
    dyn.window(24)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    nwin = 10
    e0.record()
    for _ in range(nwin):
        dyn.window(24)
    e1.record()
    torch.cuda.synchronize()
    out["window_ms_graph_physics"] = round(e0.elapsed_time(e1) / nwin, 4)
    out["roofline"] = speedy_roofline(st, forcing, bc)
    out["note"] = ("step_ms_*: one dyn_step (grtend/sptend/implic/hordif/timint, 164 transforms; with physics + "
                   "phypar on level 1, 41 more transforms) launched alone; window_ms_graph_physics: the chained "
                   "26-step window (sml_dyn_window, one hipGraph) as the hybrid step runs it")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle

        s = oracle.dyn_state_copy(st)
        rad = oracle.phys_state()
        oracle.dyn_step_physics(s, forcing["phis"], forcing["tcorh"], forcing["qcorh"], bc, rad, True, 2, 2,
                                2 * DELT, 0.5)
        t0 = time.perf_counter()
        nrep = 5
        for i in range(nrep):
            oracle.dyn_step_physics(s, forcing["phis"], forcing["tcorh"], forcing["qcorh"], bc, rad, i % 3 == 0, 2, 2,
                                    2 * DELT, 0.5)
        out["cpu_oracle_step_ms_physics"] = round((time.perf_counter() - t0) / nrep * 1e3, 3)
        out["cpu_oracle_note"] = "oracle C restatement (direct DFT instead of FFTPACK), 1 core"
    dyn.close()
    return out


def training_leg(dev, mask, args, world, rank):
    """Supplementary measurement (BASELINE configs[4]: W_out training of all 1152
    regions on 8 GPUs): every rank trains its own batch of args.train_regions
    6000-node-class regions, resident in HBM at once (144 per rank = all 1152 on 8
    ranks; no collective -- regions are independent, scaling weak).  Per batch:
    chunking_matmul Gram and cross products (hand-written fp64 MFMA kernel) over
    args.train_steps time steps in 4 batches, then regularisation + the hand-written
    batched Cholesky solve (k_chol_* / k_solve_*, replacing mldivide's dgesv,
    mod_linalg.f90:109-151).  Times are the max over ranks.  Roofline: Gram kernel
    flops / its time, and the solve's algorithmic flops (naug^3/3 potrf + 2 naug^2
    nout for the two triangular solves) / its time, both vs the measured fp64 MFMA
    rate."""
    import ctypes

    import torch
    import torch.distributed as dist

    from speedy_ml_amd import domain
    from speedy_ml_amd._lib import check, lib
    from speedy_ml_amd.training import Trainer

    per = args.train_regions
    regions = [(rank * per + i) % 1152 for i in range(per)]
    naug = [132 + domain.reservoir_sizes(r, bool(mask[r])).n for r in regions]
    nb = args.train_batches
    m = args.train_steps // nb
    gen = torch.Generator(device=dev)
    gen.manual_seed(3 + rank)
    S = torch.tanh(torch.randn(sum(naug) * m, dtype=torch.float64, device=dev, generator=gen))
    T = torch.randn(len(naug) * m * 136, dtype=torch.float64, device=dev, generator=gen)
    tr = Trainer(naug)
    if args.train_panel != 8:
        tr.set_panel(args.train_panel)
    tr.accumulate(S, T, m)  # warm-up
    tr.reset()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    for _ in range(nb):
        tr.accumulate(S, T, m)
    e1.record()
    _, info = tr.solve()
    e2.record()
    torch.cuda.synchronize()
    times = torch.tensor([e0.elapsed_time(e1), e1.elapsed_time(e2)], dtype=torch.float64, device=dev)
    ok = torch.tensor([float((info == 0).all())], device=dev)
    if world > 1:
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    gram_ms, solve_ms = (float(v) for v in times.cpu())
    npad = tr.npad
    # algorithmic flops: lower-triangle Gram (naug(naug+1)/2 dot products) + T S^T, 2 flops per FMA
    algo = sum(2.0 * (n * (n + 1) / 2 + 136 * n) * m * nb for n in naug)
    # the MFMA work actually issued: each tile's 64 x 64 wave sub-tiles that hold output
    # (k_train_gram2 skips the blocks past a region's naug, the sub-tiles above a
    # diagonal tile's diagonal and those past naug / nout)
    def live_quads(n):
        cr, q = (n + 127) // 128, 0
        for bi in range(cr):
            for bj in range(bi + 1):
                q += sum(1 for wr in (0, 1) for wc in (0, 1)
                         if bi * 128 + wr * 64 < n and bj * 128 + wc * 64 < n and not (bi == bj and wr < wc))
        for bi in range(2):
            for bj in range(cr):
                q += sum(1 for wr in (0, 1) for wc in (0, 1) if bi * 128 + wr * 64 < 136 and bj * 128 + wc * 64 < n)
        return q
    issued = sum(live_quads(n) for n in naug) * 2.0 * 64 * 64 * m * nb
    peak, ghz = ctypes.c_double(), ctypes.c_double()
    check(lib().sml_probe_mfma_f64_clock(20000, ctypes.byref(peak), ctypes.byref(ghz)))
    # the nominal peak at the clock the chip holds under back-to-back fp64 MFMA
    peak_clk = F64_MFMA_PEAK_TF * ghz.value / 2.4 if ghz.value > 0 else None
    tr.close()
    del S, T
    torch.cuda.empty_cache()
    achieved = algo / (gram_ms * 1e-3) / 1e12
    solve_algo = sum(n ** 3 / 3.0 + 2.0 * n * n * 136 for n in naug)
    solve_tf = solve_algo / (solve_ms * 1e-3) / 1e12
    return {
        "workload": f"{len(naug)} regions per rank x {world} rank(s) (naug {min(naug)}..{max(naug)}, one batch "
                    f"resident: {len(naug) * npad * npad * 8 / 1e9:.1f} GB of Gram matrices per GPU), "
                    f"{m * nb} training steps in {nb} chunking_matmul batches, then fit_chunk_hybrid "
                    "regularisation + solve",
        "regions_per_s": round(world * len(naug) / ((gram_ms + solve_ms) * 1e-3), 2),
        "scaling": "weak",
        "gram_ms": round(gram_ms, 3),
        "solve_ms": round(solve_ms, 3),
        "solve_ms_per_region": round(solve_ms / len(naug), 3),
        "solve_info_ok": bool(ok.item() == 1.0),
        "solve_roofline": {
            "kernels": "k_chol_diag_b / k_chol_panel / k_chol_upanel / k_chol_update (right-looking over panels "
                       "of 8 block columns, left-looking inside, 128-blocked, fp64 MFMA, 16-B LDS staging) + "
                       "k_solve_lpanel / k_solve_update (block forward / backward substitution: a panel's "
                       "block rows left-looking, one launch each; the rows below or above by the panel; each "
                       "panel's forward substitution on a second stream beside the later panels' factorisation)",
            "bound": "mfma", "unit": "TFLOP/s",
            "achieved": round(solve_tf, 2),
            "peak": F64_MFMA_PEAK_TF,
            "frac": round(solve_tf / F64_MFMA_PEAK_TF, 4),
            "probe_tflops": round(peak.value, 2),
            "frac_of_probe": round(solve_tf / peak.value, 4),
            "probe_clock_ghz": round(ghz.value, 3),
            "frac_at_probe_clock": round(solve_tf / peak_clk, 4) if peak_clk else None,
            "algorithmic_flops": solve_algo,
            "previous": "r04a: 290.7 ms, 39.8 TF/s (every region factored at the batch's padded size); r02: 394 ms, "
                        "29.3 TF/s (1 wave per SIMD); rocSOLVER dpotrf + dpotrs strided-batched in r01: 41.7 ms per "
                        "region",
        },
        "roofline": {
            "kernel": "k_train_gram2 (fp64 MFMA 16x16x4, 128x128 tiles, lower triangle + T S^T strip, LDS stages "
                      "double-buffered and filled by 16-B row-pair loads / stores, 2 waves per SIMD; blocks past a "
                      "region's naug and wave sub-tiles without output skipped)",
            "bound": "mfma", "unit": "TFLOP/s",
            "achieved": round(achieved, 2),
            "issued_tflops": round(issued / (gram_ms * 1e-3) / 1e12, 2),
            "peak": F64_MFMA_PEAK_TF,
            "peak_source": "nominal: 64 clk per v_mfma_f64_16x16x4_f64 (2048 flop) on each of 1024 SIMDs at 2.4 GHz; "
                           "the Gram's own inner loop from LDS operands reaches 77.35 TF/s = 0.984 of it "
                           "(tools/probe_lds_mfma.hip).  probe_tflops: back-to-back register-operand 16x16x4 MFMAs "
                           "of tools/probe_mfma_f64.hip (~47.5) -- not a ceiling",
            "frac": round(achieved / F64_MFMA_PEAK_TF, 4),
            "probe_tflops": round(peak.value, 2),
            "frac_of_probe": round(achieved / peak.value, 4),
            "probe_clock_ghz": round(ghz.value, 3),
            "peak_at_probe_clock": round(peak_clk, 2) if peak_clk else None,
            "frac_at_probe_clock": round(achieved / peak_clk, 4) if peak_clk else None,
            "algorithmic_flops": algo,
            "previous": "r04a: 462.0 ms, 47.5 TF/s (every tile of the batch's padded size issued: 57.5 TF/s); r02: "
                        "k_train_gram (single-buffered LDS, 1 wave per SIMD) 636 ms, 34.3 TF/s",
        },
    }


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_baseline(nreg: int, mask, threads: int):
    """The reference's CPU path of one hybrid step, timed on this host (rank 0, N=1):

      predict      all nreg regions with the reference's arithmetic -- COO SpMV,
                   the DENSE W_in matmul (mod_reservoir.f90:1443, 26.5 MB per region),
                   W_out GEMV, unstandardize -- fp64 weights as read_trained_res holds
                   them: the oracle's C restatement (oracle/speedy_oracle.c
                   orc_predict, pinned statement by statement), OpenMP over regions;
      exchange     assemble + tile of every region (the root's serial loops,
                   mpires.f90:300-751), oracle C, one thread;
      window       the REFERENCE's own SPEEDY code (oracle/_ref/libspeedy_ref_dyn.so,
                   dyn_* / phy_* / spe_* compiled as-is) through iogrid(30), stepone,
                   24 leapfrog steps and iogrid(31), one thread, as the reference runs
                   it on its root rank (oracle/ref_window_timing.py, a subprocess).

    One full step each with `threads` OpenMP threads (the value) and with one thread
    (reported beside it); no sample is extrapolated."""
    import subprocess

    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights

    t_gen = time.perf_counter()
    regs, fbs, lms, xs = [], [], [], []
    for r in range(nreg):
        w = region_weights(r, bool(mask[r]))
        regs.append({"rows": w.rows, "cols": w.cols, "vals": w.vals.astype(np.float64),
                     "win": w.win.astype(np.float64), "wout": w.wout.astype(np.float64), "mean": w.mean,
                     "std": w.std})
        fbs.append(feedback_vector(r, w.ninp))
        lms.append(local_model_vector(r))
        xs.append(initial_state(r, w.n))
    t_gen = time.perf_counter() - t_gen
    wbytes = sum(r["win"].nbytes + r["wout"].nbytes for r in regs)
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    counts = sorted({1, threads} | ({share} if 1 < share < threads else set()))
    pred = {}
    for th in counts:
        oracle.predict_regions(regs[:th], fbs[:th], lms[:th], xs[:th], nthreads=th)  # page the threads in
        t0 = time.perf_counter()
        outvecs = oracle.predict_regions(regs, fbs, lms, xs, nthreads=th)
        pred[th] = time.perf_counter() - t0
    del regs
    # exchange on the host: assemble + tile every region
    t0 = time.perf_counter()
    g4, g2, pr = oracle.assemble(outvecs)
    ms = np.ones(36)
    for r in range(nreg):
        oracle.tile_feedback(r, g4, g2, pr, np.zeros(36), ms, np.zeros(16))
        oracle.tile_local_model(r, g4, g2, np.zeros(36), ms)
    t_xchg = time.perf_counter() - t0
    # the reference's window, in a subprocess (its stack, its prints)
    out = subprocess.run([sys.executable, os.path.join(REPO, "oracle", "ref_window_timing.py"), "2"],
                         capture_output=True, text=True, timeout=300)
    win = json.loads(out.stdout.strip().splitlines()[-1])
    t_win = win["window_s"]
    step = {th: pred[th] + t_xchg + t_win for th in pred}
    best = min((th for th in pred if th > 1), key=lambda th: step[th], default=1)
    quota = None
    try:  # the cgroup's CPU quota (cgroup v2 cpu.max "quota period"), when there is one
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {
        "value": round(1.0 / step[best], 4),
        "unit": "hybrid timesteps/s",
        "cores": best,
        "kind": "port",
        "sample": f"one full hybrid step, no extrapolation: predict of all {nreg} regions with the reference's "
                  f"arithmetic (dense fp64 W_in, {wbytes / 1e9:.1f} GB of weights), OpenMP over regions, timed at "
                  + ", ".join(f"{th} thread{'s' if th > 1 else ''} {pred[th] * 1e3:.0f} ms" for th in counts)
                  + f" (value: the fastest, {best} threads; {1.0 / step[1]:.3f} steps/s single-core); host "
                  f"assemble + tile of every region {t_xchg * 1e3:.1f} ms; the reference's own SPEEDY window "
                  f"(compiled reference Fortran, oracle/_ref, 1 thread: iogrid(30), stepone, 24 leapfrog steps, "
                  f"iogrid(31)) {t_win * 1e3:.0f} ms -- agcm_init's per-window set-up (namelist, boundary files, "
                  f"coupler init) is excluded; host: {_cpu_model()}, {len(os.sched_getaffinity(0))} CPUs in the "
                  f"affinity mask, cgroup CPU quota {quota if quota is not None else 'none'}, "
                  f"OMP_NUM_THREADS={share or 'unset'}; weight generation {t_gen:.0f} s untimed",
        "single_thread_value": round(1.0 / step[1], 4),
        "threads_timed": counts,
        "affinity_cpus": len(os.sched_getaffinity(0)),
        "cgroup_cpu_quota": quota,
        "cpu_model": _cpu_model(),
        "predict_ms": {str(k): round(v * 1e3, 1) for k, v in pred.items()},
        "exchange_ms": round(t_xchg * 1e3, 2),
        "window_ms": round(t_win * 1e3, 1),
        "window_excludes": "agcm_init (per-window namelist / boundary-file / coupler set-up of agcm_main)",
    }


if __name__ == "__main__":
    main()

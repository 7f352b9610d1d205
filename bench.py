#!/usr/bin/env python3
"""bench.py -- SPEEDY-ML hybrid hot path on MI355X (one process per GPU).

One "step" = one hybrid-step pass over the reservoir side of the hot path for all
1152 subdomains (BASELINE.json configs[1], sharded per configs[3]):

  1. predict for every local region: A x + W_in u -> tanh -> W_out [model; x~],
     unstandardize                       (mod_reservoir.f90:1416-1487, 2 kernels)
  2. exchange: all-gather of every rank's outvecs over RCCL (N > 1)
                                         (replaces mpires.f90:338-716 MPI p2p)
  3. assemble the global T30L8 grid + clips (mpires.f90:300-478)
  4. re-tile every local region's next feedback (overlap tiles, standardized) and
     its standardized SPEEDY local vector (mpires.f90:558-751)

The SPEEDY window itself (26 dyn_steps with physics) is not part of this step yet:
the SPEEDY forecast grids consumed in (4) are a fixed synthetic T30L8 state.  Data
are synthetic, weights random with the trained structure, 6000-node-class
reservoirs (n = 5760/6160/6048/5880), fp64 arithmetic, weights held at their fp32
file precision (exact).

Usage: python bench.py [--gpus N --steps K --warmup W]
       python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--regions", type=int, default=1152)
    p.add_argument("--weights", choices=("f32", "f64"), default="f32")
    p.add_argument("--cpu-sample", type=int, default=96, help="regions in the CPU-baseline sample (0 = skip)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--train-regions", type=int, default=8,
                   help="regions in the supplementary W_out-training leg (0 = skip)")
    p.add_argument("--train-steps", type=int, default=4096, help="training time steps per region in that leg")
    p.add_argument("--hybrid-steps", type=int, default=10,
                   help="hybrid steps timed in the supplementary configs[2] leg (reservoir + SPEEDY dynamics "
                        "window; 0 = skip)")
    p.add_argument("--speedy-steps", type=int, default=48,
                   help="leapfrog steps timed in the supplementary SPEEDY-dynamics leg (0 = skip)")
    return p.parse_args()


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from speedy_ml_amd import domain
    from speedy_ml_amd.exchange import OutvecExchange
    from speedy_ml_amd.reservoir import Reservoirs
    from speedy_ml_amd.synthetic import initial_state, region_weights, synthetic_grids

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
    regions = domain.processor_decomposition(nreg, world, rank)

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
    fb, lm, ov = res.alloc_io(dev)
    exchange = OutvecExchange(nreg, world, rank, device=dev)
    g4h, g2h, prh = synthetic_grids(11)
    f4h, f2h, _ = synthetic_grids(12)
    g4 = torch.from_numpy(g4h).to(dev)
    g2 = torch.from_numpy(g2h).to(dev)
    pr = torch.from_numpy(prh).to(dev)
    f4 = torch.from_numpy(f4h).to(dev)
    f2 = torch.from_numpy(f2h).to(dev)
    tisr = torch.from_numpy(np.random.default_rng(13).standard_normal((len(regions), 16))).to(dev)
    # initial inputs from the synthetic analysis state (start_prediction analogue)
    res.tile_inputs(g4, g2, pr, f4, f2, tisr, fb, lm)
    torch.cuda.synchronize()
    log(rank, f"setup {time.time() - t_setup:.1f}s, {len(regions)} regions on rank 0")

    def step():
        res.predict(fb, lm, ov)
        glob = exchange(ov)  # RCCL all-gather over xGMI when world > 1
        res.assemble(glob, g4, g2, pr)
        res.tile_inputs(g4, g2, pr, f4, f2, tisr, fb, lm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    res.enable_timing(args.steps)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    upd_ms, rd_ms = res.kernel_times()
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # ---- roofline of the dominant kernel (readout: streams W_out)
    wb = 4 if args.weights == "f32" else 8
    rd_bytes = sum(wb * 136 * (132 + s.n) + 8 * (132 + s.n) + 8 * 136 + 2 * 36 * 8 for s in sizes)
    rd_bytes_f64 = sum(8 * 136 * (132 + s.n) + 8 * (132 + s.n) + 8 * 136 + 2 * 36 * 8 for s in sizes)
    rd_avg_s = float(np.mean(rd_ms)) * 1e-3
    upd_avg_s = float(np.mean(upd_ms)) * 1e-3
    achieved = rd_bytes / rd_avg_s / 1e9
    _, algo_step = res.footprint()
    traffic = None
    pmc_path = os.path.join(REPO, "profiles", "readout_pmc.json")
    if os.path.exists(pmc_path) and world == 1 and nreg == 1152 and args.weights == "f32":
        try:
            traffic = json.load(open(pmc_path)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.cpu_sample > 0:
        cpu = cpu_baseline(args.cpu_sample, nreg, mask)
    speedy = speedy_leg(dev, world, rank, args) if args.speedy_steps > 0 else None
    hybrid = None
    if args.hybrid_steps > 0:
        hybrid = hybrid_leg(dev, world, res, exchange, (fb, lm, ov), (g4, g2, pr, f4, f2, tisr), args)
    training = training_leg(dev, mask, args) if args.train_regions > 0 and world == 1 else None

    if rank == 0:
        steps_per_s = args.steps / dt
        line = {
            "metric": "hybrid timesteps/sec, T30L8 + 1152x6k-node reservoirs; 1/2/4/8-GPU scaling",
            "value": round(steps_per_s, 3),
            "unit": "hybrid timesteps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded T30L8 state, random weights with the trained structure)",
            "config": {
                "workload": "configs[1]: batched reservoir forward for all 1152 subdomains + RCCL outvec "
                            "all-gather + global-grid assembly + feedback/local-model re-tiling; SPEEDY "
                            "window not included (fixed synthetic forecast grids)",
                "regions": nreg,
                "regions_per_gpu": len(regions),
                "reservoir_nodes": "5760/6160/6048/5880 (NINT(6000/ninp)*ninp)",
                "weights": f"{args.weights} storage ({'exact file precision' if args.weights == 'f32' else 'fp64'}), "
                           "fp64 arithmetic",
                "parallelism": f"res_domain sharded over {world} GPU(s)",
            },
            "roofline": {
                "kernel": "k_res_readout (W_out GEMV, 17 waves x 8 rows per region)",
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
                "step_algorithmic_bytes": algo_step,
            },
            "cpu_baseline": cpu,
            "speedy_dynamics": speedy,
            "hybrid_with_dynamics": hybrid,
            "training": training,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def speedy_leg(dev, world, rank, args):
    """Supplementary measurement, outside the headline step: SPEEDY's dynamical core
    (dyn_step without physics) on the GPU, timed per leapfrog step with HIP events,
    launched step by step and replayed from a hipGraph, plus the oracle's step on
    one host core.  A 6-h window is stepone + 24 leapfrog steps (nsteps = 96/day)."""
    import torch

    from speedy_ml_amd.dynamics import DELT, Dynamics
    from speedy_ml_amd.synthetic import dyn_state

    st, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    out = {}
    for mode, graph in (("launch", False), ("graph", True)):
        dyn.set_state(st)
        dyn.stepone()
        dyn.leapfrog(4, DELT, graph=graph)  # warm-up (and graph capture)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        dyn.leapfrog(args.speedy_steps, DELT, graph=graph)
        e1.record()
        torch.cuda.synchronize()
        out[f"step_ms_{mode}"] = round(e0.elapsed_time(e1) / args.speedy_steps, 4)
    out["window_ms_graph"] = round(26 * out["step_ms_graph"], 3)
    out["note"] = ("dynamics only (grtend/sptend/implic/hordif/timint, 164 transforms as 7 batched launches); "
                   "physics not on the GPU, not part of the headline value")
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle

        s = oracle.dyn_state_copy(st)
        oracle.dyn_step(s, forcing["phis"], forcing["tcorh"], forcing["qcorh"], None, 2, 2, 2 * DELT, 0.5)
        t0 = time.perf_counter()
        nrep = 5
        for _ in range(nrep):
            oracle.dyn_step(s, forcing["phis"], forcing["tcorh"], forcing["qcorh"], None, 2, 2, 2 * DELT, 0.5)
        out["cpu_oracle_step_ms"] = round((time.perf_counter() - t0) / nrep * 1e3, 3)
        out["cpu_oracle_note"] = "oracle C restatement (long-double DFT instead of FFTPACK), 1 core"
    dyn.close()
    return out


def hybrid_leg(dev, world, res, exchange, io, grids, args):
    """Supplementary measurement, BASELINE configs[2] shape (dynamics only): one
    hybrid step = predict for every local region -> RCCL all-gather -> assemble ->
    iogrid(30) -> stepone + 24 leapfrog steps of the dynamical core -> iogrid(31)
    -> re-tile feedback and local model.  Every stage on the GPU, no host sync
    inside the step.  Physics (phypar) is not computed (zero tendencies), so this
    is not the reference's full window and not the headline value."""
    import torch
    import torch.distributed as dist

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state

    fb, lm, ov = io
    g4, g2, pr, f4, f2, tisr = grids
    _, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)

    def hstep():
        res.predict(fb, lm, ov)
        glob = exchange(ov)
        res.assemble(glob, g4, g2, pr)
        dyn.from_grid(g4, g2)   # iogrid(30), min/max for the safety check stay on the device
        dyn.window(24)          # stepone + 24 x step(2,2) (hipGraph replay)
        dyn.to_grid(f4, f2)     # iogrid(31)
        res.tile_inputs(g4, g2, pr, f4, f2, tisr, fb, lm)

    for _ in range(2):
        hstep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.hybrid_steps):
        hstep()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    _, safe = dyn.from_grid(g4.cpu().numpy(), g2.cpu().numpy())
    dyn.close()
    return {
        "value": round(args.hybrid_steps / dt, 3),
        "unit": "hybrid timesteps/s",
        "ms_per_step": round(dt / args.hybrid_steps * 1e3, 4),
        "steps": args.hybrid_steps,
        "last_window_safe": bool(safe),
        "note": "configs[2] shape without physics: SPEEDY window = iogrid(30) + stepone + 24 leapfrog dynamics "
                "steps + iogrid(31), replicated on every rank; phypar not on the GPU yet",
    }


def training_leg(dev, mask, args):
    """Supplementary measurement (BASELINE configs[4] shape on one GPU): W_out ridge
    training for a batch of 6000-node-class regions -- chunking_matmul Gram and
    cross products (hand-written fp64 MFMA kernel) over args.train_steps time steps
    in 4 batches, then regularisation + batched Cholesky solve (rocSOLVER).
    Roofline: Gram kernel flops / its time vs the measured fp64 MFMA rate."""
    import ctypes

    import torch

    from speedy_ml_amd import domain
    from speedy_ml_amd._lib import check, lib
    from speedy_ml_amd.training import Trainer

    regions = [r * (1152 // args.train_regions) for r in range(args.train_regions)]
    naug = [132 + domain.reservoir_sizes(r, bool(mask[r])).n for r in regions]
    nb = 4
    m = args.train_steps // nb
    gen = torch.Generator(device=dev)
    gen.manual_seed(3)
    S = torch.tanh(torch.randn(sum(naug) * m, dtype=torch.float64, device=dev, generator=gen))
    T = torch.randn(len(naug) * m * 136, dtype=torch.float64, device=dev, generator=gen)
    tr = Trainer(naug)
    tr.accumulate(S, T, m)  # warm-up
    tr.reset()
    torch.cuda.synchronize()
    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    e0.record()
    for _ in range(nb):
        tr.accumulate(S, T, m)
    e1.record()
    _, info = tr.solve()
    e2.record()
    torch.cuda.synchronize()
    gram_ms = e0.elapsed_time(e1)
    solve_ms = e1.elapsed_time(e2)
    npad = tr.npad
    # algorithmic flops: lower-triangle Gram (naug(naug+1)/2 dot products) + T S^T, 2 flops per FMA
    algo = sum(2.0 * (n * (n + 1) / 2 + 136 * n) * m * nb for n in naug)
    # executed by the tiles (128 x 128, padded): the MFMA work actually issued
    C = npad // 128
    issued = len(naug) * (C * (C + 1) // 2 + 2 * C) * 2.0 * 128 * 128 * m * nb
    peak = ctypes.c_double()
    check(lib().sml_probe_mfma_f64(20000, ctypes.byref(peak)))
    tr.close()
    achieved = algo / (gram_ms * 1e-3) / 1e12
    return {
        "workload": f"{len(naug)} regions (naug {min(naug)}..{max(naug)}), {m * nb} training steps in {nb} "
                    "chunking_matmul batches, then fit_chunk_hybrid regularisation + solve",
        "gram_ms": round(gram_ms, 3),
        "solve_ms": round(solve_ms, 3),
        "solve_info_ok": bool((info == 0).all()),
        "roofline": {
            "kernel": "k_train_gram (fp64 MFMA 16x16x4, 128x128 tiles, lower triangle + T S^T strip)",
            "bound": "mfma", "unit": "TFLOP/s",
            "achieved": round(achieved, 2),
            "issued_tflops": round(issued / (gram_ms * 1e-3) / 1e12, 2),
            "peak": round(peak.value, 2),
            "peak_source": "measured: back-to-back v_mfma_f64_16x16x4_f64 on every SIMD (sml_probe_mfma_f64)",
            "frac": round(achieved / peak.value, 4),
            "algorithmic_flops": algo,
        },
    }


def cpu_baseline(sample: int, nreg: int, mask):
    """The oracle's restatement of predict (dense W_in matmul, COO SpMV, dense W_out
    GEMV: the reference's arithmetic) timed on one host core over a bounded sample
    of regions spread over the shape classes, plus the exchange/tiling oracle on
    every region; extrapolated to one hybrid step of all 1152 regions."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    from speedy_ml_amd import domain
    from speedy_ml_amd.synthetic import feedback_vector, initial_state, local_model_vector, region_weights

    stride = max(1, nreg // sample)
    picks = list(range(0, nreg, stride))[:sample]
    t_pred = 0.0
    for r in picks:
        w = region_weights(r, bool(mask[r]))
        win = w.win.astype(np.float64)
        wout = w.wout.astype(np.float64)
        vals = w.vals.astype(np.float64)
        x = initial_state(r, w.n)
        fb = feedback_vector(r, w.ninp)
        lm = local_model_vector(r)
        t0 = time.perf_counter()
        oracle.predict(w.rows, w.cols, vals, win, wout, fb, lm, x, w.mean, w.std)
        t_pred += time.perf_counter() - t0
    per_region = t_pred / len(picks)
    # exchange on the host: assemble + tile every region (root-serial in the reference)
    outvecs = np.random.default_rng(0).standard_normal((nreg, 136))
    g4, g2, pr = (None, None, None)
    t0 = time.perf_counter()
    g4, g2, pr = oracle.assemble(outvecs)
    ms = np.ones(36)
    for r in range(nreg):
        oracle.tile_feedback(r, g4, g2, pr, np.zeros(36), ms, np.zeros(16))
        oracle.tile_local_model(r, g4, g2, np.zeros(36), ms)
    t_xchg = time.perf_counter() - t0
    step_s = per_region * nreg + t_xchg
    return {
        "value": round(1.0 / step_s, 4),
        "unit": "hybrid timesteps/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle predict (dense W_in as the reference) timed on {len(picks)} of {nreg} regions "
                  f"(every {stride}th, all shape classes), {per_region * 1e3:.3f} ms/region, extrapolated to "
                  f"{nreg}; + host assemble/tile of all regions {t_xchg * 1e3:.1f} ms; "
                  f"host {platform.processor() or platform.machine()}, {os.cpu_count()} logical CPUs visible",
    }


if __name__ == "__main__":
    main()

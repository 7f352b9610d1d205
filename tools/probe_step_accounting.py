"""The N = 1 step accounting: where the bench's 0.88-ms step goes
against the window's 0.74 ms alone.  Runs the bench's loop (full size, overlap +
pipelined + slab ocean + date forcing, run_speedy polled per step) with the timeline
build of the library (sml_timeline.hpp: per-block plain stores, no atomics), then the same window alone and the same begin
alone, and prints one table:

  * each piece of the window in the loop vs alone: its span, the 26 row kernels, the
    26 per-m kernels, the kernel boundaries between them;
  * the begin (update + v_ml readout) in the loop vs alone;
  * the chain between two windows, kernel by kernel (start / end after the window's
    last kernel): the exit, the forecast hop's store, the finish (from the forecast's
    arrival), the grid hop's signal, the re-tiling, the entry specx (from the grid's
    arrival), k_io_entry, the next window's first row kernel.

    bash tools/build_variant.sh tl 'EXTRA=-DSML_TL'
    SML_LIB=abx/tl/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_step_accounting.py \
        [--sim-ranks N] [--json OUT]

--sim-ranks N: rank 0's share of an N-rank decomposition with bench.py --sim-ranks'
stand-in exchange (the chain at N > 1: the finish, the exchange copy, k_assemble).

wall_clock64 stamps (100 MHz) from thread 0 of every block; untraced.  The timeline
build's step rate is printed beside the table (its stamps cost a load at each block's
start and two stores at its end)."""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
from speedy_ml_amd import domain  # noqa: E402
from speedy_ml_amd._lib import check, lib, ptr  # noqa: E402
from speedy_ml_amd.dynamics import Dynamics  # noqa: E402
from speedy_ml_amd.exchange import OutvecExchange  # noqa: E402
from speedy_ml_amd.hybrid import HybridLoop, SlabOcean  # noqa: E402
from speedy_ml_amd.reservoir import Reservoirs  # noqa: E402
from speedy_ml_amd.synthetic import (dyn_state, initial_state, phys_boundary, region_weights, slab_fields,  # noqa: E402
                                     slab_start_outvec, slab_weights, surface_climatology, synthetic_grids)

KINDS = ("entry_specx", "io_entry", "row", "spec", "exit_gridx", "exit_store", "finish", "hop_signal", "tile_feedback",
         "update", "readout", "fordate", "check_minmax", "assemble")
WARMUP, STEPS = 20, 300


RING = (1024, 1024, 16384, 16384, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024, 1024)  # sml_timeline.hpp
BLOCKS = (64, 64, 64, 64, 64, 1, 2048, 1, 1024, 2048, 8192, 32, 4, 1024)
MAX_BLOCKS = 8192


class Timeline:
    """sml_dbg_timeline's buffer: per kind, a ring of launches x recorded blocks of
    (start, end) wall_clock64 pairs, and per (kind, block) the launches recorded."""

    def __init__(self):
        self.reset()

    def reset(self):
        d, n = ctypes.c_void_p(), ctypes.c_int64()
        check(lib().sml_dbg_timeline(ctypes.byref(d), ctypes.byref(n), 1))
        self.d, self.size = d.value, n.value

    def read(self):
        raw = np.zeros(self.size // 8, np.uint64)
        check(lib().sml_copy_to_host(ptr(raw), ctypes.c_void_p(self.d), raw.nbytes))
        cnt = raw[:len(KINDS) * MAX_BLOCKS // 2].view(np.uint32).reshape(len(KINDS), MAX_BLOCKS)
        logs, o = {}, len(KINDS) * MAX_BLOCKS // 2
        for k, name in enumerate(KINDS):
            n = RING[k] * BLOCKS[k] * 5
            logs[name] = raw[o:o + n].reshape(RING[k], BLOCKS[k], 5).astype(np.int64)
            o += n
        return cnt, logs


def launches(rd, kind, clock=False):
    """(start, end) in us of every launch of a kind since the last reset, in order;
    clock: the median over its blocks of the shader clock (GHz) they ran at instead.
    Block b's records advance only in launches of more than b blocks: walk block 0's
    records (every launch) with a cursor per block."""
    cnt, logs = rd
    k = KINDS.index(kind)
    n = int(cnt[k, 0])
    lg = logs[kind]
    R, B = lg.shape[0], lg.shape[1]
    assert n <= R, (kind, n)
    cur = np.zeros(B, np.int64)
    out = []
    for c in range(n):
        g = int(min(lg[c % R, 0, 4], B))  # this launch's grid (recorded blocks)
        idx = cur[:g] % R
        rec = lg[idx, np.arange(g)]
        cur[:g] += 1
        s, e = rec[:, 0], rec[:, 1]
        ok = s > 0
        if clock:
            dw, dc = (e - s)[ok], (rec[:, 3] - rec[:, 2])[ok]
            good = dw > 50  # blocks of at least 0.5 us
            out.append(float(np.median(dc[good] / (dw[good] * 10.0))) if good.any() else float("nan"))
        else:
            out.append((s[ok].min() / 100.0, e[ok].max() / 100.0))  # 100 MHz ticks -> us
    return out


def build(dev, sim):
    """sim > 1: rank 0's share of a sim-rank decomposition with bench.py --sim-ranks'
    stand-in exchange (the other ranks' rows copied once from this rank's)."""
    mask = domain.load_sst_mask()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    regions = domain.processor_decomposition(1152, sim, 0)
    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in regions]
    res = Reservoirs(regions, [mask[r] for r in regions], [s.n for s in sizes], [s.k for s in sizes])
    for i, r in enumerate(regions):
        w = region_weights(r, bool(mask[r]), climatology=True)
        res.load_region_weights(i, w)
        res.set_state(i, initial_state(r, w.n))
    sreg = [r for r in regions if mask[r]]
    sws = [slab_weights(r) for r in sreg]
    slab = Reservoirs(sreg, [0] * len(sreg), [w.n for w in sws], [w.k for w in sws], chunk_speedy=0, nout=4,
                      ninp=[w.ninp for w in sws], out_index=[35] * 4)
    for j, w in enumerate(sws):
        slab.load_region_weights(j, w)
        slab.set_state(j, initial_state(sreg[j], w.n, seed=17))
    base, smask, sice, tice = slab_fields()
    st0, forcing = dyn_state()
    dyn = Dynamics()
    dyn.set_forcing(**forcing)
    dyn.set_state(st0)
    bc = phys_boundary(dyn, forcing["phis"])
    surf, clim = surface_climatology(bc["fmask1"])
    bc["fmask1"] = surf["fmask_l"]
    dyn.set_physics(bc)
    dyn.set_surface(surf)
    dyn.set_climatology(clim)
    check(lib().sml_dyn_set_sea_ice(dyn._h, ptr(np.ascontiguousarray(sice)), ptr(np.ascontiguousarray(tice))))
    tisr = t(np.random.default_rng(13).standard_normal((len(regions), 16)))
    so = SlabOcean(slab, t(base), t(smask))
    exchange = OutvecExchange(1152, 1, 0, device=dev, nout=140)
    if sim > 1:
        glob = torch.zeros((1152, 140), dtype=torch.float64, device=dev)
        filled = []

        def exchange(ov_local):
            if not filled:
                glob.copy_(ov_local[torch.arange(1152, device=dev) % len(regions)])
                filled.append(True)
            glob[:len(regions)].copy_(ov_local)
            return glob
    loop = HybridLoop(res, dyn, exchange, dev, tisr=tisr, slab=so)
    loop.set_calendar(1981, 24 * 365, 6)
    loop.set_pipelined(True)
    g4, g2, pr = synthetic_grids(11)
    f4, f2, _ = synthetic_grids(12)
    loop.start(t(g4), t(g2), t(pr), t(f4), t(f2))
    loop.start_slab(t(np.stack([slab_start_outvec(r) for r in sreg])))
    loop.sync()
    return loop, slab


def med(v):
    return statistics.median(v) if v else float("nan")


def window_pieces(rows, specs):
    span = specs[-1][1] - rows[0][0]
    rk = sum(b - a for a, b in rows)
    sk = sum(b - a for a, b in specs)
    return {"span": span, "row_kernels": rk, "per_m_kernels": sk, "boundaries": span - rk - sk}


def main():
    dev = torch.device("cuda", 0)
    sim = int(sys.argv[sys.argv.index("--sim-ranks") + 1]) if "--sim-ranks" in sys.argv else 1
    tl = Timeline()
    loop, slab = build(dev, sim)
    poll = (lambda: True) if sim > 1 else loop.run_speedy  # (the stand-in exchange's other ranks stay stale)
    for _ in range(WARMUP):
        loop.step()
        assert poll()
    loop.sync()
    torch.cuda.synchronize()
    tl.reset()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        loop.step()
        assert poll()
    loop.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rd = tl.read()
    n = {k: int(rd[0][i, 0]) for i, k in enumerate(KINDS)}
    print(f"timeline build: {STEPS / dt:.1f} steps/s ({dt / STEPS * 1e3:.4f} ms per step); launches {n}")
    get = lambda k: launches(rd, k)  # noqa: E731
    io = get("io_entry")
    rows, specs = get("row"), get("spec")
    assert len(rows) == 26 * len(io) and len(specs) == 26 * len(io), (len(rows), len(specs), len(io))
    wins = [window_pieces(rows[26 * i:26 * i + 26], specs[26 * i:26 * i + 26]) for i in range(len(io))]
    upd, rdo = get("update"), get("readout")
    upd_min = sorted(b - a for a, b in upd)[len(upd) // 2]  # the atmo launches are the majority
    rdo_min = sorted(b - a for a, b in rdo)[len(rdo) // 2]
    # the slab steps add a slab begin (update + readout of the slab reservoirs): the atmo
    # begin is the launch pair that starts right after each step's tiling
    tiles = get("tile_feedback")
    exit_g, store, fin, hop, ent = get("exit_gridx"), get("exit_store"), get("finish"), get("hop_signal"), get("entry_specx")
    ford = get("fordate")
    # per step i (window i): chain from window i's end to window i+1's first row kernel
    asm = get("assemble")
    chain = {k: [] for k in ("exit_gridx", "exit_store", "finish", "assemble", "hop_signal", "tile_feedback",
                             "entry_specx", "io_entry", "next_row")}
    begin_in = []
    for i in range(len(io) - 1):
        w_end = specs[26 * i + 25][1]
        nxt = rows[26 * (i + 1)][0]

        def after(lst, key):
            c = [x for x in lst if x[0] >= w_end - 1.0 and x[0] <= nxt + 1.0]
            if c:
                chain[key].append((c[0][0] - w_end, c[0][1] - w_end))
        after(exit_g, "exit_gridx")
        after(store, "exit_store")
        after(fin, "finish")
        after(asm, "assemble")
        after(hop, "hop_signal")
        after(tiles, "tile_feedback")
        after(ent, "entry_specx")
        after(io, "io_entry")
        chain["next_row"].append((nxt - w_end, nxt - w_end))
        # the begin issued after this step's tiling: the atmo update + v_ml readout
        # starting after it (a slab step's slab predict launches the same kernels for
        # 4032-node reservoirs, far shorter: the first long launch of each is the atmo's)
        tl_i = [x for x in tiles if x[0] >= w_end - 1.0 and x[0] <= nxt + 1.0]
        if tl_i and i + 1 < len(io):
            u = [x for x in upd if x[0] >= tl_i[0][1] - 1.0 and x[1] - x[0] >= 0.5 * upd_min][:1]
            r_ = [x for x in rdo if u and x[0] >= u[0][1] - 1.0 and x[1] - x[0] >= 0.5 * rdo_min][:1]
            if u and r_:
                begin_in.append({"update": u[0][1] - u[0][0], "readout": r_[0][1] - r_[0][0],
                                 "begin": r_[0][1] - u[0][0], "begin_start_after_window_start": u[0][0] - nxt,
                                 "begin_end_before_next_window_end": specs[26 * (i + 1) + 25][1] - r_[0][1]})
    period = [io[i + 1][0] - io[i][0] for i in range(len(io) - 1)]
    # per step of the window (0 = stepone's first half step ... 25): row / per-m kernel
    # durations and the boundary after each, in the loop
    def per_step(rw, sp, nwin):
        out = []
        for q in range(26):
            r_ = [rw[26 * i + q][1] - rw[26 * i + q][0] for i in range(nwin)]
            s_ = [sp[26 * i + q][1] - sp[26 * i + q][0] for i in range(nwin)]
            b_ = [sp[26 * i + q][0] - rw[26 * i + q][1] for i in range(nwin)]
            out.append((med(r_), med(s_), med(b_)))
        return out
    ps_in = per_step(rows, specs, len(io))
    clk_in = {"row": med(launches(rd, "row", True)), "spec": med(launches(rd, "spec", True)),
              "readout": med(launches(rd, "readout", True))}
    # ---- the window alone (dyn.window, the same context, nothing beside it)
    tl.reset()
    dyn = loop.dyn
    for _ in range(30):
        dyn.window(24)
    torch.cuda.synchronize()
    rda = tl.read()
    ga = lambda k: launches(rda, k)  # noqa: E731
    ra, sa = ga("row"), ga("spec")
    alone = [window_pieces(ra[26 * i:26 * i + 26], sa[26 * i:26 * i + 26]) for i in range(5, len(ra) // 26)]
    ps_alone = per_step(ra[130:], sa[130:], len(ra) // 26 - 5)
    clk_alone = {"row": med(launches(rda, "row", True)[130:]), "spec": med(launches(rda, "spec", True)[130:])}
    # ---- run_model alone from the loop's last assembled grid (the same entry state the
    # in-step windows start from; nothing beside it): in-step vs alone with the same data
    tl.reset()
    f4b, f2b = torch.zeros_like(loop.f4), torch.zeros_like(loop.f2)
    for _ in range(30):
        dyn.run_model(loop.g4, loop.g2, f4b, f2b, stream=loop.side)
    torch.cuda.synchronize()
    rdm = tl.read()
    rm, sm_ = launches(rdm, "row"), launches(rdm, "spec")
    alone_rm = [window_pieces(rm[26 * i:26 * i + 26], sm_[26 * i:26 * i + 26]) for i in range(5, len(rm) // 26)]
    # ---- the begin alone on the reservoir's stream (its 192 CUs, nothing beside it)
    tl.reset()
    res = loop.res
    for _ in range(20):
        res.predict_finish(loop.lm, loop.ov, stream=loop.main)
        res.predict_begin(loop.fb, stream=loop.main)
    torch.cuda.synchronize()
    rdb = tl.read()
    gb = lambda k: launches(rdb, k)  # noqa: E731
    ub, rb = gb("update"), gb("readout")
    begin_alone = [{"update": u[1] - u[0], "readout": r[1] - r[0], "begin": r[1] - u[0]} for u, r in zip(ub[2:], rb[2:])]
    out = {"sim_ranks": sim, "steps_per_s_timeline_build": STEPS / dt, "step_period_us": med(period),
           "window": {"in_step": {k: med([w[k] for w in wins]) for k in wins[0]},
                      "alone": {k: med([w[k] for w in alone]) for k in alone[0]},
                      "run_model_alone": {k: med([w[k] for w in alone_rm]) for k in alone_rm[0]}},
           "begin": {"in_step": {k: med([b[k] for b in begin_in]) for k in begin_in[0]} if begin_in else {},
                     "alone": {k: med([b[k] for b in begin_alone]) for k in begin_alone[0]}},
           "chain_after_window_end_us": {k: {"start": med([v[0] for v in vs]), "end": med([v[1] for v in vs]),
                                             "n": len(vs)} for k, vs in chain.items()},
           "fordate_us": med([b - a for a, b in ford]), "fordates": len(ford),
           "per_window_step_us": {"in_step": ps_in, "alone": ps_alone},
           "shader_clock_ghz": {"in_step": clk_in, "alone": clk_alone}}
    print(f"step period (io_entry to io_entry) {out['step_period_us']:.1f} us")
    print(f"{'window (us)':24s} {'in step':>9s} {'alone':>9s} {'diff':>8s} {'run_model alone':>16s}")
    for k in ("span", "row_kernels", "per_m_kernels", "boundaries"):
        a, b = out["window"]["in_step"][k], out["window"]["alone"][k]
        print(f"  {k:22s} {a:9.1f} {b:9.1f} {a - b:8.1f} {out['window']['run_model_alone'][k]:16.1f}")
    print(f"{'begin (us)':24s} {'in step':>9s} {'alone':>9s}")
    for k in ("update", "readout", "begin"):
        print(f"  {k:22s} {out['begin']['in_step'].get(k, float('nan')):9.1f} {out['begin']['alone'][k]:9.1f}")
    for k in ("begin_start_after_window_start", "begin_end_before_next_window_end"):
        print(f"  {k:38s} {out['begin']['in_step'].get(k, float('nan')):9.1f}")
    print("chain after the window's last kernel (us):  start    end")
    for k, v in out["chain_after_window_end_us"].items():
        print(f"  {k:38s} {v['start']:7.1f} {v['end']:7.1f}  (n {v['n']})")
    print(f"shader clock (GHz, median over blocks): in step {clk_in}, alone {clk_alone}")
    print("per window step: row kernel / per-m kernel / row->per-m boundary, in step minus alone (us)")
    for q in range(26):
        a, b = ps_in[q], ps_alone[q]
        print(f"  step {q:2d}  row {a[0]:6.2f} ({a[0] - b[0]:+5.2f})  per-m {a[1]:6.2f} ({a[1] - b[1]:+5.2f})  "
              f"boundary {a[2]:5.2f} ({a[2] - b[2]:+5.2f})")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    loop.close()
    slab.close()


if __name__ == "__main__":
    main()

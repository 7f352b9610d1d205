"""The N = 1 step accounting: where the bench's 0.88-ms step goes
against the window's 0.74 ms alone.  Runs the bench's loop (full size, overlap +
pipelined + slab ocean + date forcing, run_speedy polled per step) with the timeline
build of the library (sml_timeline.hpp), then the same window alone and the same begin
alone, and prints one table:

  * each piece of the window in the loop vs alone: its span, the 26 row kernels, the
    26 per-m kernels, the kernel boundaries between them;
  * the begin (update + v_ml readout) in the loop vs alone;
  * the chain between two windows, kernel by kernel (start / end after the window's
    last kernel): the exit, the forecast hop's store, the finish (from the forecast's
    arrival), the grid hop's signal, the re-tiling, the entry specx (from the grid's
    arrival), k_io_entry, the next window's first row kernel.

    bash tools/build_variant.sh tl 'EXTRA=-DSML_TL'
    SML_LIB=abx/tl/speedy-ml-1_amd/lib/libspeedyml.so python tools/probe_step_accounting.py [--json OUT]

wall_clock64 stamps (100 MHz) from thread 0 of every block; untraced.  The timeline
build's stamps cost a few atomics per block: its step rate is printed beside the table."""
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
         "update", "readout", "fordate", "check_minmax")
WARMUP, STEPS = 20, 300


class Timeline:
    def __init__(self):
        d, k, r = ctypes.c_void_p(), ctypes.c_int(), ctypes.c_int()
        check(lib().sml_dbg_timeline(ctypes.byref(d), ctypes.byref(k), ctypes.byref(r)))
        assert k.value == len(KINDS), k.value
        self.d, self.kinds, self.ring = d.value, k.value, r.value
        self.off_t0 = ((8 * self.kinds + 4 * self.kinds) + 7) // 8 * 8
        self.size = self.off_t0 + 2 * self.kinds * self.ring * 8

    def read(self):
        raw = np.zeros(self.size // 8, np.uint64)
        check(lib().sml_copy_to_host(ptr(raw), ctypes.c_void_p(self.d), raw.nbytes))
        seq = raw[:self.kinds].astype(np.int64)
        t = raw[self.off_t0 // 8:].reshape(2, self.kinds, self.ring)
        return seq, t[0], t[1]


def launches(tl_read, kind, lo, hi):
    """(start, end) in us of launches lo..hi-1 of a kind."""
    seq, t0, t1 = tl_read
    k = KINDS.index(kind)
    out = []
    for s in range(lo, hi):
        a, b = int(t0[k, s % 16384]), int(t1[k, s % 16384])
        out.append((a / 100.0, b / 100.0))  # 100 MHz ticks -> us
    return out


def build(dev):
    mask = domain.load_sst_mask()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    sizes = [domain.reservoir_sizes(r, bool(mask[r])) for r in range(1152)]
    res = Reservoirs(list(range(1152)), mask, [s.n for s in sizes], [s.k for s in sizes])
    for r in range(1152):
        w = region_weights(r, bool(mask[r]), climatology=True)
        res.load_region_weights(r, w)
        res.set_state(r, initial_state(r, w.n))
    sreg = [r for r in range(1152) if mask[r]]
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
    tisr = t(np.random.default_rng(13).standard_normal((1152, 16)))
    so = SlabOcean(slab, t(base), t(smask))
    loop = HybridLoop(res, dyn, OutvecExchange(1152, 1, 0, device=dev, nout=140), dev, tisr=tisr, slab=so)
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
    tl = Timeline()
    loop, slab = build(dev)
    for _ in range(WARMUP):
        loop.step()
        assert loop.run_speedy()
    loop.sync()
    torch.cuda.synchronize()
    seq0 = tl.read()[0].copy()
    t0 = time.perf_counter()
    for _ in range(STEPS):
        loop.step()
        assert loop.run_speedy()
    loop.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    rd = tl.read()
    seq1 = rd[0].copy()
    n = {k: int(seq1[i] - seq0[i]) for i, k in enumerate(KINDS)}
    print(f"timeline build: {STEPS / dt:.1f} steps/s ({dt / STEPS * 1e3:.4f} ms per step); launches {n}")
    get = lambda k: launches(rd, k, int(seq0[KINDS.index(k)]), int(seq1[KINDS.index(k)]))  # noqa: E731
    io = get("io_entry")
    rows, specs = get("row"), get("spec")
    assert len(rows) == 26 * len(io) and len(specs) == 26 * len(io), (len(rows), len(specs), len(io))
    wins = [window_pieces(rows[26 * i:26 * i + 26], specs[26 * i:26 * i + 26]) for i in range(len(io))]
    upd, rdo = get("update"), get("readout")
    # the slab steps add a slab begin (update + readout of the slab reservoirs): the atmo
    # begin is the launch pair that starts right after each step's tiling
    tiles = get("tile_feedback")
    exit_g, store, fin, hop, ent = get("exit_gridx"), get("exit_store"), get("finish"), get("hop_signal"), get("entry_specx")
    ford = get("fordate")
    # per step i (window i): chain from window i's end to window i+1's first row kernel
    chain = {k: [] for k in ("exit_gridx", "exit_store", "finish", "hop_signal", "tile_feedback", "entry_specx",
                             "io_entry", "next_row")}
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
        after(hop, "hop_signal")
        after(tiles, "tile_feedback")
        after(ent, "entry_specx")
        after(io, "io_entry")
        chain["next_row"].append((nxt - w_end, nxt - w_end))
        # the begin issued after this step's tiling: update + readout starting after it
        tl_i = [x for x in tiles if x[0] >= w_end - 1.0 and x[0] <= nxt + 1.0]
        if tl_i:
            u = [x for x in upd if x[0] >= tl_i[0][1] - 1.0][:1]
            r_ = [x for x in rdo if u and x[0] >= u[0][1] - 1.0][:1]
            if u and r_:
                begin_in.append({"update": u[0][1] - u[0][0], "readout": r_[0][1] - r_[0][0],
                                 "begin": r_[0][1] - u[0][0], "begin_start_after_window_start": u[0][0] - nxt,
                                 "begin_end_after_next_window_end": r_[0][1] - specs[26 * (i + 1) + 25][1]})
    period = [io[i + 1][0] - io[i][0] for i in range(len(io) - 1)]
    # ---- the window alone (dyn.window, the same context, nothing beside it)
    seqa = tl.read()[0].copy()
    dyn = loop.dyn
    for _ in range(30):
        dyn.window(24)
    torch.cuda.synchronize()
    rda = tl.read()
    ga = lambda k: launches(rda, k, int(seqa[KINDS.index(k)]), int(rda[0][KINDS.index(k)]))  # noqa: E731
    ra, sa = ga("row"), ga("spec")
    alone = [window_pieces(ra[26 * i:26 * i + 26], sa[26 * i:26 * i + 26]) for i in range(5, len(ra) // 26)]
    # ---- the begin alone on the reservoir's stream (its 192 CUs, nothing beside it)
    seqb = tl.read()[0].copy()
    res = loop.res
    for _ in range(20):
        res.predict_finish(loop.lm, loop.ov, stream=loop.main)
        res.predict_begin(loop.fb, stream=loop.main)
    torch.cuda.synchronize()
    rdb = tl.read()
    gb = lambda k: launches(rdb, k, int(seqb[KINDS.index(k)]), int(rdb[0][KINDS.index(k)]))  # noqa: E731
    ub, rb = gb("update"), gb("readout")
    begin_alone = [{"update": u[1] - u[0], "readout": r[1] - r[0], "begin": r[1] - u[0]} for u, r in zip(ub[2:], rb[2:])]
    out = {"steps_per_s_timeline_build": STEPS / dt, "step_period_us": med(period),
           "window": {"in_step": {k: med([w[k] for w in wins]) for k in wins[0]},
                      "alone": {k: med([w[k] for w in alone]) for k in alone[0]}},
           "begin": {"in_step": {k: med([b[k] for b in begin_in]) for k in begin_in[0]} if begin_in else {},
                     "alone": {k: med([b[k] for b in begin_alone]) for k in begin_alone[0]}},
           "chain_after_window_end_us": {k: {"start": med([v[0] for v in vs]), "end": med([v[1] for v in vs]),
                                             "n": len(vs)} for k, vs in chain.items()},
           "fordate_us": med([b - a for a, b in ford]), "fordates": len(ford)}
    print(f"step period (io_entry to io_entry) {out['step_period_us']:.1f} us")
    print(f"{'window (us)':24s} {'in step':>9s} {'alone':>9s} {'diff':>8s}")
    for k in ("span", "row_kernels", "per_m_kernels", "boundaries"):
        a, b = out["window"]["in_step"][k], out["window"]["alone"][k]
        print(f"  {k:22s} {a:9.1f} {b:9.1f} {a - b:8.1f}")
    print(f"{'begin (us)':24s} {'in step':>9s} {'alone':>9s}")
    for k in ("update", "readout", "begin"):
        print(f"  {k:22s} {out['begin']['in_step'].get(k, float('nan')):9.1f} {out['begin']['alone'][k]:9.1f}")
    for k in ("begin_start_after_window_start", "begin_end_after_next_window_end"):
        print(f"  {k:38s} {out['begin']['in_step'].get(k, float('nan')):9.1f}")
    print("chain after the window's last kernel (us):  start    end")
    for k, v in out["chain_after_window_end_us"].items():
        print(f"  {k:38s} {v['start']:7.1f} {v['end']:7.1f}  (n {v['n']})")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)
    loop.close()
    slab.close()


if __name__ == "__main__":
    main()

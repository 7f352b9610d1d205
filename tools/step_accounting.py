"""Where the hybrid step's time goes: from a rocprofv3 kernel
trace of bench.py (profiles/collect.sh's trace pass), one table of

  * the window's pieces in the loop (beside the reservoir's begin) against the same
    window alone (the bench's speedy leg, dyn.window): the 26 row kernels
    (k_st_gridspec_p), the 26 per-m kernels (k_st_spec), the boundaries between them;
  * each kernel of the serial chain between two windows: run_model's exit (k_gridx),
    the forecast hop's store, the v_p finish (+ the one-rank assembly), the grid hop's
    signal, iogrid(30)'s entry specx, k_io_entry, and the gaps between them.

    python tools/step_accounting.py TRACE.csv [--json OUT.json]

Medians over the steps; microseconds.  A traced run dispatches a little slower than
an untraced one, so the step period here is longer than the bench's; the split of the
period is what the table is for."""
import csv
import json
import statistics
import sys


def load(path):
    rows = []
    for x in csv.DictReader(open(path)):
        n = x["Kernel_Name"]
        rows.append((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), n, x["Queue_Id"]))
    rows.sort()
    return rows


def short(name):
    for k in ("k_st_gridspec_p", "k_st_spec", "k_io_entry", "k_specx", "k_gridx", "k_flag_store", "k_hop_signal",
              "k_res_finish_grid", "k_res_update_bal", "k_res_readout", "k_tile_feedback", "k_slab_ring",
              "k_fordate", "k_io_minmax", "k_gridy", "k_st_inv", "k_state_to_m", "k_assemble", "k_specy",
              "k_hop_wait", "k_sst_grid", "k_sst_feedback", "k_hybrid_sst", "k_slab_avg", "k_slab_rows",
              "k_res_update", "k_tile_local_model"):
        if k in name:
            return k
    return name[:40]


def windows(rows, queue):
    """Runs of 26 (row kernel, per-m kernel) pairs on SPEEDY's queue, with what precedes them."""
    q = [r for r in rows if r[3] == queue]
    out = []
    i = 0
    while i < len(q):
        if short(q[i][2]) == "k_st_gridspec_p":
            j = i
            ks = []
            while j < len(q) and short(q[j][2]) in ("k_st_gridspec_p", "k_st_spec"):
                ks.append(q[j])
                j += 1
            prev = short(q[i - 1][2]) if i > 0 else ""
            out.append((prev, ks, i, j))
            i = j
        else:
            i += 1
    return q, out


def window_pieces(ks):
    g = [k for k in ks if short(k[2]) == "k_st_gridspec_p"]
    s = [k for k in ks if short(k[2]) == "k_st_spec"]
    gaps = [ks[t + 1][0] - ks[t][1] for t in range(len(ks) - 1)]
    return {"span": (ks[-1][1] - ks[0][0]) / 1e3, "row_kernels": sum(e - b for b, e, *_ in g) / 1e3,
            "per_m_kernels": sum(e - b for b, e, *_ in s) / 1e3, "boundaries": sum(gaps) / 1e3,
            "n_row": len(g), "n_m": len(s)}


def main():
    path = sys.argv[1]
    rows = load(path)
    # SPEEDY's queue: the one running the row kernels inside the loop (after k_io_entry)
    qs = {}
    for r in rows:
        if short(r[2]) == "k_io_entry":
            qs[r[3]] = qs.get(r[3], 0) + 1
    squeue = max(qs, key=qs.get)
    q, wins = windows(rows, squeue)
    in_step = [w for w in wins if w[0] == "k_io_entry" and len(w[1]) == 52]
    alone = [w for w in wins if w[0] in ("k_st_inv", "k_state_to_m") and len(w[1]) == 52]
    med = lambda v: statistics.median(v) if v else float("nan")  # noqa: E731
    table = {}
    for name, ws in (("in_step", in_step), ("alone", alone)):
        p = [window_pieces(w[1]) for w in ws]
        table[name] = {k: med([x[k] for x in p]) for k in ("span", "row_kernels", "per_m_kernels", "boundaries")}
        table[name]["windows"] = len(ws)
    # the chain around each in-loop window: SPEEDY's queue from the window's end to the
    # next window's first row kernel, the main queue's kernels in that interval
    chain = []
    for a, b in zip(in_step, in_step[1:]):
        t_end = a[1][-1][1]
        t_next = b[1][0][0]
        seg = [r for r in rows if t_end - 1 <= r[0] <= t_next]
        items = []
        for r in seg:
            items.append((short(r[2]), r[3] == squeue, (r[0] - t_end) / 1e3, (r[1] - t_end) / 1e3))
        chain.append(((t_next - t_end) / 1e3, items))
    # per chain kernel: median start / end after the window's last kernel
    keyed = {}
    for total, items in chain:
        seen = {}
        for nm, sp, s0, s1 in items:
            k = (nm, "speedy" if sp else "other")
            if k in seen:
                continue
            seen[k] = (s0, s1)
        for k, v in seen.items():
            keyed.setdefault(k, []).append(v)
    chain_tab = sorted(((med([v[0] for v in vs]), med([v[1] for v in vs]), k, len(vs)) for k, vs in keyed.items()),
                       key=lambda x: x[0])
    period = [b[1][0][0] - a[1][0][0] for a, b in zip(in_step, in_step[1:])]
    out = {"trace": path, "speedy_queue": squeue, "steps": len(in_step), "step_period_us": med(period) / 1e3,
           "window": table, "chain_us_after_window_end": [
               {"kernel": k[0], "queue": k[1], "start": round(s0, 2), "end": round(s1, 2), "dur": round(s1 - s0, 2),
                "n": n} for s0, s1, k, n in chain_tab if n >= len(chain) // 2],
           "window_end_to_next_window_us": med([c[0] for c in chain])}
    print(f"trace {path}: {len(in_step)} in-loop windows, {len(alone)} alone; step period "
          f"{out['step_period_us']:.1f} us (traced)")
    print(f"{'window piece (us)':28s} {'in step':>10s} {'alone':>10s} {'diff':>9s}")
    for k in ("span", "row_kernels", "per_m_kernels", "boundaries"):
        a, b = table["in_step"][k], table["alone"][k]
        print(f"  {k:26s} {a:10.1f} {b:10.1f} {a - b:9.1f}")
    print(f"chain: window end -> next window's first row kernel {out['window_end_to_next_window_us']:.1f} us")
    print(f"  {'kernel':22s} {'queue':7s} {'start':>8s} {'end':>8s} {'dur':>7s}")
    for e in out["chain_us_after_window_end"]:
        print(f"  {e['kernel']:22s} {e['queue']:7s} {e['start']:8.1f} {e['end']:8.1f} {e['dur']:7.1f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()

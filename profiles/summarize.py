"""Condense rocprofv3 output (profiles/collect.sh) into committed summaries.

    python profiles/summarize.py gpurun_out/prof_r01 r01

Writes profiles/<round>_kernel_stats.csv (rocprofv3 --stats, verbatim),
profiles/<round>_summary.md (per-kernel average duration and HBM bytes per
launch) and profiles/readout_pmc.json (the readout kernel's measured HBM traffic,
read by bench.py for roofline.traffic).

HBM bytes follow MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE counts exactly half the bytes of a wide coalesced
streaming read, so the read side is doubled for the 16-B-per-lane streaming
kernels (k_res_readout); other kernels report raw and doubled reads.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys
from collections import defaultdict

HERE = os.path.dirname(os.path.abspath(__file__))


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def _find(root, pattern):
    hits = sorted(glob.glob(os.path.join(root, "**", pattern), recursive=True))
    return hits[0] if hits else None


def _short(name: str) -> str:
    if "k_res_readout" in name:  # <WT, mode[, rows]>: 0 = v_ml half (step_begin), 1 = finish, 2 = one pass
        m = re.search(r"k_res_readout<(\w+), (\d)", name)
        wt = m.group(1) if m else ("float" if ("<float" in name or "IfL" in name) else "double")
        mode = m.group(2) if m else ("1" if "Li1E" in name else "2" if "Li2E" in name else "0")
        return f"k_res_readout_{ {'0': 'ml', '1': 'finish', '2': 'full'}[mode]}<{wt}>"
    for key in ("k_res_readout", "k_res_update_bal", "k_res_update", "k_res_finish_grid", "k_tile_feedback", "k_tile_local_model", "k_assemble",
                "k_gridy", "k_gridx", "k_specx", "k_specy", "k_vds", "k_uvspec"):
        if key in name:
            if "IfE" in name or "<float>" in name:
                return key + "<float>"
            if "IdE" in name or "<double>" in name:
                return key + "<double>"
            return key
    return name[:60]


def counters(root, counter):
    path = _find(root, "*counter_collection.csv")
    if not path:
        return {}
    per = defaultdict(list)
    for r in _rows(path):
        name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
        if (r.get("Counter_Name") or "") != counter:
            continue
        per[_short(name)].append(float(r.get("Counter_Value") or 0.0))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    root, rnd = sys.argv[1], sys.argv[2]
    stats = _find(os.path.join(root, "trace"), "*kernel_stats.csv")
    if not stats:
        raise SystemExit(f"no kernel_stats.csv under {root}/trace")
    shutil.copy(stats, os.path.join(HERE, f"{rnd}_kernel_stats.csv"))
    fetch = counters(os.path.join(root, "fetch"), "FETCH_SIZE")
    write = counters(os.path.join(root, "write"), "WRITE_SIZE")
    rows = []
    for r in _rows(stats):
        name = _short(r["Name"])
        avg_us = float(r["AverageNs"]) / 1e3
        rows.append((name, int(r["Calls"]), avg_us, float(r.get("Percentage", 0.0)), fetch.get(name), write.get(name)))
    try:
        commit = subprocess.run(["git", "-C", HERE, "rev-parse", "--short", "HEAD"], capture_output=True,
                                text=True).stdout.strip()
    except Exception:
        commit = ""
    bench = {}
    try:
        bench = json.loads(open(os.path.join(root, "trace_bench.json")).read().strip().splitlines()[-1])
    except Exception:
        pass
    lines = [f"# rocprofv3 summary, round {rnd}", "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 20 --warmup 3 "
             "--no-cpu-baseline --train-regions 0 --speedy-steps 8 --reservoir-steps 10` (1 x MI355X), then one `--pmc FETCH_SIZE` and one `--pmc WRITE_SIZE` pass "
             f"of the same command.  Source commit: {commit or 'n/a'}.", "",
             "| kernel | calls | avg us | % time | FETCH_SIZE KiB/launch (raw) | WRITE_SIZE KiB/launch |",
             "|---|---|---|---|---|---|"]
    for name, calls, avg, pct, fk, wk in sorted(rows, key=lambda x: -x[2] * x[1]):
        lines.append(f"| {name} | {calls} | {avg:.2f} | {pct:.1f} | "
                     f"{'' if fk is None else f'{fk:.0f}'} | {'' if wk is None else f'{wk:.0f}'} |")
    if bench:
        lines += ["", "bench line of the traced run (profiled clocks run lower, MI355X_MICROARCH.md "
                      "DVFS item 2):", "", "```", json.dumps(bench), "```"]
    # the dominant readout launch: one-pass (full) by default, the v_ml half with --overlap
    rd = sorted([r for r in rows if r[0].startswith(("k_res_readout_full", "k_res_readout_ml"))],
                key=lambda r: -r[1] * r[2])
    if rd and rd[0][4] is not None and rd[0][5] is not None:
        name, calls, avg, _, fk, wk = rd[0]
        hbm = (2.0 * fk + wk) * 1024.0
        out = {"kernel": name, "round": rnd, "commit": commit, "avg_duration_us_rocprof": avg,
               "fetch_kib_raw": fk, "write_kib": wk, "hbm_bytes_per_launch": hbm,
               "correction": "FETCH_SIZE x2 (gfx950 counts half of 16-B/lane streaming reads)"}
        if bench:
            out["algorithmic_bytes_per_launch"] = bench.get("roofline", {}).get("algorithmic_bytes_per_launch")
        json.dump(out, open(os.path.join(HERE, "readout_pmc.json"), "w"), indent=1)
        lines += ["", f"{name} HBM traffic per launch (2 x FETCH + WRITE): {hbm / 1e9:.3f} GB"]
    # the state update (k_res_update_bal beside the window; k_res_update when not balanced)
    up = sorted([r for r in rows if r[0].startswith(("k_res_update_bal", "k_res_update"))], key=lambda r: -r[1] * r[2])
    if up and up[0][4] is not None and up[0][5] is not None:
        name, calls, avg, _, fk, wk = up[0]
        hbm_raw = (fk + wk) * 1024.0
        hbm_x2 = (2.0 * fk + wk) * 1024.0
        ab = (bench.get("roofline", {}) or {}).get("update_algorithmic_bytes")
        lines += ["", f"{name} HBM traffic per launch: {hbm_raw / 1e6:.1f} MB (FETCH raw + WRITE), "
                      f"{hbm_x2 / 1e6:.1f} MB (FETCH x2 + WRITE)" + (f"; algorithmic {ab / 1e6:.1f} MB" if ab else "")]
    open(os.path.join(HERE, f"{rnd}_summary.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()

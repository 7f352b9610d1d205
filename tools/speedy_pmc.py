"""SPEEDY window counters: the Legendre MFMA utilisation and the f64 VALU work of the
fused step kernels (k_st_gridspec: a latitude row's FFTs, grid-point dynamics and
phypar; k_st_spec: a zonal wavenumber's specy, spectral tail and gridy).

    python tools/speedy_pmc.py run [windows]          # the workload (launched, no graph)
    python tools/speedy_pmc.py summarize DIR ROUND    # -> DIR/speedy_pmc.json (commit as profiles/speedy_pmc.json)

`run` integrates `windows` SPEEDY windows (stepone + 24 leapfrog steps with physics)
launched step by step so every kernel is one dispatch of its own.  Collect with one
counter pass (at most 8 SQ counters, 2 GRBM):

    rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 \
        SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE -d DIR -o pmc --output-format csv -- python3 tools/speedy_pmc.py run

Counter meaning (rocprofv3 --list-avail on gfx950): MfmaFlopsF64 =
SQ_INSTS_VALU_MFMA_MOPS_F64 x 512; MfmaUtil = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE
x SIMDs), but GRBM_GUI_ACTIVE sums the chip's instances, so bench.py takes the
utilisation from the flops and its own phase durations; the SQ_INSTS_VALU_*_F64 counters count wave instructions (x 64 lanes; an FMA
is 2 flops).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_st_gridspec", "k_st_spec", "k_st_inv", "k_state_to_m")


def run(nwin: int) -> None:
    sys.path.insert(0, os.path.join(REPO, "speedy-ml-1_amd"))
    import torch

    from speedy_ml_amd.dynamics import Dynamics
    from speedy_ml_amd.synthetic import dyn_state, phys_boundary

    st, forcing = dyn_state()
    d = Dynamics()
    d.set_forcing(**forcing)
    d.set_state(st)
    d.set_physics(phys_boundary(d, forcing["phis"]))
    d.set_clock(1, True)
    for _ in range(nwin):
        d.window(24, graph=False)
    torch.cuda.synchronize()
    d.close()


def _short(name: str) -> str | None:
    for k in KERNELS:
        if k in name:
            return k
    return None


def summarize(out_dir: str, rnd: str) -> dict:
    rows = []
    for path in glob.glob(os.path.join(out_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(path, newline="") as f:
            rows += list(csv.DictReader(f))
    if not rows:
        raise SystemExit(f"no counter_collection.csv under {out_dir}")
    # one row per (dispatch, counter); values summed over the dimensions rocprofv3 reports
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in rows:
        k = _short(r.get("Kernel_Name", ""))
        if k is None:
            continue
        disp = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[(k, disp)][r["Counter_Name"]] += float(r["Counter_Value"])
        names[k] = r.get("Kernel_Name", k)
    durs = defaultdict(list)
    for path in glob.glob(os.path.join(out_dir, "**", "*kernel_trace.csv"), recursive=True):
        with open(path, newline="") as f:
            for r in csv.DictReader(f):
                k = _short(r.get("Kernel_Name", ""))
                if k:
                    durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"round": rnd, "tool": "tools/speedy_pmc.py", "kernels": {}}
    try:
        out["commit"] = subprocess.run(["git", "-C", REPO, "rev-parse", "--short", "HEAD"], capture_output=True,
                                       text=True).stdout.strip() or None
    except OSError:
        out["commit"] = None
    for k in KERNELS:
        disp = [v for (kk, _), v in per.items() if kk == k]
        if not disp:
            continue
        n = len(disp)
        avg = {c: sum(d.get(c, 0.0) for d in disp) / n for c in disp[0]}
        mfma_flops = avg.get("SQ_INSTS_VALU_MFMA_MOPS_F64", 0.0) * 512
        valu_flops = 64 * (2 * avg.get("SQ_INSTS_VALU_FMA_F64", 0.0) + avg.get("SQ_INSTS_VALU_ADD_F64", 0.0)
                           + avg.get("SQ_INSTS_VALU_MUL_F64", 0.0))
        e = {
            "dispatches": n,
            "avg_duration_us_trace": round(sum(durs[k]) / len(durs[k]), 3) if durs.get(k) else None,
            "counters_per_dispatch": {c: round(v, 1) for c, v in sorted(avg.items())},
            "mfma_f64_flops_per_dispatch": mfma_flops,
            "valu_f64_flops_per_dispatch": valu_flops,
            "valu_f64_trans_insts_per_dispatch": avg.get("SQ_INSTS_VALU_TRANS_F64", 0.0),
        }
        out["kernels"][k] = e
    # written next to the raw output; copy to profiles/speedy_pmc.json to commit it
    path = os.path.join(out_dir, "speedy_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    if len(sys.argv) >= 2 and sys.argv[1] == "run":
        run(int(sys.argv[2]) if len(sys.argv) > 2 else 3)
    elif len(sys.argv) >= 4 and sys.argv[1] == "summarize":
        summarize(sys.argv[2], sys.argv[3])
    else:
        raise SystemExit(__doc__)

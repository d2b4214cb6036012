"""Decompose a run of back-to-back training steps from a rocprofv3 kernel trace (run_kernel_trace.csv): for every
kernel name the median duration, and the median gap from the previous kernel's end to its start, over the dispatches
of the trace (or of the last --last dispatches), plus the median start-to-start period of the first kernel named
--period-kernel (one training step).

    python tools/trace_steps.py gpurun_out/prof/run_kernel_trace.csv [--last 400] [--period-kernel train]
"""
from __future__ import annotations

import argparse
import csv
import json
from collections import defaultdict

import numpy as np


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--period-kernel", default="")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    if args.last:
        ev = ev[-args.last:]
    dur, gap = defaultdict(list), defaultdict(list)
    starts = []
    for i, (s, e, n) in enumerate(ev):
        key = n.split("(")[0][:80]
        dur[key].append((e - s) / 1e3)
        if i:
            gap[key].append((s - ev[i - 1][1]) / 1e3)
        if args.period_kernel and args.period_kernel in n:
            starts.append(s)
    out = {k: {"n": len(v), "median_us": round(float(np.median(v)), 3),
               "median_gap_before_us": round(float(np.median(gap[k])), 3) if gap[k] else None} for k, v in dur.items()}
    res = {"kernels": out}
    if len(starts) > 2:
        res["period_us_median"] = round(float(np.median(np.diff(starts))) / 1e3, 3)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Timed-window breakdown from a rocprofv3 ``--kernel-trace`` CSV of ``bench.py``.

    python tools/boundary_trace.py <trace_kernel_trace.csv> [--steps 20] [--kernel rollout_]

The bench's timed window is its last ``--steps`` rollout launches (plus whatever else was
enqueued between them: the episode-summary reduction at the boundary). Prints every launch in
the window with its duration and the idle gap before it, the window length from the first
launch's start to the last's end, and the model (steps - b) * t_step + b * t_reset that the
verdict asks the bench line to agree with (b = boundary steps in the window).
"""
from __future__ import annotations

import argparse
import csv
import json
import statistics


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def analyse(rows, steps, kernel):
    idx = [i for i, r in enumerate(rows) if kernel in r[2]]
    win = idx[-steps:]
    first, last = win[0], win[-1]
    seq = rows[first:last + 1]
    launches = []
    prev_end = None
    for s, e, name in seq:
        launches.append({"kernel": name[:60], "us": (e - s) / 1e3,
                         "gap_before_us": None if prev_end is None else (s - prev_end) / 1e3})
        prev_end = e
    roll = [(rows[i][1] - rows[i][0]) / 1e3 for i in win]
    med = statistics.median(roll)
    resets = [t for t in roll if t > 1.8 * med]
    plain = [t for t in roll if t <= 1.8 * med]
    window_us = (rows[last][1] - rows[first][0]) / 1e3
    model_us = sum(plain) + sum(resets)
    t_step = statistics.mean(plain)
    t_reset = statistics.mean(resets) if resets else None
    return {"steps": steps, "window_us": window_us, "us_per_step_window": window_us / steps,
            "t_step_us": t_step, "t_reset_us": t_reset, "boundary_steps": len(resets),
            "model_us": model_us, "model_us_per_step": model_us / steps,
            "gaps_us_total": window_us - sum(l["us"] for l in launches),
            "other_kernels_us": sum(l["us"] for l in launches) - sum(roll),
            "launches": launches}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--kernel", default="rollout_")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    r = analyse(load(a.csv), a.steps, a.kernel)
    if a.json:
        print(json.dumps(r, indent=1))
        return
    for l in r["launches"]:
        g = "" if l["gap_before_us"] is None else "%7.2f" % l["gap_before_us"]
        print("%8.2f us  gap %7s  %s" % (l["us"], g, l["kernel"]))
    for k in ("window_us", "us_per_step_window", "t_step_us", "t_reset_us", "boundary_steps", "model_us_per_step",
              "gaps_us_total", "other_kernels_us"):
        print("%-20s %s" % (k, r[k]))


if __name__ == "__main__":
    main()

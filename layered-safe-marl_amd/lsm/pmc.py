"""Reduce rocprofv3 output of a bench run to the numbers the bench line cites.

    python -m lsm.pmc stats  <kernel-trace dir>              -> per-kernel duration summary
    python -m lsm.pmc traffic <fetch dir> <write dir> --config 3 --envs 4096 [--out profiles/pmc_traffic.json]

``traffic`` reads the two separate PMC passes (FETCH_SIZE and WRITE_SIZE do not fit
one TCC pass on gfx950) and applies the gfx950 corrections of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section): FETCH_SIZE is in KiB and
counts half the bytes of wide coalesced reads (x2), WRITE_SIZE is exact for
16-B/lane streaming stores.  Values are per launch of ``rollout_kernel``
(mean over the profiled dispatches, warm-up launches excluded). Each entry records the
``lsm_build_id()`` of the library that was profiled; bench.py quotes an entry only for that build.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import statistics

KERNEL = "lsm::rollout"   # substring of every step-kernel variant (one-wave, team, workgroup)


def _rows(d, suffix):
    files = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    if not files:
        raise FileNotFoundError("no *%s under %s" % (suffix, d))
    for f in files:
        with open(f, newline="") as fh:
            yield from csv.DictReader(fh)


def counter_per_launch(d, counter, kernel=KERNEL, skip=5):
    """Mean over dispatches of `kernel` of the counter summed over its instances."""
    per = {}
    for r in _rows(d, "counter_collection.csv"):
        if kernel not in r.get("Kernel_Name", "") or r.get("Counter_Name") != counter:
            continue
        k = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    vals = [per[k] for k in sorted(per)][skip:]
    if not vals:
        raise ValueError("counter %s not found for %s in %s" % (counter, kernel, d))
    return statistics.fmean(vals), len(vals)


def kernel_stats(d):
    out = []
    for r in _rows(d, "kernel_stats.csv"):
        out.append({"name": r["Name"][:80], "calls": int(r["Calls"]),
                    "avg_us": float(r["AverageNs"]) / 1e3, "pct": float(r["Percentage"])})
    return out


def launch_durations(d, kernel=KERNEL):
    """Per-dispatch durations (us) of `kernel` in dispatch order (kernel_trace.csv)."""
    rows = []
    for r in _rows(d, "kernel_trace.csv"):
        if kernel in r.get("Kernel_Name", ""):
            rows.append((int(r.get("Dispatch_Id") or 0),
                         (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    return [us for _, us in sorted(rows)]


def main():
    ap = argparse.ArgumentParser()
    sub = ap.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("stats")
    s.add_argument("dir")
    ln = sub.add_parser("launches")
    ln.add_argument("dir")
    ln.add_argument("--kernel", default=KERNEL)
    t = sub.add_parser("traffic")
    t.add_argument("fetch_dir")
    t.add_argument("write_dir")
    t.add_argument("--config", type=int, required=True)
    t.add_argument("--envs", type=int, required=True)
    t.add_argument("--out", default=None)
    t.add_argument("--kernel", default=KERNEL)
    t.add_argument("--round", default=None, help="profile tag (e.g. r05) recorded with the entry")
    c = sub.add_parser("counters")
    c.add_argument("dirs", nargs="+")
    c.add_argument("--kernel", default=KERNEL)
    a = ap.parse_args()
    if a.cmd == "counters":
        for d in a.dirs:
            names = sorted({r["Counter_Name"] for r in _rows(d, "counter_collection.csv")})
            for n in names:
                v, k = counter_per_launch(d, n, a.kernel)
                print("%-24s %16.1f  (mean of %d launches)" % (n, v, k))
        return
    if a.cmd == "launches":
        us = launch_durations(a.dir, a.kernel)
        srt = sorted(us)
        q = lambda f: srt[min(len(srt) - 1, int(f * len(srt)))]
        print(json.dumps({"kernel": a.kernel, "launches": len(us), "mean_us": statistics.fmean(us),
                          "p50_us": q(0.5), "p90_us": q(0.9), "max_us": srt[-1],
                          "slowest": [(i, round(v, 2)) for i, v in sorted(enumerate(us), key=lambda x: -x[1])[:4]],
                          # the two launches after each of those (the steps right after an auto-reset)
                          "after_slowest": [[(j, round(us[j], 2)) for j in (i + 1, i + 2) if j < len(us)]
                                            for i, _ in sorted(enumerate(us), key=lambda x: -x[1])[:4]],
                          "note": "the slowest launches are the auto-reset steps (MT19937 scenario replay)"}))
        return
    if a.cmd == "stats":
        for r in kernel_stats(a.dir):
            print("%-80s %6d %10.2f us %6.2f%%" % (r["name"], r["calls"], r["avg_us"], r["pct"]))
        return
    fetch_kib, nf = counter_per_launch(a.fetch_dir, "FETCH_SIZE", a.kernel)
    write_kib, nw = counter_per_launch(a.write_dir, "WRITE_SIZE", a.kernel)
    from . import capi
    bid = capi.load_library().lsm_build_id().decode()
    rec = {"num_envs": a.envs, "kernel": a.kernel, "build_id": bid, "round": a.round,
           "fetch_size_kib_raw": fetch_kib, "write_size_kib": write_kib,
           "fetch_bytes_corrected": 2 * fetch_kib * 1024, "write_bytes": write_kib * 1024,
           "hbm_bytes_per_launch": 2 * fetch_kib * 1024 + write_kib * 1024,
           "dispatches": [nf, nw],
           "correction": "FETCH_SIZE x2 (gfx950, MI355X_MICROARCH.md HBM section); KiB -> bytes"}
    print(json.dumps(rec))
    if a.out:
        db = {}
        if os.path.exists(a.out):
            with open(a.out) as fh:
                db = json.load(fh)
        db["config%d" % a.config] = rec
        with open(a.out, "w") as fh:
            json.dump(db, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()

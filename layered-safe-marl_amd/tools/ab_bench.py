"""A/B timing of kernel variants in one GPU session (boxes differ by a few %, so variants are
only compared within one run). Each variant = a library (LSM_LIB, see lsm.build variant) and
environment settings; the variants are run round-robin `--reps` times.

    python layered-safe-marl_amd/tools/ab_bench.py --config 3 --reps 2 \\
        base: team2:KSEL=team=2 nosplit:LSM_LIB=liblsm_rollout_nosplit.so

A variant is NAME:K=V,K=V (LSM_LIB relative to csrc/; KSEL=field=value;field=value passes
bench.py --kernel-select). Prints one line per variant: the median ms per step and each run's.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")


def parse(v):
    name, _, kv = v.partition(":")
    env = {}
    for item in filter(None, kv.split(",")):
        k, _, val = item.partition("=")
        env[k] = os.path.join(CSRC, val) if k == "LSM_LIB" else val
    ksel = env.pop("KSEL", "").replace(";", ",")
    return name, env, ksel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--allow-old", action="store_true",
                    help="libraries older than the Python side may lack newer entry points (LSM_LIB_AB=1)")
    ap.add_argument("--bench-args", default="", help="extra bench.py arguments (e.g. '--steps 20')")
    a = ap.parse_args()
    vs = [parse(v) for v in a.variants]
    res = {n: [] for n, _, _ in vs}
    for _ in range(a.reps):
        for name, extra, ksel in vs:
            env = dict(os.environ, **extra)
            if a.allow_old:
                env["LSM_LIB_AB"] = "1"
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", str(a.config), "--steps",
                   str(a.steps), "--warmup", str(a.warmup), "--no-cpu-baseline"] + a.bench_args.split()
            if ksel:
                cmd += ["--kernel-select", ksel]
            out = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(name, "FAILED", out.stderr[-2000:], flush=True)
                sys.exit(1)
            d = json.loads(out.stdout.strip().splitlines()[-1])
            res[name].append(d["ms_per_step"] * 1e3)
            print("%-12s %8.2f us  (%s)" % (name, res[name][-1], d["roofline"]["kernel"]), flush=True)
    print("---- config %d, median us/step over %d reps" % (a.config, a.reps))
    for name, _, _ in vs:
        print("%-12s %8.2f   %s" % (name, statistics.median(res[name]), " ".join("%.2f" % x for x in res[name])))


if __name__ == "__main__":
    main()

"""Build the oracle's C restatements (TEST INFRASTRUCTURE): oracle/csrc/*.c -> oracle/liboracle_ref.so.

gcc with -ffp-contract=off, so only the fma() calls the restatement writes out are fused. The .so
is git-ignored and travels to the GPU box with the tree (it is only loaded by tests, smoke() and
bench.py's cpu_baseline leg)."""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
SRCS = [os.path.join(HERE, "csrc", "rk45_ref.c")]
OUT = os.path.join(HERE, "liboracle_ref.so")


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and os.path.exists(OUT) and all(os.path.getmtime(s) <= os.path.getmtime(OUT) for s in SRCS):
        return OUT
    cmd = ["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC", "-o", OUT + ".tmp"] + SRCS + ["-lm"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force=True)

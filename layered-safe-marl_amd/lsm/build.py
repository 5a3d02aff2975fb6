"""Build ``liblsm_rollout.so`` in-tree with hipcc for gfx950 (no JIT cache, no CMake).

``python -m lsm.build`` (from ``layered-safe-marl_amd/``) or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
SRC = os.path.join(CSRC, "lsm_rollout.hip")
OUT = os.path.join(CSRC, "liblsm_rollout.so")
DEPS = [SRC, os.path.join(CSRC, "lsm_numeric.h"), os.path.join(CSRC, "lsm_scenario.h"),
        os.path.join(CSRC, "lsm_block.h"),
        os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "lsm_rollout.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
         # reproduce numpy's float64 expression order exactly; explicit fma() only where
         # OpenBLAS fuses (lsm_numeric.h)
         "-ffp-contract=off", "-Wno-unused-result"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(d) > t for d in DEPS if os.path.exists(d))


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)

"""Build ``liblsm_rollout.so`` in-tree with hipcc for gfx950 (no JIT cache, no CMake).

``python -m lsm.build`` (from ``layered-safe-marl_amd/``) or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
SRC = os.path.join(CSRC, "lsm_rollout.hip")   # the rollout TU (diagnostic builds recompile it alone)
OUT = os.path.join(CSRC, "liblsm_rollout.so")
HDR = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "lsm_rollout.h")
# translation units -> their dependencies (each compiled to its own object, then linked)
UNITS = {
    "lsm_rollout.hip": ["lsm_numeric.h", "lsm_scenario.h", "lsm_block.h", "lsm_rk45.h", "lsm_pow_tables.h", "lsm_team.h"],
    "lsm_edges.hip": [],
    "lsm_buffer.hip": [],
    "lsm_metrics.hip": [],
}

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # reproduce numpy's float64 expression order exactly; explicit fma() only where
         # OpenBLAS fuses (lsm_numeric.h)
         "-ffp-contract=off", "-Wno-unused-result"]


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _obj(unit: str) -> str:
    return os.path.join(CSRC, unit.rsplit(".", 1)[0] + ".o")


def needs_build() -> bool:
    objs = [_obj(u) for u in UNITS]
    return _stale(OUT, objs) or any(
        _stale(_obj(u), [os.path.join(CSRC, u), HDR] + [os.path.join(CSRC, d) for d in deps])
        for u, deps in UNITS.items())


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    objs = []
    for u, deps in UNITS.items():
        o = _obj(u)
        objs.append(o)
        if force or _stale(o, [os.path.join(CSRC, u), HDR] + [os.path.join(CSRC, d) for d in deps]):
            cmd = [HIPCC] + FLAGS + ["-c", "-o", o + ".tmp", u]
            if verbose:
                print(" ".join(cmd), flush=True)
            subprocess.check_call(cmd, cwd=CSRC)
            os.replace(o + ".tmp", o)
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_variant(name: str, defines, verbose: bool = True) -> str:
    """A/B experiments: the rollout TU rebuilt with extra -D flags and linked with the product's
    other objects into csrc/liblsm_rollout_<name>.so (select it with LSM_LIB=...). Never the
    product library."""
    build(verbose=verbose)
    out = os.path.join(CSRC, "liblsm_rollout_%s.so" % name)
    obj = out[:-3] + ".o"
    cmd = [HIPCC] + FLAGS + ["-D%s" % d for d in defines] + ["-c", "-o", obj, "lsm_rollout.hip"]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    objs = [obj] + [_obj(u) for u in UNITS if u != "lsm_rollout.hip"]
    subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, cwd=CSRC)
    os.remove(obj)
    return out


def build_variants(specs, verbose: bool = True):
    """Several A/B variants at once: the product library and each variant's rollout object
    compile in parallel (one hipcc process each), then each variant links. specs: NAME:D1,D2."""
    import threading
    t = threading.Thread(target=build, kwargs={"verbose": verbose})
    t.start()
    procs = []
    for spec in specs:
        name, _, defs = spec.partition(":")
        obj = os.path.join(CSRC, "liblsm_rollout_%s.o" % name)
        cmd = [HIPCC] + FLAGS + ["-D%s" % d for d in filter(None, defs.split(","))] + ["-c", "-o", obj, "lsm_rollout.hip"]
        if verbose:
            print(" ".join(cmd), flush=True)
        procs.append((name, obj, subprocess.Popen(cmd, cwd=CSRC, stderr=subprocess.DEVNULL)))
    t.join()
    for name, obj, pr in procs:
        if pr.wait() != 0:
            raise RuntimeError("variant %s failed to compile" % name)
        out = os.path.join(CSRC, "liblsm_rollout_%s.so" % name)
        objs = [obj] + [_obj(u) for u in UNITS if u != "lsm_rollout.hip"]
        subprocess.check_call([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs, cwd=CSRC)
        os.remove(obj)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        # python -m lsm.build variant NAME DEF1 [DEF2 ...]
        build_variant(sys.argv[2], sys.argv[3:])
    elif len(sys.argv) > 2 and sys.argv[1] == "variants":
        # python -m lsm.build variants NAME:DEF1,DEF2 NAME2:DEF3 ...
        build_variants(sys.argv[2:])
    else:
        build(force="--force" in sys.argv)

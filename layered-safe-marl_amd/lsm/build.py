"""Build ``liblsm_rollout.so`` in-tree with hipcc for gfx950 (no JIT cache, no CMake).

``python -m lsm.build`` (from ``layered-safe-marl_amd/``) or ``__graft_entry__.build()``.

The rollout translation unit instantiates ~25 kernels; it is compiled as ``ROLLOUT_PARTS``
objects in parallel (``-DLSM_PART=0`` the host code, ``-DLSM_PART=g`` kernel group g, see the
group table in ``csrc/lsm_rollout.hip``) and linked with the other units.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
SRC = os.path.join(CSRC, "lsm_rollout.hip")   # the rollout TU
OUT = os.path.join(CSRC, "liblsm_rollout.so")
HDR = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "lsm_rollout.h")
ROLLOUT_DEPS = ["lsm_numeric.h", "lsm_scenario.h", "lsm_block.h", "lsm_rk45.h", "lsm_pow_tables.h", "lsm_team.h"]
ROLLOUT_PARTS = 9
# the other translation units -> their dependencies (each compiled to its own object, then linked)
UNITS = {
    "lsm_edges.hip": [],
    "lsm_buffer.hip": [],
    "lsm_metrics.hip": [],
}

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
         # reproduce numpy's float64 expression order exactly; explicit fma() only where
         # OpenBLAS fuses (lsm_numeric.h)
         "-ffp-contract=off", "-Wno-unused-result", "-Wno-unused-function"]
# Variant / diagnostic builds define this; csrc/lsm_rollout.hip refuses its diagnostic switches
# (LSM_XP_*: bounds with wrong results, LSM_STAMPS) without it, so the product build cannot get one.
DIAG_DEFINE = "LSM_DIAGNOSTIC_BUILD"


def _stale(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _obj(unit: str) -> str:
    return os.path.join(CSRC, unit.rsplit(".", 1)[0] + ".o")


def _part_obj(part: int, tag: str = "") -> str:
    return os.path.join(CSRC, "lsm_rollout%s_p%d.o" % (tag, part))


def _rollout_deps():
    return [SRC, HDR] + [os.path.join(CSRC, d) for d in ROLLOUT_DEPS]


def _run_parallel(jobs, verbose=True):
    """jobs: [(cmd, out)] -- each compiles into out + '.tmp', renamed on success."""
    limit = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4))))
    pending = list(jobs)
    running = []
    failed = []
    while pending or running:
        while pending and len(running) < limit:
            cmd, out = pending.pop(0)
            if verbose:
                print(" ".join(cmd), flush=True)
            running.append((subprocess.Popen(cmd, cwd=CSRC), out))
        p, out = running.pop(0)
        if p.wait() != 0:
            failed.append(out)
        elif os.path.exists(out + ".tmp"):
            os.replace(out + ".tmp", out)
    if failed:
        raise RuntimeError("compile failed: %s" % ", ".join(os.path.basename(f) for f in failed))


def build_id(defines=()) -> str:
    """sha256 of the step kernel's sources, the header, the compiler flags and the variant's -D
    flags (16 hex digits): lsm_build_id() of the library built from them."""
    import hashlib
    h = hashlib.sha256()
    for f in _rollout_deps():
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    h.update(" ".join(FLAGS + sorted(defines)).encode())
    return h.hexdigest()[:16]


def _rollout_jobs(defines=(), tag="", force=True, parts=None):
    jobs = []
    bid = build_id(defines)
    for part in (range(ROLLOUT_PARTS) if parts is None else parts):
        o = _part_obj(part, tag)
        if force or _stale(o, _rollout_deps()):
            cmd = [HIPCC] + FLAGS + ["-D%s" % d for d in defines] + ['-DLSM_BUILD_ID="%s"' % bid] + \
                ["-DLSM_PART=%d" % part, "-c", "-o", o + ".tmp", "lsm_rollout.hip"]
            jobs.append((cmd, o))
    return jobs


def needs_build() -> bool:
    objs = [_obj(u) for u in UNITS] + [_part_obj(p) for p in range(ROLLOUT_PARTS)]
    return _stale(OUT, objs) or any(_stale(_part_obj(p), _rollout_deps()) for p in range(ROLLOUT_PARTS)) or any(
        _stale(_obj(u), [os.path.join(CSRC, u), HDR] + [os.path.join(CSRC, d) for d in deps])
        for u, deps in UNITS.items())


def _link(objs, out, verbose=True):
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out + ".tmp"] + objs
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd, cwd=CSRC)
    os.replace(out + ".tmp", out)


def build(force: bool = False, verbose: bool = True) -> str:
    if not force and not needs_build():
        return OUT
    jobs = _rollout_jobs(force=force)
    for u, deps in UNITS.items():
        o = _obj(u)
        if force or _stale(o, [os.path.join(CSRC, u), HDR] + [os.path.join(CSRC, d) for d in deps]):
            jobs.append(([HIPCC] + FLAGS + ["-c", "-o", o + ".tmp", u], o))
    _run_parallel(jobs, verbose)
    _link([_part_obj(p) for p in range(ROLLOUT_PARTS)] + [_obj(u) for u in UNITS], OUT, verbose)
    return OUT


def variant_path(name: str) -> str:
    return os.path.join(CSRC, "liblsm_rollout_%s.so" % name)


def build_variants(specs, verbose: bool = True):
    """A/B experiments and diagnostic builds: the rollout TU rebuilt with extra -D flags and linked
    with the product's other objects into csrc/liblsm_rollout_<name>.so (select it with LSM_LIB=...).
    Never the product library. specs: ["NAME:D1,D2", ...], or "NAME:D1,D2@3,4" to recompile only
    those kernel groups (the others are the product's objects: for defines that only touch those
    groups' kernels); all recompiled parts of all variants compile in parallel."""
    build(verbose=verbose)
    jobs, variants = [], []
    for spec in specs:
        name, _, rest = spec.partition(":")
        defs, _, only = rest.partition("@")
        defines = [d for d in defs.split(",") if d] + [DIAG_DEFINE]
        parts = sorted({int(x) for x in only.split(",") if x}) if only else list(range(ROLLOUT_PARTS))
        jobs += _rollout_jobs(defines, tag="_" + name, parts=parts)
        variants.append((name, parts))
    _run_parallel(jobs, verbose)
    for name, parts in variants:
        objs = [_part_obj(p, "_" + name) if p in parts else _part_obj(p) for p in range(ROLLOUT_PARTS)]
        _link(objs + [_obj(u) for u in UNITS], variant_path(name), verbose)
        for p in parts:
            os.remove(_part_obj(p, "_" + name))
    return [variant_path(n) for n, _ in variants]


def build_variant(name: str, defines, verbose: bool = True) -> str:
    return build_variants(["%s:%s" % (name, ",".join(defines))], verbose)[0]


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "variant":
        # python -m lsm.build variant NAME DEF1 [DEF2 ...]
        build_variant(sys.argv[2], sys.argv[3:])
    elif len(sys.argv) > 2 and sys.argv[1] == "variants":
        # python -m lsm.build variants NAME:DEF1,DEF2 NAME2:DEF3 ...
        build_variants(sys.argv[2:])
    else:
        build(force="--force" in sys.argv)

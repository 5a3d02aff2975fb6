"""Import and drive the *reference itself* in this container (TEST INFRASTRUCTURE ONLY).

Used only by ``tests/golden/make_golden.py`` to record golden vectors. It needs
``/root/reference`` (absent on the GPU box) and never runs there.

Recipe: put ``oracle/ref_stubs`` first on ``sys.path`` so the
absent third-party packages (gym, pyglet, absl, jax, hj_reachability,
hj_reachability_utils, cvxpy, casadi) resolve to local stubs, disable bytecode
writing (``/root/reference`` must stay untouched), and run from a scratch working
directory holding the ``data/*.pkl`` files the reference opens by relative path
(``multiagent/config.py:29-30,62``) -- written here from synthetic tables.
"""
from __future__ import annotations

import argparse
import os
import pickle
import sys

import numpy as np

REF_ROOT = "/root/reference"
_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
_STUBS = os.path.join(_HERE, "ref_stubs")


def reference_available() -> bool:
    return os.path.isdir(os.path.join(REF_ROOT, "multiagent"))


def _install_paths():
    sys.dont_write_bytecode = True
    for p in (REF_ROOT, _REPO, _STUBS):
        if p in sys.path:
            sys.path.remove(p)
    sys.path.insert(0, REF_ROOT)
    sys.path.insert(0, _REPO)
    sys.path.insert(0, _STUBS)


def write_data_files(workdir: str, di_table=None, at_table=None, ttr_table=None):
    """Pickle synthetic HJ / TTR tables where the reference expects them."""
    _install_paths()
    from hj_reachability_utils.common import GridMetaData, HjValueData, TtrData
    os.makedirs(os.path.join(workdir, "data"), exist_ok=True)

    def dump(name, obj):
        with open(os.path.join(workdir, "data", name), "wb") as f:
            pickle.dump(obj, f)

    if di_table is not None:
        g = di_table
        dump("crazyflies_value_function.pkl",
             HjValueData(g["values"], GridMetaData(g["lo"], g["hi"], g["shape"], g["periodic"]),
                         g["separation_distance"]))
    if at_table is not None:
        g = at_table
        dump("airtaxi_value_function.pkl",
             HjValueData(g["values"], GridMetaData(g["lo"], g["hi"], g["shape"], g["periodic"]),
                         g["separation_distance"]))
    if ttr_table is not None:
        g = ttr_table
        dump("airtaxi_ttr_function.pkl",
             TtrData(g["values"], GridMetaData(g["lo"], g["hi"], g["shape"], g["periodic"]),
                     g["ttr_max"]))


def default_args(**over) -> argparse.Namespace:
    """The env-side argparse fields ``make_world`` reads (train.sh + onpolicy/config.py)."""
    a = dict(
        scenario_name="navigation_graph_safe", num_agents=3, num_landmarks=2,
        num_obstacles=0, num_walls=0, num_scripted_agents=0, collaborative=False,
        use_dones=False, episode_length=250, num_env_steps=250 * 4, n_rollout_threads=1,
        dynamics_type="double_integrator", world_size=4, graph_feat_type="relative",
        use_safety_filter=False, num_internal_step=1, use_masking=True,
        discrete_action=True, zeroshift=0, seed=0, algorithm_name="rmappo",
    )
    a.update(over)
    return argparse.Namespace(**a)


def make_reference_env(args: argparse.Namespace, workdir: str, seed: int):
    """``GraphMPEEnv(args)`` + ``env.seed(seed)`` exactly as scripts/train_mpe.py:23-45."""
    _install_paths()
    old = os.getcwd()
    os.chdir(workdir)
    try:
        from multiagent.MPE_env import GraphMPEEnv
        env = GraphMPEEnv(args)
        env.seed(seed)
    finally:
        os.chdir(old)
    return env


def run_in(workdir, fn, *a, **k):
    old = os.getcwd()
    os.chdir(workdir)
    try:
        return fn(*a, **k)
    finally:
        os.chdir(old)


def one_hot_actions(idx: np.ndarray, n_act: int = 25):
    """Runner-style one-hot actions (graph_mpe_runner.py:432-433)."""
    idx = np.asarray(idx)
    out = np.zeros(idx.shape + (n_act,), dtype=np.float64)
    np.put_along_axis(out, idx[..., None], 1.0, axis=-1)
    return out

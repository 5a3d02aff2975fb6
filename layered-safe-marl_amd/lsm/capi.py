"""ctypes binding of the C ABI in ``include/lsm_rollout.h`` (``liblsm_rollout.so``).

This is the Python stub a maintainer of the reference would add (see
INTEGRATION.md): plain pointers and sizes only, no torch types cross the ABI.
The library is built in-tree by ``lsm.build`` (``hipcc --offload-arch=gfx950``);
if it is missing the import fails loudly -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSM_LIB") or os.path.join(os.path.dirname(_HERE), "csrc", "liblsm_rollout.so")

LSM_DOUBLE_INTEGRATOR, LSM_AIRTAXI = 0, 1
LSM_ACTIONS_INDEX_I32, LSM_ACTIONS_ONEHOT_F32, LSM_ACTIONS_ONEHOT_F64 = 0, 1, 2
(OUT_OBS, OUT_NODE_OBS, OUT_ADJ, OUT_REWARD, OUT_DONE, OUT_RESET_FLAG, OUT_EP_INFO, OUT_INFO,
 OUT_EDGES, OUT_STATE, OUT_DEBUG_STAMPS, OUT_ADJ_MASK, OUT_SHARE_OBS, OUT_MASKS, OUT_ACTIVE_MASKS,
 OUT_COLLISION_FORCE, OUT_DEPARTED, OUT_ADJ_NNZ) = range(18)
NUM_OUT = 18
LSM_SCENARIO_TRAIN, LSM_SCENARIO_LAYOUT, LSM_SCENARIO_DEPARTURES = 0, 1, 2
LSM_RNG_MT19937, LSM_RNG_PHILOX = 0, 1
ADJ_REFERENCE, ADJ_COMPACT = 0, 1
# lsm_config.reward_terms bits: RewardBinaryConfig's optional reward terms (multiagent/config.py:78-83)
REWARD_BITS = {"safety_violation": 1, "potential_conflict": 2, "diff_from_filtered_action": 4, "hj_value": 8}
INFO_FIELDS = ("individual_reward", "min_relative_distance", "Dist_to_goal", "Time_req_to_goal",
               "Num_agent_collisions", "Distance_mean", "Distance_variance", "Dists_traveled",
               "Time_mean", "Time_stddev", "Min_time_to_goal", "Safety filtered", "Safety violated",
               "deconflicting_agent_index", "action_diff", "reached_goal", "position_x", "position_y")

# Every symbol include/lsm_rollout.h declares (checked by tests/test_capi.py).
EXPORTED = ("lsm_create", "lsm_destroy", "lsm_last_error", "lsm_set_value_table", "lsm_set_ttr_table",
            "lsm_bind_output", "lsm_output_bytes", "lsm_reset", "lsm_step", "lsm_num_entities",
            "lsm_node_features", "lsm_obs_dim", "lsm_host_mt_uniforms", "lsm_host_scenario",
            "lsm_set_agent_state", "lsm_edges_workspace_bytes", "lsm_edges_count", "lsm_edges_emit", "lsm_edges_emit_dev",
            "lsm_edges_last_error", "lsm_bind_output_ring", "lsm_select_ring", "lsm_buffer_insert",
            "lsm_buffer_last_error", "lsm_host_rk45_di", "lsm_host_glibc_pow", "lsm_action_errors",
            "lsm_kernel_name", "lsm_reset_layout", "lsm_layout_doubles", "lsm_host_philox_uniforms",
            "lsm_host_philox4x32", "lsm_episode_summary", "lsm_build_id", "lsm_test_set_mt_stage",
            "lsm_create_select", "lsm_edges_scan_emit")


class LsmConfig(C.Structure):
    _fields_ = [("dynamics", C.c_int32), ("num_envs", C.c_int32), ("num_agents", C.c_int32),
                ("num_landmarks", C.c_int32), ("episode_length", C.c_int32),
                ("use_safety_filter", C.c_int32), ("use_masking", C.c_int32),
                ("auto_reset", C.c_int32), ("emit_edges", C.c_int32), ("adj_layout", C.c_int32),
                ("world_size", C.c_double), ("seed", C.c_int64), ("env_offset", C.c_int64),
                ("collision_forces", C.c_int32), ("scenario", C.c_int32), ("rng", C.c_int32),
                ("num_internal_step", C.c_int32), ("reward_terms", C.c_int32), ("collaborative", C.c_int32)]


class LsmKernelSelect(C.Structure):
    """lsm_kernel_select: kernel choice for parity tests and A/B runs (the library reads no
    environment variables). ``kernel_select(**overrides)`` fills the defaults."""
    _fields_ = [(n, C.c_int32) for n in ("workgroup_per_env", "lanes_per_env", "team", "generic", "lean",
                                         "filter_search", "bounds_shift")]


KERNEL_SELECT_DEFAULTS = dict(workgroup_per_env=0, lanes_per_env=0, team=-1, generic=0, lean=-1, filter_search=-1,
                              bounds_shift=0)


def kernel_select(**overrides) -> LsmKernelSelect:
    bad = set(overrides) - set(KERNEL_SELECT_DEFAULTS)
    if bad:
        raise ValueError("unknown kernel_select fields: %s" % sorted(bad))
    return LsmKernelSelect(**dict(KERNEL_SELECT_DEFAULTS, **overrides))


class LsmCurriculum(C.Structure):
    _fields_ = [(n, C.c_double) for n in (
        "curriculum_ratio", "sloped", "stair", "ratio_airtaxi", "ratio_scenario",
        "goal_heading_error_thresh", "goal_speed_error_thresh", "min_dist_thresh",
        "separation_distance", "engagement_distance", "world_use_safety_filter", "stair_is_int")]


class LsmError(RuntimeError):
    pass


_lib = None


def load_library(path: str = LIB_PATH):
    """Load liblsm_rollout.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise LsmError("liblsm_rollout.so not built (%s); run __graft_entry__.build() or "
                       "python -m lsm.build -- there is no CPU fallback" % path)
    lib = C.CDLL(path)
    P, I32, I64, U32, D, SZ = C.c_void_p, C.c_int32, C.c_int64, C.c_uint32, C.c_double, C.c_size_t
    sig = {
        "lsm_create": (I32, [C.POINTER(LsmConfig), C.POINTER(P)]),
        "lsm_create_select": (I32, [C.POINTER(LsmConfig), C.POINTER(LsmKernelSelect), C.POINTER(P)]),
        "lsm_destroy": (None, [P]),
        "lsm_last_error": (C.c_char_p, [P]),
        "lsm_set_value_table": (I32, [P, I32, P, P, P, P, P, P, D]),
        "lsm_set_ttr_table": (I32, [P, I32, P, P, P, P, P, D]),
        "lsm_bind_output": (I32, [P, I32, P, SZ]),
        "lsm_output_bytes": (SZ, [P, I32]),
        "lsm_reset": (I32, [P, C.POINTER(LsmCurriculum), P]),
        "lsm_step": (I32, [P, P, I32, C.POINTER(LsmCurriculum), P]),
        "lsm_num_entities": (I32, [P]),
        "lsm_node_features": (I32, [P]),
        "lsm_obs_dim": (I32, [P]),
        "lsm_host_mt_uniforms": (I32, [U32, I32, D, D, P]),
        "lsm_host_scenario": (I32, [C.POINTER(LsmConfig), C.POINTER(LsmCurriculum), U32, P, P]),
        "lsm_set_agent_state": (I32, [P, I32, P, P, P]),
        "lsm_edges_workspace_bytes": (SZ, [I64]),
        "lsm_edges_count": (I32, [P, P, I64, I32, I32, P, P, SZ, P]),
        "lsm_edges_emit": (I32, [P, P, I64, I32, I32, P, I64, P, P, P]),
        "lsm_edges_emit_dev": (I32, [P, P, I64, I32, I32, P, I64, P, P, P]),
        "lsm_edges_scan_emit": (I32, [P, P, I64, I32, I32, P, P, P, SZ, I64, P, P, P, P]),
        "lsm_edges_last_error": (C.c_char_p, []),
        "lsm_bind_output_ring": (I32, [P, I32, P, SZ, I32, I32]),
        "lsm_select_ring": (I32, [P, I32]),
        "lsm_buffer_insert": (I32, [P, P, I32, I32, I32, I32, P, P, P, P, P, P]),
        "lsm_buffer_last_error": (C.c_char_p, []),
        "lsm_host_rk45_di": (I32, [P, D, D, D, P]),
        "lsm_host_glibc_pow": (D, [D, D]),
        "lsm_action_errors": (I32, [P, P]),
        "lsm_kernel_name": (C.c_char_p, [P]),
        "lsm_reset_layout": (I32, [P, C.POINTER(LsmCurriculum), P, P]),
        "lsm_layout_doubles": (I32, [P]),
        "lsm_host_philox_uniforms": (I32, [U32, U32, I32, D, D, P]),
        "lsm_host_philox4x32": (I32, [P, P, P]),
        "lsm_episode_summary": (I32, [P, I32, P, P]),
        "lsm_build_id": (C.c_char_p, []),
        "lsm_test_set_mt_stage": (I32, [P, I32]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name, None)
        if fn is None and os.environ.get("LSM_LIB_AB") == "1":
            continue   # tools/ab_bench.py --allow-old: an older library may lack a newer entry point
        if fn is None:
            raise AttributeError("%s: missing symbol %s" % (path, name))
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, handle=None):
    if rc != 0:
        lib = load_library()
        msg = lib.lsm_last_error(handle).decode() if handle else "lsm call failed"
        raise LsmError(msg)

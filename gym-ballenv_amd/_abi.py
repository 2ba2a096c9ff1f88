"""ctypes mirror of include/ballenv.h and the loader for libballenv.so.

The shared library is built in-tree (``__graft_entry__.build()`` or
``python -m gym_ballenv_amd.build``).  There is no fallback: if the library is
missing or was built for another ABI version, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os

ABI_VERSION = 7
MAX_STATIC, MAX_DYNAMIC, MAX_GOALS, MAX_ACTIONS, MAX_WINDOW = 64, 32, 16, 16, 64

BE_OK, BE_E_INVALID, BE_E_HIP, BE_E_NOMEM, BE_E_DEVICE = 0, -1, -2, -3, -4
STATUS_BITS = {1: "reset tape exhausted", 2: "reset rejection limit", 4: "action index out of range",
               8: "dynamic obstacle left the int16 coordinate range",
               16: "goal change with no other goal (the reference raises ValueError)"}

LIB_NAME = "libballenv.so"
LIB_PATH = os.environ.get("BALLENV_LIB") or os.path.join(os.path.dirname(os.path.realpath(__file__)), LIB_NAME)
# BALLENV_LIB: load a diagnostics build (tools/) instead of the in-tree libballenv.so

# Names declared in include/ballenv.h (checked by tests/test_abi.py).
EXPORTS = ("be_abi_version", "be_config_default", "be_config_check", "be_step_bytes", "be_stats_slots",
           "be_last_error", "be_kernel_name",
           "be_create", "be_destroy", "be_reset", "be_step", "be_step_n", "be_rollout", "be_observe", "be_sample_actions",
           "be_status", "be_state_blob_bytes", "be_save_state", "be_load_state",
           "be_pool_fill", "be_pool_invalidate", "be_pool_set_period", "be_pool_period", "be_pool_bytes", "be_pool_entry", "be_policy_create", "be_policy_destroy", "be_policy_load", "be_policy_act",
           "be_policy_rollout", "be_policy_bytes", "be_observe_blocks",
           "be_board_config_default", "be_board_create", "be_board_destroy", "be_board_last_error",
           "be_board_reset", "be_board_step", "be_board_rollout", "be_board_observe", "be_board_status",
           "be_board_pool_bytes")
BOARD_MAX_STATIC, BOARD_MAX_ACTIONS, BOARD_FEATURES = 32, 16, 20


class BeConfig(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("window", C.c_int32), ("env_offset", C.c_int64), ("seed", C.c_uint64),
        ("screen_width", C.c_int32), ("screen_height", C.c_int32),
        ("strip_obs_x", C.c_int32), ("strip_obs_y", C.c_int32),
        ("strip_goal_x", C.c_int32), ("strip_goal_y", C.c_int32),
        ("strip_agent_x", C.c_int32), ("strip_agent_y", C.c_int32),
        ("radius_obstacle", C.c_int32), ("radius_agent", C.c_int32),
        ("speed_x", C.c_int32), ("speed_y", C.c_int32),
        ("threshold_goal", C.c_double), ("time_penalty", C.c_double), ("min_spawn_dist", C.c_double),
        ("num_static", C.c_int32), ("num_dynamic", C.c_int32),
        ("static_penalty", C.c_double), ("dynamic_penalty", C.c_double),
        ("goal_change_step", C.c_int32), ("obs_certainty", C.c_int32), ("num_goals", C.c_int32),
        ("goals", (C.c_int32 * 2) * MAX_GOALS), ("obstacle_speed", C.c_int32 * MAX_DYNAMIC),
        ("num_actions", C.c_int32), ("actions", (C.c_int32 * 2) * MAX_ACTIONS),
        ("time_limit", C.c_int32), ("autoreset", C.c_int32),
    ]


class BeState(C.Structure):
    _fields_ = [("agent", C.c_void_p), ("goal", C.c_void_p), ("prev_dist", C.c_void_p),
                ("total_dist", C.c_void_p), ("ep_return", C.c_void_p), ("ep_len", C.c_void_p), ("episode", C.c_void_p),
                ("static_obs", C.c_void_p), ("dyn_obs", C.c_void_p), ("dyn_goal", C.c_void_p)]


class BeOut(C.Structure):
    _fields_ = [("obs", C.c_void_p), ("obs_f32", C.c_void_p), ("reward", C.c_void_p), ("done", C.c_void_p),
                ("truncated", C.c_void_p), ("terminal_obs", C.c_void_p), ("final_return", C.c_void_p),
                ("final_len", C.c_void_p), ("stats", C.c_void_p)]


class BeActOut(C.Structure):
    _fields_ = [("action", C.c_void_p), ("log_prob", C.c_void_p), ("value", C.c_void_p), ("probs", C.c_void_p)]


class BeBoardConfig(C.Structure):
    _fields_ = [
        ("num_envs", C.c_int32), ("num_static", C.c_int32), ("env_offset", C.c_int64), ("seed", C.c_uint64),
        ("screen_width", C.c_int32), ("screen_height", C.c_int32),
        ("strip_obs_x", C.c_int32), ("strip_obs_y", C.c_int32),
        ("strip_goal_x", C.c_int32), ("strip_goal_y", C.c_int32),
        ("strip_agent_x", C.c_int32), ("strip_agent_y", C.c_int32),
        ("agent_radius", C.c_double), ("static_radius", C.c_double), ("obstacle_feature_radius", C.c_double),
        ("goal_threshold", C.c_double), ("min_spawn_dist", C.c_double),
        ("spawn_thresh_agent", C.c_double), ("spawn_thresh_goal", C.c_double),
        ("num_actions", C.c_int32), ("actions", (C.c_double * 2) * 16),
        ("time_limit", C.c_int32), ("autoreset", C.c_int32),
    ]


class BeBoardState(C.Structure):
    _fields_ = [("agent", C.c_void_p), ("goal", C.c_void_p), ("dist", C.c_void_p), ("total_dist", C.c_void_p),
                ("ep_return", C.c_void_p), ("ep_len", C.c_void_p), ("episode", C.c_void_p),
                ("static_obs", C.c_void_p)]


class BeBoardOut(C.Structure):
    _fields_ = [("features", C.c_void_p), ("reward", C.c_void_p), ("done", C.c_void_p), ("truncated", C.c_void_p)]


class BallEnvError(RuntimeError):
    pass


_lib = None


def lib() -> C.CDLL:
    """Load libballenv.so (raises if it is absent: there is no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise BallEnvError(f"{LIB_PATH} not found: build it with __graft_entry__.build() "
                           "or `python -m gym_ballenv_amd.build` (no CPU fallback exists)")
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    P = C.POINTER
    sig = {
        "be_abi_version": (C.c_int, []),
        "be_config_default": (C.c_int, [P(BeConfig), i32, i32]),
        "be_config_check": (C.c_int, [P(BeConfig), C.c_char_p, i32]),
        "be_step_bytes": (i64, [P(BeConfig)]),
        "be_stats_slots": (i64, [P(BeConfig)]),
        "be_last_error": (C.c_char_p, [vp]),
        "be_kernel_name": (C.c_char_p, [vp, i32]),
        "be_create": (C.c_int, [P(BeConfig), i32, P(vp)]),
        "be_destroy": (C.c_int, [vp]),
        "be_reset": (C.c_int, [vp, P(BeState), vp, vp, i32, P(BeOut), vp]),
        "be_step": (C.c_int, [vp, P(BeState), vp, vp, vp, P(BeOut), vp]),
        "be_rollout": (C.c_int, [vp, P(BeState), vp, C.c_int32, P(BeOut), vp]),
        "be_step_n": (C.c_int, [vp, P(BeState), vp, C.c_int32, P(BeOut), vp]),
        "be_observe": (C.c_int, [vp, P(BeState), P(BeOut), vp]),
        "be_sample_actions": (C.c_int, [vp, vp, i32, u64, vp]),
        "be_status": (C.c_int, [vp, P(i32), vp]),
        "be_state_blob_bytes": (i64, [P(BeConfig)]),
        "be_save_state": (C.c_int, [vp, P(BeState), vp, vp]),
        "be_load_state": (C.c_int, [vp, P(BeState), vp, vp]),
        "be_pool_fill": (C.c_int, [vp, P(BeState), vp]),
        "be_pool_invalidate": (C.c_int, [vp, vp]),
        "be_pool_set_period": (C.c_int, [vp, i32]),
        "be_pool_bytes": (i64, [vp]),
        "be_pool_period": (i32, [vp]),
        "be_pool_entry": (C.c_int, [vp, i32, i32, P(C.c_uint32), P(C.c_double), i32]),
        "be_policy_create": (C.c_int, [vp, i32, i32, P(vp)]),
        "be_policy_destroy": (C.c_int, [vp]),
        "be_policy_load": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, vp]),
        "be_policy_act": (C.c_int, [vp, P(BeState), vp, P(BeActOut), u64, vp]),
        "be_policy_rollout": (C.c_int, [vp, P(BeState), vp, vp, i32, P(BeOut), P(BeActOut), u64, vp]),
        "be_policy_bytes": (i64, [vp]),
        "be_observe_blocks": (C.c_int, [vp, P(BeState), vp, vp, vp]),
        "be_board_config_default": (C.c_int, [P(BeBoardConfig), i32, i32]),
        "be_board_create": (C.c_int, [P(BeBoardConfig), i32, P(vp)]),
        "be_board_destroy": (C.c_int, [vp]),
        "be_board_last_error": (C.c_char_p, [vp]),
        "be_board_reset": (C.c_int, [vp, P(BeBoardState), vp, vp, i32, P(BeBoardOut), vp]),
        "be_board_step": (C.c_int, [vp, P(BeBoardState), vp, vp, P(BeBoardOut), vp]),
        "be_board_rollout": (C.c_int, [vp, P(BeBoardState), vp, vp, i32, P(BeBoardOut), vp]),
        "be_board_observe": (C.c_int, [vp, P(BeBoardState), P(BeBoardOut), vp]),
        "be_board_status": (C.c_int, [vp, P(i32), vp]),
        "be_board_pool_bytes": (i64, [vp]),
    }
    # a BALLENV_LIB diagnostics build from an earlier commit (tools/build_rev_lib.sh, A/B runs) may
    # predate the newest entry points and ABI version; the in-tree library must match exactly
    diag = bool(os.environ.get("BALLENV_LIB"))
    for name, (res, args) in sig.items():
        fn = getattr(L, name, None)
        if fn is None and diag and (name.startswith("be_pool_") or name == "be_board_pool_bytes"):
            continue
        if fn is None:
            raise BallEnvError(f"{LIB_PATH} does not export {name}: rebuild it")
        fn.restype, fn.argtypes = res, args
    v = L.be_abi_version()
    if v != ABI_VERSION and not (diag and v >= 6):
        raise BallEnvError(f"{LIB_PATH} has ABI {v}, expected {ABI_VERSION}: rebuild it")
    _lib = L
    return L


def check(rc: int, ctx=None) -> None:
    if rc != BE_OK:
        msg = lib().be_last_error(ctx)
        raise BallEnvError(f"libballenv error {rc}: {msg.decode() if msg else ''}")


def default_config(num_envs: int, window: int) -> BeConfig:
    c = BeConfig()
    check(lib().be_config_default(C.byref(c), num_envs, window))
    return c


def config_check(c: BeConfig) -> str:
    """'' if valid, else the library's message (pure host code, no GPU needed)."""
    buf = C.create_string_buffer(256)
    rc = lib().be_config_check(C.byref(c), buf, 256)
    return "" if rc == BE_OK else buf.value.decode()


def step_bytes(c: BeConfig) -> int:
    return int(lib().be_step_bytes(C.byref(c)))


def stats_slots(c: BeConfig) -> int:
    return int(lib().be_stats_slots(C.byref(c)))


def board_check(rc: int, board=None) -> None:
    if rc != BE_OK:
        msg = lib().be_board_last_error(board)
        raise BallEnvError(f"libballenv board error {rc}: {msg.decode() if msg else ''}")

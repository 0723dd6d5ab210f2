"""ctypes binding of libsacx (include/sacx.h).

This is the product path's only way to the GPU: there is no CPU fallback.  If
the shared library is missing the import raises, loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SACX_LIBPATH") or os.path.join(os.path.dirname(_HERE), "lib", "libsacx.so")

SACX_ABI_VERSION = 8
MAX_DEPTH = 4                   # SACX_MAX_DEPTH: hidden layers per net
MAX_MODELS = 8                  # SACX_MAX_MODELS: --num_models
STAGE_FLOATS = 65536            # SACX_STAGE_FLOATS (include/sacx.h)
ACT = {"relu": 0, "tanh": 1, "elu": 2}
DTYPES = {0: "f32", 1: "i32", 2: "i64", 3: "u32", 4: "f64"}
STEP_EXTERNAL_RANDOMS = 1
STEP_EAGER = 2
ROLE_WORK, ROLE_PARAM, ROLE_TARGET, ROLE_STATE = 0, 1, 2, 3
DIAG_DISC = 1
DIAG_EXPERT_ACTIONS = 2
STAT_NAMES = ["q1_loss", "q2_loss", "p_loss", "alpha_loss", "alpha", "mse_loss", "nlp_mean", "step"]

# every symbol include/sacx.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "sacx_create", "sacx_destroy", "sacx_last_error", "sacx_arena_bytes", "sacx_layout", "sacx_bind",
    "sacx_buffer_append", "sacx_buffer_append_host", "sacx_actor_act_host",
    "sacx_buffer_append_host_seeds", "sacx_actor_act_host_seeds", "sacx_expert_set", "sacx_perm_push", "sacx_rng_seed", "sacx_rng_set_state",
    "sacx_rng_get_state", "sacx_sac_step", "sacx_model_fit", "sacx_sync", "sacx_plan_info", "sacx_model_plan_info", "sacx_profile",
    "sacx_time_graph", "sacx_actor_act", "sacx_time_kernels", "sacx_rollout",
    "sacx_dp_unique_id", "sacx_dp_init", "sacx_dp_init_local", "sacx_dp_local_step", "sacx_expert_diag", "sacx_resync", "sacx_seed_stride",
    "sacx_seed_select", "sacx_prepare", "sacx_actor_evaluate", "sacx_critic_forward", "sacx_model_forward",
    "sacx_model_loss", "sacx_spec_hits", "sacx_settle", "sacx_model_sample",
]


class Config(ctypes.Structure):
    _fields_ = [
        ("abi_version", ctypes.c_int32),
        ("s_dim", ctypes.c_int32),
        ("a_dim", ctypes.c_int32),
        ("hidden", ctypes.c_int32 * 2),
        ("activation", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("buffer_capacity", ctypes.c_int64),
        ("per_state_std", ctypes.c_int32),
        ("use_expert", ctypes.c_int32),
        ("expert_capacity", ctypes.c_int32),
        ("expert_batch", ctypes.c_int32),
        ("model_hidden", ctypes.c_int32 * 2),
        ("model_activation", ctypes.c_int32),
        ("model_batch", ctypes.c_int32),
        ("target_update_int", ctypes.c_int32),
        ("graph_steps", ctypes.c_int32),
        ("stats_capacity", ctypes.c_int32),
        ("perm_capacity", ctypes.c_int32),
        ("gamma", ctypes.c_float),
        ("tau", ctypes.c_float),
        ("lr_q", ctypes.c_float),
        ("lr_pi", ctypes.c_float),
        ("lr_alpha", ctypes.c_float),
        ("lr_model", ctypes.c_float),
        ("init_temperature", ctypes.c_float),
        ("target_entropy", ctypes.c_float),
        ("act_limit", ctypes.c_float),
        ("epsilon", ctypes.c_float),
        ("reward_loss_coef", ctypes.c_float),
        ("gemm_bf16", ctypes.c_int32),
        ("seeds", ctypes.c_int32),
        ("actor_gaussian", ctypes.c_int32),
        ("actor_std_mult", ctypes.c_float),
        ("actor_output_norm", ctypes.c_int32),
        ("actor_layer_norm", ctypes.c_int32),
        ("num_models", ctypes.c_int32),
        ("model_max_grad_norm", ctypes.c_float),
        ("delta_clip_loss", ctypes.c_float),
        ("reward_clip_loss", ctypes.c_float),
        ("act_per_layer", ctypes.c_int32),
        ("act_layers", (ctypes.c_int32 * 2) * 3),
        ("delta_clip_pred", ctypes.c_float),
        ("single_seed_plan", ctypes.c_int32),
        # ABI 7
        ("gaussian_model", ctypes.c_int32),
        ("scale_model_loss", ctypes.c_int32),
        ("separate_reward_nn", ctypes.c_int32),
        ("reward_hidden", ctypes.c_int32 * 2),
        ("reward_act_layers", ctypes.c_int32 * 2),
        ("critic_hidden", ctypes.c_int32 * 2),
        # ABI 8: every net's hidden layers [actor, critics, world models, reward nets] (0: the fields above)
        ("net_depth", ctypes.c_int32 * 4),
        ("net_hidden", (ctypes.c_int32 * 4) * 4),
        ("net_acts", (ctypes.c_int32 * 4) * 4),
    ]


class Segment(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 48),
        ("offset", ctypes.c_uint64),
        ("rows", ctypes.c_int64),
        ("cols", ctypes.c_int64),
        ("dtype", ctypes.c_int32),
        ("role", ctypes.c_int32),
    ]


class LaunchInfo(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 32),
        ("kernel", ctypes.c_char * 32),
        ("grid", ctypes.c_int32),
        ("block", ctypes.c_int32),
        ("flops", ctypes.c_double),
        ("bytes", ctypes.c_double),
    ]


_lib = None


def lib():
    """Loads libsacx.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libsacx.so not found at {LIB_PATH}: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(the HIP engine is required; there is no CPU fallback)")
    L = ctypes.CDLL(LIB_PATH)
    vp, i32, i64, u32, f32, f64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32,
                                   ctypes.c_float, ctypes.c_double)
    P = ctypes.POINTER
    sig = {
        "sacx_create": (ctypes.c_int, [P(Config), P(vp)]),
        "sacx_destroy": (None, [vp]),
        "sacx_last_error": (ctypes.c_char_p, [vp]),
        "sacx_arena_bytes": (i64, [vp]),
        "sacx_seed_stride": (i64, [vp]),
        "sacx_seed_select": (i32, [vp, i32]),
        "sacx_layout": (ctypes.c_int, [vp, P(Segment), i32, P(i32)]),
        "sacx_bind": (ctypes.c_int, [vp, vp, ctypes.c_uint64, vp]),
        "sacx_buffer_append": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64]),
        "sacx_expert_set": (ctypes.c_int, [vp, vp, vp, i32, f32]),
        "sacx_perm_push": (ctypes.c_int, [vp, vp, i64]),
        "sacx_rng_seed": (ctypes.c_int, [vp, u32]),
        "sacx_rng_set_state": (ctypes.c_int, [vp, vp, i32, i32, f64]),
        "sacx_rng_get_state": (ctypes.c_int, [vp, vp, P(i32), P(i32), P(f64)]),
        "sacx_sac_step": (ctypes.c_int, [vp, i64, i64, i32, i32]),
        "sacx_prepare": (ctypes.c_int, [vp, i64, i32]),
        "sacx_model_fit": (ctypes.c_int, [vp, vp, i64, i32]),
        "sacx_sync": (ctypes.c_int, [vp]),
        "sacx_settle": (ctypes.c_int, [vp]),
        "sacx_plan_info": (ctypes.c_int, [vp, P(LaunchInfo), i32, P(i32)]),
        "sacx_model_plan_info": (ctypes.c_int, [vp, P(LaunchInfo), i32, P(i32)]),
        "sacx_spec_hits": (i64, [vp]),
        "sacx_profile": (ctypes.c_int, [vp, i64, P(f64), i32]),
        "sacx_time_graph": (ctypes.c_int, [vp, i64, ctypes.c_char_p, P(f64)]),
        "sacx_actor_act": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "sacx_buffer_append_host": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64]),
        "sacx_actor_act_host": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "sacx_buffer_append_host_seeds": (ctypes.c_int, [vp, vp, vp, vp, vp, vp, i64]),
        "sacx_actor_act_host_seeds": (ctypes.c_int, [vp, vp, i64, i32, vp]),
        "sacx_actor_evaluate": (ctypes.c_int, [vp, vp, i64, vp, vp]),
        "sacx_critic_forward": (ctypes.c_int, [vp, i32, vp, vp, i64, i32, vp]),
        "sacx_model_forward": (ctypes.c_int, [vp, i32, vp, vp, i64, f32, f32, vp, vp, vp]),
        "sacx_model_sample": (ctypes.c_int, [vp, i32, vp, vp, i64, i32, f32, f32, vp, vp, vp]),
        "sacx_model_loss": (ctypes.c_int, [vp, i32, vp, vp, vp, vp, i64, f32, f32, vp]),
        "sacx_time_kernels": (ctypes.c_int, [vp, ctypes.c_char_p, i32, P(f64), P(f64), P(i64)]),
        "sacx_dp_unique_id": (ctypes.c_int, [vp, i32]),
        "sacx_resync": (ctypes.c_int, [vp]),
        "sacx_expert_diag": (ctypes.c_int, [vp, vp, vp, vp, i32, i32, f32, vp]),
        "sacx_dp_init": (ctypes.c_int, [vp, vp, i32, i32]),
        "sacx_dp_init_local": (ctypes.c_int, [vp, i32, i32]),
        "sacx_dp_local_step": (ctypes.c_int, [vp, i32, i64, i64, i32]),
        "sacx_rollout": (ctypes.c_int, [vp, i32, vp, i64, i32, i32, f32, f32, vp, vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


class SacxError(RuntimeError):
    pass


def check(rc: int, handle=None, what: str = "") -> None:
    if rc != 0:
        msg = lib().sacx_last_error(handle)
        raise SacxError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")

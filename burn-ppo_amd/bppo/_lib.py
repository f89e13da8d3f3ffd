"""ctypes binding of libbppo.so (include/bppo.h).

The library is built in-tree (burn-ppo_amd/bppo/libbppo.so, `make -C burn-ppo_amd`).
There is no fallback: if the shared object is missing or fails to load, every
entry point raises.  The product path never touches the CPU oracle.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# BPPO_LIB_PATH: a diagnostic build of the same library (e.g. libbppo_stamps.so)
LIB_PATH = os.environ.get("BPPO_LIB_PATH") or os.path.join(HERE, "libbppo.so")

OK, ERR_ARG, ERR_NONFINITE, ERR_EMPTY_MASK, ERR_HIP, ERR_COMM, ERR_UNSUPPORTED = range(7)
ENV_CARTPOLE, ENV_CONNECT_FOUR, ENV_LIARS_DICE = 0, 1, 2
ENV_SKULL = 3
ENV_KINDS = {"cartpole": ENV_CARTPOLE, "connect_four": ENV_CONNECT_FOUR, "liars_dice": ENV_LIARS_DICE,
             "skull": ENV_SKULL}
MAX_PLAYERS = 6


class BppoError(RuntimeError):
    def __init__(self, status, msg):
        super().__init__(f"bppo status {status}: {msg}")
        self.status = status


class Config(C.Structure):
    _fields_ = [("env_kind", C.c_int32), ("num_envs", C.c_int32), ("num_steps", C.c_int32),
                ("hidden_size", C.c_int32), ("num_hidden", C.c_int32), ("relu", C.c_int32),
                ("ctde", C.c_int32), ("critic_hidden_size", C.c_int32), ("critic_num_hidden", C.c_int32),
                ("num_epochs", C.c_int32), ("num_minibatches", C.c_int32),
                ("normalize_obs", C.c_int32), ("normalize_returns", C.c_int32), ("clip_value", C.c_int32),
                ("gamma", C.c_double), ("gae_lambda", C.c_double), ("clip_epsilon", C.c_double),
                ("value_coef", C.c_double), ("max_grad_norm", C.c_double), ("adam_epsilon", C.c_double),
                ("target_kl", C.c_double), ("return_clip", C.c_double),
                ("reward_shaping_coef", C.c_double), ("seed", C.c_uint64), ("env_seed_base", C.c_uint64),
                ("rng_stream", C.c_uint64),
                ("cnn", C.c_int32), ("num_conv_layers", C.c_int32), ("conv_channels", C.c_int32 * 4),
                ("kernel_size", C.c_int32), ("cnn_fc_hidden_size", C.c_int32), ("cnn_num_fc_layers", C.c_int32),
                ("normalize_values", C.c_int32), ("player_count", C.c_int32), ("split_networks", C.c_int32),
                ("shuffle_windows", C.c_int32)]


class Episode(C.Structure):
    _fields_ = [("total_reward", C.c_float * MAX_PLAYERS), ("length", C.c_int32), ("env_index", C.c_int32),
                ("step", C.c_int32), ("pad", C.c_int32)]


class RolloutInfo(C.Structure):
    _fields_ = [("episodes", C.c_int32), ("mean_return", C.c_float), ("mean_length", C.c_float),
                ("pad", C.c_int32), ("rng_word_pos", C.c_uint64)]


METRIC_NAMES = ("policy_loss", "value_loss", "entropy", "entropy_scaled", "approx_kl", "clip_fraction",
                "explained_variance", "total_loss", "value_mean", "returns_mean", "adv_mean_raw",
                "adv_std_raw", "adv_min_raw", "adv_max_raw", "value_error_mean", "value_error_std",
                "value_error_max", "avg_valid_actions", "entropy_valid_pct")


# PopArt metrics (ppo.rs:2061-2068; NaN when the reference's Option is None)
POPART_METRICS = ("value_norm_target_mean", "value_norm_target_std", "value_norm_rescale_mag")


class UpdateMetrics(C.Structure):
    _fields_ = [(n, C.c_float) for n in METRIC_NAMES] + [("num_updates", C.c_int32),
                                                          ("epochs_run", C.c_int32)] + \
        [(n, C.c_float) for n in POPART_METRICS]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_size_t, C.c_void_p)

# every symbol declared in include/bppo.h (tests check the .so exports them all)
EXPORTS = (
    "bppo_create", "bppo_destroy", "bppo_last_error", "bppo_version", "bppo_num_params",
    "bppo_params_set", "bppo_params_get", "bppo_forward", "bppo_rng_get", "bppo_rng_set",
    "bppo_vecenv_reset", "bppo_vecenv_observe", "bppo_vecenv_step", "bppo_vecenv_set_step", "bppo_set_reward_shaping_schedule",
    "bppo_obs_norm_get", "bppo_obs_norm_set", "bppo_ret_norm_get", "bppo_ret_norm_set",
    "bppo_collect_rollouts", "bppo_rollout_episodes", "bppo_compute_gae", "bppo_ppo_update", "bppo_train_step", "bppo_train_steps",
    "bppo_set_allreduce", "bppo_set_allreduce_async", "bppo_get_stream", "bppo_opponents_set", "bppo_opponents_get_envs", "bppo_buffer_get", "bppo_buffer_set", "bppo_gae_device", "bppo_gae_rows_device",
    "bppo_gae_mp_device", "bppo_last_kernel_ms", "bppo_debug_libm", "bppo_debug_shuffle_chain", "bppo_debug_chain_walk2", "bppo_minibatch_rows",
    "bppo_debug_fisher_yates", "bppo_debug_gemm", "bppo_debug_shuffle_engine", "bppo_debug_sample",
    "bppo_rng_fill_bytes", "bppo_rng_from_seed", "bppo_rng_key_get", "bppo_num_param_tensors",
    "bppo_optimizer_get", "bppo_optimizer_set", "bppo_popart_get", "bppo_popart_set",
    "bppo_config_size", "bppo_update_metrics_size", "bppo_episode_size", "bppo_rollout_info_size",
    "bppo_set_explained_variance_mode", "bppo_set_minibatch_kernel", "bppo_set_rank",
    "bppo_debug_record_params",
)

# ABI struct -> the library's sizeof export (checked when the library loads)
STRUCT_SIZES = {"bppo_config_size": Config, "bppo_update_metrics_size": UpdateMetrics,
                "bppo_episode_size": Episode, "bppo_rollout_info_size": RolloutInfo}

_lib = None


def lib():
    """Load libbppo.so (raises if it is absent: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process: the PyTorch wheel ships its own libamdhip64.
    # Loading torch first makes libbppo bind to that already-loaded runtime; the
    # other order leaves torch unable to see the GPU ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} is missing; build it with `make -C burn-ppo_amd` "
                           f"(or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    vp, u64, sz, i32 = C.c_void_p, C.c_uint64, C.c_size_t, C.c_int32
    fp = C.POINTER(C.c_float)
    dp = C.POINTER(C.c_double)
    sig = {
        "bppo_create": (i32, [C.POINTER(Config), C.c_int, vp, C.POINTER(vp)]),
        "bppo_destroy": (None, [vp]),
        "bppo_last_error": (C.c_char_p, [vp]),
        "bppo_version": (C.c_char_p, []),
        "bppo_num_params": (sz, [vp]),
        "bppo_params_set": (i32, [vp, vp, sz]),
        "bppo_params_get": (i32, [vp, vp, sz]),
        "bppo_forward": (i32, [vp, vp, vp, i32, vp, vp]),
        "bppo_rng_get": (i32, [vp, C.POINTER(u64)]),
        "bppo_rng_set": (i32, [vp, u64]),
        "bppo_vecenv_reset": (i32, [vp]),
        "bppo_vecenv_observe": (i32, [vp, vp, vp, vp, vp]),
        "bppo_vecenv_step": (i32, [vp, vp, vp, vp, vp, vp, i32, C.POINTER(i32)]),
        "bppo_vecenv_set_step": (i32, [vp, u64]),
        "bppo_set_reward_shaping_schedule": (i32, [vp, vp, vp, i32]),
        "bppo_obs_norm_get": (i32, [vp, vp, vp, dp]),
        "bppo_obs_norm_set": (i32, [vp, vp, vp, C.c_double]),
        "bppo_ret_norm_get": (i32, [vp, vp, vp]),
        "bppo_ret_norm_set": (i32, [vp, vp, vp]),
        "bppo_collect_rollouts": (i32, [vp, C.POINTER(RolloutInfo)]),
        "bppo_rollout_episodes": (i32, [vp, vp, i32, C.POINTER(i32)]),
        "bppo_compute_gae": (i32, [vp]),
        "bppo_ppo_update": (i32, [vp, C.c_double, C.c_double, C.POINTER(UpdateMetrics)]),
        "bppo_train_step": (i32, [vp, C.c_double, C.c_double, C.POINTER(RolloutInfo), C.POINTER(UpdateMetrics)]),
        "bppo_train_steps": (i32, [vp, i32, vp, vp, C.c_uint64, vp, vp, vp, i32, vp]),
        "bppo_set_allreduce": (i32, [vp, ALLREDUCE_FN, vp, i32]),
        "bppo_set_allreduce_async": (i32, [vp, ALLREDUCE_FN, vp, i32]),
        "bppo_set_rank": (i32, [vp, i32]),
        "bppo_get_stream": (i32, [vp, C.POINTER(vp)]),
        "bppo_opponents_set": (i32, [vp, i32, vp, vp, vp, vp, i32, vp, vp, vp]),
        "bppo_opponents_get_envs": (i32, [vp, vp, vp]),
        "bppo_buffer_get": (i32, [vp, C.c_char_p, vp, sz]),
        "bppo_buffer_set": (i32, [vp, C.c_char_p, vp, sz]),
        "bppo_gae_device": (i32, [vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp, vp]),
        "bppo_gae_rows_device": (i32, [vp, vp, vp, vp, i32, i32, C.c_float, C.c_float, vp, vp, vp, vp]),
        "bppo_gae_mp_device": (i32, [vp, vp, vp, vp, vp, i32, i32, i32, C.c_float, C.c_float, vp, vp,
                                     vp]),
        "bppo_last_kernel_ms": (i32, [vp, C.c_char_p, fp]),
        "bppo_debug_libm": (i32, [i32, i32, vp, vp, sz]),
        "bppo_debug_shuffle_chain": (i32, [u64, u64, u64, C.c_uint32, vp, C.POINTER(u64)]),
        "bppo_minibatch_rows": (i32, [vp, vp, i32, C.POINTER(i32)]),
        "bppo_debug_chain_walk2": (i32, [u64, u64, u64, u64, C.c_uint32, C.c_uint32, C.POINTER(u64), C.POINTER(u64)]),
        "bppo_debug_fisher_yates": (i32, [i32, vp, C.c_uint32, vp]),
        "bppo_debug_gemm": (i32, [i32, i32, i32, i32, vp, vp, vp, i32, vp, vp]),
        "bppo_debug_shuffle_engine": (i32, [u64, u64, u64, C.c_uint32, i32, u64, i32, i32, vp, vp, vp]),
        "bppo_debug_sample": (i32, [i32, i32, vp, vp, u64, u64, u64, vp, vp]),
        "bppo_rng_fill_bytes": (i32, [vp, vp, sz]),
        "bppo_rng_from_seed": (i32, [vp, vp]),
        "bppo_rng_key_get": (i32, [vp, vp]),
        "bppo_num_param_tensors": (sz, [vp]),
        "bppo_optimizer_get": (i32, [vp, vp, vp, vp, sz]),
        "bppo_optimizer_set": (i32, [vp, vp, vp, vp, sz]),
        "bppo_popart_get": (i32, [vp, vp]),
        "bppo_popart_set": (i32, [vp, vp]),
        "bppo_set_explained_variance_mode": (i32, [vp, i32]),
        "bppo_set_minibatch_kernel": (i32, [vp, i32]),
        "bppo_debug_record_params": (i32, [vp, vp, i32]),
    }
    for name in STRUCT_SIZES:
        sig[name] = (sz, [])
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    for name, struct in STRUCT_SIZES.items():
        if getattr(L, name)() != C.sizeof(struct):
            raise RuntimeError(f"{LIB_PATH}: {name}() = {getattr(L, name)()} but ctypes {struct.__name__} is "
                               f"{C.sizeof(struct)} bytes (binding out of date with include/bppo.h)")
    _lib = L
    return L


def check(status, ctx=None):
    if status != OK:
        msg = lib().bppo_last_error(ctx).decode() if ctx else ""
        raise BppoError(status, msg)


def ptr(a):
    """data pointer of a numpy array or torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        assert a.flags["C_CONTIGUOUS"]
        return a.ctypes.data
    return a.data_ptr()

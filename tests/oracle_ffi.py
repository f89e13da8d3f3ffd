"""ctypes bindings for the CPU oracle (oracle/build/liboracle.so).

TEST INFRASTRUCTURE ONLY: the oracle is the parity checker and the timed CPU
baseline.  The product path (burn-ppo_amd/bppo -> libbppo.so) never imports
this module.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "build", "liboracle.so")

ENV_CARTPOLE, ENV_CONNECT_FOUR, ENV_LIARS_DICE, ENV_SKULL = 0, 1, 2, 3


def _num_players(kind):
    return {ENV_CARTPOLE: 1, ENV_CONNECT_FOUR: 2, ENV_LIARS_DICE: 4, ENV_SKULL: 6}[kind]


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


class Rng(C.Structure):
    _fields_ = [("key", C.c_uint32 * 8), ("stream", C.c_uint64), ("word_pos", C.c_uint64),
                ("cached_block", C.c_uint64), ("block", C.c_uint32 * 16), ("rounds", C.c_int)]


class CartPole(C.Structure):
    _fields_ = [("x", C.c_float), ("x_dot", C.c_float), ("theta", C.c_float),
                ("theta_dot", C.c_float), ("steps", C.c_int32), ("rng", Rng)]


class ConnectFour(C.Structure):
    _fields_ = [("board", (C.c_int8 * 7) * 6), ("current", C.c_int8), ("game_over", C.c_int8),
                ("winner", C.c_int8)]


class LiarsDice(C.Structure):
    _fields_ = [("dice", (C.c_uint8 * 2) * 4), ("num_dice", C.c_uint8 * 4), ("current", C.c_uint8),
                ("has_bid", C.c_int8), ("bid_qty", C.c_uint8), ("bid_face", C.c_uint8),
                ("last_bidder", C.c_int8), ("bid_count", C.c_int32),
                ("hist_player", C.c_uint8 * 16), ("hist_qty", C.c_uint8 * 16),
                ("hist_face", C.c_uint8 * 16), ("hist_len", C.c_int32),
                ("elim_order", C.c_int8 * 4), ("num_elim", C.c_int32), ("game_over", C.c_int8),
                ("global_step", C.c_uint64), ("rng", Rng)]


class Skull(C.Structure):
    _fields_ = [("n", C.c_int32), ("has_trap", C.c_uint8 * 6), ("rose_count", C.c_uint8 * 6),
                ("wins", C.c_uint8 * 6), ("stack_len", C.c_uint8 * 6), ("stack", (C.c_uint8 * 4) * 6),
                ("passed", C.c_uint8 * 6), ("revealed", C.c_uint8 * 6),
                ("phase", C.c_int32), ("current", C.c_int32), ("round_starter", C.c_int32),
                ("current_bid", C.c_int32), ("current_bidder", C.c_int32), ("hist_len", C.c_int32),
                ("hist_player", C.c_uint8 * 8), ("hist_bid", C.c_uint8 * 8),
                ("roses_found", C.c_int32), ("must_reveal_own", C.c_int32), ("last_skull_owner", C.c_int32),
                ("elim_order", C.c_int8 * 6), ("num_elim", C.c_int32), ("game_over", C.c_int32),
                ("winner", C.c_int32), ("rng", Rng)]


class ObsNorm(C.Structure):
    _fields_ = [("dim", C.c_int), ("mean", C.POINTER(C.c_double)), ("var", C.POINTER(C.c_double)),
                ("count", C.c_double), ("clip", C.c_float)]


class RetNorm(C.Structure):
    _fields_ = [("num_envs", C.c_int), ("num_players", C.c_int), ("returns", C.POINTER(C.c_double)),
                ("var", C.c_double), ("mean", C.c_double), ("count", C.c_double), ("gamma", C.c_double),
                ("epsilon", C.c_double), ("clip", C.c_float)]


class PopArt(C.Structure):
    _fields_ = [("mean", C.c_double), ("var", C.c_double), ("count", C.c_double), ("epsilon", C.c_double)]


class Adam(C.Structure):
    _fields_ = [("m1", C.POINTER(C.c_float)), ("m2", C.POINTER(C.c_float)), ("time", C.POINTER(C.c_int32)),
                ("has_state", C.c_int)]


class Episode(C.Structure):
    _fields_ = [("total_rewards", C.c_float * 6), ("length", C.c_int32), ("env_index", C.c_int32)]


class NetDesc(C.Structure):
    _fields_ = [("ctde", C.c_int), ("obs_dim", C.c_int), ("priv_dim", C.c_int), ("act_dim", C.c_int),
                ("relu", C.c_int), ("n_actor", C.c_int), ("actor_width", C.c_int),
                ("n_critic", C.c_int), ("critic_width", C.c_int), ("n_params", C.c_size_t),
                ("cnn", C.c_int), ("n_conv", C.c_int), ("conv_ch", C.c_int * 4), ("ksize", C.c_int),
                ("H", C.c_int), ("W", C.c_int), ("C", C.c_int), ("split", C.c_int)]


class PpoCfg(C.Structure):
    _fields_ = [("num_epochs", C.c_int), ("num_minibatches", C.c_int), ("clip_epsilon", C.c_float),
                ("clip_epsilon_d", C.c_double), ("value_coef", C.c_double),
                ("max_grad_norm", C.c_double), ("adam_epsilon", C.c_float),
                ("target_kl", C.c_double), ("clip_value", C.c_int)]


class TrainCfg(C.Structure):
    _fields_ = [("env_kind", C.c_int), ("num_envs", C.c_int), ("num_steps", C.c_int),
                ("hidden", C.c_int), ("num_hidden", C.c_int), ("relu", C.c_int), ("ctde", C.c_int),
                ("critic_hidden", C.c_int), ("critic_num_hidden", C.c_int),
                ("normalize_obs", C.c_int), ("normalize_returns", C.c_int),
                ("return_clip", C.c_float), ("gamma", C.c_double), ("gae_lambda", C.c_double),
                ("lr", C.c_double), ("ent_coef", C.c_double), ("reward_shaping", C.c_double),
                ("ppo", PpoCfg), ("seed", C.c_uint64), ("threads", C.c_int),
                ("cnn", C.c_int), ("num_conv", C.c_int), ("conv_ch", C.c_int * 4), ("ksize", C.c_int),
                ("normalize_values", C.c_int), ("player_count", C.c_int), ("split_networks", C.c_int),
                ("env_seed_offset", C.c_uint64), ("rng_stream", C.c_uint64), ("shuffle_windows", C.c_int)]


class UpdateMetrics(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "policy_loss", "value_loss", "entropy", "entropy_scaled", "approx_kl", "clip_fraction",
        "explained_variance", "total_loss", "value_mean", "returns_mean", "adv_mean_raw",
        "adv_std_raw", "adv_min_raw", "adv_max_raw", "value_error_mean", "value_error_std",
        "value_error_max", "avg_valid_actions", "entropy_valid_pct")] + [
        ("num_updates", C.c_int32), ("epochs_run", C.c_int32)] + [
        (n, C.c_float) for n in ("value_norm_target_mean", "value_norm_target_std", "value_norm_rescale_mag")]


class MbStats(C.Structure):
    _fields_ = [(n, C.c_float) for n in (
        "loss", "policy_loss", "value_loss", "entropy", "approx_kl", "clip_fraction", "value_mean",
        "returns_mean", "value_error_mean", "value_error_std", "value_error_max",
        "avg_valid_actions", "entropy_valid_pct")]


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        fp = np.ctypeslib.ndpointer
        f32 = fp(np.float32, flags="C_CONTIGUOUS")
        f64 = fp(np.float64, flags="C_CONTIGUOUS")
        i32 = fp(np.int32, flags="C_CONTIGUOUS")
        u32 = fp(np.uint32, flags="C_CONTIGUOUS")
        u8 = fp(np.uint8, flags="C_CONTIGUOUS")
        sig = {
            "or_chacha_block": (None, [u32, C.c_uint64, C.c_uint64, C.c_int, u32]),
            "or_rng_seed_u64": (None, [C.POINTER(Rng), C.c_uint64]),
            "or_rng_next_u32": (C.c_uint32, [C.POINTER(Rng)]),
            "or_rng_next_u64": (C.c_uint64, [C.POINTER(Rng)]),
            "or_rng_fill_bytes": (None, [C.POINTER(Rng), u8, C.c_size_t]),
            "or_gen_range_f32": (C.c_float, [C.POINTER(Rng), C.c_float, C.c_float]),
            "or_gen_range_u32": (C.c_uint32, [C.POINTER(Rng), C.c_uint32, C.c_uint32]),
            "or_gen_range_u8_incl": (C.c_uint8, [C.POINTER(Rng), C.c_uint8, C.c_uint8]),
            "or_shuffle_u32": (None, [C.POINTER(Rng), u32, C.c_size_t]),
            "or_shuffle_targets": (None, [C.POINTER(Rng), u32, C.c_size_t]),
            "or_apply_swaps": (None, [u32, u32, C.c_size_t]),
            "or_rng_words": (None, [C.c_uint64, C.c_uint64, u32, C.c_size_t]),
            "or_rng_words_key": (None, [u32, C.c_int, C.c_uint64, u32, C.c_size_t]),
            "or_rng_seed_key": (None, [C.c_uint64, u32]),
            "or_cartpole_new": (None, [C.POINTER(CartPole), C.c_uint64]),
            "or_cartpole_reset": (None, [C.POINTER(CartPole), f32]),
            "or_cartpole_step": (None, [C.POINTER(CartPole), C.c_int32, f32, C.POINTER(C.c_float),
                                        C.POINTER(C.c_int)]),
            "or_c4_new": (None, [C.POINTER(ConnectFour)]),
            "or_c4_reset": (None, [C.POINTER(ConnectFour), f32]),
            "or_c4_step": (None, [C.POINTER(ConnectFour), C.c_int32, f32, f32, C.POINTER(C.c_int)]),
            "or_c4_mask": (None, [C.POINTER(ConnectFour), u8]),
            "or_c4_get_obs": (None, [C.POINTER(ConnectFour), f32]),
            "or_ld_new": (None, [C.POINTER(LiarsDice), C.c_uint64]),
            "or_ld_reset": (None, [C.POINTER(LiarsDice), f32]),
            "or_ld_step": (None, [C.POINTER(LiarsDice), C.c_int32, C.c_float, f32, f32,
                                  C.POINTER(C.c_int)]),
            "or_ld_mask": (None, [C.POINTER(LiarsDice), u8]),
            "or_ld_priv": (None, [C.POINTER(LiarsDice), f32]),
            "or_ld_get_obs": (None, [C.POINTER(LiarsDice), f32]),
            "or_skull_new": (None, [C.POINTER(Skull), C.c_int, C.c_uint64]),
            "or_skull_reset": (None, [C.POINTER(Skull), C.c_void_p]),
            "or_skull_step": (None, [C.POINTER(Skull), C.c_int32, C.c_float, C.c_void_p, f32,
                                     C.POINTER(C.c_int), C.POINTER(C.c_int)]),
            "or_skull_mask": (None, [C.POINTER(Skull), u8]),
            "or_skull_get_obs": (None, [C.POINTER(Skull), f32]),
            "or_skull_priv": (None, [C.POINTER(Skull), f32]),
            "or_skull_placements": (None, [C.POINTER(Skull), i32]),
            "or_skull_final_rewards": (None, [C.POINTER(Skull), f32]),
            "or_skull_outcome": (None, [C.POINTER(Skull), i32]),
            "or_vecenv_new": (C.c_void_p, [C.c_int, C.c_int, C.c_uint64]),
            "or_vecenv_new_np": (C.c_void_p, [C.c_int, C.c_int, C.c_uint64, C.c_int]),
            "or_vecenv_invalid": (C.c_int, [C.c_void_p]),
            "or_vecenv_free": (None, [C.c_void_p]),
            "or_vecenv_get_obs": (None, [C.c_void_p, f32]),
            "or_vecenv_get_players": (None, [C.c_void_p, i32]),
            "or_vecenv_get_masks": (C.c_int, [C.c_void_p, u8]),
            "or_vecenv_get_priv": (None, [C.c_void_p, f32]),
            "or_vecenv_set_shaping": (None, [C.c_void_p, C.c_float]),
            "or_vecenv_step": (C.c_int, [C.c_void_p, i32, f32, f32, u8, C.POINTER(Episode), C.c_int]),
            "or_vecenv_env_ptr": (C.c_void_p, [C.c_void_p, C.c_int]),
            "or_net_num_params": (C.c_size_t, [C.POINTER(NetDesc)]),
            "or_linear": (None, [f32, f32, f32, C.c_size_t, C.c_int, C.c_int, C.c_int, f32]),
            "or_linear_dx": (None, [f32, f32, C.c_size_t, C.c_int, C.c_int, f32]),
            "or_set_relu_masks": (None, [C.c_void_p, C.c_int]),
            "or_net_forward": (None, [C.POINTER(NetDesc), f32, f32, C.c_void_p, C.c_size_t, f32, f32]),
            "or_sample_categorical": (None, [C.POINTER(Rng), f32, C.c_size_t, C.c_int, i32]),
            "or_log_prob": (C.c_float, [f32, C.c_int, C.c_int32]),
            "or_entropy": (C.c_float, [f32, C.c_int]),
            "or_compute_gae": (None, [f32, f32, f32, f32, C.c_int, C.c_int, C.c_float, C.c_float,
                                      f32, f32]),
            "or_compute_gae_mp": (None, [f32, i32, f32, f32, f32, C.c_int, C.c_int, C.c_int,
                                         C.c_float, C.c_float, f32, f32]),
            "or_explained_variance": (C.c_float, [f32, f32, C.c_size_t]),
            "or_normalize_advantages": (None, [f32, C.c_size_t, f32, C.POINTER(C.c_float),
                                               C.POINTER(C.c_float), C.POINTER(C.c_float),
                                               C.POINTER(C.c_float)]),
            "or_minibatch_loss_grad": (None, [C.POINTER(NetDesc), f32, C.c_size_t, f32, C.c_void_p,
                                              i32, f32, f32, f32, f32, C.c_void_p, C.POINTER(PpoCfg),
                                              C.c_double, f32, C.POINTER(MbStats)]),
            "or_trainer_new": (C.c_void_p, [C.POINTER(TrainCfg), f32]),
            "or_trainer_free": (None, [C.c_void_p]),
            "or_trainer_num_params": (C.c_size_t, [C.c_void_p]),
            "or_trainer_get_params": (None, [C.c_void_p, f32]),
            "or_trainer_set_params": (None, [C.c_void_p, f32]),
            "or_trainer_rng_pos": (C.c_uint64, [C.c_void_p]),
            "or_trainer_collect": (C.c_int, [C.c_void_p]),
            "or_trainer_gae": (None, [C.c_void_p]),
            "or_trainer_update": (None, [C.c_void_p, C.POINTER(UpdateMetrics)]),
            "or_trainers_update": (None, [C.c_void_p, C.c_int, C.c_void_p]),
            "or_trainer_set_buffer": (C.c_int, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]),
            "or_trainer_mb_log": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
            "or_trainer_buffer": (C.c_size_t, [C.c_void_p, C.c_char_p, C.c_void_p, C.c_size_t]),
            "or_trainer_obs_norm_state": (None, [C.c_void_p, f64, f64, C.POINTER(C.c_double)]),
            "or_trainer_ret_norm_state": (None, [C.c_void_p, f64, C.c_void_p]),
            "or_trainer_episodes": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
            "or_trainer_last_phase_seconds": (C.c_double, [C.c_void_p, C.c_int]),
            "or_trainer_set_opponents": (None, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p,
                                                C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]),
            "or_trainer_opponent_envs": (None, [C.c_void_p, C.c_void_p, C.c_void_p]),
            "or_shuffle_positions": (None, [C.c_void_p, C.c_int, i32, C.c_void_p, i32]),
            "or_gen_range_u64": (C.c_uint64, [C.c_void_p, C.c_uint64, C.c_uint64]),
            "or_set_mlp_parallel": (None, [C.c_int]),
            "or_obs_norm_init": (None, [C.POINTER(ObsNorm), C.c_int, C.c_float]),
            "or_obs_norm_free": (None, [C.POINTER(ObsNorm)]),
            "or_obs_norm_update_batch": (None, [C.POINTER(ObsNorm), f32, C.c_size_t]),
            "or_obs_norm_normalize_batch": (None, [C.POINTER(ObsNorm), f32, C.c_size_t]),
            "or_ret_norm_init": (None, [C.POINTER(RetNorm), C.c_int, C.c_int, C.c_double, C.c_float]),
            "or_ret_norm_free": (None, [C.POINTER(RetNorm)]),
            "or_ret_norm_update_return": (None, [C.POINTER(RetNorm), C.c_int, C.c_int, C.c_float]),
            "or_ret_norm_update_variance": (None, [C.POINTER(RetNorm), C.c_int, C.c_int]),
            "or_ret_norm_normalize": (C.c_float, [C.POINTER(RetNorm), C.c_float]),
            "or_ret_norm_reset_player": (None, [C.POINTER(RetNorm), C.c_int, C.c_int]),
            "or_ret_norm_reset_env": (None, [C.POINTER(RetNorm), C.c_int]),
            "or_ret_norm_update_and_normalize_all": (None, [C.POINTER(RetNorm), f32, u8]),
            "or_apply_action_mask": (C.c_long, [f32, u8, C.c_size_t, C.c_int]),
            "or_trainer_set_rng": (None, [C.c_void_p, u32, C.c_uint64]),
            "or_trainer_set_shaping": (None, [C.c_void_p, C.c_float]),
            "or_schedule_get": (C.c_double, [C.c_void_p, C.c_void_p, C.c_int, C.c_uint64]),
            "or_trainer_set_adam": (None, [C.c_void_p, f32, f32, i32, C.c_int]),
            "or_trainer_popart": (None, [C.c_void_p, C.c_void_p, C.c_void_p]),
            "or_popart_init": (None, [C.POINTER(PopArt)]),
            "or_popart_std": (C.c_double, [C.POINTER(PopArt)]),
            "or_popart_update": (None, [C.POINTER(PopArt), f32, C.c_size_t, C.POINTER(C.c_double),
                                        C.POINTER(C.c_double)]),
            "or_popart_normalize": (None, [C.POINTER(PopArt), f32, C.c_size_t, f32]),
            "or_popart_denormalize": (None, [C.POINTER(PopArt), f32, C.c_size_t]),
            "or_trainer_get_adam": (None, [C.c_void_p, f32, f32, i32, C.c_int]),
            "or_trainer_set_norms": (None, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p,
                                            C.c_void_p]),
            "or_adam_init": (None, [C.POINTER(Adam), C.POINTER(NetDesc)]),
            "or_adam_free": (None, [C.POINTER(Adam)]),
            "or_adam_step": (None, [C.POINTER(NetDesc), C.POINTER(Adam), f32, f32, C.c_double, C.c_float,
                                    C.c_float]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


# ------------------------------------------------------------- helpers ---
def chacha_block(key_words, counter, stream=0, rounds=20):
    out = np.zeros(16, np.uint32)
    lib().or_chacha_block(np.asarray(key_words, np.uint32), counter, stream, rounds, out)
    return out


def stdrng_words(seed, n, skip=0):
    out = np.zeros(n, np.uint32)
    lib().or_rng_words(seed, skip, out, n)
    return out


def seed_key(seed):
    k = np.zeros(8, np.uint32)
    lib().or_rng_seed_key(seed, k)
    return k


def new_rng(seed):
    r = Rng()
    lib().or_rng_seed_u64(C.byref(r), seed)
    return r


def mlp_desc(obs_dim, act_dim, hidden, num_hidden, relu=True, split=False):
    """shared trunk, or split_networks (a critic trunk of the same shape on obs)"""
    d = NetDesc(ctde=0, obs_dim=obs_dim, priv_dim=0, act_dim=act_dim, relu=int(relu),
                n_actor=num_hidden, actor_width=hidden, n_critic=num_hidden if split else 0,
                critic_width=hidden if split else 0, split=int(split))
    d.n_params = lib().or_net_num_params(C.byref(d))
    return d


def cnn_desc(act_dim, conv_ch, ksize, fc_hidden, n_fc, relu=True, split=False):
    """Connect Four CNN (obs 86, shape (6, 7, 2)); split: the critic's own conv + FC trunk"""
    d = NetDesc(ctde=0, obs_dim=86, priv_dim=0, act_dim=act_dim, relu=int(relu), n_actor=n_fc,
                actor_width=fc_hidden, n_critic=n_fc if split else 0, critic_width=fc_hidden if split else 0,
                cnn=1, n_conv=len(conv_ch),
                conv_ch=(C.c_int * 4)(*[conv_ch[min(i, len(conv_ch) - 1)] for i in range(4)]), ksize=ksize,
                H=6, W=7, C=2, split=int(split))
    d.n_params = lib().or_net_num_params(C.byref(d))
    return d


def ctde_desc(obs_dim, priv_dim, act_dim, hidden, num_hidden, critic_hidden, critic_num_hidden,
              relu=True):
    d = NetDesc(ctde=1, obs_dim=obs_dim, priv_dim=priv_dim, act_dim=act_dim, relu=int(relu),
                n_actor=num_hidden, actor_width=hidden, n_critic=critic_num_hidden,
                critic_width=critic_hidden)
    d.n_params = lib().or_net_num_params(C.byref(d))
    return d


def net_forward(desc, params, obs, priv=None):
    B = obs.shape[0]
    logits = np.zeros((B, desc.act_dim), np.float32)
    values = np.zeros(B, np.float32)
    pp = None if priv is None else np.ascontiguousarray(priv, np.float32)
    lib().or_net_forward(C.byref(desc), np.ascontiguousarray(params, np.float32),
                         np.ascontiguousarray(obs, np.float32),
                         None if pp is None else pp.ctypes.data, B, logits, values)
    return logits, values


_mb_stats_fn = None


def minibatch_stats(desc, params, obs, priv, actions, old_logp, adv_norm, returns, old_values, masks, pc, ent):
    """or_minibatch_loss_grad's statistics alone (grads = NULL: forward and loss, no backward)"""
    global _mb_stats_fn
    if _mb_stats_fn is None:
        f = lib()["or_minibatch_loss_grad"]          # a second function object: its own argtypes
        vp = C.c_void_p
        f.restype = None
        f.argtypes = [C.POINTER(NetDesc), vp, C.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp, C.POINTER(PpoCfg),
                      C.c_double, vp, C.POINTER(MbStats)]
        _mb_stats_fn = f
    arrs = [np.ascontiguousarray(a, t) if a is not None else None
            for a, t in ((params, np.float32), (obs, np.float32), (priv, np.float32), (actions, np.int32),
                         (old_logp, np.float32), (adv_norm, np.float32), (returns, np.float32),
                         (old_values, np.float32), (masks, np.float32))]
    ptr = [None if a is None else a.ctypes.data for a in arrs]
    ms = MbStats()
    _mb_stats_fn(C.byref(desc), ptr[0], len(arrs[1]) if arrs[1].ndim == 1 else arrs[1].shape[0], ptr[1], ptr[2],
                 ptr[3], ptr[4], ptr[5], ptr[6], ptr[7], ptr[8], C.byref(pc), ent, None, C.byref(ms))
    return {f: getattr(ms, f) for f, _ in MbStats._fields_}


def linear(x, W, b, relu):
    """or_linear: y = act(x W + b) in matrixmultiply's KC=256 fma-chain order (relu: 1, 0 tanh, -1 none)"""
    B, K = x.shape
    N = W.shape[1]
    y = np.zeros((B, N), np.float32)
    lib().or_linear(np.ascontiguousarray(x, np.float32), np.ascontiguousarray(W, np.float32),
                    np.ascontiguousarray(b, np.float32), B, K, N, relu, y)
    return y


def linear_dx(dz, W):
    """or_linear_dx: dx [B][in] = dz [B][out] W^T, W [in][out], an f32 fma chain over out from 0"""
    B, out = dz.shape
    dx = np.zeros((B, W.shape[0]), np.float32)
    lib().or_linear_dx(np.ascontiguousarray(dz, np.float32), np.ascontiguousarray(W, np.float32), B, W.shape[0],
                       out, dx)
    return dx


def compute_gae(rewards, dones, values, last_values, gamma, lam):
    T, N = rewards.shape
    adv = np.zeros((T, N), np.float32)
    ret = np.zeros((T, N), np.float32)
    lib().or_compute_gae(np.ascontiguousarray(rewards, np.float32), np.ascontiguousarray(dones, np.float32),
                         np.ascontiguousarray(values, np.float32),
                         np.ascontiguousarray(last_values, np.float32), T, N, gamma, lam, adv, ret)
    return adv, ret


def compute_gae_mp(all_rewards, players, dones, values, last_v_pp, gamma, lam):
    T, N, P = all_rewards.shape
    adv = np.zeros((T, N), np.float32)
    ret = np.zeros((T, N), np.float32)
    lib().or_compute_gae_mp(np.ascontiguousarray(all_rewards, np.float32),
                            np.ascontiguousarray(players, np.int32),
                            np.ascontiguousarray(dones, np.float32),
                            np.ascontiguousarray(values, np.float32),
                            np.ascontiguousarray(last_v_pp, np.float32), T, N, P, gamma, lam, adv, ret)
    return adv, ret


def ppo_cfg(num_epochs=4, num_minibatches=4, clip=0.2, value_coef=0.5, max_grad_norm=0.5,
            adam_eps=1e-5, target_kl=None, clip_value=False):
    return PpoCfg(num_epochs=num_epochs, num_minibatches=num_minibatches, clip_epsilon=clip,
                  clip_epsilon_d=clip, value_coef=value_coef, max_grad_norm=max_grad_norm,
                  adam_epsilon=adam_eps, target_kl=-1.0 if target_kl is None else target_kl,
                  clip_value=int(clip_value))


def train_cfg(env_kind=ENV_CARTPOLE, num_envs=8, num_steps=128, hidden=64, num_hidden=2, relu=True,
              ctde=False, critic_hidden=0, critic_num_hidden=0, normalize_obs=True,
              normalize_returns=True, return_clip=10.0, gamma=0.99, gae_lambda=0.95, lr=1e-3,
              ent_coef=0.01, reward_shaping=0.0, seed=42, threads=0, cnn=None, normalize_values=False,
              player_count=0, split=False, env_seed_offset=0, rng_stream=0, shuffle_windows=False, **ppo):
    """cnn: None, or (conv_channels per layer, kernel_size); hidden / num_hidden are
    then cnn_fc_hidden_size / cnn_num_fc_layers"""
    extra = {}
    if cnn is not None:
        ch, ks = cnn
        extra = dict(cnn=1, num_conv=len(ch), conv_ch=(C.c_int * 4)(*[ch[min(i, len(ch) - 1)] for i in range(4)]),
                     ksize=ks)
    return TrainCfg(**extra, normalize_values=int(normalize_values), player_count=player_count,
                    env_seed_offset=env_seed_offset, rng_stream=rng_stream, shuffle_windows=int(shuffle_windows),
                    split_networks=int(split), env_kind=env_kind, num_envs=num_envs, num_steps=num_steps, hidden=hidden,
                    num_hidden=num_hidden, relu=int(relu), ctde=int(ctde), critic_hidden=critic_hidden,
                    critic_num_hidden=critic_num_hidden, normalize_obs=int(normalize_obs),
                    normalize_returns=int(normalize_returns), return_clip=return_clip, gamma=gamma,
                    gae_lambda=gae_lambda, lr=lr, ent_coef=ent_coef, reward_shaping=reward_shaping,
                    ppo=ppo_cfg(**ppo), seed=seed, threads=threads)


class Trainer:
    """One oracle training run (main.rs:684-988 restated)."""

    def __init__(self, cfg, params):
        self.cfg = cfg
        self.h = lib().or_trainer_new(C.byref(cfg), np.ascontiguousarray(params, np.float32))
        self.n_params = lib().or_trainer_num_params(self.h)

    def close(self):
        if self.h:
            lib().or_trainer_free(self.h)
            self.h = None

    __del__ = close

    def collect(self):
        return lib().or_trainer_collect(self.h)

    def gae(self):
        lib().or_trainer_gae(self.h)

    def update(self):
        m = UpdateMetrics()
        lib().or_trainer_update(self.h, C.byref(m))
        return {k: getattr(m, k) for k, _ in UpdateMetrics._fields_}

    @staticmethod
    def update_ranks(trainers):
        """or_trainers_update: one data-parallel update of W rank trainers in lockstep
        (per-rank shuffles and advantage statistics, gradients summed over the ranks
        and scaled by 1/W before clip + Adam) -> W metric dicts"""
        W = len(trainers)
        hs = (C.c_void_p * W)(*[t.h for t in trainers])
        ms = (UpdateMetrics * W)()
        lib().or_trainers_update(hs, W, ms)
        return [{k: getattr(m, k) for k, _ in UpdateMetrics._fields_} for m in ms]

    def params(self):
        out = np.zeros(self.n_params, np.float32)
        lib().or_trainer_get_params(self.h, out)
        return out

    def episodes(self):
        """the last collect's EpisodeStats in the reference's order (step, then env index):
        (total_rewards[0] bits, length, env_index)"""
        n = lib().or_trainer_episodes(self.h, None, 0)
        eps = (Episode * max(n, 1))()
        lib().or_trainer_episodes(self.h, eps, n)
        return [(np.float32(eps[i].total_rewards[0]).view(np.uint32).item(), eps[i].length, eps[i].env_index)
                for i in range(n)]

    def rng_pos(self):
        return lib().or_trainer_rng_pos(self.h)

    def buffer(self, name, dtype=np.float32):
        n = lib().or_trainer_buffer(self.h, name.encode(), None, 0)
        out = np.zeros(n // 4, dtype)
        lib().or_trainer_buffer(self.h, name.encode(), out.ctypes.data, n)
        return out

    def minibatch_log(self):
        """the last update's per-minibatch statistics in run order: list of dicts"""
        n = lib().or_trainer_mb_log(self.h, None, 0)
        arr = (MbStats * max(n, 1))()
        lib().or_trainer_mb_log(self.h, arr, n)
        return [{f: getattr(arr[i], f) for f, _ in MbStats._fields_} for i in range(n)]

    def set_buffer(self, name, arr):
        a = np.ascontiguousarray(arr)
        assert lib().or_trainer_set_buffer(self.h, name.encode(), a.ctypes.data, a.nbytes) == 0, name

    def obs_norm_state(self, dim):
        mean = np.zeros(dim, np.float64)
        var = np.zeros(dim, np.float64)
        cnt = C.c_double()
        lib().or_trainer_obs_norm_state(self.h, mean, var, C.byref(cnt))
        return mean, var, cnt.value

    def ret_norm_state(self, returns=False):
        mvc = np.zeros(3, np.float64)
        if not returns:
            lib().or_trainer_ret_norm_state(self.h, mvc, None)
            return mvc
        r = np.zeros(self.cfg.num_envs * _num_players(self.cfg.env_kind), np.float64)
        lib().or_trainer_ret_norm_state(self.h, mvc, r.ctypes.data)
        return mvc, r

    def set_opponents(self, params, norms, n_opp, learner_pos, pos_to_opp, current_opp):
        """ppo.rs:537-1063 opponent pool: params [K, n_params]; norms: per model
        (mean [D], m2 [D], count) or None; seat state of envs [0, n_opp)."""
        params = np.ascontiguousarray(params, np.float32)
        K = params.shape[0] if params.ndim == 2 else 0
        D = lib().or_trainer_buffer(self.h, b"obs", None, 0) // 4 // (self.cfg.num_steps * self.cfg.num_envs)
        mean = np.zeros((max(K, 1), D)); m2 = np.zeros((max(K, 1), D)); cnt = np.zeros(max(K, 1))
        for k, nm in enumerate(norms or []):
            if nm is not None:
                mean[k], m2[k], cnt[k] = nm
        self._keep = [params, mean, m2, cnt, np.ascontiguousarray(learner_pos, np.int32),
                      np.ascontiguousarray(pos_to_opp, np.int32), np.ascontiguousarray(current_opp, np.int32)]
        k = self._keep
        lib().or_trainer_set_opponents(self.h, K, k[0].ctypes.data, k[1].ctypes.data, k[2].ctypes.data,
                                       k[3].ctypes.data, n_opp, k[4].ctypes.data, k[5].ctypes.data,
                                       k[6].ctypes.data)

    def opponent_envs(self, n_opp, P):
        lp = np.zeros(max(n_opp, 1), np.int32); po = np.zeros(max(n_opp, 1) * P, np.int32)
        lib().or_trainer_opponent_envs(self.h, lp.ctypes.data, po.ctypes.data)
        return lp[:n_opp], po[:n_opp * P]

    def popart(self, set4=None):
        g = np.zeros(4)
        lib().or_trainer_popart(self.h, g.ctypes.data, None)
        if set4 is not None:
            s4 = np.ascontiguousarray(set4, np.float64)
            lib().or_trainer_popart(self.h, None, s4.ctypes.data)
        return g

    def phase_seconds(self, ph):
        return lib().or_trainer_last_phase_seconds(self.h, ph)

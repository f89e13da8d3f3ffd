"""The reference's hot-path surfaces, MI355X-native underneath.

Mirrors burn-ppo's in-process interfaces with the same names and argument
meaning, so a caller of the reference finds the same calls:

    VecEnv                 env.rs:270-487  (new / step / get_observations / ...)
    ActorCritic            network/mod.rs:28-189 (forward / params)
    RolloutBuffer          ppo.rs:52-200  (device-resident; fields exported on demand)
    collect_rollouts       ppo.rs:213-500
    compute_gae            ppo.rs:1069-1124 (bootstrap from main.rs:877-947)
    ppo_update             ppo.rs:1661-2112
    Trainer.train_update   one iteration of run_training's loop, main.rs:684-988

All state lives in HBM inside one libbppo context (bppo_ctx); these wrappers only
marshal host arrays.  Errors that the reference panics on (NaN log-probs,
empty action masks) raise BppoError.
"""
import ctypes as C
from collections import deque

import numpy as np

from . import _lib as L
from .host import ENV_DIMS, make_config, orthogonal_init, schedule_get, shaping_schedule, to_struct


class Context:
    """Owns one bppo_ctx (device buffers, env state, params, Adam, RNG)."""

    def __init__(self, cfg, device=0, stream=None, rank=0, world=1, envs_per_rank=None):
        self.cfg = cfg
        self.rank, self.world = rank, world
        self.struct = to_struct(cfg, rank, world, envs_per_rank)
        h = C.c_void_p()
        st = L.lib().bppo_create(C.byref(self.struct), device, stream, C.byref(h))
        self.h = h
        if st != L.OK:
            msg = L.lib().bppo_last_error(h).decode() if h else ""
            if h:
                L.lib().bppo_destroy(h)
            self.h = None
            raise L.BppoError(st, msg)
        self.N = self.struct.num_envs
        self.T = self.struct.num_steps
        sched = shaping_schedule(cfg)
        if len(sched) != 1 or sched[0][1] != 0:
            self.set_reward_shaping_schedule(sched)
        self.n_params = L.lib().bppo_num_params(self.h)
        self.obs_dim, self.num_actions, self.num_players, priv = ENV_DIMS[cfg["env"]]
        # the device keeps privileged rows only for CTDE nets
        self.priv_dim = priv if cfg["network_type"] == "ctde" else 0
        # seated players (opponent-pool seat tables): Skull's player_count, else NUM_PLAYERS
        self.seats = int(cfg.get("player_count", 4)) if cfg["env"] == "skull" else self.num_players
        self.has_masks = cfg["env"] != "cartpole"
        self._ar_keep = None

    def close(self):
        if self.h:
            L.lib().bppo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, st):
        L.check(st, self.h)

    # parity hooks -------------------------------------------------------
    def buffer(self, name, dtype=np.float32, shape=None):
        TN = self.T * self.N
        n = {"obs": TN * self.obs_dim, "last_values": self.N, "grad": self.n_params,
             "priv": TN * self.priv_dim, "masks": TN * self.num_actions,
             "all_rewards": TN * self.num_players, "last_v_pp": self.N * self.num_players}.get(name, TN)
        if shape is not None:
            n = int(np.prod(shape))
        out = np.zeros(n, dtype)
        self._chk(L.lib().bppo_buffer_get(self.h, name.encode(), out.ctypes.data, out.nbytes))
        return out.reshape(shape) if shape else out

    def minibatch_rows(self):
        """the last update's per-minibatch metric rows [runs, width] (bppo_minibatch_rows):
        columns 0-4 = sums of policy loss, 2 x value loss, entropy, approx KL, clip
        fraction; column 10 = the minibatch's row count"""
        w = C.c_int32()
        n = L.lib().bppo_minibatch_rows(self.h, None, 0, C.byref(w))
        out = np.zeros((max(n, 0), w.value), np.float32)
        if n > 0:
            L.lib().bppo_minibatch_rows(self.h, out.ctypes.data, n, C.byref(w))
        return out

    def set_buffer(self, name, arr):
        arr = np.ascontiguousarray(arr)
        self._chk(L.lib().bppo_buffer_set(self.h, name.encode(), arr.ctypes.data, arr.nbytes))

    def rng_pos(self):
        p = C.c_uint64()
        self._chk(L.lib().bppo_rng_get(self.h, C.byref(p)))
        return p.value

    def set_rng_pos(self, p):
        self._chk(L.lib().bppo_rng_set(self.h, p))

    def obs_norm(self):
        m = np.zeros(self.obs_dim); v = np.zeros(self.obs_dim); c = C.c_double()
        self._chk(L.lib().bppo_obs_norm_get(self.h, m.ctypes.data, v.ctypes.data, C.byref(c)))
        return m, v, c.value

    def set_obs_norm(self, mean, m2, count):
        mean = np.ascontiguousarray(mean, np.float64); m2 = np.ascontiguousarray(m2, np.float64)
        self._chk(L.lib().bppo_obs_norm_set(self.h, mean.ctypes.data, m2.ctypes.data, float(count)))

    def ret_norm(self):
        """-> ([mean, M2, count], rolling returns [N * num_players]) (normalization.rs:121-134)"""
        mvc = np.zeros(3); r = np.zeros(self.N * self.num_players)
        self._chk(L.lib().bppo_ret_norm_get(self.h, mvc.ctypes.data, r.ctypes.data))
        return mvc, r

    def set_ret_norm(self, mvc, returns):
        mvc = np.ascontiguousarray(mvc, np.float64); r = np.ascontiguousarray(returns, np.float64)
        if r.size != self.N * self.num_players:
            raise ValueError(f"returns must hold num_envs * num_players = {self.N * self.num_players} values")
        self._chk(L.lib().bppo_ret_norm_set(self.h, mvc.ctypes.data, r.ctypes.data))

    def set_reward_shaping_schedule(self, milestones):
        """reward_shaping_coef: Schedule [(value, step), ...] (config.rs:761-762)."""
        v = np.ascontiguousarray([float(a) for a, _ in milestones], np.float64)
        st = np.ascontiguousarray([int(b) for _, b in milestones], np.uint64)
        self._chk(L.lib().bppo_set_reward_shaping_schedule(self.h, v.ctypes.data, st.ctypes.data, len(v)))

    def popart(self):
        """PopArtNormalizer state [mean, M2, count, epsilon] (normalization.rs:275-284)"""
        st = np.zeros(4)
        self._chk(L.lib().bppo_popart_get(self.h, st.ctypes.data))
        return st

    def set_popart(self, st):
        st = np.ascontiguousarray(st, np.float64)
        self._chk(L.lib().bppo_popart_set(self.h, st.ctypes.data))

    def set_opponents(self, params, norms, num_opponent_envs, learner_pos, pos_to_opp, current_opp):
        """Opponent-pool rollouts (ppo.rs:537-1063): params [K, n_params] of the
        loaded opponents, norms[k] = (mean, m2, count) or None, seat state of envs
        [0, num_opponent_envs) (EnvState, opponent_pool.rs:80-124), current_opp
        [P - 1] = OpponentPool::sample_all_slots."""
        params = np.ascontiguousarray(params, np.float32).reshape(-1, self.n_params)
        K, D, P = params.shape[0], self.obs_dim, self.seats
        mean = np.zeros((max(K, 1), D)); m2 = np.zeros((max(K, 1), D)); cnt = np.zeros(max(K, 1))
        for k, nm in enumerate(norms or []):
            if nm is not None:
                mean[k], m2[k], cnt[k] = nm
        lp = np.ascontiguousarray(learner_pos, np.int32)
        po = np.ascontiguousarray(pos_to_opp, np.int32)
        co = np.ascontiguousarray(current_opp, np.int32)
        self._chk(L.lib().bppo_opponents_set(self.h, K, params.ctypes.data, mean.ctypes.data, m2.ctypes.data,
                                             cnt.ctypes.data, int(num_opponent_envs), lp.ctypes.data,
                                             po.ctypes.data, co.ctypes.data))
        self._n_opp = int(num_opponent_envs)

    def opponent_envs(self):
        """-> (learner_pos [n_opp], pos_to_opp [n_opp, P]) after the last rollout"""
        n = getattr(self, "_n_opp", 0)
        lp = np.zeros(max(n, 1), np.int32); po = np.zeros(max(n, 1) * self.seats, np.int32)
        self._chk(L.lib().bppo_opponents_get_envs(self.h, lp.ctypes.data, po.ctypes.data))
        return lp[:n], po[:n * self.seats].reshape(n, self.seats)

    def kernel_ms(self, name):
        f = C.c_float()
        self._chk(L.lib().bppo_last_kernel_ms(self.h, name.encode(), C.byref(f)))
        return f.value

    def set_explained_variance_mode(self, mode):
        """0: f64 sums on the device (default); 1: the reference's f32 sequential sums,
        bit for bit (ppo.rs:1268-1294), on a host thread beside the update"""
        self._chk(L.lib().bppo_set_explained_variance_mode(self.h, int(mode)))

    def set_minibatch_kernel(self, mode):
        """0: exact f32 kernel for the update's first minibatch, split-bf16 for the rest
        (default); 1: exact for every minibatch; 2: split for every minibatch (parity hook)"""
        self._chk(L.lib().bppo_set_minibatch_kernel(self.h, int(mode)))

    def record_params(self, max_minibatches):
        """parity hook (bppo_debug_record_params): the next updates copy the parameters of
        each minibatch they run into the returned [max_minibatches, n_params] array
        (record_params(0) stops it)"""
        if max_minibatches <= 0:
            self._chk(L.lib().bppo_debug_record_params(self.h, None, 0))
            self._rec = None
            return None
        self._rec = np.zeros((max_minibatches, self.n_params), np.float32)
        self._chk(L.lib().bppo_debug_record_params(self.h, self._rec.ctypes.data, max_minibatches))
        return self._rec

    def set_allreduce(self, fn, world, stream_ordered=False):
        """fn(device_ptr:int, n:int) -> None must leave the SUM over ranks in place.
        stream_ordered: fn only enqueues the reduction on `self.stream` (no host
        wait per minibatch; bppo_set_allreduce_async)."""
        def _cb(p, n, user):
            try:
                fn(p, n)
                return 0
            except Exception:
                return 1
        self._ar_keep = L.ALLREDUCE_FN(_cb)
        setter = L.lib().bppo_set_allreduce_async if stream_ordered else L.lib().bppo_set_allreduce
        self._chk(L.lib().bppo_set_rank(self.h, self.rank))     # PopArt's W > 1 all-gather slot
        self._chk(setter(self.h, self._ar_keep, None, world))

    @property
    def stream(self):
        """The context's HIP stream (hipStream_t as int)."""
        s = C.c_void_p()
        self._chk(L.lib().bppo_get_stream(self.h, C.byref(s)))
        return s.value or 0


class VecEnv:
    """env.rs VecEnv over the device-resident envs (CartPole, Connect Four, Liar's Dice)."""

    def __init__(self, ctx):
        self.ctx = ctx

    @classmethod
    def new(cls, ctx):
        """VecEnv::new(num_envs, |i| E::new(seed + i)) — env.rs:281-302."""
        v = cls(ctx)
        v.ctx._chk(L.lib().bppo_vecenv_reset(ctx.h))
        return v

    def num_envs(self):
        return self.ctx.N

    def get_observations(self):
        o = np.zeros(self.ctx.N * self.ctx.obs_dim, np.float32)
        self.ctx._chk(L.lib().bppo_vecenv_observe(self.ctx.h, o.ctypes.data, None, None, None))
        return o

    def get_current_players(self):
        p = np.zeros(self.ctx.N, np.int32)
        self.ctx._chk(L.lib().bppo_vecenv_observe(self.ctx.h, None, p.ctypes.data, None, None))
        return p

    def get_action_masks(self):
        """env.rs:350-362: [N*A] bool, None when the env has no masks (CartPole)."""
        if not self.ctx.has_masks:
            return None
        m = np.zeros(self.ctx.N * self.ctx.num_actions, np.uint8)
        self.ctx._chk(L.lib().bppo_vecenv_observe(self.ctx.h, None, None, m.ctypes.data, None))
        return m.astype(bool)

    def get_privileged_obs(self):
        """env.rs:365-376: [N*G] (Liar's Dice 120, Skull 200) for CTDE contexts, None otherwise."""
        if not self.ctx.priv_dim:
            return None
        g = np.zeros(self.ctx.N * self.ctx.priv_dim, np.float32)
        self.ctx._chk(L.lib().bppo_vecenv_observe(self.ctx.h, None, None, None, g.ctypes.data))
        return g

    def set_step(self, step):
        self.ctx._chk(L.lib().bppo_vecenv_set_step(self.ctx.h, int(step)))

    def step(self, actions):
        """-> (obs [N*obs], rewards [N][P], dones [N] bool, completed episodes)"""
        N = self.ctx.N
        a = np.ascontiguousarray(actions, np.int32)
        obs = np.zeros(N * self.ctx.obs_dim, np.float32)
        P = self.ctx.num_players
        rew = np.zeros(N * P, np.float32)
        dn = np.zeros(N, np.uint8)
        cap = N
        eps = (L.Episode * cap)()
        n = C.c_int32()
        self.ctx._chk(L.lib().bppo_vecenv_step(self.ctx.h, a.ctypes.data, obs.ctypes.data, rew.ctypes.data,
                                               dn.ctypes.data, eps, cap, C.byref(n)))
        done_eps = [dict(total_rewards=list(eps[i].total_reward[:P]), length=eps[i].length,
                         env_index=eps[i].env_index) for i in range(min(n.value, cap))]
        return obs, rew.reshape(N, P), dn.astype(bool), done_eps


class ActorCritic:
    """ActorCriticNetwork (network/mod.rs): flat params in Burn record order."""

    def __init__(self, ctx):
        self.ctx = ctx

    def is_ctde(self):
        return self.ctx.cfg["network_type"] == "ctde"

    def get_params(self):
        out = np.zeros(self.ctx.n_params, np.float32)
        self.ctx._chk(L.lib().bppo_params_get(self.ctx.h, out.ctypes.data, out.size))
        return out

    def set_params(self, p):
        p = np.ascontiguousarray(p, np.float32)
        self.ctx._chk(L.lib().bppo_params_set(self.ctx.h, p.ctypes.data, p.size))

    def forward(self, obs, priv=None):
        """network/mod.rs:93-114 (MLP) / forward_actor + forward_critic (CTDE, ctde.rs:132-183)
        -> (logits [B, A], values [B, 1]); priv [B, G] is required for CTDE."""
        obs = np.ascontiguousarray(obs, np.float32).reshape(-1, self.ctx.obs_dim)
        B = obs.shape[0]
        pr = None
        if priv is not None:
            pr = np.ascontiguousarray(priv, np.float32).reshape(B, -1)
        lg = np.zeros((B, self.ctx.num_actions), np.float32)
        v = np.zeros(B, np.float32)
        self.ctx._chk(L.lib().bppo_forward(self.ctx.h, obs.ctypes.data, None if pr is None else pr.ctypes.data,
                                           B, lg.ctypes.data, v.ctypes.data))
        return lg, v.reshape(B, 1)


class RolloutBuffer:
    """ppo.rs:52-200; the [T, N, ...] fields stay in HBM and are exported on demand."""

    def __init__(self, ctx):
        self.ctx = ctx

    def __getattr__(self, name):
        ctx = self.__dict__["ctx"]
        T, N = ctx.T, ctx.N
        if name == "observations":
            return ctx.buffer("obs").reshape(T, N, ctx.obs_dim)
        if name == "actions":
            return ctx.buffer("actions", np.int32).reshape(T, N)
        if name in ("rewards", "dones", "values", "log_probs", "advantages", "returns"):
            return ctx.buffer(name).reshape(T, N)
        if name == "privileged_obs" and ctx.priv_dim:
            return ctx.buffer("priv").reshape(T, N, ctx.priv_dim)
        if name == "action_masks" and ctx.has_masks:
            return ctx.buffer("masks").reshape(T, N, ctx.num_actions)
        if name == "acting_players":
            return ctx.buffer("players", np.int32).reshape(T, N)
        if name == "all_rewards":
            return ctx.buffer("all_rewards").reshape(T, N, ctx.num_players)
        raise AttributeError(name)


def collect_rollouts(ctx):
    """ppo.rs:213-500.  Returns (rollout info, last_value_per_player is implicit
    on device).  The main RNG advances by T*N*A words exactly as the reference."""
    info = L.RolloutInfo()
    ctx._chk(L.lib().bppo_collect_rollouts(ctx.h, C.byref(info)))
    return info


def rollout_episodes(ctx):
    """EpisodeStats of the last rollout in the reference's order: by step, then
    env index (env.rs:470-483 appends completed envs in env order each step)."""
    n = C.c_int32()
    ctx._chk(L.lib().bppo_rollout_episodes(ctx.h, None, 0, C.byref(n)))
    cap = n.value
    if cap == 0:
        return []
    eps = (L.Episode * cap)()
    ctx._chk(L.lib().bppo_rollout_episodes(ctx.h, eps, cap, C.byref(n)))
    P = ctx.num_players
    return [dict(total_rewards=list(eps[i].total_reward[:P]), length=eps[i].length, env_index=eps[i].env_index,
                 step=eps[i].step) for i in range(min(n.value, cap))]


def compute_gae(ctx):
    """main.rs:877-947 bootstrap (updated obs stats) + ppo.rs:1069-1124."""
    ctx._chk(L.lib().bppo_compute_gae(ctx.h))


def _metrics_dict(m):
    d = {k: getattr(m, k) for k in L.METRIC_NAMES + L.POPART_METRICS}
    d["num_updates"] = m.num_updates
    d["epochs_run"] = m.epochs_run
    return d


def ppo_update(ctx, learning_rate, entropy_coef):
    """ppo.rs:1661-2112 -> UpdateMetrics dict."""
    m = L.UpdateMetrics()
    ctx._chk(L.lib().bppo_ppo_update(ctx.h, float(learning_rate), float(entropy_coef), C.byref(m)))
    return _metrics_dict(m)


def train_step(ctx, learning_rate, entropy_coef):
    """collect_rollouts + bootstrap/GAE + ppo_update in one call (bppo_train_step):
    enqueued back to back, one host wait.  -> (rollout info, UpdateMetrics dict)."""
    info, m = L.RolloutInfo(), L.UpdateMetrics()
    ctx._chk(L.lib().bppo_train_step(ctx.h, float(learning_rate), float(entropy_coef), C.byref(info), C.byref(m)))
    return info, _metrics_dict(m)


def perf_scalars(env_steps, seconds, rollout_ms, gae_ms, update_ms):
    """The reference's perf/* scalars (main.rs:1092-1132) over one logging interval:
    perf/sps = env steps / wall seconds, perf/{rollout,gae,update}_time = the phases' summed
    seconds, perf/{rollout,update}_pct of their sum.  The phase times here are the device
    times of the phases (HIP events on the context's stream; the reference times its host
    calls, which on the device path only enqueue), so the reference's dashboards read the
    same names with the same meaning."""
    r, g, u = rollout_ms * 1e-3, gae_ms * 1e-3, update_ms * 1e-3
    tot = r + g + u
    out = {"perf/sps": env_steps / seconds if seconds > 0 else 0.0, "perf/rollout_time": r, "perf/gae_time": g,
           "perf/update_time": u}
    if tot > 0:
        out["perf/rollout_pct"] = r / tot * 100.0
        out["perf/update_pct"] = u / tot * 100.0
    return out


class Trainer:
    """run_training's per-update loop body (main.rs:684-988) on one GPU (or one
    rank of a data-parallel job)."""

    def __init__(self, cfg=None, device=0, params=None, init_seed=0, **kw):
        self.cfg = cfg or make_config("cartpole")
        self.ctx = Context(self.cfg, device=device, **kw)
        self.model = ActorCritic(self.ctx)
        self.vec_env = VecEnv(self.ctx)
        self.buffer = RolloutBuffer(self.ctx)
        self.model.set_params(orthogonal_init(self.cfg, init_seed) if params is None else params)
        self.global_step = 0
        # main.rs:988 global_step += num_steps * num_envs, num_envs of the whole job (every
        # rank's shard) so the lr / entropy / shaping schedules see the job's env steps
        self.steps_per_update = self.ctx.T * self.ctx.N * self.ctx.world
        # main.rs:850-853: the last 100 completed episodes' returns (player 0)
        self.recent_returns = deque(maxlen=100)

    def mean_recent_return(self):
        return float(np.mean(self.recent_returns)) if self.recent_returns else float("nan")

    def train_update(self, track_returns=False):
        """one iteration of main.rs:684-988.  track_returns: push this rollout's
        completed episodes into the 100-episode window (main.rs:842-853)."""
        lr = schedule_get(self.cfg["learning_rate"], self.global_step)         # main.rs:706
        ent = schedule_get(self.cfg["entropy_coef"], self.global_step)         # main.rs:716
        self.vec_env.set_step(self.global_step)
        if track_returns:
            info = collect_rollouts(self.ctx)
            for ep in rollout_episodes(self.ctx):
                self.recent_returns.append(ep["total_rewards"][0])
            compute_gae(self.ctx)
            metrics = ppo_update(self.ctx, lr, ent)
        else:
            info, metrics = train_step(self.ctx, lr, ent)        # the same three steps, one host wait
        self.global_step += self.steps_per_update                             # main.rs:988
        metrics["episodes"] = info.episodes
        metrics["mean_return"] = info.mean_return
        metrics["rng_word_pos"] = info.rng_word_pos
        return metrics

    def train_updates(self, n, phase_keys=()):
        """n iterations of train_update in one pipelined call (bppo_train_steps): the
        same results as n train_update(track_returns=False) calls, the GPU never idle
        between them.  -> (list of metrics dicts, {key: sum of last_kernel_ms(key)})."""
        lr = np.array([schedule_get(self.cfg["learning_rate"], self.global_step + k * self.steps_per_update)
                       for k in range(n)], np.float64)
        ent = np.array([schedule_get(self.cfg["entropy_coef"], self.global_step + k * self.steps_per_update)
                        for k in range(n)], np.float64)
        infos, ms = (L.RolloutInfo * max(n, 1))(), (L.UpdateMetrics * max(n, 1))()
        keys = (C.c_char_p * max(len(phase_keys), 1))(*[k.encode() for k in phase_keys])
        sums = np.zeros(max(len(phase_keys), 1), np.float32)
        self.ctx._chk(L.lib().bppo_train_steps(self.ctx.h, n, lr.ctypes.data, ent.ctypes.data, self.global_step,
                                                infos, ms, keys, len(phase_keys), sums.ctypes.data))
        out = []
        for k in range(n):
            d = _metrics_dict(ms[k])
            d["episodes"] = infos[k].episodes
            d["mean_return"] = infos[k].mean_return
            d["rng_word_pos"] = infos[k].rng_word_pos
            out.append(d)
        self.global_step += n * self.steps_per_update
        return out, {k: float(sums[i]) for i, k in enumerate(phase_keys)}

    def close(self):
        self.ctx.close()

/*
 * bppo.h — C-ABI of libbppo.so, the MI355X-native replacement for burn-ppo's
 * rollout -> GAE -> PPO-update hot path.
 *
 * Plain pointers and sizes only.  Host pointers are marked "host"; the few
 * entry points taking device pointers say so.  Every entry point returns a
 * bppo_status; the reference's panics (NaN log-probs ppo.rs:363-366, empty
 * action mask utils.rs:115-123) become status codes, never aborts.
 * A context is not thread-safe: one context per host thread per GPU.
 *
 * Reference surfaces each group replaces (bhansconnect/burn-ppo):
 *   bppo_create / bppo_vecenv_*   Environment + VecEnv       env.rs:24-173, 281-487
 *   bppo_params_* / bppo_forward  ActorCriticNetwork         network/mod.rs:53-189
 *   bppo_collect_rollouts         collect_rollouts           ppo.rs:213-500
 *   bppo_compute_gae              bootstrap + compute_gae[_multiplayer]
 *                                                            main.rs:877-947, ppo.rs:1069-1264
 *   bppo_ppo_update               ppo_update (+ Adam/clip)   ppo.rs:1661-2112, main.rs:264-268
 *   bppo_gae_device               compute_gae on caller device buffers  ppo.rs:1069-1124
 *   bppo_rng_*                    the shared &mut StdRng     main.rs:189, checkpoint.rs:390-426
 *   bppo_optimizer_*              Adam record (checkpoint)   checkpoint.rs:291-335
 *   bppo_obs_norm_* / ret_norm_*  ObsNormalizer / ReturnNormalizer  normalization.rs:12-260
 */
#ifndef BPPO_H
#define BPPO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    BPPO_OK = 0,
    BPPO_ERR_ARG = 1,          /* bad argument / shape mismatch */
    BPPO_ERR_NONFINITE = 2,    /* ppo.rs:363-366 "NaN/Inf in log probs" */
    BPPO_ERR_EMPTY_MASK = 3,   /* utils.rs:115-123 "Empty action mask" */
    BPPO_ERR_HIP = 4,          /* HIP runtime failure (message in bppo_last_error) */
    BPPO_ERR_COMM = 5,         /* all-reduce callback failed */
    BPPO_ERR_UNSUPPORTED = 6   /* configuration not implemented on the device path */
} bppo_status;

typedef enum { BPPO_ENV_CARTPOLE = 0, BPPO_ENV_CONNECT_FOUR = 1, BPPO_ENV_LIARS_DICE = 2, BPPO_ENV_SKULL = 3 } bppo_env_kind;
/* the widest player axis (Skull: MAX_PLAYERS = 6, envs/skull.rs:13) */
#define BPPO_MAX_PLAYERS 6

/* Mirrors the subset of config.rs:747-924 the hot path reads. */
typedef struct {
    int32_t env_kind;            /* bppo_env_kind */
    int32_t num_envs;            /* envs on THIS rank */
    int32_t num_steps;           /* T */
    int32_t hidden_size, num_hidden, relu;   /* activation == "relu" (else tanh) */
    int32_t ctde, critic_hidden_size, critic_num_hidden;
    int32_t num_epochs, num_minibatches;
    int32_t normalize_obs, normalize_returns, clip_value;
    double gamma, gae_lambda, clip_epsilon, value_coef, max_grad_norm, adam_epsilon;
    double target_kl;            /* < 0 : None */
    double return_clip;          /* ReturnNormalizer clip (config.rs:966-968) */
    double reward_shaping_coef;  /* Liar's Dice / Skull shaping (constant schedule; see below) */
    uint64_t seed;               /* main StdRng seed (main.rs:189) */
    uint64_t env_seed_base;      /* env i is seeded env_seed_base + i (main.rs:1964) */
    uint64_t rng_stream;         /* ChaCha stream id of the main RNG: 0 = reference; rank for W>1 */
    /* network_type = "cnn" (network/cnn.rs:24-50; Connect Four, OBSERVATION_SHAPE (6, 7, 2)):
     * num_conv_layers conv layers (stride 1, same padding, odd kernel_size, relu),
     * conv_channels per layer (the last repeated past the list, cnn.rs:84-90),
     * cnn_num_fc_layers FC layers of cnn_fc_hidden_size, then the heads */
    int32_t cnn, num_conv_layers, conv_channels[4], kernel_size, cnn_fc_hidden_size, cnn_num_fc_layers;
    /* normalize_values (config.rs:827-832, default false): PopArt value normalization
     * with value-head rescaling (normalization.rs:262-366, ppo.rs:1599-1653) */
    int32_t normalize_values;
    /* Skull: player_count (config.rs:767 PlayerCountMode, get_fixed_count, main.rs:1998);
     * 2..6, 0 = the default 4.  The player axis of the buffers stays NUM_PLAYERS = 6. */
    int32_t player_count;
    /* split_networks (config.rs:860, default false): separate actor and critic trunks.
     * MLP (mlp.rs:40-130, 139-206): a critic trunk of num_hidden x hidden_size on the
     * observation; flat parameters in Burn record order: layers (actor), critic_layers,
     * policy_head, value_head.  CNN (cnn.rs:116-135, 264-302): the critic's own conv stack
     * and FC layers; record order conv, fc, critic conv, critic fc, heads.  CTDE nets ignore
     * it (ctde.rs).  Any net: at most 16 layers in all (hidden / conv / FC layers + the two
     * heads), else bppo_create returns BPPO_ERR_UNSUPPORTED. */
    int32_t split_networks;
    /* shuffle_windows (not in the reference; for data-parallel ranks):
     * 0 = the reference: each epoch's shuffle (ppo.rs:1816) continues the main RNG where
     * the previous one ended.  1 = epoch e of an update draws from word S + e * (2 B + 2^20)
     * of the main stream (S = the update's first shuffle word, B = rows shuffled) and the
     * next rollout starts at S + epochs * (2 B + 2^20): every shuffle's start is known in
     * advance, so the host walks the epochs at once instead of speculating (a fraction of
     * the host CPU: what an 8-rank node can give each rank).  Self-play only. */
    int32_t shuffle_windows;
} bppo_config;

typedef struct {
    float total_reward[BPPO_MAX_PLAYERS];   /* players >= the env's NUM_PLAYERS: 0 */
    int32_t length;
    int32_t env_index;
    int32_t step;                /* rollout step t at which it ended */
    int32_t pad;
} bppo_episode;

typedef struct {
    int32_t episodes;            /* completed this rollout */
    float mean_return;           /* of player 0 */
    float mean_length;
    int32_t pad;
    uint64_t rng_word_pos;       /* main RNG position after the rollout */
} bppo_rollout_info;

/* UpdateMetrics, ppo.rs:1342-1369 */
typedef struct {
    float policy_loss, value_loss, entropy, entropy_scaled, approx_kl, clip_fraction;
    float explained_variance, total_loss, value_mean, returns_mean;
    float adv_mean_raw, adv_std_raw, adv_min_raw, adv_max_raw;
    float value_error_mean, value_error_std, value_error_max;
    float avg_valid_actions, entropy_valid_pct;
    int32_t num_updates, epochs_run;
    /* PopArt (ppo.rs:2061-2068, 1799-1804): NaN when the reference's Option is None */
    float value_norm_target_mean, value_norm_target_std, value_norm_rescale_mag;
} bppo_update_metrics;

typedef struct bppo_ctx bppo_ctx;

/* ---- lifecycle ---------------------------------------------------------- */
/* hip_stream may be NULL (the context creates its own).  Resets the VecEnv
 * (VecEnv::new semantics, env.rs:281-302) and zero-initialises parameters. */
bppo_status bppo_create(const bppo_config *cfg, int hip_device, void *hip_stream, bppo_ctx **out);
void bppo_destroy(bppo_ctx *ctx);
const char *bppo_last_error(const bppo_ctx *ctx);
const char *bppo_version(void);
/* sizeof the ABI structs as this library was built: a binding (Rust #[repr(C)], ctypes)
 * asserts its own struct sizes against these before the first bppo_create */
size_t bppo_config_size(void);
size_t bppo_update_metrics_size(void);
size_t bppo_episode_size(void);
size_t bppo_rollout_info_size(void);

/* ---- ActorCritic -------------------------------------------------------- */
/* flat parameters in Burn record order: per Linear W[in][out] then b[out];
 * MLP: hidden..., policy head, value head; CTDE: actor hidden..., policy head,
 * critic hidden..., value head (mlp.rs:47-62, ctde.rs:26-44). */
size_t bppo_num_params(const bppo_ctx *ctx);
bppo_status bppo_params_set(bppo_ctx *ctx, const float *host, size_t n);
bppo_status bppo_params_get(bppo_ctx *ctx, float *host, size_t n);
/* forward on B rows of host obs [B*obs_dim] (+ priv [B*priv_dim] for CTDE) */
bppo_status bppo_forward(bppo_ctx *ctx, const float *obs, const float *priv, int32_t B,
                         float *logits, float *values);

/* ---- main RNG (StdRng = ChaCha12; state = seed key + word position) ------- */
bppo_status bppo_rng_get(bppo_ctx *ctx, uint64_t *word_pos);
bppo_status bppo_rng_set(bppo_ctx *ctx, uint64_t word_pos);
/* checkpoint.rs:390-400 save_rng_state: fill_bytes from the main RNG (ceil(n/4)
 * words, little-endian; advances the position like the reference's draw) */
bppo_status bppo_rng_fill_bytes(bppo_ctx *ctx, uint8_t *dst, size_t n);
/* checkpoint.rs:405-426 load_rng_state: the main RNG becomes StdRng::from_seed(seed[32]) */
bppo_status bppo_rng_from_seed(bppo_ctx *ctx, const uint8_t *seed);
bppo_status bppo_rng_key_get(bppo_ctx *ctx, uint32_t key[8]);

/* ---- optimizer (Adam) state, for checkpoint.rs save/load_optimizer ------- */
/* m1, m2 flat like the parameters; steps[bppo_num_param_tensors] = Adam time per
 * parameter tensor (W then b of every Linear, record order) */
size_t bppo_num_param_tensors(const bppo_ctx *ctx);
bppo_status bppo_optimizer_get(bppo_ctx *ctx, float *m1, float *m2, int32_t *steps, size_t n);
bppo_status bppo_optimizer_set(bppo_ctx *ctx, const float *m1, const float *m2, const int32_t *steps, size_t n);

/* ---- VecEnv ------------------------------------------------------------- */
bppo_status bppo_vecenv_reset(bppo_ctx *ctx);  /* VecEnv::new: factory(i) + reset() */
/* current state: obs [N*obs_dim] raw, players [N], masks [N*A] (0/1), priv [N*priv]; any may be NULL */
bppo_status bppo_vecenv_observe(bppo_ctx *ctx, float *obs, int32_t *players, uint8_t *masks,
                                float *priv);
/* VecEnv::step (env.rs:400-487): actions [N]; rewards [N*P]; dones [N];
 * completed episodes in env order (up to cap), count in *n_eps */
bppo_status bppo_vecenv_step(bppo_ctx *ctx, const int32_t *actions, float *obs, float *rewards,
                             uint8_t *dones, bppo_episode *eps, int32_t cap, int32_t *n_eps);
/* VecEnv::set_step (env.rs:329-333, main.rs:727): the step schedulable env
 * parameters are evaluated at (Liar's Dice shaping, liars_dice.rs:535, 635) */
bppo_status bppo_vecenv_set_step(bppo_ctx *ctx, uint64_t global_step);
/* reward_shaping_coef: Schedule (config.rs:761-762, schedule.rs:29-78) as n
 * (value, step) milestones, sorted by step as Schedule::parse_cli / Deserialize
 * leave them; replaces the constant config.reward_shaping_coef.  n = 0: empty
 * schedule (0.0).  BPPO_ERR_ARG when the initial value is < 0 (config.rs:1514). */
bppo_status bppo_set_reward_shaping_schedule(bppo_ctx *ctx, const double *values, const uint64_t *steps,
                                             int32_t n);

/* ---- normalizers (f64 state, normalization.rs) ------------------------ */
bppo_status bppo_obs_norm_get(bppo_ctx *ctx, double *mean, double *m2, double *count);
bppo_status bppo_obs_norm_set(bppo_ctx *ctx, const double *mean, const double *m2, double count);
/* mvc = {mean, M2, count}; returns = per (env, player) rolling returns [N*P] */
bppo_status bppo_ret_norm_get(bppo_ctx *ctx, double *mvc, double *returns);
bppo_status bppo_ret_norm_set(bppo_ctx *ctx, const double *mvc, const double *returns);
/* PopArtNormalizer state {mean, M2, count, epsilon} (normalization.rs:275-284) */
bppo_status bppo_popart_get(bppo_ctx *ctx, double *state4);
bppo_status bppo_popart_set(bppo_ctx *ctx, const double *state4);

/* ---- the hot path ------------------------------------------------------- */
bppo_status bppo_collect_rollouts(bppo_ctx *ctx, bppo_rollout_info *info);
bppo_status bppo_rollout_episodes(bppo_ctx *ctx, bppo_episode *eps, int32_t cap, int32_t *n);
bppo_status bppo_compute_gae(bppo_ctx *ctx);
bppo_status bppo_ppo_update(bppo_ctx *ctx, double lr, double ent_coef, bppo_update_metrics *m);
/* the three calls above as one (main.rs:860-947 then ppo.rs:1661-2112): enqueued back to
 * back with one host wait at the end; the rollout's error statuses are reported after
 * the update (info may be NULL) */
bppo_status bppo_train_step(bppo_ctx *ctx, double lr, double ent_coef, bppo_rollout_info *info,
                            bppo_update_metrics *m);
/* n bppo_train_step iterations (main.rs:684-988 loop body, lr[k] / ent_coef[k], env step
 * global_step0 + k*T*N*world_size), software-pipelined: each iteration's rollout is enqueued behind the
 * previous update before the host waits for that update, so the GPU does not idle between
 * iterations.  Same results as n bppo_train_step calls; the stream is drained on return.
 * After an error status the next iteration's rollout may already have run (the RNG and
 * the envs are past it): it stays the context's next rollout, which bppo_collect_rollouts,
 * bppo_train_step and bppo_train_steps use instead of drawing another one (bppo_compute_gae
 * consumes it too).  A setter of the state it was drawn with (bppo_params_set,
 * bppo_rng_set / _from_seed, bppo_obs_norm_set, bppo_ret_norm_set, bppo_popart_set,
 * bppo_vecenv_reset) discards it; the next rollout is then drawn anew (bppo_optimizer_set
 * keeps it: a rollout does not read the Adam moments).
 * infos / ms: n entries each (may be NULL); phase_keys (bppo_last_kernel_ms names, nkeys of
 * them): per-key sums over the n iterations into phase_sums */
bppo_status bppo_train_steps(bppo_ctx *ctx, int32_t n, const double *lr, const double *ent_coef,
                             uint64_t global_step0, bppo_rollout_info *infos, bppo_update_metrics *ms,
                             const char *const *phase_keys, int32_t nkeys, float *phase_sums);

/* multi-GPU: called once per minibatch with the flat f32 gradient (+ metric
 * partials) in DEVICE memory, on the context's stream, before clip + Adam.
 * The callback must leave the SUM over ranks in place; the context divides
 * by world_size.  (RCCL all-reduce over xGMI, one per minibatch.) */
typedef int (*bppo_allreduce_fn)(float *device_buf, size_t n, void *user);
/* W = world_size > 1 semantics (the reference is single-process; DESIGN.md section 7,
 * pinned by tests/test_gpu_multirank.py against the oracle's W-rank update): each rank's
 * gradient is the mean over its own minibatch rows with its own advantage normalization;
 * the SUM over ranks is scaled by 1/W before clip + Adam, so all ranks take the same step.
 * The metric partials ride along, so the UpdateMetrics are those of all ranks' rows
 * together, except value_error_max, adv_*_raw and explained_variance, which stay per rank.
 * normalize_values (PopArt) at W > 1: every rank's running return statistics absorb ALL
 * ranks' returns, rank by rank in rank order (each rank's batch statistics travel through
 * the same callback as an exact all-gather), so the value-head rescale and the normalized
 * targets are identical on every rank; needs bppo_set_rank.  Opponent pools at W > 1: each
 * rank trains on its own learner rows, cut into num_minibatches of its own sizes; the
 * minibatch slots run in lockstep (one callback each), a rank without rows in a slot
 * contributing a zero gradient and zero metric partials (its value_error_max for the slot is
 * -inf).  The SUM is scaled by 1/W in every slot, empty contributions included, so a slot
 * that some ranks have no rows for takes a proportionally smaller step (the oracle's
 * or_trainers_update does the same). */
bppo_status bppo_set_allreduce(bppo_ctx *ctx, bppo_allreduce_fn fn, void *user, int32_t world_size);
/* this context's rank among the all-reduce's world_size ranks (0-based; unset by default):
 * the slot of its PopArt batch statistics in the W > 1 all-gather.  Required for
 * normalize_values at W > 1: an update without it returns BPPO_ERR_ARG, and so does one whose
 * gathered statistics show two contexts in one slot (a duplicated rank) */
bppo_status bppo_set_rank(bppo_ctx *ctx, int32_t rank);

/* stream-ordered variant: fn is called WITHOUT draining the stream, right after
 * the minibatch's gradient kernels are enqueued; it must enqueue the SUM
 * all-reduce of device_buf on the context's stream (bppo_get_stream) and
 * return.  Clip + Adam are enqueued after it, so the host never waits per
 * minibatch (replaces the ncclAllReduce-on-stream call a Rust host would make
 * in ppo.rs's update loop; the reference has no multi-GPU path). */
bppo_status bppo_set_allreduce_async(bppo_ctx *ctx, bppo_allreduce_fn fn, void *user, int32_t world_size);
bppo_status bppo_get_stream(bppo_ctx *ctx, void **hip_stream);

/* Opponent-pool training (multi-player envs): replaces collect_rollouts_with_opponents
 * (ppo.rs:537-1063) and the learner-row filter of ppo_update (ppo.rs:165-180,
 * 1696-1753).  The host keeps the pool (OpponentPool, opponent_pool.rs: checkpoint
 * loading, win-rate sampling, rotation) and hands over the loaded models:
 *   n_models (<= 15) parameter vectors of the learner's architecture, packed
 *   [n_models][n_params]; per model an optional observation normalizer
 *   (norm_mean/norm_m2 [n_models][obs_dim], norm_count [n_models]; count < 2 or
 *   NULL arrays = none);
 *   envs [0, num_opponent_envs) play against them (main.rs:621-637), with seat
 *   state learner_pos [num_opponent_envs] and pos_to_opp [num_opponent_envs][P]
 *   (model index per seat, -1 on the learner's seat) (EnvState, opponent_pool.rs:80-124);
 *   current_opp [P - 1]: OpponentPool::sample_all_slots, the models a finished game
 *   is given before its seats are reshuffled from the main RNG.  P here is the
 *   seated player count (main.rs:552: Skull's player_count, else NUM_PLAYERS).
 * Opponent batches sample in ascending model index (the reference iterates a
 * HashMap, whose order is unspecified).  num_opponent_envs = 0 switches it off.
 * Buffer "valid" holds the learner-turn flags of the last rollout; ppo_update
 * trains on those rows only. */
bppo_status bppo_opponents_set(bppo_ctx *ctx, int32_t n_models, const float *params, const double *norm_mean,
                               const double *norm_m2, const double *norm_count, int32_t num_opponent_envs,
                               const int32_t *learner_pos, const int32_t *pos_to_opp, const int32_t *current_opp);
/* the seat state after the last rollout's reshuffles */
bppo_status bppo_opponents_get_envs(bppo_ctx *ctx, int32_t *learner_pos, int32_t *pos_to_opp);

/* parity hooks: export / import a RolloutBuffer field.  names: "obs", "priv",
 * "actions" (i32), "rewards", "dones", "values", "log_probs", "advantages",
 * "returns", "players" (i32), "all_rewards", "masks", "last_v_pp", "perm" (u32,
 * last epoch's shuffled indices), "grad" (the last minibatch's gradient); export only,
 * multi-player nets: "hidden:<l>" = FC hidden layer l's activations of the last forward
 * ([rows_max][width] f32, rows_max = max(num_envs, ceil(T N / num_minibatches)); the last
 * minibatch's rows in "perm" order -- the device's ReLU decisions for
 * tests/test_gpu_gemm_split.py) */
/* the last update's per-minibatch metric rows in run order (parity diagnosis: which
 * minibatch's statistics first leave the bar): row k = the minibatch's sums
 * [policy_loss, 2*value_loss, entropy, approx_kl, clip_fraction, value, return, |v-R|,
 * (v-R)^2, max |v-R|, rows, ...] then 4 advantage statistics; returns the row count,
 * copies up to max_rows rows of *row_width floats into out (may be NULL) */
int32_t bppo_minibatch_rows(bppo_ctx *ctx, float *out, int32_t max_rows, int32_t *row_width);
bppo_status bppo_buffer_get(bppo_ctx *ctx, const char *name, void *host, size_t bytes);
bppo_status bppo_buffer_set(bppo_ctx *ctx, const char *name, const void *host, size_t bytes);

/* ---- standalone device kernels on caller-owned DEVICE buffers ------------ */
/* compute_gae (ppo.rs:1069-1124) on [T,N] device arrays; stream may be NULL */
bppo_status bppo_gae_device(const float *rewards, const float *dones, const float *values,
                            const float *last_values, int32_t T, int32_t N, float gamma,
                            float lambda, float *advantages, float *returns, void *hip_stream);
/* the same, plus the [advantage, return] pair of every row, pairs [T*N][2] floats (row
 * t*N+e), as the update path writes them for its minibatch gathers;
 * BPPO_ERR_UNSUPPORTED unless N % 4 == 0, T <= 128 and the arrays are 16-byte aligned */
bppo_status bppo_gae_rows_device(const float *rewards, const float *dones, const float *values,
                                 const float *last_values, int32_t T, int32_t N, float gamma,
                                 float lambda, float *advantages, float *returns, float *pairs,
                                 void *hip_stream);
/* compute_gae_multiplayer (ppo.rs:1140-1264): all_rewards [T,N,P], players [T,N] i32,
 * last_v_pp [N,P] */
bppo_status bppo_gae_mp_device(const float *all_rewards, const int32_t *players,
                               const float *dones, const float *values, const float *last_v_pp,
                               int32_t T, int32_t N, int32_t P, float gamma, float lambda,
                               float *advantages, float *returns, void *hip_stream);

/* UpdateMetrics.explained_variance (ppo.rs:1268-1294): mode 0 (default) = f64 sums on the
 * device (within 1e-6 of the exact value; the reference's f32 sums drift ~1e-3 at 10^6
 * rows); mode 1 = the reference's own arithmetic, bit for bit: four sequential f32 sums
 * over the buffer, on a host thread from device->host copies made beside the update
 * (it waits for them at the update's end: ~10 ms of one CPU per 8.4 M rows) */
bppo_status bppo_set_explained_variance_mode(bppo_ctx *ctx, int32_t mode);

/* which minibatch kernels run (a parity / A-B hook).  CartPole's 2x64 relu MLP (CfgB):
 * mode 0 (default) runs the update's first minibatch on the exact f32 kernel (it runs with
 * the rollout's parameters, so the ratio is exactly 1 and the forward equals the rollout's
 * bit for bit) and every later one on the f32-accurate split-bf16 kernel; 1 the exact kernel
 * for every minibatch; 2 the split kernel for every minibatch, the first included (its
 * gradient from the rollout's parameters can then be compared with the oracle's,
 * tests/test_gpu_split_kernel.py).  The GEMM path (Connect Four, Liar's Dice, Skull, other
 * nets; wide_api.hip wide_minibatch):
 *   mode 0 (default), minibatches below 32,768 rows (WIDE_SPLIT_MIN_ROWS): the exact forward
 *     and input-gradient f32 chains, weight gradients summed in f64 on the f64 MFMA;
 *     from 32,768 rows, MLP / CTDE nets: the update's first minibatch keeps the exact forward
 *     (ratio exactly 1) and runs its backward (input and weight gradients) on the split-bf16
 *     contraction, every later minibatch runs all its GEMMs split; CNN nets: the exact
 *     chains with f32 split-K weight gradients;
 *   mode 1: the exact chains, weight gradients in f64 row by row in order (the oracle's
 *     arithmetic exactly; a latency-bound parity mode);
 *   mode 2: MLP / CTDE nets run every minibatch's forward and backward on the split-bf16
 *     contraction (the first included); CNN nets the exact chains with f32 split-K weight
 *     gradients. */
bppo_status bppo_set_minibatch_kernel(bppo_ctx *ctx, int32_t mode);

/* parity hook: while host != NULL, every bppo_ppo_update copies the parameters it runs each
 * minibatch with (the first max_minibatches in run order) to host[k * num_params], so each
 * minibatch's statistics can be recomputed from the device's own parameters at any size
 * (tests/test_gpu_fullsize.py); "perm_ep:<e>" (bppo_buffer_get) is epoch e's permutation */
bppo_status bppo_debug_record_params(bppo_ctx *ctx, float *host, int32_t max_minibatches);

/* device timing of the last call of each phase kernel (ms), for bench.py's roofline */
bppo_status bppo_last_kernel_ms(bppo_ctx *ctx, const char *kernel, float *ms);

/* libm parity hook: which 0 = logf, 1 = sinf, 2 = cosf, 3 = gumbel(-ln(-ln u)), 4 = expf, 5 = tanhf;
 * device = 0 runs the host build of the same source, 1 runs the HIP kernel */
bppo_status bppo_debug_libm(int32_t which, int32_t device, const float *x, float *y, size_t n);

/* shuffle parity hooks (ppo.rs:1816, rand 0.8.5 SliceRandom::shuffle on StdRng):
 * the host draw chain alone — J[i] = gen_range(0..i+1) for i = n-1..1 from word
 * position word_pos of StdRng(seed) stream `stream`, *end_pos = position after —
 * and the device Fisher-Yates permutation of 0..n-1 for given swap targets J */
bppo_status bppo_debug_shuffle_chain(uint64_t seed, uint64_t stream, uint64_t word_pos, uint32_t n,
                                     uint32_t *J, uint64_t *end_pos);
bppo_status bppo_debug_fisher_yates(int32_t device, const uint32_t *J, uint32_t n, uint32_t *perm);
/* host only: two draw chains of n (from word positions pos_a, pos_b) walked together by
 * the interleaved two-chain walker the shuffle_windows engine uses, over words handed
 * over in pieces ending at multiples of `piece` words; *end_a / *end_b = the positions
 * after each shuffle (must equal bppo_debug_shuffle_chain's) */
bppo_status bppo_debug_chain_walk2(uint64_t seed, uint64_t stream, uint64_t pos_a, uint64_t pos_b, uint32_t n,
                                   uint32_t piece, uint64_t *end_a, uint64_t *end_b);
/* the whole shuffle engine (GPU-made ChaCha words, speculative walks, J rebuilt on
 * the GPU) for `jobs` updates of `epochs` shuffles of n: the first from word
 * position start, each next update `gap` words after the previous one's last
 * shuffle.  J [jobs][epochs][n], end word positions [jobs][epochs], met = checkpoints
 * walked before meeting a speculative walk (-1 = none; may be NULL).  Must equal
 * chained shuffle_chain calls.  windows = 1: the shuffle_windows layout (epoch e of
 * an update from its start + e * (2 n + 2^20), the next update gap words after its
 * start + epochs * (2 n + 2^20)): must equal shuffle_chain calls from those starts. */
bppo_status bppo_debug_shuffle_engine(uint64_t seed, uint64_t stream, uint64_t start, uint32_t n, int32_t epochs,
                                      uint64_t gap, int32_t jobs, int32_t windows, uint32_t *J, uint64_t *ends,
                                      int32_t *met);

/* sampling parity hook: apply_action_mask + sample_categorical + log_prob_categorical
 * (utils.rs:10-45, 96-135) for B host rows of A logits (A in {2, 7, 49}) on the device
 * sampler; Gumbel words from StdRng(seed) stream `stream` at word_pos, row-major;
 * masks [B*A] 0/1 or NULL.  Returns BPPO_ERR_EMPTY_MASK for a row with no valid
 * action (the reference panics, utils.rs:115-123) and BPPO_ERR_NONFINITE for a
 * non-finite log-prob (ppo.rs:363-366). */
bppo_status bppo_debug_sample(int32_t A, int32_t B, const float *logits, const uint8_t *masks, uint64_t seed,
                              uint64_t stream, uint64_t word_pos, int32_t *actions, float *log_probs);

/* GEMM engine parity hook (host buffers).  mode 0: out[M][N] = act(A[M][K] B[K][N] + bias[N])
 * with matrixmultiply's KC=256 fma-chain order (Burn Linear forward, mlp.rs:140-206);
 * (act: 0 none, 1 relu, 2 tanh); mode 1: out[M][N] = (A[M][K] B[N][K]^T) * act'(H) with H = bias_or_H
 * the layer output (may be NULL): act 2 -> (1 - H^2), otherwise [H > 0];
 * mode 2: out[M][N] = A[K][M]^T B[K][N] (weight gradient), out2[N] = column sums of B */
bppo_status bppo_debug_gemm(int32_t mode, int32_t M, int32_t N, int32_t K, const float *A, const float *B,
                            const float *bias_or_H, int32_t act, float *out, float *out2);

#ifdef __cplusplus
}
#endif
#endif

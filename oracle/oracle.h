/*
 * oracle.h — CPU restatement of burn-ppo's rollout -> GAE -> PPO-update hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the timed
 * CPU baseline ("kind": "port").  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product (libbppo.so) never
 * links, loads or calls anything under oracle/.
 *
 * Every function cites the reference file:line it restates
 * (/root/reference = bhansconnect/burn-ppo).  Third-party arithmetic that is
 * not vendored in the reference (rand 0.8.5, rand_core 0.6.4, rand_chacha
 * 0.3.1, burn 0.20 ndarray/autodiff/optim, matrixmultiply 0.3.10) is restated
 * from the published algorithms and marked "restated, verify" where nothing in
 * the reference's own tests pins it.  Transcendentals (logf, sinf, cosf, expf)
 * come from the platform glibc libm, exactly as the reference's Rust code gets
 * them (f32::ln / sin / cos / exp lower to libm calls).
 *
 * Compiled with -ffp-contract=off: every fused multiply-add below is an
 * explicit fmaf(), mirroring Rust's `mul_add` call sites; Rust never contracts
 * `a*b+c` by itself.
 */
#ifndef BPPO_ORACLE_H
#define BPPO_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ RNG -- */
/* rand 0.8.5 StdRng = rand_chacha 0.3.1 ChaCha12Rng behind rand_core 0.6.4
 * BlockRng.  The stream is the plain ChaCha keystream (64-bit block counter in
 * state words 12-13, stream id 0 in 14-15) read as little-endian u32 words, so
 * the whole generator state is (key, word position). */
typedef struct {
    uint32_t key[8];
    uint64_t stream;    /* nonce words 14-15; 0 for StdRng */
    uint64_t word_pos;  /* index of the next u32 to hand out */
    uint64_t cached_block;
    uint32_t block[16];
    int rounds;         /* 12 for StdRng; 20 only for the RFC/OpenSSL KAT */
} or_rng;

void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream,
                     int rounds, uint32_t out[16]);
void or_rng_seed_u64(or_rng *r, uint64_t seed);
void or_rng_from_key(or_rng *r, const uint32_t key[8], int rounds);
uint32_t or_rng_next_u32(or_rng *r);
uint64_t or_rng_next_u64(or_rng *r);
void or_rng_fill_bytes(or_rng *r, uint8_t *dst, size_t n);
float or_gen_range_f32(or_rng *r, float low, float high);
uint32_t or_gen_range_u32(or_rng *r, uint32_t low, uint32_t high);     /* [low, high) */
uint8_t or_gen_range_u8_incl(or_rng *r, uint8_t low, uint8_t high);    /* [low, high] */
uint64_t or_gen_range_u64(or_rng *r, uint64_t low, uint64_t high);     /* [low, high), usize */
void or_shuffle_u32(or_rng *r, uint32_t *v, size_t n);
void or_shuffle_targets(or_rng *r, uint32_t *J, size_t n);
void or_apply_swaps(const uint32_t *J, uint32_t *v, size_t n);
/* helpers for ctypes: run n draws and return them */
void or_rng_words(uint64_t seed, uint64_t skip, uint32_t *out, size_t n);
void or_rng_words_key(const uint32_t key[8], int rounds, uint64_t skip, uint32_t *out, size_t n);
void or_rng_seed_key(uint64_t seed, uint32_t key_out[8]);

/* ----------------------------------------------------------------- envs -- */
enum { OR_ENV_CARTPOLE = 0, OR_ENV_CONNECT_FOUR = 1, OR_ENV_LIARS_DICE = 2, OR_ENV_SKULL = 3 };

#define OR_CP_OBS 5
#define OR_CP_ACT 2
typedef struct {
    float x, x_dot, theta, theta_dot;
    int32_t steps;
    or_rng rng;
} or_cartpole;
void or_cartpole_new(or_cartpole *e, uint64_t seed);
void or_cartpole_reset(or_cartpole *e, float *obs);
void or_cartpole_step(or_cartpole *e, int32_t action, float *obs, float *reward, int *done);
void or_cartpole_get_obs(const or_cartpole *e, float *obs);

#define OR_C4_OBS 86
#define OR_C4_ACT 7
typedef struct {
    int8_t board[6][7]; /* 0 empty, 1 = Player1, 2 = Player2 */
    int8_t current;     /* 1 or 2 */
    int8_t game_over;
    int8_t winner;      /* 0 none/draw, 1, 2 */
} or_connect_four;
void or_c4_new(or_connect_four *e);
void or_c4_reset(or_connect_four *e, float *obs);
void or_c4_step(or_connect_four *e, int32_t action, float *obs, float rewards[2], int *done);
void or_c4_get_obs(const or_connect_four *e, float *obs);
void or_c4_mask(const or_connect_four *e, uint8_t mask[7]);
int or_c4_current_player(const or_connect_four *e);

#define OR_LD_PLAYERS 4
#define OR_LD_DICE 2
#define OR_LD_OBS 270
#define OR_LD_ACT 49
#define OR_LD_PRIV 120
#define OR_LD_HIST 16
typedef struct {
    uint8_t dice[OR_LD_PLAYERS][OR_LD_DICE];
    uint8_t num_dice[OR_LD_PLAYERS];
    uint8_t current;
    int8_t has_bid;
    uint8_t bid_qty, bid_face;
    int8_t last_bidder;           /* -1 none */
    int32_t bid_count;            /* bids this round */
    uint8_t hist_player[OR_LD_HIST], hist_qty[OR_LD_HIST], hist_face[OR_LD_HIST];
    int32_t hist_len;             /* valid entries (<= 16), newest last */
    int8_t elim_order[OR_LD_PLAYERS];
    int32_t num_elim;
    int8_t game_over;
    uint64_t global_step;
    or_rng rng;
} or_liars_dice;
void or_ld_new(or_liars_dice *e, uint64_t seed);
void or_ld_reset(or_liars_dice *e, float *obs);
void or_ld_step(or_liars_dice *e, int32_t action, float shaping, float *obs, float rewards[4], int *done);
void or_ld_get_obs(const or_liars_dice *e, float *obs);
void or_ld_mask(const or_liars_dice *e, uint8_t mask[49]);
void or_ld_priv(const or_liars_dice *e, float *priv);
int or_ld_current_player(const or_liars_dice *e);

#define OR_SK_MAXP 6
#define OR_SK_CARDS 4
#define OR_SK_ROSES 3
#define OR_SK_MAXBID 24
#define OR_SK_WINS 2
#define OR_SK_OBS 135
#define OR_SK_ACT 33
#define OR_SK_PRIV 200
#define OR_SK_HIST 8
typedef struct {
    int32_t n;                                  /* num_players, 2..6 */
    uint8_t has_trap[OR_SK_MAXP], rose_count[OR_SK_MAXP], wins[OR_SK_MAXP];
    uint8_t stack_len[OR_SK_MAXP], stack[OR_SK_MAXP][OR_SK_CARDS];   /* 1 = skull, bottom first */
    uint8_t passed[OR_SK_MAXP], revealed[OR_SK_MAXP];
    int32_t phase, current, round_starter, current_bid, current_bidder;   /* bidder -1: None */
    int32_t hist_len;
    uint8_t hist_player[OR_SK_HIST], hist_bid[OR_SK_HIST];              /* bid 0 = pass */
    int32_t roses_found, must_reveal_own, last_skull_owner;
    int8_t elim_order[OR_SK_MAXP];
    int32_t num_elim, game_over, winner;        /* winner -1: None */
    or_rng rng;
} or_skull;
void or_skull_new(or_skull *e, int num_players, uint64_t seed);
void or_skull_reset(or_skull *e, float *obs);
void or_skull_step(or_skull *e, int32_t action, float shaping, float *obs, float rewards[6], int *done,
                   int *invalid);
void or_skull_get_obs(const or_skull *e, float *obs);
void or_skull_mask(const or_skull *e, uint8_t mask[33]);
void or_skull_priv(const or_skull *e, float *priv);
int or_skull_current_player(const or_skull *e);
void or_skull_outcome(const or_skull *e, int32_t out[6]);
void or_skull_placements(const or_skull *e, int32_t out[6]);
void or_skull_final_rewards(const or_skull *e, float r[6]);

/* -------------------------------------------------------------- VecEnv --- */
typedef struct or_vecenv or_vecenv;
or_vecenv *or_vecenv_new(int env_kind, int num_envs, uint64_t seed_base);
/* Skull: player_count (config.rs:767, Fixed count; 0 = the default 4) */
or_vecenv *or_vecenv_new_np(int env_kind, int num_envs, uint64_t seed_base, int player_count);
int or_vecenv_invalid(const or_vecenv *v);   /* an action outside the mask was stepped (panic) */
void or_vecenv_free(or_vecenv *v);
int or_vecenv_obs_dim(const or_vecenv *v);
int or_vecenv_act_dim(const or_vecenv *v);
int or_vecenv_players(const or_vecenv *v);
int or_vecenv_priv_dim(const or_vecenv *v);
void or_vecenv_set_shaping(or_vecenv *v, float coef);
double or_schedule_get(const double *values, const uint64_t *steps, int n, uint64_t step);
void or_vecenv_get_obs(const or_vecenv *v, float *obs);
void or_vecenv_get_players(const or_vecenv *v, int32_t *players);
int or_vecenv_get_masks(const or_vecenv *v, uint8_t *masks);  /* returns 0 if env has no masks */
void or_vecenv_get_priv(const or_vecenv *v, float *priv);
/* step: rewards [N*P]; dones [N]; episode stats appended (up to cap) */
typedef struct {
    float total_rewards[6];
    int32_t length;
    int32_t env_index;
} or_episode;
int or_vecenv_step(or_vecenv *v, const int32_t *actions, float *obs_out, float *rewards,
                   uint8_t *dones, or_episode *eps, int eps_cap);
void *or_vecenv_env_ptr(or_vecenv *v, int i);

/* ---------------------------------------------------------- normalizers -- */
typedef struct {
    int dim;
    double *mean, *var;   /* var is the Welford M2 accumulator */
    double count;
    float clip;
} or_obs_norm;
void or_obs_norm_init(or_obs_norm *n, int dim, float clip);
void or_obs_norm_free(or_obs_norm *n);
void or_obs_norm_update_batch(or_obs_norm *n, const float *obs, size_t rows);
void or_obs_norm_normalize_batch(const or_obs_norm *n, float *obs, size_t rows);

typedef struct {
    int num_envs, num_players;
    double *returns;      /* [num_envs * num_players] */
    double var, mean, count, gamma, epsilon;
    float clip;
} or_ret_norm;
void or_ret_norm_init(or_ret_norm *n, int num_envs, int num_players, double gamma, float clip);
void or_ret_norm_free(or_ret_norm *n);
void or_ret_norm_update_return(or_ret_norm *n, int env, int player, float r);
void or_ret_norm_update_variance(or_ret_norm *n, int env, int player);
float or_ret_norm_normalize(const or_ret_norm *n, float r);
void or_ret_norm_reset_player(or_ret_norm *n, int env, int player);
void or_ret_norm_reset_env(or_ret_norm *n, int env);
void or_ret_norm_update_and_normalize_all(or_ret_norm *n, float *rewards, const uint8_t *dones);

/* ----------------------------------------------------------- networks ---- */
/* Flat parameter layout = Burn module record order: for every Linear, W[in][out]
 * (row-major) then b[out].  MLP: hidden layers, policy head, value head.  CTDE:
 * actor hidden, policy head, critic hidden, value head. */
typedef struct {
    int ctde;
    int obs_dim, priv_dim, act_dim;
    int relu;
    int n_actor;              /* number of actor hidden layers */
    int actor_width;
    int n_critic;             /* CTDE critic hidden layers (0 for MLP) */
    int critic_width;
    size_t n_params;
    /* CNN (network/cnn.rs; Connect Four OBSERVATION_SHAPE (H, W, C) = (6, 7, 2)):
     * n_conv conv layers of conv_ch[l] channels, odd kernel ksize, stride 1, same
     * padding, relu; then n_actor FC layers of actor_width, then the heads */
    int cnn, n_conv, conv_ch[4], ksize, H, W, C;
    /* split_networks (mlp.rs:40-130, 139-206): a critic trunk of n_critic x critic_width on
     * obs alone (priv_dim 0), structured like CTDE; record order: actor hidden, critic
     * hidden, policy head, value head */
    int split;
} or_net_desc;
size_t or_net_num_params(const or_net_desc *d);
void or_net_value_head(const or_net_desc *d, size_t *w, size_t *b, int *in);   /* value head W offset, b offset, in */
/* forward for B rows; logits [B*A], values [B] */
void or_net_forward(const or_net_desc *d, const float *params, const float *obs,
                    const float *priv, size_t B, float *logits, float *values);
/* MLP forward/backward row parallelism (OpenMP); off = single-threaded MLP */
void or_set_mlp_parallel(int on);
/* one linear layer y = x W + b with the matrixmultiply summation order */
void or_linear(const float *x, const float *W, const float *b, size_t B, int in, int out,
               int relu, float *y);
/* test hook: ReLU decisions of FC layer l's backward taken from masks[l] (u8 [mb][out]),
 * NULL entries / NULL masks = the forward's own (y > 0) */
void or_set_relu_masks(const uint8_t *const *masks, int n);
/* the input gradient of one Linear as the backward computes it (test hook) */
void or_linear_dx(const float *dz, const float *W, size_t B, int in, int out, float *dx);

/* ------------------------------------------------------------- policy ---- */
void or_sample_categorical(or_rng *rng, const float *logits, size_t B, int A, int32_t *actions);
long or_apply_action_mask(float *logits, const uint8_t *mask, size_t B, int A);   /* -1 ok, else empty row */
void or_log_softmax_row(const float *x, int A, float *out);
float or_log_prob(const float *logits, int A, int32_t a);
float or_entropy(const float *logits, int A);

/* ---------------------------------------------------------------- GAE ---- */
void or_compute_gae(const float *rewards, const float *dones, const float *values,
                    const float *last_values, int T, int N, float gamma, float lambda,
                    float *adv, float *ret);
void or_compute_gae_mp(const float *all_rewards, const int32_t *players, const float *dones,
                       const float *values, const float *last_v_pp, int T, int N, int P,
                       float gamma, float lambda, float *adv, float *ret);
float or_explained_variance(const float *values, const float *returns, size_t n);

/* ---------------------------------------------------------- PPO update --- */
typedef struct {
    int num_epochs, num_minibatches;
    float clip_epsilon;      /* as f64 in the reference; bounds cast to f32 */
    double clip_epsilon_d;
    double value_coef;
    double max_grad_norm;
    float adam_epsilon;
    double target_kl;        /* < 0 means None */
    int clip_value;
} or_ppo_cfg;

typedef struct {
    float *m1, *m2;          /* Adam moments, flat like params */
    int32_t *time;           /* per-tensor step counter */
    int has_state;
} or_adam;

typedef struct {
    float policy_loss, value_loss, entropy, entropy_scaled, approx_kl, clip_fraction;
    float explained_variance, total_loss, value_mean, returns_mean;
    float adv_mean_raw, adv_std_raw, adv_min_raw, adv_max_raw;
    float value_error_mean, value_error_std, value_error_max;
    float avg_valid_actions, entropy_valid_pct;
    int32_t num_updates;
    int32_t epochs_run;
    float value_norm_target_mean, value_norm_target_std, value_norm_rescale_mag;   /* NaN = None */
} or_update_metrics;

/* PopArtNormalizer (normalization.rs:262-366) */
typedef struct { double mean, var, count, epsilon; } or_popart;
void or_popart_init(or_popart *p);
double or_popart_std(const or_popart *p);
void or_popart_update(or_popart *p, const float *returns, size_t n, double *old_mean, double *old_std);
void or_popart_normalize(const or_popart *p, const float *x, size_t n, float *out);
void or_popart_denormalize(const or_popart *p, float *v, size_t n);

/* per-minibatch loss/grad: grads [n_params]; returns loss. Used by the update and by tests */
typedef struct {
    float loss, policy_loss, value_loss, entropy, approx_kl, clip_fraction;
    float value_mean, returns_mean, value_error_mean, value_error_std, value_error_max;
    float avg_valid_actions, entropy_valid_pct;
} or_mb_stats;
void or_minibatch_loss_grad(const or_net_desc *d, const float *params, size_t mb,
                            const float *obs, const float *priv, const int32_t *actions,
                            const float *old_logp, const float *adv_norm, const float *returns,
                            const float *old_values, const float *masks, const or_ppo_cfg *c,
                            double ent_coef, float *grads, or_mb_stats *st);
void or_normalize_advantages(const float *adv, size_t n, float *out, float *mean, float *std,
                             float *mn, float *mx);
void or_adam_init(or_adam *a, const or_net_desc *d);
void or_adam_free(or_adam *a);
void or_adam_step(const or_net_desc *d, or_adam *a, float *params, float *grads, double lr,
                  float max_grad_norm, float eps);

/* ---------------------------------------------------------- trainer ------ */
typedef struct or_trainer or_trainer;
#define OR_MB_LOG_MAX 256
/* the last update's per-minibatch statistics in run order (the metrics of all ranks'
 * rows at W > 1); returns how many minibatches ran, copies up to max */
int or_trainer_mb_log(const or_trainer *t, or_mb_stats *out, int max);
typedef struct {
    int env_kind;
    int num_envs, num_steps;
    int hidden, num_hidden, relu;
    int ctde, critic_hidden, critic_num_hidden;
    int normalize_obs, normalize_returns;
    float return_clip;
    double gamma, gae_lambda, lr, ent_coef;
    double reward_shaping;
    or_ppo_cfg ppo;
    uint64_t seed;
    int threads;             /* env-step threads (rayon equivalent); 0 = all */
    int cnn, num_conv, conv_ch[4], ksize;   /* network_type = "cnn" (Connect Four) */
    int normalize_values;    /* PopArt (config.rs:827-832) */
    int player_count;        /* Skull (config.rs:767), 0 = 4 */
    int split_networks;      /* config.rs:860 (MLP nets) */
    /* data-parallel rank r of W (libbppo's W > 1 semantics): envs are
     * seeded seed + env_seed_offset + i (offset = r * num_envs) and the main RNG is
     * StdRng::seed_from_u64(seed) on ChaCha stream rng_stream (= r).  Zero: the reference. */
    uint64_t env_seed_offset;
    uint64_t rng_stream;
    /* shuffle_windows (libbppo's bppo_config field, not the reference): epoch e of an
     * update shuffles from word S + e * OR_SHUFFLE_WINDOW(B) (S = the update's first
     * shuffle word) and the update leaves the RNG at S + epochs * OR_SHUFFLE_WINDOW(B) */
    int shuffle_windows;
} or_train_cfg;
#define OR_SHUFFLE_WINDOW(B) (2 * (uint64_t)(B) + ((uint64_t)1 << 20))
or_trainer *or_trainer_new(const or_train_cfg *c, const float *init_params);
void or_trainer_free(or_trainer *t);
size_t or_trainer_num_params(const or_trainer *t);
void or_trainer_get_params(const or_trainer *t, float *out);
void or_trainer_set_params(or_trainer *t, const float *in);
uint64_t or_trainer_rng_pos(const or_trainer *t);
void or_trainer_set_rng(or_trainer *t, const uint32_t key[8], uint64_t pos);
/* main.rs:720-727: reward_shaping_coef.get(global_step) for the next rollout */
void or_trainer_set_shaping(or_trainer *t, float coef);
void or_trainer_set_adam(or_trainer *t, const float *m1, const float *m2, const int32_t *steps, int n_tensors);
void or_trainer_get_adam(const or_trainer *t, float *m1, float *m2, int32_t *steps, int n_tensors);
void or_trainer_popart(or_trainer *t, double *get4, const double *set4);
void or_trainer_set_norms(or_trainer *t, const double *mean, const double *m2, double count, const double *mvc,
                          const double *returns);
/* phases of one update, so tests can compare buffers phase by phase */
int or_trainer_collect(or_trainer *t);                     /* returns episodes completed (all, not only those stored) */
void or_trainer_gae(or_trainer *t);
void or_trainer_update(or_trainer *t, or_update_metrics *m);
/* the same update for W data-parallel ranks in lockstep (gradients summed over the
 * ranks then scaled by 1/W before clip + Adam; ms[W]); W = 1 is or_trainer_update */
void or_trainers_update(or_trainer **ts, int W, or_update_metrics *ms);
/* buffer export: name in {"obs","actions","rewards","dones","values","log_probs",
   "advantages","returns","players","all_rewards","masks","priv","last_v_pp"} */
size_t or_trainer_buffer(const or_trainer *t, const char *name, void *out, size_t bytes);
int or_trainer_set_buffer(or_trainer *t, const char *name, const void *src, size_t bytes);  /* values, advantages, returns, rewards, log_probs */
void or_trainer_obs_norm_state(const or_trainer *t, double *mean, double *var, double *count);
void or_trainer_ret_norm_state(const or_trainer *t, double *mean_var_count3, double *returns);
int or_trainer_episodes(const or_trainer *t, or_episode *out, int cap);  /* last collect */
/* Opponent-pool training (ppo.rs:537-1063, main.rs:621-651): K opponent
 * parameter sets of the learner's architecture, each with an optional
 * observation normalizer (count < 2: none); envs [0, n_opp) are opponent envs
 * with seat state learner_pos [n_opp], pos_to_opp [n_opp * P] (model index, -1
 * for the learner's seat); current_opp [P - 1] is OpponentPool::sample_all_slots
 * (the models a finished game is reassigned).  Opponent batches run in
 * ascending model index (the reference iterates a HashMap).  n_opp = 0 turns
 * it off.  The update then trains on the learner rows only (buffer "valid"). */
void or_trainer_set_opponents(or_trainer *t, int K, const float *params, const double *mean,
                              const double *m2, const double *count, int n_opp, const int32_t *learner_pos,
                              const int32_t *pos_to_opp, const int32_t *current_opp);
void or_trainer_opponent_envs(const or_trainer *t, int32_t *learner_pos, int32_t *pos_to_opp);
/* EnvState::shuffle_positions (opponent_pool.rs:107-123) on caller state */
void or_shuffle_positions(or_rng *r, int P, const int32_t *assigned, int32_t *learner_pos, int32_t *pos_to_opp);
double or_trainer_last_phase_seconds(const or_trainer *t, int phase);   /* 0 rollout, 1 gae, 2 update */

#ifdef __cplusplus
}
#endif
#endif

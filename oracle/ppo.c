/*
 * ppo.c — GAE (ppo.rs:1069-1264), explained variance (ppo.rs:1268-1294) and a
 * trainer that restates one update of run_training (main.rs:684-988):
 * collect_rollouts (ppo.rs:213-500) -> bootstrap + GAE (main.rs:877-947) ->
 * ppo_update (ppo.rs:1661-2112).  TEST INFRASTRUCTURE ONLY.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include "oracle.h"

/* ppo.rs:1094-1123 — fmaf exactly where the reference calls mul_add. */
void or_compute_gae(const float *r, const float *d, const float *v, const float *last_v, int T,
                    int N, float gamma, float lambda, float *adv, float *ret) {
    float *last = calloc((size_t)N, sizeof(float));
    for (int t = T - 1; t >= 0; t--)
        for (int e = 0; e < N; e++) {
            size_t i = (size_t)t * N + e;
            float nv = t == T - 1 ? last_v[e] : v[i + N];
            float delta = fmaf(gamma * nv, 1.0f - d[i], r[i]) - v[i];
            last[e] = fmaf(gamma * lambda * (1.0f - d[i]), last[e], delta);
            adv[i] = last[e];
        }
    if (ret) for (size_t i = 0; i < (size_t)T * N; i++) ret[i] = adv[i] + v[i];
    free(last);
}

/* ppo.rs:1174-1263 — two reverse passes with per-player carries. */
void or_compute_gae_mp(const float *all_r, const int32_t *pl, const float *d, const float *v,
                       const float *last_v_pp, int T, int N, int P, float gamma, float lambda,
                       float *adv, float *ret) {
    size_t TN = (size_t)T * N;
    float *ar = malloc(sizeof(float) * TN);
    float *carry = calloc((size_t)N * P, sizeof(float));
    for (int t = T - 1; t >= 0; t--)
        for (int e = 0; e < N; e++) {
            size_t i = (size_t)t * N + e;
            int a = pl[i];
            float *c = carry + (size_t)e * P;
            if (d[i] > 0.5f) for (int p = 0; p < P; p++) c[p] = 0.0f;
            ar[i] = all_r[i * P + a] + c[a];
            c[a] = 0.0f;
            for (int p = 0; p < P; p++) if (p != a) c[p] += all_r[i * P + p];
        }
    float *gc = calloc((size_t)N * P, sizeof(float));
    float *nv = malloc(sizeof(float) * (size_t)N * P);
    memcpy(nv, last_v_pp, sizeof(float) * (size_t)N * P);
    for (int t = T - 1; t >= 0; t--)
        for (int e = 0; e < N; e++) {
            size_t i = (size_t)t * N + e;
            int a = pl[i];
            float *g = gc + (size_t)e * P, *n = nv + (size_t)e * P;
            if (d[i] > 0.5f) {
                for (int p = 0; p < P; p++) g[p] = 0.0f;
                for (int p = 0; p < P; p++) if (p != a) n[p] = 0.0f;
            }
            float delta = fmaf(gamma * n[a], 1.0f - d[i], ar[i]) - v[i];
            float A = fmaf(gamma * lambda * (1.0f - d[i]), g[a], delta);
            adv[i] = A;
            g[a] = A;
            n[a] = v[i];
        }
    if (ret) for (size_t i = 0; i < TN; i++) ret[i] = adv[i] + v[i];
    free(ar); free(carry); free(gc); free(nv);
}

/* ppo.rs:1268-1294 — f32 sequential sums, population variance. */
float or_explained_variance(const float *values, const float *returns, size_t n_) {
    float n = (float)n_;
    if (n < 2.0f) return 0.0f;
    float s = 0.0f;
    for (size_t i = 0; i < n_; i++) s += returns[i];
    float mr = s / n, vr = 0.0f;
    for (size_t i = 0; i < n_; i++) { float q = returns[i] - mr; vr += q * q; }
    vr /= n;
    if (vr < 1e-8f) return 0.0f;
    float sr = 0.0f;
    for (size_t i = 0; i < n_; i++) sr += returns[i] - values[i];
    float mres = sr / n, vres = 0.0f;
    for (size_t i = 0; i < n_; i++) { float q = (returns[i] - values[i]) - mres; vres += q * q; }
    vres /= n;
    return 1.0f - vres / vr;
}

/* ================================================================ trainer == */
struct or_trainer {
    or_train_cfg c;
    or_net_desc net;
    float *params;
    or_adam adam;
    or_vecenv *env;
    or_obs_norm on;
    or_ret_norm rn;
    or_popart pa;
    or_rng rng;
    int T, N, D, A, P, G;
    float *obs, *priv, *rewards, *dones, *values, *logp, *all_r, *masks, *adv, *ret, *raw, *lvpp;
    int32_t *actions, *players;
    int has_masks;
    or_episode *eps;
    int n_eps, eps_cap;
    long n_eps_total;        /* episodes completed in the last collect (n_eps of them stored) */
    double phase_s[3];
    /* opponent pool (ppo.rs:537-1063) */
    int K, n_opp;
    float *opp_params;
    or_obs_norm *opp_on;
    int *opp_has_norm;
    int32_t *lpos, *p2o, *curopp;
    int Pa;                  /* seated players: EnvState's num_players (main.rs:552, 649) */
    float *valid;
    /* the last update's per-minibatch statistics, in run order (parity diagnosis) */
    or_mb_stats mblog[OR_MB_LOG_MAX];
    int n_mblog;
};

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

or_trainer *or_trainer_new(const or_train_cfg *c, const float *init_params) {
    or_trainer *t = calloc(1, sizeof *t);
    t->c = *c;
    t->env = or_vecenv_new_np(c->env_kind, c->num_envs, c->seed + c->env_seed_offset, c->player_count);
    or_vecenv_set_shaping(t->env, (float)c->reward_shaping);
    t->T = c->num_steps; t->N = c->num_envs;
    t->D = or_vecenv_obs_dim(t->env); t->A = or_vecenv_act_dim(t->env);
    t->P = or_vecenv_players(t->env); t->G = c->ctde ? or_vecenv_priv_dim(t->env) : 0;
    t->Pa = c->env_kind == OR_ENV_SKULL ? (c->player_count > 0 ? c->player_count : 4) : t->P;
    t->net.ctde = c->ctde; t->net.obs_dim = t->D; t->net.priv_dim = t->G; t->net.act_dim = t->A;
    t->net.relu = c->relu; t->net.n_actor = c->num_hidden; t->net.actor_width = c->hidden;
    t->net.split = c->split_networks && !c->ctde;   /* mlp.rs:100-130, cnn.rs:116-135 */
    t->net.n_critic = c->ctde ? c->critic_num_hidden : t->net.split ? c->num_hidden : 0;
    t->net.critic_width = c->ctde ? c->critic_hidden : t->net.split ? c->hidden : 0;
    if (c->cnn) {   /* cnn.rs:66-150 */
        t->net.cnn = 1; t->net.n_conv = c->num_conv; t->net.ksize = c->ksize;
        for (int l = 0; l < 4; l++) t->net.conv_ch[l] = c->conv_ch[l];
        t->net.H = 6; t->net.W = 7; t->net.C = 2;
    }
    t->net.n_params = or_net_num_params(&t->net);
    t->params = malloc(sizeof(float) * t->net.n_params);
    memcpy(t->params, init_params, sizeof(float) * t->net.n_params);
    or_adam_init(&t->adam, &t->net);
    or_obs_norm_init(&t->on, t->D, 10.0f);
    or_ret_norm_init(&t->rn, t->N, t->P, c->gamma, c->return_clip);
    or_popart_init(&t->pa);
    or_rng_seed_u64(&t->rng, c->seed);   /* main.rs:189 */
    t->rng.stream = c->rng_stream;       /* rank r of a data-parallel job: stream r */
    size_t TN = (size_t)t->T * t->N;
    t->obs = malloc(sizeof(float) * TN * t->D);
    t->raw = malloc(sizeof(float) * TN * t->D);
    t->priv = t->G ? malloc(sizeof(float) * TN * t->G) : NULL;
    t->rewards = malloc(sizeof(float) * TN);
    t->dones = malloc(sizeof(float) * TN);
    t->values = malloc(sizeof(float) * TN);
    t->logp = malloc(sizeof(float) * TN);
    t->all_r = malloc(sizeof(float) * TN * t->P);
    t->masks = c->env_kind != OR_ENV_CARTPOLE ? malloc(sizeof(float) * TN * t->A) : NULL;
    t->adv = malloc(sizeof(float) * TN);
    t->ret = malloc(sizeof(float) * TN);
    t->actions = malloc(sizeof(int32_t) * TN);
    t->players = malloc(sizeof(int32_t) * TN);
    t->lvpp = calloc((size_t)t->N * t->P, sizeof(float));
    t->eps_cap = t->N * 4 + 1024;
    t->eps = malloc(sizeof(or_episode) * t->eps_cap);
    return t;
}

void or_trainer_free(or_trainer *t) {
    if (!t) return;
    or_vecenv_free(t->env); or_adam_free(&t->adam); or_obs_norm_free(&t->on); or_ret_norm_free(&t->rn);
    free(t->params); free(t->obs); free(t->raw); free(t->priv); free(t->rewards); free(t->dones);
    free(t->values); free(t->logp); free(t->all_r); free(t->masks); free(t->adv); free(t->ret);
    free(t->actions); free(t->players); free(t->lvpp); free(t->eps);
    for (int k = 0; k < t->K; k++) or_obs_norm_free(&t->opp_on[k]);
    free(t->opp_on); free(t->opp_has_norm); free(t->opp_params);
    free(t->lpos); free(t->p2o); free(t->curopp); free(t->valid); free(t);
}

/* opponent_pool.rs:107-123 EnvState::shuffle_positions: the learner's seat is
 * gen_range(0..P) (usize -> u64 draw), the other seats ascending, shuffled
 * (u32 gen_index), then mapped to the assigned opponents in order */
void or_shuffle_positions(or_rng *r, int P, const int32_t *assigned, int32_t *learner_pos, int32_t *pos_to_opp) {
    const int lp = (int)or_gen_range_u64(r, 0, (uint64_t)P);
    uint32_t other[8];
    int no = 0;
    for (int p = 0; p < P; p++) if (p != lp) other[no++] = (uint32_t)p;
    or_shuffle_u32(r, other, (size_t)no);
    *learner_pos = lp;
    for (int p = 0; p < P; p++) pos_to_opp[p] = -1;
    for (int i = 0; i < no; i++) pos_to_opp[other[i]] = assigned[i];
}

void or_trainer_set_opponents(or_trainer *t, int K, const float *params, const double *mean,
                              const double *m2, const double *count, int n_opp, const int32_t *learner_pos,
                              const int32_t *pos_to_opp, const int32_t *current_opp) {
    for (int k = 0; k < t->K; k++) or_obs_norm_free(&t->opp_on[k]);
    free(t->opp_on); free(t->opp_has_norm); free(t->opp_params);
    free(t->lpos); free(t->p2o); free(t->curopp);
    const size_t np = t->net.n_params;
    t->K = K; t->n_opp = n_opp;
    t->opp_params = malloc(sizeof(float) * np * (K > 0 ? K : 1));
    if (K) memcpy(t->opp_params, params, sizeof(float) * np * K);
    t->opp_on = calloc(K > 0 ? K : 1, sizeof(or_obs_norm));
    t->opp_has_norm = calloc(K > 0 ? K : 1, sizeof(int));
    for (int k = 0; k < K; k++) {
        or_obs_norm_init(&t->opp_on[k], t->D, 10.0f);
        if (count && count[k] >= 2.0) {
            memcpy(t->opp_on[k].mean, mean + (size_t)k * t->D, sizeof(double) * t->D);
            memcpy(t->opp_on[k].var, m2 + (size_t)k * t->D, sizeof(double) * t->D);
            t->opp_on[k].count = count[k];
            t->opp_has_norm[k] = 1;
        }
    }
    t->lpos = malloc(sizeof(int32_t) * (n_opp > 0 ? n_opp : 1));
    t->p2o = malloc(sizeof(int32_t) * (size_t)(n_opp > 0 ? n_opp : 1) * t->Pa);
    t->curopp = malloc(sizeof(int32_t) * t->Pa);
    if (n_opp) {
        memcpy(t->lpos, learner_pos, sizeof(int32_t) * n_opp);
        memcpy(t->p2o, pos_to_opp, sizeof(int32_t) * (size_t)n_opp * t->Pa);
    }
    memcpy(t->curopp, current_opp, sizeof(int32_t) * (t->Pa - 1));
    if (!t->valid) t->valid = malloc(sizeof(float) * (size_t)t->T * t->N);
}

void or_trainer_opponent_envs(const or_trainer *t, int32_t *learner_pos, int32_t *pos_to_opp) {
    if (!t->n_opp) return;
    if (learner_pos) memcpy(learner_pos, t->lpos, sizeof(int32_t) * t->n_opp);
    if (pos_to_opp) memcpy(pos_to_opp, t->p2o, sizeof(int32_t) * (size_t)t->n_opp * t->Pa);
}

/* resume hooks (checkpoint.rs:405-465 load_*): main RNG = StdRng::from_seed(key
 * bytes) at word position pos, Adam moments + per-tensor steps, normalizer state */
void or_trainer_set_shaping(or_trainer *t, float coef) { or_vecenv_set_shaping(t->env, coef); }

void or_trainer_set_rng(or_trainer *t, const uint32_t key[8], uint64_t pos) {
    or_rng_from_key(&t->rng, key, 12);
    t->rng.word_pos = pos;
}
void or_trainer_set_adam(or_trainer *t, const float *m1, const float *m2, const int32_t *steps, int n_tensors) {
    memcpy(t->adam.m1, m1, sizeof(float) * t->net.n_params);
    memcpy(t->adam.m2, m2, sizeof(float) * t->net.n_params);
    for (int i = 0; i < n_tensors; i++) t->adam.time[i] = steps[i];
    t->adam.has_state = 1;
}
void or_trainer_get_adam(const or_trainer *t, float *m1, float *m2, int32_t *steps, int n_tensors) {
    memcpy(m1, t->adam.m1, sizeof(float) * t->net.n_params);
    memcpy(m2, t->adam.m2, sizeof(float) * t->net.n_params);
    for (int i = 0; i < n_tensors; i++) steps[i] = t->adam.time[i];
}
void or_trainer_set_norms(or_trainer *t, const double *mean, const double *m2, double count, const double *mvc,
                          const double *returns) {
    if (mean) {
        memcpy(t->on.mean, mean, sizeof(double) * t->D);
        memcpy(t->on.var, m2, sizeof(double) * t->D);
        t->on.count = count;
    }
    if (mvc) {
        t->rn.mean = mvc[0]; t->rn.var = mvc[1]; t->rn.count = mvc[2];
        if (returns) memcpy(t->rn.returns, returns, sizeof(double) * (size_t)t->N * t->P);
    }
}

void or_trainer_popart(or_trainer *t, double *get4, const double *set4) {
    if (get4) { get4[0] = t->pa.mean; get4[1] = t->pa.var; get4[2] = t->pa.count; get4[3] = t->pa.epsilon; }
    if (set4) { t->pa.mean = set4[0]; t->pa.var = set4[1]; t->pa.count = set4[2]; t->pa.epsilon = set4[3]; }
}

size_t or_trainer_num_params(const or_trainer *t) { return t->net.n_params; }
void or_trainer_get_params(const or_trainer *t, float *o) { memcpy(o, t->params, sizeof(float) * t->net.n_params); }
void or_trainer_set_params(or_trainer *t, const float *i) { memcpy(t->params, i, sizeof(float) * t->net.n_params); }
uint64_t or_trainer_rng_pos(const or_trainer *t) { return t->rng.word_pos; }
double or_trainer_last_phase_seconds(const or_trainer *t, int ph) { return t->phase_s[ph]; }

static void forward_rows(or_trainer *t, const float *obs, const float *priv, size_t B,
                         float *logits, float *values) {
    or_net_forward(&t->net, t->params, obs, priv, B, logits, values);
}

/* one masked categorical draw per row of a group (ppo.rs:337-339 / :735-737 / :849-850):
 * -inf masking (panics on an empty mask), Gumbel-max from the main RNG */
static void mask_rows(float *logits, const uint8_t *mk, const int32_t *rows, int n, int A) {
    for (int j = 0; j < n; j++) {
        const uint8_t *m = mk + (size_t)rows[j] * A;
        int any = 0;
        for (int a = 0; a < A; a++) any |= m[a];
        if (!any) { fprintf(stderr, "Empty action mask: env %d\n", rows[j]); abort(); }
        for (int a = 0; a < A; a++) logits[(size_t)j * A + a] += m[a] ? 0.0f : -INFINITY;
    }
}

/* ppo.rs:537-1063 collect_rollouts_with_opponents.  Per step: partition into the
 * learner's rows (self-play envs and opponent envs on the learner's seat) and
 * each opponent model's rows; the learner batch samples first, then the
 * opponent batches in ascending model index, all from the main RNG; env step;
 * every finished opponent game gets the current opponents and reshuffled seats
 * (main RNG, env order); then every row is stored, with the learner-turn flag
 * evaluated against the seats AFTER that reshuffle (ppo.rs:904-911: the
 * reference's order, replicated). */
static int collect_opp(or_trainer *t) {
    double t0 = now_s();
    const int N = t->N, D = t->D, A = t->A, P = t->P, G = t->G;
    const size_t np = t->net.n_params;
    float *raw = malloc(sizeof(float) * N * D), *xo = malloc(sizeof(float) * N * D);
    float *xp = G ? malloc(sizeof(float) * N * G) : NULL, *privs = G ? malloc(sizeof(float) * N * G) : NULL;
    float *logits = malloc(sizeof(float) * N * A), *vals = malloc(sizeof(float) * N);
    float *rw = malloc(sizeof(float) * N * P), *alogp = malloc(sizeof(float) * N), *aval = malloc(sizeof(float) * N);
    uint8_t *dn = malloc(N), *mk = malloc((size_t)N * A);
    int32_t *cp = malloc(sizeof(int32_t) * N), *act = malloc(sizeof(int32_t) * N);
    int32_t *rows = malloc(sizeof(int32_t) * N), *sact = malloc(sizeof(int32_t) * N);
    t->n_eps = 0; t->n_eps_total = 0;
    memset(t->lvpp, 0, sizeof(float) * (size_t)N * P);
    for (int s = 0; s < t->T; s++) {
        const size_t base = (size_t)s * N;
        or_vecenv_get_players(t->env, cp);                                   /* :614 */
        or_vecenv_get_obs(t->env, raw);                                      /* :617 */
        memcpy(t->raw + base * D, raw, sizeof(float) * N * D);               /* :620-622 */
        if (G) { or_vecenv_get_priv(t->env, privs); memcpy(t->priv + base * G, privs, sizeof(float) * N * G); }
        int hm = or_vecenv_get_masks(t->env, mk);                            /* :647 */
        t->has_masks = hm;
        if (!hm) memset(mk, 1, (size_t)N * A);
        if (hm) for (size_t q = 0; q < (size_t)N * A; q++) t->masks[base * A + q] = mk[q] ? 1.0f : 0.0f;
        for (int e = 0; e < N; e++) { act[e] = 0; alogp[e] = 0.0f; aval[e] = 0.0f; }
        /* learner batch (:636-640, :668-775) */
        int n = 0;
        for (int e = 0; e < N; e++) if (e >= t->n_opp || cp[e] == t->lpos[e]) rows[n++] = e;
        if (n) {
            for (int j = 0; j < n; j++) {
                memcpy(xo + (size_t)j * D, raw + (size_t)rows[j] * D, sizeof(float) * D);
                if (G) memcpy(xp + (size_t)j * G, privs + (size_t)rows[j] * G, sizeof(float) * G);
            }
            if (t->c.normalize_obs) or_obs_norm_normalize_batch(&t->on, xo, n);
            forward_rows(t, xo, xp, n, logits, vals);
            if (t->c.normalize_values) or_popart_denormalize(&t->pa, vals, (size_t)n);   /* :759-763 */
            if (hm) mask_rows(logits, mk, rows, n, A);
            or_sample_categorical(&t->rng, logits, n, A, sact);
            for (int j = 0; j < n; j++) {
                const int e = rows[j];
                float lp = or_log_prob(logits + (size_t)j * A, A, sact[j]);
                if (!isfinite(lp)) { fprintf(stderr, "NaN/Inf in log probs\n"); abort(); }
                act[e] = sact[j]; alogp[e] = lp; aval[e] = vals[j];
                t->lvpp[(size_t)e * P + cp[e]] = vals[j];                    /* :770-772 */
            }
        }
        /* opponent batches (:777-864), ascending model index */
        for (int k = 0; k < t->K; k++) {
            n = 0;
            for (int e = 0; e < t->n_opp; e++)
                if (cp[e] != t->lpos[e] && t->p2o[(size_t)e * t->Pa + cp[e]] == k) rows[n++] = e;
            if (!n) continue;
            for (int j = 0; j < n; j++) {
                memcpy(xo + (size_t)j * D, raw + (size_t)rows[j] * D, sizeof(float) * D);
                if (G) memcpy(xp + (size_t)j * G, privs + (size_t)rows[j] * G, sizeof(float) * G);
            }
            if (t->opp_has_norm[k]) or_obs_norm_normalize_batch(&t->opp_on[k], xo, n);
            or_net_forward(&t->net, t->opp_params + (size_t)k * np, xo, xp, n, logits, vals);
            if (hm) mask_rows(logits, mk, rows, n, A);
            or_sample_categorical(&t->rng, logits, n, A, sact);
            for (int j = 0; j < n; j++) act[rows[j]] = sact[j];
        }
        int cap = t->eps_cap - t->n_eps;
        int ne = or_vecenv_step(t->env, act, NULL, rw, dn, t->eps + t->n_eps, cap);   /* :867-871 */
        t->n_eps += ne < cap ? ne : cap;
        t->n_eps_total += ne;
        for (int e = 0; e < t->n_opp; e++)                                   /* :874-925 */
            if (dn[e]) or_shuffle_positions(&t->rng, t->Pa, t->curopp, &t->lpos[e], &t->p2o[(size_t)e * t->Pa]);
        for (int e = 0; e < N; e++) {                                        /* :928-1003 */
            const int cur = cp[e];
            const int valid = e >= t->n_opp || cur == t->lpos[e];
            t->valid[base + e] = valid ? 1.0f : 0.0f;
            float r = rw[(size_t)e * P + cur];
            if (t->c.normalize_returns) {
                or_ret_norm_update_return(&t->rn, e, cur, r);
                if (valid) or_ret_norm_update_variance(&t->rn, e, cur);
                r = or_ret_norm_normalize(&t->rn, r);
                if (dn[e]) or_ret_norm_reset_player(&t->rn, e, cur);
            }
            t->rewards[base + e] = r;
            for (int q = 0; q < P; q++) t->all_r[(base + e) * P + q] = q == cur ? r : rw[(size_t)e * P + q];
            t->actions[base + e] = act[e];
            t->logp[base + e] = alogp[e];
            t->values[base + e] = aval[e];
            t->dones[base + e] = dn[e] ? 1.0f : 0.0f;
            t->players[base + e] = cur;
        }
        memcpy(t->obs + base * D, raw, sizeof(float) * N * D);              /* :943-948 learner-normalized */
        if (t->c.normalize_obs) or_obs_norm_normalize_batch(&t->on, t->obs + base * D, N);
    }
    if (t->c.normalize_obs) or_obs_norm_update_batch(&t->on, t->raw, (size_t)t->T * N);   /* :1058-1060 */
    free(raw); free(xo); free(xp); free(privs); free(logits); free(vals); free(rw); free(alogp); free(aval);
    free(dn); free(mk); free(cp); free(act); free(rows); free(sact);
    t->phase_s[0] = now_s() - t0;
    return (int)t->n_eps_total;
}

/* ppo.rs:213-500 collect_rollouts (self-play / single-player path). */
int or_trainer_collect(or_trainer *t) {
    if (t->n_opp > 0) return collect_opp(t);
    double t0 = now_s();
    const int N = t->N, D = t->D, A = t->A, P = t->P, G = t->G;
    float *obs = malloc(sizeof(float) * N * D);
    float *logits = malloc(sizeof(float) * N * A);
    float *vals = malloc(sizeof(float) * N);
    float *rw = malloc(sizeof(float) * N * P);
    uint8_t *dn = malloc(N);
    uint8_t *mk = malloc((size_t)N * A);
    int32_t *cp = malloc(sizeof(int32_t) * N);
    int32_t *act = malloc(sizeof(int32_t) * N);
    t->n_eps = 0; t->n_eps_total = 0;
    memset(t->lvpp, 0, sizeof(float) * (size_t)N * P);
    for (int s = 0; s < t->T; s++) {
        size_t base = (size_t)s * N;
        or_vecenv_get_players(t->env, cp);                       /* :275 */
        or_vecenv_get_obs(t->env, obs);                          /* :278 */
        if (G) or_vecenv_get_priv(t->env, t->priv + base * G);   /* :282 */
        memcpy(t->raw + base * D, obs, sizeof(float) * N * D);   /* :287-289 */
        if (t->c.normalize_obs) or_obs_norm_normalize_batch(&t->on, obs, N); /* :292-294 lagged */
        int hm = or_vecenv_get_masks(t->env, mk);                /* :297 */
        t->has_masks = hm;
        if (hm)
            for (size_t q = 0; q < (size_t)N * A; q++) t->masks[base * A + q] = mk[q] ? 1.0f : 0.0f;
        forward_rows(t, obs, G ? t->priv + base * G : NULL, N, logits, vals);  /* :322-333 */
        if (t->c.normalize_values) or_popart_denormalize(&t->pa, vals, (size_t)N);   /* :355-359 */
        if (hm) {                                                /* :337 apply_action_mask */
            long bad = or_apply_action_mask(logits, mk, (size_t)N, A);
            if (bad >= 0) { fprintf(stderr, "Empty action mask: env %ld\n", bad); abort(); }
        }
        or_sample_categorical(&t->rng, logits, N, A, act);       /* :338 */
        for (int e = 0; e < N; e++) {                            /* :339 */
            float lp = or_log_prob(logits + (size_t)e * A, A, act[e]);
            if (!isfinite(lp)) { fprintf(stderr, "NaN/Inf in log probs\n"); abort(); }
            t->logp[base + e] = lp;
        }
        int ne = or_vecenv_step(t->env, act, NULL, rw, dn, t->eps + t->n_eps,
                                t->eps_cap - t->n_eps);         /* :374-378 */
        t->n_eps += ne < t->eps_cap - t->n_eps ? ne : t->eps_cap - t->n_eps;
        t->n_eps_total += ne;
        for (int e = 0; e < N; e++) {                            /* :382-408 */
            int p = cp[e];
            float r = rw[(size_t)e * P + p];
            if (t->c.normalize_returns) {
                or_ret_norm_update_return(&t->rn, e, p, r);
                or_ret_norm_update_variance(&t->rn, e, p);
                r = or_ret_norm_normalize(&t->rn, r);
                if (dn[e]) or_ret_norm_reset_player(&t->rn, e, p);
            }
            t->rewards[base + e] = r;
            for (int q = 0; q < P; q++)                          /* :412-428 */
                t->all_r[(base + e) * P + q] = q == p ? r : rw[(size_t)e * P + q];
        }
        memcpy(t->obs + base * D, obs, sizeof(float) * N * D);  /* :431-440 */
        for (int e = 0; e < N; e++) {
            t->actions[base + e] = act[e];
            t->dones[base + e] = dn[e] ? 1.0f : 0.0f;
            t->values[base + e] = vals[e];
            t->players[base + e] = cp[e];
            t->lvpp[(size_t)e * P + cp[e]] = vals[e];           /* :443-445 */
        }
    }
    if (t->c.normalize_obs) or_obs_norm_update_batch(&t->on, t->raw, (size_t)t->T * N); /* :495-497 */
    free(obs); free(logits); free(vals); free(rw); free(dn); free(mk); free(cp); free(act);
    t->phase_s[0] = now_s() - t0;
    return (int)t->n_eps_total;
}

/* main.rs:877-947 bootstrap (UPDATED normalizer stats) then GAE dispatch. */
void or_trainer_gae(or_trainer *t) {
    double t0 = now_s();
    const int N = t->N, D = t->D, A = t->A, P = t->P, G = t->G;
    float *obs = malloc(sizeof(float) * N * D);
    float *priv = G ? malloc(sizeof(float) * N * G) : NULL;
    float *logits = malloc(sizeof(float) * N * A);
    float *lv = malloc(sizeof(float) * N);
    or_vecenv_get_obs(t->env, obs);
    if (t->c.normalize_obs) or_obs_norm_normalize_batch(&t->on, obs, N);
    if (G) or_vecenv_get_priv(t->env, priv);
    forward_rows(t, obs, priv, N, logits, lv);
    if (t->c.normalize_values) or_popart_denormalize(&t->pa, lv, (size_t)N);   /* main.rs:898-907 */
    if (P > 1) {
        int32_t *cp = malloc(sizeof(int32_t) * N);
        or_vecenv_get_players(t->env, cp);
        for (int e = 0; e < N; e++) t->lvpp[(size_t)e * P + cp[e]] = lv[e];
        or_compute_gae_mp(t->all_r, t->players, t->dones, t->values, t->lvpp, t->T, N, P,
                          (float)t->c.gamma, (float)t->c.gae_lambda, t->adv, t->ret);
        free(cp);
    } else {
        or_compute_gae(t->rewards, t->dones, t->values, lv, t->T, N, (float)t->c.gamma,
                       (float)t->c.gae_lambda, t->adv, t->ret);
    }
    free(obs); free(priv); free(logits); free(lv);
    t->phase_s[1] = now_s() - t0;
}

/* ppo.rs:1661-2112 ppo_update, for W ranks stepped in lockstep (W = 1: the
 * reference's single-process update).  W > 1 restates libbppo's data-parallel
 * semantics (the reference has no multi-GPU
 * path): each rank shuffles its own rows with its own main-RNG stream, gathers
 * its minibatch and normalizes the advantages over its own rows, and computes
 * its loss gradient (mean over its rows).  The gradients are then SUMMED over
 * the ranks in f32, in rank order, and scaled by 1/W (the all-reduce between
 * loss.backward() and optimizer.step, ppo.rs:1953-1988), so every rank takes
 * the same clip + Adam step.  The minibatch metrics are the ones of the W
 * minibatches together (sums over all ranks' rows, as the device's metric
 * partials travel with the gradient), except value_error_max and the raw
 * advantage statistics, which stay per rank; the KL early stop reads the
 * combined approx_kl, so all ranks stop together.  PopArt: each rank's running
 * statistics absorb every rank's returns in rank order before the rescale.  Opponent
 * pools: each rank trains on its own learner rows, cut into num_minibatches of its own
 * sizes; the slots run in lockstep, a rank without rows in one adding a zero gradient. */
typedef struct {
    uint32_t *vidx, *idx;
    size_t B, sz, start;
    float *grads, *mo, *mp, *mm, *mlp, *madv, *mret, *mov, *madvn;
    int32_t *ma;
    float am, as, amn, amx;
    or_mb_stats st;
    float tam, tas, tamin, tamax, tvemax;
    float rescale_mag;
    double tsum, tsq, tcnt;
} rank_ws;

void or_trainers_update(or_trainer **ts, int W, or_update_metrics *ms) {
    double t0 = now_s();
    if (W < 1) return;
    or_trainer *t0r = ts[0];
    const int D = t0r->D, A = t0r->A, G = t0r->G;
    const or_ppo_cfg *c = &t0r->c.ppo;
    const size_t np = t0r->net.n_params;
    rank_ws *ws = calloc((size_t)W, sizeof *ws);
    size_t mbmax = 0;
    for (int r = 0; r < W; r++) {
        or_trainer *t = ts[r];
        rank_ws *w = &ws[r];
        w->B = (size_t)t->T * t->N;
        /* opponent-pool training: only the learner rows, in (t, e) order (ppo.rs:1696-1720) */
        if (t->n_opp > 0) {
            w->vidx = malloc(sizeof(uint32_t) * w->B);
            size_t nv = 0;
            for (size_t i = 0; i < w->B; i++) if (t->valid[i] > 0.5f) w->vidx[nv++] = (uint32_t)i;
            w->B = nv;
        }
    }
    for (int r = 0; r < W; r++) {
        or_trainer *t = ts[r];
        rank_ws *w = &ws[r];
        /* ppo.rs:1787-1808 PopArt: statistics over the (learner) returns, then rescale the value head */
        w->rescale_mag = NAN;
        if (t->c.normalize_values) {
            double om, os;
            if (W == 1) {
                float *rr = malloc(sizeof(float) * (w->B ? w->B : 1));
                for (size_t i = 0; i < w->B; i++) rr[i] = t->ret[w->vidx ? w->vidx[i] : i];
                or_popart_update(&t->pa, rr, w->B, &om, &os);
                free(rr);
            } else {
                /* W > 1: every rank's statistics absorb ALL ranks' returns, rank by rank (the
                 * device all-gathers the ranks' batch statistics and merges them in rank order),
                 * so the value-head rescale below is the same on every rank */
                double dm, ds;
                om = t->pa.mean; os = or_popart_std(&t->pa);
                for (int q = 0; q < W; q++) {
                    const rank_ws *wq = &ws[q];
                    float *rr = malloc(sizeof(float) * (wq->B ? wq->B : 1));
                    for (size_t i = 0; i < wq->B; i++) rr[i] = ts[q]->ret[wq->vidx ? wq->vidx[i] : i];
                    or_popart_update(&t->pa, rr, wq->B, &dm, &ds);
                    free(rr);
                }
            }
            if (t->pa.count >= 2.0) {
                size_t vw, vb; int vin;
                or_net_value_head(&t->net, &vw, &vb, &vin);    /* ppo.rs:1599-1653 */
                const double nm = t->pa.mean, ns = or_popart_std(&t->pa), sc = os / ns;
                for (int i = 0; i < vin; i++) t->params[vw + i] = (float)((double)t->params[vw + i] * sc);
                t->params[vb] = (float)(((double)t->params[vb] * os + om - nm) / ns);
                w->rescale_mag = (float)fabs(sc);
            }
        }
        size_t mbm = w->B / c->num_minibatches + 1;
        if (mbm > mbmax) mbmax = mbm;
    }
    for (int r = 0; r < W; r++) {
        rank_ws *w = &ws[r];
        w->idx = malloc(sizeof(uint32_t) * (w->B ? w->B : 1));
        w->grads = malloc(sizeof(float) * np);
        w->mo = malloc(sizeof(float) * mbmax * D);
        w->mp = G ? malloc(sizeof(float) * mbmax * G) : NULL;
        w->mm = ts[r]->has_masks ? malloc(sizeof(float) * mbmax * A) : NULL;
        w->ma = malloc(sizeof(int32_t) * mbmax);
        w->mlp = malloc(sizeof(float) * mbmax); w->madv = malloc(sizeof(float) * mbmax);
        w->mret = malloc(sizeof(float) * mbmax); w->mov = malloc(sizeof(float) * mbmax);
        w->madvn = malloc(sizeof(float) * mbmax);
        w->tamin = INFINITY; w->tamax = -INFINITY; w->tvemax = -INFINITY;
    }
    /* W > 1: the combined minibatch (stats only) and the summed gradient */
    const size_t cmax = W > 1 ? (size_t)W * mbmax : 1;
    float *co = W > 1 ? malloc(sizeof(float) * cmax * D) : NULL;
    float *cp = W > 1 && G ? malloc(sizeof(float) * cmax * G) : NULL;
    float *cm = W > 1 && t0r->has_masks ? malloc(sizeof(float) * cmax * A) : NULL;
    int32_t *ca = W > 1 ? malloc(sizeof(int32_t) * cmax) : NULL;
    float *clp = W > 1 ? malloc(sizeof(float) * cmax) : NULL, *cadv = W > 1 ? malloc(sizeof(float) * cmax) : NULL;
    float *cret = W > 1 ? malloc(sizeof(float) * cmax) : NULL, *cov = W > 1 ? malloc(sizeof(float) * cmax) : NULL;
    float *gsum = malloc(sizeof(float) * np), *gstep = malloc(sizeof(float) * np);
    float tp = 0, tv = 0, th = 0, tk = 0, tc = 0, tl = 0, tvm = 0, trm = 0;
    float tvem = 0, tves = 0, tav = 0, tevp = 0;
    int nup = 0, epochs_run = 0, stop = 0;
    for (int r = 0; r < W; r++) ts[r]->n_mblog = 0;
    uint64_t S[64];                      /* each rank's first shuffle word (shuffle_windows) */
    for (int r = 0; r < W && r < 64; r++) S[r] = ts[r]->rng.word_pos;
    const int windows = t0r->c.shuffle_windows;
    if (windows && (W > 64 || ws[0].vidx)) { fprintf(stderr, "or_trainers_update: shuffle_windows: self-play only\n"); abort(); }
    for (int ep = 0; ep < c->num_epochs && !stop; ep++) {
        epochs_run++;
        for (int r = 0; r < W; r++) {
            rank_ws *w = &ws[r];
            for (size_t i = 0; i < w->B; i++) w->idx[i] = (uint32_t)i;  /* :1815 */
            if (windows) ts[r]->rng.word_pos = S[r] + (uint64_t)ep * OR_SHUFFLE_WINDOW(w->B);
            or_shuffle_u32(&ts[r]->rng, w->idx, w->B);                    /* :1816 */
            w->start = 0;
        }
        /* each rank cuts its own rows into num_minibatches (its learner-row count under an
         * opponent pool); W > 1 runs every slot on every rank in lockstep, a rank without
         * rows in a slot adding a zero gradient (the device's all-reduce count must match) */
        for (int mbi = 0; mbi < c->num_minibatches; mbi++) {
            size_t sz_any = 0;
            for (int r = 0; r < W; r++) {
                const size_t Br = ws[r].B;
                ws[r].sz = Br / c->num_minibatches + ((size_t)mbi < Br % c->num_minibatches ? 1 : 0);
                sz_any += ws[r].sz;
            }
            if (W == 1 && sz_any == 0) continue;
            for (int r = 0; r < W; r++) {
                or_trainer *t = ts[r];
                rank_ws *w = &ws[r];
                const size_t sz = w->sz;
                if (sz == 0) {
                    memset(w->grads, 0, sizeof(float) * np);
                    memset(&w->st, 0, sizeof w->st);
                    w->am = w->as = 0.0f; w->amn = INFINITY; w->amx = -INFINITY;
                    w->st.value_error_max = -INFINITY;
                    continue;
                }
                for (size_t q = 0; q < sz; q++) {                    /* :1833-1857 gather */
                    size_t i = w->vidx ? w->vidx[w->idx[w->start + q]] : w->idx[w->start + q];
                    memcpy(w->mo + q * D, t->obs + i * D, sizeof(float) * D);
                    if (G) memcpy(w->mp + q * G, t->priv + i * G, sizeof(float) * G);
                    if (w->mm) memcpy(w->mm + q * A, t->masks + i * A, sizeof(float) * A);
                    w->ma[q] = t->actions[i]; w->mlp[q] = t->logp[i]; w->madv[q] = t->adv[i];
                    w->mret[q] = t->ret[i]; w->mov[q] = t->values[i];
                }
                if (t->c.normalize_values) {                        /* ppo.rs:1859-1897 */
                    or_popart_normalize(&t->pa, w->mret, sz, w->mret);
                    or_popart_normalize(&t->pa, w->mov, sz, w->mov);
                    for (size_t q = 0; q < sz; q++) {
                        w->tsum += (double)w->mret[q]; w->tsq += (double)w->mret[q] * w->mret[q]; w->tcnt += 1.0;
                    }
                }
                or_normalize_advantages(w->madv, sz, w->madvn, &w->am, &w->as, &w->amn, &w->amx);
                or_minibatch_loss_grad(&t->net, t->params, sz, w->mo, w->mp, w->ma, w->mlp, w->madvn, w->mret,
                                       w->mov, w->mm, c, t->c.ent_coef, w->grads, &w->st);
            }
            or_mb_stats stg = ws[0].st;
            if (W == 1) {
                memcpy(gstep, ws[0].grads, sizeof(float) * np);
            } else {
                /* the SUM all-reduce in rank order, then 1/W before clip + Adam */
                memcpy(gsum, ws[0].grads, sizeof(float) * np);
                for (int r = 1; r < W; r++)
                    for (size_t k = 0; k < np; k++) gsum[k] += ws[r].grads[k];
                const float inv_world = 1.0f / (float)W;
                for (size_t k = 0; k < np; k++) gstep[k] = gsum[k] * inv_world;
                /* the metrics of all ranks' rows together */
                size_t o = 0;
                for (int r = 0; r < W; r++) {
                    rank_ws *w = &ws[r];
                    const size_t sz = w->sz;
                    memcpy(co + o * D, w->mo, sizeof(float) * sz * D);
                    if (G) memcpy(cp + o * G, w->mp, sizeof(float) * sz * G);
                    if (cm) memcpy(cm + o * A, w->mm, sizeof(float) * sz * A);
                    memcpy(ca + o, w->ma, sizeof(int32_t) * sz); memcpy(clp + o, w->mlp, sizeof(float) * sz);
                    memcpy(cadv + o, w->madvn, sizeof(float) * sz); memcpy(cret + o, w->mret, sizeof(float) * sz);
                    memcpy(cov + o, w->mov, sizeof(float) * sz);
                    o += sz;
                }
                or_minibatch_loss_grad(&t0r->net, t0r->params, o, co, cp, ca, clp, cadv, cret, cov, cm, c,
                                       t0r->c.ent_coef, NULL, &stg);
            }
            for (int r = 0; r < W; r++) {
                or_trainer *t = ts[r];
                float *g = gstep;
                if (r + 1 < W) { memcpy(gsum, gstep, sizeof(float) * np); g = gsum; }   /* the step clips in place */
                or_adam_step(&t->net, &t->adam, t->params, g, t->c.lr, (float)c->max_grad_norm, c->adam_epsilon);
                rank_ws *w = &ws[r];
                w->tam += w->am; w->tas += w->as;
                w->tamin = fminf(w->tamin, w->amn); w->tamax = fmaxf(w->tamax, w->amx);
                w->tvemax = fmaxf(w->tvemax, w->st.value_error_max);
                w->start += w->sz;
            }
            for (int r = 0; r < W; r++)
                if (ts[r]->n_mblog < OR_MB_LOG_MAX) ts[r]->mblog[ts[r]->n_mblog++] = stg;
            tp += stg.policy_loss; tv += stg.value_loss; th += stg.entropy; tk += stg.approx_kl;
            tc += stg.clip_fraction; tl += stg.loss; tvm += stg.value_mean; trm += stg.returns_mean;
            tvem += stg.value_error_mean; tves += stg.value_error_std;
            tav += stg.avg_valid_actions; tevp += stg.entropy_valid_pct;
            nup++;
            if (c->target_kl >= 0 && stg.approx_kl > (float)c->target_kl) { stop = 1; break; } /* :2019-2023 */
        }
    }
    if (windows)
        for (int r = 0; r < W; r++) ts[r]->rng.word_pos = S[r] + (uint64_t)c->num_epochs * OR_SHUFFLE_WINDOW(ws[r].B);
    for (int r = 0; r < W; r++) {
        or_trainer *t = ts[r];
        rank_ws *w = &ws[r];
        or_update_metrics *m = ms ? &ms[r] : NULL;
        if (!m) continue;
        const size_t B = w->B;
        float n = (float)nup;
        memset(m, 0, sizeof *m);
        m->policy_loss = tp / n; m->value_loss = tv / n; m->entropy = th / n;
        m->entropy_scaled = m->entropy / logf((float)A);
        m->approx_kl = tk / n; m->clip_fraction = tc / n;
        if (w->vidx) {                                                /* ppo.rs:2047-2056 */
            float *fv = malloc(sizeof(float) * (B ? B : 1)), *fr = malloc(sizeof(float) * (B ? B : 1));
            for (size_t i = 0; i < B; i++) { fv[i] = t->values[w->vidx[i]]; fr[i] = t->ret[w->vidx[i]]; }
            m->explained_variance = or_explained_variance(fv, fr, B);
            free(fv); free(fr);
        } else {
            m->explained_variance = or_explained_variance(t->values, t->ret, B);
        }
        m->total_loss = tl / n; m->value_mean = tvm / n; m->returns_mean = trm / n;
        m->adv_mean_raw = w->tam / n; m->adv_std_raw = w->tas / n; m->adv_min_raw = w->tamin; m->adv_max_raw = w->tamax;
        m->value_error_mean = tvem / n; m->value_error_std = tves / n; m->value_error_max = w->tvemax;
        m->avg_valid_actions = t->has_masks ? tav / n : 0.0f;
        m->entropy_valid_pct = t->has_masks ? tevp / n : 0.0f;
        m->num_updates = nup; m->epochs_run = epochs_run;
        m->value_norm_rescale_mag = w->rescale_mag;
        m->value_norm_target_mean = m->value_norm_target_std = NAN;
        if (w->tcnt > 0) {                                             /* ppo.rs:2061-2068 */
            const double mean = w->tsum / w->tcnt, var = w->tsq / w->tcnt - mean * mean;
            m->value_norm_target_mean = (float)mean;
            m->value_norm_target_std = (float)sqrt(var > 0.0 ? var : 0.0);
        }
    }
    for (int r = 0; r < W; r++) {
        rank_ws *w = &ws[r];
        free(w->vidx); free(w->idx); free(w->grads); free(w->mo); free(w->mp); free(w->mm); free(w->ma);
        free(w->mlp); free(w->madv); free(w->mret); free(w->mov); free(w->madvn);
    }
    free(ws); free(co); free(cp); free(cm); free(ca); free(clp); free(cadv); free(cret); free(cov);
    free(gsum); free(gstep);
    for (int r = 0; r < W; r++) ts[r]->phase_s[2] = now_s() - t0;
}

void or_trainer_update(or_trainer *t, or_update_metrics *m) { or_trainers_update(&t, 1, m); }

size_t or_trainer_buffer(const or_trainer *t, const char *name, void *out, size_t bytes) {
    size_t TN = (size_t)t->T * t->N;
    const void *src = NULL; size_t n = 0;
    if (!strcmp(name, "obs")) { src = t->obs; n = TN * t->D * 4; }
    else if (!strcmp(name, "raw_obs")) { src = t->raw; n = TN * t->D * 4; }
    else if (!strcmp(name, "priv")) { src = t->priv; n = t->G ? TN * t->G * 4 : 0; }
    else if (!strcmp(name, "actions")) { src = t->actions; n = TN * 4; }
    else if (!strcmp(name, "rewards")) { src = t->rewards; n = TN * 4; }
    else if (!strcmp(name, "dones")) { src = t->dones; n = TN * 4; }
    else if (!strcmp(name, "values")) { src = t->values; n = TN * 4; }
    else if (!strcmp(name, "log_probs")) { src = t->logp; n = TN * 4; }
    else if (!strcmp(name, "advantages")) { src = t->adv; n = TN * 4; }
    else if (!strcmp(name, "returns")) { src = t->ret; n = TN * 4; }
    else if (!strcmp(name, "players")) { src = t->players; n = TN * 4; }
    else if (!strcmp(name, "all_rewards")) { src = t->all_r; n = TN * t->P * 4; }
    else if (!strcmp(name, "masks")) { src = t->masks; n = t->masks ? TN * t->A * 4 : 0; }
    else if (!strcmp(name, "last_v_pp")) { src = t->lvpp; n = (size_t)t->N * t->P * 4; }
    else if (!strcmp(name, "valid")) { src = t->valid; n = t->valid ? TN * 4 : 0; }
    if (!src) return 0;
    if (out && bytes >= n) memcpy(out, src, n);
    return n;
}

/* parity hook: overwrite a RolloutBuffer field (names as or_trainer_buffer) */
int or_trainer_set_buffer(or_trainer *t, const char *name, const void *src, size_t bytes) {
    size_t n = or_trainer_buffer(t, name, NULL, 0);
    if (!n || n != bytes) return -1;
    void *dst = NULL;
    if (!strcmp(name, "values")) dst = t->values;
    else if (!strcmp(name, "advantages")) dst = t->adv;
    else if (!strcmp(name, "returns")) dst = t->ret;
    else if (!strcmp(name, "rewards")) dst = t->rewards;
    else if (!strcmp(name, "log_probs")) dst = t->logp;
    if (!dst) return -1;
    memcpy(dst, src, bytes);
    return 0;
}

void or_trainer_obs_norm_state(const or_trainer *t, double *mean, double *var, double *count) {
    if (mean) memcpy(mean, t->on.mean, sizeof(double) * t->D);
    if (var) memcpy(var, t->on.var, sizeof(double) * t->D);
    if (count) *count = t->on.count;
}

void or_trainer_ret_norm_state(const or_trainer *t, double *mvc, double *returns) {
    if (mvc) { mvc[0] = t->rn.mean; mvc[1] = t->rn.var; mvc[2] = t->rn.count; }
    if (returns) memcpy(returns, t->rn.returns, sizeof(double) * (size_t)t->N * t->P);
}

int or_trainer_episodes(const or_trainer *t, or_episode *out, int cap) {
    int n = t->n_eps < cap ? t->n_eps : cap;
    if (out) memcpy(out, t->eps, sizeof(or_episode) * n);
    return t->n_eps;
}

int or_trainer_mb_log(const or_trainer *t, or_mb_stats *out, int max) {
    const int n = t->n_mblog < max ? t->n_mblog : max;
    if (out) memcpy(out, t->mblog, sizeof(or_mb_stats) * (size_t)n);
    return t->n_mblog;
}

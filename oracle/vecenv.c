/*
 * vecenv.c — VecEnv semantics (env.rs:270-487) and the two normalizers
 * (normalization.rs:12-260).  TEST INFRASTRUCTURE ONLY.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

struct or_vecenv {
    int kind, n, obs_dim, act_dim, players, priv_dim, invalid;
    float shaping;
    void *envs;
    size_t env_size;
    float *obs;           /* obs_buffer [N*obs] */
    float *ep_rewards;    /* [N*P] */
    int32_t *ep_len;      /* [N] */
};

static void *env_at(const or_vecenv *v, int i) { return (char *)v->envs + (size_t)i * v->env_size; }
void *or_vecenv_env_ptr(or_vecenv *v, int i) { return env_at(v, i); }

static void env_reset(or_vecenv *v, int i, float *obs) {
    switch (v->kind) {
    case OR_ENV_CARTPOLE: or_cartpole_reset(env_at(v, i), obs); break;
    case OR_ENV_CONNECT_FOUR: or_c4_reset(env_at(v, i), obs); break;
    case OR_ENV_SKULL: or_skull_reset(env_at(v, i), obs); break;
    default: or_ld_reset(env_at(v, i), obs); break;
    }
}

/* env.rs:281-302 — factory(i) (main.rs:1964 seed+i) then reset() AGAIN. */
or_vecenv *or_vecenv_new(int kind, int n, uint64_t seed_base) { return or_vecenv_new_np(kind, n, seed_base, 0); }
int or_vecenv_invalid(const or_vecenv *v) { return v->invalid; }

or_vecenv *or_vecenv_new_np(int kind, int n, uint64_t seed_base, int np) {
    or_vecenv *v = calloc(1, sizeof *v);
    if (np <= 0) np = 4;                               /* PlayerCountMode::default (config.rs:667-671) */
    v->kind = kind; v->n = n;
    switch (kind) {
    case OR_ENV_CARTPOLE:
        v->obs_dim = OR_CP_OBS; v->act_dim = OR_CP_ACT; v->players = 1; v->priv_dim = 0;
        v->env_size = sizeof(or_cartpole);
        break;
    case OR_ENV_CONNECT_FOUR:
        v->obs_dim = OR_C4_OBS; v->act_dim = OR_C4_ACT; v->players = 2; v->priv_dim = 0;
        v->env_size = sizeof(or_connect_four);
        break;
    case OR_ENV_SKULL:   /* Environment::NUM_PLAYERS = MAX_PLAYERS (skull.rs:1049) */
        v->obs_dim = OR_SK_OBS; v->act_dim = OR_SK_ACT; v->players = OR_SK_MAXP; v->priv_dim = OR_SK_PRIV;
        v->env_size = sizeof(or_skull);
        break;
    default:
        v->obs_dim = OR_LD_OBS; v->act_dim = OR_LD_ACT; v->players = 4; v->priv_dim = OR_LD_PRIV;
        v->env_size = sizeof(or_liars_dice);
        break;
    }
    v->envs = calloc((size_t)n, v->env_size);
    v->obs = calloc((size_t)n * v->obs_dim, sizeof(float));
    v->ep_rewards = calloc((size_t)n * v->players, sizeof(float));
    v->ep_len = calloc((size_t)n, sizeof(int32_t));
    for (int i = 0; i < n; i++) {
        uint64_t s = seed_base + (uint64_t)i;
        switch (kind) {
        case OR_ENV_CARTPOLE: or_cartpole_new(env_at(v, i), s); break;
        case OR_ENV_CONNECT_FOUR: or_c4_new(env_at(v, i)); break;
        case OR_ENV_SKULL: or_skull_new(env_at(v, i), np, s); break;   /* main.rs:2008-2014 */
        default: or_ld_new(env_at(v, i), s); break;
        }
        env_reset(v, i, v->obs + (size_t)i * v->obs_dim);
    }
    return v;
}

void or_vecenv_free(or_vecenv *v) {
    if (!v) return;
    free(v->envs); free(v->obs); free(v->ep_rewards); free(v->ep_len); free(v);
}

int or_vecenv_obs_dim(const or_vecenv *v) { return v->obs_dim; }
int or_vecenv_act_dim(const or_vecenv *v) { return v->act_dim; }
int or_vecenv_players(const or_vecenv *v) { return v->players; }
int or_vecenv_priv_dim(const or_vecenv *v) { return v->priv_dim; }
void or_vecenv_set_shaping(or_vecenv *v, float c) { v->shaping = c; }

/* schedule.rs:54-78 Schedule::get over n (value, step) milestones */
double or_schedule_get(const double *v, const uint64_t *s, int n, uint64_t step) {
    if (n <= 0) return 0.0;
    if (n == 1 || step <= s[0]) return v[0];
    for (int i = 0; i < n - 1; i++) {
        if (step >= s[i] && step < s[i + 1]) {
            double t = (double)(step - s[i]) / (double)(s[i + 1] - s[i]);
            return v[i] + (v[i + 1] - v[i]) * t;
        }
    }
    return v[n - 1];
}

/* env.rs:336-376 */
void or_vecenv_get_obs(const or_vecenv *v, float *obs) {
    memcpy(obs, v->obs, sizeof(float) * (size_t)v->n * v->obs_dim);
}
void or_vecenv_get_players(const or_vecenv *v, int32_t *p) {
    for (int i = 0; i < v->n; i++) {
        switch (v->kind) {
        case OR_ENV_CARTPOLE: p[i] = 0; break;
        case OR_ENV_CONNECT_FOUR: p[i] = or_c4_current_player(env_at(v, i)); break;
        case OR_ENV_SKULL: p[i] = or_skull_current_player(env_at(v, i)); break;
        default: p[i] = or_ld_current_player(env_at(v, i)); break;
        }
    }
}
int or_vecenv_get_masks(const or_vecenv *v, uint8_t *m) {
    if (v->kind == OR_ENV_CARTPOLE) return 0;
    for (int i = 0; i < v->n; i++) {
        if (v->kind == OR_ENV_CONNECT_FOUR) or_c4_mask(env_at(v, i), m + (size_t)i * 7);
        else if (v->kind == OR_ENV_SKULL) or_skull_mask(env_at(v, i), m + (size_t)i * OR_SK_ACT);
        else or_ld_mask(env_at(v, i), m + (size_t)i * 49);
    }
    return 1;
}
void or_vecenv_get_priv(const or_vecenv *v, float *g) {
    if (v->kind == OR_ENV_SKULL) {
        for (int i = 0; i < v->n; i++) or_skull_priv(env_at(v, i), g + (size_t)i * OR_SK_PRIV);
        return;
    }
    if (v->kind != OR_ENV_LIARS_DICE) return;
    for (int i = 0; i < v->n; i++) or_ld_priv(env_at(v, i), g + (size_t)i * OR_LD_PRIV);
}

/* env.rs:400-487 — parallel step (rayon there, OpenMP here), accumulate
 * episode reward/length, auto-reset on done, completed stats in env order. */
int or_vecenv_step(or_vecenv *v, const int32_t *actions, float *obs_out, float *rewards,
                   uint8_t *dones, or_episode *eps, int eps_cap) {
    const int P = v->players, D = v->obs_dim;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < v->n; i++) {
        float r[6] = {0, 0, 0, 0, 0, 0};
        int done = 0, bad = 0;
        float *o = v->obs + (size_t)i * D;
        switch (v->kind) {
        case OR_ENV_CARTPOLE: or_cartpole_step(env_at(v, i), actions[i], o, &r[0], &done); break;
        case OR_ENV_CONNECT_FOUR: or_c4_step(env_at(v, i), actions[i], o, r, &done); break;
        case OR_ENV_SKULL:
            or_skull_step(env_at(v, i), actions[i], v->shaping, o, r, &done, &bad);
            if (bad) {
#pragma omp atomic write
                v->invalid = 1;
            }
            break;
        default: or_ld_step(env_at(v, i), actions[i], v->shaping, o, r, &done); break;
        }
        for (int p = 0; p < P; p++) {
            v->ep_rewards[(size_t)i * P + p] += r[p];
            rewards[(size_t)i * P + p] = r[p];
        }
        v->ep_len[i] += 1;
        dones[i] = (uint8_t)done;
    }
    int n_eps = 0;
    for (int i = 0; i < v->n; i++) {
        if (!dones[i]) continue;
        if (eps && n_eps < eps_cap) {
            or_episode *e = &eps[n_eps];
            memset(e, 0, sizeof *e);
            for (int p = 0; p < P; p++) e->total_rewards[p] = v->ep_rewards[(size_t)i * P + p];
            e->length = v->ep_len[i];
            e->env_index = i;
        }
        n_eps++;
        for (int p = 0; p < P; p++) v->ep_rewards[(size_t)i * P + p] = 0.0f;
        v->ep_len[i] = 0;
    }
    /* resets consume each env's own RNG stream only: order-independent */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < v->n; i++)
        if (dones[i]) env_reset(v, i, v->obs + (size_t)i * D);
    if (obs_out) memcpy(obs_out, v->obs, sizeof(float) * (size_t)v->n * D);
    return n_eps;
}

/* ============================================================ ObsNormalizer */
void or_obs_norm_init(or_obs_norm *n, int dim, float clip) {
    n->dim = dim;
    n->mean = calloc((size_t)dim, sizeof(double));
    n->var = calloc((size_t)dim, sizeof(double));
    n->count = 0.0;
    n->clip = clip;
}
void or_obs_norm_free(or_obs_norm *n) { free(n->mean); free(n->var); }

/* normalization.rs:37-53 — sequential Welford over rows in (t, e) order */
void or_obs_norm_update_batch(or_obs_norm *n, const float *obs, size_t rows) {
    for (size_t i = 0; i < rows; i++) {
        n->count += 1.0;
        for (int j = 0; j < n->dim; j++) {
            double x = (double)obs[i * n->dim + j];
            double delta = x - n->mean[j];
            n->mean[j] += delta / n->count;
            double delta2 = x - n->mean[j];
            n->var[j] += delta * delta2;
        }
    }
}

/* normalization.rs:58-75 */
void or_obs_norm_normalize_batch(const or_obs_norm *n, float *obs, size_t rows) {
    if (n->count < 2.0) return;
    for (size_t i = 0; i < rows; i++)
        for (int j = 0; j < n->dim; j++) {
            double variance = n->var[j] / n->count;
            double sd = sqrt(variance);
            if (sd < 1e-8) sd = 1e-8;
            float z = (float)(((double)obs[i * n->dim + j] - n->mean[j]) / sd);
            if (z < -n->clip) z = -n->clip;
            if (z > n->clip) z = n->clip;
            obs[i * n->dim + j] = z;
        }
}

/* ========================================================= ReturnNormalizer */
void or_ret_norm_init(or_ret_norm *n, int num_envs, int num_players, double gamma, float clip) {
    n->num_envs = num_envs; n->num_players = num_players;
    n->returns = calloc((size_t)num_envs * num_players, sizeof(double));
    n->var = n->mean = n->count = 0.0;
    n->gamma = gamma; n->epsilon = 1e-8; n->clip = clip;
}
void or_ret_norm_free(or_ret_norm *n) { free(n->returns); }
/* normalization.rs:156-160 */
void or_ret_norm_update_return(or_ret_norm *n, int e, int p, float r) {
    double *x = &n->returns[(size_t)e * n->num_players + p];
    *x = *x * n->gamma + (double)r;
}
/* normalization.rs:171-181 */
void or_ret_norm_update_variance(or_ret_norm *n, int e, int p) {
    double x = n->returns[(size_t)e * n->num_players + p];
    n->count += 1.0;
    double delta = x - n->mean;
    n->mean += delta / n->count;
    double delta2 = x - n->mean;
    n->var += delta * delta2;
}
/* normalization.rs:187-197 */
float or_ret_norm_normalize(const or_ret_norm *n, float r) {
    if (n->count < 2.0) return r;
    double variance = n->var / n->count;
    double sd = sqrt(variance + n->epsilon);
    float z = (float)((double)r / sd);
    if (z < -n->clip) z = -n->clip;
    if (z > n->clip) z = n->clip;
    return z;
}
void or_ret_norm_reset_player(or_ret_norm *n, int e, int p) {
    n->returns[(size_t)e * n->num_players + p] = 0.0;
}
/* normalization.rs:202-210 */
void or_ret_norm_reset_env(or_ret_norm *n, int e) {
    for (int p = 0; p < n->num_players; p++) n->returns[(size_t)e * n->num_players + p] = 0.0;
}
/* normalization.rs:220-243 (single-player convenience): per env update the
 * rolling return, the variance stats, normalize in place, reset on done */
void or_ret_norm_update_and_normalize_all(or_ret_norm *n, float *rewards, const uint8_t *dones) {
    for (int e = 0; e < n->num_envs; e++) {
        const float r = rewards[e];
        or_ret_norm_update_return(n, e, 0, r);
        or_ret_norm_update_variance(n, e, 0);
        rewards[e] = or_ret_norm_normalize(n, r);
        if (dones[e]) or_ret_norm_reset_player(n, e, 0);
    }
}

/* ======================================================== PopArtNormalizer */
void or_popart_init(or_popart *p) { p->mean = 0.0; p->var = 0.0; p->count = 0.0; p->epsilon = 1e-4; }
/* normalization.rs:299-305 */
double or_popart_std(const or_popart *p) { return p->count < 2.0 ? 1.0 : sqrt(p->var / p->count + p->epsilon); }
/* normalization.rs:316-332: sequential Welford; returns the stats before the batch */
void or_popart_update(or_popart *p, const float *r, size_t n, double *old_mean, double *old_std) {
    *old_mean = p->mean;
    *old_std = or_popart_std(p);
    for (size_t i = 0; i < n; i++) {
        const double x = (double)r[i];
        p->count += 1.0;
        const double d = x - p->mean;
        p->mean += d / p->count;
        p->var += d * (x - p->mean);
    }
}
/* normalization.rs:337-348 */
void or_popart_normalize(const or_popart *p, const float *x, size_t n, float *out) {
    if (p->count < 2.0) { memmove(out, x, sizeof(float) * n); return; }
    const double sd = or_popart_std(p);
    for (size_t i = 0; i < n; i++) out[i] = (float)(((double)x[i] - p->mean) / sd);
}
/* normalization.rs:351-360 */
void or_popart_denormalize(const or_popart *p, float *v, size_t n) {
    if (p->count < 2.0) return;
    const double sd = or_popart_std(p);
    for (size_t i = 0; i < n; i++) v[i] = (float)((double)v[i] * sd + p->mean);
}

/*
 * envs.c — CartPole, Connect Four, Liar's Dice restated from the reference
 * (TEST INFRASTRUCTURE ONLY).
 */
#include <math.h>
#include <string.h>
#include "oracle.h"

/* ============================================================ CartPole ==== */
/* envs/cartpole.rs:11-23 — f32 constants evaluated like rustc const-folds them. */
#define CP_GRAVITY 9.8f
#define CP_POLE_MASS 0.1f
#define CP_TOTAL_MASS (1.0f + 0.1f)
#define CP_HALF_LEN 0.5f
#define CP_MASS_LEN (0.1f * 0.5f)
#define CP_FORCE 10.0f
#define CP_TAU 0.02f
#define CP_X_THRESH 2.4f
#define CP_MAX_STEPS 500

static float cp_theta_threshold(void) {
    /* cartpole.rs:22: 12.0 * PI / 180.0 in f32, left to right */
    volatile float twelve = 12.0f, pi = 3.14159265358979323846f, d = 180.0f;
    return twelve * pi / d;
}

/* cartpole.rs:75-84 */
void or_cartpole_get_obs(const or_cartpole *e, float *obs) {
    obs[0] = e->x; obs[1] = e->x_dot; obs[2] = e->theta; obs[3] = e->theta_dot;
    obs[4] = (float)e->steps / (float)CP_MAX_STEPS;
}

/* cartpole.rs:272-281 — four gen_range(-0.05..0.05) draws: x, x_dot, theta, theta_dot */
void or_cartpole_reset(or_cartpole *e, float *obs) {
    e->x = or_gen_range_f32(&e->rng, -0.05f, 0.05f);
    e->x_dot = or_gen_range_f32(&e->rng, -0.05f, 0.05f);
    e->theta = or_gen_range_f32(&e->rng, -0.05f, 0.05f);
    e->theta_dot = or_gen_range_f32(&e->rng, -0.05f, 0.05f);
    e->steps = 0;
    if (obs) or_cartpole_get_obs(e, obs);
}

/* cartpole.rs:92-106 — new() seeds StdRng and resets once. */
void or_cartpole_new(or_cartpole *e, uint64_t seed) {
    memset(e, 0, sizeof *e);
    or_rng_seed_u64(&e->rng, seed);
    or_cartpole_reset(e, NULL);
}

/* cartpole.rs:50-66 physics_step (mul_add == fmaf; powi(2) == x*x), then
 * cartpole.rs:283-301 step/is_terminal/reward. */
void or_cartpole_step(or_cartpole *e, int32_t action, float *obs, float *reward, int *done) {
    float force = action == 0 ? -CP_FORCE : CP_FORCE;
    float cos_t = cosf(e->theta);
    float sin_t = sinf(e->theta);
    float temp = fmaf(CP_MASS_LEN * (e->theta_dot * e->theta_dot), sin_t, force) / CP_TOTAL_MASS;
    float theta_acc = fmaf(CP_GRAVITY, sin_t, -(cos_t * temp)) /
                      (CP_HALF_LEN * (4.0f / 3.0f - CP_POLE_MASS * (cos_t * cos_t) / CP_TOTAL_MASS));
    float x_acc = temp - CP_MASS_LEN * theta_acc * cos_t / CP_TOTAL_MASS;
    e->x_dot += CP_TAU * x_acc;
    e->x += CP_TAU * e->x_dot;
    e->theta_dot += CP_TAU * theta_acc;
    e->theta += CP_TAU * e->theta_dot;
    e->steps += 1;
    int d = fabsf(e->x) > CP_X_THRESH || fabsf(e->theta) > cp_theta_threshold() ||
            e->steps >= CP_MAX_STEPS;
    *reward = (d && e->steps < CP_MAX_STEPS) ? 0.0f : 1.0f;
    *done = d;
    if (obs) or_cartpole_get_obs(e, obs);
}

/* ========================================================= Connect Four ==== */
/* envs/connect_four.rs:186-206: P1 plane, P2 plane (absolute), turn one-hot. */
void or_c4_get_obs(const or_connect_four *e, float *obs) {
    memset(obs, 0, sizeof(float) * OR_C4_OBS);
    for (int r = 0; r < 6; r++)
        for (int c = 0; c < 7; c++) {
            int idx = r * 7 + c;
            if (e->board[r][c] == 1) obs[idx] = 1.0f;
            else if (e->board[r][c] == 2) obs[42 + idx] = 1.0f;
        }
    obs[84 + (e->current - 1)] = 1.0f;
}

int or_c4_current_player(const or_connect_four *e) { return e->current - 1; }

/* connect_four.rs:225-240 new/reset (seed ignored). */
void or_c4_new(or_connect_four *e) {
    memset(e, 0, sizeof *e);
    e->current = 1;
}
void or_c4_reset(or_connect_four *e, float *obs) {
    or_c4_new(e);
    if (obs) or_c4_get_obs(e, obs);
}

/* connect_four.rs:126-170 */
static int c4_check_winner(const or_connect_four *e, int row, int col, int player) {
    static const int dirs[4][2] = {{0, 1}, {1, 0}, {1, 1}, {1, -1}};
    for (int d = 0; d < 4; d++) {
        int dr = dirs[d][0], dc = dirs[d][1], count = 1;
        for (int i = 1; i < 4; i++) {
            int r = row + dr * i, c = col + dc * i;
            if (r < 0 || r >= 6 || c < 0 || c >= 7) break;
            if (e->board[r][c] == player) count++; else break;
        }
        for (int i = 1; i < 4; i++) {
            int r = row - dr * i, c = col - dc * i;
            if (r < 0 || r >= 6 || c < 0 || c >= 7) break;
            if (e->board[r][c] == player) count++; else break;
        }
        if (count >= 4) return 1;
    }
    return 0;
}

/* connect_four.rs:249-283 (win +1/-1, draw 0/0, invalid -> done, no reward) */
void or_c4_step(or_connect_four *e, int32_t action, float *obs, float rewards[2], int *done) {
    int cur = e->current - 1, other = 1 - cur;
    rewards[0] = rewards[1] = 0.0f;
    if (action < 0 || action >= 7 || e->board[0][action] != 0 || e->game_over) {
        *done = 1;
        if (obs) or_c4_get_obs(e, obs);
        return;
    }
    int row = -1;
    for (int r = 5; r >= 0; r--)
        if (e->board[r][action] == 0) { e->board[r][action] = e->current; row = r; break; }
    if (row >= 0 && c4_check_winner(e, row, action, e->current)) {
        e->game_over = 1;
        e->winner = e->current;
        rewards[cur] = 1.0f;
        rewards[other] = -1.0f;
        *done = 1;
        if (obs) or_c4_get_obs(e, obs);
        return;
    }
    int full = 1;
    for (int c = 0; c < 7; c++) if (e->board[0][c] == 0) { full = 0; break; }
    if (full) {
        e->game_over = 1;
        *done = 1;
        if (obs) or_c4_get_obs(e, obs);
        return;
    }
    e->current = e->current == 1 ? 2 : 1;
    *done = 0;
    if (obs) or_c4_get_obs(e, obs);
}

/* connect_four.rs:289-295 */
void or_c4_mask(const or_connect_four *e, uint8_t mask[7]) {
    for (int c = 0; c < 7; c++) mask[c] = e->board[0][c] == 0;
}

/* =========================================================== Liar's Dice === */
#define LD_P OR_LD_PLAYERS
#define LD_D OR_LD_DICE

/* liars_dice.rs:191-197 */
static void ld_roll_all(or_liars_dice *e) {
    for (int p = 0; p < LD_P; p++)
        for (int d = 0; d < e->num_dice[p]; d++) e->dice[p][d] = or_gen_range_u8_incl(&e->rng, 1, 6);
}

static int ld_total_dice(const or_liars_dice *e) {
    int s = 0;
    for (int p = 0; p < LD_P; p++) s += e->num_dice[p];
    return s;
}

static int ld_alive(const or_liars_dice *e) {
    int s = 0;
    for (int p = 0; p < LD_P; p++) s += e->num_dice[p] > 0;
    return s;
}

/* liars_dice.rs:211-230 (wild 1s; bids on 1 count only 1s) */
static int ld_count(const or_liars_dice *e, int face) {
    int c = 0;
    for (int p = 0; p < LD_P; p++)
        for (int d = 0; d < e->num_dice[p]; d++) {
            int v = e->dice[p][d];
            if (face == 1 ? v == 1 : (v == face || v == 1)) c++;
        }
    return c;
}

/* liars_dice.rs:233-250 */
static int ld_valid_bid(const or_liars_dice *e, int q, int f) {
    if (q == 0 || q > ld_total_dice(e)) return 0;
    if (f == 0 || f > 6) return 0;
    if (!e->has_bid) return 1;
    return q > e->bid_qty || (q == e->bid_qty && f > e->bid_face);
}

/* liars_dice.rs:253-264 */
static int ld_next_alive(const or_liars_dice *e, int from) {
    int next = (from + 1) % LD_P;
    while (e->num_dice[next] == 0) {
        next = (next + 1) % LD_P;
        if (next == from) break;
    }
    return next;
}

/* liars_dice.rs:266-305 */
static void ld_start_new_round(or_liars_dice *e, int loser) {
    if (e->num_dice[loser] > 0) e->num_dice[loser]--;
    if (e->num_dice[loser] == 0) e->elim_order[e->num_elim++] = (int8_t)loser;
    if (ld_alive(e) <= 1) {
        e->game_over = 1;
        for (int p = 0; p < LD_P; p++)
            if (e->num_dice[p] > 0) { e->elim_order[e->num_elim++] = (int8_t)p; break; }
        return;
    }
    e->has_bid = 0; e->bid_qty = 0; e->bid_face = 0;
    e->last_bidder = -1;
    e->bid_count = 0;
    e->hist_len = 0;
    e->current = e->num_dice[loser] > 0 ? (uint8_t)loser : (uint8_t)ld_next_alive(e, loser);
    ld_roll_all(e);
}

/* liars_dice.rs:309-374 (relative indexing, 270 floats) */
void or_ld_get_obs(const or_liars_dice *e, float *obs) {
    memset(obs, 0, sizeof(float) * OR_LD_OBS);
    int cur = e->current, idx = 0;
    for (int d = 0; d < e->num_dice[cur]; d++) {
        obs[idx + e->dice[cur][d] - 1] = 1.0f;
        idx += 6;
    }
    idx = 12;
    for (int r = 0; r < LD_P; r++) obs[idx++] = (float)e->num_dice[(r + cur) % LD_P] / 2.0f;
    for (int r = 0; r < LD_P; r++) obs[idx++] = e->num_dice[(r + cur) % LD_P] > 0 ? 1.0f : 0.0f;
    obs[idx + cur] = 1.0f;
    idx += 4;
    if (e->has_bid) obs[idx + (e->bid_qty - 1) * 6 + (e->bid_face - 1)] = 1.0f;
    idx += 48;
    obs[idx++] = e->has_bid ? 1.0f : 0.0f;
    {
        float bc = (float)e->bid_count / 20.0f;
        obs[idx++] = bc < 1.0f ? bc : 1.0f;
    }
    if (e->last_bidder >= 0) obs[idx + (e->last_bidder + LD_P - cur) % LD_P] = 1.0f;
    idx += 4;
    /* liars_dice.rs:113-137 BidHistory::to_observation_relative */
    for (int i = 0; i < e->hist_len; i++) {
        int base = idx + i * 12;
        obs[base + (e->hist_player[i] + LD_P - cur) % LD_P] = 1.0f;
        obs[base + 4] = (float)e->hist_qty[i] / 8.0f;
        obs[base + 5 + (e->hist_face[i] - 1)] = 1.0f;
        obs[base + 11] = 1.0f;
    }
}

int or_ld_current_player(const or_liars_dice *e) { return e->current; }

/* liars_dice.rs:171-188 new_with_config (rolls once) */
void or_ld_new(or_liars_dice *e, uint64_t seed) {
    memset(e, 0, sizeof *e);
    for (int p = 0; p < LD_P; p++) e->num_dice[p] = LD_D;
    e->last_bidder = -1;
    or_rng_seed_u64(&e->rng, seed);
    ld_roll_all(e);
}

/* liars_dice.rs:464-478 reset (rolls again) */
void or_ld_reset(or_liars_dice *e, float *obs) {
    for (int p = 0; p < LD_P; p++) e->num_dice[p] = LD_D;
    e->current = 0;
    e->has_bid = 0; e->bid_qty = 0; e->bid_face = 0;
    e->last_bidder = -1;
    e->bid_count = 0;
    e->hist_len = 0;
    e->num_elim = 0;
    e->game_over = 0;
    ld_roll_all(e);
    if (obs) or_ld_get_obs(e, obs);
}

/* liars_dice.rs:481-551; shaping = reward_shaping_coef.get(step) as f32 */
void or_ld_step(or_liars_dice *e, int32_t action, float shaping, float *obs, float rewards[4],
                int *done) {
    for (int p = 0; p < LD_P; p++) rewards[p] = 0.0f;
    if (e->game_over || e->num_dice[e->current] == 0) {
        *done = 1;
        if (obs) or_ld_get_obs(e, obs);
        return;
    }
    if (action != 48) {
        int q = action / 6 + 1, f = action % 6 + 1;
        if (!ld_valid_bid(e, q, f)) {
            e->game_over = 1;
            *done = 1;
            if (obs) or_ld_get_obs(e, obs);
            return;
        }
        /* BidHistory::push: ring of 16, drop oldest */
        if (e->hist_len >= OR_LD_HIST) {
            memmove(e->hist_player, e->hist_player + 1, OR_LD_HIST - 1);
            memmove(e->hist_qty, e->hist_qty + 1, OR_LD_HIST - 1);
            memmove(e->hist_face, e->hist_face + 1, OR_LD_HIST - 1);
            e->hist_len = OR_LD_HIST - 1;
        }
        e->hist_player[e->hist_len] = e->current;
        e->hist_qty[e->hist_len] = (uint8_t)q;
        e->hist_face[e->hist_len] = (uint8_t)f;
        e->hist_len++;
        e->has_bid = 1; e->bid_qty = (uint8_t)q; e->bid_face = (uint8_t)f;
        e->last_bidder = (int8_t)e->current;
        e->bid_count++;
        e->current = (uint8_t)ld_next_alive(e, e->current);
        *done = 0;
        if (obs) or_ld_get_obs(e, obs);
        return;
    }
    if (!e->has_bid) {
        e->game_over = 1;
        *done = 1;
        if (obs) or_ld_get_obs(e, obs);
        return;
    }
    int actual = ld_count(e, e->bid_face);
    int caller_correct = actual < e->bid_qty;
    int caller = e->current, bidder = e->last_bidder;
    int loser = caller_correct ? bidder : caller;
    ld_start_new_round(e, loser);
    for (int p = 0; p < LD_P; p++)
        if (e->num_dice[p] > 0) rewards[p] += shaping;
    if (e->game_over) {
        static const float place_r[4] = {1.0f, 0.33f, -0.33f, -1.0f};
        for (int o = 0; o < e->num_elim; o++) {
            int placement = LD_P - o;
            rewards[e->elim_order[o]] = place_r[placement - 1];
        }
    }
    *done = e->game_over;
    if (obs) or_ld_get_obs(e, obs);
}

/* liars_dice.rs:557-580 */
void or_ld_mask(const or_liars_dice *e, uint8_t mask[49]) {
    memset(mask, 0, 49);
    if (e->num_dice[e->current] == 0 || e->game_over) return;
    mask[48] = e->has_bid ? 1 : 0;
    int maxq = ld_total_dice(e);
    for (int q = 1; q <= maxq; q++)
        for (int f = 1; f <= 6; f++)
            if (ld_valid_bid(e, q, f)) mask[(q - 1) * 6 + (f - 1)] = 1;
}

/* liars_dice.rs:639-739 (110 floats, zero-padded to 120) */
void or_ld_priv(const or_liars_dice *e, float *g) {
    int i = 0;
    memset(g, 0, sizeof(float) * OR_LD_PRIV);
    g[i++] = (float)e->current / 4.0f;
    if (e->has_bid) {
        g[i++] = (float)e->bid_qty / 8.0f;
        g[i++] = (float)e->bid_face / 6.0f;
    } else {
        g[i++] = 0.0f; g[i++] = 0.0f;
    }
    g[i++] = e->last_bidder >= 0 ? (float)e->last_bidder / 4.0f : -1.0f;
    g[i++] = (float)e->bid_count / 12.0f;
    for (int k = 0; k < OR_LD_HIST; k++) {
        if (k < e->hist_len) {
            int j = e->hist_len - 1 - k; /* newest first */
            g[i++] = (float)e->hist_player[j] / 4.0f;
            g[i++] = (float)e->hist_qty[j] / 8.0f;
            g[i++] = (float)e->hist_face[j] / 6.0f;
        } else {
            g[i++] = 0.0f; g[i++] = 0.0f; g[i++] = 0.0f;
        }
    }
    g[i++] = e->game_over ? 1.0f : 0.0f;
    for (int s = 0; s < LD_P; s++) {
        g[i++] = (float)e->num_dice[s] / 2.0f;
        g[i++] = e->num_dice[s] > 0 ? 1.0f : 0.0f;
        for (int d = 0; d < LD_D; d++) {
            for (int f = 1; f <= 6; f++)
                g[i++] = (d < e->num_dice[s] && e->dice[s][d] == f) ? 1.0f : 0.0f;
        }
    }
}

// bppo_envs.h — Connect Four and Liar's Dice on the device (one lane per env).
//
//  Connect Four: envs/connect_four.rs:105-295.  Board as two 42-bit planes
//  (bit r*7+c, row 0 = top) + player to move (1|2) + game-over flag.
//  Liar's Dice:  envs/liars_dice.rs:91-739.  4 players x 2 dice, bid history
//  ring of 16, each env's own StdRng(seed+i) read at a counter-addressed word
//  position (dice rolls: rand 0.8.5 gen_range(1u8..=6), rejection included).
// Observation rows are built in LDS by the owning lane and written out by the
// whole block (contiguous rows => coalesced stores), see k_wide.hip.
#pragma once
#include "bppo_device.h"

namespace bppo {

// ============================================================ Connect Four ==
constexpr int C4_OBS = 86, C4_ACT = 7;
struct C4State {
    uint64_t p[2];      // piece planes of Player1 / Player2
    int32_t cur;        // 1 or 2
    int32_t over;
};

__device__ __forceinline__ int c4_at(const C4State &s, int r, int c) {
    const uint64_t b = 1ull << (r * 7 + c);
    return (s.p[0] & b) ? 1 : ((s.p[1] & b) ? 2 : 0);
}

// connect_four.rs:126-170: count through the placed piece in 4 directions
__device__ __forceinline__ bool c4_check_winner(const C4State &s, int row, int col, int player) {
    const uint64_t mine = s.p[player - 1];
    const int dr[4] = {0, 1, 1, 1}, dc[4] = {1, 0, 1, -1};
#pragma unroll
    for (int d = 0; d < 4; d++) {
        int count = 1;
        for (int i = 1; i < 4; i++) {
            const int r = row + dr[d] * i, c = col + dc[d] * i;
            if (r < 0 || r >= 6 || c < 0 || c >= 7) break;
            if (mine & (1ull << (r * 7 + c))) count++; else break;
        }
        for (int i = 1; i < 4; i++) {
            const int r = row - dr[d] * i, c = col - dc[d] * i;
            if (r < 0 || r >= 6 || c < 0 || c >= 7) break;
            if (mine & (1ull << (r * 7 + c))) count++; else break;
        }
        if (count >= 4) return true;
    }
    return false;
}

__device__ __forceinline__ void c4_reset(C4State &s) { s.p[0] = s.p[1] = 0; s.cur = 1; s.over = 0; }

// connect_four.rs:249-283: win +1/-1 done, full board 0/0 done, invalid or full
// column: done with zero rewards, otherwise switch player
__device__ __forceinline__ void c4_step(C4State &s, int action, float r[2], int &done) {
    const int cur = s.cur - 1, other = 1 - cur;
    r[0] = r[1] = 0.0f;
    const uint64_t occ = s.p[0] | s.p[1];
    if (action < 0 || action >= 7 || (occ & (1ull << action)) || s.over) { done = 1; return; }
    int row = -1;
    for (int rr = 5; rr >= 0; rr--)
        if (!(occ & (1ull << (rr * 7 + action)))) { row = rr; break; }
    s.p[cur] |= 1ull << (row * 7 + action);
    if (c4_check_winner(s, row, action, s.cur)) {
        s.over = 1;
        r[cur] = 1.0f; r[other] = -1.0f;
        done = 1;
        return;
    }
    const uint64_t occ2 = s.p[0] | s.p[1];
    if ((occ2 & 0x7Full) == 0x7Full) { s.over = 1; done = 1; return; }
    s.cur = s.cur == 1 ? 2 : 1;
    done = 0;
}

// connect_four.rs:186-206 (absolute planes + turn one-hot); row pre-zeroed
__device__ __forceinline__ void c4_obs(const C4State &s, float *row) {
    for (int i = 0; i < 42; i++) {
        const uint64_t b = 1ull << i;
        if (s.p[0] & b) row[i] = 1.0f;
        else if (s.p[1] & b) row[42 + i] = 1.0f;
    }
    row[84 + (s.cur - 1)] = 1.0f;
}

__device__ __forceinline__ void c4_mask(const C4State &s, uint8_t *m) {
    const uint64_t occ = s.p[0] | s.p[1];
    for (int c = 0; c < 7; c++) m[c] = (occ & (1ull << c)) ? 0 : 1;
}

// ============================================================ Liar's Dice ===
constexpr int LD_P = 4, LD_D = 2, LD_OBS = 270, LD_ACT = 49, LD_PRIV = 120, LD_HIST = 16;
struct LDState {
    uint8_t dice[LD_P][LD_D];
    uint8_t num_dice[LD_P];
    uint8_t current, has_bid, bid_qty, bid_face;
    int8_t last_bidder;
    uint8_t hist_len, num_elim, game_over;
    int8_t elim_order[LD_P];
    int32_t bid_count;
    uint8_t hist_player[LD_HIST], hist_qty[LD_HIST], hist_face[LD_HIST];
    uint64_t rng_pos;      // word position of this env's StdRng(seed + i)
};

// rand 0.8.5 UniformInt<u8>::sample_single_inclusive(1, 6) (liars_dice.rs:194)
__device__ __forceinline__ uint8_t ld_roll(WordCursor &c) {
    const uint32_t range = 6u, zone = 0xFFFFFFFFu - ((0u - range) % range);
    for (;;) {
        const uint64_t m = (uint64_t)c.next() * range;
        if ((uint32_t)m <= zone) return (uint8_t)(1 + (uint32_t)(m >> 32));
    }
}

// liars_dice.rs:191-197
__device__ __forceinline__ void ld_roll_all(LDState &s, WordCursor &c) {
    for (int p = 0; p < LD_P; p++)
        for (int d = 0; d < s.num_dice[p]; d++) s.dice[p][d] = ld_roll(c);
}

__device__ __forceinline__ int ld_total(const LDState &s) {
    int t = 0;
    for (int p = 0; p < LD_P; p++) t += s.num_dice[p];
    return t;
}
__device__ __forceinline__ int ld_alive(const LDState &s) {
    int t = 0;
    for (int p = 0; p < LD_P; p++) t += s.num_dice[p] > 0;
    return t;
}
// liars_dice.rs:211-230 (1s wild; a bid on 1s counts only 1s)
__device__ __forceinline__ int ld_count(const LDState &s, int face) {
    int n = 0;
    for (int p = 0; p < LD_P; p++)
        for (int d = 0; d < s.num_dice[p]; d++) {
            const int v = s.dice[p][d];
            n += face == 1 ? (v == 1) : (v == face || v == 1);
        }
    return n;
}
// liars_dice.rs:233-250
__device__ __forceinline__ bool ld_valid_bid(const LDState &s, int total, int q, int f) {
    if (q == 0 || q > total) return false;
    if (f == 0 || f > 6) return false;
    if (!s.has_bid) return true;
    return q > s.bid_qty || (q == s.bid_qty && f > s.bid_face);
}
// liars_dice.rs:253-264
__device__ __forceinline__ int ld_next_alive(const LDState &s, int from) {
    int next = (from + 1) % LD_P;
    while (s.num_dice[next] == 0) {
        next = (next + 1) % LD_P;
        if (next == from) break;
    }
    return next;
}
// liars_dice.rs:266-305
__device__ __forceinline__ void ld_start_new_round(LDState &s, int loser, WordCursor &c) {
    if (s.num_dice[loser] > 0) s.num_dice[loser]--;
    if (s.num_dice[loser] == 0) s.elim_order[s.num_elim++] = (int8_t)loser;
    if (ld_alive(s) <= 1) {
        s.game_over = 1;
        for (int p = 0; p < LD_P; p++)
            if (s.num_dice[p] > 0) { s.elim_order[s.num_elim++] = (int8_t)p; break; }
        return;
    }
    s.has_bid = 0; s.bid_qty = 0; s.bid_face = 0;
    s.last_bidder = -1;
    s.bid_count = 0;
    s.hist_len = 0;
    s.current = s.num_dice[loser] > 0 ? (uint8_t)loser : (uint8_t)ld_next_alive(s, loser);
    ld_roll_all(s, c);
}

// liars_dice.rs:464-478 reset (rolls all dice)
__device__ __forceinline__ void ld_reset(LDState &s, WordCursor &c) {
    for (int p = 0; p < LD_P; p++) s.num_dice[p] = LD_D;
    s.current = 0; s.has_bid = 0; s.bid_qty = 0; s.bid_face = 0;
    s.last_bidder = -1; s.bid_count = 0; s.hist_len = 0; s.num_elim = 0; s.game_over = 0;
    ld_roll_all(s, c);
}

// liars_dice.rs:171-188 new_with_config: zeroed state, 2 dice each, first roll
__device__ __forceinline__ void ld_new(LDState &s, WordCursor &c) {
    uint8_t *raw = reinterpret_cast<uint8_t *>(&s);
    for (size_t i = 0; i < sizeof(LDState); i++) raw[i] = 0;
    for (int p = 0; p < LD_P; p++) s.num_dice[p] = LD_D;
    s.last_bidder = -1;
    ld_roll_all(s, c);
}

// liars_dice.rs:481-551; shaping = reward_shaping_coef.get(step) as f32
__device__ __forceinline__ void ld_step(LDState &s, int action, float shaping, float r[4], int &done,
                                        WordCursor &c) {
    for (int p = 0; p < LD_P; p++) r[p] = 0.0f;
    if (s.game_over || s.num_dice[s.current] == 0) { done = 1; return; }
    if (action != 48) {
        const int q = action / 6 + 1, f = action % 6 + 1;
        if (!ld_valid_bid(s, ld_total(s), q, f)) { s.game_over = 1; done = 1; return; }
        if (s.hist_len >= LD_HIST) {   // BidHistory::push drops the oldest
            for (int i = 0; i < LD_HIST - 1; i++) {
                s.hist_player[i] = s.hist_player[i + 1];
                s.hist_qty[i] = s.hist_qty[i + 1];
                s.hist_face[i] = s.hist_face[i + 1];
            }
            s.hist_len = LD_HIST - 1;
        }
        s.hist_player[s.hist_len] = s.current;
        s.hist_qty[s.hist_len] = (uint8_t)q;
        s.hist_face[s.hist_len] = (uint8_t)f;
        s.hist_len++;
        s.has_bid = 1; s.bid_qty = (uint8_t)q; s.bid_face = (uint8_t)f;
        s.last_bidder = (int8_t)s.current;
        s.bid_count++;
        s.current = (uint8_t)ld_next_alive(s, s.current);
        done = 0;
        return;
    }
    if (!s.has_bid) { s.game_over = 1; done = 1; return; }
    const int actual = ld_count(s, s.bid_face);
    const bool caller_correct = actual < s.bid_qty;
    const int loser = caller_correct ? s.last_bidder : s.current;
    ld_start_new_round(s, loser, c);
    for (int p = 0; p < LD_P; p++)
        if (s.num_dice[p] > 0) r[p] = __fadd_rn(r[p], shaping);
    if (s.game_over) {
        const float place_r[4] = {1.0f, 0.33f, -0.33f, -1.0f};
        for (int o = 0; o < s.num_elim; o++) r[s.elim_order[o]] = place_r[LD_P - o - 1];
    }
    done = s.game_over;
}

// liars_dice.rs:309-374 (relative seats, 270 floats); row pre-zeroed
__device__ __forceinline__ void ld_obs(const LDState &s, float *o) {
    const int cur = s.current;
    for (int d = 0; d < s.num_dice[cur]; d++) o[d * 6 + s.dice[cur][d] - 1] = 1.0f;
    int idx = 12;
    for (int r = 0; r < LD_P; r++) o[idx++] = __fdiv_rn((float)s.num_dice[(r + cur) % LD_P], 2.0f);
    for (int r = 0; r < LD_P; r++) o[idx++] = s.num_dice[(r + cur) % LD_P] > 0 ? 1.0f : 0.0f;
    o[idx + cur] = 1.0f;
    idx += 4;
    if (s.has_bid) o[idx + (s.bid_qty - 1) * 6 + (s.bid_face - 1)] = 1.0f;
    idx += 48;
    o[idx++] = s.has_bid ? 1.0f : 0.0f;
    const float bc = __fdiv_rn((float)s.bid_count, 20.0f);
    o[idx++] = bc < 1.0f ? bc : 1.0f;
    if (s.last_bidder >= 0) o[idx + (s.last_bidder + LD_P - cur) % LD_P] = 1.0f;
    idx += 4;
    for (int i = 0; i < s.hist_len; i++) {   // BidHistory::to_observation_relative (113-137)
        const int base = idx + i * 12;
        o[base + (s.hist_player[i] + LD_P - cur) % LD_P] = 1.0f;
        o[base + 4] = __fdiv_rn((float)s.hist_qty[i], 8.0f);
        o[base + 5 + (s.hist_face[i] - 1)] = 1.0f;
        o[base + 11] = 1.0f;
    }
}

// liars_dice.rs:557-580
__device__ __forceinline__ void ld_mask(const LDState &s, uint8_t *m) {
    for (int a = 0; a < LD_ACT; a++) m[a] = 0;
    if (s.num_dice[s.current] == 0 || s.game_over) return;
    m[48] = s.has_bid ? 1 : 0;
    const int total = ld_total(s);
    for (int q = 1; q <= total; q++)
        for (int f = 1; f <= 6; f++)
            if (ld_valid_bid(s, total, q, f)) m[(q - 1) * 6 + (f - 1)] = 1;
}

// liars_dice.rs:639-739 privileged obs (110 floats, zero-padded to 120); row pre-zeroed
__device__ __forceinline__ void ld_priv(const LDState &s, float *g) {
    int i = 0;
    g[i++] = __fdiv_rn((float)s.current, 4.0f);
    if (s.has_bid) {
        g[i++] = __fdiv_rn((float)s.bid_qty, 8.0f);
        g[i++] = __fdiv_rn((float)s.bid_face, 6.0f);
    } else {
        i += 2;
    }
    g[i++] = s.last_bidder >= 0 ? __fdiv_rn((float)s.last_bidder, 4.0f) : -1.0f;
    g[i++] = __fdiv_rn((float)s.bid_count, 12.0f);
    for (int k = 0; k < LD_HIST; k++) {
        if (k < s.hist_len) {
            const int j = s.hist_len - 1 - k;   // newest first
            g[i++] = __fdiv_rn((float)s.hist_player[j], 4.0f);
            g[i++] = __fdiv_rn((float)s.hist_qty[j], 8.0f);
            g[i++] = __fdiv_rn((float)s.hist_face[j], 6.0f);
        } else {
            i += 3;
        }
    }
    g[i++] = s.game_over ? 1.0f : 0.0f;
    for (int p = 0; p < LD_P; p++) {
        g[i++] = __fdiv_rn((float)s.num_dice[p], 2.0f);
        g[i++] = s.num_dice[p] > 0 ? 1.0f : 0.0f;
        for (int d = 0; d < LD_D; d++)
            for (int f = 1; f <= 6; f++) g[i++] = (d < s.num_dice[p] && s.dice[p][d] == f) ? 1.0f : 0.0f;
    }
}

}  // namespace bppo

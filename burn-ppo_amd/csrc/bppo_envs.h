// bppo_envs.h — Connect Four and Liar's Dice on the device (one lane per env).
//
//  Connect Four: envs/connect_four.rs:105-295.  Board as two 42-bit planes
//  (bit r*7+c, row 0 = top) + player to move (1|2) + game-over flag.
//  Liar's Dice:  envs/liars_dice.rs:91-739.  4 players x 2 dice, bid history
//  ring of 16, each env's own StdRng(seed+i) read at a counter-addressed word
//  position (dice rolls: rand 0.8.5 gen_range(1u8..=6), rejection included).
//  Skull:        envs/skull.rs:118-1605.  2-6 players (num_players kept in the
//  state), MAX_PLAYERS = 6 seat slots; stacks as a length + skull bitmask
//  (bottom first); lose_coaster's gen_range(0..total) over usize from the env's
//  StdRng(seed+i) at a counter-addressed word position.
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

// ================================================================== Skull ==
constexpr int SK_P = 6, SK_CARDS = 4, SK_ROSES = 3, SK_MAXBID = 24, SK_WINS = 2;
constexpr int SK_OBS = 135, SK_ACT = 33, SK_PRIV = 200, SK_HIST = 8;
constexpr int SK_PASS = 2 + SK_MAXBID, SK_REVEAL0 = SK_PASS + 1;
enum { SK_PLACING = 0, SK_BIDDING = 1, SK_REVEALING = 2 };
struct SKState {
    uint8_t n;                            // num_players
    uint8_t phase, current, round_starter, current_bid, hist_len, roses_found, must_reveal, num_elim, game_over;
    int8_t bidder, last_skull, winner;    // -1: None
    uint8_t has_trap[SK_P], rose[SK_P], wins[SK_P], slen[SK_P], sbits[SK_P], passed[SK_P], revealed[SK_P];
    uint8_t hist_player[SK_HIST], hist_bid[SK_HIST];   // bid 0 = pass
    int8_t elim[SK_P];
};

// rand 0.8.5 UniformInt<u64>::sample_single(0, range) (usize on 64-bit): next_u64
// (two words, low first), 64x64 -> 128 multiply, zone (range << lz) - 1
__device__ __forceinline__ uint64_t sk_gen_range_u64(WordCursor &c, uint64_t range) {
    const uint64_t zone = (range << __clzll((long long)range)) - 1ull;
    for (;;) {
        const uint64_t lo32 = c.next(), hi32 = c.next();
        const uint64_t v = (hi32 << 32) | lo32;
        const uint64_t lo = v * range, hi = __umul64hi(v, range);
        if (lo <= zone) return hi;
    }
}

__device__ __forceinline__ bool sk_alive(const SKState &s, int p) {          // skull.rs:204-206
    return p < s.n && (s.has_trap[p] || s.rose[p] > 0);
}
__device__ __forceinline__ int sk_coasters(const SKState &s, int p) {        // :209-215
    return p >= s.n ? 0 : (int)s.has_trap[p] + (int)s.rose[p];
}
__device__ __forceinline__ int sk_alive_count(const SKState &s) {
    int c = 0;
    for (int p = 0; p < s.n; p++) c += sk_alive(s, p);
    return c;
}
__device__ __forceinline__ int sk_next_alive(const SKState &s, int from) {    // :223-236
    int next = (from + 1) % s.n;
    const int start = next;
    for (;;) {
        if (sk_alive(s, next)) return next;
        next = (next + 1) % s.n;
        if (next == start) return from;
    }
}
__device__ __forceinline__ int sk_next_non_passed(const SKState &s, int from) {   // :239-251, -1 = None
    int next = (from + 1) % s.n;
    const int start = next;
    for (;;) {
        if (sk_alive(s, next) && !s.passed[next]) return next;
        next = (next + 1) % s.n;
        if (next == start) return -1;
    }
}
__device__ __forceinline__ int sk_non_passed(const SKState &s) {
    int c = 0;
    for (int p = 0; p < s.n; p++) c += sk_alive(s, p) && !s.passed[p];
    return c;
}
__device__ __forceinline__ int sk_total(const SKState &s) {
    int t = 0;
    for (int p = 0; p < s.n; p++) t += s.slen[p];
    return t;
}
__device__ __forceinline__ int sk_skulls(const SKState &s, int p) { return __popc(s.sbits[p] & ((1u << s.slen[p]) - 1u)); }
__device__ __forceinline__ bool sk_trap_in_hand(const SKState &s, int p) { return s.has_trap[p] && sk_skulls(s, p) == 0; }
__device__ __forceinline__ int sk_roses_in_hand(const SKState &s, int p) {    // :271-277 (saturating)
    const int in_stack = s.slen[p] - sk_skulls(s, p);
    return s.rose[p] > in_stack ? s.rose[p] - in_stack : 0;
}
__device__ __forceinline__ int sk_unrevealed(const SKState &s, int p) {
    return s.slen[p] > s.revealed[p] ? s.slen[p] - s.revealed[p] : 0;
}

__device__ __forceinline__ void sk_start_round(SKState &s, int starter) {    // :379-401
    for (int i = 0; i < SK_P; i++) { s.slen[i] = 0; s.sbits[i] = 0; s.passed[i] = 0; s.revealed[i] = 0; }
    s.phase = SK_PLACING; s.current_bid = 0; s.bidder = -1; s.hist_len = 0;
    s.roses_found = 0; s.must_reveal = 0; s.last_skull = -1;
    s.current = (uint8_t)(sk_alive(s, starter) ? starter : sk_next_alive(s, starter));
    s.round_starter = s.current;
}
__device__ __forceinline__ void sk_hist_push(SKState &s, int player, int bid, bool drop_oldest) {
    if (drop_oldest && s.hist_len >= SK_HIST) {   // VecDeque::pop_front
        for (int i = 0; i < SK_HIST - 1; i++) { s.hist_player[i] = s.hist_player[i + 1]; s.hist_bid[i] = s.hist_bid[i + 1]; }
        s.hist_len--;
    }
    s.hist_player[s.hist_len] = (uint8_t)player;
    s.hist_bid[s.hist_len] = (uint8_t)bid;
    s.hist_len++;
}
__device__ __forceinline__ void sk_to_revealing(SKState &s) {               // :695-705
    s.phase = SK_REVEALING; s.current = (uint8_t)s.bidder; s.must_reveal = 1; s.roses_found = 0;
    for (int i = 0; i < SK_P; i++) s.revealed[i] = 0;
}
__device__ __forceinline__ void sk_check_bidding_end(SKState &s) {          // :708-720
    if (sk_non_passed(s) == 1) {
        int b = -1;
        for (int p = 0; p < s.n && b < 0; p++)
            if (sk_alive(s, p) && !s.passed[p]) b = p;
        s.bidder = (int8_t)b;
        sk_to_revealing(s);
    } else {
        const int next = sk_next_non_passed(s, s.current);
        if (next >= 0) s.current = (uint8_t)next;
    }
}

// :472-529 competition ranking on (is_winner, wins, coasters, elimination rank)
__device__ __forceinline__ void sk_placements(const SKState &s, int pl[SK_P]) {
    int key[SK_P][4];
    for (int p = 0; p < s.n; p++) {
        int er = s.num_elim;
        for (int k = s.num_elim - 1; k >= 0; k--)
            if (s.elim[k] == p) er = k;
        key[p][0] = s.winner == p; key[p][1] = s.wins[p]; key[p][2] = sk_coasters(s, p); key[p][3] = er;
    }
    for (int p = 0; p < s.n; p++) {
        int better = 0;
        for (int q = 0; q < s.n; q++) {
            int c = 0;
            for (int k = 0; k < 4 && c == 0; k++) c = (key[q][k] > key[p][k]) - (key[q][k] < key[p][k]);
            better += c > 0;
        }
        pl[p] = 1 + better;
    }
}
// :406-443 reward(pl) = 1 - 2 (pl - 1) / (n - 1), averaged over a tie group (f32)
__device__ __forceinline__ void sk_final_rewards(const SKState &s, float r[SK_P]) {
    int pl[SK_P];
    sk_placements(s, pl);
    const int n = s.n;
    for (int p = 0; p < SK_P; p++) r[p] = 0.0f;
    for (int p = 0; p < n; p++) {
        int g = 0;
        for (int q = 0; q < n; q++) g += pl[q] == pl[p];
        float total = 0.0f;
        for (int o = 0; o < g; o++) {
            const float ep = (float)(pl[p] + o);
            total = __fadd_rn(total, n > 1 ? __fsub_rn(1.0f, __fdiv_rn(__fmul_rn(2.0f, __fsub_rn(ep, 1.0f)),
                                                                        __fsub_rn((float)n, 1.0f)))
                                           : 0.0f);
        }
        r[p] = __fdiv_rn(total, (float)g);
    }
}

// skull.rs:1067-1097 reset (the env RNG is not reseeded); n from new_with_players
__device__ __forceinline__ void sk_reset(SKState &s, int n) {
    s.n = (uint8_t)n;
    for (int i = 0; i < SK_P; i++) {
        s.has_trap[i] = i < n; s.rose[i] = i < n ? SK_ROSES : 0; s.wins[i] = 0;
        s.slen[i] = 0; s.sbits[i] = 0; s.passed[i] = 0; s.revealed[i] = 0; s.elim[i] = -1;
    }
    for (int i = 0; i < SK_HIST; i++) { s.hist_player[i] = 0; s.hist_bid[i] = 0; }
    s.phase = SK_PLACING; s.current = 0; s.round_starter = 0; s.current_bid = 0; s.bidder = -1;
    s.hist_len = 0; s.roses_found = 0; s.must_reveal = 0; s.last_skull = -1;
    s.num_elim = 0; s.game_over = 0; s.winner = -1;
}

// skull.rs:1254-1336
__device__ __forceinline__ void sk_mask(const SKState &s, uint8_t *m) {
    for (int a = 0; a < SK_ACT; a++) m[a] = 0;
    if (s.game_over) return;
    const int p = s.current;
    if (s.phase == SK_PLACING) {
        if (sk_trap_in_hand(s, p)) m[0] = 1;
        if (sk_roses_in_hand(s, p) > 0) m[1] = 1;
        if (s.slen[p] > 0) {
            const int tc = sk_total(s), lo = s.current_bid + 1 > 1 ? s.current_bid + 1 : 1;
            for (int b = lo; b <= tc; b++) m[2 + b - 1] = 1;
        }
    } else if (s.phase == SK_BIDDING) {
        const int tc = sk_total(s);
        for (int b = s.current_bid + 1; b <= tc; b++) m[2 + b - 1] = 1;
        if (!s.passed[p] && sk_non_passed(s) > 1) m[SK_PASS] = 1;
    } else if (p == s.bidder) {
        const int b = s.bidder;
        if (s.must_reveal && sk_unrevealed(s, b) > 0) {
            m[SK_REVEAL0 + b] = 1;
        } else {
            if (sk_unrevealed(s, b) > 0) m[SK_REVEAL0 + b] = 1;
            for (int q = 0; q < s.n; q++)
                if (q != b && sk_unrevealed(s, q) > 0) m[SK_REVEAL0 + q] = 1;
        }
    }
}

// skull.rs:1103-1252.  r[SK_P] (seats >= n stay 0, env.rs:477); shaping =
// reward_shaping_coef.get(step) as f32; an action outside the mask (a panic
// in the reference) sets *bad and leaves the state unchanged
__device__ __forceinline__ void sk_step(SKState &s, int action, float shaping, float r[SK_P], int &done, int &bad,
                                        WordCursor &c) {
    for (int p = 0; p < SK_P; p++) r[p] = 0.0f;
    bad = 0;
    if (s.game_over) { done = 1; return; }
    const int pl = s.current;
    uint8_t m[SK_ACT];
    sk_mask(s, m);
    if (action < 0 || action >= SK_ACT || !m[action]) { bad = 1; done = 0; return; }
    if (s.phase == SK_PLACING) {
        if (action == 0 || action == 1) {
            if (action == 0) s.sbits[pl] |= (uint8_t)(1u << s.slen[pl]);
            s.slen[pl]++;
            s.current = (uint8_t)sk_next_alive(s, pl);
        } else if (action < SK_PASS) {                    // transition_to_bidding (:673-692)
            const int bid = action - 1;
            s.phase = SK_BIDDING; s.current_bid = (uint8_t)bid; s.bidder = (int8_t)pl;
            sk_hist_push(s, pl, bid, false);
            if (bid == sk_total(s)) sk_to_revealing(s);
            else {
                const int next = sk_next_non_passed(s, pl);
                if (next >= 0) s.current = (uint8_t)next;
                else sk_check_bidding_end(s);
            }
        }
    } else if (s.phase == SK_BIDDING) {
        if (action >= 2 && action < SK_PASS) {
            const int bid = action - 1;
            s.current_bid = (uint8_t)bid; s.bidder = (int8_t)pl;
            sk_hist_push(s, pl, bid, true);
            if (bid == sk_total(s)) sk_to_revealing(s);
            else {
                const int next = sk_next_non_passed(s, pl);
                if (next >= 0) s.current = (uint8_t)next;
                else sk_check_bidding_end(s);
            }
        } else if (action == SK_PASS) {
            s.passed[pl] = 1;
            sk_hist_push(s, pl, 0, true);
            sk_check_bidding_end(s);
        }
    } else {
        const int bidder = s.bidder, target = action - SK_REVEAL0;
        const int idx = s.slen[target] - 1 - s.revealed[target];       // reveal_card (:293-302)
        const bool skull = (s.sbits[target] >> idx) & 1u;
        s.revealed[target]++;
        if (!skull) s.roses_found++;
        if (target == bidder && sk_unrevealed(s, bidder) == 0) s.must_reveal = 0;
        if (skull) {
            s.last_skull = (int8_t)target;
            const int total = sk_coasters(s, bidder);                  // lose_coaster (:305-323)
            if (total > 0) {
                const uint64_t choice = sk_gen_range_u64(c, (uint64_t)total);
                if (s.has_trap[bidder] && choice == 0) s.has_trap[bidder] = 0;
                else s.rose[bidder]--;
                if (sk_coasters(s, bidder) == 0) s.elim[s.num_elim++] = (int8_t)bidder;
            }
            if (shaping > 0.0f) r[bidder] = __fsub_rn(r[bidder], __fmul_rn(0.25f, shaping));   // :446-462
            if (sk_alive_count(s) <= 1) {
                s.game_over = 1;
                s.winner = -1;
                for (int p = 0; p < s.n && s.winner < 0; p++)
                    if (sk_alive(s, p)) s.winner = (int8_t)p;
                sk_final_rewards(s, r);
            } else {
                const int nxt = sk_alive(s, bidder) ? bidder : (sk_alive(s, target) ? target : sk_next_alive(s, target));
                sk_start_round(s, nxt);
            }
        } else if (s.roses_found >= s.current_bid) {
            s.wins[bidder]++;
            if (shaping > 0.0f) r[bidder] = __fadd_rn(r[bidder], shaping);
            if (s.wins[bidder] >= SK_WINS || sk_alive_count(s) == 1) {
                s.game_over = 1;
                s.winner = (int8_t)bidder;
                sk_final_rewards(s, r);
            } else {
                sk_start_round(s, bidder);
            }
        }
    }
    done = s.game_over;
}

// skull.rs:533-670 (relative seats, 135 floats); row pre-zeroed
__device__ __forceinline__ void sk_obs(const SKState &s, float *o) {
    const int pl = s.current, n = s.n;
    o[0] = sk_trap_in_hand(s, pl) ? 1.0f : 0.0f;
    const int rh = sk_roses_in_hand(s, pl);
    for (int i = 0; i < SK_ROSES; i++) o[1 + i] = i < rh ? 1.0f : 0.0f;
    for (int i = 0; i < SK_CARDS && i < s.slen[pl]; i++) o[4 + i] = ((s.sbits[pl] >> i) & 1u) ? 1.0f : 0.0f;
    for (int r = 0; r < SK_P && r < n; r++) {
        const int a = (r + pl) % n;
        o[8 + r] = __fdiv_rn((float)s.slen[a], 4.0f);
        o[14 + r] = __fdiv_rn((float)sk_coasters(s, a), 4.0f);
        o[20 + r] = sk_alive(s, a) ? 1.0f : 0.0f;
        o[26 + r] = 1.0f;
        o[48 + r] = s.passed[a] ? 1.0f : 0.0f;
        o[54 + r] = __fdiv_rn((float)s.wins[a], 2.0f);
        o[60 + r] = __fdiv_rn((float)s.revealed[a], 4.0f);
    }
    o[32 + pl] = 1.0f;
    o[38 + s.phase] = 1.0f;
    o[41] = __fdiv_rn((float)s.current_bid, 24.0f);
    if (s.bidder >= 0) o[42 + (s.bidder + n - pl) % n] = 1.0f;
    if (n >= 2 && n <= SK_P) o[66 + n - 2] = 1.0f;
    for (int i = 0; i < s.hist_len; i++) {
        const int b = 71 + i * (SK_P + 2);
        o[b + (s.hist_player[i] + n - pl) % n] = 1.0f;
        if (s.hist_bid[i] == 0) o[b + SK_P + 1] = 1.0f;
        else o[b + SK_P] = __fdiv_rn((float)s.hist_bid[i], 24.0f);
    }
}

// skull.rs:1480-1605 privileged obs (103 floats, zero-padded to 200); row pre-zeroed
__device__ __forceinline__ void sk_priv(const SKState &s, float *g) {
    int k = 0;
    g[k + s.phase] = 1.0f; k += 3;
    g[k++] = __fdiv_rn((float)s.current, 6.0f);
    g[k++] = __fdiv_rn((float)s.round_starter, 6.0f);
    if (s.current_bid > 0) {
        g[k++] = __fdiv_rn((float)s.current_bid, 24.0f);
        g[k++] = s.bidder >= 0 ? __fdiv_rn((float)s.bidder, 6.0f) : -1.0f;
    } else {
        g[k++] = 0.0f;
        g[k++] = -1.0f;
    }
    const int hl = s.hist_len < 10 ? s.hist_len : 10;
    for (int i = 0; i < hl; i++) {                                  // newest first
        const int j = s.hist_len - 1 - i;
        g[k + 3 * i] = __fdiv_rn((float)s.hist_player[j], 6.0f);
        g[k + 3 * i + 1] = __fdiv_rn((float)s.hist_bid[j], 24.0f);
        g[k + 3 * i + 2] = s.hist_bid[j] == 0 ? 1.0f : 0.0f;
    }
    k += 30;
    g[k++] = s.game_over ? 1.0f : 0.0f;
    for (int i = 2; i <= SK_P; i++) g[k++] = s.n == i ? 1.0f : 0.0f;
    for (int p = 0; p < SK_P; p++) {
        const int sk = sk_skulls(s, p);
        g[k++] = p < s.n ? 1.0f : 0.0f;
        g[k++] = __fdiv_rn((float)s.wins[p], 2.0f);
        g[k++] = (s.has_trap[p] || s.rose[p] > 0) ? 1.0f : 0.0f;
        g[k++] = s.has_trap[p] ? 1.0f : 0.0f;
        g[k++] = __fdiv_rn((float)s.rose[p], 3.0f);
        g[k++] = __fdiv_rn((float)s.slen[p], 4.0f);
        g[k++] = __fdiv_rn((float)sk, 4.0f);
        g[k++] = __fdiv_rn((float)(s.slen[p] - sk), 4.0f);
        g[k++] = s.passed[p] ? 1.0f : 0.0f;
        g[k++] = __fdiv_rn((float)s.revealed[p], 4.0f);
    }
}

}  // namespace bppo

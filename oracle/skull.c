/*
 * skull.c — Skull & Roses, 2-6 players (envs/skull.rs).  TEST INFRASTRUCTURE ONLY.
 *
 * Player-indexed arrays hold MAX_PLAYERS = 6 slots; seats >= num_players do not
 * exist (no coasters).  A stack is bottom-first (push = place, skull.rs:287-289);
 * revealing takes the top unrevealed card (skull.rs:293-302).  The env RNG is
 * StdRng::seed_from_u64(seed) (skull.rs:186), used only by lose_coaster's
 * gen_range(0..total) over usize (skull.rs:312).
 */
#include <string.h>
#include "oracle.h"

enum { SK_PLACING = 0, SK_BIDDING = 1, SK_REVEALING = 2 };
#define SK_PASS (2 + OR_SK_MAXBID)           /* 26 */
#define SK_REVEAL0 (SK_PASS + 1)             /* 27 .. 32 */

/* skull.rs:204-206 */
static int is_alive(const or_skull *e, int p) {
    return p < e->n && (e->has_trap[p] || e->rose_count[p] > 0);
}
/* skull.rs:209-215 */
static int coaster_count(const or_skull *e, int p) {
    return p >= e->n ? 0 : (int)e->has_trap[p] + (int)e->rose_count[p];
}
/* skull.rs:218-220 */
static int alive_count(const or_skull *e) {
    int c = 0;
    for (int p = 0; p < e->n; p++) c += is_alive(e, p);
    return c;
}
/* skull.rs:223-236 */
static int next_alive(const or_skull *e, int from) {
    int next = (from + 1) % e->n;
    const int start = next;
    for (;;) {
        if (is_alive(e, next)) return next;
        next = (next + 1) % e->n;
        if (next == start) return from;
    }
}
/* skull.rs:239-251: -1 = None */
static int next_non_passed(const or_skull *e, int from) {
    int next = (from + 1) % e->n;
    const int start = next;
    for (;;) {
        if (is_alive(e, next) && !e->passed[next]) return next;
        next = (next + 1) % e->n;
        if (next == start) return -1;
    }
}
/* skull.rs:254-258 */
static int non_passed_count(const or_skull *e) {
    int c = 0;
    for (int p = 0; p < e->n; p++) c += is_alive(e, p) && !e->passed[p];
    return c;
}
/* skull.rs:261-263 */
static int total_cards(const or_skull *e) {
    int t = 0;
    for (int p = 0; p < e->n; p++) t += e->stack_len[p];
    return t;
}
static int skulls_in_stack(const or_skull *e, int p) {
    int c = 0;
    for (int i = 0; i < e->stack_len[p]; i++) c += e->stack[p][i];
    return c;
}
/* skull.rs:266-268 */
static int trap_in_hand(const or_skull *e, int p) { return e->has_trap[p] && skulls_in_stack(e, p) == 0; }
/* skull.rs:271-277 (saturating) */
static int roses_in_hand(const or_skull *e, int p) {
    const int in_stack = e->stack_len[p] - skulls_in_stack(e, p);
    return e->rose_count[p] > in_stack ? e->rose_count[p] - in_stack : 0;
}
/* skull.rs:280-284 */
static int unrevealed(const or_skull *e, int p) {
    return e->stack_len[p] > e->revealed[p] ? e->stack_len[p] - e->revealed[p] : 0;
}

/* skull.rs:293-302 -> 1 if the revealed card is the skull */
static int reveal_card(or_skull *e, int p) {
    const int idx = e->stack_len[p] - 1 - e->revealed[p];
    const int skull = e->stack[p][idx];
    e->revealed[p]++;
    if (!skull) e->roses_found++;
    return skull;
}

/* skull.rs:305-323 */
static void lose_coaster(or_skull *e, int p) {
    const int total = coaster_count(e, p);
    if (total == 0) return;
    const uint64_t choice = or_gen_range_u64(&e->rng, 0, (uint64_t)total);
    if (e->has_trap[p] && choice == 0) e->has_trap[p] = 0;
    else e->rose_count[p]--;
    if (coaster_count(e, p) == 0) e->elim_order[e->num_elim++] = (int8_t)p;
}

/* skull.rs:379-401 */
static void start_new_round(or_skull *e, int starter) {
    for (int i = 0; i < OR_SK_MAXP; i++) { e->stack_len[i] = 0; e->passed[i] = 0; e->revealed[i] = 0; }
    e->phase = SK_PLACING;
    e->current_bid = 0;
    e->current_bidder = -1;
    e->hist_len = 0;
    e->roses_found = 0;
    e->must_reveal_own = 0;
    e->last_skull_owner = -1;
    e->current = is_alive(e, starter) ? starter : next_alive(e, starter);
    e->round_starter = e->current;
}

static void hist_push(or_skull *e, int player, int bid, int drop_oldest) {
    if (drop_oldest && e->hist_len >= OR_SK_HIST) {          /* VecDeque::pop_front */
        memmove(e->hist_player, e->hist_player + 1, OR_SK_HIST - 1);
        memmove(e->hist_bid, e->hist_bid + 1, OR_SK_HIST - 1);
        e->hist_len--;
    }
    e->hist_player[e->hist_len] = (uint8_t)player;
    e->hist_bid[e->hist_len] = (uint8_t)bid;
    e->hist_len++;
}

/* skull.rs:695-705 */
static void to_revealing(or_skull *e) {
    e->phase = SK_REVEALING;
    e->current = e->current_bidder;
    e->must_reveal_own = 1;
    e->roses_found = 0;
    for (int i = 0; i < OR_SK_MAXP; i++) e->revealed[i] = 0;
}

/* skull.rs:708-720 */
static void check_bidding_end(or_skull *e) {
    if (non_passed_count(e) == 1) {
        int b = -1;
        for (int p = 0; p < e->n && b < 0; p++)
            if (is_alive(e, p) && !e->passed[p]) b = p;
        e->current_bidder = b;
        to_revealing(e);
    } else {
        const int next = next_non_passed(e, e->current);
        if (next >= 0) e->current = next;
    }
}

/* skull.rs:673-692 */
static void to_bidding(or_skull *e, int bidder, int bid) {
    e->phase = SK_BIDDING;
    e->current_bid = bid;
    e->current_bidder = bidder;
    hist_push(e, bidder, bid, 0);
    if (bid == total_cards(e)) {
        to_revealing(e);
    } else {
        const int next = next_non_passed(e, bidder);
        if (next >= 0) e->current = next;
        else check_bidding_end(e);
    }
}

/* skull.rs:472-529 competition ranking (1224): 1 + #players strictly better on
 * (is_winner, wins, coasters, elimination rank) */
static void placements(const or_skull *e, int out[OR_SK_MAXP]) {
    int key[OR_SK_MAXP][4];
    for (int p = 0; p < e->n; p++) {
        int er = e->num_elim;
        for (int k = 0; k < e->num_elim; k++)
            if (e->elim_order[k] == p) { er = k; break; }
        key[p][0] = e->winner == p; key[p][1] = e->wins[p]; key[p][2] = coaster_count(e, p); key[p][3] = er;
    }
    for (int p = 0; p < e->n; p++) {
        int better = 0;
        for (int q = 0; q < e->n; q++) {
            int c = 0;
            for (int k = 0; k < 4 && c == 0; k++) c = (key[q][k] > key[p][k]) - (key[q][k] < key[p][k]);
            better += c > 0;
        }
        out[p] = 1 + better;
    }
}

/* skull.rs:406-443: reward(pl) = 1 - 2 (pl - 1) / (n - 1), averaged over a tie group */
static void final_rewards(const or_skull *e, float r[OR_SK_MAXP]) {
    int pl[OR_SK_MAXP];
    placements(e, pl);
    const int n = e->n;
    for (int p = 0; p < n; p++) {
        int g = 0;
        for (int q = 0; q < n; q++) g += pl[q] == pl[p];
        float total = 0.0f;
        for (int o = 0; o < g; o++) {
            const float ep = (float)(pl[p] + o);
            total += n > 1 ? 1.0f - 2.0f * (ep - 1.0f) / ((float)n - 1.0f) : 0.0f;
        }
        r[p] = total / (float)g;
    }
    for (int p = n; p < OR_SK_MAXP; p++) r[p] = 0.0f;
}

/* skull.rs:446-462 */
static void round_rewards(int success, int bidder, float rsc, float r[OR_SK_MAXP]) {
    for (int p = 0; p < OR_SK_MAXP; p++) r[p] = 0.0f;
    if (rsc > 0.0f) {
        if (success) r[bidder] += rsc;
        else r[bidder] -= 1.0f / (float)OR_SK_CARDS * rsc;
    }
}

/* skull.rs:158-201 new_with_players */
void or_skull_new(or_skull *e, int num_players, uint64_t seed) {
    memset(e, 0, sizeof *e);
    e->n = num_players;
    for (int i = 0; i < OR_SK_MAXP; i++) {
        e->has_trap[i] = i < num_players;
        e->rose_count[i] = i < num_players ? OR_SK_ROSES : 0;
    }
    e->phase = SK_PLACING;
    e->current_bidder = -1;
    e->last_skull_owner = -1;
    e->winner = -1;
    or_rng_seed_u64(&e->rng, seed);
}

/* skull.rs:1067-1097 (the RNG is not reseeded) */
void or_skull_reset(or_skull *e, float *obs) {
    for (int i = 0; i < OR_SK_MAXP; i++) {
        e->has_trap[i] = i < e->n;
        e->rose_count[i] = i < e->n ? OR_SK_ROSES : 0;
        e->wins[i] = 0; e->stack_len[i] = 0; e->passed[i] = 0; e->revealed[i] = 0;
    }
    e->phase = SK_PLACING;
    e->current = 0; e->round_starter = 0;
    e->current_bid = 0; e->current_bidder = -1;
    e->hist_len = 0; e->roses_found = 0; e->must_reveal_own = 0; e->last_skull_owner = -1;
    e->num_elim = 0; e->game_over = 0; e->winner = -1;
    if (obs) or_skull_get_obs(e, obs);
}

int or_skull_current_player(const or_skull *e) { return e->current; }

/* skull.rs:1254-1336 */
void or_skull_mask(const or_skull *e, uint8_t m[OR_SK_ACT]) {
    memset(m, 0, OR_SK_ACT);
    if (e->game_over) return;
    const int p = e->current;
    if (e->phase == SK_PLACING) {
        if (trap_in_hand(e, p)) m[0] = 1;
        if (roses_in_hand(e, p) > 0) m[1] = 1;
        if (e->stack_len[p] > 0) {
            const int tc = total_cards(e);
            const int lo = e->current_bid + 1 > 1 ? e->current_bid + 1 : 1;
            for (int b = lo; b <= tc; b++) m[2 + b - 1] = 1;
        }
    } else if (e->phase == SK_BIDDING) {
        const int tc = total_cards(e);
        for (int b = e->current_bid + 1; b <= tc; b++) m[2 + b - 1] = 1;
        if (!e->passed[p] && non_passed_count(e) > 1) m[SK_PASS] = 1;
    } else {
        const int b = e->current_bidder;
        if (p == b) {
            if (e->must_reveal_own && unrevealed(e, b) > 0) {
                m[SK_REVEAL0 + b] = 1;
            } else {
                if (unrevealed(e, b) > 0) m[SK_REVEAL0 + b] = 1;
                for (int q = 0; q < e->n && q < OR_SK_MAXP; q++)
                    if (q != b && unrevealed(e, q) > 0) m[SK_REVEAL0 + q] = 1;
            }
        }
    }
}

/* skull.rs:533-670 get_observation (relative seats: 0 = current player) */
void or_skull_get_obs(const or_skull *e, float *o) {
    memset(o, 0, sizeof(float) * OR_SK_OBS);
    const int pl = e->current, n = e->n;
    o[0] = trap_in_hand(e, pl) ? 1.0f : 0.0f;
    const int rh = roses_in_hand(e, pl);
    for (int i = 0; i < OR_SK_ROSES; i++) o[1 + i] = i < rh ? 1.0f : 0.0f;
    for (int i = 0; i < OR_SK_CARDS; i++)
        if (i < e->stack_len[pl]) o[4 + i] = e->stack[pl][i] ? 1.0f : 0.0f;
    for (int r = 0; r < OR_SK_MAXP && r < n; r++) {
        const int a = (r + pl) % n;
        o[8 + r] = (float)e->stack_len[a] / (float)OR_SK_CARDS;
        o[14 + r] = (float)coaster_count(e, a) / (float)OR_SK_CARDS;
        o[20 + r] = is_alive(e, a) ? 1.0f : 0.0f;
        o[26 + r] = 1.0f;
        o[48 + r] = e->passed[a] ? 1.0f : 0.0f;
        o[54 + r] = (float)e->wins[a] / (float)OR_SK_WINS;
        o[60 + r] = (float)e->revealed[a] / (float)OR_SK_CARDS;
    }
    o[32 + pl] = 1.0f;
    o[38 + e->phase] = 1.0f;
    o[41] = (float)e->current_bid / (float)OR_SK_MAXBID;
    if (e->current_bidder >= 0) o[42 + (e->current_bidder + n - pl) % n] = 1.0f;
    if (n >= 2 && n <= OR_SK_MAXP) o[66 + n - 2] = 1.0f;
    for (int i = 0; i < e->hist_len; i++) {
        const int b = 71 + i * (OR_SK_MAXP + 2);
        o[b + (e->hist_player[i] + n - pl) % n] = 1.0f;
        if (e->hist_bid[i] == 0) o[b + OR_SK_MAXP + 1] = 1.0f;
        else o[b + OR_SK_MAXP] = (float)e->hist_bid[i] / (float)OR_SK_MAXBID;
    }
}

/* skull.rs:1480-1605 privileged_obs (absolute seats), padded to 200 */
void or_skull_priv(const or_skull *e, float *g) {
    memset(g, 0, sizeof(float) * OR_SK_PRIV);
    int k = 0;
    g[k + e->phase] = 1.0f; k += 3;
    g[k++] = (float)e->current / (float)OR_SK_MAXP;
    g[k++] = (float)e->round_starter / (float)OR_SK_MAXP;
    if (e->current_bid > 0) {
        g[k++] = (float)e->current_bid / (float)OR_SK_MAXBID;
        g[k++] = e->current_bidder >= 0 ? (float)e->current_bidder / (float)OR_SK_MAXP : -1.0f;
    } else {
        g[k++] = 0.0f;
        g[k++] = -1.0f;
    }
    const int hl = e->hist_len < 10 ? e->hist_len : 10;
    for (int i = 0; i < hl; i++) {                        /* newest first */
        const int j = e->hist_len - 1 - i;
        g[k + 3 * i] = (float)e->hist_player[j] / (float)OR_SK_MAXP;
        g[k + 3 * i + 1] = (float)e->hist_bid[j] / (float)OR_SK_MAXBID;
        g[k + 3 * i + 2] = e->hist_bid[j] == 0 ? 1.0f : 0.0f;
    }
    k += 30;
    g[k++] = e->game_over ? 1.0f : 0.0f;
    for (int i = 2; i <= OR_SK_MAXP; i++) g[k++] = e->n == i ? 1.0f : 0.0f;
    for (int s = 0; s < OR_SK_MAXP; s++) {
        const int sk = skulls_in_stack(e, s);
        g[k++] = s < e->n ? 1.0f : 0.0f;
        g[k++] = (float)e->wins[s] / (float)OR_SK_WINS;
        g[k++] = (e->has_trap[s] || e->rose_count[s] > 0) ? 1.0f : 0.0f;
        g[k++] = e->has_trap[s] ? 1.0f : 0.0f;
        g[k++] = (float)e->rose_count[s] / (float)OR_SK_ROSES;
        g[k++] = (float)e->stack_len[s] / (float)OR_SK_CARDS;
        g[k++] = (float)sk / (float)OR_SK_CARDS;
        g[k++] = (float)(e->stack_len[s] - sk) / (float)OR_SK_CARDS;
        g[k++] = e->passed[s] ? 1.0f : 0.0f;
        g[k++] = (float)e->revealed[s] / (float)OR_SK_CARDS;
    }
}

/* skull.rs:1103-1252.  rewards [6] (seats >= num_players stay 0, env.rs:477);
 * an action outside the mask panics in the reference: *invalid = 1, no change */
void or_skull_step(or_skull *e, int32_t action, float shaping, float *obs, float r[OR_SK_MAXP], int *done,
                   int *invalid) {
    for (int p = 0; p < OR_SK_MAXP; p++) r[p] = 0.0f;
    if (invalid) *invalid = 0;
    if (e->game_over) { *done = 1; if (obs) or_skull_get_obs(e, obs); return; }
    const int pl = e->current;
    uint8_t m[OR_SK_ACT];
    or_skull_mask(e, m);
    if (action < 0 || action >= OR_SK_ACT || !m[action]) {
        if (invalid) *invalid = 1;
        *done = 0;
        if (obs) or_skull_get_obs(e, obs);
        return;
    }
    if (e->phase == SK_PLACING) {
        if (action == 0 || action == 1) {
            e->stack[pl][e->stack_len[pl]++] = action == 0;
            e->current = next_alive(e, pl);
        } else if (action >= 2 && action < SK_PASS) {
            to_bidding(e, pl, action - 2 + 1);
        }
    } else if (e->phase == SK_BIDDING) {
        if (action >= 2 && action < SK_PASS) {
            const int bid = action - 2 + 1;
            e->current_bid = bid;
            e->current_bidder = pl;
            hist_push(e, pl, bid, 1);
            if (bid == total_cards(e)) {
                to_revealing(e);
            } else {
                const int next = next_non_passed(e, pl);
                if (next >= 0) e->current = next;
                else check_bidding_end(e);
            }
        } else if (action == SK_PASS) {
            e->passed[pl] = 1;
            hist_push(e, pl, 0, 1);
            check_bidding_end(e);
        }
    } else {
        const int bidder = e->current_bidder;
        const int target = action - SK_REVEAL0;
        const int skull = reveal_card(e, target);
        if (target == bidder && unrevealed(e, bidder) == 0) e->must_reveal_own = 0;
        if (skull) {
            e->last_skull_owner = target;
            lose_coaster(e, bidder);
            round_rewards(0, bidder, shaping, r);
            if (alive_count(e) <= 1) {
                e->game_over = 1;
                e->winner = -1;
                for (int p = 0; p < e->n && e->winner < 0; p++)
                    if (is_alive(e, p)) e->winner = p;
                final_rewards(e, r);
            } else {
                const int nxt = is_alive(e, bidder) ? bidder : (is_alive(e, target) ? target : next_alive(e, target));
                start_new_round(e, nxt);
            }
        } else if (e->roses_found >= e->current_bid) {
            e->wins[bidder]++;
            round_rewards(1, bidder, shaping, r);
            if (e->wins[bidder] >= OR_SK_WINS || alive_count(e) == 1) {
                e->game_over = 1;
                e->winner = bidder;
                final_rewards(e, r);
            } else {
                start_new_round(e, bidder);
            }
        }
    }
    *done = e->game_over;
    if (obs) or_skull_get_obs(e, obs);
}

/* test hooks: compute_placements / calculate_final_rewards (skull.rs:406, 472) */
void or_skull_placements(const or_skull *e, int32_t out[OR_SK_MAXP]) {
    int pl[OR_SK_MAXP];
    placements(e, pl);
    for (int p = 0; p < OR_SK_MAXP; p++) out[p] = p < e->n ? pl[p] : 0;
}
void or_skull_final_rewards(const or_skull *e, float r[OR_SK_MAXP]) { final_rewards(e, r); }

/* skull.rs:1338-1343 game_outcome: placements, 0 while the game runs */
void or_skull_outcome(const or_skull *e, int32_t out[OR_SK_MAXP]) {
    int pl[OR_SK_MAXP];
    for (int p = 0; p < OR_SK_MAXP; p++) out[p] = 0;
    if (!e->game_over) return;
    placements(e, pl);
    for (int p = 0; p < e->n; p++) out[p] = pl[p];
}

// k_wide.hip — device kernels of the GEMM-engine ("wide") path: Connect Four,
// Liar's Dice and Skull VecEnv (env.rs:281-487) with action masks -- and CartPole
// for the nets the fused CartPole kernels do not cover (other widths / depths,
// split_networks) -- masked Gumbel-max
// sampling (utils.rs:10-31, 96-135), the masked clipped-surrogate loss and its
// logit/value gradients (ppo.rs:1385-1592), and the small helpers around the
// GEMM engine (row gather, head packing, metric reduction).
#include "bppo_internal.h"
#include "bppo_envs.h"
#include "bppo_wide.h"

namespace bppo {

// ------------------------------------------------------------ env traits --
template <int ENV> struct EnvT;
// CartPole (cartpole.rs:50-106, 272-301): no action mask (all actions valid, so the
// -inf / (mask - 1) * 1e9 masking adds exactly 0), one player
template <> struct EnvT<BPPO_ENV_CARTPOLE> {
    using S = CartPoleState;
    static constexpr int D = 5, A = 2, P = 1, G = 0;
    // CartPole::new(seed) resets (cartpole.rs:104), VecEnv::new resets again (env.rs:289-293)
    __device__ static void reset_new(S &s, const Key8 &k, uint64_t &pos, int) {
        WordCursor c; c.init(k, 0, 0);
        cartpole_reset(s, c);
        cartpole_reset(s, c);
        pos = c.pos;
    }
    __device__ static void reset(S &s, const Key8 &k, uint64_t &pos) {
        WordCursor c; c.init(k, 0, pos);
        cartpole_reset(s, c);
        pos = c.pos;
    }
    __device__ static int player(const S &) { return 0; }
    __device__ static void step(S &s, int a, float, float r[BPPO_MAX_PLAYERS], int &done, int &, const Key8 &,
                                uint64_t &) {
        float rw = 0.0f;
        done = cartpole_step(s, a, rw) ? 1 : 0;
        r[0] = rw;
    }
    __device__ static void obs(const S &s, float *row) {
        float o[5];
        cartpole_obs(s, o);
        for (int i = 0; i < 5; i++) row[i] = o[i];
    }
    __device__ static void priv(const S &, float *) {}
    __device__ static void mask(const S &, uint8_t *m) { m[0] = 1; m[1] = 1; }
};
template <> struct EnvT<BPPO_ENV_CONNECT_FOUR> {
    using S = C4State;
    static constexpr int D = C4_OBS, A = C4_ACT, P = 2, G = 0;
    __device__ static void reset_new(S &s, const Key8 &, uint64_t &, int) { c4_reset(s); }   // new() ignores the seed
    __device__ static void reset(S &s, const Key8 &, uint64_t &) { c4_reset(s); }
    __device__ static int player(const S &s) { return s.cur - 1; }
    __device__ static void step(S &s, int a, float, float r[BPPO_MAX_PLAYERS], int &done, int &, const Key8 &,
                                uint64_t &) {
        c4_step(s, a, r, done);
    }
    __device__ static void obs(const S &s, float *row) { c4_obs(s, row); }
    __device__ static void priv(const S &, float *) {}
    __device__ static void mask(const S &s, uint8_t *m) { c4_mask(s, m); }
};
template <> struct EnvT<BPPO_ENV_LIARS_DICE> {
    using S = LDState;
    static constexpr int D = LD_OBS, A = LD_ACT, P = 4, G = LD_PRIV;
    // VecEnv::new: new_with_config rolls once, reset() rolls again (liars_dice.rs:186, 476)
    __device__ static void reset_new(S &s, const Key8 &k, uint64_t &pos, int) {
        WordCursor c; c.init(k, 0, 0);
        ld_new(s, c);
        ld_reset(s, c);
        pos = c.pos;
    }
    __device__ static void reset(S &s, const Key8 &k, uint64_t &pos) {
        WordCursor c; c.init(k, 0, pos);
        ld_reset(s, c);
        pos = c.pos;
    }
    __device__ static int player(const S &s) { return s.current; }
    __device__ static void step(S &s, int a, float shaping, float r[BPPO_MAX_PLAYERS], int &done, int &,
                                const Key8 &k, uint64_t &pos) {
        WordCursor c; c.init(k, 0, pos);
        ld_step(s, a, shaping, r, done, c);
        pos = c.pos;
    }
    __device__ static void obs(const S &s, float *row) { ld_obs(s, row); }
    __device__ static void priv(const S &s, float *row) { ld_priv(s, row); }
    __device__ static void mask(const S &s, uint8_t *m) { ld_mask(s, m); }
};
template <> struct EnvT<BPPO_ENV_SKULL> {
    using S = SKState;
    static constexpr int D = SK_OBS, A = SK_ACT, P = SK_P, G = SK_PRIV;
    // VecEnv::new: new_with_players(n, shaping, seed + i) then reset(); neither draws
    __device__ static void reset_new(S &s, const Key8 &, uint64_t &pos, int players) { sk_reset(s, players); pos = 0; }
    __device__ static void reset(S &s, const Key8 &, uint64_t &) { sk_reset(s, s.n); }
    __device__ static int player(const S &s) { return s.current; }
    __device__ static void step(S &s, int a, float shaping, float r[BPPO_MAX_PLAYERS], int &done, int &bad,
                                const Key8 &k, uint64_t &pos) {
        WordCursor c; c.init(k, 0, pos);
        sk_step(s, a, shaping, r, done, bad, c);
        pos = c.pos;
    }
    __device__ static void obs(const S &s, float *row) { sk_obs(s, row); }
    __device__ static void priv(const S &s, float *row) { sk_priv(s, row); }
    __device__ static void mask(const S &s, uint8_t *m) { sk_mask(s, m); }
};

template <int ENV>
__device__ __forceinline__ typename EnvT<ENV>::S *env_state(void *base) {
    return reinterpret_cast<typename EnvT<ENV>::S *>(base);
}

// VecEnv::new (env.rs:281-302): factory(seed_base + i) then reset()
template <int ENV>
__global__ void k_wide_reset(int N, uint64_t seed_base, int players, void *state, uint64_t *env_pos, float *ep_ret,
                             int32_t *ep_len) {
    using E = EnvT<ENV>;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    typename E::S s;
    uint64_t pos = 0;
    const Key8 k = seed_key(seed_base + (uint64_t)e);
    E::reset_new(s, k, pos, players);
    env_state<ENV>(state)[e] = s;
    env_pos[e] = pos;
    for (int p = 0; p < E::P; p++) ep_ret[(size_t)e * E::P + p] = 0.0f;
    ep_len[e] = 0;
}

// get_privileged_obs / get_observations / get_action_masks / get_current_players
// (env.rs:336-376) for 64 envs per block: rows [priv(G) | obs(D)] built in LDS,
// then stored by the whole block (the 64 rows are contiguous in HBM)
template <int ENV, bool PRIV>
__global__ void __launch_bounds__(64) k_wide_observe(int N, const void *state, float *xc, uint8_t *mask,
                                                     int32_t *players) {
    using E = EnvT<ENV>;
    constexpr int G = PRIV ? E::G : 0;
    constexpr int L = G + E::D;
    __shared__ __attribute__((aligned(16))) float rows[64 * L];
    const int e0 = blockIdx.x * 64, e = e0 + threadIdx.x;
    static_assert((64 * L) % 4 == 0, "observation tile in float4s");
    for (int i = threadIdx.x; i < 64 * L / 4; i += 64) reinterpret_cast<float4 *>(rows)[i] = make_float4(0, 0, 0, 0);
    __syncthreads();
    if (e < N) {
        const typename E::S s = env_state<ENV>(const_cast<void *>(state))[e];
        float *row = rows + threadIdx.x * L;
        if constexpr (PRIV) E::priv(s, row);
        E::obs(s, row + G);
        if (mask) E::mask(s, mask + (size_t)e * E::A);
        if (players) players[e] = E::player(s);
    }
    __syncthreads();
    const int nrows = min(64, N - e0);
    float *dst = xc + (size_t)e0 * L;
    // float4 stores when the tile's start is 16-B aligned (e0 L a multiple of 4), then the tail
    int i0 = 0;
    if (((size_t)e0 * L) % 4 == 0) {
        const int n4 = nrows * L / 4;
        for (int i = threadIdx.x; i < n4; i += 64) reinterpret_cast<float4 *>(dst)[i] = reinterpret_cast<const float4 *>(rows)[i];
        i0 = 4 * n4;
    }
    for (int i = i0 + threadIdx.x; i < nrows * L; i += 64) dst[i] = rows[i];
}

// VecEnv::step (env.rs:400-487) + the reward bookkeeping of collect_rollouts
// (ppo.rs:382-428, return normalisation off): all_rewards [N][P], the acting
// player's reward, done flag, episode accumulators, completed-episode records
// and auto-reset.
template <int ENV>
__global__ void k_wide_step(WideStepArgs a) {
    using E = EnvT<ENV>;
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.N) return;
    typename E::S s = env_state<ENV>(a.state)[e];
    const int act = a.actions[e];
    const int p_act = E::player(s);
    const Key8 k = seed_key(a.seed_base + (uint64_t)e);
    uint64_t pos = a.env_pos[e];
    float r[BPPO_MAX_PLAYERS] = {0, 0, 0, 0, 0, 0};
    int done = 0, bad = 0;
    E::step(s, act, a.shaping, r, done, bad, k, pos);
    if (bad && a.err) atomicOr(a.err, 8);
    float *er = a.ep_ret + (size_t)e * E::P;
    for (int p = 0; p < E::P; p++) {
        er[p] = __fadd_rn(er[p], r[p]);
        if (a.all_r) a.all_r[(size_t)e * E::P + p] = r[p];
    }
    const int len = a.ep_len[e] + 1;
    if (a.rew_act) a.rew_act[e] = r[p_act];
    if (a.done_f) a.done_f[e] = done ? 1.0f : 0.0f;
    if (a.done_u8) a.done_u8[e] = (uint8_t)done;
    const int slot = wave_episode_slot(done != 0, a.ep_count);
    if (done) {
        if (slot < a.eps_cap) {
            EpisodeRec rec;
            for (int p = 0; p < BPPO_MAX_PLAYERS; p++) rec.total_reward[p] = p < E::P ? er[p] : 0.0f;
            rec.length = len; rec.env_index = e; rec.step = a.t; rec.pad = 0;
            a.eps[slot] = rec;
        }
        for (int p = 0; p < E::P; p++) er[p] = 0.0f;
        a.ep_len[e] = 0;
        E::reset(s, k, pos);
    } else {
        a.ep_len[e] = len;
    }
    env_state<ENV>(a.state)[e] = s;
    a.env_pos[e] = pos;
}

// apply_action_mask + sample_categorical + log_prob_categorical (ppo.rs:337-366):
// masked logits get -inf; Gumbel u from the main stream at word
// base + e*A + a (row-major [env][action], one word per draw); first argmax.
// The A words of a row span at most NB ChaCha blocks; every lane makes exactly NB blocks
// (the same instructions in every lane) into its own LDS row and reads word a at its row
// offset.  A WordCursor walk here made a block whenever ANY lane of the wave crossed a
// block boundary -- with A = 49 every draw index is some lane's boundary, so each wave ran
// up to 49 divergent blocks per step instead of 4 (110 us per CfgD step)
constexpr int SAMPLE_THREADS = 64;
template <int A>
__global__ void __launch_bounds__(SAMPLE_THREADS) k_sample_masked(SampleArgs g) {
    constexpr int NB = (15 + A - 1) / 16 + 1;
    constexpr int WS = 16 * NB + 1;               // odd row stride: the lanes' rows on distinct banks
    __shared__ uint32_t wbuf[SAMPLE_THREADS * WS];
    __shared__ MathLds T;
    T.load();
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= g.N) return;
    float x[A];
    uint8_t mk[A];
    bool any = false;
#pragma unroll
    for (int a = 0; a < A; a++) { mk[a] = g.mask[(size_t)e * A + a]; x[a] = g.logits[(size_t)e * A + a]; }
    // (all loads above, the masking after: `ok ? logits[i] : -inf` became a branch around
    // each load with a wait at its end -- 2 A round trips per row)
#pragma unroll
    for (int a = 0; a < A; a++) {
        const bool ok = mk[a] != 0;
        any |= ok;
        x[a] = ok ? __fadd_rn(x[a], 0.0f) : -INFINITY;
    }
    if (!any) { atomicOr(g.err, 2); return; }   // utils.rs:115-123 "Empty action mask"
    const uint64_t row = g.gpos ? (uint64_t)g.gpos[e] : (uint64_t)e;   // ppo.rs:737 / :850 batch order
    const uint64_t w0 = (g.dbase ? *g.dbase : g.base) + row * A;
    uint32_t *words = wbuf + threadIdx.x * WS;
#pragma unroll 1
    for (int j = 0; j < NB; j++) {
        uint32_t blk[16];
        chacha12_block(g.key, (w0 >> 4) + j, g.stream, blk);
#pragma unroll
        for (int w = 0; w < 16; w++) words[16 * j + w] = blk[w];
    }
    const int off = (int)(w0 & 15);
    int best = 0;
    float bv = 0.0f;
#pragma unroll
    for (int a = 0; a < A; a++) {
        const float v = __fadd_rn(x[a], T.gumbel(words[off + a]));
        if (a == 0 || v > bv) { bv = v; best = a; }
    }
    g.act[e] = best;
    if (g.group && g.group[e] != 0) {              // opponent's move: no log-prob / value (ppo.rs:849-861)
        g.logp[e] = 0.0f;
        g.val[e] = 0.0f;
        return;
    }
    const float lp = log_prob_row<A>(x, best, T);
    if (!isfinite(lp)) atomicOr(g.err, 1);       // ppo.rs:363-366
    float v = g.values[e];
    if (g.pa_on) v = (float)((double)v * g.pa_std + g.pa_mean);
    g.logp[e] = lp;
    g.val[e] = v;
    const int p = g.players[e];
    g.lvpp[(size_t)e * g.P + p] = v;               // ppo.rs:443-445
}

// bootstrap (main.rs:918-927): last_value_per_player[e][current player] = V(s_T)
__global__ void k_boot_lvpp(int N, int P, const float *values, const int32_t *players, float *lvpp) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    lvpp[(size_t)e * P + players[e]] = values[e];
}

// minibatch gather (ppo.rs:1833-1857): dst[r][:] = src[perm[start + r]][:].  One wave per
// row: the row index loaded once, the row's loads (64 consecutive floats per instruction,
// clamped so none is conditional) all issued before its stores.  The element-per-thread
// form (a 64-bit division and a dependent perm -> src load pair per element) moved
// ~2 TB/s: 575 us per CfgD observation gather
constexpr int GATHER_U = 8;
__global__ void __launch_bounds__(256) k_gather_rows(const uint32_t *perm, uint32_t start, uint32_t n,
                                                     const float *src, int L, float *dst) {
    const int lane = threadIdx.x & 63;
    const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
    for (size_t r = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r < n; r += nw) {
        const float *s = src + (size_t)perm[start + r] * L;
        float *d = dst + r * L;
        for (int c0 = 0; c0 < L; c0 += 64 * GATHER_U) {
            float v[GATHER_U];
#pragma unroll
            for (int u = 0; u < GATHER_U; u++) v[u] = s[min(c0 + 64 * u + lane, L - 1)];
#pragma unroll
            for (int u = 0; u < GATHER_U; u++)
                if (c0 + 64 * u + lane < L) d[c0 + 64 * u + lane] = v[u];
        }
    }
}

// packed shared-trunk heads [K][A+1] = [W_policy | W_value], bias [A+1]
__global__ void k_pack_heads(const float *params, int K, int A, size_t wp, size_t bp, size_t wv, size_t bv,
                             float *W, float *b) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int A1 = A + 1;
    if (i < K * A1) {
        const int k = i / A1, j = i % A1;
        W[i] = j < A ? params[wp + (size_t)k * A + j] : params[wv + k];
    }
    if (i < A1) b[i] = i < A ? params[bp + i] : params[bv];
}

// compute_minibatch_loss (ppo.rs:1385-1502) + metrics (1507-1592) per row, with
// the masked log-softmax of the update ((mask - 1) * 1e9, ppo.rs:1436-1441):
// writes dOut[r] = [dL/dlogits (A) | dL/dvalue] and per-block metric partials.
template <int A>
__global__ void __launch_bounds__(256) k_wide_loss(LossArgs g) {
    __shared__ double red[WM_COUNT][256 / 64];
    __shared__ MathLds T;
    T.load();
    double m[WM_COUNT];
#pragma unroll
    for (int k = 0; k < WM_COUNT; k++) m[k] = 0.0;
    m[WM_VEMAX] = -INFINITY;
    const float mean = g.mb_stats[0], denom = __fadd_rn(g.mb_stats[1], 1e-8f);
    for (uint32_t r = blockIdx.x * blockDim.x + threadIdx.x; r < g.n; r += gridDim.x * blockDim.x) {
        const uint32_t idx = g.perm[g.start + r];
        const int act = g.act[idx];
        const float olp = g.logp[idx], R = g.ret[idx];
        const float An = __fdiv_rn(__fsub_rn(g.adv[idx], mean), denom);   // utils.rs:88
        float x[A];
        int nvalid = 0;
        float mx = -INFINITY;
#pragma unroll
        for (int a = 0; a < A; a++) {
            const float mk = g.mask[(size_t)idx * A + a] ? 1.0f : 0.0f;
            x[a] = __fadd_rn(g.logits[(size_t)r * A + a], __fmul_rn(__fsub_rn(mk, 1.0f), 1e9f));
            nvalid += mk > 0.5f;
            mx = x[a] > mx ? x[a] : mx;
        }
        float s = 0.0f;
#pragma unroll
        for (int a = 0; a < A; a++) s = __fadd_rn(s, T.expf(__fsub_rn(x[a], mx)));
        const float lse = T.logf(s);
        float H = 0.0f, newlp = 0.0f;
        float pr[A];                                          // exp(log_softmax), reused below
#pragma unroll
        for (int a = 0; a < A; a++) {
            x[a] = __fsub_rn(__fsub_rn(x[a], mx), lse);      // log_softmax
            pr[a] = T.expf(x[a]);
            H = __fadd_rn(H, __fmul_rn(pr[a], x[a]));
            newlp = a == act ? x[a] : newlp;
        }
        H = -H;
        const float log_ratio = __fsub_rn(newlp, olp);
        const float ratio = T.expf(log_ratio);
        const float na = -An;
        const float pl1 = __fmul_rn(na, ratio);
        const float rc = ratio < g.lo ? g.lo : (ratio > g.hi ? g.hi : ratio);
        const float pl2 = __fmul_rn(na, rc);
        const bool rhs = pl1 < pl2;
        const float pl = rhs ? pl2 : pl1;
        const float v = g.values[r];
        float vl, dvl;
        if (g.clip_value) {
            const float ov = g.val[idx];
            const float dlt = __fsub_rn(v, ov);
            const float dc = dlt < -g.ceps ? -g.ceps : (dlt > g.ceps ? g.ceps : dlt);
            const float vc = __fadd_rn(ov, dc);
            const float l1 = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
            const float l2 = __fmul_rn(__fsub_rn(vc, R), __fsub_rn(vc, R));
            if (l1 < l2) { vl = l2; dvl = (dlt >= -g.ceps && dlt <= g.ceps) ? 2.0f * __fsub_rn(vc, R) : 0.0f; }
            else { vl = l1; dvl = 2.0f * __fsub_rn(v, R); }
        } else {
            vl = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
            dvl = 2.0f * __fsub_rn(v, R);
        }
        // dL/dlogits and dL/dvalue in f64, each rounded once to f32 (ppo.rs:1923-1959 through
        // the oracle's restatement of the autodiff, oracle/net.c or_minibatch_loss_grad)
        const double g_ratio = (!rhs || (ratio >= g.lo && ratio <= g.hi)) ? -(double)An * g.inv_mb_d : 0.0;
        const double g_lr = g_ratio * (double)ratio;
        const double ecd = g.ent_coef_d * g.inv_mb_d;
        float *d = g.dout + (size_t)r * (A + 1);
#pragma unroll
        for (int a = 0; a < A; a++) {
            const double p = (double)pr[a];
            double gd = g_lr * ((a == act ? 1.0 : 0.0) - p);
            gd += ecd * p * ((double)x[a] + (double)H);
            d[a] = (float)gd;
        }
        d[A] = (float)(g.value_coef_d * 0.5 * g.inv_mb_d * (double)dvl);
        const float ve = fabsf(__fsub_rn(v, R));
        m[WM_PL] += pl; m[WM_VL] += vl; m[WM_H] += H;
        m[WM_KL] += (double)__fsub_rn(__fsub_rn(ratio, 1.0f), log_ratio);
        m[WM_CF] += fabsf(__fsub_rn(ratio, 1.0f)) > g.ceps ? 1.0 : 0.0;
        m[WM_V] += v; m[WM_R] += R; m[WM_VE] += ve; m[WM_VE2] += (double)ve * ve;
        m[WM_VEMAX] = fmax(m[WM_VEMAX], (double)ve);
        m[WM_N] += 1.0;
        m[WM_VALID] += nvalid;
        if (nvalid > 1) {
            m[WM_NCHOICE] += 1.0;
            m[WM_HV] += (double)__fdiv_rn(H, T.logf((float)nvalid));
        }
    }
    // block reduction: wave shuffles, then waves through LDS, fixed order
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < WM_COUNT; k++) {
        double v = m[k];
        for (int off = 32; off > 0; off >>= 1) {
            const double o = __shfl_xor(v, off, 64);
            v = k == WM_VEMAX ? fmax(v, o) : v + o;
        }
        if (lane == 0) red[k][w] = v;
    }
    __syncthreads();
    if (threadIdx.x < WM_COUNT) {
        const int k = threadIdx.x;
        double v = red[k][0];
        for (int i = 1; i < 4; i++) v = k == WM_VEMAX ? fmax(v, red[k][i]) : v + red[k][i];
        g.part[(size_t)blockIdx.x * WM_COUNT + k] = v;
    }
}

// fixed-order reduction of the loss partials into the metric slots after the
// gradient (d_grad[np + k]), where the all-reduce callback picks them up: one
// wave per metric, lane-strided sums then a fixed shuffle tree
static_assert(WM_COUNT == GRAD_METRIC_SLOTS && WM_VEMAX == GRAD_VEMAX, "metric slot layout");
__global__ void __launch_bounds__(64) k_wide_metric_reduce(const double *part, int nblk, float *out) {
    const int k = blockIdx.x, lane = threadIdx.x;
    const bool is_max = k == WM_VEMAX;
    double v = is_max ? -INFINITY : 0.0;
    for (int b = lane; b < nblk; b += 64) {
        const double x = part[(size_t)b * WM_COUNT + k];
        v = is_max ? fmax(v, x) : v + x;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const double o = __shfl_xor(v, off, 64);
        v = is_max ? fmax(v, o) : v + o;
    }
    if (lane == 0) {
        out[k] = (float)v;
        if (is_max) out[GRAD_VEMAX_LOCAL] = (float)v;   // kept out of the W > 1 SUM all-reduce
    }
}

// ------------------------------------------------------------- launchers --
#define ENV_DISPATCH(kind, KERNEL, grid, block, ...)                                        \
    do {                                                                                    \
        if ((kind) == BPPO_ENV_CONNECT_FOUR)                                                \
            hipLaunchKernelGGL(KERNEL<BPPO_ENV_CONNECT_FOUR>, grid, block, 0, st, __VA_ARGS__); \
        else if ((kind) == BPPO_ENV_CARTPOLE)                                               \
            hipLaunchKernelGGL(KERNEL<BPPO_ENV_CARTPOLE>, grid, block, 0, st, __VA_ARGS__);    \
        else if ((kind) == BPPO_ENV_SKULL)                                                  \
            hipLaunchKernelGGL(KERNEL<BPPO_ENV_SKULL>, grid, block, 0, st, __VA_ARGS__);       \
        else                                                                                \
            hipLaunchKernelGGL(KERNEL<BPPO_ENV_LIARS_DICE>, grid, block, 0, st, __VA_ARGS__);  \
    } while (0)

hipError_t wide_env_reset(int kind, hipStream_t st, int N, uint64_t seed_base, int players, void *state,
                          uint64_t *env_pos, float *ep_ret, int32_t *ep_len) {
    ENV_DISPATCH(kind, k_wide_reset, dim3((N + 255) / 256), dim3(256), N, seed_base, players, state, env_pos, ep_ret,
                 ep_len);
    return hipGetLastError();
}

hipError_t wide_env_observe(int kind, int with_priv, hipStream_t st, int N, const void *state, float *xc,
                            uint8_t *mask, int32_t *players) {
    const dim3 grid((N + 63) / 64), block(64);
    if (kind == BPPO_ENV_CONNECT_FOUR)
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_CONNECT_FOUR, false>), grid, block, 0, st, N, state, xc, mask, players);
    else if (kind == BPPO_ENV_CARTPOLE)
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_CARTPOLE, false>), grid, block, 0, st, N, state, xc, mask, players);
    else if (kind == BPPO_ENV_SKULL && with_priv)
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_SKULL, true>), grid, block, 0, st, N, state, xc, mask, players);
    else if (kind == BPPO_ENV_SKULL)
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_SKULL, false>), grid, block, 0, st, N, state, xc, mask, players);
    else if (with_priv)
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_LIARS_DICE, true>), grid, block, 0, st, N, state, xc, mask, players);
    else
        hipLaunchKernelGGL((k_wide_observe<BPPO_ENV_LIARS_DICE, false>), grid, block, 0, st, N, state, xc, mask, players);
    return hipGetLastError();
}

hipError_t wide_env_step(int kind, hipStream_t st, const WideStepArgs &a) {
    ENV_DISPATCH(kind, k_wide_step, dim3((a.N + 255) / 256), dim3(256), a);
    return hipGetLastError();
}

hipError_t wide_sample(int A, hipStream_t st, const SampleArgs &g) {
    const dim3 grid((g.N + SAMPLE_THREADS - 1) / SAMPLE_THREADS), block(SAMPLE_THREADS);
    if (A == 2) hipLaunchKernelGGL(k_sample_masked<2>, grid, block, 0, st, g);   // CartPole (GEMM path, bppo_debug_sample)
    else if (A == C4_ACT) hipLaunchKernelGGL(k_sample_masked<C4_ACT>, grid, block, 0, st, g);
    else if (A == LD_ACT) hipLaunchKernelGGL(k_sample_masked<LD_ACT>, grid, block, 0, st, g);
    else if (A == SK_ACT) hipLaunchKernelGGL(k_sample_masked<SK_ACT>, grid, block, 0, st, g);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t wide_boot_lvpp(hipStream_t st, int N, int P, const float *values, const int32_t *players, float *lvpp) {
    hipLaunchKernelGGL(k_boot_lvpp, dim3((N + 255) / 256), dim3(256), 0, st, N, P, values, players, lvpp);
    return hipGetLastError();
}

hipError_t wide_gather(hipStream_t st, const uint32_t *perm, uint32_t start, uint32_t n, const float *src, int L,
                       float *dst) {
    if (n == 0 || L <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)std::min<size_t>(((size_t)n + 3) / 4, 8192);   // 4 rows (waves) per block
    hipLaunchKernelGGL(k_gather_rows, dim3(blocks), dim3(256), 0, st, perm, start, n, src, L, dst);
    return hipGetLastError();
}

hipError_t wide_pack_heads(hipStream_t st, const float *params, int K, int A, size_t wp, size_t bp, size_t wv,
                           size_t bv, float *W, float *b) {
    const int n = K * (A + 1);
    hipLaunchKernelGGL(k_pack_heads, dim3((n + 255) / 256), dim3(256), 0, st, params, K, A, wp, bp, wv, bv, W, b);
    return hipGetLastError();
}

hipError_t wide_loss(int A, hipStream_t st, const LossArgs &g, int blocks, float *metrics_out) {
    if (A == 2) hipLaunchKernelGGL(k_wide_loss<2>, dim3(blocks), dim3(256), 0, st, g);   // CartPole
    else if (A == C4_ACT) hipLaunchKernelGGL(k_wide_loss<C4_ACT>, dim3(blocks), dim3(256), 0, st, g);
    else if (A == LD_ACT) hipLaunchKernelGGL(k_wide_loss<LD_ACT>, dim3(blocks), dim3(256), 0, st, g);
    else if (A == SK_ACT) hipLaunchKernelGGL(k_wide_loss<SK_ACT>, dim3(blocks), dim3(256), 0, st, g);
    else return hipErrorInvalidValue;
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_wide_metric_reduce, dim3(WM_COUNT), dim3(64), 0, st, g.part, blocks, metrics_out);
    return hipGetLastError();
}

}  // namespace bppo

namespace bppo {
size_t wide_state_bytes(int kind) {
    return kind == BPPO_ENV_CONNECT_FOUR ? sizeof(C4State) : kind == BPPO_ENV_SKULL ? sizeof(SKState)
         : kind == BPPO_ENV_CARTPOLE ? sizeof(CartPoleState) : sizeof(LDState);
}
}  // namespace bppo

// k_rollout.hip — CartPole VecEnv + fused rollout kernels.
//
// One lane owns one environment for the whole rollout (SoA env state in HBM,
// kept in VGPRs across the T steps).  Per step, exactly as collect_rollouts
// (ppo.rs:271-446): lagged obs normalisation (normalization.rs:58-75), MLP
// forward (mlp.rs:140-206) with weights staged in LDS, Gumbel-max sampling
// from the main ChaCha12 stream at word base + (t*N + e)*A + a (utils.rs:10-31),
// log-prob (utils.rs:38-45), env step + auto-reset (env.rs:413-467,
// cartpole.rs:272-301).  Raw rewards are written; the return normaliser runs as
// a post-pass scan (k_gae.hip) because normalised rewards only feed GAE.
#include "bppo_internal.h"
#include "bppo_mlp64.h"

namespace bppo {

// ObsNormalizer::normalize_batch (normalization.rs:58-75) from device stats
// on = {mean[D], M2[D], count}.  The stats are fixed for a whole rollout, so
// the per-dim std is derived once (same f64 ops as per call) and each step only
// does (raw - mean) / sd.
struct ObsNorm5 {
    double mean[5], sd[5];
    bool on;
    __device__ __forceinline__ void load(const double *__restrict__ st, int norm_on) {
        const double cnt = st[10];
        on = norm_on && cnt >= 2.0;
#pragma unroll
        for (int d = 0; d < 5; d++) {
            const double var = st[5 + d] / cnt;
            double s = sqrt(var);
            sd[d] = s < 1e-8 ? 1e-8 : s;
            mean[d] = st[d];
        }
    }
    __device__ __forceinline__ void apply(const float (&raw)[5], float (&out)[5]) const {
#pragma unroll
        for (int d = 0; d < 5; d++) {
            if (!on) { out[d] = raw[d]; continue; }
            float z = (float)(((double)raw[d] - mean[d]) / sd[d]);
            z = z < -10.0f ? -10.0f : z;
            z = z > 10.0f ? 10.0f : z;
            out[d] = z;
        }
    }
};

// per-env raw-observation statistics of one rollout (count T) for the
// normalizer update (normalization.rs:37-53): sums shifted by the first
// observation, no division per step; mean / M2 at the end match the
// sequential Welford values to f64 rounding (Chan-merged afterwards)
struct ObsAcc5 {
    double x0[5], s1[5], s2[5];
    __device__ __forceinline__ void init(const float (&raw)[5]) {
#pragma unroll
        for (int d = 0; d < 5; d++) { x0[d] = (double)raw[d]; s1[d] = s2[d] = 0.0; }
    }
    __device__ __forceinline__ void push(const float (&raw)[5]) {
#pragma unroll
        for (int d = 0; d < 5; d++) {
            const double dd = (double)raw[d] - x0[d];
            s1[d] += dd;
            s2[d] += dd * dd;
        }
    }
    __device__ __forceinline__ void store(double T, double *part) const {
#pragma unroll
        for (int d = 0; d < 5; d++) {
            part[d] = x0[d] + s1[d] / T;
            const double m2 = s2[d] - s1[d] * s1[d] / T;
            part[5 + d] = m2 > 0.0 ? m2 : 0.0;
        }
    }
};

__device__ __forceinline__ void load_state(const float *cp, const int32_t *steps, int N, int e,
                                           CartPoleState &s) {
    s.x = cp[e]; s.x_dot = cp[N + e]; s.theta = cp[2 * N + e]; s.theta_dot = cp[3 * N + e];
    s.steps = steps[e];
}
__device__ __forceinline__ void store_state(float *cp, int32_t *steps, int N, int e,
                                            const CartPoleState &s) {
    cp[e] = s.x; cp[N + e] = s.x_dot; cp[2 * N + e] = s.theta; cp[3 * N + e] = s.theta_dot;
    steps[e] = s.steps;
}

// VecEnv::new: CartPole::new(seed+i) resets once, VecEnv::new resets again
// (cartpole.rs:104, env.rs:289-293) => words 0-3 discarded, state from 4-7.
__global__ void k_cartpole_reset(int N, uint64_t seed_base, float *cp, int32_t *steps,
                                 uint64_t *env_pos, float *ep_ret, int32_t *ep_len, float *obs) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    WordCursor c;
    c.init(seed_key(seed_base + (uint64_t)e), 0, 0);
    CartPoleState s;
    cartpole_reset(s, c);
    cartpole_reset(s, c);
    store_state(cp, steps, N, e, s);
    env_pos[e] = c.pos;
    ep_ret[e] = 0.0f;
    ep_len[e] = 0;
    if (obs) {
        float o[5];
        cartpole_obs(s, o);
        for (int d = 0; d < 5; d++) obs[e * 5 + d] = o[d];
    }
}

struct RolloutArgs {
    int N, T;
    uint64_t seed_base;
    float *cp; int32_t *steps; uint64_t *env_pos; float *ep_ret; int32_t *ep_len;
    Key8 key; uint64_t stream; uint64_t base_pos;
    const float *params; int n_params;
    const double *on; int norm_on;
    float *obs, *rew_raw, *done, *val, *logp; int32_t *act;
    double *obs_part;
    EpisodeRec *eps; int32_t *ep_count; int eps_cap;
    int32_t *err;
    float4 *rows;        // MFMA rollout: also the update's rows A [B][2] float4 (k_update.hip load_row), or null
    unsigned long long *stamps;   // diagnostic build only (BPPO_RO_STAMPS): per-wave segment cycles
    const float4 *rpool; const uint64_t *rpos; int rpool_k;   // 64-lane MFMA rollout: k_reset_pool's states
};

// diagnostic build (-DBPPO_RO_STAMPS): s_memtime segment sums per wave of the 64-lane CfgB
// rollout (cdna_hip_programming.md section 7 in-kernel stamps); read the shares, not the time
#ifdef BPPO_RO_STAMPS
constexpr int RO_NSEG = 8;
#define RO_STAMP(k)                                                                              \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long t_;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        ro_acc[k] += t_ - ro_prev;                                                               \
        ro_prev = t_;                                                                            \
    } while (0)
#else
#define RO_STAMP(k) \
    do {            \
    } while (0)
#endif

template <int H, int NL, int ACT>
__global__ void __launch_bounds__(256) k_cartpole_rollout(RolloutArgs a) {
    extern __shared__ __attribute__((aligned(16))) float sP[];
    constexpr CpOffsets O = cp_offsets<H, NL>();
    for (int i = threadIdx.x; i < O.n; i += blockDim.x) sP[i] = a.params[i];
    __syncthreads();
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= a.N) return;
    const int N = a.N;
    CartPoleState s;
    load_state(a.cp, a.steps, N, e, s);
    WordCursor ec;
    ec.init(seed_key(a.seed_base + (uint64_t)e), 0, a.env_pos[e]);
    float ep_ret = a.ep_ret[e];
    int32_t ep_len = a.ep_len[e];
    ObsNorm5 nz;
    nz.load(a.on, a.norm_on);
    ObsAcc5 oa;
    {
        float raw0[5];
        cartpole_obs(s, raw0);
        oa.init(raw0);
    }
    int32_t bad = 0;
#pragma unroll 1
    for (int t = 0; t < a.T; t++) {
        float raw[5], x[5];
        cartpole_obs(s, raw);
        oa.push(raw);
        nz.apply(raw, x);
        const size_t row = (size_t)t * N + e;
#pragma unroll
        for (int d = 0; d < 5; d++) a.obs[row * 5 + d] = x[d];
        float lg[2], v;
        int zero = 0;
        asm volatile("" : "+v"(zero));   // keep weight reads inside the step loop (no LICM spill)
        cp_forward<H, NL, ACT>(sP + zero, x, lg, v, sP + cp_stage_ofs<H, NL>() + threadIdx.x, blockDim.x);
        // Gumbel-max: words base + row*2 + {0,1}
        const uint64_t p0 = a.base_pos + row * 2;
        uint32_t blk[16];
        chacha12_block(a.key, p0 >> 4, a.stream, blk);
        const uint32_t l0 = (uint32_t)(p0 & 15);
        uint32_t w0 = blk[0], w1 = blk[1];
#pragma unroll
        for (int i = 1; i < 16; i++) w0 = l0 == (uint32_t)i ? blk[i] : w0;
#pragma unroll
        for (int i = 0; i < 15; i++) w1 = l0 == (uint32_t)i ? blk[i + 1] : w1;
        if (l0 == 15) {
            uint32_t b2[16];
            chacha12_block(a.key, (p0 >> 4) + 1, a.stream, b2);
            w1 = b2[0];
        }
        const float n0 = __fadd_rn(lg[0], gumbel_from_word(w0));
        const float n1 = __fadd_rn(lg[1], gumbel_from_word(w1));
        const int act = n1 > n0 ? 1 : 0;               // argmax, first maximum
        const float lp = log_prob_row<2>(lg, act);
        bad |= !isfinite(lp);
        float r;
        const bool done = cartpole_step(s, act, r);
        ep_ret = __fadd_rn(ep_ret, r);
        ep_len += 1;
        const int32_t k = wave_episode_slot(done, a.ep_count);
        if (done) {
            if (k < a.eps_cap) {
                EpisodeRec rec;
                rec.total_reward[0] = ep_ret;
                for (int p = 1; p < BPPO_MAX_PLAYERS; p++) rec.total_reward[p] = 0.0f;
                rec.length = ep_len; rec.env_index = e; rec.step = t; rec.pad = 0;
                a.eps[k] = rec;
            }
            cartpole_reset(s, ec);
            ep_ret = 0.0f;
            ep_len = 0;
        }
        a.act[row] = act;
        a.rew_raw[row] = r;
        a.done[row] = done ? 1.0f : 0.0f;
        a.val[row] = v;
        a.logp[row] = lp;
    }
    store_state(a.cp, a.steps, N, e, s);
    a.env_pos[e] = ec.pos;
    a.ep_ret[e] = ep_ret;
    a.ep_len[e] = ep_len;
    oa.store((double)a.T, a.obs_part + (size_t)e * 10);
    if (bad) atomicOr(a.err, 1);
}

// Gumbel noise of a whole rollout, ahead of it (utils.rs:10-31): g[i] for the
// word at base + i, i < count (row-major [t][env][action], one word per draw).
// One ChaCha12 block per thread; the rollout reads two floats per env-step.  The
// block's 16 x 256 noise floats are transposed through LDS so every store
// instruction writes 256 consecutive floats (a thread's own 16 words would be
// a 64-B-strided store per word)
constexpr int GUM_THREADS = 256;
// zero0 / zero1 (optional): the rollout's episode counter and error flags, set to 0 here
// (one store each) instead of by two fill launches ahead of it
__global__ void __launch_bounds__(GUM_THREADS) k_gumbel_words(Key8 key, uint64_t stream, uint64_t base,
                                                              uint64_t count, float *__restrict__ g,
                                                              int32_t *zero0, int32_t *zero1) {
    __shared__ float tile[16 * GUM_THREADS + GUM_THREADS / 2];
    if (zero0 && blockIdx.x == 0 && threadIdx.x == 0) { *zero0 = 0; *zero1 = 0; }
    const uint64_t blk0 = (base >> 4) + blockIdx.x * (uint64_t)GUM_THREADS;
    const uint64_t b = blk0 + threadIdx.x, wb = blk0 * 16;
    if (b * 16 < base + count) {
        uint32_t blk[16];
        chacha12_block(key, b, stream, blk);
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const int k = threadIdx.x * 16 + j;
            tile[k + (k >> 5)] = gumbel_from_word(blk[j]);   // one pad float per 32: conflict-free writes
        }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; j++) {
        const int k = j * GUM_THREADS + threadIdx.x;
        const uint64_t w = wb + k;
        if (w >= base && w < base + count) g[w - base] = tile[k + (k >> 5)];
    }
}

// The next K reset states of every env, drawn ahead of the 64-lane rollout from the env's
// own stream (cartpole.rs:275-278: four gen_range draws with rejection, from env_pos on),
// with the stream position after each.  In the rollout a reset is then a register copy of
// a prefetched entry instead of a ChaCha block evaluated under divergence: any of a wave's
// 64 lanes finishing an episode made the whole wave wait on one (segment stamps: 1.7k of
// 23.7k cycles per step, profiles/r05b/rollout_stamps.txt).  Entries [j][e]: the threads
// of a wave write consecutive envs.  An env that resets more than K times in one rollout
// falls back to drawing in the kernel (bit-identical: the same cursor, from the position
// after entry K - 1).
__global__ void __launch_bounds__(256) k_reset_pool(int N, int K, uint64_t seed_base, const uint64_t *__restrict__ env_pos,
                                                    float4 *__restrict__ pool, uint64_t *__restrict__ ppos) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    WordCursor c;
    c.init(seed_key(seed_base + (uint64_t)e), 0, env_pos[e]);
    for (int j = 0; j < K; j++) {
        CartPoleState s;
        cartpole_reset(s, c);
        pool[(size_t)j * N + e] = make_float4(s.x, s.x_dot, s.theta, s.theta_dot);
        ppos[(size_t)j * N + e] = c.pos;
    }
}

// The CfgB rollout (64x2 relu MLP) with the MLP on v_mfma_f32_32x32x2_f32: each
// wave owns 32 envs for all T steps (lanes 0-31 hold the env state; all 64
// lanes run the MFMAs), 8 waves per block, 2 per SIMD.  Per step: obs ->
// normalise (lagged stats) -> H1, H2 on MFMA in natural k order (bit-equal to
// the VALU chain) -> heads on the VALU -> Gumbel-max with the precomputed noise
// -> log-prob -> CartPole step / auto-reset; same outputs as k_cartpole_rollout.
__global__ void __launch_bounds__(512, 2) k_cartpole_rollout_mfma(RolloutArgs a, const float *__restrict__ gum) {
    using namespace mmb;
    extern __shared__ __attribute__((aligned(16))) float smem[];
    Params &S = *reinterpret_cast<Params *>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    Wave &B = reinterpret_cast<Wave *>(smem + sizeof(Params) / 4)[wv];
    load_params(S, a.params);
    __syncthreads();
    const int c = lane & 31, h = lane >> 5;
    const int N = a.N;
    const int e = (blockIdx.x * WAVES + wv) * TR + c;
    const bool mine = h == 0 && e < N;
    float b0k[2], b1k[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) { b0k[ct] = S.b0[c + 32 * ct]; b1k[ct] = S.b1[c + 32 * ct]; }
    CartPoleState s{};
    WordCursor ec;
    float ep_ret = 0.0f;
    int32_t ep_len = 0;
    if (mine) {
        load_state(a.cp, a.steps, N, e, s);
        ec.init(seed_key(a.seed_base + (uint64_t)e), 0, a.env_pos[e]);
        ep_ret = a.ep_ret[e];
        ep_len = a.ep_len[e];
    }
    ObsNorm5 nz;
    nz.load(a.on, a.norm_on);
    ObsAcc5 oa;
    if (mine) {
        float raw0[5];
        cartpole_obs(s, raw0);
        oa.init(raw0);
    }
    int32_t bad = 0;
#pragma unroll 1
    for (int t = 0; t < a.T; t++) {
        const size_t row = (size_t)t * N + e;
        // this step's Gumbel pair, loaded before the MLP so its HBM latency hides under it
        const float2 gz = mine ? *reinterpret_cast<const float2 *>(gum + row * 2) : make_float2(0.0f, 0.0f);
        float4 xa = make_float4(0.f, 0.f, 0.f, 0.f);
        float x4 = 0.0f;
        if (h == 0) {
            float x[5] = {0, 0, 0, 0, 0};
            if (mine) {
                float raw[5];
                cartpole_obs(s, raw);
                oa.push(raw);
                nz.apply(raw, x);
#pragma unroll
                for (int d = 0; d < 5; d++) a.obs[row * 5 + d] = x[d];
                xa = make_float4(x[0], x[1], x[2], x[3]);
                x4 = x[4];
            }
#pragma unroll
            for (int d = 0; d < 5; d++) B.X[c * 9 + d] = x[d];
            B.X[c * 9 + 5] = 0.0f;
        }
        wave_sync();
        f32x16_t h1[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) h1[ct][q] = 0.0f;
#pragma unroll
        for (int st = 0; st < 3; st++) {
            const float av = B.X[c * 9 + 2 * st + h];
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
                h1[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, S.W0[(2 * st + h) * H + c + 32 * ct], h1[ct], 0, 0, 0);
        }
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const float v = __fadd_rn(h1[ct][q], b0k[ct]);
                B.T[cd_row(q, h) * RS + c + 32 * ct] = v > 0.0f ? v : 0.0f;
            }
        wave_sync();
        f32x16_t h2[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) h2[ct][q] = 0.0f;
#pragma unroll 8
        for (int st = 0; st < 32; st++) {
            const float av = B.T[c * RS + 2 * st + h];
            h2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, S.W1[(2 * st + h) * RS + c], h2[0], 0, 0, 0);
            h2[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, S.W1[(2 * st + h) * RS + c + 32], h2[1], 0, 0, 0);
        }
        wave_sync();
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const float v = __fadd_rn(h2[ct][q], b1k[ct]);
                B.T[cd_row(q, h) * RS + c + 32 * ct] = v > 0.0f ? v : 0.0f;
            }
        wave_sync();
        // heads: lane half h runs the k-ordered chain of logit h, both run the value
        // chain (two chains per lane instead of three on the low half alone; each
        // chain is the same fma sequence, so the values are bit-identical)
        float lh = 0.0f, vv = 0.0f;
        if (e < N) {
            const float *hr = B.T + c * RS;
            const float2 *pv = S.PV[h];
#pragma unroll 16
            for (int k = 0; k < H; k++) {
                const float hk = hr[k];
                const float2 w = pv[k];
                lh = __builtin_fmaf(hk, w.x, lh);
                vv = __builtin_fmaf(hk, w.y, vv);
            }
        }
        const float lx = __shfl_xor(lh, 32, 64);
        if (mine) {
            const float l0 = lh, l1 = lx;
            float lg[2];
            lg[0] = __fadd_rn(l0, S.bp[0]);
            lg[1] = __fadd_rn(l1, S.bp[1]);
            const float v = __fadd_rn(vv, S.bv[0]);
            const float n0 = __fadd_rn(lg[0], gz.x);
            const float n1 = __fadd_rn(lg[1], gz.y);
            const int act = n1 > n0 ? 1 : 0;               // argmax, first maximum
            const float lp = log_prob_row<2>(lg, act);
            bad |= !isfinite(lp);
            float r;
            const bool done = cartpole_step(s, act, r);
            ep_ret = __fadd_rn(ep_ret, r);
            ep_len += 1;
            const int32_t k = wave_episode_slot(done, a.ep_count);
            if (done) {
                if (k < a.eps_cap) {
                    EpisodeRec rec;
                    rec.total_reward[0] = ep_ret;
                    for (int p = 1; p < BPPO_MAX_PLAYERS; p++) rec.total_reward[p] = 0.0f;
                    rec.length = ep_len; rec.env_index = e; rec.step = t; rec.pad = 0;
                    a.eps[k] = rec;
                }
                cartpole_reset(s, ec);
                ep_ret = 0.0f;
                ep_len = 0;
            }
            a.act[row] = act;
            a.rew_raw[row] = r;
            a.done[row] = done ? 1.0f : 0.0f;
            a.val[row] = v;
            a.logp[row] = lp;
            // the row's 32 bytes in one pair of stores (adjacent lanes: adjacent rows)
            if (a.rows) { a.rows[row * 2] = xa; a.rows[row * 2 + 1] = make_float4(x4, __int_as_float(act), lp, v); }
        }
        wave_sync();
    }
    if (mine) {
        store_state(a.cp, a.steps, N, e, s);
        a.env_pos[e] = ec.pos;
        a.ep_ret[e] = ep_ret;
        a.ep_len[e] = ep_len;
        oa.store((double)a.T, a.obs_part + (size_t)e * 10);
        if (bad) atomicOr(a.err, 1);
    }
}

// The CfgB rollout with every lane owning an env: a wave
// holds 64 envs as two 32-env MFMA tiles (lane l = env l; tile A = lanes 0-31,
// tile B = lanes 32-63 of the wave's 64 envs) and runs both layers TRANSPOSED
// (H^T = W^T X^T on v_mfma_f32_32x32x2_f32, units on the MFMA rows, envs on
// its columns), with no LDS round trip for H1:
//  * layer 1's K pairs (x0,x1) (x2,x3) (x4,1) come from the env lanes through one
//    v_permlane32_swap per pair; b0 rides in the K pad (fma(1, b0, acc) is the
//    reference's separate + b0, rounded once);
//  * layer 1's output rows are hidden units permuted so that accumulator
//    register m of lane half h holds unit 2m + h: register m is then directly the
//    B operand of layer 2's K step m (k = 2m on half 0, 2m + 1 on half 1), in
//    natural k order (same fma chain as the reference's matmul);
//  * layer 2's output rows are permuted so register m holds unit 32h + m; the
//    registers go to the wave's [env][unit] tile and lane l reads env l's row for the
//    heads' k-ordered chains (+ b1, relu, three fma chains per lane).  (Swapping them
//    with v_permlane32_swap instead kept 64 more registers live: 475 per wave, no room
//    for other kernels' waves; r04 first form, profiles/r04_rollout/rollout_ab.txt);
//  * W0 (+b0) lives in VGPRs for the whole rollout, W1's operands in LDS (one
//    conflict-free ds_read_b64 per K step for both tiles); H2 goes through a per-wave
//    [env][unit] LDS tile (stride 65) to the heads, whose {wp0, wp1, wv, b1} rows are LDS
//    broadcasts; expf/logf tables in LDS.
// One wave per SIMD (CfgB: 65,536 envs = 1,024 waves) in 269 registers and 84 KB of LDS
// per block, which leaves room on every CU for the side-stream shuffle kernels' waves.
namespace mmr {
constexpr int H = 64, WAVES = 4;
struct Params {
    uint64_t exp2tab[32];
    double linvc[16], llogc[16];
    float4 hw[H];                 // {Wp[2k], Wp[2k+1], Wv[k], b1[k]}
    float bp[2], bv[2];
    __device__ __forceinline__ float expf(float x) const { return bppo_math::expf_glibc_tab(x, exp2tab); }
    __device__ __forceinline__ float logf(float x) const { return bppo_math::logf_glibc_tab(x, linvc, llogc); }
};
// MFMA output row r (0..63) -> hidden unit, layer 1 / layer 2
__device__ __forceinline__ int unit1(int r) {
    const int rr = r & 31, ct = r >> 5, q = (rr & 3) + 4 * (rr >> 3), hh = (rr >> 2) & 1;
    return 2 * (q + 16 * ct) + hh;
}
__device__ __forceinline__ int unit2(int r) {
    const int rr = r & 31, ct = r >> 5, q = (rr & 3) + 4 * (rr >> 3), hh = (rr >> 2) & 1;
    return 32 * hh + q + 16 * ct;
}
__device__ __forceinline__ void swap_halves(float &lo, float &hi) {
    // lanes 32-63 of `lo` <-> lanes 0-31 of `hi`
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(lo), __float_as_uint(hi), false, false);
    lo = __uint_as_float(r[0]);
    hi = __uint_as_float(r[1]);
}
__device__ __forceinline__ float log_prob2(const Params &S, const float (&x)[2], int a) {
    const float m = x[1] > x[0] ? x[1] : x[0];
    float s = 0.0f;
    s = __fadd_rn(s, S.expf(__fsub_rn(x[0], m)));
    s = __fadd_rn(s, S.expf(__fsub_rn(x[1], m)));
    const float lse = S.logf(s);
    return __fsub_rn(__fsub_rn(a ? x[1] : x[0], m), lse);
}
}  // namespace mmr

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 2))) k_cartpole_rollout_mfma64(RolloutArgs a, const float *__restrict__ gum) {
    using namespace mmr;
    constexpr CpOffsets O = cp_offsets<64, 2>();
    __shared__ Params S;
    __shared__ float2 w1r[32][64];                // layer 2's A operands [K step][lane] = {ct 0, ct 1}
    __shared__ float T2[WAVES][64 * 65];          // H2 [env][unit], row stride 65 (conflict-free both ways)
    const float *__restrict__ P = a.params;
    for (int i = threadIdx.x; i < H; i += blockDim.x)
        S.hw[i] = make_float4(P[O.wp + 2 * i], P[O.wp + 2 * i + 1], P[O.wv + i], P[O.b1 + i]);
    if (threadIdx.x < 32) S.exp2tab[threadIdx.x] = bppo_math::kExp2fTab[threadIdx.x];
    if (threadIdx.x < 16) {
        S.linvc[threadIdx.x] = bppo_math::kLogfInvc[threadIdx.x];
        S.llogc[threadIdx.x] = bppo_math::kLogfLogc[threadIdx.x];
    }
    if (threadIdx.x < 2) S.bp[threadIdx.x] = P[O.bp + threadIdx.x];
    if (threadIdx.x == 0) S.bv[0] = P[O.bv];
    __syncthreads();

    const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const int N = a.N;
    const int e = (blockIdx.x * WAVES + (threadIdx.x >> 6)) * 64 + lane;
    const bool mine = e < N;
    for (int i = threadIdx.x; i < 32 * 64; i += blockDim.x) {
        const int st = i >> 6, l = i & 63, lc = l & 31, lh = l >> 5;
        w1r[st][l] = make_float2(P[O.w1 + (2 * st + lh) * H + unit2(lc)], P[O.w1 + (2 * st + lh) * H + unit2(lc + 32)]);
    }
    __syncthreads();
    float *Tw = T2[threadIdx.x >> 6];
    // layer 1's A operands stay in registers for the whole rollout
    float w0r[3][2];
#pragma unroll
    for (int st = 0; st < 3; st++)
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const int d = 2 * st + h, u = unit1(c + 32 * ct);
            w0r[st][ct] = d < 5 ? P[O.w0 + d * H + u] : P[O.b0 + u];
        }

    CartPoleState s{};
    uint64_t env_pos = 0;
    float ep_ret = 0.0f;
    int32_t ep_len = 0;
    if (mine) {
        load_state(a.cp, a.steps, N, e, s);
        env_pos = a.env_pos[e];
        ep_ret = a.ep_ret[e];
        ep_len = a.ep_len[e];
    }
    ObsNorm5 nz;
    nz.load(a.on, a.norm_on);
    ObsAcc5 oa;
    {
        float raw0[5];
        cartpole_obs(s, raw0);
        oa.init(raw0);
    }
    int32_t bad = 0;
    // the next reset state: k_reset_pool entry rj, read at every step's start (an L2 hit
    // until the entry is used) so that no load is waited on in the step's reset branch
    int rj = 0;
    // the previous step's finished episodes: the slot counter's atomic return is read one
    // step later (under this step's MFMAs) instead of stalling the wave where it is issued
    uint64_t pm = 0;          // ballot of the previous step's done lanes
    int32_t pbase = 0;        // its leader lane's atomicAdd return
    float pret = 0.0f;
    int32_t plen = 0;
    auto flush_eps = [&](int step) {
        if (pm == 0) return;
        const int leader = __ffsll((unsigned long long)pm) - 1;
        const int32_t base = __builtin_amdgcn_readlane(pbase, leader);
        if ((pm >> lane) & 1ull) {
            const int32_t k = base + (int32_t)__popcll(pm & ((1ull << lane) - 1ull));
            if (k < a.eps_cap) {
                EpisodeRec rec;
                rec.total_reward[0] = pret;
                for (int p = 1; p < BPPO_MAX_PLAYERS; p++) rec.total_reward[p] = 0.0f;
                rec.length = plen; rec.env_index = e; rec.step = step; rec.pad = 0;
                a.eps[k] = rec;
            }
        }
    };
#ifdef BPPO_RO_STAMPS
    unsigned long long ro_acc[RO_NSEG] = {}, ro_prev;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(ro_prev)::"memory");
#endif
    // the prologue's loads (W0 fragments, state) complete before the step loop: left pending
    // at the loop header, the wait-count pass waited on every step's fresh loads (the Gumbel
    // pair, the reset entry) at layer 1's first use of the W0 registers
    __builtin_amdgcn_s_waitcnt(0);
#pragma unroll 1
    for (int t = 0; t < a.T; t++) {
        const size_t row = (size_t)t * N + e;
        // the next step's Gumbel pair, in flight under this step's MFMAs
        // this step's Gumbel pair: in flight under the layer MFMAs, first used by the argmax (a
        // pair prefetched a step ahead needs a register copy at the loop latch, where the
        // wait-count pass then waited for the whole step's stores)
        float2 gz = make_float2(0.0f, 0.0f);
        if (mine) gz = *reinterpret_cast<const float2 *>(gum + row * 2);
        float4 rnx = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        uint64_t rnpos = 0;
        if (mine && rj < a.rpool_k) { rnx = a.rpool[(size_t)rj * N + e]; rnpos = a.rpos[(size_t)rj * N + e]; }
        float x[6] = {0, 0, 0, 0, 0, 1.0f};
        if (mine) {
            float raw[5], z[5];
            cartpole_obs(s, raw);
            oa.push(raw);
            nz.apply(raw, z);
#pragma unroll
            for (int d = 0; d < 5; d++) x[d] = z[d];
        }
        RO_STAMP(0);
        // ---- layer 1 (transposed): H1^T = [W0; b0]^T [x, 1]^T, two env tiles
        f32x16_t h1[2][2];
#pragma unroll
        for (int tl = 0; tl < 2; tl++)
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
#pragma unroll
                for (int q = 0; q < 16; q++) h1[tl][ct][q] = 0.0f;
#pragma unroll
        for (int st = 0; st < 3; st++) {
            float pa = x[2 * st], pb = x[2 * st + 1];
            swap_halves(pa, pb);         // pa: tile A's (k = 2st, 2st + 1), pb: tile B's
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                h1[0][ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0r[st][ct], pa, h1[0][ct], 0, 0, 0);
                h1[1][ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(w0r[st][ct], pb, h1[1][ct], 0, 0, 0);
            }
        }
#pragma unroll
        for (int tl = 0; tl < 2; tl++)
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
#pragma unroll
                for (int q = 0; q < 16; q++) {
                    const float v = h1[tl][ct][q];
                    h1[tl][ct][q] = v > 0.0f ? v : 0.0f;
                }
        RO_STAMP(1);
        // ---- layer 2 (transposed): register m of h1 is K step m
        f32x16_t h2[2][2];
#pragma unroll
        for (int tl = 0; tl < 2; tl++)
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
#pragma unroll
                for (int q = 0; q < 16; q++) h2[tl][ct][q] = 0.0f;
        int zero1 = 0;
        asm volatile("" : "+v"(zero1));   // the operand reads stay in the step loop
        const float2 *w1p = &w1r[0][lane] + zero1;
#pragma unroll
        for (int st = 0; st < 32; st++) {
            const float2 w = w1p[st * 64];
#pragma unroll
            for (int tl = 0; tl < 2; tl++) {
                h2[tl][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.x, h1[tl][st >> 4][st & 15], h2[tl][0], 0, 0, 0);
                h2[tl][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(w.y, h1[tl][st >> 4][st & 15], h2[tl][1], 0, 0, 0);
            }
        }
        RO_STAMP(2);
        // H2 -> the wave's [env][unit] tile (register m of lane (c, h) holds unit 32h + m of
        // env c of tile tl), then lane l reads env l's row
#pragma unroll
        for (int tl = 0; tl < 2; tl++)
#pragma unroll
            for (int m = 0; m < 32; m++) Tw[(32 * tl + c) * 65 + 32 * h + m] = h2[tl][m >> 4][m & 15];
        wave_sync();
        RO_STAMP(3);
        // ---- heads: + b1, relu, the k-ordered chains of logit 0, logit 1, value
        // (the row reads stay in the step loop: hoisted, they would pin 256 VGPRs)
        int zero = 0;
        asm volatile("" : "+v"(zero));
        const float4 *hw = S.hw + zero;
        const float *hrow = Tw + lane * 65 + zero;
        // batches of 8 units: the batch's 8 weight rows and 8 activations are all read before
        // its chains consume them, one LDS round trip per batch (the per-unit form waited on
        // every read: 24% of the step under the segment stamps; a double-buffered 4-unit form
        // measured no better, profiles/r05c/rollout_stamps.txt)
        float l0 = 0.0f, l1 = 0.0f, vv = 0.0f;
#pragma unroll 1
        for (int k0 = 0; k0 < H; k0 += 8) {
            float4 w[8];
            float hz[8];
#pragma unroll
            for (int j = 0; j < 8; j++) { w[j] = hw[k0 + j]; hz[j] = hrow[k0 + j]; }
#pragma unroll
            for (int j = 0; j < 8; j++) {
                float z = __fadd_rn(hz[j], w[j].w);
                z = z > 0.0f ? z : 0.0f;
                l0 = __builtin_fmaf(z, w[j].x, l0);
                l1 = __builtin_fmaf(z, w[j].y, l1);
                vv = __builtin_fmaf(z, w[j].z, vv);
            }
        }
        float lg[2];
        lg[0] = __fadd_rn(l0, S.bp[0]);
        lg[1] = __fadd_rn(l1, S.bp[1]);
        const float v = __fadd_rn(vv, S.bv[0]);
        const float n0 = __fadd_rn(lg[0], gz.x);
        const float n1 = __fadd_rn(lg[1], gz.y);
        const int act = n1 > n0 ? 1 : 0;               // argmax, first maximum
        RO_STAMP(4);
        const float lp = log_prob2(S, lg, act);
        bool done = false;
        float r = 0.0f;
        RO_STAMP(5);
        if (mine) {
            bad |= !isfinite(lp);
            done = cartpole_step(s, act, r);
            ep_ret = __fadd_rn(ep_ret, r);
            ep_len += 1;
        }
        // episode records: the previous step's slots, then this step's counter reservation
        flush_eps(t - 1);
        const uint64_t m = (uint64_t)__ballot(done ? 1 : 0);
        if (m) {
            const int leader = __ffsll((unsigned long long)m) - 1;
            if (lane == leader) pbase = atomicAdd(a.ep_count, (int32_t)__popcll(m));
        }
        pm = m;
        if (done) {
            pret = ep_ret;
            plen = ep_len;
            if (rj < a.rpool_k) {
                s.x = rnx.x; s.x_dot = rnx.y; s.theta = rnx.z; s.theta_dot = rnx.w; s.steps = 0;
                env_pos = rnpos;
                rj++;
            } else {
                WordCursor ec;
                ec.init(seed_key(a.seed_base + (uint64_t)e), 0, env_pos);
                cartpole_reset(s, ec);
                env_pos = ec.pos;
            }
            ep_ret = 0.0f;
            ep_len = 0;
        }
        RO_STAMP(6);
        if (mine) {
#pragma unroll
            for (int d = 0; d < 5; d++) a.obs[row * 5 + d] = x[d];
            a.act[row] = act;
            a.rew_raw[row] = r;
            a.done[row] = done ? 1.0f : 0.0f;
            a.val[row] = v;
            a.logp[row] = lp;
            if (a.rows) {
                a.rows[row * 2] = make_float4(x[0], x[1], x[2], x[3]);
                a.rows[row * 2 + 1] = make_float4(x[4], __int_as_float(act), lp, v);
            }
        }
        wave_sync();                      // this step's tile reads done before the next step's writes
        RO_STAMP(7);
    }
    flush_eps(a.T - 1);
#ifdef BPPO_RO_STAMPS
    if (lane == 0 && a.stamps)
        for (int k = 0; k < RO_NSEG; k++) a.stamps[(size_t)(e >> 6) * RO_NSEG + k] = ro_acc[k];
#endif
    if (mine) {
        store_state(a.cp, a.steps, N, e, s);
        a.env_pos[e] = env_pos;
        a.ep_ret[e] = ep_ret;
        a.ep_len[e] = ep_len;
        oa.store((double)a.T, a.obs_part + (size_t)e * 10);
        if (bad) atomicOr(a.err, 1);
    }
}

// VecEnv::step surface (env.rs:400-487) for host-driven stepping.
__global__ void k_cartpole_step(int N, uint64_t seed_base, float *cp, int32_t *steps,
                                uint64_t *env_pos, float *ep_ret, int32_t *ep_len,
                                const int32_t *actions, float *rew, uint8_t *dn, float *obs,
                                EpisodeRec *eps, int32_t *ep_count, int cap) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    CartPoleState s;
    load_state(cp, steps, N, e, s);
    float r;
    bool done = cartpole_step(s, actions[e], r);
    float er = __fadd_rn(ep_ret[e], r);
    int32_t el = ep_len[e] + 1;
    const int32_t k = wave_episode_slot(done, ep_count);
    if (done) {
        if (k < cap) {
            EpisodeRec rec;
            rec.total_reward[0] = er;
            for (int p = 1; p < BPPO_MAX_PLAYERS; p++) rec.total_reward[p] = 0.0f;
            rec.length = el; rec.env_index = e; rec.step = 0; rec.pad = 0;
            eps[k] = rec;
        }
        WordCursor c;
        c.init(seed_key(seed_base + (uint64_t)e), 0, env_pos[e]);
        cartpole_reset(s, c);
        env_pos[e] = c.pos;
        er = 0.0f; el = 0;
    }
    store_state(cp, steps, N, e, s);
    ep_ret[e] = er; ep_len[e] = el;
    rew[e] = r;
    dn[e] = done ? 1 : 0;
    if (obs) {
        float o[5];
        cartpole_obs(s, o);
        for (int d = 0; d < 5; d++) obs[e * 5 + d] = o[d];
    }
}

__global__ void k_cartpole_observe(int N, const float *cp, const int32_t *steps, float *obs) {
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    CartPoleState s;
    load_state(cp, steps, N, e, s);
    float o[5];
    cartpole_obs(s, o);
    for (int d = 0; d < 5; d++) obs[e * 5 + d] = o[d];
}

// bootstrap (main.rs:878-896): current obs normalised with the UPDATED stats
template <int H, int NL, int ACT>
__global__ void __launch_bounds__(256) k_cartpole_bootstrap(int N, const float *cp,
                                                            const int32_t *steps,
                                                            const float *params, const double *on,
                                                            int norm_on, float *last_v) {
    extern __shared__ __attribute__((aligned(16))) float sP[];
    constexpr CpOffsets O = cp_offsets<H, NL>();
    for (int i = threadIdx.x; i < O.n; i += blockDim.x) sP[i] = params[i];
    __syncthreads();
    int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    CartPoleState s;
    load_state(cp, steps, N, e, s);
    float raw[5], x[5], lg[2], v;
    cartpole_obs(s, raw);
    ObsNorm5 nz;
    nz.load(on, norm_on);
    nz.apply(raw, x);
    cp_forward<H, NL, ACT>(sP, x, lg, v, sP + cp_stage_ofs<H, NL>() + threadIdx.x, blockDim.x);
    last_v[e] = v;
}

template <int H, int NL, int ACT>
__global__ void __launch_bounds__(256) k_cartpole_forward_rows(int B, const float *obs,
                                                               const float *params, float *logits,
                                                               float *values) {
    extern __shared__ __attribute__((aligned(16))) float sP[];
    constexpr CpOffsets O = cp_offsets<H, NL>();
    for (int i = threadIdx.x; i < O.n; i += blockDim.x) sP[i] = params[i];
    __syncthreads();
    int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= B) return;
    float x[5], lg[2], v;
    for (int d = 0; d < 5; d++) x[d] = obs[(size_t)r * 5 + d];
    cp_forward<H, NL, ACT>(sP, x, lg, v, sP + cp_stage_ofs<H, NL>() + threadIdx.x, blockDim.x);
    logits[(size_t)r * 2] = lg[0];
    logits[(size_t)r * 2 + 1] = lg[1];
    values[r] = v;
}

// Merge per-env Welford partials (count T each) into the running stats
// (normalization.rs:37-53 is a sequential Welford over T*N rows; Chan merges
// give the same statistics to f64 rounding).  Two passes with a fixed merge
// order: OBS_PART_BLOCKS blocks each merge a contiguous range of envs (thread-
// sequential, then a block tree), then one thread per dim merges the block
// results in block order into the running stats.
constexpr int OBS_PART_BLOCKS = 64, OBS_MAX_D = 8;
__global__ void __launch_bounds__(256) k_obs_norm_part(int N, int D, double T, const double *part, double *bp) {
    __shared__ double sn[256], sm[256][OBS_MAX_D], sq[256][OBS_MAX_D];
    const int per = (N + gridDim.x - 1) / gridDim.x;
    const int e0 = blockIdx.x * per, e1 = min(N, e0 + per);
    double n = 0.0, mean[OBS_MAX_D], m2[OBS_MAX_D];
    for (int d = 0; d < OBS_MAX_D; d++) mean[d] = m2[d] = 0.0;
    for (int e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const double *pe = part + (size_t)e * 2 * D;
        const double nn = n + T, f = T / nn, g = n * T / nn;
        for (int d = 0; d < D; d++) {
            const double delta = pe[d] - mean[d];
            mean[d] += delta * f;
            m2[d] += pe[D + d] + delta * delta * g;
        }
        n = nn;
    }
    sn[threadIdx.x] = n;
    for (int d = 0; d < D; d++) { sm[threadIdx.x][d] = mean[d]; sq[threadIdx.x][d] = m2[d]; }
    __syncthreads();
    for (int st = blockDim.x / 2; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            const double na = sn[threadIdx.x], nb = sn[threadIdx.x + st], nn = na + nb;
            if (nb > 0) {
                const double f = na > 0 ? nb / nn : 1.0, g = na * nb / nn;
                for (int d = 0; d < D; d++) {
                    const double delta = sm[threadIdx.x + st][d] - sm[threadIdx.x][d];
                    sm[threadIdx.x][d] += delta * f;
                    sq[threadIdx.x][d] += sq[threadIdx.x + st][d] + delta * delta * g;
                }
                sn[threadIdx.x] = nn;
            }
        }
        __syncthreads();
    }
    if (threadIdx.x < D) {
        double *o = bp + ((size_t)blockIdx.x * OBS_MAX_D + threadIdx.x) * 3;
        o[0] = sn[0]; o[1] = sm[0][threadIdx.x]; o[2] = sq[0][threadIdx.x];
    }
}
__global__ void k_obs_norm_final(int D, int nblk, const double *bp, double *on) {
    const int d = threadIdx.x;
    if (d >= D) return;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    // the block partials of 16 blocks are loaded before the in-order merge consumes
    // them: one load round trip per 16 blocks instead of one per block
    constexpr int U = 16;
    for (int b0 = 0; b0 < nblk; b0 += U) {
        double pn[U], pm[U], p2[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const double *o = bp + ((size_t)min(b0 + k, nblk - 1) * OBS_MAX_D + d) * 3;
            pn[k] = o[0]; pm[k] = o[1]; p2[k] = o[2];
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            if (b0 + k >= nblk) break;
            const double nb = pn[k];
            if (nb <= 0) continue;
            const double nn = n + nb, delta = pm[k] - mean;
            mean = n > 0 ? mean + delta * (nb / nn) : pm[k];
            m2 += p2[k] + (n > 0 ? delta * delta * (n * nb / nn) : 0.0);
            n = nn;
        }
    }
    // old stats (count on[2D]) merged with the batch
    const double na = on[2 * D], nn = na + n, delta = mean - on[d];
    const double ma = on[d];
    on[d] = na > 0 ? ma + delta * (n / nn) : mean;
    on[D + d] = on[D + d] + m2 + (na > 0 ? delta * delta * (na * n / nn) : 0.0);
    __syncthreads();
    if (d == 0) on[2 * D] = nn;
}

// ------------------------------------------------------------- launchers ---
// shape x activation: relu (configs/*.toml) or tanh (config.rs:990-992 default)
#define CP_DISPATCH(H_, NL_, CALL)                                                 \
    if (h == H_ && nl == NL_) {                                                    \
        if (c->cfg.relu) CALL(H_, NL_, ACT_RELU); else CALL(H_, NL_, ACT_TANH);   \
        return launch_check(c, __func__);                                          \
    }

static bool cp_supported(int h, int nl) {
    return (h == 16 || h == 32 || h == 64) && (nl == 1 || nl == 2);
}

bppo_status launch_cartpole_reset(bppo_ctx *c) {
    int N = c->N;
    hipLaunchKernelGGL(k_cartpole_reset, dim3((N + 255) / 256), dim3(256), 0, c->stream, N,
                       c->cfg.env_seed_base, c->d_cp, c->d_steps, c->d_env_pos, c->d_ep_ret,
                       c->d_ep_len, nullptr);
    TRY(launch_check(c, __func__));
    if (c->ev_env) BPPO_HIP(c, hipEventRecord(c->ev_env, c->stream));   // env state written
    return BPPO_OK;
}

static bppo_status launch_cartpole_rollout_kernels(bppo_ctx *c, uint64_t base_pos, int norm_on);
// every CartPole rollout variant, then ev_env: the env state it wrote (and the 64-lane
// kernel's Gumbel words / reset pool it read) -- what the next rollout's prep_stream waits for
bppo_status launch_cartpole_rollout(bppo_ctx *c, uint64_t base_pos, const double *, const double *,
                                    int norm_on) {
    const bppo_status s = launch_cartpole_rollout_kernels(c, base_pos, norm_on);
    if (s == BPPO_OK && c->ev_env) BPPO_HIP(c, hipEventRecord(c->ev_env, c->stream));
    return s;
}

static bppo_status launch_cartpole_rollout_kernels(bppo_ctx *c, uint64_t base_pos, int norm_on) {
    const int h = c->cfg.hidden_size, nl = c->cfg.num_hidden;
    // the episode counter and error flags at 0 before the rollout: in the Gumbel kernel when it
    // runs on the update stream (below), else two fills here
    static const bool prep_side = getenv("BPPO_PREP_SIDE") && atoi(getenv("BPPO_PREP_SIDE")) == 1;
    const bool lanes64 = !(getenv("BPPO_ROLLOUT_LANES64") && atoi(getenv("BPPO_ROLLOUT_LANES64")) == 0);
    const bool gum_path = h == 64 && nl == 2 && c->cfg.relu && c->d_gumbel;
    const bool side = gum_path && lanes64 && prep_side && c->prep_stream && c->ev_env && c->ev_prep;
    if (!gum_path || side) {
        BPPO_HIP(c, hipMemsetAsync(c->d_ep_count, 0, 4, c->stream));
        BPPO_HIP(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
    }
    if (!cp_supported(h, nl)) {
        c->err = "CartPole rollout kernel supports MLPs with hidden in {16,32,64} x {1,2} layers";
        return BPPO_ERR_UNSUPPORTED;
    }
    RolloutArgs a;
    a.N = c->N; a.T = c->T; a.seed_base = c->cfg.env_seed_base;
    a.cp = c->d_cp; a.steps = c->d_steps; a.env_pos = c->d_env_pos; a.ep_ret = c->d_ep_ret;
    a.ep_len = c->d_ep_len; a.key = c->rng_key; a.stream = c->cfg.rng_stream; a.base_pos = base_pos;
    a.params = c->d_params; a.n_params = (int)c->net.n_params; a.on = c->d_on; a.norm_on = norm_on;
    a.obs = c->d_obs; a.rew_raw = c->d_rew_raw; a.done = c->d_done; a.val = c->d_val;
    a.logp = c->d_logp; a.act = c->d_act; a.obs_part = c->d_obs_part; a.eps = c->d_eps;
    a.ep_count = c->d_ep_count; a.eps_cap = c->eps_cap; a.err = c->d_err;
    a.rows = nullptr;
    a.stamps = nullptr;
    a.rpool = nullptr; a.rpos = nullptr; a.rpool_k = 0;
    c->rows_from_rollout = false;
    if (gum_path) {
        // the update's packed rows (obs, action, log-prob, value) written by the rollout
        // itself; GAE adds advantage and return, so k_pack_rows is not needed (PopArt
        // trains on normalized values computed at update start: packed there instead)
        if (c->d_rowA && !c->cfg.normalize_values && !getenv("BPPO_NO_FUSED_PACK")) {
            a.rows = c->d_rowA;
            c->rows_from_rollout = true;
        }
        // Gumbel noise for every (t, env, action) first, then the MFMA rollout
        const uint64_t count = (uint64_t)c->T * c->N * 2;
        const uint64_t blocks = ((base_pos + count + 15) >> 4) - (base_pos >> 4);
        // BPPO_PREP_SIDE=1 (r06, A/B): the 64-lane rollout's inputs (Gumbel words, reset pool)
        // on prep_stream, which waits only for the last env-state writer (the previous
        // rollout), so they run beside the previous update instead of between its last
        // minibatch and this rollout.  Kernel traces: the gap before the rollout 285-607 ->
        // 121-295 us, but the update's minibatches 0.2-0.45 ms longer beside them (update span
        // 11.04 / 12.39 vs 11.36 / 12.24 ms, profiles/r06p/): off by default
        hipStream_t ps = side ? c->prep_stream : c->stream;
        if (side) BPPO_HIP(c, hipStreamWaitEvent(ps, c->ev_env, 0));
        hipLaunchKernelGGL(k_gumbel_words, dim3((unsigned)((blocks + 255) / 256)), dim3(256), 0, ps, c->rng_key,
                           (uint64_t)c->cfg.rng_stream, base_pos, count, c->d_gumbel,
                           side ? nullptr : c->d_ep_count, side ? nullptr : (int32_t *)c->d_err);
        TRY(launch_check(c, "k_gumbel_words"));
        // default: the 64-lane kernel (269 registers and 84 KB of LDS per 4-wave block, so
        // the side-stream Fisher-Yates passes still share its CUs): device-bound A/B
        // 0.1-0.28 ms/update faster than r03's half-wave kernel (profiles/r04_rollout/
        // rollout_ab.txt).  BPPO_ROLLOUT_LANES64=0: the half-wave kernel.
        if (!lanes64) {
            const int waves = (c->N + mmb::TR - 1) / mmb::TR;
            hipLaunchKernelGGL(k_cartpole_rollout_mfma, dim3((waves + mmb::WAVES - 1) / mmb::WAVES), dim3(64 * mmb::WAVES),
                               mmb::LDS, c->stream, a, (const float *)c->d_gumbel);
        } else {
            const int waves = (c->N + 63) / 64;
            // BPPO_RESET_POOL_K (tests): a shorter pool (exercises the in-kernel fallback), 0: none
            int pk = RPOOL_K;
            if (const char *v = getenv("BPPO_RESET_POOL_K")) pk = std::max(0, std::min(RPOOL_K, atoi(v)));
            if (c->d_rpool && pk > 0) {
                hipLaunchKernelGGL(k_reset_pool, dim3((c->N + 255) / 256), dim3(256), 0, ps, c->N, pk,
                                   c->cfg.env_seed_base, (const uint64_t *)c->d_env_pos, c->d_rpool, c->d_rpos);
                TRY(launch_check(c, "k_reset_pool"));
                a.rpool = c->d_rpool; a.rpos = c->d_rpos; a.rpool_k = pk;
            }
#ifdef BPPO_RO_STAMPS
            static unsigned long long *d_st = nullptr;
            if (!d_st) BPPO_HIP(c, hipMalloc((void **)&d_st, sizeof(unsigned long long) * (size_t)waves * RO_NSEG));
            a.stamps = d_st;
#endif
            if (side) {
                BPPO_HIP(c, hipEventRecord(c->ev_prep, ps));
                BPPO_HIP(c, hipStreamWaitEvent(c->stream, c->ev_prep, 0));
            }
            hipLaunchKernelGGL(k_cartpole_rollout_mfma64, dim3((waves + mmr::WAVES - 1) / mmr::WAVES),
                               dim3(64 * mmr::WAVES), 0, c->stream, a, (const float *)c->d_gumbel);
#ifdef BPPO_RO_STAMPS
            {   // mean per-wave cycles per segment over every launch; printed every 4 launches
                static double acc_s[RO_NSEG] = {};
                static int nl = 0;
                std::vector<unsigned long long> hs((size_t)waves * RO_NSEG);
                BPPO_HIP(c, hipMemcpyAsync(hs.data(), d_st, hs.size() * 8, hipMemcpyDeviceToHost, c->stream));
                BPPO_HIP(c, hipStreamSynchronize(c->stream));
                for (int w = 0; w < waves; w++)
                    for (int k = 0; k < RO_NSEG; k++) acc_s[k] += (double)hs[(size_t)w * RO_NSEG + k] / waves;
                if (++nl % 4 == 0) {
                    double tot = 0;
                    for (int k = 0; k < RO_NSEG; k++) tot += acc_s[k];
                    fprintf(stderr, "[rostamp] launches=%d cycles/wave/step=%.0f shares:", nl, tot / nl / c->T);
                    for (int k = 0; k < RO_NSEG; k++) fprintf(stderr, " s%d=%.3f", k, acc_s[k] / tot);
                    fprintf(stderr, "\n");
                }
            }
#endif
        }
        TRY(launch_check(c, __func__));
        return BPPO_OK;
    }
    dim3 grid((c->N + 255) / 256), blk(256);
#define L(H_, NL_, A_) hipLaunchKernelGGL((k_cartpole_rollout<H_, NL_, A_>), grid, blk, (cp_lds<H_, NL_>(A_, 256)), c->stream, a)
    CP_DISPATCH(16, 1, L) CP_DISPATCH(16, 2, L) CP_DISPATCH(32, 1, L) CP_DISPATCH(32, 2, L)
    CP_DISPATCH(64, 1, L) CP_DISPATCH(64, 2, L)
#undef L
    return BPPO_ERR_UNSUPPORTED;
}

bppo_status launch_bootstrap(bppo_ctx *c, const double *, const double *, int norm_on) {
    const int h = c->cfg.hidden_size, nl = c->cfg.num_hidden;
    dim3 grid((c->N + 255) / 256), blk(256);
#define L(H_, NL_, A_)                                                                          \
    hipLaunchKernelGGL((k_cartpole_bootstrap<H_, NL_, A_>), grid, blk, (cp_lds<H_, NL_>(A_, 256)), c->stream, c->N, c->d_cp, \
                       c->d_steps, c->d_params, c->d_on, norm_on, c->d_last_v)
    CP_DISPATCH(16, 1, L) CP_DISPATCH(16, 2, L) CP_DISPATCH(32, 1, L) CP_DISPATCH(32, 2, L)
    CP_DISPATCH(64, 1, L) CP_DISPATCH(64, 2, L)
#undef L
    return BPPO_ERR_UNSUPPORTED;
}

bppo_status launch_forward_rows(bppo_ctx *c, const float *d_obs, int B, float *d_logits,
                                float *d_values) {
    const int h = c->cfg.hidden_size, nl = c->cfg.num_hidden;
    dim3 grid((B + 255) / 256), blk(256);
#define L(H_, NL_, A_)                                                                            \
    hipLaunchKernelGGL((k_cartpole_forward_rows<H_, NL_, A_>), grid, blk, (cp_lds<H_, NL_>(A_, 256)), c->stream, B, d_obs, \
                       c->d_params, d_logits, d_values)
    CP_DISPATCH(16, 1, L) CP_DISPATCH(16, 2, L) CP_DISPATCH(32, 1, L) CP_DISPATCH(32, 2, L)
    CP_DISPATCH(64, 1, L) CP_DISPATCH(64, 2, L)
#undef L
    return BPPO_ERR_UNSUPPORTED;
}

bppo_status launch_cartpole_vecenv_step(bppo_ctx *c, const int32_t *d_actions, float *d_rew,
                                        uint8_t *d_done, float *d_obs_out) {
    int N = c->N;
    hipLaunchKernelGGL(k_cartpole_step, dim3((N + 255) / 256), dim3(256), 0, c->stream, N,
                       c->cfg.env_seed_base, c->d_cp, c->d_steps, c->d_env_pos, c->d_ep_ret,
                       c->d_ep_len, d_actions, d_rew, d_done, d_obs_out, c->d_eps, c->d_ep_count,
                       c->eps_cap);
    TRY(launch_check(c, __func__));
    if (c->ev_env) BPPO_HIP(c, hipEventRecord(c->ev_env, c->stream));   // env state written
    return BPPO_OK;
}

bppo_status launch_cartpole_observe(bppo_ctx *c, float *d_obs_out) {
    int N = c->N;
    hipLaunchKernelGGL(k_cartpole_observe, dim3((N + 255) / 256), dim3(256), 0, c->stream, N,
                       c->d_cp, c->d_steps, d_obs_out);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// ---- multi-player envs (D = 86 / 270): the obs columns of the [priv | obs]
// rows normalized in place with the lagged stats (normalization.rs:57-74,
// ppo.rs:292-294; privileged obs stay raw), the raw values kept for the update
__global__ void __launch_bounds__(256) k_obs_norm_rows(int rows, int D, int ld, float *x, float *raw,
                                                       const double *on, float clip) {
    const double cnt = on[2 * D];
    const size_t n = (size_t)rows * D;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / D;
        const int d = (int)(i - r * D);
        float *p = x + r * ld + d;
        const float v = *p;
        if (raw) raw[i] = v;
        if (cnt >= 2.0) {
            double sd = sqrt(on[D + d] / cnt);
            sd = sd < 1e-8 ? 1e-8 : sd;
            float z = (float)(((double)v - on[d]) / sd);
            z = z < -clip ? -clip : z;
            z = z > clip ? clip : z;
            *p = z;
        }
    }
}
bppo_status launch_obs_norm_rows(bppo_ctx *c, int rows, float *x, int ld, float *raw) {
    return launch_obs_norm_rows_on(c, rows, x, ld, raw, c->d_on);
}
bppo_status launch_obs_norm_rows_on(bppo_ctx *c, int rows, float *x, int ld, float *raw, const double *on) {
    const size_t n = (size_t)rows * c->D;
    hipLaunchKernelGGL(k_obs_norm_rows, dim3((unsigned)std::min<size_t>((n + 255) / 256, 8192)), dim3(256), 0,
                       c->stream, rows, c->D, ld, x, raw, on, 10.0f);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// update_batch over all T*N raw rows (normalization.rs:37-53): column-parallel
// per chunk of rows (thread = dim, coalesced along the row), sums shifted by the
// chunk's first row, then the chunks Chan-merged in order into the running stats
constexpr int OBSW_CHUNKS = 256;
__global__ void __launch_bounds__(256) k_obsw_part(size_t rows, int D, const float *raw, double *part) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    const size_t per = (rows + gridDim.y - 1) / gridDim.y;
    const size_t r0 = blockIdx.y * per, r1 = r0 + per < rows ? r0 + per : rows;
    double n = 0.0, s1 = 0.0, s2 = 0.0, k = 0.0;
    if (r0 < r1) k = raw[r0 * D + d];
    for (size_t r = r0; r < r1; r++) {
        const double y = (double)raw[r * D + d] - k;
        s1 += y;
        s2 += y * y;
        n += 1.0;
    }
    double *o = part + ((size_t)blockIdx.y * D + d) * 3;
    o[0] = n;
    o[1] = n > 0 ? k + s1 / n : 0.0;
    o[2] = n > 0 ? s2 - s1 * (s1 / n) : 0.0;
}
__global__ void k_obsw_final(int D, int nchunk, const double *part, double *on) {
    const int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int b = 0; b < nchunk; b++) {
        const double *o = part + ((size_t)b * D + d) * 3;
        const double nb = o[0];
        if (nb <= 0) continue;
        const double nn = n + nb, delta = o[1] - mean;
        mean = n > 0 ? mean + delta * (nb / nn) : o[1];
        m2 += o[2] + (n > 0 ? delta * delta * (n * nb / nn) : 0.0);
        n = nn;
    }
    const double na = on[2 * D], nn = na + n, delta = mean - on[d];
    const double ma = on[d];
    on[d] = na > 0 ? ma + delta * (n / nn) : mean;
    on[D + d] = on[D + d] + m2 + (na > 0 ? delta * delta * (na * n / nn) : 0.0);
}
__global__ void k_obsw_count(int D, double add, double *on) { on[2 * D] += add; }

bppo_status launch_obs_norm_merge(bppo_ctx *c) {
    if (c->wide) {
        const size_t rows = (size_t)c->T * c->N;
        if ((size_t)OBSW_CHUNKS * c->D * 3 > c->obsw_part_n) { c->err = "obs normalizer scratch too small"; return BPPO_ERR_ARG; }
        hipLaunchKernelGGL(k_obsw_part, dim3((c->D + 255) / 256, OBSW_CHUNKS), dim3(256), 0, c->stream, rows, c->D,
                           c->d_obs_raw, c->d_obsw_part);
        hipLaunchKernelGGL(k_obsw_final, dim3((c->D + 255) / 256), dim3(256), 0, c->stream, c->D, OBSW_CHUNKS,
                           c->d_obsw_part, c->d_on);
        hipLaunchKernelGGL(k_obsw_count, dim3(1), dim3(1), 0, c->stream, c->D, (double)rows, c->d_on);
        TRY(launch_check(c, __func__));
        return BPPO_OK;
    }
    if (c->D > OBS_MAX_D) { c->err = "observation normalizer: obs dim > 8"; return BPPO_ERR_UNSUPPORTED; }
    const int nblk = std::min(OBS_PART_BLOCKS, std::max(1, (c->N + 255) / 256));
    hipLaunchKernelGGL(k_obs_norm_part, dim3(nblk), dim3(256), 0, c->stream, c->N, c->D, (double)c->T,
                       c->d_obs_part, c->d_red);
    hipLaunchKernelGGL(k_obs_norm_final, dim3(1), dim3(64), 0, c->stream, c->D, nblk, c->d_red, c->d_on);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// the rollout's completed-episode summary (mean return of player 0, mean length)
// for bppo_rollout_info: per-block f64 partial sums in a fixed order, combined on
// the host — no episode records cross PCIe (there are ~N * T / 20 of them)
// host_slot: the rollout's slot of the pinned host buffer (its device address): [count, err]
// as two int32 in double 0, then the partials -- written here instead of copied after
__global__ void __launch_bounds__(256) k_ep_summary(const EpisodeRec *eps, const int32_t *count, const int32_t *err,
                                                    int cap, double *host_slot) {
    const int cnt = *count;
    const int n = min(cnt, cap);
    double *part = host_slot + 2;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        int32_t *hv = reinterpret_cast<int32_t *>(host_slot);
        hv[0] = cnt;
        hv[1] = *err;
    }
    double sr = 0.0, sl = 0.0;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        sr += (double)eps[i].total_reward[0];
        sl += (double)eps[i].length;
    }
    __shared__ double sh[2][4];
    for (int o = 32; o > 0; o >>= 1) { sr += __shfl_down(sr, o, 64); sl += __shfl_down(sl, o, 64); }
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = sr; sh[1][w] = sl; }
    __syncthreads();
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
        part[2 * blockIdx.x + 1] = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    }
}

bppo_status launch_episode_summary(bppo_ctx *c, double *host_slot) {
    hipLaunchKernelGGL(k_ep_summary, dim3(EP_SUMMARY_BLOCKS), dim3(256), 0, c->stream, c->d_eps, c->d_ep_count,
                       (const int32_t *)c->d_err, c->eps_cap, host_slot);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

}  // namespace bppo

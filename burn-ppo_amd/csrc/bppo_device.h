// bppo_device.h — device-side building blocks shared by the HIP kernels.
//
//  * ChaCha12 block (rand_chacha 0.3.1 layout) and the rand 0.8.5 samplers the
//    reference draws with, evaluated at counter-addressable word positions;
//  * CartPole physics (envs/cartpole.rs:50-106, 272-301) with the glibc
//    sinf/cosf restatement, so transitions are bit-identical to the reference;
//  * the per-row MLP forward with matrixmultiply's summation order (a k-ordered
//    fma chain from 0, bias added after), shared by the rollout, bootstrap and
//    update kernels so the first-minibatch PPO ratio is exactly 1 (ppo.rs:1452).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bppo_math.h"

namespace bppo {

// ------------------------------------------------------------------ ChaCha --
__host__ __device__ __forceinline__ uint32_t rotl32(uint32_t v, int n) { return (v << n) | (v >> (32 - n)); }

#define BPPO_QR(a, b, c, d)                                  \
    a += b; d ^= a; d = rotl32(d, 16);                       \
    c += d; b ^= c; b = rotl32(b, 12);                       \
    a += b; d ^= a; d = rotl32(d, 8);                        \
    c += d; b ^= c; b = rotl32(b, 7);

struct Key8 { uint32_t k[8]; };

// One ChaCha12 block: constants, key, 64-bit block counter (words 12-13),
// stream id (words 14-15).  rand_chacha guts.rs refill_wide.
__host__ __device__ __forceinline__ void chacha12_block(const Key8 &key, uint64_t ctr, uint64_t stream,
                                               uint32_t out[16]) {
    uint32_t x0 = 0x61707865u, x1 = 0x3320646eu, x2 = 0x79622d32u, x3 = 0x6b206574u;
    uint32_t x4 = key.k[0], x5 = key.k[1], x6 = key.k[2], x7 = key.k[3];
    uint32_t x8 = key.k[4], x9 = key.k[5], x10 = key.k[6], x11 = key.k[7];
    uint32_t x12 = (uint32_t)ctr, x13 = (uint32_t)(ctr >> 32);
    uint32_t x14 = (uint32_t)stream, x15 = (uint32_t)(stream >> 32);
#pragma unroll
    for (int r = 0; r < 6; r++) {
        BPPO_QR(x0, x4, x8, x12); BPPO_QR(x1, x5, x9, x13);
        BPPO_QR(x2, x6, x10, x14); BPPO_QR(x3, x7, x11, x15);
        BPPO_QR(x0, x5, x10, x15); BPPO_QR(x1, x6, x11, x12);
        BPPO_QR(x2, x7, x8, x13); BPPO_QR(x3, x4, x9, x14);
    }
    out[0] = x0 + 0x61707865u; out[1] = x1 + 0x3320646eu; out[2] = x2 + 0x79622d32u;
    out[3] = x3 + 0x6b206574u;
    out[4] = x4 + key.k[0]; out[5] = x5 + key.k[1]; out[6] = x6 + key.k[2]; out[7] = x7 + key.k[3];
    out[8] = x8 + key.k[4]; out[9] = x9 + key.k[5]; out[10] = x10 + key.k[6];
    out[11] = x11 + key.k[7];
    out[12] = x12 + (uint32_t)ctr; out[13] = x13 + (uint32_t)(ctr >> 32);
    out[14] = x14 + (uint32_t)stream; out[15] = x15 + (uint32_t)(stream >> 32);
}

// word at absolute stream position pos (one block evaluation; callers that read
// several consecutive words use WordCursor).
__device__ __forceinline__ uint32_t chacha12_word(const Key8 &key, uint64_t stream, uint64_t pos) {
    uint32_t blk[16];
    chacha12_block(key, pos >> 4, stream, blk);
    uint32_t w = blk[0];
    const uint32_t lane = (uint32_t)(pos & 15);
#pragma unroll
    for (int i = 1; i < 16; i++) w = lane == (uint32_t)i ? blk[i] : w;
    return w;
}

// sequential reader (BlockRng semantics) caching the current block in registers
// slot of this lane's episode record: one atomicAdd per wave for all of its
// lanes that finished an episode this step (a per-lane atomic on the one counter
// serialises ~N/20 atomics per step early in training).  Call with every lane
// that may be done active; returns -1 for lanes that are not done.  Record order
// in the buffer is not part of the contract (bppo_rollout_episodes sorts).
__device__ __forceinline__ int32_t wave_episode_slot(bool done, int32_t *count) {
    const uint64_t m = (uint64_t)__ballot(done ? 1 : 0);
    if (m == 0) return -1;
    const int lane = (int)__lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    int32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (int32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    return done ? base + (int32_t)__popcll(m & ((1ull << lane) - 1ull)) : -1;
}

struct WordCursor {
    Key8 key;
    uint64_t stream, pos, cached;
    uint32_t blk[16];
    __device__ __forceinline__ void init(const Key8 &k, uint64_t s, uint64_t p) {
        key = k; stream = s; pos = p; cached = ~0ull;
    }
    __device__ __forceinline__ uint32_t next() {
        uint64_t b = pos >> 4;
        if (b != cached) { chacha12_block(key, b, stream, blk); cached = b; }
        const uint32_t lane = (uint32_t)(pos & 15);
        uint32_t w = blk[0];
#pragma unroll
        for (int i = 1; i < 16; i++) w = lane == (uint32_t)i ? blk[i] : w;
        pos++;
        return w;
    }
};

// rand_core 0.6.4 seed_from_u64 (PCG32 fill)
__host__ __device__ __forceinline__ Key8 seed_key(uint64_t state) {
    Key8 k;
    for (int i = 0; i < 8; i++) {
        state = state * 6364136223846793005ULL + 11634580027462260723ULL;
        uint32_t xs = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        k.k[i] = (xs >> rot) | (xs << ((32 - rot) & 31));
    }
    return k;
}

// rand 0.8.5 UniformFloat<f32> value from one word: (w >> 9 | 1.0 exponent) - 1
__device__ __forceinline__ float unit_from_word(uint32_t w) {
    return __uint_as_float((w >> 9) | 0x3F800000u) - 1.0f;
}

// gen_range(low..high) f32 with rejection (cartpole.rs:275-278)
__device__ __forceinline__ float gen_range_f32(WordCursor &c, float low, float high) {
    const float scale = high - low;
    for (;;) {
        float v = unit_from_word(c.next());
        float res = __fadd_rn(__fmul_rn(v, scale), low);
        if (res < high) return res;
    }
}

// Gumbel noise from one word (utils.rs:20-25): u = gen_range(1e-10..1.0) with
// scale (1.0 - 1e-10)f32 == 1.0 (never rejects), g = -ln(-ln u) with glibc logf.
__device__ __forceinline__ float gumbel_from_word(uint32_t w) {
    float u = __fadd_rn(__fmul_rn(unit_from_word(w), 1.0f), 1e-10f);
    return -bppo_math::logf_glibc(-bppo_math::logf_glibc(u));
}

// the glibc expf / logf tables staged in LDS by a kernel whose lanes each evaluate many of
// them (the masked sampler's 2 A logf, the wide loss's 3 A expf per row): a lane-varying
// index into the __constant__ copies is a vector global load per evaluation, each waited
// on in turn (k_wide_loss<49>: 152 table loads per row)
struct MathLds {
    uint64_t exp2tab[32];
    double linvc[16], llogc[16];
    __device__ __forceinline__ void load() {     // every thread of the block; then a barrier
        if (threadIdx.x < 32) exp2tab[threadIdx.x] = bppo_math::kExp2fTab[threadIdx.x];
        if (threadIdx.x < 16) { linvc[threadIdx.x] = bppo_math::kLogfInvc[threadIdx.x]; llogc[threadIdx.x] = bppo_math::kLogfLogc[threadIdx.x]; }
        __syncthreads();
    }
    __device__ __forceinline__ float expf(float x) const { return bppo_math::expf_glibc_tab(x, exp2tab); }
    __device__ __forceinline__ float logf(float x) const { return bppo_math::logf_glibc_tab(x, linvc, llogc); }
    __device__ __forceinline__ float gumbel(uint32_t w) const {
        float u = __fadd_rn(__fmul_rn(unit_from_word(w), 1.0f), 1e-10f);
        return -logf(-logf(u));
    }
};

// ---------------------------------------------------------------- CartPole --
struct CartPoleState {
    float x, x_dot, theta, theta_dot;
    int32_t steps;
};

// cartpole.rs:11-23 constants as rustc const-folds them (f32)
#define CP_TOTAL_MASS (1.0f + 0.1f)
#define CP_MASS_LEN (0.1f * 0.5f)

__device__ __forceinline__ void cartpole_obs(const CartPoleState &s, float o[5]) {
    o[0] = s.x; o[1] = s.x_dot; o[2] = s.theta; o[3] = s.theta_dot;
    o[4] = __fdiv_rn((float)s.steps, 500.0f);
}

__device__ __forceinline__ void cartpole_reset(CartPoleState &s, WordCursor &c) {
    s.x = gen_range_f32(c, -0.05f, 0.05f);
    s.x_dot = gen_range_f32(c, -0.05f, 0.05f);
    s.theta = gen_range_f32(c, -0.05f, 0.05f);
    s.theta_dot = gen_range_f32(c, -0.05f, 0.05f);
    s.steps = 0;
}

// physics_step + step (cartpole.rs:50-66, 283-301); returns done, writes reward
__device__ __forceinline__ bool cartpole_step(CartPoleState &s, int action, float &reward) {
    const float force = action == 0 ? -10.0f : 10.0f;
    const float cos_t = bppo_math::cosf_glibc(s.theta);
    const float sin_t = bppo_math::sinf_glibc(s.theta);
    const float temp =
        __fdiv_rn(__builtin_fmaf(__fmul_rn(CP_MASS_LEN, __fmul_rn(s.theta_dot, s.theta_dot)), sin_t, force),
                  CP_TOTAL_MASS);
    const float den = __fmul_rn(0.5f, __fsub_rn(4.0f / 3.0f,
                                               __fdiv_rn(__fmul_rn(0.1f, __fmul_rn(cos_t, cos_t)), CP_TOTAL_MASS)));
    const float theta_acc = __fdiv_rn(__builtin_fmaf(9.8f, sin_t, -__fmul_rn(cos_t, temp)), den);
    const float x_acc =
        __fsub_rn(temp, __fdiv_rn(__fmul_rn(__fmul_rn(CP_MASS_LEN, theta_acc), cos_t), CP_TOTAL_MASS));
    s.x_dot = __fadd_rn(s.x_dot, __fmul_rn(0.02f, x_acc));
    s.x = __fadd_rn(s.x, __fmul_rn(0.02f, s.x_dot));
    s.theta_dot = __fadd_rn(s.theta_dot, __fmul_rn(0.02f, theta_acc));
    s.theta = __fadd_rn(s.theta, __fmul_rn(0.02f, s.theta_dot));
    s.steps += 1;
    const float theta_thr = __fdiv_rn(__fmul_rn(12.0f, 3.14159265358979323846f), 180.0f);
    const bool done = fabsf(s.x) > 2.4f || fabsf(s.theta) > theta_thr || s.steps >= 500;
    reward = (done && s.steps < 500) ? 0.0f : 1.0f;
    return done;
}

// ------------------------------------------------------------------ policy --
// log_softmax (Burn activation::log_softmax: (x - max) - ln(sum(exp(x - max))))
// with glibc expf/logf; returns log-prob of `a`, entropy optionally.
struct MathConst {               // the __constant__ tables (kernels without an LDS copy)
    __device__ __forceinline__ float expf(float x) const { return bppo_math::expf_glibc(x); }
    __device__ __forceinline__ float logf(float x) const { return bppo_math::logf_glibc(x); }
};
template <int A, typename M = MathConst>
__device__ __forceinline__ float log_prob_row(const float x[A], int a, const M &T = M{}) {
    float m = x[0];
#pragma unroll
    for (int i = 1; i < A; i++) m = x[i] > m ? x[i] : m;
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < A; i++) s = __fadd_rn(s, T.expf(__fsub_rn(x[i], m)));
    const float lse = T.logf(s);
    float xa = x[0];
#pragma unroll
    for (int i = 1; i < A; i++) xa = a == i ? x[i] : xa;
    return __fsub_rn(__fsub_rn(xa, m), lse);
}

// ------------------------------------------------------------------- MLP ----
// hidden activation (mlp.rs:79, :187-191): relu if configured, else tanh
enum { ACT_NONE = 0, ACT_RELU = 1, ACT_TANH = 2 };
template <int ACT>
__device__ __forceinline__ float act_fwd(float v) {
    if constexpr (ACT == ACT_RELU) return v > 0.0f ? v : 0.0f;
    else if constexpr (ACT == ACT_TANH) return bppo_math::tanhf_glibc_bf(v);
    else return v;
}
// Burn autodiff backward through the activation given its OUTPUT y:
// relu -> g where y > 0; tanh -> g * (1 - y^2) (powi 2, neg, add 1, mul)
template <int ACT>
__device__ __forceinline__ float act_bwd(float g, float y) {
    if constexpr (ACT == ACT_RELU) return y > 0.0f ? g : 0.0f;
    else if constexpr (ACT == ACT_TANH) return __fmul_rn(g, __fsub_rn(1.0f, __fmul_rn(y, y)));
    else return g;
}

// y[o] = act( (sum_k x[k] W[k][o], k-ordered fma chain from 0) + b[o] )
// W row-major [IN][OUT] in LDS (or global).  IN <= 256 (one matrixmultiply KC block).
// tanh: the OUT pre-activations go through this thread's column of an LDS stage
// (element o at stage[o * ss], ss = threads sharing the stage, so a wave's
// accesses are conflict-free) and one rolled loop applies tanh; an unrolled
// per-unit tanh is too large to schedule without spilling.
template <int IN, int OUT, int ACT>
__device__ __forceinline__ void linear_fwd(const float *__restrict__ W, const float *__restrict__ b,
                                           const float (&x)[IN], float (&y)[OUT],
                                           float *stage = nullptr, int ss = 0) {
    static_assert(IN <= 256, "K > KC needs the split-chain path");
#pragma unroll
    for (int o = 0; o < OUT; o++) y[o] = 0.0f;
#pragma unroll
    for (int k = 0; k < IN; k++) {
        const float xk = x[k];
        // one weight row per step: an opaque row pointer stops the scheduler from
        // hoisting all IN*OUT LDS reads ahead of the FMAs (register blow-up)
        int kofs = k * OUT;
        // opaque offset (keeps the LDS address space) that depends on the previous
        // step's accumulator: weight rows are fetched at most one step ahead
        asm volatile("" : "+v"(kofs) : "v"(y[OUT - 1]));
        const float *Wk = W + kofs;
#pragma unroll
        for (int o = 0; o < OUT; o++) y[o] = __builtin_fmaf(xk, Wk[o], y[o]);
    }
    if constexpr (ACT == ACT_TANH) {
#pragma unroll
        for (int o = 0; o < OUT; o++) stage[o * ss] = __fadd_rn(y[o], b[o]);
#pragma unroll 1
        for (int o = 0; o < OUT; o++) stage[o * ss] = bppo_math::tanhf_glibc_bf(stage[o * ss]);
#pragma unroll
        for (int o = 0; o < OUT; o++) y[o] = stage[o * ss];
    } else {
#pragma unroll
        for (int o = 0; o < OUT; o++) y[o] = act_fwd<ACT>(__fadd_rn(y[o], b[o]));
    }
}

// CartPole MLP (obs 5, actions 2) parameter offsets in Burn record order
struct CpOffsets {
    int w0, b0, w1, b1, wp, bp, wv, bv, n;
};
template <int H, int NL>
__host__ __device__ constexpr CpOffsets cp_offsets() {
    // Burn record order: layers[0..NL), policy_head, value_head (mlp.rs:47-62)
    CpOffsets o{};
    int off = 0;
    o.w0 = off; off += 5 * H; o.b0 = off; off += H;
    if (NL == 2) { o.w1 = off; off += H * H; o.b1 = off; off += H; }
    else { o.w1 = o.b1 = -1; }
    o.wp = off; off += H * 2; o.bp = off; off += 2;
    o.wv = off; off += H; o.bv = off; off += 1;
    o.n = off;
    return o;
}

// dynamic LDS of the per-env forward kernels: the parameters, then (tanh) the
// activation stage [H][threads]
template <int H, int NL>
__host__ __device__ constexpr int cp_stage_ofs() { return (cp_offsets<H, NL>().n + 3) & ~3; }
template <int H, int NL>
inline size_t cp_lds(int act, int threads) {
    return (size_t)(cp_stage_ofs<H, NL>() + (act == ACT_TANH ? H * threads : 0)) * sizeof(float);
}

// (stage/ss: the tanh LDS stage of linear_fwd, unused for relu)
template <int H, int NL, int ACT>
__device__ __forceinline__ void cp_forward(const float *__restrict__ P, const float (&x)[5],
                                           float (&lg)[2], float &v, float *stage = nullptr, int ss = 0) {
    constexpr CpOffsets O = cp_offsets<H, NL>();
    float h[H];
    linear_fwd<5, H, ACT>(P + O.w0, P + O.b0, x, h, stage, ss);
    if constexpr (NL == 2) {
        float h2[H];
        linear_fwd<H, H, ACT>(P + O.w1, P + O.b1, h, h2, stage, ss);
        linear_fwd<H, 2, ACT_NONE>(P + O.wp, P + O.bp, h2, lg);
        float vv[1];
        linear_fwd<H, 1, ACT_NONE>(P + O.wv, P + O.bv, h2, vv);
        v = vv[0];
    } else {
        linear_fwd<H, 2, ACT_NONE>(P + O.wp, P + O.bp, h, lg);
        float vv[1];
        linear_fwd<H, 1, ACT_NONE>(P + O.wv, P + O.bv, h, vv);
        v = vv[0];
    }
}

}  // namespace bppo

// k_gae.hip — GAE and the return-normaliser scan.
//
// GAE is a reverse linear recurrence over T per env and embarrassingly parallel
// over N: one lane per env walks t = T-1..0, loading (reward, done, value) rows
// with coalesced 256-B wave accesses (lane = env), UNROLL steps in flight, and
// the carry in registers.  The arithmetic is the reference's op-for-op
// (ppo.rs:1109-1112: delta = fma(gamma*nv, 1-d, r) - v; A = fma(gamma*lambda*(1-d), A, delta)),
// so advantages are bit-identical.  The multiplayer variant fuses the two
// reverse passes of ppo.rs:1179-1253 into one walk with per-player carries in
// registers, keeping each element's op order.
//
// ReturnNormalizer (normalization.rs:115-202, applied at ppo.rs:390-408): the
// rolling return per (env) is a per-env scan; its Welford statistics are a
// global inclusive scan in (t, e) order, done here as a Chan-merge scan in f64.
#include "bppo_internal.h"
#include <algorithm>

namespace bppo {

constexpr int GAE_UNROLL = 8;

__global__ void __launch_bounds__(256) k_gae_1p(const float *__restrict__ r,
                                                const float *__restrict__ d,
                                                const float *__restrict__ v,
                                                const float *__restrict__ lv, int T, int N,
                                                float gamma, float lambda, float *__restrict__ adv,
                                                float *__restrict__ ret) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const float gl = gamma * lambda;    // `gamma * gae_lambda * (1 - d)` is left-assoc
    float last = 0.0f;
    float nv = lv[e];
    int t = T - 1;
    for (; t >= GAE_UNROLL - 1; t -= GAE_UNROLL) {
        float rr[GAE_UNROLL], dd[GAE_UNROLL], vv[GAE_UNROLL];
#pragma unroll
        for (int u = 0; u < GAE_UNROLL; u++) {
            const size_t i = (size_t)(t - u) * N + e;
            rr[u] = r[i]; dd[u] = d[i]; vv[u] = v[i];
        }
#pragma unroll
        for (int u = 0; u < GAE_UNROLL; u++) {
            const size_t i = (size_t)(t - u) * N + e;
            const float om = 1.0f - dd[u];
            const float delta = __fsub_rn(__builtin_fmaf(gamma * nv, om, rr[u]), vv[u]);
            last = __builtin_fmaf(gl * om, last, delta);
            adv[i] = last;
            ret[i] = __fadd_rn(last, vv[u]);
            nv = vv[u];
        }
    }
    for (; t >= 0; t--) {
        const size_t i = (size_t)t * N + e;
        const float vv = v[i], om = 1.0f - d[i];
        const float delta = __fsub_rn(__builtin_fmaf(gamma * nv, om, r[i]), vv);
        last = __builtin_fmaf(gl * om, last, delta);
        adv[i] = last;
        ret[i] = __fadd_rn(last, vv);
        nv = vv;
    }
}

// The CfgB shape (N % 4 == 0, T <= GSEG_WAVES * GSEG_L): one block per 256 envs
// (each lane owns 4 consecutive envs: dwordx4 loads and stores), T cut into
// GSEG_WAVES contiguous segments of L steps, one wave per segment.  Every wave
// issues all of its segment's loads at once (3 L + 1 dwordx4 per lane), turns
// them into delta_t and c_t = gamma*lambda*(1-d_t) elementwise, then the serial
// chain A_t = fma(c_t, A_{t+1}, delta_t) runs segment by segment from the last
// (the carry between waves goes through LDS), so each element sees exactly the
// reference's op sequence and the result is bit-identical to k_gae_1p.  16
// waves per block keep ~16 waves per CU and ~25 x 1 KB loads in flight per wave.
constexpr int GSEG_WAVES = 16, GSEG_L = 8;
__global__ void __launch_bounds__(GSEG_WAVES * 64) k_gae_1p_seg(const float4 *__restrict__ r,
                                                                 const float4 *__restrict__ d,
                                                                 const float4 *__restrict__ v,
                                                                 const float4 *__restrict__ lv, int T, int N4,
                                                                 int L, float gamma, float lambda,
                                                                 float4 *__restrict__ adv, float4 *__restrict__ ret,
                                                                 float2 *__restrict__ pairs) {
    __shared__ float4 carry[GSEG_WAVES][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = blockIdx.x * 64 + lane;
    const bool ok = g < N4;
    const int t0 = w * L, n = max(0, min(T, t0 + L) - t0);   // this wave's steps [t0, t0 + n)
    const float gl = gamma * lambda;
    float4 x0[GSEG_L], x1[GSEG_L], vv[GSEG_L], vnext = make_float4(0.f, 0.f, 0.f, 0.f);
    if (ok) {
#pragma unroll
        for (int u = 0; u < GSEG_L; u++)
            if (u < n) {
                const size_t i = (size_t)(t0 + u) * N4 + g;
                x0[u] = r[i]; x1[u] = d[i]; vv[u] = v[i];
            }
        if (n > 0) vnext = t0 + n < T ? v[(size_t)(t0 + n) * N4 + g] : lv[g];
    }
    // elementwise: x0 <- delta_t = fma(gamma * v_{t+1}, 1 - d_t, r_t) - v_t, x1 <- gamma*lambda*(1 - d_t)
#pragma unroll
    for (int u = 0; u < GSEG_L; u++) {
        if (u >= n) continue;
        const float4 nv = u + 1 < n ? vv[u + 1 < GSEG_L ? u + 1 : u] : vnext;
        float4 &a = x0[u], &b = x1[u];
        const float4 vu = vv[u];
        float om;
        om = 1.0f - b.x; a.x = __fsub_rn(__builtin_fmaf(gamma * nv.x, om, a.x), vu.x); b.x = gl * om;
        om = 1.0f - b.y; a.y = __fsub_rn(__builtin_fmaf(gamma * nv.y, om, a.y), vu.y); b.y = gl * om;
        om = 1.0f - b.z; a.z = __fsub_rn(__builtin_fmaf(gamma * nv.z, om, a.z), vu.z); b.z = gl * om;
        om = 1.0f - b.w; a.w = __fsub_rn(__builtin_fmaf(gamma * nv.w, om, a.w), vu.w); b.w = gl * om;
    }
    // the serial chain, last segment first
    for (int k = GSEG_WAVES - 1; k >= 0; k--) {
        if (w == k) {
            float4 A = k == GSEG_WAVES - 1 ? make_float4(0.f, 0.f, 0.f, 0.f) : carry[k + 1][lane];
#pragma unroll
            for (int u = GSEG_L - 1; u >= 0; u--) {
                if (u >= n) continue;
                A.x = __builtin_fmaf(x1[u].x, A.x, x0[u].x);
                A.y = __builtin_fmaf(x1[u].y, A.y, x0[u].y);
                A.z = __builtin_fmaf(x1[u].z, A.z, x0[u].z);
                A.w = __builtin_fmaf(x1[u].w, A.w, x0[u].w);
                x0[u] = A;
            }
            carry[k][lane] = A;
        }
        __syncthreads();
    }
    if (!ok) return;
#pragma unroll
    for (int u = 0; u < GSEG_L; u++) {
        if (u >= n) continue;
        const size_t i = (size_t)(t0 + u) * N4 + g;
        const float4 A = x0[u], vu = vv[u];
        adv[i] = A;
        const float4 R = make_float4(__fadd_rn(A.x, vu.x), __fadd_rn(A.y, vu.y), __fadd_rn(A.z, vu.z), __fadd_rn(A.w, vu.w));
        ret[i] = R;
        if (pairs) {
            // the update rows' [advantage, return] pairs of these 4 envs: 32 contiguous
            // bytes per lane, adjacent lanes adjacent (2 KB per wave store pair).  The
            // same pairs stored into 64-byte interleaved rows, 8 B per row per lane, cost
            // 241 us of stores at CfgB against 13.5 us for this pattern
            // (scripts/probes/row_store_probe.hip, profiles/r03_row_store_probe.txt)
            float4 *o = reinterpret_cast<float4 *>(pairs + 4 * i);
            o[0] = make_float4(A.x, R.x, A.y, R.y);
            o[1] = make_float4(A.z, R.z, A.w, R.w);
        }
    }
}

template <int P>
__global__ void __launch_bounds__(256) k_gae_mp(const float *__restrict__ ar,
                                                const int32_t *__restrict__ pl,
                                                const float *__restrict__ d,
                                                const float *__restrict__ v,
                                                const float *__restrict__ lvpp, int T, int N,
                                                float gamma, float lambda, float *__restrict__ adv,
                                                float *__restrict__ ret) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    const float gl = gamma * lambda;
    float carry[P], gc[P], nv[P];
#pragma unroll
    for (int p = 0; p < P; p++) { carry[p] = 0.0f; gc[p] = 0.0f; nv[p] = lvpp[(size_t)e * P + p]; }
    for (int t = T - 1; t >= 0; t--) {
        const size_t i = (size_t)t * N + e;
        const int a = pl[i];
        const float dn = d[i], vv = v[i];
        float rw[P];
#pragma unroll
        for (int p = 0; p < P; p++) rw[p] = ar[i * P + p];
        // pass 1 (ppo.rs:1179-1203)
        if (dn > 0.5f) {
#pragma unroll
            for (int p = 0; p < P; p++) carry[p] = 0.0f;
        }
        float ca = 0.0f, ra = 0.0f;
#pragma unroll
        for (int p = 0; p < P; p++) if (p == a) { ca = carry[p]; ra = rw[p]; }
        const float attributed = __fadd_rn(ra, ca);
#pragma unroll
        for (int p = 0; p < P; p++) carry[p] = p == a ? 0.0f : __fadd_rn(carry[p], rw[p]);
        // pass 2 (ppo.rs:1217-1253)
        if (dn > 0.5f) {
#pragma unroll
            for (int p = 0; p < P; p++) { gc[p] = 0.0f; if (p != a) nv[p] = 0.0f; }
        }
        float nva = 0.0f, gca = 0.0f;
#pragma unroll
        for (int p = 0; p < P; p++) if (p == a) { nva = nv[p]; gca = gc[p]; }
        const float om = 1.0f - dn;
        const float delta = __fsub_rn(__builtin_fmaf(gamma * nva, om, attributed), vv);
        const float A = __builtin_fmaf(gl * om, gca, delta);
        adv[i] = A;
        ret[i] = __fadd_rn(A, vv);
#pragma unroll
        for (int p = 0; p < P; p++) if (p == a) { gc[p] = A; nv[p] = vv; }
    }
}

// k_gae_mp with T split over GSEG_WAVES waves of a block (lane = env, 64 envs per
// block): each wave loads its segment's players, dones, values and rewards at once,
// then the per-env state of the two reverse passes (carry[P], gc[P], nv[P]) walks the
// segments from the last to the first through LDS, one wave at a time, with the op
// sequence of k_gae_mp per element (bit-identical).  At CfgD (N = 32768) the one-lane-
// per-env kernel had 2 waves per CU; this one has 32, and every load is issued up front.
template <int P>
__global__ void __launch_bounds__(GSEG_WAVES * 64) k_gae_mp_seg(const float *__restrict__ ar,
                                                               const int32_t *__restrict__ pl,
                                                               const float *__restrict__ d,
                                                               const float *__restrict__ v,
                                                               const float *__restrict__ lvpp, int T, int N, int L,
                                                               float gamma, float lambda, float *__restrict__ adv,
                                                               float *__restrict__ ret) {
    __shared__ float st[3 * P][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;
    const bool ok = e < N;
    const int t0 = w * L, n = max(0, min(T, t0 + L) - t0);
    const float gl = gamma * lambda;
    int a_[GSEG_L];
    float dn_[GSEG_L], v_[GSEG_L], rw_[GSEG_L][P];
    if (ok) {
#pragma unroll
        for (int u = 0; u < GSEG_L; u++)
            if (u < n) {
                const size_t i = (size_t)(t0 + u) * N + e;
                a_[u] = pl[i]; dn_[u] = d[i]; v_[u] = v[i];
#pragma unroll
                for (int p = 0; p < P; p++) rw_[u][p] = ar[i * P + p];
            }
    }
    float out_a[GSEG_L];
    for (int k = GSEG_WAVES - 1; k >= 0; k--) {
        if (w == k && ok) {
            float carry[P], gc[P], nv[P];
#pragma unroll
            for (int p = 0; p < P; p++) {
                if (k == GSEG_WAVES - 1) { carry[p] = 0.0f; gc[p] = 0.0f; nv[p] = lvpp[(size_t)e * P + p]; }
                else { carry[p] = st[p][lane]; gc[p] = st[P + p][lane]; nv[p] = st[2 * P + p][lane]; }
            }
#pragma unroll
            for (int u = GSEG_L - 1; u >= 0; u--) {
                if (u >= n) continue;
                const int a = a_[u];
                const float dn = dn_[u], vv = v_[u];
                if (dn > 0.5f) {
#pragma unroll
                    for (int p = 0; p < P; p++) carry[p] = 0.0f;
                }
                float ca = 0.0f, ra = 0.0f;
#pragma unroll
                for (int p = 0; p < P; p++) if (p == a) { ca = carry[p]; ra = rw_[u][p]; }
                const float attributed = __fadd_rn(ra, ca);
#pragma unroll
                for (int p = 0; p < P; p++) carry[p] = p == a ? 0.0f : __fadd_rn(carry[p], rw_[u][p]);
                if (dn > 0.5f) {
#pragma unroll
                    for (int p = 0; p < P; p++) { gc[p] = 0.0f; if (p != a) nv[p] = 0.0f; }
                }
                float nva = 0.0f, gca = 0.0f;
#pragma unroll
                for (int p = 0; p < P; p++) if (p == a) { nva = nv[p]; gca = gc[p]; }
                const float om = 1.0f - dn;
                const float delta = __fsub_rn(__builtin_fmaf(gamma * nva, om, attributed), vv);
                const float A = __builtin_fmaf(gl * om, gca, delta);
                out_a[u] = A;
#pragma unroll
                for (int p = 0; p < P; p++) if (p == a) { gc[p] = A; nv[p] = vv; }
            }
#pragma unroll
            for (int p = 0; p < P; p++) { st[p][lane] = carry[p]; st[P + p][lane] = gc[p]; st[2 * P + p][lane] = nv[p]; }
        }
        __syncthreads();
    }
    if (!ok) return;
#pragma unroll
    for (int u = 0; u < GSEG_L; u++) {
        if (u >= n) continue;
        const size_t i = (size_t)(t0 + u) * N + e;
        adv[i] = out_a[u];
        ret[i] = __fadd_rn(out_a[u], v_[u]);
    }
}

bppo_status launch_gae_1p(const float *r, const float *d, const float *v, const float *lv, int T,
                          int N, float gamma, float lambda, float *adv, float *ret, hipStream_t s,
                          float2 *pairs, bool *pairs_done, hipError_t *herr) {
    if (pairs_done) *pairs_done = false;
    if (T <= 0 || N <= 0) return BPPO_OK;
    const bool al = ((uintptr_t)r | (uintptr_t)d | (uintptr_t)v | (uintptr_t)lv | (uintptr_t)adv | (uintptr_t)ret |
                     (uintptr_t)pairs) % 16 == 0;   // k_gae_1p_seg stores the pairs as float4
    if (N % 4 == 0 && T <= GSEG_WAVES * GSEG_L && al) {
        const int N4 = N / 4, L = (T + GSEG_WAVES - 1) / GSEG_WAVES;
        hipLaunchKernelGGL(k_gae_1p_seg, dim3((N4 + 63) / 64), dim3(GSEG_WAVES * 64), 0, s, (const float4 *)r,
                           (const float4 *)d, (const float4 *)v, (const float4 *)lv, T, N4, L, gamma, lambda,
                           (float4 *)adv, (float4 *)ret, pairs);
        if (pairs_done) *pairs_done = pairs != nullptr;
    } else {
        hipLaunchKernelGGL(k_gae_1p, dim3((N + 255) / 256), dim3(256), 0, s, r, d, v, lv, T, N, gamma,
                           lambda, adv, ret);
    }
    const hipError_t e = hipGetLastError();
    if (herr) *herr = e;
    return e == hipSuccess ? BPPO_OK : BPPO_ERR_HIP;
}

bppo_status launch_gae_mp(const float *ar, const int32_t *pl, const float *d, const float *v,
                          const float *lvpp, int T, int N, int P, float gamma, float lambda,
                          float *adv, float *ret, hipStream_t s, hipError_t *herr) {
    if (T <= 0 || N <= 0) return BPPO_OK;
    if (T <= GSEG_WAVES * GSEG_L && P >= 1 && P <= 6) {
        const int L = (T + GSEG_WAVES - 1) / GSEG_WAVES;
        const dim3 gs((N + 63) / 64), bs(GSEG_WAVES * 64);
#define MPSEG(P_) hipLaunchKernelGGL(k_gae_mp_seg<P_>, gs, bs, 0, s, ar, pl, d, v, lvpp, T, N, L, gamma, lambda, adv, ret)
        switch (P) {
        case 1: MPSEG(1); break;
        case 2: MPSEG(2); break;
        case 3: MPSEG(3); break;
        case 4: MPSEG(4); break;
        case 5: MPSEG(5); break;
        default: MPSEG(6); break;
        }
#undef MPSEG
        const hipError_t e = hipGetLastError();
        if (herr) *herr = e;
        return e == hipSuccess ? BPPO_OK : BPPO_ERR_HIP;
    }
    dim3 g((N + 255) / 256), b(256);
    switch (P) {
    case 1: hipLaunchKernelGGL(k_gae_mp<1>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    case 2: hipLaunchKernelGGL(k_gae_mp<2>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    case 3: hipLaunchKernelGGL(k_gae_mp<3>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    case 4: hipLaunchKernelGGL(k_gae_mp<4>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    case 5: hipLaunchKernelGGL(k_gae_mp<5>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    case 6: hipLaunchKernelGGL(k_gae_mp<6>, g, b, 0, s, ar, pl, d, v, lvpp, T, N, gamma, lambda, adv, ret); break;
    default: return BPPO_ERR_ARG;
    }
    const hipError_t e = hipGetLastError();
    if (herr) *herr = e;
    return e == hipSuccess ? BPPO_OK : BPPO_ERR_HIP;
}

// --------------------------------------------------------- ReturnNormalizer --
__device__ __forceinline__ Welford wmerge(Welford a, Welford b) {
    if (b.n == 0.0) return a;
    if (a.n == 0.0) return b;
    const double n = a.n + b.n, dl = b.mean - a.mean;
    Welford r;
    r.n = n;
    r.mean = a.mean + dl * (b.n / n);
    r.m2 = a.m2 + b.m2 + dl * dl * (a.n * b.n / n);
    return r;
}
// normalization.rs:171-181 single-sample update
__device__ __forceinline__ void wpush(Welford &s, double x) {
    s.n += 1.0;
    const double delta = x - s.mean;
    s.mean += delta / s.n;
    s.m2 += delta * (x - s.mean);
}

constexpr int RN_IPT = 16, RN_BLOCK = 256, RN_SEG = RN_IPT * RN_BLOCK;

// per-env rolling returns (update_return / reset_player after the stats update).
// One thread per env walks T: the reward/done loads of RN_TU steps are issued
// before the chain that consumes them (one load round trip per RN_TU steps, not
// per step).  Alone it runs 75 us at CfgB; in the loop it shares the GPU with the
// side-stream shuffle passes (~300 us, the same with one-wave blocks: r02r)
constexpr int RN_TU = 16;
__global__ void k_rn_returns(int T, int N, double gamma, const float *__restrict__ rew_raw,
                             const float *__restrict__ done, double *__restrict__ returns_state,
                             double *__restrict__ X) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    double x = returns_state[e];
    // whole RN_TU blocks without a break inside (a conditional exit let the compiler sink
    // every load next to its use: one round trip per step), then the tail
    int t0 = 0;
    for (; t0 + RN_TU <= T; t0 += RN_TU) {
        float r[RN_TU], d[RN_TU];
#pragma unroll
        for (int k = 0; k < RN_TU; k++) {
            const size_t i = (size_t)(t0 + k) * N + e;
            r[k] = rew_raw[i];
            d[k] = done[i];
        }
#pragma unroll
        for (int k = 0; k < RN_TU; k++) {
            x = x * gamma + (double)r[k];
            X[(size_t)(t0 + k) * N + e] = x;
            if (d[k] != 0.0f) x = 0.0;
        }
    }
    for (; t0 < T; t0++) {
        const size_t i = (size_t)t0 * N + e;
        x = x * gamma + (double)rew_raw[i];
        X[i] = x;
        if (done[i] != 0.0f) x = 0.0;
    }
    returns_state[e] = x;
}

// multi-player (ppo.rs:388-408): one rolling return per (env, player), updated
// and pushed for the ACTING player only (normalization.rs:163-186), reset for
// that player when the step ends the episode.  X in (t, e) order as above.
// valid (opponent pool, nullable): only learner turns enter the variance stats
// (ppo.rs:982-989); other rows carry a NaN in X, which the scan skips
__global__ void k_rn_returns_mp(int T, int N, int P, double gamma, const float *rew_raw, const float *done,
                                const int32_t *players, const float *valid, double *returns_state, double *X) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    double R0 = returns_state[(size_t)e * P], R1 = P > 1 ? returns_state[(size_t)e * P + 1] : 0.0;
    double R2 = P > 2 ? returns_state[(size_t)e * P + 2] : 0.0, R3 = P > 3 ? returns_state[(size_t)e * P + 3] : 0.0;
    auto step = [&](size_t i, int p, float r, float d, bool ok) {
        double x = p == 0 ? R0 : p == 1 ? R1 : p == 2 ? R2 : R3;
        x = x * gamma + (double)r;
        X[i] = ok ? x : __longlong_as_double(0x7ff8000000000000ll);
        if (d != 0.0f) x = 0.0;
        R0 = p == 0 ? x : R0; R1 = p == 1 ? x : R1; R2 = p == 2 ? x : R2; R3 = p == 3 ? x : R3;
    };
    const bool has_valid = valid != nullptr;
    const float *vsrc = has_valid ? valid : done;  // read unconditionally (a guarded load was a branch + wait)
    int t0 = 0;
    for (; t0 + RN_TU <= T; t0 += RN_TU) {       // the loads of RN_TU steps ahead of their chain
        int pl[RN_TU];
        float r[RN_TU], d[RN_TU], vv[RN_TU];
#pragma unroll
        for (int k = 0; k < RN_TU; k++) {
            const size_t i = (size_t)(t0 + k) * N + e;
            pl[k] = players[i]; r[k] = rew_raw[i]; d[k] = done[i]; vv[k] = vsrc[i];
        }
        bool ok[RN_TU];
#pragma unroll
        for (int k = 0; k < RN_TU; k++) ok[k] = !has_valid || vv[k] > 0.5f;
#pragma unroll
        for (int k = 0; k < RN_TU; k++) step((size_t)(t0 + k) * N + e, pl[k], r[k], d[k], ok[k]);
    }
    for (; t0 < T; t0++) {
        const size_t i = (size_t)t0 * N + e;
        step(i, players[i], rew_raw[i], done[i], !valid || valid[i] > 0.5f);
    }
    returns_state[(size_t)e * P] = R0;
    if (P > 1) returns_state[(size_t)e * P + 1] = R1;
    if (P > 2) returns_state[(size_t)e * P + 2] = R2;
    if (P > 3) returns_state[(size_t)e * P + 3] = R3;
}

// ppo.rs:412-428: the acting player's entry of all_rewards is the normalized
// acting reward; the other players keep their raw rewards
__global__ void k_rn_scatter_acting(size_t n, int P, const int32_t *players, const float *rew, float *all_r) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        all_r[i * P + players[i]] = rew[i];
}

// block-level exclusive scan of Welford states held one per thread (Hillis-Steele)
__device__ Welford block_exclusive_scan(Welford mine, Welford *sh) {
    sh[threadIdx.x] = mine;
    __syncthreads();
    for (int off = 1; off < (int)blockDim.x; off <<= 1) {
        Welford v = sh[threadIdx.x];
        Welford u = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : Welford{0, 0, 0};
        __syncthreads();
        sh[threadIdx.x] = threadIdx.x >= (unsigned)off ? wmerge(u, v) : v;
        __syncthreads();
    }
    Welford incl = sh[threadIdx.x];
    Welford excl = threadIdx.x > 0 ? sh[threadIdx.x - 1] : Welford{0, 0, 0};
    (void)incl;
    __syncthreads();
    return excl;
}

// the block's RN_SEG returns staged through LDS with coalesced loads; thread t
// then walks its RN_IPT consecutive values (one pad double per RN_IPT keeps the
// per-thread rows on distinct banks)
// (all RN_IPT loads of a thread issued before the LDS stores: the plain loop waited on
// each load in turn; the raw rewards of k_rn_apply are staged the same way)
constexpr int RN_PAD = RN_IPT + 1;
template <typename V>
__device__ __forceinline__ void rn_stage(size_t n, const V *X, V *xs) {
    const size_t base = (size_t)blockIdx.x * RN_SEG;
    V v[RN_IPT];
#pragma unroll
    for (int j = 0; j < RN_IPT; j++) {
        const size_t i = base + threadIdx.x + (size_t)j * RN_BLOCK;
        v[j] = i < n ? X[i] : (V)0;
    }
#pragma unroll
    for (int j = 0; j < RN_IPT; j++) {
        const int k = threadIdx.x + j * RN_BLOCK;
        xs[(k / RN_IPT) * RN_PAD + (k % RN_IPT)] = v[j];
    }
    __syncthreads();
}

__global__ void __launch_bounds__(RN_BLOCK) k_rn_block_agg(size_t n, const double *X, Welford *agg) {
    __shared__ Welford sh[RN_BLOCK];
    __shared__ double xs[RN_BLOCK * RN_PAD];
    rn_stage(n, X, xs);
    const size_t base = (size_t)blockIdx.x * RN_SEG + (size_t)threadIdx.x * RN_IPT;
    Welford s{0, 0, 0};
    for (int k = 0; k < RN_IPT; k++)
        if (base + k < n && !isnan(xs[threadIdx.x * RN_PAD + k])) wpush(s, xs[threadIdx.x * RN_PAD + k]);
    Welford ex = block_exclusive_scan(s, sh);
    if (threadIdx.x == blockDim.x - 1) agg[blockIdx.x] = wmerge(ex, s);
}

// exclusive scan of the block aggregates, seeded with the running stats
__global__ void __launch_bounds__(1024) k_rn_agg_scan(int nb, Welford *agg, double *stats) {
    __shared__ Welford sh[1024];
    const int per = (nb + 1023) / 1024;
    const int lo = threadIdx.x * per;
    Welford s{0, 0, 0};
    for (int k = 0; k < per; k++)
        if (lo + k < nb) s = wmerge(s, agg[lo + k]);
    Welford ex = block_exclusive_scan(s, sh);
    Welford run = wmerge(Welford{stats[2], stats[0], stats[1]}, ex);
    for (int k = 0; k < per; k++)
        if (lo + k < nb) {
            Welford a = agg[lo + k];
            agg[lo + k] = run;            // exclusive prefix of block lo+k
            run = wmerge(run, a);
        }
    if (threadIdx.x == blockDim.x - 1 || (lo < nb && lo + per >= nb)) {
        if (lo < nb && lo + per >= nb) { stats[0] = run.mean; stats[1] = run.m2; stats[2] = run.n; }
    }
}

__global__ void __launch_bounds__(RN_BLOCK) k_rn_apply(size_t n, const double *X,
                                                       const float *rew_raw, const Welford *agg,
                                                       float clip, float *rew) {
    __shared__ Welford sh[RN_BLOCK];
    __shared__ double xs[RN_BLOCK * RN_PAD];
    __shared__ float rs[RN_BLOCK * RN_PAD];
    rn_stage(n, rew_raw, rs);                     // the raw rewards, replaced in place below
    rn_stage(n, X, xs);
    const size_t base = (size_t)blockIdx.x * RN_SEG + (size_t)threadIdx.x * RN_IPT;
    Welford s{0, 0, 0};
    for (int k = 0; k < RN_IPT; k++)
        if (base + k < n && !isnan(xs[threadIdx.x * RN_PAD + k])) wpush(s, xs[threadIdx.x * RN_PAD + k]);
    Welford ex = block_exclusive_scan(s, sh);
    Welford run = wmerge(agg[blockIdx.x], ex);
    for (int k = 0; k < RN_IPT; k++) {
        const size_t i = base + k;
        if (i >= n) break;
        if (!isnan(xs[threadIdx.x * RN_PAD + k])) wpush(run, xs[threadIdx.x * RN_PAD + k]);
        float r = rs[threadIdx.x * RN_PAD + k];
        if (run.n >= 2.0) {                                  // normalization.rs:187-197
            const double sd = sqrt(run.m2 / run.n + 1e-8);
            float z = (float)((double)r / sd);
            z = z < -clip ? -clip : z;
            z = z > clip ? clip : z;
            r = z;
        }
        rs[threadIdx.x * RN_PAD + k] = r;
    }
    __syncthreads();
    const size_t b0 = (size_t)blockIdx.x * RN_SEG;
    for (int k = threadIdx.x; k < RN_SEG; k += RN_BLOCK)
        if (b0 + k < n) rew[b0 + k] = rs[(k / RN_IPT) * RN_PAD + (k % RN_IPT)];
}

bppo_status launch_return_norm(bppo_ctx *c) {
    const size_t n = (size_t)c->T * c->N;
    const int nb = (int)((n + RN_SEG - 1) / RN_SEG);
    if (c->wide)
        hipLaunchKernelGGL(k_rn_returns_mp, dim3((c->N + 255) / 256), dim3(256), 0, c->stream, c->T, c->N, c->P,
                           c->cfg.gamma, c->d_rew_raw, c->d_done, c->d_players, c->n_opp ? c->d_valid : nullptr,
                           c->d_rn_returns, c->d_X);
    else
        hipLaunchKernelGGL(k_rn_returns, dim3((c->N + 255) / 256), dim3(256), 0, c->stream, c->T, c->N,
                           c->cfg.gamma, c->d_rew_raw, c->d_done, c->d_rn_returns, c->d_X);
    hipLaunchKernelGGL(k_rn_block_agg, dim3(nb), dim3(RN_BLOCK), 0, c->stream, n, c->d_X,
                       c->d_scan_agg);
    hipLaunchKernelGGL(k_rn_agg_scan, dim3(1), dim3(1024), 0, c->stream, nb, c->d_scan_agg,
                       c->d_rn_stats);
    hipLaunchKernelGGL(k_rn_apply, dim3(nb), dim3(RN_BLOCK), 0, c->stream, n, c->d_X, c->d_rew_raw,
                       c->d_scan_agg, (float)c->cfg.return_clip, c->d_rew);
    if (c->wide)
        hipLaunchKernelGGL(k_rn_scatter_acting, dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)), dim3(256), 0,
                           c->stream, n, c->P, c->d_players, c->d_rew, c->d_allr);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

}  // namespace bppo

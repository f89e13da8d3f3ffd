// k_update.hip — ppo_update on the device (ppo.rs:1661-2112).
//
//  * shuffle: shuffle_engine.hip (host draw chain) + k_shuffle.hip (permutation);
//  * per minibatch: gather by the shuffled indices (ppo.rs:1833-1857), raw
//    advantage stats + normalisation (ppo.rs:1905-1917, utils.rs:80-89), fused
//    forward + clipped-surrogate loss + backward (ppo.rs:1385-1502) with the
//    weight-gradient reductions staged through LDS per wave, per-wave partial
//    gradients reduced in fixed order (deterministic), per-tensor norm clip +
//    Adam (main.rs:264-268).
#include <algorithm>
#include <cstdlib>
#include "bppo_internal.h"
#include "bppo_mlp64.h"

namespace bppo {

constexpr int STAT_BLOCKS = 1024;   // partial blocks of the explained-variance sums

// =========================================================== fwd + bwd ====
// metric slots appended after the parameters in the gradient slab
enum { M_PL = 0, M_VL, M_H, M_KL, M_CF, M_V, M_R, M_VE, M_VE2, M_VEMAX, M_N, NUM_M };

// per-tensor norm clip + Adam arguments (k_adam1 / k_adam, and the minibatch kernels' tail)
constexpr int ADAM_CHUNK = 4096;
struct AdamTensor { int off, len; float c1, c2; };
struct AdamArgs {
    float *params, *grad, *m1, *m2;
    double *part;
    AdamTensor t[32];
    int blk0[33];          // first block of tensor i; blk0[nt] = total blocks
    int nt;
    float lr, max_norm, eps, inv_world;
};
constexpr int SLAB_GROUPS = 32;      // the slab's block rows are summed in 32 groups, then the groups in order

struct MbArgs {
    const float *obs, *logp, *adv, *ret, *val;
    const int32_t *act;
    const uint32_t *perm;
    uint32_t start, n;
    const float *params;
    const float *mb_stats;
    float *slab;           // [waves][np + NUM_M]
    int np;
    float lo, hi, ceps;    // clip bounds
    float inv_mb, ent_coef, value_coef;
    int clip_value;
    const float4 *rowA;    // packed rows A [B][2] float4 and B [B] float2 (bppo_internal.h d_rowA / d_rowB) or nullptr
    const float2 *rowB;
    unsigned long long *stamps;   // diagnostic build only (BPPO_MB_STAMPS): per-wave segment cycles
};

// diagnostic build (-DBPPO_MB_STAMPS): s_memtime segment sums per wave
// (cdna_hip_programming.md §7 in-kernel stamps); read the shares, not the time
#ifdef BPPO_MB_STAMPS
constexpr int MB_NSEG = 11;
#define MB_STAMP(k)                                                                              \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long t_;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");               \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        st_acc[k] += t_ - st_prev;                                                               \
        st_prev = t_;                                                                            \
    } while (0)
#else
#define MB_STAMP(k) \
    do {            \
    } while (0)
#endif

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
    return v;
}

// per-wave LDS staging of 64 rows; row-major [row][H] with the column XOR-ed by
// the row, so lane-per-row writes spread over banks and row reads stay broadcast
template <int H>
struct WaveStage {
    float a[64 * H];
    float b[64 * H];
    float x[64][8];
    float l[64][4];
    __device__ __forceinline__ static int at(int row, int col) { return row * H + (col ^ (row & (H - 1))); }
};

template <int H, int NL, int ACT>
__global__ void __launch_bounds__(256, 1) k_minibatch(MbArgs g) {
    constexpr CpOffsets O = cp_offsets<H, NL>();
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float *sPbase = smem;
    WaveStage<H> *stages = reinterpret_cast<WaveStage<H> *>(smem + ((O.n + 3) & ~3));
    for (int i = threadIdx.x; i < O.n; i += blockDim.x) sPbase[i] = g.params[i];
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    WaveStage<H> &S = stages[wv];
    const int gwave = blockIdx.x * (blockDim.x >> 6) + wv;
    const int nwaves = gridDim.x * (blockDim.x >> 6);
    const float mean = g.mb_stats[0], denom = g.mb_stats[1] + 1e-8f;

    // persistent per-lane gradient accumulators (lane = output column / feature)
    float gW0[5], gb0 = 0.0f, gW1[H], gb1 = 0.0f;
    float gP0 = 0.0f, gP1 = 0.0f, gV = 0.0f, gbp0 = 0.0f, gbp1 = 0.0f, gbv = 0.0f;
#pragma unroll
    for (int k = 0; k < 5; k++) gW0[k] = 0.0f;
#pragma unroll
    for (int k = 0; k < H; k++) gW1[k] = 0.0f;
    float m_pl = 0, m_vl = 0, m_h = 0, m_kl = 0, m_cf = 0, m_v = 0, m_r = 0, m_ve = 0, m_ve2 = 0;
    float m_vemax = -INFINITY, m_n = 0;

    for (uint32_t base = (uint32_t)gwave * 64; base < g.n; base += (uint32_t)nwaves * 64) {
        const uint32_t r = base + lane;
        const bool valid = r < g.n;
        int zero = 0;
        asm volatile("" : "+v"(zero));   // keep weight reads inside the chunk loop (no LICM spill)
        const float *sP = sPbase + zero;
        float x[5] = {0, 0, 0, 0, 0};
        int a = 0;
        float olp = 0.0f, A = 0.0f, R = 0.0f, ov = 0.0f;
        if (valid) {
            const uint32_t idx = g.perm[g.start + r];
#pragma unroll
            for (int d = 0; d < 5; d++) x[d] = g.obs[(size_t)idx * 5 + d];
            a = g.act[idx]; olp = g.logp[idx]; A = g.adv[idx]; R = g.ret[idx];
            if (g.clip_value) ov = g.val[idx];
        }
        const float An = __fdiv_rn(__fsub_rn(A, mean), denom);   // utils.rs:88
        // ---- forward (same code path as the rollout: ratio == 1 at first mb)
        float h1[H];
        linear_fwd<5, H, ACT>(sP + O.w0, sP + O.b0, x, h1, S.a + lane, 64);   // tanh stage: S.a column-major
        // relu: the backward needs only the sign bits; tanh re-reads y from LDS
        uint64_t m1 = 0, m2 = 0;
#pragma unroll
        for (int k = 0; k < H; k++) m1 |= (h1[k] > 0.0f ? 1ull : 0ull) << k;
        float hl[H];
        if constexpr (NL == 2) {
            linear_fwd<H, H, ACT>(sP + O.w1, sP + O.b1, h1, hl, S.a + lane, 64);
        } else {
#pragma unroll
            for (int k = 0; k < H; k++) hl[k] = h1[k];
        }
#pragma unroll
        for (int k = 0; k < H; k++) m2 |= (hl[k] > 0.0f ? 1ull : 0ull) << k;
        float lg[2], vv[1];
        linear_fwd<H, 2, ACT_NONE>(sP + O.wp, sP + O.bp, hl, lg);
        linear_fwd<H, 1, ACT_NONE>(sP + O.wv, sP + O.bv, hl, vv);
        const float v = vv[0];
        // ---- loss terms (ppo.rs:1444-1487)
        float mx = lg[0] > lg[1] ? lg[0] : lg[1];
        const float e0 = bppo_math::expf_glibc(__fsub_rn(lg[0], mx));
        const float e1 = bppo_math::expf_glibc(__fsub_rn(lg[1], mx));
        const float lse = bppo_math::logf_glibc(__fadd_rn(e0, e1));
        const float ls0 = __fsub_rn(__fsub_rn(lg[0], mx), lse);
        const float ls1 = __fsub_rn(__fsub_rn(lg[1], mx), lse);
        const float p0 = bppo_math::expf_glibc(ls0), p1 = bppo_math::expf_glibc(ls1);
        const float Hn = -__fadd_rn(__fmul_rn(p0, ls0), __fmul_rn(p1, ls1));
        const float newlp = a == 1 ? ls1 : ls0;
        const float log_ratio = __fsub_rn(newlp, olp);
        const float ratio = bppo_math::expf_glibc(log_ratio);
        const float na = -An;
        const float pl1 = __fmul_rn(na, ratio);
        const float rc = ratio < g.lo ? g.lo : (ratio > g.hi ? g.hi : ratio);
        const float pl2 = __fmul_rn(na, rc);
        const bool rhs = pl1 < pl2;
        const float pl = rhs ? pl2 : pl1;
        float vl, dvl;
        if (g.clip_value) {
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
        // gradients of the loss w.r.t. logits and value
        const float g_ratio = (!rhs || (ratio >= g.lo && ratio <= g.hi)) ? -An * g.inv_mb : 0.0f;
        const float g_lr = g_ratio * ratio;
        const float ec = g.ent_coef * g.inv_mb;
        float dl0 = g_lr * ((a == 0 ? 1.0f : 0.0f) - p0) + ec * p0 * (ls0 + Hn);
        float dl1 = g_lr * ((a == 1 ? 1.0f : 0.0f) - p1) + ec * p1 * (ls1 + Hn);
        float dv = g.value_coef * 0.5f * g.inv_mb * dvl;
        if (!valid) { dl0 = dl1 = dv = 0.0f; }
        if (valid) {
            const float ve = fabsf(__fsub_rn(v, R));
            m_pl += pl; m_vl += vl; m_h += Hn; m_kl += (ratio - 1.0f) - log_ratio;
            m_cf += fabsf(ratio - 1.0f) > g.ceps ? 1.0f : 0.0f;
            m_v += v; m_r += R; m_ve += ve; m_ve2 += ve * ve; m_vemax = fmaxf(m_vemax, ve);
            m_n += 1.0f;
        }
        // ---- head gradients: dWp[k][a] = sum_r hl[r][k] dl[r][a] (lane = k)
#pragma unroll
        for (int k = 0; k < H; k++) S.a[WaveStage<H>::at(lane, k)] = valid ? hl[k] : 0.0f;
        S.l[lane][0] = dl0; S.l[lane][1] = dl1; S.l[lane][2] = dv;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        #pragma unroll 2
        for (int rr = 0; rr < 64; rr++) {
            const float q0 = S.l[rr][0], q1 = S.l[rr][1], q2 = S.l[rr][2];
            gbp0 += q0; gbp1 += q1; gbv += q2;
            if (lane < H) {
                const float hv = S.a[WaveStage<H>::at(rr, lane)];
                gP0 = __builtin_fmaf(hv, q0, gP0);
                gP1 = __builtin_fmaf(hv, q1, gP1);
                gV = __builtin_fmaf(hv, q2, gV);
            }
        }
        // ---- dz of the last hidden layer
        float dz[H];
#pragma unroll
        for (int o = 0; o < H; o++) {
            float s = __builtin_fmaf(dl0, sP[O.wp + o * 2], 0.0f);
            s = __builtin_fmaf(dl1, sP[O.wp + o * 2 + 1], s);
            s = __builtin_fmaf(dv, sP[O.wv + o], s);
            // S.a still holds this lane's row of hl (0 for an absent row, whose s is 0)
            if constexpr (ACT == ACT_RELU) dz[o] = ((m2 >> o) & 1ull) ? s : 0.0f;
            else dz[o] = act_bwd<ACT>(s, S.a[WaveStage<H>::at(lane, o)]);
        }
        __builtin_amdgcn_wave_barrier();
        float dz1[H];
        if constexpr (NL == 2) {
            // dW1[k][o] = sum_r h1[r][k] dz2[r][o]   (lane = o)
#pragma unroll
            for (int k = 0; k < H; k++) { S.a[WaveStage<H>::at(lane, k)] = valid ? h1[k] : 0.0f; S.b[WaveStage<H>::at(lane, k)] = dz[k]; }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            if (lane < H) {
                #pragma unroll 2
                for (int rr = 0; rr < 64; rr++) {
                    const float dzo = S.b[WaveStage<H>::at(rr, lane)];
                    gb1 += dzo;
#pragma unroll
                    for (int k = 0; k < H; k++) gW1[k] = __builtin_fmaf(S.a[WaveStage<H>::at(rr, k)], dzo, gW1[k]);
                }
            }
            // dh1 = dz2 W1^T, dz1 = dh1 * act'(h1) (S.a holds h1 now)
            float prev = 0.0f;
#pragma unroll
            for (int k = 0; k < H; k++) {
                int kofs = O.w1 + k * H;
                asm volatile("" : "+v"(kofs) : "v"(prev));   // W1 row k fetched one step ahead
                const float *Wk = sP + kofs;
                float s = 0.0f;
#pragma unroll
                for (int o = 0; o < H; o++) s = __builtin_fmaf(dz[o], Wk[o], s);
                if constexpr (ACT == ACT_RELU) dz1[k] = ((m1 >> k) & 1ull) ? s : 0.0f;
                else dz1[k] = act_bwd<ACT>(s, S.a[WaveStage<H>::at(lane, k)]);
                prev = s;
            }
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int k = 0; k < H; k++) dz1[k] = dz[k];
        }
        // dW0[k][o] = sum_r x[r][k] dz1[r][o]   (lane = o)
#pragma unroll
        for (int k = 0; k < H; k++) S.b[WaveStage<H>::at(lane, k)] = dz1[k];
#pragma unroll
        for (int d = 0; d < 5; d++) S.x[lane][d] = x[d];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (lane < H) {
            #pragma unroll 2
            for (int rr = 0; rr < 64; rr++) {
                const float dzo = S.b[WaveStage<H>::at(rr, lane)];
                gb0 += dzo;
#pragma unroll
                for (int d = 0; d < 5; d++) gW0[d] = __builtin_fmaf(S.x[rr][d], dzo, gW0[d]);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    // ---- write this wave's partial gradient row
    float *row = g.slab + (size_t)gwave * (g.np + NUM_M);
    if (lane < H) {
#pragma unroll
        for (int d = 0; d < 5; d++) row[O.w0 + d * H + lane] = gW0[d];
        row[O.b0 + lane] = gb0;
        if constexpr (NL == 2) {
#pragma unroll
            for (int k = 0; k < H; k++) row[O.w1 + k * H + lane] = gW1[k];
            row[O.b1 + lane] = gb1;
        }
        row[O.wp + lane * 2] = gP0;
        row[O.wp + lane * 2 + 1] = gP1;
        row[O.wv + lane] = gV;
    }
    if (lane == 0) { row[O.bp] = gbp0; row[O.bp + 1] = gbp1; row[O.bv] = gbv; }
    const float s_pl = wave_sum(m_pl), s_vl = wave_sum(m_vl), s_h = wave_sum(m_h);
    const float s_kl = wave_sum(m_kl), s_cf = wave_sum(m_cf), s_v = wave_sum(m_v);
    const float s_r = wave_sum(m_r), s_ve = wave_sum(m_ve), s_ve2 = wave_sum(m_ve2);
    const float s_mx = wave_max(m_vemax), s_n = wave_sum(m_n);
    if (lane == 0) {
        float *mm = row + g.np;
        mm[M_PL] = s_pl; mm[M_VL] = s_vl; mm[M_H] = s_h; mm[M_KL] = s_kl; mm[M_CF] = s_cf;
        mm[M_V] = s_v; mm[M_R] = s_r; mm[M_VE] = s_ve; mm[M_VE2] = s_ve2; mm[M_VEMAX] = s_mx;
        mm[M_N] = s_n;
    }
}

// one minibatch row (ppo.rs:1833-1857 gather), loaded branch-free: an absent
// row (idx = ~0) reads row 0 and is zeroed by selects, so the record stays in
// registers (a branchy per-member fill lands it in scratch)
// a row as loaded one tile ahead: the raw values and whether the row exists.  The loads
// are unconditional (a missing row reads row 0) and the zeroing of a missing row waits
// for the consumer (row_used): selects right after the loads made the wave wait for the
// gather at once (s_waitcnt vmcnt(0) behind the prefetch), exposing its latency every tile
struct RowData {
    float x0, x1, x2, x3, x4;
    int a;
    float olp, A, R, ov;
    bool ok;
    __device__ __forceinline__ float x(int d) const { return d == 0 ? x0 : d == 1 ? x1 : d == 2 ? x2 : d == 3 ? x3 : x4; }
};
__device__ __forceinline__ RowData load_row(const MbArgs &g, uint32_t idx) {
    const bool ok = idx != 0xFFFFFFFFu;
    const size_t i = ok ? idx : 0;
    RowData d;
    d.ok = ok;
    if (g.rowA) {                     // one 32-byte sector [obs 0..3][obs 4, action, log-prob, value] + [adv, ret]
        const float4 a = g.rowA[i * 2], b = g.rowA[i * 2 + 1];
#ifdef BPPO_DIAG_NO_ROWB   // diagnostic build (wrong results): the gather without the second line
        const float2 c = make_float2(a.x * 0.5f, b.x * 0.25f);
#else
        const float2 c = g.rowB[i];
#endif
        d.x0 = a.x; d.x1 = a.y; d.x2 = a.z; d.x3 = a.w;
        d.x4 = b.x; d.a = __float_as_int(b.y); d.olp = b.z; d.ov = b.w;
        d.A = c.x; d.R = c.y;
        return d;
    }
    const float *o = g.obs + i * 5;
    d.x0 = o[0]; d.x1 = o[1]; d.x2 = o[2]; d.x3 = o[3]; d.x4 = o[4];
    d.a = g.act[i]; d.olp = g.logp[i]; d.A = g.adv[i]; d.R = g.ret[i];
    d.ov = g.clip_value ? g.val[i] : 0.0f;
    return d;
}
// the row as the kernel uses it: a missing row all zeros, the old value only with clip_value
__device__ __forceinline__ RowData row_used(const RowData &r, int clip_value) {
    RowData d;
    d.ok = r.ok;
    d.x0 = r.ok ? r.x0 : 0.0f; d.x1 = r.ok ? r.x1 : 0.0f; d.x2 = r.ok ? r.x2 : 0.0f;
    d.x3 = r.ok ? r.x3 : 0.0f; d.x4 = r.ok ? r.x4 : 0.0f;
    d.a = r.ok ? r.a : 0;
    d.olp = r.ok ? r.olp : 0.0f; d.A = r.ok ? r.A : 0.0f; d.R = r.ok ? r.R : 0.0f;
    d.ov = (r.ok && clip_value) ? r.ov : 0.0f;
    return d;
}

// the update's rows packed once per update: [obs 0..3][obs 4, action, log-prob, value]
// (rows A, 32 B) and [advantage, return] (rows B, 8 B), so the shuffled minibatch
// gather touches two sectors per row instead of six buffers (when the rollout and GAE
// did not write them already)
__global__ void __launch_bounds__(256) k_pack_rows(size_t B, const float *obs, const int32_t *act, const float *logp,
                                                   const float *adv, const float *ret, const float *val,
                                                   float4 *rowA, float2 *rowB) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < B; i += (size_t)gridDim.x * blockDim.x) {
        const float *o = obs + i * 5;
        rowA[i * 2] = make_float4(o[0], o[1], o[2], o[3]);
        rowA[i * 2 + 1] = make_float4(o[4], __int_as_float(act[i]), logp[i], val[i]);
        rowB[i] = make_float2(adv[i], ret[i]);
    }
}
bppo_status launch_pack_rows(bppo_ctx *c) {
    const size_t B = (size_t)c->T * c->N;
    hipLaunchKernelGGL(k_pack_rows, dim3(2048), dim3(256), 0, c->stream, B, c->d_obs, c->d_act, c->d_logp, c->d_adv,
                       c->u_ret, c->u_val, c->d_rowA, c->d_rowB);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// ================================================ MFMA minibatch (H=64, NL=2) ==
// The CfgB network (5 -> 64 -> 64 -> {2, 1}, relu) per wave tile of 32 rows on
// v_mfma_f32_32x32x2_f32:
//   forward   H1 = relu(X W0 + b0), H2 = relu(H1 W1 + b1): natural k order (the
//             MFMA is a k-ordered fma chain), so values equal the rollout's VALU
//             forward bit for bit and the first-minibatch ratio is exactly 1;
//             the heads run on the VALU, lane = row, in k order.
//   backward  dW1 += H1^T dZ2 takes both accumulators straight from the C/D
//             layout (rows in registers: a permuted but fixed row order inside
//             the gradient sum); dZ1 = (dZ2 W1^T) * [H1 > 0] on MFMA after one
//             LDS transpose of dZ2; dW0, biases and the head gradients on the VALU.
// 8 waves per block (2 per SIMD), one block per CU, persistent over the minibatch.
__global__ void __launch_bounds__(512, 2) k_minibatch_mfma(MbArgs g) {
    using namespace mmb;
    constexpr CpOffsets O = cp_offsets<64, 2>();
    extern __shared__ __attribute__((aligned(16))) float smem[];
    Params &S = *reinterpret_cast<Params *>(smem);
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    WaveB &B = reinterpret_cast<WaveB *>(smem + sizeof(Params) / 4)[wv];
    load_params(S, g.params);
    __syncthreads();
#ifdef BPPO_MB_STAMPS
    unsigned long long st_acc[MB_NSEG] = {}, st_prev;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
#endif

    const int c = lane & 31, h = lane >> 5;
    const int gwave = blockIdx.x * WAVES + wv, nwaves = gridDim.x * WAVES;
    const float mean = g.mb_stats[0], denom = g.mb_stats[1] + 1e-8f;
    float b0k[2], b1k[2], wpk0[2], wpk1[2], wvk[2];
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        const int k = c + 32 * ct;
        b0k[ct] = S.b0[k]; b1k[ct] = S.b1[k];
        wpk0[ct] = S.Wp[2 * k]; wpk1[ct] = S.Wp[2 * k + 1]; wvk[ct] = S.Wv[k];
    }
    f32x16_t dW1[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int q = 0; q < 16; q++) dW1[i][j][q] = 0.0f;
    float gW0[5][2], gb0[2] = {0, 0}, gb1[2] = {0, 0}, gP0[2] = {0, 0}, gP1[2] = {0, 0}, gV[2] = {0, 0};
#pragma unroll
    for (int d = 0; d < 5; d++) gW0[d][0] = gW0[d][1] = 0.0f;
    float gbp0 = 0, gbp1 = 0, gbv = 0;
    float m_pl = 0, m_vl = 0, m_h = 0, m_kl = 0, m_cf = 0, m_v = 0, m_r = 0, m_ve = 0, m_ve2 = 0;
    float m_vemax = -INFINITY, m_n = 0;

    // software pipeline of the gather (ppo.rs:1833-1857): the shuffled index two
    // tiles ahead, the row data one tile ahead, so the dependent loads of the next
    // tile run under this tile's MFMAs
    const uint32_t stride = (uint32_t)nwaves * TR;
    auto idx_of = [&](uint32_t b) -> uint32_t {
        const uint32_t rr = b + c;
        return (h == 0 && rr < g.n) ? g.perm[g.start + rr] : 0xFFFFFFFFu;
    };
    RowData nxt;
    uint32_t idx_next = idx_of((uint32_t)gwave * TR + stride);
    nxt = load_row(g, idx_of((uint32_t)gwave * TR));
    // the first tile's loads drained before the loop: loads still pending at the loop
    // header made the wait-count pass wait on EVERY tile's prefetch right after issuing it
    // (its counts for the prologue's registers applied to the loop's in-order counter)
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t base = (uint32_t)gwave * TR; base < g.n; base += stride) {
        const uint32_t r = base + c;
        const bool valid = h == 0 && r < g.n;
        const RowData cur = row_used(nxt, g.clip_value);
        // re-derive the lane coordinates from an opaque copy each iteration: every
        // LDS address below is then one base VGPR + an immediate offset, instead
        // of ~100 loop-invariant addresses hoisted out of the loop (and spilled)
        int ln_ = lane;
        asm volatile("" : "+v"(ln_));
        const int c = ln_ & 31, h = ln_ >> 5;
        const uint32_t idx_after = idx_of(base + 2 * stride);
        nxt = load_row(g, idx_next);
        idx_next = idx_after;
        const int a = cur.a;
        const float olp = cur.olp, A = cur.A, R = cur.R, ov = cur.ov;
        if (h == 0) {
#pragma unroll
            for (int d = 0; d < 5; d++) B.X[c * 5 + d] = cur.x(d);
        }
        wave_sync();
        MB_STAMP(0);
        __builtin_amdgcn_s_setprio(3);   // matrix segment (see layer 2)
        // ---- layer 1 (K = 5 padded to 6: the pad operand is 0)
        f32x16_t acc[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[ct][q] = 0.0f;
#pragma unroll
        for (int s = 0; s < 3; s++) {
            const float av = (s == 2 && h == 1) ? 0.0f : B.X[c * 5 + 2 * s + h];
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, S.W0[(2 * s + h) * H + c + 32 * ct], acc[ct], 0, 0, 0);
        }
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const float v = __fadd_rn(acc[ct][q], b0k[ct]);
                B.T1[cd_row(q, h) * RS + c + 32 * ct] = v > 0.0f ? v : 0.0f;
            }
        wave_sync();
        __builtin_amdgcn_s_setprio(0);
        MB_STAMP(1);
        // ---- layer 2 (K = 64)
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[ct][q] = 0.0f;
        // the two matrix segments (layer 2, dZ1/dW1) run at wave priority 3: when both
        // waves of a SIMD are ready, the one feeding the matrix pipe issues first
        // (A/B: launch minimum 0.553 -> 0.548 ms, mean -1 %; with layer 1 too, a further
        // -0.5 % / -0.7 %: profiles/r03_mb_setprio_ab.txt)
        __builtin_amdgcn_s_setprio(3);
#pragma unroll 8
        for (int s = 0; s < 32; s++) {
            const float av = B.T1[c * RS + 2 * s + h];
            const float bv0 = S.W1[(2 * s + h) * RS + c], bv1 = S.W1[(2 * s + h) * RS + c + 32];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv1, acc[1], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        MB_STAMP(2);
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const float v = __fadd_rn(acc[ct][q], b1k[ct]);
                B.T2[cd_row(q, h) * RS + c + 32 * ct] = v > 0.0f ? v : 0.0f;
            }
        wave_sync();
        MB_STAMP(3);
        // ---- heads + loss, lane = row c on both lane halves: half h runs the k-ordered
        // chain of logit h and both run the value chain (two chains per lane instead
        // of three; each chain is the same fma sequence as before, so bit-identical);
        // the row's exp pairs -- softmax terms, probabilities -- run one per half;
        // the rest of the loss, dl and the metrics on the low half
        {
            float lh = 0.0f, vv = 0.0f;
            const float *hr = B.T2 + c * RS;
            const float2 *pv = S.PV[h];
#pragma unroll 16
            for (int k = 0; k < H; k++) {
                const float hk = hr[k];
                const float2 w = pv[k];
                lh = __builtin_fmaf(hk, w.x, lh);
                vv = __builtin_fmaf(hk, w.y, vv);
            }
            const float lx = __shfl_xor(lh, 32, 64);
            const float l0 = h ? lx : lh, l1 = h ? lh : lx;
            MB_STAMP(9);
            const float lg0 = __fadd_rn(l0, S.bp[0]), lg1 = __fadd_rn(l1, S.bp[1]), v = __fadd_rn(vv, S.bv[0]);
            const float mx = lg0 > lg1 ? lg0 : lg1;
            const float eh = S.expf(__fsub_rn(h ? lg1 : lg0, mx));
            const float eo = __shfl_xor(eh, 32, 64);
            const float e0 = h ? eo : eh, e1 = h ? eh : eo;
            const float lse = S.logf(__fadd_rn(e0, e1));
            const float ls0 = __fsub_rn(__fsub_rn(lg0, mx), lse);
            const float ls1 = __fsub_rn(__fsub_rn(lg1, mx), lse);
            const float ph = S.expf(h ? ls1 : ls0);
            const float po = __shfl_xor(ph, 32, 64);
            const float p0 = h ? po : ph, p1 = h ? ph : po;
          if (h == 0) {
            const float An = __fdiv_rn(__fsub_rn(A, mean), denom);   // utils.rs:88
            const float Hn = -__fadd_rn(__fmul_rn(p0, ls0), __fmul_rn(p1, ls1));
            const float newlp = a == 1 ? ls1 : ls0;
            const float log_ratio = __fsub_rn(newlp, olp);
            const float ratio = S.expf(log_ratio);
            const float na = -An;
            const float pl1 = __fmul_rn(na, ratio);
            const float rc = ratio < g.lo ? g.lo : (ratio > g.hi ? g.hi : ratio);
            const float pl2 = __fmul_rn(na, rc);
            const bool rhs = pl1 < pl2;
            const float pl = rhs ? pl2 : pl1;
            float vl, dvl;
            if (g.clip_value) {
                const float dlt = __fsub_rn(v, ov);
                const float dc = dlt < -g.ceps ? -g.ceps : (dlt > g.ceps ? g.ceps : dlt);
                const float vc = __fadd_rn(ov, dc);
                const float q1 = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
                const float q2 = __fmul_rn(__fsub_rn(vc, R), __fsub_rn(vc, R));
                if (q1 < q2) { vl = q2; dvl = (dlt >= -g.ceps && dlt <= g.ceps) ? 2.0f * __fsub_rn(vc, R) : 0.0f; }
                else { vl = q1; dvl = 2.0f * __fsub_rn(v, R); }
            } else {
                vl = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
                dvl = 2.0f * __fsub_rn(v, R);
            }
            const float g_ratio = (!rhs || (ratio >= g.lo && ratio <= g.hi)) ? -An * g.inv_mb : 0.0f;
            const float g_lr = g_ratio * ratio;
            const float ec = g.ent_coef * g.inv_mb;
            float dl0 = g_lr * ((a == 0 ? 1.0f : 0.0f) - p0) + ec * p0 * (ls0 + Hn);
            float dl1 = g_lr * ((a == 1 ? 1.0f : 0.0f) - p1) + ec * p1 * (ls1 + Hn);
            float dv = g.value_coef * 0.5f * g.inv_mb * dvl;
            if (!valid) { dl0 = dl1 = dv = 0.0f; }
            else {
                const float ve = fabsf(__fsub_rn(v, R));
                m_pl += pl; m_vl += vl; m_h += Hn; m_kl += (ratio - 1.0f) - log_ratio;
                m_cf += fabsf(ratio - 1.0f) > g.ceps ? 1.0f : 0.0f;
                m_v += v; m_r += R; m_ve += ve; m_ve2 += ve * ve; m_vemax = fmaxf(m_vemax, ve);
                m_n += 1.0f;
            }
            gbp0 += dl0; gbp1 += dl1; gbv += dv;
            B.dl[c * 4 + 0] = dl0; B.dl[c * 4 + 1] = dl1; B.dl[c * 4 + 2] = dv; B.dl[c * 4 + 3] = 0.0f;
          }
        }
        wave_sync();
        MB_STAMP(10);
        MB_STAMP(4);
        // ---- head weight gradients dWp, dWv += H2^T [dl | dv] (lane = hidden unit)
#pragma unroll 4
        for (int q = 0; q < 16; q++) {
            const int row = cd_row(q, h);
            const float d0 = B.dl[row * 4], d1 = B.dl[row * 4 + 1], dvr = B.dl[row * 4 + 2];
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const float hv = B.T2[row * RS + c + 32 * ct];
                gP0[ct] = __builtin_fmaf(hv, d0, gP0[ct]);
                gP1[ct] = __builtin_fmaf(hv, d1, gP1[ct]);
                gV[ct] = __builtin_fmaf(hv, dvr, gV[ct]);
            }
        }
        // ---- dZ2 before the relu mask: [dl0 dl1 dv 0] [Wp0; Wp1; Wv; 0] per (row, k)
        // as two k-steps of the MFMA (the same k-ordered fma chain as the VALU
        // form d0*wp0 -> +d1*wp1 -> +dv*wv), already in the C/D layout
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[ct][q] = 0.0f;
        {
            const float a0 = B.dl[c * 4 + h], a1 = B.dl[c * 4 + 2 + h];
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, h ? wpk1[ct] : wpk0[ct], acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, h ? 0.0f : wvk[ct], acc[ct], 0, 0, 0);
            }
        }
        // dZ2 = that * [H2 > 0], over H2 in place (each lane rewrites only its own
        // C/D elements)
#pragma unroll
        for (int q = 0; q < 16; q++) {
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const int ad = cd_row(q, h) * RS + c + 32 * ct;
                const float dz = B.T2[ad] > 0.0f ? acc[ct][q] : 0.0f;
                gb1[ct] += dz;
                B.T2[ad] = dz;
            }
            if ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound the LDS read hoisting
        }
        wave_sync();
        MB_STAMP(5);
        // ---- dZ1 = dZ2 W1^T (32 k-steps) interleaved with dW1 += H1^T dZ2 (16
        // k-steps over row pairs): both operands of every MFMA come from LDS
#pragma unroll
        for (int jt = 0; jt < 2; jt++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[jt][q] = 0.0f;
        __builtin_amdgcn_s_setprio(3);
#pragma unroll 4
        for (int s2 = 0; s2 < 16; s2++) {
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int s = 2 * s2 + u;
                const float av = B.T2[c * RS + 2 * s + h];
                const float bw0 = S.W1[c * RS + 2 * s + h], bw1 = S.W1[(c + 32) * RS + 2 * s + h];
                acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bw0, acc[0], 0, 0, 0);
                acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bw1, acc[1], 0, 0, 0);
            }
            const int rr = (2 * s2 + h) * RS;
            const float a0 = B.T1[rr + c], a1 = B.T1[rr + c + 32];
            const float z0 = B.T2[rr + c], z1 = B.T2[rr + c + 32];
            dW1[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, z0, dW1[0][0], 0, 0, 0);
            dW1[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, z1, dW1[0][1], 0, 0, 0);
            dW1[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, z0, dW1[1][0], 0, 0, 0);
            dW1[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, z1, dW1[1][1], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        MB_STAMP(6);
        // dZ1 masked by relu'(H1); dW0 and db0 on the VALU (lane = hidden unit)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int row = cd_row(q, h);
            float xr[5];
#pragma unroll
            for (int d = 0; d < 5; d++) xr[d] = B.X[row * 5 + d];
#pragma unroll
            for (int jt = 0; jt < 2; jt++) {
                const float dzv = B.T1[row * RS + c + 32 * jt] > 0.0f ? acc[jt][q] : 0.0f;
                gb0[jt] += dzv;
#pragma unroll
                for (int d = 0; d < 5; d++) gW0[d][jt] = __builtin_fmaf(xr[d], dzv, gW0[d][jt]);
            }
            if ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);   // bound the LDS read hoisting
        }
        wave_sync();
        MB_STAMP(7);
    }
    // ---- this wave's partial gradient row (lane halves hold different rows: combine)
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        gb0[ct] += __shfl_xor(gb0[ct], 32, 64); gb1[ct] += __shfl_xor(gb1[ct], 32, 64);
        gP0[ct] += __shfl_xor(gP0[ct], 32, 64); gP1[ct] += __shfl_xor(gP1[ct], 32, 64);
        gV[ct] += __shfl_xor(gV[ct], 32, 64);
#pragma unroll
        for (int d = 0; d < 5; d++) gW0[d][ct] += __shfl_xor(gW0[d][ct], 32, 64);
    }
    // the block's 8 wave rows meet in LDS (all tiles done: the staging is free)
    // and are summed in wave order into one slab row per block
    const int W_ = g.np + NUM_M;
    __syncthreads();
    float *row = smem + (size_t)wv * W_;
    if (h == 0) {
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const int k = c + 32 * ct;
#pragma unroll
            for (int d = 0; d < 5; d++) row[O.w0 + d * H + k] = gW0[d][ct];
            row[O.b0 + k] = gb0[ct];
            row[O.b1 + k] = gb1[ct];
            row[O.wp + 2 * k] = gP0[ct];
            row[O.wp + 2 * k + 1] = gP1[ct];
            row[O.wv + k] = gV[ct];
        }
    }
    // dW1[k][o]: accumulator (it, jt) row k = (q&3) + 8(q>>2) + 4h + 32 it, col o = c + 32 jt
#pragma unroll
    for (int it = 0; it < 2; it++)
#pragma unroll
        for (int jt = 0; jt < 2; jt++)
#pragma unroll
            for (int q = 0; q < 16; q++)
                row[O.w1 + ((q & 3) + 8 * (q >> 2) + 4 * h + 32 * it) * H + c + 32 * jt] = dW1[it][jt][q];
    const float s_bp0 = wave_sum(gbp0), s_bp1 = wave_sum(gbp1), s_bv = wave_sum(gbv);
    const float s_pl = wave_sum(m_pl), s_vl = wave_sum(m_vl), s_h = wave_sum(m_h);
    const float s_kl = wave_sum(m_kl), s_cf = wave_sum(m_cf), s_v = wave_sum(m_v);
    const float s_r = wave_sum(m_r), s_ve = wave_sum(m_ve), s_ve2 = wave_sum(m_ve2);
    const float s_mx = wave_max(m_vemax), s_n = wave_sum(m_n);
    if (lane == 0) {
        row[O.bp] = s_bp0; row[O.bp + 1] = s_bp1; row[O.bv] = s_bv;
        float *mm = row + g.np;
        mm[M_PL] = s_pl; mm[M_VL] = s_vl; mm[M_H] = s_h; mm[M_KL] = s_kl; mm[M_CF] = s_cf;
        mm[M_V] = s_v; mm[M_R] = s_r; mm[M_VE] = s_ve; mm[M_VE2] = s_ve2; mm[M_VEMAX] = s_mx;
        mm[M_N] = s_n;
    }
    __syncthreads();
    for (int p = tid; p < W_; p += blockDim.x) {
        float acc = smem[p];
        if (p == g.np + M_VEMAX) {
            for (int w = 1; w < WAVES; w++) acc = fmaxf(acc, smem[(size_t)w * W_ + p]);
        } else {
            for (int w = 1; w < WAVES; w++) acc += smem[(size_t)w * W_ + p];
        }
        g.slab[(size_t)blockIdx.x * W_ + p] = acc;
    }
#ifdef BPPO_MB_STAMPS
    MB_STAMP(8);
    if (lane == 0)
        for (int k = 0; k < MB_NSEG; k++) g.stamps[(size_t)gwave * MB_NSEG + k] = st_acc[k];
#endif
}

// ============================================ split-bf16 minibatch (H=64, NL=2) ==
// Every minibatch but the update's first.  The first minibatch runs with the rollout's
// parameters, where the forward must reproduce the rollout's values bit for bit (ratio
// exactly 1: k_minibatch_mfma, k-ordered f32 MFMA chains).  After the first Adam step the
// parameters already differ from the reference's in the last bits (gradient summation
// order), so the later minibatches only need f32 ACCURACY, not the reference's rounding.
// Here the three 64x64 contractions -- layer 2, dZ1 = dZ2 W1^T, dW1 = H1^T dZ2 -- run on
// v_mfma_f32_32x32x16_bf16 (1/16 the cycles of the f32 MFMA per FLOP) with every f32
// operand split exactly into three bf16 pieces x = x0 + x1 + x2 (8 significand bits each)
// and the six products of order <= 2 accumulated in f32 (x0y0, x0y1, x1y0, x0y2, x1y1,
// x2y0).  |x1| <= 2^-8 |x| and |x2| <= 2^-16 |x|, so each dropped product (x1y2, x2y1,
// x2y2) is at most 2^-24 |xy|, together <= (2^-23 + 2^-32) |xy|; with the f32 additions a
// product is within 2^-22 of xy (tests/test_split_bf16.py), and the kernel's gradient is
// checked against the oracle from identical parameters (tests/test_gpu_split_kernel.py):
// 48 bf16 MFMAs of 32 cycles per contraction per 32-row tile instead of 64 f32 MFMAs of
// 64 cycles.
//   layer 1 twice on the f32 MFMA (K = 6, b0 folded into the pad row): transposed
//     (H1^T: units in registers, rows on lanes = layer 2's A fragments, no LDS) and in
//     the C/D orientation (rows in registers = dW1's A fragments and the relu mask);
//   heads on the VALU with ILP (lane = row, each lane half over 32 units);
//   W1 split once per block into ONE bf16 image [j1][j2] (r06; r05 kept a second,
//   transposed copy): dZ1's B fragments read its rows (ds_read_b128), layer 2's B fragments
//   -- k = j1 in the accumulator's permuted row order -- its columns through the
//   transposing ds_read_b64_tr_b16; 128-B rows with the 16-B chunks XOR-swizzled so both
//   reads are conflict-free (w1_at);
//   dZ2 split once (r06): its pieces go to a [j2][row] image (Z, over the H2 tile) that
//   dW1 reads back per lane (B fragments, k = rows) and dZ1 reads transposed (A fragments,
//   k = j2) -- r05 split the same values twice, once per layout.
namespace mmf {
constexpr int H = 64, TR = 32, WS = 68;
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
struct Params {
    uint64_t exp2tab[32];
    double linvc[16], llogc[16];
    float W0[6 * H];              // [d][j1]; row 5 = b0 (the K pad multiplies a 1)
    float b1[H];
    float4 Wh[H];                 // {wp0, wp1, wv, 0} per hidden unit
    float bp[2], bv[2];
    float2 PV[2][H];              // exact heads: {Wp[2k + h], Wv[k]} per lane half h (k_minibatch_mfma's pairs)
    __bf16 W1[3][H * H];          // W1 pieces [j1][j2], chunks swizzled (w1_at)
    __device__ __forceinline__ float expf(float x) const { return bppo_math::expf_glibc_tab(x, exp2tab); }
    __device__ __forceinline__ float logf(float x) const { return bppo_math::logf_glibc_tab(x, linvc, llogc); }
};
constexpr int MET_STRIDE = 20;
// EXACT_FWD (the update's first minibatch) keeps dZ2 in f32 in the tile and splits it per
// use (its f32 W1 copy for the exact layer 2 leaves no LDS for the piece image)
template <bool EXACT_FWD>
struct Wave {
    float X[TR * 5];
    union {
        float T[TR * WS];             // H2, then (EXACT_FWD) dZ2 [row][j2]
        __bf16 Z[EXACT_FWD ? 4 : 3 * H * TR];   // dZ2 pieces [j2][row], chunks swizzled (z_at)
    };
    float dl[TR * 4];
    // per row lane: the metric sums and head-bias gradients (MT_*); row stride 20 floats,
    // not 16: lanes c and c+4 of a b128 access then fall in different bank groups
    // (stride 16 put 4 lanes on the same banks: r04g counted 6.5M conflict cycles/launch)
    float met[TR * MET_STRIDE];
};
enum { MT_PL = 0, MT_VL, MT_H, MT_KL, MT_CF, MT_V, MT_R, MT_VE, MT_VE2, MT_VEMAX, MT_N, MT_BP0, MT_BP1, MT_BV };
constexpr int WAVES = 8;
constexpr size_t W1F_BYTES = H * H * sizeof(float);   // EXACT_FWD: W1 in f32 after Params
template <bool EXACT_FWD>
constexpr size_t lds_tiles() { return sizeof(Params) + (EXACT_FWD ? W1F_BYTES : 0) + WAVES * sizeof(Wave<EXACT_FWD>); }
static_assert(lds_tiles<false>() <= 160 * 1024 && lds_tiles<true>() <= 160 * 1024,
              "split minibatch kernel LDS over the gfx950 limit");
static_assert(sizeof(Params) % 16 == 0 && offsetof(Params, W1) % 16 == 0 && sizeof(Wave<false>) % 16 == 0 &&
              sizeof(Wave<true>) % 16 == 0, "LDS images 16-B aligned");
// W1 image: 16-B chunk k of row j1 stored at chunk k ^ w1_swz(j1), w1_swz a bijection of
// bits 1-3 of j1.  Row reads (dZ1, ds_read_b128: 16 lanes j1, one chunk) then land on
// (j1 & 1, chunk) pairs that differ within each lane group; the transposed reads (layer 2:
// rows j1 .. j1+3, j1 = 0 mod 4, 32 columns per lane half) put rows j1 and j1+2 in
// different 64-B halves of the bank space (bit 2 of the swizzle = bit 1 of j1)
__device__ __forceinline__ int w1_swz(int j1) { return (((j1 >> 1) & 1) << 2) | (((j1 >> 2) & 1) << 1) | ((j1 >> 3) & 1); }
__device__ __forceinline__ int w1_at(int j1, int j2) { return j1 * H + ((((j2 >> 3) ^ w1_swz(j1)) << 3) | (j2 & 7)); }
// Z image: [j2][row] rows of 64 B, 8-B chunk k (rows 4k .. 4k+3) stored at k ^ z_swz(j2):
// conflict-free for the ds_write_b64 stores (16 lanes j2, one chunk), the per-lane
// ds_read_b64 reads (32 lanes j2) and the transposed reads (4 rows j2 x 32 columns)
__device__ __forceinline__ int z_swz(int j2) { return ((j2 >> 2) & 7) ^ (((j2 >> 1) & 1) << 2); }
__device__ __forceinline__ int z_at(int j2, int row) { return j2 * TR + ((((row >> 2) ^ z_swz(j2)) << 2) | (row & 3)); }
// ds_read_b64_tr_b16: lane 4q + p of each 16-lane group addresses row q, columns 4p .. 4p+3
// of a 4 x 16 block; lane i receives column i, row q in element q
__device__ __forceinline__ s16x4_t lds_tr4(const __bf16 *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t *)p);
}
__device__ __forceinline__ bf16x8_t cat8(s16x4_t lo, s16x4_t hi) {
    return __builtin_bit_cast(bf16x8_t, (s16x8_t)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}
struct Split8 { bf16x8_t p[3]; };
// exact three-piece split of 8 f32 values, a pair at a time: one v_cvt_pk_bf16_f32 per
// piece pair, the pieces' f32 values taken back from the packed word (<< 16, & 0xffff0000)
// and the residuals as one packed subtract -- the per-element form converted every value
// twice (once alone for its residual, once paired for the operand) plus moves
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    uint32_t u = __builtin_bit_cast(uint32_t, bf16x2_t{(__bf16)a, (__bf16)b});
    asm("" : "+v"(u));      // opaque: the halves are read back from THIS word (no re-conversion)
    return u;
}
union Pieces8 { bf16x8_t v; uint32_t u[4]; };
__device__ __forceinline__ Split8 split8(const float (&x)[8]) {
#ifdef BPPO_SPLIT8_SCALAR       // A/B build: each element converted on its own (r04 form)
    Split8 t;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        t.p[0][j] = a; t.p[1][j] = b; t.p[2][j] = (__bf16)(r - (float)b);
    }
    return t;
#endif
    Pieces8 p0, p1, p2;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const float xa = x[2 * j], xb = x[2 * j + 1];
        const uint32_t A = pk_bf16(xa, xb);
        const float ra = xa - __uint_as_float(A << 16), rb = xb - __uint_as_float(A & 0xffff0000u);
        const uint32_t B = pk_bf16(ra, rb);
        const float sa = ra - __uint_as_float(B << 16), sb = rb - __uint_as_float(B & 0xffff0000u);
        p0.u[j] = A; p1.u[j] = B; p2.u[j] = pk_bf16(sa, sb);
    }
    Split8 s;
    s.p[0] = p0.v; s.p[1] = p1.v; s.p[2] = p2.v;
    return s;
}
// relu as a signed-integer max of the bits (a negative float is a negative int; -0 -> +0):
// one v_max_i32, where `v > 0 ? v : 0` is a v_max_f32 behind a canonicalising v_max_f32
// (IEEE mode).  Differs only for a NaN with a clear sign bit, which it passes on
// (split launches 0.481 -> 0.462 ms mean in the bench, profiles/r05d/r05z_ab_*.log)
__device__ __forceinline__ float relu_bits(float v) {
    const int b = __float_as_int(v);
    return __int_as_float(b > 0 ? b : 0);
}
__device__ __forceinline__ void mfma6(f32x16_t &acc, const Split8 &a, const Split8 &b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[2], b.p[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[1], b.p[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.p[0], b.p[0], acc, 0, 0, 0);
}
// dZ1's B fragment: W1[j1][j2 .. j2+7] (j2 = 0 mod 8), one ds_read_b128 per piece
__device__ __forceinline__ Split8 w1_row_pieces(const __bf16 (*W1)[H * H], int j1, int j2) {
    Split8 s;
    const int off = w1_at(j1, j2);
#pragma unroll
    for (int p = 0; p < 3; p++) s.p[p] = *reinterpret_cast<const bf16x8_t *>(W1[p] + off);
    return s;
}
// layer 2's B fragment: W1[j1 + 8e + q][j2] for e = 0, 1 and q = 0..3 (elements 4e + q),
// two transposed reads per piece; off[e] = the lane's offset of its block row (tr_off)
__device__ __forceinline__ Split8 w1_tr_pieces(const __bf16 (*W1)[H * H], int base, const int (&off)[2]) {
    Split8 s;
#pragma unroll
    for (int p = 0; p < 3; p++) s.p[p] = cat8(lds_tr4(W1[p] + base + off[0]), lds_tr4(W1[p] + base + off[1]));
    return s;
}
template <bool EXACT_FWD>
__device__ __forceinline__ void load_params_split(Params &S, float *W1f, const float *__restrict__ P) {
    constexpr CpOffsets O = cp_offsets<64, 2>();
    for (int i = threadIdx.x; i < 6 * H; i += blockDim.x) S.W0[i] = i < 5 * H ? P[O.w0 + i] : P[O.b0 + i - 5 * H];
    // W1 [in = j1][out = j2]: one 8-value chunk per thread, split and stored as three 16-B
    // pieces (r05: 2-B stores into two images, 1.37 M bank-conflict cycles per launch)
    for (int t = threadIdx.x; t < H * H / 8; t += blockDim.x) {
        const int j1 = t >> 3, j2 = (t & 7) * 8;
        float w[8];
#pragma unroll
        for (int j = 0; j < 8; j++) w[j] = P[O.w1 + 8 * t + j];
        const Split8 sp = split8(w);
        const int off = w1_at(j1, j2);
#pragma unroll
        for (int p = 0; p < 3; p++) *reinterpret_cast<bf16x8_t *>(S.W1[p] + off) = sp.p[p];
        if (EXACT_FWD) {
#pragma unroll
            for (int j = 0; j < 8; j++) W1f[8 * t + j] = w[j];
        }
    }
    for (int i = threadIdx.x; i < H; i += blockDim.x) {
        S.b1[i] = P[O.b1 + i];
        S.Wh[i] = make_float4(P[O.wp + 2 * i], P[O.wp + 2 * i + 1], P[O.wv + i], 0.0f);
        if (EXACT_FWD) {
            S.PV[0][i] = make_float2(P[O.wp + 2 * i], P[O.wv + i]);
            S.PV[1][i] = make_float2(P[O.wp + 2 * i + 1], P[O.wv + i]);
        }
    }
    if (threadIdx.x < 32) S.exp2tab[threadIdx.x] = bppo_math::kExp2fTab[threadIdx.x];
    if (threadIdx.x < 16) {
        S.linvc[threadIdx.x] = bppo_math::kLogfInvc[threadIdx.x];
        S.llogc[threadIdx.x] = bppo_math::kLogfLogc[threadIdx.x];
    }
    if (threadIdx.x < 2) S.bp[threadIdx.x] = P[O.bp + threadIdx.x];
    if (threadIdx.x == 0) S.bv[0] = P[O.bv];
}
}  // namespace mmf

// EXACT_FWD (r06): the update's first minibatch, which runs with the rollout's parameters, so
// the ratio must be exactly 1: the forward of k_minibatch_mfma -- layer 1 as below (the same
// k-ordered MFMA chain, b0 added as the K pad's 1 * b0, i.e. after the five products), layer 2
// as the f32 MFMA chain in natural k order from an [j1][row] LDS image of H1, both heads as
// k-ordered fma chains over all 64 units (lane half h: logit h, both: the value) -- and the
// backward of the split kernel (dW1 and dZ1 on the split-bf16 contraction): VERDICT r5 item 6
template <bool EXACT_FWD>
__global__ void __launch_bounds__(512, 2) k_minibatch_split(MbArgs g) {
    using namespace mmf;
    using mmb::cd_row;
    constexpr CpOffsets O = cp_offsets<64, 2>();
    extern __shared__ __attribute__((aligned(16))) float smem[];
    Params &S = *reinterpret_cast<Params *>(smem);
    float *W1f = smem + sizeof(Params) / 4;          // EXACT_FWD only
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    Wave<EXACT_FWD> &B = reinterpret_cast<Wave<EXACT_FWD> *>(smem + (sizeof(Params) + (EXACT_FWD ? W1F_BYTES : 0)) / 4)[wv];
    load_params_split<EXACT_FWD>(S, W1f, g.params);
    __syncthreads();
#ifdef BPPO_MB_STAMPS
    unsigned long long st_acc[MB_NSEG] = {}, st_prev;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_prev)::"memory");
#endif

    const int c = lane & 31, h = lane >> 5;
    const int gwave = blockIdx.x * WAVES + wv, nwaves = gridDim.x * WAVES;
    const float mean = g.mb_stats[0], denom = g.mb_stats[1] + 1e-8f;
    // transposed reads: lane 4q + p of its 16-lane group (column block gq = bit 4 of the lane)
    // layer 2: W1 rows 4h + 8e + q (+ 32 it + 16 s2), columns 32 ct + 16 gq + 4p
    int w1tr[2][2];
    {
        const int q = (lane >> 2) & 3, p = lane & 3, gq = (lane >> 4) & 1;
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int e = 0; e < 2; e++) w1tr[ct][e] = w1_at(4 * h + 8 * e + q, 32 * ct + 16 * gq + 4 * p);
    }
    f32x16_t dW1[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int q = 0; q < 16; q++) dW1[i][j][q] = 0.0f;
    float gW0[5][2], gb0[2] = {0, 0}, gb1[2] = {0, 0}, gP0[2] = {0, 0}, gP1[2] = {0, 0}, gV[2] = {0, 0};
#pragma unroll
    for (int d = 0; d < 5; d++) gW0[d][0] = gW0[d][1] = 0.0f;
    // the per-row metric sums live in LDS (lane c of the low half owns row slot c), not
    // in 14 loop-carried registers per lane
    if (h == 0) {
        float4 *mp = reinterpret_cast<float4 *>(B.met + c * MET_STRIDE);
        mp[0] = make_float4(0, 0, 0, 0); mp[1] = make_float4(0, 0, 0, 0);
        mp[2] = make_float4(0, -INFINITY, 0, 0); mp[3] = make_float4(0, 0, 0, 0);
    }

    const uint32_t stride = (uint32_t)nwaves * TR;
    auto idx_of = [&](uint32_t b) -> uint32_t {
        const uint32_t rr = b + c;
        return (h == 0 && rr < g.n) ? g.perm[g.start + rr] : 0xFFFFFFFFu;
    };
    RowData nxt;
    uint32_t idx_next = idx_of((uint32_t)gwave * TR + stride);
    nxt = load_row(g, idx_of((uint32_t)gwave * TR));
    // the first tile's loads drained before the loop: loads still pending at the loop
    // header made the wait-count pass wait on EVERY tile's prefetch right after issuing it
    // (its counts for the prologue's registers applied to the loop's in-order counter)
    __builtin_amdgcn_s_waitcnt(0);
    for (uint32_t base = (uint32_t)gwave * TR; base < g.n; base += stride) {
        const uint32_t r = base + c;
        const bool valid = h == 0 && r < g.n;
        const RowData cur = row_used(nxt, g.clip_value);
        int ln_ = lane;
        asm volatile("" : "+v"(ln_));
        const int c = ln_ & 31, h = ln_ >> 5;
        const uint32_t idx_after = idx_of(base + 2 * stride);
        nxt = load_row(g, idx_next);
        idx_next = idx_after;
        const int a = cur.a;
        const float olp = cur.olp, A = cur.A, R = cur.R, ov = cur.ov;
        if (h == 0) {
#pragma unroll
            for (int d = 0; d < 5; d++) B.X[c * 5 + d] = cur.x(d);
        }
        wave_sync();
        MB_STAMP(0);   // gather: row loads issued, this tile's X staged
        // ---- layer 1, transposed: H1^T[j1][row c] (j1 = cd_row(q, h) + 32 it)
        float xs[3];
#pragma unroll
        for (int s = 0; s < 3; s++) xs[s] = (s == 2 && h == 1) ? 1.0f : B.X[c * 5 + 2 * s + h];
        // ---- layer 2 (C/D orientation): A = H1 from the layer-1 registers (one 32-unit
        // tile of layer 1 at a time), B = W1 pieces
        f32x16_t h2[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) h2[ct][q] = 0.0f;
        // matrix segments at wave priority 3 (the other wave's VALU segments take the
        // leftover issue slots): launch mean 0.487 -> 0.466-0.476 ms, update -0.17 ms
        // (A/B, profiles/r04_windows/split_prio_ab.txt)
        __builtin_amdgcn_s_setprio(3);
#pragma unroll
        for (int it = 0; it < 2; it++) {
            f32x16_t a1;
#pragma unroll
            for (int q = 0; q < 16; q++) a1[q] = 0.0f;
#pragma unroll
            for (int s = 0; s < 3; s++)
                a1 = __builtin_amdgcn_mfma_f32_32x32x2f32(S.W0[(2 * s + h) * H + c + 32 * it], xs[s], a1, 0, 0, 0);
            if (EXACT_FWD) {
                // H1 as an [j1][row] image in the H2 tile: the C/D layout itself (row j1 =
                // cd_row(q, h) + 32 it, column = row c), consecutive lanes, consecutive banks
#pragma unroll
                for (int q = 0; q < 16; q++) B.T[(cd_row(q, h) + 32 * it) * TR + c] = relu_bits(a1[q]);
                continue;
            }
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                float v8[8];
#pragma unroll
                for (int j = 0; j < 8; j++) v8[j] = relu_bits(a1[8 * s2 + j]);
                const Split8 Af = split8(v8);
#pragma unroll
                for (int ct = 0; ct < 2; ct++)
                    mfma6(h2[ct], Af, w1_tr_pieces(S.W1, (32 * it + 16 * s2) * H, w1tr[ct]));
                __builtin_amdgcn_sched_barrier(0);   // bound the piece-load hoisting (registers)
            }
        }
        if (EXACT_FWD) {
            // layer 2 as k_minibatch_mfma: k = 2s + h per 32x32x2 step, natural order
            wave_sync();
#pragma unroll 4
            for (int s = 0; s < 32; s++) {
                const float av = B.T[(2 * s + h) * TR + c];
                const float bv0 = W1f[(2 * s + h) * H + c], bv1 = W1f[(2 * s + h) * H + c + 32];
                h2[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv0, h2[0], 0, 0, 0);
                h2[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv1, h2[1], 0, 0, 0);
            }
        }
        __builtin_amdgcn_s_setprio(0);
        MB_STAMP(1);   // layers 1 and 2
        // H2 = relu(. + b1) -> the row-major tile for the heads
        if (EXACT_FWD) wave_sync();          // every lane's last H1 read precedes the H2 stores
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const float v = h2[ct][q] + S.b1[c + 32 * ct];
                B.T[cd_row(q, h) * WS + c + 32 * ct] = relu_bits(v);
            }
        wave_sync();
        MB_STAMP(2);   // H2 epilogue
        // ---- heads: lane = row c, lane half h over units [32 h, 32 h + 32), 2 chains each
        // (EXACT_FWD: k_minibatch_mfma's k-ordered chains over all 64 units)
        float l0, l1, vv;
        if (EXACT_FWD) {
            float lh = 0.0f, vc = 0.0f;
            const float *hr = B.T + c * WS;
            const float2 *pv = S.PV[h];
#pragma unroll 2
            for (int k = 0; k < H; k += 4) {
                const float4 x = *reinterpret_cast<const float4 *>(hr + k);
                const float xs4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const float2 w = pv[k + u];
                    lh = __builtin_fmaf(xs4[u], w.x, lh);
                    vc = __builtin_fmaf(xs4[u], w.y, vc);
                }
            }
            const float lx = __shfl_xor(lh, 32, 64);
            l0 = h ? lx : lh; l1 = h ? lh : lx; vv = vc;
        } else {
            float pa[3] = {0, 0, 0}, pb[3] = {0, 0, 0};
            const float *hr = B.T + c * WS + 32 * h;
#pragma unroll
            for (int k = 0; k < 32; k += 4) {
                const float4 x = *reinterpret_cast<const float4 *>(hr + k);
                const float4 w0 = S.Wh[32 * h + k], w1 = S.Wh[32 * h + k + 1];
                const float4 w2 = S.Wh[32 * h + k + 2], w3 = S.Wh[32 * h + k + 3];
                pa[0] = __builtin_fmaf(x.x, w0.x, pa[0]); pa[1] = __builtin_fmaf(x.x, w0.y, pa[1]); pa[2] = __builtin_fmaf(x.x, w0.z, pa[2]);
                pb[0] = __builtin_fmaf(x.y, w1.x, pb[0]); pb[1] = __builtin_fmaf(x.y, w1.y, pb[1]); pb[2] = __builtin_fmaf(x.y, w1.z, pb[2]);
                pa[0] = __builtin_fmaf(x.z, w2.x, pa[0]); pa[1] = __builtin_fmaf(x.z, w2.y, pa[1]); pa[2] = __builtin_fmaf(x.z, w2.z, pa[2]);
                pb[0] = __builtin_fmaf(x.w, w3.x, pb[0]); pb[1] = __builtin_fmaf(x.w, w3.y, pb[1]); pb[2] = __builtin_fmaf(x.w, w3.z, pb[2]);
            }
            float t0 = pa[0] + pb[0], t1 = pa[1] + pb[1], t2 = pa[2] + pb[2];
            t0 += __shfl_xor(t0, 32, 64); t1 += __shfl_xor(t1, 32, 64); t2 += __shfl_xor(t2, 32, 64);
            l0 = t0; l1 = t1; vv = t2;
        }
        MB_STAMP(3);   // heads
        // ---- loss (as k_minibatch_mfma), dl per row
        {
            const float lg0 = __fadd_rn(l0, S.bp[0]), lg1 = __fadd_rn(l1, S.bp[1]), v = __fadd_rn(vv, S.bv[0]);
            const float mx = lg0 > lg1 ? lg0 : lg1;
            const float eh = S.expf(__fsub_rn(h ? lg1 : lg0, mx));
            const float eo = __shfl_xor(eh, 32, 64);
            const float e0 = h ? eo : eh, e1 = h ? eh : eo;
            const float lse = S.logf(__fadd_rn(e0, e1));
            const float ls0 = __fsub_rn(__fsub_rn(lg0, mx), lse);
            const float ls1 = __fsub_rn(__fsub_rn(lg1, mx), lse);
            const float ph = S.expf(h ? ls1 : ls0);
            const float po = __shfl_xor(ph, 32, 64);
            const float p0 = h ? po : ph, p1 = h ? ph : po;
          if (h == 0) {
            const float An = __fdiv_rn(__fsub_rn(A, mean), denom);   // utils.rs:88
            const float Hn = -__fadd_rn(__fmul_rn(p0, ls0), __fmul_rn(p1, ls1));
            const float newlp = a == 1 ? ls1 : ls0;
            const float log_ratio = __fsub_rn(newlp, olp);
            const float ratio = S.expf(log_ratio);
            const float na = -An;
            const float pl1 = __fmul_rn(na, ratio);
            const float rc = ratio < g.lo ? g.lo : (ratio > g.hi ? g.hi : ratio);
            const float pl2 = __fmul_rn(na, rc);
            const bool rhs = pl1 < pl2;
            const float pl = rhs ? pl2 : pl1;
            float vl, dvl;
            if (g.clip_value) {
                const float dlt = __fsub_rn(v, ov);
                const float dc = dlt < -g.ceps ? -g.ceps : (dlt > g.ceps ? g.ceps : dlt);
                const float vc = __fadd_rn(ov, dc);
                const float q1 = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
                const float q2 = __fmul_rn(__fsub_rn(vc, R), __fsub_rn(vc, R));
                if (q1 < q2) { vl = q2; dvl = (dlt >= -g.ceps && dlt <= g.ceps) ? 2.0f * __fsub_rn(vc, R) : 0.0f; }
                else { vl = q1; dvl = 2.0f * __fsub_rn(v, R); }
            } else {
                vl = __fmul_rn(__fsub_rn(v, R), __fsub_rn(v, R));
                dvl = 2.0f * __fsub_rn(v, R);
            }
            const float g_ratio = (!rhs || (ratio >= g.lo && ratio <= g.hi)) ? -An * g.inv_mb : 0.0f;
            const float g_lr = g_ratio * ratio;
            const float ec = g.ent_coef * g.inv_mb;
            float dl0 = g_lr * ((a == 0 ? 1.0f : 0.0f) - p0) + ec * p0 * (ls0 + Hn);
            float dl1 = g_lr * ((a == 1 ? 1.0f : 0.0f) - p1) + ec * p1 * (ls1 + Hn);
            float dv = g.value_coef * 0.5f * g.inv_mb * dvl;
            if (!valid) { dl0 = dl1 = dv = 0.0f; }
            else {
                const float ve = fabsf(__fsub_rn(v, R));
                float4 *mp = reinterpret_cast<float4 *>(B.met + c * MET_STRIDE);
                float4 m0 = mp[0], m1 = mp[1], m2 = mp[2], m3 = mp[3];
                m0.x += pl; m0.y += vl; m0.z += Hn; m0.w += (ratio - 1.0f) - log_ratio;
                m1.x += fabsf(ratio - 1.0f) > g.ceps ? 1.0f : 0.0f;
                m1.y += v; m1.z += R; m1.w += ve; m2.x += ve * ve; m2.y = fmaxf(m2.y, ve);
                m2.z += 1.0f; m2.w += dl0; m3.x += dl1; m3.y += dv;
                mp[0] = m0; mp[1] = m1; mp[2] = m2; mp[3] = m3;
            }
            *reinterpret_cast<float4 *>(B.dl + c * 4) = make_float4(dl0, dl1, dv, 0.0f);
          }
        }
        wave_sync();
        MB_STAMP(4);   // loss
        // ---- head weight gradients (lane = hidden unit), dZ2 before the mask on the f32 MFMA
#pragma unroll 4
        for (int q = 0; q < 16; q++) {
            const int row = cd_row(q, h);
            const float4 d = *reinterpret_cast<const float4 *>(B.dl + row * 4);
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const float hv = B.T[row * WS + c + 32 * ct];
                gP0[ct] = __builtin_fmaf(hv, d.x, gP0[ct]);
                gP1[ct] = __builtin_fmaf(hv, d.y, gP1[ct]);
                gV[ct] = __builtin_fmaf(hv, d.z, gV[ct]);
            }
        }
        f32x16_t acc[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) acc[ct][q] = 0.0f;
        {
            const float a0 = B.dl[c * 4 + h], a1 = B.dl[c * 4 + 2 + h];
#pragma unroll
            for (int ct = 0; ct < 2; ct++) {
                const float4 w = S.Wh[c + 32 * ct];
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, h ? w.y : w.x, acc[ct], 0, 0, 0);
                acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, h ? 0.0f : w.z, acc[ct], 0, 0, 0);
            }
        }
        // dZ2 = that * [H2 > 0]
        if (EXACT_FWD) {
            // written over H2 in f32, split per use below
#pragma unroll
            for (int q = 0; q < 16; q++) {
#pragma unroll
                for (int ct = 0; ct < 2; ct++) {
                    const int ad = cd_row(q, h) * WS + c + 32 * ct;
                    const float dz = B.T[ad] > 0.0f ? acc[ct][q] : 0.0f;
                    gb1[ct] += dz;
                    B.T[ad] = dz;
                }
                if ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);
            }
        } else {
#pragma unroll
            for (int q = 0; q < 16; q++)
#pragma unroll
                for (int ct = 0; ct < 2; ct++) {
                    acc[ct][q] = B.T[cd_row(q, h) * WS + c + 32 * ct] > 0.0f ? acc[ct][q] : 0.0f;
                    gb1[ct] += acc[ct][q];
                }
            wave_sync();    // every lane's H2 reads before the piece image overwrites the tile
            // split once: this lane's column j2 = c + 32 t, rows cd_row(8 s2 + j, h) -> the
            // [j2][row] image, 8 B (rows 16 s2 + 8e + 4h .. +3) per piece and half e
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    float z[8];
#pragma unroll
                    for (int j = 0; j < 8; j++) z[j] = acc[t][8 * s2 + j];
                    const Split8 P = split8(z);
#pragma unroll
                    for (int p = 0; p < 3; p++) {
                        const uint4 u = __builtin_bit_cast(uint4, P.p[p]);
                        *reinterpret_cast<uint2 *>(B.Z + p * H * TR + z_at(c + 32 * t, 16 * s2 + 4 * h)) = make_uint2(u.x, u.y);
                        *reinterpret_cast<uint2 *>(B.Z + p * H * TR + z_at(c + 32 * t, 16 * s2 + 8 + 4 * h)) = make_uint2(u.z, u.w);
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
        }
        MB_STAMP(5);   // head gradients, dZ2
        __builtin_amdgcn_s_setprio(3);
        // ---- layer 1 again, C/D orientation: H1[row][j1] (rows in registers)
        f32x16_t h1[2];
#pragma unroll
        for (int jt = 0; jt < 2; jt++)
#pragma unroll
            for (int q = 0; q < 16; q++) h1[jt][q] = 0.0f;
#pragma unroll
        for (int s = 0; s < 3; s++) {
            const float xv = (s == 2 && h == 1) ? 1.0f : B.X[c * 5 + 2 * s + h];
#pragma unroll
            for (int jt = 0; jt < 2; jt++)
                h1[jt] = __builtin_amdgcn_mfma_f32_32x32x2f32(xv, S.W0[(2 * s + h) * H + c + 32 * jt], h1[jt], 0, 0, 0);
        }
        uint32_t m1 = 0;                         // relu mask of H1, bit q + 16 jt
#pragma unroll
        for (int jt = 0; jt < 2; jt++)
#pragma unroll
            for (int q = 0; q < 16; q++) {
                h1[jt][q] = relu_bits(h1[jt][q]);
                const uint32_t hb = __float_as_uint(h1[jt][q]);
                m1 |= (hb < 1u ? hb : 1u) << (q + 16 * jt);
            }
        MB_STAMP(6);   // layer 1 again, relu mask
        // ---- dW1 += H1^T dZ2: both operands straight from the C/D registers (k = rows)
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++) {
            Split8 Bz[2];
#pragma unroll
            for (int t = 0; t < 2; t++) {
                if (EXACT_FWD) {
                    float z[8];      // this lane's own dZ2 elements, back from the tile
#pragma unroll
                    for (int j = 0; j < 8; j++) z[j] = B.T[cd_row(8 * s2 + j, h) * WS + c + 32 * t];
                    Bz[t] = split8(z);
                } else {
                    // this lane's own pieces, back from the image
#pragma unroll
                    for (int p = 0; p < 3; p++) {
                        const uint2 lo = *reinterpret_cast<const uint2 *>(B.Z + p * H * TR + z_at(c + 32 * t, 16 * s2 + 4 * h));
                        const uint2 hi = *reinterpret_cast<const uint2 *>(B.Z + p * H * TR + z_at(c + 32 * t, 16 * s2 + 8 + 4 * h));
                        Bz[t].p[p] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
                    }
                }
            }
#pragma unroll
            for (int it = 0; it < 2; it++) {
                float u[8];
#pragma unroll
                for (int j = 0; j < 8; j++) u[j] = h1[it][8 * s2 + j];
                const Split8 Ah = split8(u);
#pragma unroll
                for (int jt = 0; jt < 2; jt++) mfma6(dW1[it][jt], Ah, Bz[jt]);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        wave_sync();
        MB_STAMP(7);   // dW1
        // ---- dZ1 = dZ2 W1^T: A = dZ2 rows (natural k = j2) from the tile, B = W1 pieces
        f32x16_t dz1[2];
#pragma unroll
        for (int ct = 0; ct < 2; ct++)
#pragma unroll
            for (int q = 0; q < 16; q++) dz1[ct][q] = 0.0f;
#pragma unroll
        for (int ks = 0; ks < 4; ks++) {
            Split8 Az;
            if (EXACT_FWD) {
                const float *zr = B.T + c * WS + 16 * ks + 8 * h;
                const float4 z0 = *reinterpret_cast<const float4 *>(zr), z1 = *reinterpret_cast<const float4 *>(zr + 4);
                const float zz[8] = {z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w};
                Az = split8(zz);
            } else {
                // transposed: lane 4q + p of its group reads j2 = 16 ks + 8h + 4e + q, rows
                // 16 gq + 4p .. +3; lane c receives row c, element 4e + q
                const int q = (lane >> 2) & 3, pp = lane & 3, gq = (lane >> 4) & 1;
#pragma unroll
                for (int p = 0; p < 3; p++)
                    Az.p[p] = cat8(lds_tr4(B.Z + p * H * TR + z_at(16 * ks + 8 * h + q, 16 * gq + 4 * pp)),
                                   lds_tr4(B.Z + p * H * TR + z_at(16 * ks + 8 * h + 4 + q, 16 * gq + 4 * pp)));
            }
#pragma unroll
            for (int ct = 0; ct < 2; ct++)
                mfma6(dz1[ct], Az, w1_row_pieces(S.W1, c + 32 * ct, 16 * ks + 8 * h));
            __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_setprio(0);
        MB_STAMP(8);   // dZ1
        // dZ1 masked by relu'(H1); dW0 and db0 on the VALU (lane = hidden unit)
#pragma unroll
        for (int q = 0; q < 16; q++) {
            const int row = cd_row(q, h);
            float xr[5];
#pragma unroll
            for (int d = 0; d < 5; d++) xr[d] = B.X[row * 5 + d];
#pragma unroll
            for (int jt = 0; jt < 2; jt++) {
                // bit q + 16 jt of m1 sign-extended to a 0 / all-ones mask
                const int mk = (int)(m1 << (31 - (q + 16 * jt))) >> 31;
                const float dzv = __int_as_float(__float_as_int(dz1[jt][q]) & mk);
                gb0[jt] += dzv;
#pragma unroll
                for (int d = 0; d < 5; d++) gW0[d][jt] = __builtin_fmaf(xr[d], dzv, gW0[d][jt]);
            }
            if ((q & 3) == 3) __builtin_amdgcn_sched_barrier(0);
        }
        wave_sync();
        MB_STAMP(9);   // dW0
    }
    // ---- this wave's partial gradient row (as k_minibatch_mfma)
#pragma unroll
    for (int ct = 0; ct < 2; ct++) {
        gb0[ct] += __shfl_xor(gb0[ct], 32, 64); gb1[ct] += __shfl_xor(gb1[ct], 32, 64);
        gP0[ct] += __shfl_xor(gP0[ct], 32, 64); gP1[ct] += __shfl_xor(gP1[ct], 32, 64);
        gV[ct] += __shfl_xor(gV[ct], 32, 64);
#pragma unroll
        for (int d = 0; d < 5; d++) gW0[d][ct] += __shfl_xor(gW0[d][ct], 32, 64);
    }
    float mt[14];
#pragma unroll
    for (int k = 0; k < 14; k++) mt[k] = h == 0 ? B.met[c * MET_STRIDE + k] : (k == MT_VEMAX ? -INFINITY : 0.0f);
    const int W_ = g.np + NUM_M;
    __syncthreads();
    float *row = smem + (size_t)wv * W_;
    if (h == 0) {
#pragma unroll
        for (int ct = 0; ct < 2; ct++) {
            const int k = c + 32 * ct;
#pragma unroll
            for (int d = 0; d < 5; d++) row[O.w0 + d * H + k] = gW0[d][ct];
            row[O.b0 + k] = gb0[ct];
            row[O.b1 + k] = gb1[ct];
            row[O.wp + 2 * k] = gP0[ct];
            row[O.wp + 2 * k + 1] = gP1[ct];
            row[O.wv + k] = gV[ct];
        }
    }
#pragma unroll
    for (int it = 0; it < 2; it++)
#pragma unroll
        for (int jt = 0; jt < 2; jt++)
#pragma unroll
            for (int q = 0; q < 16; q++)
                row[O.w1 + ((q & 3) + 8 * (q >> 2) + 4 * h + 32 * it) * H + c + 32 * jt] = dW1[it][jt][q];
    float st[14];
#pragma unroll
    for (int k = 0; k < 14; k++) st[k] = k == MT_VEMAX ? wave_max(mt[k]) : wave_sum(mt[k]);
    if (lane == 0) {
        row[O.bp] = st[MT_BP0]; row[O.bp + 1] = st[MT_BP1]; row[O.bv] = st[MT_BV];
        float *mm = row + g.np;
        static_assert(MT_PL == M_PL && MT_VEMAX == M_VEMAX && MT_N == M_N, "metric slots");
#pragma unroll
        for (int k = 0; k <= MT_N; k++) mm[k] = st[k];
    }
    __syncthreads();
    for (int p = tid; p < W_; p += blockDim.x) {
        float a2 = smem[p];
        if (p == g.np + M_VEMAX) {
            for (int w = 1; w < WAVES; w++) a2 = fmaxf(a2, smem[(size_t)w * W_ + p]);
        } else {
            for (int w = 1; w < WAVES; w++) a2 += smem[(size_t)w * W_ + p];
        }
        g.slab[(size_t)blockIdx.x * W_ + p] = a2;
    }
#ifdef BPPO_MB_STAMPS
    MB_STAMP(10);  // the block's gradient row
    if (lane == 0)
        for (int k = 0; k < MB_NSEG; k++) g.stamps[(size_t)gwave * MB_NSEG + k] = st_acc[k];
#endif
}

// fixed-order reduction of the wave partials, grad[p] = sum_w slab[w][p]: SLAB_GROUPS
// row groups each summed in f64 in row order, then the groups in order.
// both passes in one launch, same association (bit-identical grad): a block owns 16
// columns and all 32 row groups, thread (column tid % 16, group tid / 16), the group sums
// through LDS, then 16 threads add the groups in order.  ~300 blocks for the CfgB width
// (r02-r04: 64 columns per block, 75 blocks of 16 waves each looping over two groups --
// 35 us mean per minibatch in the loop)
constexpr int SLAB1_COLS = 16;
__global__ void __launch_bounds__(SLAB1_COLS * SLAB_GROUPS) k_slab_reduce1(const float *__restrict__ slab, int rows,
                                                                           int width, float *__restrict__ grad,
                                                                           float *__restrict__ vemax_local) {
    __shared__ double part[SLAB_GROUPS][SLAB1_COLS];
    const int c = threadIdx.x % SLAB1_COLS, g = threadIdx.x / SLAB1_COLS;
    const int p = blockIdx.x * SLAB1_COLS + c;
    const bool live = p < width, is_max = p == width - NUM_M + M_VEMAX;
    const int per = (rows + SLAB_GROUPS - 1) / SLAB_GROUPS;
    if (live) {
        const int w0 = g * per, w1 = min(rows, w0 + per);
        double s = is_max ? -INFINITY : 0.0;
#pragma unroll 8
        for (int w = w0; w < w1; w++) {
            const double v = slab[(size_t)w * width + p];
            s = is_max ? fmax(s, v) : s + v;
        }
        part[g][c] = s;
    }
    __syncthreads();
    if (g == 0 && live) {
        double s = is_max ? -INFINITY : 0.0;
        for (int q = 0; q < SLAB_GROUPS; q++) s = is_max ? fmax(s, part[q][c]) : s + part[q][c];
        grad[p] = (float)s;
        if (is_max) *vemax_local = (float)s;     // kept out of the W > 1 SUM all-reduce
    }
}

// per-tensor norm clip + Adam (burn-optim 0.20 restated).  Each tensor is cut
// into ADAM_CHUNK-element blocks: pass 1 writes every block's sum of squares,
// pass 2 sums its tensor's partials in block order (deterministic) and updates.
__device__ __forceinline__ int adam_tensor_of(const AdamArgs &a, int b) {
    int t = 0;
    while (t + 1 < a.nt && a.blk0[t + 1] <= b) t++;
    return t;
}
__global__ void __launch_bounds__(256) k_adam_norm(AdamArgs a) {
    __shared__ double red[256];
    const int ti = adam_tensor_of(a, blockIdx.x);
    const AdamTensor T = a.t[ti];
    const int i0 = (blockIdx.x - a.blk0[ti]) * ADAM_CHUNK, i1 = min(T.len, i0 + ADAM_CHUNK);
    double ss = 0.0;
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        const float gi = a.grad[T.off + i] * a.inv_world;
        ss += (double)gi * (double)gi;
    }
    red[threadIdx.x] = ss;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) a.part[blockIdx.x] = red[0];
}
// adam_sqrt_note: the square root is sqrtf (correctly rounded under -fno-fast-math), not
// __fsqrt_rn: on this toolchain __fsqrt_rn lowers to the 1-ulp hardware approximation
// and differs from the host's sqrtf in ~15% of operands (scripts/probes/
// fp_rounding_probe.hip, profiles/r05b/fp_rounding_probe.txt) — one ulp in an update
// that the chaotic CNN trajectory then amplifies past 1e-5 within a few minibatches
__global__ void __launch_bounds__(256) k_adam(AdamArgs a) {
    __shared__ double tot;
    const int ti = adam_tensor_of(a, blockIdx.x);
    const AdamTensor T = a.t[ti];
    if (threadIdx.x == 0) {
        double s = 0.0;
        for (int b = a.blk0[ti]; b < a.blk0[ti + 1]; b++) s += a.part[b];
        tot = s;
    }
    __syncthreads();
    const int i0 = (blockIdx.x - a.blk0[ti]) * ADAM_CHUNK, i1 = min(T.len, i0 + ADAM_CHUNK);
    const float norm = (float)sqrt(tot);
    const float scale = norm > a.max_norm ? __fdiv_rn(a.max_norm, norm) : 1.0f;
    const bool clip = norm > a.max_norm;
    const float b1 = 0.9f, b2 = 0.999f, f1 = 1.0f - 0.9f, f2 = 1.0f - 0.999f;
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        float gi = a.grad[T.off + i] * a.inv_world;
        if (clip) gi = __fmul_rn(gi, scale);
        const float m1 = __fadd_rn(__fmul_rn(a.m1[T.off + i], b1), __fmul_rn(gi, f1));
        const float m2 = __fadd_rn(__fmul_rn(a.m2[T.off + i], b2), __fmul_rn(__fmul_rn(gi, gi), f2));
        a.m1[T.off + i] = m1;
        a.m2[T.off + i] = m2;
        const float m1c = __fdiv_rn(m1, T.c1), m2c = __fdiv_rn(m2, T.c2);
        const float upd = __fdiv_rn(m1c, __fadd_rn(sqrtf(m2c), a.eps));   // sqrtf: see adam_sqrt_note
        a.params[T.off + i] = __fsub_rn(a.params[T.off + i], __fmul_rn(upd, a.lr));
    }
}

// every tensor within one ADAM_CHUNK (the CfgB net): one block per tensor does
// pass 1 (the same per-thread sums and tree as k_adam_norm) and pass 2 (the
// update) back to back; block 0 also copies the minibatch's metric row.  The norm
// uses the first 256 threads exactly as k_adam_norm does (bit-identical); the
// elementwise update spreads over all ADAM1_THREADS (4 elements per thread for a
// 64x64 weight instead of 16 in a serial chain)
constexpr int ADAM1_THREADS = 1024;
__global__ void __launch_bounds__(ADAM1_THREADS) k_adam1(AdamArgs a, const float *gtail, const float *mb_stats,
                                                         int nm, float *metric_dst) {
    __shared__ double red[256];
    const AdamTensor T = a.t[blockIdx.x];
    if (threadIdx.x < 256) {
        double ss = 0.0;
#pragma unroll 4
        for (int i = threadIdx.x; i < T.len; i += 256) {
            const float gi = a.grad[T.off + i] * a.inv_world;
            ss += (double)gi * (double)gi;
        }
        red[threadIdx.x] = ss;
    }
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    const double tot = red[0];
    const float norm = (float)sqrt(tot);
    const float scale = norm > a.max_norm ? __fdiv_rn(a.max_norm, norm) : 1.0f;
    const bool clip = norm > a.max_norm;
    const float b1 = 0.9f, b2 = 0.999f, f1 = 1.0f - 0.9f, f2 = 1.0f - 0.999f;
#pragma unroll 2
    for (int i = threadIdx.x; i < T.len; i += ADAM1_THREADS) {
        float gi = a.grad[T.off + i] * a.inv_world;
        if (clip) gi = __fmul_rn(gi, scale);
        const float m1 = __fadd_rn(__fmul_rn(a.m1[T.off + i], b1), __fmul_rn(gi, f1));
        const float m2 = __fadd_rn(__fmul_rn(a.m2[T.off + i], b2), __fmul_rn(__fmul_rn(gi, gi), f2));
        a.m1[T.off + i] = m1;
        a.m2[T.off + i] = m2;
        const float m1c = __fdiv_rn(m1, T.c1), m2c = __fdiv_rn(m2, T.c2);
        const float upd = __fdiv_rn(m1c, __fadd_rn(sqrtf(m2c), a.eps));   // sqrtf: see adam_sqrt_note
        a.params[T.off + i] = __fsub_rn(a.params[T.off + i], __fmul_rn(upd, a.lr));
    }
    if (blockIdx.x == 0 && metric_dst) {
        const int i = threadIdx.x;
        if (i < nm) metric_dst[i] = gtail[i == GRAD_VEMAX ? GRAD_VEMAX_LOCAL : i];
        else if (i < nm + 4) metric_dst[i] = mb_stats[i - nm];
    }
}

// explained variance partial sums (ppo.rs:1268-1294)
__global__ void __launch_bounds__(256) k_ev(size_t n, const float *val, const float *ret, const float *valid,
                                             double *part) {
    __shared__ double sh[4][256];
    double s[4] = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (valid && !(valid[i] > 0.5f)) continue;      // opponent pool: learner rows only (ppo.rs:2047-2056)
        const double R = ret[i], res = (double)(ret[i] - val[i]);
        s[0] += R; s[1] += R * R; s[2] += res; s[3] += res * res;
    }
    for (int k = 0; k < 4; k++) sh[k][threadIdx.x] = s[k];
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st)
            for (int k = 0; k < 4; k++) sh[k][threadIdx.x] += sh[k][threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int k = 0; k < 4; k++) part[blockIdx.x * 4 + k] = sh[k][0];
}

// ------------------------------------------------------------- launchers ---
// advantage stats of every minibatch of one epoch in one pass (ppo.rs:1905-1913,
// utils.rs:80-89): f64 sum and sum of squares, min, max over each minibatch's
// shuffled rows.  Block b owns positions [b C, (b + 1) C) (EpochSplit in
// bppo_internal.h); the final pass adds the block partials of each minibatch in
// block order (deterministic).  On the ranged shuffle path the partials come
// from the fused Fisher-Yates final pass (k_shuffle.hip k_fy_final_ranged).
// 1024 threads per block, ADV_U positions per thread in flight (perm then adv are
// two dependent random-ish loads; one pair at a time left the block latency bound)
constexpr int ADV_THREADS = 1024, ADV_U = 4;
__global__ void __launch_bounds__(ADV_THREADS) k_adv_epoch(const float *__restrict__ adv,
                                                           const uint32_t *__restrict__ perm, EpochSplit sp,
                                                           uint32_t C, double *part) {
    __shared__ double red[ADV_THREADS / 64][2][4];
    const uint32_t i0 = blockIdx.x * C, i1 = min(sp.B, i0 + C);
    const uint32_t m0 = mb_of(i0, sp);
    double s[2] = {0.0, 0.0}, q[2] = {0.0, 0.0};
    float mn[2] = {INFINITY, INFINITY}, mx[2] = {-INFINITY, -INFINITY};
    for (uint32_t b = i0 + threadIdx.x; b < i1; b += ADV_THREADS * ADV_U) {
        uint32_t pi[ADV_U];
        float a[ADV_U];
#pragma unroll
        for (int k = 0; k < ADV_U; k++) pi[k] = perm[min(b + k * ADV_THREADS, i1 - 1)];
#pragma unroll
        for (int k = 0; k < ADV_U; k++) a[k] = adv[pi[k]];
#pragma unroll
        for (int k = 0; k < ADV_U; k++) {
            const uint32_t i = b + k * ADV_THREADS;
            if (i >= i1) continue;
            const double d = (double)a[k];
            if (mb_of(i, sp) != m0) { s[1] += d; q[1] += d * d; mn[1] = fminf(mn[1], a[k]); mx[1] = fmaxf(mx[1], a[k]); }
            else { s[0] += d; q[0] += d * d; mn[0] = fminf(mn[0], a[k]); mx[0] = fmaxf(mx[0], a[k]); }
        }
    }
    // wave reduction, then the block's waves in order (deterministic)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < 2; k++) {
        double x = s[k], y = q[k];
        float u = mn[k], v = mx[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64);
            u = fminf(u, __shfl_xor(u, o, 64)); v = fmaxf(v, __shfl_xor(v, o, 64));
        }
        if (lane == 0) { red[w][k][0] = x; red[w][k][1] = y; red[w][k][2] = u; red[w][k][3] = v; }
    }
    __syncthreads();
    if (threadIdx.x < 2) {
        const int k = threadIdx.x;
        double x = 0.0, y = 0.0, u = INFINITY, v = -INFINITY;
        for (int ww = 0; ww < ADV_THREADS / 64; ww++) {
            x += red[ww][k][0]; y += red[ww][k][1]; u = fmin(u, red[ww][k][2]); v = fmax(v, red[ww][k][3]);
        }
        double *o = part + ((size_t)blockIdx.x * 2 + k) * 4;
        o[0] = x; o[1] = y; o[2] = u; o[3] = v;
    }
}
// one block per minibatch: its rows' partials in block order -> [mean, std, min, max]
__global__ void __launch_bounds__(256) k_adv_epoch_final(const double *part, int nblk, uint32_t C, EpochSplit sp,
                                                         float *stats) {
    __shared__ double ss[256], sq[256], smn[256], smx[256];
    const uint32_t m = blockIdx.x;
    double s = 0.0, q = 0.0, mn = INFINITY, mx = -INFINITY;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
        const uint32_t m0 = mb_of((uint32_t)b * C, sp);
        if (m != m0 && m != m0 + 1) continue;
        const double *o = part + ((size_t)b * 2 + (m != m0)) * 4;
        s += o[0]; q += o[1]; mn = fmin(mn, o[2]); mx = fmax(mx, o[3]);
    }
    ss[threadIdx.x] = s; sq[threadIdx.x] = q; smn[threadIdx.x] = mn; smx[threadIdx.x] = mx;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            ss[threadIdx.x] += ss[threadIdx.x + st]; sq[threadIdx.x] += sq[threadIdx.x + st];
            smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + st]);
            smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const double n = (double)(sp.base + (m < sp.rem ? 1u : 0u));
    const double mean = ss[0] / n;
    stats[m * 4 + 0] = (float)mean;
    stats[m * 4 + 1] = n > 1.0 ? sqrtf((float)(fmax(sq[0] - ss[0] * mean, 0.0) / (n - 1.0))) : NAN;
    stats[m * 4 + 2] = (float)smn[0];
    stats[m * 4 + 3] = (float)smx[0];
}

// The same statistics from the inverse permutation (inv[r] = shuffled position of
// row r, written by the Fisher-Yates final pass on the side stream): rows stream
// in order, adv[r] and inv[r] coalesced, each added to the bins of its minibatch
// mb_of(inv[r]) (MB >= M bins in registers).  Block b owns rows [b C, (b+1) C);
// every block writes MB partials, summed per minibatch in block order.
template <int MB>
__global__ void __launch_bounds__(256) k_adv_stream(const float *__restrict__ adv, const uint32_t *__restrict__ inv,
                                                    EpochSplit sp, uint32_t C, double *part) {
    constexpr int U = 16;   // rows per thread per load round (a thread still adds its rows in order)
    __shared__ double red[4][MB][4];
    double s[MB], q[MB];
    float mn[MB], mx[MB];
#pragma unroll
    for (int k = 0; k < MB; k++) { s[k] = 0.0; q[k] = 0.0; mn[k] = INFINITY; mx[k] = -INFINITY; }
    const uint32_t r0 = blockIdx.x * C, r1 = min(sp.B, r0 + C);
    for (uint32_t b = r0 + threadIdx.x; b < r1; b += 256 * U) {
        float a[U];
        uint32_t p[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const uint32_t r = min(b + u * 256, r1 - 1);
            a[u] = adv[r];
            p[u] = inv[r];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (b + u * 256 >= r1) continue;
            const uint32_t m = mb_of(p[u], sp);
            const double d = (double)a[u];
#pragma unroll
            for (int k = 0; k < MB; k++) {
                const bool hit = m == (uint32_t)k;
                s[k] += hit ? d : 0.0;
                q[k] += hit ? d * d : 0.0;
                mn[k] = hit ? fminf(mn[k], a[u]) : mn[k];
                mx[k] = hit ? fmaxf(mx[k], a[u]) : mx[k];
            }
        }
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < MB; k++) {
        double x = s[k], y = q[k];
        float u = mn[k], v = mx[k];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            x += __shfl_xor(x, o, 64); y += __shfl_xor(y, o, 64);
            u = fminf(u, __shfl_xor(u, o, 64)); v = fmaxf(v, __shfl_xor(v, o, 64));
        }
        if (lane == 0) { red[w][k][0] = x; red[w][k][1] = y; red[w][k][2] = u; red[w][k][3] = v; }
    }
    __syncthreads();
    if (threadIdx.x < MB) {
        const int k = threadIdx.x;
        double x = 0.0, y = 0.0, u = INFINITY, v = -INFINITY;
        for (int ww = 0; ww < 4; ww++) {
            x += red[ww][k][0]; y += red[ww][k][1]; u = fmin(u, red[ww][k][2]); v = fmax(v, red[ww][k][3]);
        }
        double *o = part + ((size_t)blockIdx.x * MB + k) * 4;
        o[0] = x; o[1] = y; o[2] = u; o[3] = v;
    }
}
// one block per minibatch: the block partials in block order -> [mean, std, min, max]
__global__ void __launch_bounds__(256) k_adv_stream_final(const double *part, int nblk, int MB, EpochSplit sp,
                                                          float *stats) {
    __shared__ double ss[256], sq[256], smn[256], smx[256];
    const uint32_t m = blockIdx.x;
    double s = 0.0, q = 0.0, mn = INFINITY, mx = -INFINITY;
    for (int b = threadIdx.x; b < nblk; b += blockDim.x) {
        const double *o = part + ((size_t)b * MB + m) * 4;
        s += o[0]; q += o[1]; mn = fmin(mn, o[2]); mx = fmax(mx, o[3]);
    }
    ss[threadIdx.x] = s; sq[threadIdx.x] = q; smn[threadIdx.x] = mn; smx[threadIdx.x] = mx;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            ss[threadIdx.x] += ss[threadIdx.x + st]; sq[threadIdx.x] += sq[threadIdx.x + st];
            smn[threadIdx.x] = fmin(smn[threadIdx.x], smn[threadIdx.x + st]);
            smx[threadIdx.x] = fmax(smx[threadIdx.x], smx[threadIdx.x + st]);
        }
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const double n = (double)(sp.base + (m < sp.rem ? 1u : 0u));
    const double mean = ss[0] / n;
    stats[m * 4 + 0] = (float)mean;
    stats[m * 4 + 1] = n > 1.0 ? sqrtf((float)(fmax(sq[0] - ss[0] * mean, 0.0) / (n - 1.0))) : NAN;
    stats[m * 4 + 2] = (float)smn[0];
    stats[m * 4 + 3] = (float)smx[0];
}

bppo_status launch_epoch_adv_stats(bppo_ctx *c, uint32_t B, int M, const uint32_t *inv) {
    const EpochSplit sp{B, B / (uint32_t)M, B % (uint32_t)M, (uint32_t)M};
    if (inv && M <= ADV_STREAM_MAXM && sp.base > 0) {
        const uint32_t C = (B + ADV_STREAM_BLOCKS - 1) / ADV_STREAM_BLOCKS;
        const int nblk = (int)((B + C - 1) / C);
        const int MB = M <= 4 ? 4 : (M <= 8 ? 8 : 16);
        if (MB == 4) hipLaunchKernelGGL(k_adv_stream<4>, dim3(nblk), dim3(256), 0, c->stream, c->d_adv, inv, sp, C, c->d_advpart);
        else if (MB == 8) hipLaunchKernelGGL(k_adv_stream<8>, dim3(nblk), dim3(256), 0, c->stream, c->d_adv, inv, sp, C, c->d_advpart);
        else hipLaunchKernelGGL(k_adv_stream<16>, dim3(nblk), dim3(256), 0, c->stream, c->d_adv, inv, sp, C, c->d_advpart);
        hipLaunchKernelGGL(k_adv_stream_final, dim3(M), dim3(256), 0, c->stream, c->d_advpart, nblk, MB, sp, c->d_mb_stats);
        TRY(launch_check(c, __func__));
        return BPPO_OK;
    }
    uint32_t C = (B + 511) / 512;
    if (sp.base > 0 && C > sp.base) C = sp.base;
    if (sp.base == 0) C = 1;
    const uint32_t nblk = (B + C - 1) / C;
    if ((size_t)nblk * 8 > 4 * 1024 + 64) { c->err = "epoch advantage stats: too many minibatches"; return BPPO_ERR_UNSUPPORTED; }
    hipLaunchKernelGGL(k_adv_epoch, dim3(nblk), dim3(ADV_THREADS), 0, c->stream, c->d_adv, c->d_perm, sp, C, c->d_red);
    hipLaunchKernelGGL(k_adv_epoch_final, dim3(M), dim3(256), 0, c->stream, c->d_red, (int)nblk, C, sp, c->d_mb_stats);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

static AdamArgs adam_args(bppo_ctx *c, float lr, const float *c1, const float *c2) {
    AdamArgs a;
    a.params = c->d_params; a.grad = c->d_grad; a.m1 = c->d_m1; a.m2 = c->d_m2;
    a.nt = 2 * c->net.n_layers;
    for (int l = 0; l < c->net.n_layers; l++) {
        a.t[2 * l] = AdamTensor{(int)c->net.w[l], c->net.in[l] * c->net.out[l], c1[2 * l], c2[2 * l]};
        a.t[2 * l + 1] = AdamTensor{(int)c->net.b[l], c->net.out[l], c1[2 * l + 1], c2[2 * l + 1]};
    }
    a.lr = lr; a.max_norm = (float)c->cfg.max_grad_norm; a.eps = (float)c->cfg.adam_epsilon;
    a.inv_world = 1.0f / (float)c->world;
    a.part = c->d_red;
    int nb = 0;
    for (int t = 0; t < a.nt; t++) { a.blk0[t] = nb; nb += (a.t[t].len + ADAM_CHUNK - 1) / ADAM_CHUNK; }
    a.blk0[a.nt] = nb;
    return a;
}

bppo_status launch_minibatch(bppo_ctx *c, uint32_t start, uint32_t n, float ent_coef, bool exact) {
    const int h = c->cfg.hidden_size, nl = c->cfg.num_hidden;
    MbArgs g;
    g.obs = c->d_obs; g.logp = c->d_logp; g.adv = c->d_adv; g.ret = c->u_ret; g.val = c->u_val;
    g.act = c->d_act; g.perm = c->d_perm; g.start = start; g.n = n; g.params = c->d_params;
    g.mb_stats = c->d_mb_cur; g.slab = c->d_slab; g.np = (int)c->net.n_params;
    g.lo = (float)(1.0 - c->cfg.clip_epsilon); g.hi = (float)(1.0 + c->cfg.clip_epsilon);
    g.ceps = (float)c->cfg.clip_epsilon;
    g.inv_mb = (float)(1.0 / (double)n); g.ent_coef = ent_coef; g.value_coef = (float)c->cfg.value_coef;
    g.clip_value = c->cfg.clip_value;
    g.rowA = c->d_rowA; g.rowB = c->d_rowB;
    g.stamps = nullptr;
#ifdef BPPO_MB_STAMPS
    static unsigned long long *d_st = nullptr;
    if (!d_st) (void)hipMalloc((void **)&d_st, sizeof(unsigned long long) * 2048 * MB_NSEG);
    (void)hipMemsetAsync(d_st, 0, sizeof(unsigned long long) * 2048 * MB_NSEG, c->stream);
    g.stamps = d_st;
#endif
    int blocks = 256;
    const size_t params_bytes = ((c->net.n_params + 3) & ~(size_t)3) * sizeof(float);
    if (h == 64 && nl == 2 && c->relu_mfma) {
        if ((size_t)mmb::WAVES * (c->net.n_params + NUM_M) * sizeof(float) > mmb::LDSB) {
            c->err = "minibatch kernel: gradient rows exceed LDS";
            return BPPO_ERR_UNSUPPORTED;
        }
        c->slab_used = blocks;
        // the update's first minibatch runs with the rollout's parameters: its forward is the
        // exact f32 one, so the ratio is exactly 1 -- since r06 the split kernel's exact-forward
        // variant (k_minibatch_split<true>: the backward on the split-bf16 contraction; was
        // k_minibatch_mfma, exact throughout); the others on the split-bf16 kernel
        // (BPPO_MB_EXACT_ALL=1: the exact kernel for every minibatch; BPPO_MB_FIRST_MFMA=1:
        // k_minibatch_mfma for the first, as r05 -- A/B runs)
        // (bppo_set_minibatch_kernel: 1 = exact for every minibatch, 2 = split for every one)
        static const bool exact_all = getenv("BPPO_MB_EXACT_ALL") != nullptr;
        static const bool first_mfma = getenv("BPPO_MB_FIRST_MFMA") && atoi(getenv("BPPO_MB_FIRST_MFMA")) == 1;
        const bool use_exact = c->mb_kernel == 1 || (c->mb_kernel == 0 && (exact_all || (exact && first_mfma)));
        const bool exact_fwd = !use_exact && c->mb_kernel == 0 && exact;
        const size_t lds_rows = (size_t)mmf::WAVES * (c->net.n_params + NUM_M) * sizeof(float);
        const size_t lds_split = std::max(mmf::lds_tiles<false>(), lds_rows);
        const size_t lds_split_x = std::max(mmf::lds_tiles<true>(), lds_rows);
        // HIP timer events around the launch (bench.py's roofline): every launch by default;
        // BPPO_MB_EVENTS=k times every k-th launch of an update (0: none), for A/B runs of the
        // timestamp markers' cost on the stream
        static const int ev_every = getenv("BPPO_MB_EVENTS") ? atoi(getenv("BPPO_MB_EVENTS")) : 1;
        const bool timed = ev_every > 0 && c->mb_launch++ % ev_every == 0;
        const int ei = timed && c->mb_ev_n < bppo_ctx::MB_EV ? c->mb_ev_n++ : -1;
        // (the roofline's "exact" share: the update's first minibatch, whichever kernel runs it)
        if (ei >= 0) { c->mb_ev_split[ei] = !use_exact && !exact_fwd; BPPO_HIP(c, hipEventRecord(c->mb_ev[ei][0], c->stream)); }
        if (use_exact)
            hipLaunchKernelGGL(k_minibatch_mfma, dim3(blocks), dim3(64 * mmb::WAVES), mmb::LDSB, c->stream, g);
        else if (exact_fwd)
            hipLaunchKernelGGL(k_minibatch_split<true>, dim3(blocks), dim3(64 * mmf::WAVES), lds_split_x, c->stream, g);
        else
            hipLaunchKernelGGL(k_minibatch_split<false>, dim3(blocks), dim3(64 * mmf::WAVES), lds_split, c->stream, g);
        if (ei >= 0) BPPO_HIP(c, hipEventRecord(c->mb_ev[ei][1], c->stream));
#ifdef BPPO_MB_STAMPS
        if ((!use_exact && !exact_fwd) || getenv("BPPO_MB_STAMPS_EXACT")) {
            // mean per-wave cycles per segment of the split launches (the exact kernel's with
            // BPPO_MB_STAMPS_EXACT), accumulated over launches; printed every 16
            static double acc_s[MB_NSEG] = {};
            static int nl = 0;
            std::vector<unsigned long long> h((size_t)blocks * mmb::WAVES * MB_NSEG);
            (void)hipMemcpyAsync(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost, c->stream);
            (void)hipStreamSynchronize(c->stream);
            for (size_t w = 0; w < (size_t)blocks * mmb::WAVES; w++)
                for (int k = 0; k < MB_NSEG; k++) acc_s[k] += (double)h[w * MB_NSEG + k] / (blocks * mmb::WAVES);
            if (++nl % 16 == 0) {
                double tot = 0;
                for (int k = 0; k < MB_NSEG; k++) tot += acc_s[k];
                fprintf(stderr, "[mbstamp] launches=%d cycles/wave=%.0f shares:", nl, tot / nl);
                for (int k = 0; k < MB_NSEG; k++) fprintf(stderr, " s%d=%.3f", k, acc_s[k] / tot);
                fprintf(stderr, "\n");
            }
        }
#endif
    } else
#define L(H_, NL_)                                                                                 \
    if (h == H_ && nl == NL_) {                                                                     \
        size_t lds = params_bytes + 4 * sizeof(WaveStage<H_>);                                      \
        c->slab_used = blocks * 4;                                                                  \
        if (c->cfg.relu)                                                                            \
            hipLaunchKernelGGL((k_minibatch<H_, NL_, ACT_RELU>), dim3(blocks), dim3(256), lds, c->stream, g); \
        else                                                                                        \
            hipLaunchKernelGGL((k_minibatch<H_, NL_, ACT_TANH>), dim3(blocks), dim3(256), lds, c->stream, g); \
    } else
    L(16, 1) L(16, 2) L(32, 1) L(32, 2) L(64, 1) L(64, 2) {
        c->err = "minibatch kernel: unsupported MLP shape";
        return BPPO_ERR_UNSUPPORTED;
    }
#undef L
    TRY(launch_check(c, __func__));
    const int width = (int)c->net.n_params + NUM_M;
    static_assert(M_VEMAX == GRAD_VEMAX && NUM_M <= GRAD_METRIC_SLOTS, "metric slot layout");
    hipLaunchKernelGGL(k_slab_reduce1, dim3((width + SLAB1_COLS - 1) / SLAB1_COLS), dim3(SLAB1_COLS * SLAB_GROUPS), 0,
                       c->stream, c->d_slab,
                       c->slab_used, width, c->d_grad, c->d_grad + c->net.n_params + GRAD_VEMAX_LOCAL);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// one minibatch's metric sums (grad tail) and advantage stats into the update's rows
__global__ void k_metric_row(const float *gtail, const float *mb_stats, int nm, float *dst) {
    const int i = threadIdx.x;
    if (i < nm) dst[i] = gtail[i == GRAD_VEMAX ? GRAD_VEMAX_LOCAL : i];
    else if (i < nm + 4) dst[i] = mb_stats[i - nm];
}
bppo_status launch_metric_row(bppo_ctx *c, float *dst, int nm) {
    hipLaunchKernelGGL(k_metric_row, dim3(1), dim3(64), 0, c->stream, c->d_grad + c->net.n_params, c->d_mb_cur, nm,
                       dst);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

bppo_status launch_adam(bppo_ctx *c, float lr, const float *c1, const float *c2, float *metric_dst, int nm) {
    const AdamArgs a = adam_args(c, lr, c1, c2);
    const int nb = a.blk0[a.nt];
    if (nb == a.nt && metric_dst) {       // one chunk per tensor: fused
        hipLaunchKernelGGL(k_adam1, dim3(nb), dim3(ADAM1_THREADS), 0, c->stream, a, c->d_grad + c->net.n_params,
                           c->d_mb_cur, nm, metric_dst);
        TRY(launch_check(c, __func__));
        return BPPO_OK;
    }
    hipLaunchKernelGGL(k_adam_norm, dim3(nb), dim3(256), 0, c->stream, a);
    hipLaunchKernelGGL(k_adam, dim3(nb), dim3(256), 0, c->stream, a);
    TRY(launch_check(c, __func__));
    if (metric_dst) return launch_metric_row(c, metric_dst, nm);
    return BPPO_OK;
}

// enqueue: block sums into pinned h_red; explained_variance_sums reads them once the
// caller has waited for the stream
bppo_status launch_explained_variance(bppo_ctx *c, const float *valid) {
    const size_t n = (size_t)c->T * c->N;
    // BPPO_ZERO_COPY=1: the block sums straight into the pinned buffer (its device address)
    const bool zc = zero_copy();
    hipLaunchKernelGGL(k_ev, dim3(STAT_BLOCKS), dim3(256), 0, c->stream, n, c->d_val, c->d_ret, valid,
                       zc ? c->hd_red : c->d_red);
    TRY(launch_check(c, __func__));
    if (!zc)
        BPPO_HIP(c, hipMemcpyAsync(c->h_red, c->d_red, sizeof(double) * 4 * STAT_BLOCKS,
                                   hipMemcpyDeviceToHost, c->stream));
    return BPPO_OK;
}
void explained_variance_sums(bppo_ctx *c, double *out4) {
    for (int k = 0; k < 4; k++) out4[k] = 0.0;
    for (int b = 0; b < STAT_BLOCKS; b++)
        for (int k = 0; k < 4; k++) out4[k] += c->h_red[b * 4 + k];
}

}  // namespace bppo

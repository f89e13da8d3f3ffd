// popart.hip — value normalization with value-head rescaling (PopArt;
// normalization.rs:262-366 PopArtNormalizer, ppo.rs:1599-1653 rescale, ppo.rs:
// 1780-1808 and 1859-1897 in ppo_update; config normalize_values, default off).
//
//   rollout / bootstrap  the network outputs normalized values: stored and
//                        bootstrap values are denormalized, v*std + mean in f64
//                        then f32 (ppo.rs:355-359, main.rs:898-907) — an
//                        elementwise pass (CartPole) or inside the sampler
//                        (k_sample_masked, multi-player);
//   update begin         the running (count, mean, M2) absorbs every return of
//                        the buffer (learner rows under an opponent pool): block
//                        Welford partials in f64, Chan-merged in block order;
//                        then, once count >= 2, the value head is rescaled,
//                        W *= old_std / new_std, b = (b old_std + old_mean -
//                        new_mean) / new_std (f64 math, f32 results);
//   minibatches          returns and old values enter the loss normalized,
//                        ((x - mean) / std) as f32: one elementwise pass into
//                        the update's return / value buffers (the statistics
//                        are fixed for the whole update);
//   metrics              value_norm_target_mean / std over the normalized
//                        returns of every minibatch run (f64 sums), rescale_mag.
#include "bppo_internal.h"
#include <cmath>
#include <cstring>
#include <vector>

namespace bppo {

#define PTRY(x)                                \
    do {                                       \
        bppo_status _s = (x);                  \
        if (_s != BPPO_OK) return _s;          \
    } while (0)
#define PHIP(c, expr)                                                       \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);              \
    } while (0)

double popart_std(const bppo_ctx *c) {          // normalization.rs:299-305
    return c->pa_count < 2.0 ? 1.0 : std::sqrt(c->pa_m2 / c->pa_count + c->pa_eps);
}

__global__ void k_popart_denorm(size_t n, float *v, double mean, double sd) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        v[i] = (float)((double)v[i] * sd + mean);
}

__global__ void k_popart_normalize(size_t n, const float *x, float *y, double mean, double sd) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        y[i] = (float)(((double)x[i] - mean) / sd);
}

// Welford partials of the returns, block b over the contiguous range [b C, b C + C),
// rows with valid <= 0.5 skipped; per thread a sequential Welford, then a
// fixed-order Chan tree over the block -> part[b] = {n, mean, M2}
constexpr int PA_BLOCKS = 1024;
__global__ void __launch_bounds__(256) k_popart_stats(size_t n, const float *ret, const float *valid, Welford *part) {
    __shared__ Welford sh[256];
    const size_t C = (n + gridDim.x - 1) / gridDim.x;
    const size_t i0 = (size_t)blockIdx.x * C, i1 = i0 + C < n ? i0 + C : n;
    Welford w{0.0, 0.0, 0.0};
    for (size_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
        if (valid && !(valid[i] > 0.5f)) continue;
        const double x = ret[i];
        w.n += 1.0;
        const double d = x - w.mean;
        w.mean += d / w.n;
        w.m2 += d * (x - w.mean);
    }
    sh[threadIdx.x] = w;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) {
            const Welford a = sh[threadIdx.x], b = sh[threadIdx.x + st];
            const double nn = a.n + b.n;
            Welford m{nn, a.mean, a.m2};
            if (b.n > 0) {
                const double d = b.mean - a.mean;
                m.mean = a.mean + d * (b.n / nn);
                m.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / nn);
            }
            sh[threadIdx.x] = m;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) part[blockIdx.x] = sh[0];
}

// f64 sum / sum of squares of x[idx[i]] (idx may be null: x[i]), rows with valid <= 0.5
// skipped (valid indexed like x); one partial pair per block
__global__ void __launch_bounds__(256) k_popart_sums(size_t n, const float *x, const uint32_t *idx, const float *valid,
                                                      double *part) {
    __shared__ double s1[256], s2[256];
    double a = 0.0, b = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t j = idx ? idx[i] : i;
        if (valid && !(valid[j] > 0.5f)) continue;
        const double v = x[j];
        a += v; b += v * v;
    }
    s1[threadIdx.x] = a; s2[threadIdx.x] = b;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) { s1[threadIdx.x] += s1[threadIdx.x + st]; s2[threadIdx.x] += s2[threadIdx.x + st]; }
        __syncthreads();
    }
    if (threadIdx.x == 0) { part[2 * blockIdx.x] = s1[0]; part[2 * blockIdx.x + 1] = s2[0]; }
}

// ppo.rs:1599-1653 on the value head (layer net.value): W [in][1], b [1]
__global__ void k_popart_rescale(float *params, size_t w, int len, size_t b, double scale, double old_std,
                                 double old_mean, double new_mean, double new_std) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < len) params[w + i] = (float)((double)params[w + i] * scale);
    if (i == 0) params[b] = (float)(((double)params[b] * old_std + old_mean - new_mean) / new_std);
}

static dim3 pgrid(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 4096)); }

// denormalize n values in place with the current statistics (no-op before count >= 2)
bppo_status popart_denorm(bppo_ctx *c, float *v, size_t n) {
    if (!c->cfg.normalize_values || c->pa_count < 2.0 || n == 0) return BPPO_OK;
    hipLaunchKernelGGL(k_popart_denorm, pgrid(n), dim3(256), 0, c->stream, n, v, c->pa_mean, popart_std(c));
    PHIP(c, hipGetLastError());
    return BPPO_OK;
}

bppo_status popart_alloc(bppo_ctx *c) {
    const size_t TN = (size_t)c->T * c->N;
    PHIP(c, hipMalloc((void **)&c->d_ret_n, TN * 4));
    PHIP(c, hipMalloc((void **)&c->d_val_n, TN * 4));
    PHIP(c, hipMalloc((void **)&c->d_pa_part, sizeof(Welford) * PA_BLOCKS));   // >= 2 x 256 doubles of k_popart_sums
    return BPPO_OK;
}

void popart_free(bppo_ctx *c) {
    if (c->d_ret_n) (void)hipFree(c->d_ret_n);
    if (c->d_val_n) (void)hipFree(c->d_val_n);
    if (c->d_pa_part) (void)hipFree(c->d_pa_part);
    if (c->d_pa_gather) (void)hipFree(c->d_pa_gather);
}

static void chan_merge(Welford &a, const Welford &b) {
    if (b.n <= 0) return;
    const double nn = a.n + b.n, d = b.mean - a.mean;
    a.mean = a.mean + d * (b.n / nn);
    a.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / nn);
    a.n = nn;
}

// a double as three floats, exactly: hi = fl(d), mid = fl(d - hi), lo = d - hi - mid (the
// last <= 5 significand bits of d, a float exactly); a SUM all-reduce in which every
// other rank contributes zeros then moves it bit for bit
static void split3(double d, float *o) {
    const float hi = (float)d;
    const double r1 = d - (double)hi;
    const float mid = (float)r1;
    o[0] = hi; o[1] = mid; o[2] = (float)(r1 - (double)mid);
}
static double join3(const float *o) { return ((double)o[0] + (double)o[1]) + (double)o[2]; }

// W > 1: every rank's batch statistics {n, mean, M2} (its blocks Chan-merged in order)
// all-gathered through the gradient all-reduce callback (zeros but for the own slot,
// SUM), then merged into the running statistics rank by rank -- the same arithmetic on
// every rank, so the value-head rescale keeps the ranks' parameters identical
// (every_rank_has_rows: the self-play path, where each rank's batch holds T x N > 0 returns)
static bppo_status popart_gather(bppo_ctx *c, const std::vector<Welford> &part, Welford &a, bool every_rank_has_rows) {
    const int W = c->world;
    Welford mine{0.0, 0.0, 0.0};
    for (const Welford &b : part) chan_merge(mine, b);
    std::vector<float> g((size_t)9 * W, 0.0f);
    // the slot must come from bppo_set_rank: a default would put every rank into one slot,
    // and the SUM would then scale that slot's statistics by W on every rank alike
    if (c->rank < 0) { c->err = "PopArt at W > 1 needs this context's rank (bppo_set_rank)"; return BPPO_ERR_ARG; }
    if (c->rank >= W) { c->err = "PopArt at W > 1: rank outside [0, world) (bppo_set_rank)"; return BPPO_ERR_ARG; }
    split3(mine.n, &g[9 * c->rank]); split3(mine.mean, &g[9 * c->rank + 3]); split3(mine.m2, &g[9 * c->rank + 6]);
    float own[9];
    std::memcpy(own, &g[9 * c->rank], sizeof own);
    PHIP(c, hipMemcpyAsync(c->d_pa_gather, g.data(), g.size() * 4, hipMemcpyHostToDevice, c->stream));
    if (!c->allreduce_async) PHIP(c, hipStreamSynchronize(c->stream));
    if (c->allreduce(c->d_pa_gather, g.size(), c->allreduce_user) != 0) {
        c->err = "all-reduce callback failed (PopArt statistics)";
        return BPPO_ERR_COMM;
    }
    PHIP(c, hipMemcpyAsync(g.data(), c->d_pa_gather, g.size() * 4, hipMemcpyDeviceToHost, c->stream));
    PHIP(c, hipStreamSynchronize(c->stream));
    // two contexts given one rank: the slot they share holds a sum (checked by each of them),
    // and on the self-play path some other slot stays empty (seen by every rank alike)
    if (std::memcmp(own, &g[9 * c->rank], sizeof own) != 0) {
        c->err = "PopArt at W > 1: another rank wrote this context's slot (duplicated bppo_set_rank)";
        return BPPO_ERR_ARG;
    }
    for (int q = 0; q < W && every_rank_has_rows; q++)
        if (!(join3(&g[9 * q]) > 0.0)) {
            c->err = "PopArt at W > 1: a rank's slot is empty (duplicated or missing bppo_set_rank)";
            return BPPO_ERR_ARG;
        }
    for (int q = 0; q < W; q++) chan_merge(a, Welford{join3(&g[9 * q]), join3(&g[9 * q + 3]), join3(&g[9 * q + 6])});
    return BPPO_OK;
}

// ppo.rs:1787-1808 + the normalized return / old-value buffers the minibatches read
bppo_status popart_update_begin(bppo_ctx *c, const float *valid) {
    const size_t TN = (size_t)c->T * c->N;
    c->u_ret = c->d_ret; c->u_val = c->d_val;
    c->pa_rescale_mag = NAN;
    c->pa_tsum = c->pa_tsq = 0.0; c->pa_tcount = 0.0;
    if (!c->cfg.normalize_values) return BPPO_OK;
    hipLaunchKernelGGL(k_popart_stats, dim3(PA_BLOCKS), dim3(256), 0, c->stream, TN, c->d_ret, valid,
                       (Welford *)c->d_pa_part);
    PHIP(c, hipGetLastError());
    std::vector<Welford> part(PA_BLOCKS);
    PHIP(c, hipMemcpyAsync(part.data(), c->d_pa_part, sizeof(Welford) * PA_BLOCKS, hipMemcpyDeviceToHost, c->stream));
    PHIP(c, hipStreamSynchronize(c->stream));
    const double old_mean = c->pa_mean, old_std = popart_std(c);
    Welford a{c->pa_count, c->pa_mean, c->pa_m2};
    if (c->world > 1 && c->allreduce) PTRY(popart_gather(c, part, a, valid == nullptr));
    else
        for (const Welford &b : part) chan_merge(a, b);   // Chan merge in block (= row) order
    c->pa_count = a.n; c->pa_mean = a.mean; c->pa_m2 = a.m2;
    if (c->pa_count >= 2.0) {                             // is_initialized: rescale the value head
        const double new_mean = c->pa_mean, new_std = popart_std(c);
        const NetLayout &n = c->net;
        const int len = n.in[n.value];
        hipLaunchKernelGGL(k_popart_rescale, dim3((len + 255) / 256), dim3(256), 0, c->stream, c->d_params, n.w[n.value],
                           len, n.b[n.value], old_std / new_std, old_std, old_mean, new_mean, new_std);
        PHIP(c, hipGetLastError());
        c->pa_rescale_mag = (float)std::fabs(old_std / new_std);
        if (c->wide) PTRY(wide_pack(c));
        const double sd = new_std;
        hipLaunchKernelGGL(k_popart_normalize, pgrid(TN), dim3(256), 0, c->stream, TN, (const float *)c->d_ret, c->d_ret_n,
                           new_mean, sd);
        hipLaunchKernelGGL(k_popart_normalize, pgrid(TN), dim3(256), 0, c->stream, TN, (const float *)c->d_val, c->d_val_n,
                           new_mean, sd);
        PHIP(c, hipGetLastError());
        c->u_ret = c->d_ret_n; c->u_val = c->d_val_n;
    }
    return BPPO_OK;
}

// value_norm_target statistics over the (normalized) returns of the minibatches run
// (ppo.rs:1877-1881, 2061-2068): full epochs cover every (valid) row once; a
// KL-stopped epoch covers the first `rows_done` positions of its permutation
// (d_perm, mapped to buffer rows under an opponent pool)
bppo_status popart_target_stats(bppo_ctx *c, int full_epochs, size_t rows_done, const float *valid) {
    if (!c->cfg.normalize_values) return BPPO_OK;
    const size_t TN = (size_t)c->T * c->N;
    std::vector<double> h(2 * 256 * 2);
    auto sums = [&](size_t n, const uint32_t *idx, const float *vf, double &s1, double &s2) -> bppo_status {
        s1 = s2 = 0.0;
        if (!n) return BPPO_OK;
        hipLaunchKernelGGL(k_popart_sums, dim3(256), dim3(256), 0, c->stream, n, c->u_ret, idx, vf, c->d_pa_part);
        PHIP(c, hipGetLastError());
        PHIP(c, hipMemcpyAsync(h.data(), c->d_pa_part, sizeof(double) * 512, hipMemcpyDeviceToHost, c->stream));
        PHIP(c, hipStreamSynchronize(c->stream));
        for (int b = 0; b < 256; b++) { s1 += h[2 * b]; s2 += h[2 * b + 1]; }
        return BPPO_OK;
    };
    double a1 = 0, a2 = 0, b1 = 0, b2 = 0;
    if (full_epochs > 0) PTRY(sums(TN, nullptr, valid, a1, a2));
    if (rows_done) PTRY(sums(rows_done, c->d_perm, nullptr, b1, b2));
    const double rows_all = valid ? (double)c->n_valid : (double)TN;
    c->pa_tsum = full_epochs * a1 + b1;
    c->pa_tsq = full_epochs * a2 + b2;
    c->pa_tcount = full_epochs * rows_all + (double)rows_done;
    return BPPO_OK;
}

}  // namespace bppo

// opponents.hip — opponent-pool rollouts (ppo.rs:537-1063) and the learner-only
// update filter (ppo.rs:165-180, 1696-1753) on the multi-player GEMM path.
//
// Per rollout step, on the context's stream:
//   k_opp_group   each env's mover: the learner (self-play envs [n_opp, N), and
//                 opponent envs on the learner's seat) or opponent model k; and
//                 the env's position in the step's draw order: learner rows
//                 first, then each model's rows in ascending model index, env
//                 order within a group (the reference samples the learner batch,
//                 then iterates a HashMap of opponent batches: its order is not
//                 deterministic, ours is ascending)
//   learner forward on all N rows; each model's actor forward on all N rows of
//   its own normalized copy, its rows' logits selected into the step's logits
//   sampling (k_sample_masked) at word base + position * A
//   env step, then k_opp_seats: the step's N*A Gumbel words, then for every
//   finished opponent game in env order OpponentPool::sample_all_slots and
//   EnvState::shuffle_positions from the main RNG (usize gen_range + u32
//   shuffle), then the learner-turn flags against the reshuffled seats.
// The main RNG position therefore lives on the device during the rollout and
// is read back once at its end.
#include "bppo_internal.h"
#include "bppo_wide.h"
#include <algorithm>
#include <cstring>
#include <vector>

namespace bppo {

constexpr int OPP_MAX_MODELS = 15;
constexpr int OG_THREADS = 1024;

__global__ void k_set_u64(uint64_t *p, uint64_t v) { *p = v; }

// group[e] = 0 (learner) or 1 + model; gpos[e] = the env's row in the step's
// draw order.  One block: per-thread env chunks counted per group in LDS,
// exclusive prefix per group, group bases in group order.
__global__ void __launch_bounds__(OG_THREADS) k_opp_group(int N, int n_opp, int P, int G, const int32_t *players,
                                                          const int32_t *lpos, const int32_t *p2o, int32_t *group,
                                                          int32_t *gpos, int32_t *gbase, int32_t *err) {
    __shared__ int cnt[OPP_MAX_MODELS + 1][OG_THREADS];
    __shared__ int base[OPP_MAX_MODELS + 2];
    const int tid = threadIdx.x;
    const int per = (N + OG_THREADS - 1) / OG_THREADS;
    const int e0 = tid * per, e1 = min(N, e0 + per);
    for (int g = 0; g < G; g++) cnt[g][tid] = 0;
    for (int e = e0; e < e1; e++) {
        int g = 0;
        if (e < n_opp) {
            const int cp = players[e];
            if (cp != lpos[e]) {
                const int m = p2o[(size_t)e * P + cp];
                if (m < 0 || m >= G - 1) { atomicOr(err, 4); } else g = 1 + m;
            }
        }
        group[e] = g;
        cnt[g][tid]++;
    }
    __syncthreads();
    if (tid < G) {                         // exclusive prefix of group tid over the threads
        int run = 0;
        for (int k = 0; k < OG_THREADS; k++) { const int v = cnt[tid][k]; cnt[tid][k] = run; run += v; }
        base[tid + 1] = run;
    }
    __syncthreads();
    if (tid == 0) {
        base[0] = 0;
        for (int g = 1; g <= G; g++) base[g] += base[g - 1];
        for (int g = 0; g <= G; g++) gbase[g] = base[g];
    }
    __syncthreads();
    for (int e = e0; e < e1; e++) {
        const int g = group[e];
        gpos[e] = base[g] + cnt[g][tid]++;
    }
}

// the step's raw rows in draw order: each model's rows become one contiguous slice
__global__ void k_opp_sort_rows(int N, int L, const int32_t *group, const int32_t *gpos, const float *src, float *dst) {
    const size_t n = (size_t)N * L;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t e = i / L, k = i - e * L;
        if (group[e] != 0) dst[(size_t)gpos[e] * L + k] = src[i];
    }
}

// the opponents' logits (draw order) into the step's logits for their rows
__global__ void k_opp_select(int N, int A, const int32_t *group, const int32_t *gpos, const float *src, float *dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * A) return;
    const int e = i / A;
    if (group[e] != 0) dst[i] = src[(size_t)gpos[e] * A + (i - e * A)];
}

// main-stream words from an LDS window [base, end) filled in parallel by the
// block; a position past the window (an env whose rejections run past it)
// falls back to computing its ChaCha block
struct WindowCursor {
    const uint32_t *buf;
    uint64_t base, end, pos;
    Key8 key;
    uint64_t stream;
    __device__ __forceinline__ uint32_t next() {
        uint32_t w;
        if (pos < end) {
            w = buf[pos - base];
        } else {
            uint32_t blk[16];
            chacha12_block(key, pos >> 4, stream, blk);
            w = blk[pos & 15];
        }
        pos++;
        return w;
    }
};

// rand 0.8.5 UniformInt<u64> / <u32>::sample_single on the counter-based main
// stream (same restatement as oracle/rng.c)
template <class Cur>
__device__ __forceinline__ uint64_t dev_range_u64(Cur &c, uint64_t range) {
    const uint64_t zone = (range << __clzll((long long)range)) - 1ull;
    for (;;) {
        const uint64_t lo32 = c.next(), hi32 = c.next();
        const uint64_t v = (hi32 << 32) | lo32;
        const uint64_t lo = v * range, hi = __umul64hi(v, range);
        if (lo <= zone) return hi;
    }
}
template <class Cur>
__device__ __forceinline__ uint32_t dev_range_u32(Cur &c, uint32_t range) {
    const uint32_t zone = (range << __clz((int)range)) - 1u;
    for (;;) {
        const uint64_t m = (uint64_t)c.next() * range;
        if ((uint32_t)m <= zone) return (uint32_t)(m >> 32);
    }
}

// after the env step: the step's N*A sampling words, then the seat reshuffle of
// every finished opponent game (env order, main RNG), then the learner-turn
// flags against the new seats (ppo.rs:874-925, 928-937)
constexpr int SEAT_THREADS = 1024, SEAT_CHUNK = 8192, SEAT_WORDS = 4096, SEAT_MARGIN = 64;
__global__ void __launch_bounds__(SEAT_THREADS) k_opp_seats(int N, int n_opp, int P, int A, const float *done,
                                                            const int32_t *players, Key8 key, uint64_t stream,
                                                            const int32_t *curopp, uint64_t *rngpos, int32_t *lpos,
                                                            int32_t *p2o, float *valid) {
    __shared__ int list[SEAT_CHUNK];
    __shared__ int cnt[SEAT_THREADS];
    __shared__ uint32_t words[SEAT_WORDS];
    __shared__ uint64_t pos;
    __shared__ int qnext;
    const int tid = threadIdx.x;
    if (tid == 0) pos = *rngpos + (uint64_t)N * A;
    // finished opponent games in env order, chunk by chunk: flags read in
    // parallel and compacted, the draws (sequential in the RNG) on one thread
    for (int c0 = 0; c0 < n_opp; c0 += SEAT_CHUNK) {
        const int c1 = min(n_opp, c0 + SEAT_CHUNK);
        const int per = (c1 - c0 + SEAT_THREADS - 1) / SEAT_THREADS;
        const int e0 = c0 + tid * per, e1 = min(c1, e0 + per);
        int k = 0;
        for (int e = e0; e < e1; e++) k += done[e] != 0.0f;
        cnt[tid] = k;
        __syncthreads();
        if (tid == 0) {
            int run = 0;
            for (int q = 0; q < SEAT_THREADS; q++) { const int v = cnt[q]; cnt[q] = run; run += v; }
            list[SEAT_CHUNK - 1] = run;   // count (list slot reused after the writes below)
        }
        __syncthreads();
        const int nd = list[SEAT_CHUNK - 1];
        __syncthreads();
        int o = cnt[tid];
        for (int e = e0; e < e1; e++) if (done[e] != 0.0f) list[o++] = e;
        __syncthreads();
        if (tid == 0) qnext = 0;
        __syncthreads();
        while (qnext < nd) {
            // the next SEAT_WORDS words from pos's block on, one ChaCha block per thread
            const uint64_t wbase = (pos >> 4) << 4;
            if (tid < SEAT_WORDS / 16) chacha12_block(key, (wbase >> 4) + tid, stream, (uint32_t *)&words[tid * 16]);
            __syncthreads();
            if (tid == 0) {
                WindowCursor c{words, wbase, wbase + SEAT_WORDS, pos, key, stream};
                int q = qnext;
                for (; q < nd && c.pos + SEAT_MARGIN <= c.end; q++) {
                    const int e = list[q];
                    const int lp = (int)dev_range_u64(c, (uint64_t)P);        // opponent_pool.rs:109
                    int other[BPPO_MAX_PLAYERS], no = 0;
                    for (int p = 0; p < P; p++) if (p != lp) other[no++] = p;
                    for (int i = no - 1; i >= 1; i--) {                          // :114-115 SliceRandom::shuffle
                        const int j = (int)dev_range_u32(c, (uint32_t)(i + 1));
                        const int t = other[i]; other[i] = other[j]; other[j] = t;
                    }
                    lpos[e] = lp;
                    int32_t *row = p2o + (size_t)e * P;
                    for (int p = 0; p < P; p++) row[p] = -1;
                    for (int i = 0; i < no; i++) row[other[i]] = curopp[i];
                }
                pos = c.pos;
                qnext = q;
            }
            __syncthreads();
        }
    }
    if (tid == 0) *rngpos = pos;
    __threadfence_block();
    __syncthreads();
    for (int e = tid; e < N; e += blockDim.x)
        valid[e] = (e >= n_opp || players[e] == lpos[e]) ? 1.0f : 0.0f;
}

// learner rows of the rollout in (t, e) order (ppo.rs:165-180)
__global__ void __launch_bounds__(OG_THREADS) k_compact_valid(size_t n, const float *valid, uint32_t *vidx,
                                                              uint32_t *count) {
    __shared__ uint32_t cnt[OG_THREADS];
    const int tid = threadIdx.x;
    const size_t per = (n + OG_THREADS - 1) / OG_THREADS;
    const size_t i0 = (size_t)tid * per, i1 = min(n, i0 + per);
    uint32_t k = 0;
    for (size_t i = i0; i < i1; i++) k += valid[i] > 0.5f;
    cnt[tid] = k;
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int q = 0; q < OG_THREADS; q++) { const uint32_t v = cnt[q]; cnt[q] = run; run += v; }
        *count = run;
    }
    __syncthreads();
    uint32_t o = cnt[tid];
    for (size_t i = i0; i < i1; i++)
        if (valid[i] > 0.5f) vidx[o++] = (uint32_t)i;
}

// the permutation over the learner rows, mapped to buffer rows
__global__ void k_map_perm(uint32_t n, const uint32_t *vidx, uint32_t *perm) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) perm[j] = vidx[perm[j]];
}

bool opp_active(const bppo_ctx *c) { return c->wide && c->n_opp > 0 && c->opp_K > 0; }

void opp_free(bppo_ctx *c) {
    void *ptrs[] = {c->d_opp_params, c->d_opp_on, c->d_lpos, c->d_p2o, c->d_curopp, c->d_group, c->d_gpos,
                    c->d_valid, c->d_rngpos, c->d_oraw, c->d_oxc, c->d_ologits, c->d_vidx, c->d_Jopp, c->d_nvalid,
                    c->d_gbase};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    if (c->h_gbase) (void)hipHostFree(c->h_gbase);
    c->h_gbase = nullptr; c->d_gbase = nullptr;
    c->d_opp_params = nullptr; c->d_opp_on = nullptr; c->d_lpos = c->d_p2o = c->d_curopp = nullptr;
    c->d_group = c->d_gpos = nullptr; c->d_valid = nullptr; c->d_rngpos = nullptr;
    c->d_oraw = c->d_oxc = c->d_ologits = nullptr; c->d_vidx = c->d_Jopp = c->d_nvalid = nullptr;
}

template <class T>
static bppo_status oalloc(bppo_ctx *c, T **p, size_t n) {
    if (*p) return BPPO_OK;
    BPPO_HIP(c, hipMalloc((void **)p, std::max<size_t>(n, 1) * sizeof(T)));
    BPPO_HIP(c, hipMemsetAsync(*p, 0, std::max<size_t>(n, 1) * sizeof(T), c->stream));
    return BPPO_OK;
}

bppo_status opp_alloc(bppo_ctx *c) {
    const size_t N = c->N, TN = (size_t)c->T * c->N;
    TRY(oalloc(c, &c->d_group, N));
    TRY(oalloc(c, &c->d_gpos, N));
    TRY(oalloc(c, &c->d_valid, TN));
    TRY(oalloc(c, &c->d_rngpos, 1));
    TRY(oalloc(c, &c->d_oraw, N * c->L));
    TRY(oalloc(c, &c->d_oxc, N * c->L));
    TRY(oalloc(c, &c->d_ologits, N * c->A));
    TRY(oalloc(c, &c->d_vidx, TN));
    TRY(oalloc(c, &c->d_Jopp, TN));
    TRY(oalloc(c, &c->d_nvalid, 1));
    TRY(oalloc(c, &c->d_curopp, 4));
    TRY(oalloc(c, &c->d_gbase, OPP_MAX_MODELS + 2));
    if (!c->h_gbase) BPPO_HIP(c, hipHostMalloc((void **)&c->h_gbase, sizeof(int32_t) * (OPP_MAX_MODELS + 2)));
    return BPPO_OK;
}

bppo_status opp_rollout_begin(bppo_ctx *c, uint64_t base) {
    hipLaunchKernelGGL(k_set_u64, dim3(1), dim3(1), 0, c->stream, c->d_rngpos, base);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

// raw rows kept for the opponents' forwards, then movers and draw positions
bppo_status opp_step_group(bppo_ctx *c, int t) {
    const size_t r0 = (size_t)t * c->N;
    BPPO_HIP(c, hipMemcpyAsync(c->d_oraw, c->d_xc + r0 * c->L, sizeof(float) * (size_t)c->N * c->L,
                               hipMemcpyDeviceToDevice, c->stream));
    hipLaunchKernelGGL(k_opp_group, dim3(1), dim3(OG_THREADS), 0, c->stream, c->N, c->n_opp, c->Pa, c->opp_K + 1,
                       c->d_players + r0, c->d_lpos, c->d_p2o, c->d_group, c->d_gpos, c->d_gbase, c->d_err);
    TRY(launch_check(c, __func__));
    // the per-model row counts size the opponents' GEMMs: one small read per step
    BPPO_HIP(c, hipMemcpyAsync(c->h_gbase, c->d_gbase, sizeof(int32_t) * (c->opp_K + 2), hipMemcpyDeviceToHost,
                               c->stream));
    BPPO_HIP(c, hipStreamSynchronize(c->stream));
    return BPPO_OK;
}

// each model's actor forward (its own obs normalizer, ppo.rs:809-812) on all
// rows; its rows' logits replace the learner's in d_logits
bppo_status opp_step_forwards(bppo_ctx *c) {
    const size_t np = c->net.n_params;
    const int32_t *gb = c->h_gbase;            // group g owns draw rows [gb[g], gb[g + 1])
    if (gb[c->opp_K + 1] == gb[1]) return BPPO_OK;   // no opponent moves this step
    {
        const size_t n = (size_t)c->N * c->L;
        hipLaunchKernelGGL(k_opp_sort_rows, dim3((unsigned)std::min<size_t>((n + 255) / 256, 8192)), dim3(256), 0,
                           c->stream, c->N, c->L, c->d_group, c->d_gpos, c->d_oraw, c->d_oxc);
        TRY(launch_check(c, __func__));
    }
    for (int k = 0; k < c->opp_K; k++) {
        const int r0 = gb[k + 1], rows = gb[k + 2] - gb[k + 1];
        if (rows <= 0) continue;
        float *x = c->d_oxc + (size_t)r0 * c->L;
        if (c->opp_has_norm[k])
            TRY(launch_obs_norm_rows_on(c, rows, x + c->G, c->L, nullptr, c->d_opp_on + (size_t)k * (2 * c->D + 1)));
        TRY(wide_forward_actor(c, rows, x, c->L, c->d_opp_params + (size_t)k * np, c->d_ologits + (size_t)r0 * c->A));
    }
    const int n = c->N * c->A;
    hipLaunchKernelGGL(k_opp_select, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->N, c->A, c->d_group,
                       c->d_gpos, c->d_ologits, c->d_logits);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

bppo_status opp_step_seats(bppo_ctx *c, int t) {
    const size_t r0 = (size_t)t * c->N;
    hipLaunchKernelGGL(k_opp_seats, dim3(1), dim3(SEAT_THREADS), 0, c->stream, c->N, c->n_opp, c->Pa, c->A, c->d_done + r0,
                       c->d_players + r0, c->rng_key, (uint64_t)c->cfg.rng_stream, c->d_curopp, c->d_rngpos,
                       c->d_lpos, c->d_p2o, c->d_valid + r0);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

bppo_status opp_rollout_end(bppo_ctx *c) {
    uint64_t pos = 0;
    BPPO_HIP(c, hipMemcpyAsync(&pos, c->d_rngpos, 8, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, hipStreamSynchronize(c->stream));
    c->rng_pos = pos;
    return BPPO_OK;
}

bppo_status opp_compact_valid(bppo_ctx *c) {
    const size_t TN = (size_t)c->T * c->N;
    hipLaunchKernelGGL(k_compact_valid, dim3(1), dim3(OG_THREADS), 0, c->stream, TN, c->d_valid, c->d_vidx,
                       c->d_nvalid);
    uint32_t nv = 0;
    BPPO_HIP(c, hipMemcpyAsync(&nv, c->d_nvalid, 4, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, hipStreamSynchronize(c->stream));
    c->n_valid = nv;
    return BPPO_OK;
}

bppo_status opp_map_perm(bppo_ctx *c, uint32_t n) {
    hipLaunchKernelGGL(k_map_perm, dim3((n + 255) / 256), dim3(256), 0, c->stream, n, c->d_vidx, c->d_perm);
    TRY(launch_check(c, __func__));
    return BPPO_OK;
}

}  // namespace bppo

using namespace bppo;

// ppo.rs:537-1063 / main.rs:621-651: see include/bppo.h
extern "C" bppo_status bppo_opponents_set(bppo_ctx *c, int32_t n_models, const float *params, const double *norm_mean,
                                          const double *norm_m2, const double *norm_count, int32_t num_opponent_envs,
                                          const int32_t *learner_pos, const int32_t *pos_to_opp,
                                          const int32_t *current_opp) {
    if (!c) return BPPO_ERR_ARG;
    if (!c->wide) { c->err = "opponent pool: multi-player envs only"; return BPPO_ERR_UNSUPPORTED; }
    if (n_models < 0 || n_models > OPP_MAX_MODELS) { c->err = "opponent pool: 0..15 models"; return BPPO_ERR_ARG; }
    if (num_opponent_envs < 0 || num_opponent_envs > c->N) { c->err = "opponent pool: num_opponent_envs > num_envs"; return BPPO_ERR_ARG; }
    if (num_opponent_envs > 0 && c->cfg.shuffle_windows) { c->err = "opponent pool: not with shuffle_windows"; return BPPO_ERR_UNSUPPORTED; }
    if (num_opponent_envs > 0 && (!params || !learner_pos || !pos_to_opp || !current_opp || n_models == 0)) {
        c->err = "opponent pool: models and seat state required";
        return BPPO_ERR_ARG;
    }
    const int P = c->Pa, D = c->D;   // EnvState seats: the active player count (main.rs:552, 649)
    const size_t np = c->net.n_params;
    if (num_opponent_envs > 0) {
        for (int e = 0; e < num_opponent_envs; e++) {
            if (learner_pos[e] < 0 || learner_pos[e] >= P) { c->err = "opponent pool: learner_pos out of range"; return BPPO_ERR_ARG; }
            for (int p = 0; p < P; p++) {
                const int m = pos_to_opp[(size_t)e * P + p];
                if (p == learner_pos[e] ? m != -1 : (m < 0 || m >= n_models)) {
                    c->err = "opponent pool: pos_to_opp must name a model on every non-learner seat";
                    return BPPO_ERR_ARG;
                }
            }
        }
        for (int i = 0; i < P - 1; i++)
            if (current_opp[i] < 0 || current_opp[i] >= n_models) { c->err = "opponent pool: current_opp out of range"; return BPPO_ERR_ARG; }
    }
    TRY(opp_alloc(c));
    if (c->d_opp_params) { (void)hipFree(c->d_opp_params); c->d_opp_params = nullptr; }
    if (c->d_opp_on) { (void)hipFree(c->d_opp_on); c->d_opp_on = nullptr; }
    if (c->d_lpos) { (void)hipFree(c->d_lpos); c->d_lpos = nullptr; }
    if (c->d_p2o) { (void)hipFree(c->d_p2o); c->d_p2o = nullptr; }
    c->opp_K = n_models;
    c->n_opp = num_opponent_envs;
    c->opp_has_norm.assign(std::max(n_models, 1), 0);
    TRY(oalloc(c, &c->d_opp_params, np * std::max(n_models, 1)));
    TRY(oalloc(c, &c->d_opp_on, (size_t)(2 * D + 1) * std::max(n_models, 1)));
    TRY(oalloc(c, &c->d_lpos, (size_t)std::max(num_opponent_envs, 1)));
    TRY(oalloc(c, &c->d_p2o, (size_t)std::max(num_opponent_envs, 1) * P));
    // uploads are ordered on the context stream after oalloc's zeroing memsets (a
    // blocking hipMemcpy on the null stream would not wait for that non-blocking
    // stream); the stream is drained before the host arrays may go away
    if (n_models > 0)
        BPPO_HIP(c, hipMemcpyAsync(c->d_opp_params, params, sizeof(float) * np * n_models, hipMemcpyHostToDevice, c->stream));
    std::vector<double> on((size_t)(2 * D + 1) * std::max(n_models, 1), 0.0);
    for (int k = 0; k < n_models; k++) {
        if (!norm_count || norm_count[k] < 2.0 || !norm_mean || !norm_m2) continue;
        c->opp_has_norm[k] = 1;
        std::memcpy(&on[(size_t)k * (2 * D + 1)], norm_mean + (size_t)k * D, sizeof(double) * D);
        std::memcpy(&on[(size_t)k * (2 * D + 1) + D], norm_m2 + (size_t)k * D, sizeof(double) * D);
        on[(size_t)k * (2 * D + 1) + 2 * D] = norm_count[k];
    }
    BPPO_HIP(c, hipMemcpyAsync(c->d_opp_on, on.data(), sizeof(double) * on.size(), hipMemcpyHostToDevice, c->stream));
    if (num_opponent_envs > 0) {
        BPPO_HIP(c, hipMemcpyAsync(c->d_lpos, learner_pos, sizeof(int32_t) * num_opponent_envs, hipMemcpyHostToDevice, c->stream));
        BPPO_HIP(c, hipMemcpyAsync(c->d_p2o, pos_to_opp, sizeof(int32_t) * (size_t)num_opponent_envs * P,
                                   hipMemcpyHostToDevice, c->stream));
        BPPO_HIP(c, hipMemcpyAsync(c->d_curopp, current_opp, sizeof(int32_t) * (P - 1), hipMemcpyHostToDevice, c->stream));
    }
    BPPO_HIP(c, hipStreamSynchronize(c->stream));
    return BPPO_OK;
}

extern "C" bppo_status bppo_opponents_get_envs(bppo_ctx *c, int32_t *learner_pos, int32_t *pos_to_opp) {
    if (!c) return BPPO_ERR_ARG;
    if (!c->n_opp) return BPPO_OK;
    if (learner_pos) BPPO_HIP(c, hipMemcpyAsync(learner_pos, c->d_lpos, sizeof(int32_t) * c->n_opp, hipMemcpyDeviceToHost, c->stream));
    if (pos_to_opp)
        BPPO_HIP(c, hipMemcpyAsync(pos_to_opp, c->d_p2o, sizeof(int32_t) * (size_t)c->n_opp * c->Pa, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, hipStreamSynchronize(c->stream));
    return BPPO_OK;
}

// k_shuffle.hip — the permutation of one rand 0.8.5 shuffle from its swap
// targets, in parallel and bit-identical to the sequential Fisher-Yates
//     for i = n-1 .. 1: swap(a[i], a[J[i]])          (a = 0..n-1, J[i] <= i)
//
// Position i is final once step i ran (later steps touch only indices < i), and
// it then holds the value position J[i] had just before step i.  Position j's
// value changes only at steps i' > j with J[i'] = j, each of which moves in the
// value position i' had when step i' began.  With W(i) = value at position i
// when step i begins:
//     W(i)     = W(fw(i)),  fw(i) = min{ i' > i : J[i'] = i }   (W(i) = i if none)
//     perm[i]  = W(succ(i)), succ(i) = min{ i' > i : J[i'] = J[i] } (J[i] if none)
// (i = 0 is treated as a self-swap J[0] = 0).  So: bucket the steps by target,
// order each bucket, read succ/fw off neighbours, and follow fw chains (mean
// length ~1, max ~20 at n = 2^23).  Bit-exact; no host swaps.
//
// Two bucketings.  The direct one counts and scatters with one global atomic
// per step.  The ranged one (n >= FYB_MIN_N: the per-epoch shuffles of a
// context) partitions the steps into target ranges of equal expected load —
// J[i] is uniform on [0, i], so E#{i : J[i] < x} = x (1 + ln(n/x)) — with LDS
// histograms, each block reserving its slots in a range's fixed-capacity slice with
// one global atomic per (block, range), then sorts and links each range in LDS.  A
// range over its capacity (inputs far from uniform) raises a flag and the direct
// path runs after it, gated on that flag, so any J gives the same result.
#include <algorithm>
#include <cmath>
#include <vector>
#include "bppo_internal.h"

namespace bppo {

constexpr uint32_t FY_NONE = 0xFFFFFFFFu;
constexpr int SCAN_B = 1024;           // threads per scan block
constexpr int SCAN_IPT = 8;            // elements per thread
constexpr int SCAN_TILE = SCAN_B * SCAN_IPT;

// ranged bucketing
constexpr uint32_t FYB_MIN_N = 1u << 20;
constexpr int FYB_BLOCKS = 256;        // partition blocks (one contiguous chunk of steps each)
constexpr int FYB_THREADS = 1024;
constexpr double FYB_LOAD = 2048.0;    // expected steps per range
constexpr int FYB_CAP = 4096;          // LDS capacity (steps) of one range
constexpr int FYB_RMAX = 4096;         // max targets per range
constexpr int FYB_COARSE = 11;         // coarse index: first range of each 2^11-target block
constexpr int FYB_LINK_THREADS = 512;
constexpr size_t FYB_LDS_MAX = 120 * 1024;

// gate == nullptr: always run; else run only when *gate != 0 (a range overflowed)
#define FY_GATE(g) \
    if ((g) && *(g) == 0u) return

__global__ void __launch_bounds__(256) k_fy_zero(uint32_t *p, uint32_t n, const uint32_t *gate) {
    FY_GATE(gate);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = 0u;
}

__global__ void __launch_bounds__(256) k_fy_count(const uint32_t *J, uint32_t n, uint32_t *cnt, const uint32_t *gate) {
    FY_GATE(gate);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        atomicAdd(&cnt[J[i]], 1u);
}

// ---- exclusive scan of u32 counts (three passes: tile sums, scan of sums, tiles)
__device__ __forceinline__ uint32_t block_exclusive_u32(uint32_t v, uint32_t *sh, uint32_t *total) {
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) sh[w] = x;
    __syncthreads();
    if (w == 0) {
        uint32_t s = lane < (int)(blockDim.x >> 6) ? sh[lane] : 0u;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(s, o, 64);
            if (lane >= o) s += y;
        }
        if (lane < (int)(blockDim.x >> 6)) sh[lane] = s;
    }
    __syncthreads();
    const uint32_t wpre = w ? sh[w - 1] : 0u;
    *total = sh[(blockDim.x >> 6) - 1];
    __syncthreads();
    return wpre + x - v;
}

__global__ void __launch_bounds__(SCAN_B) k_scan_tiles(const uint32_t *in, uint32_t n, uint32_t *tile_sum,
                                                       const uint32_t *gate) {
    FY_GATE(gate);
    __shared__ uint32_t sh[SCAN_B / 64];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_IPT;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_IPT; k++) s += base + k < n ? in[base + k] : 0u;
    uint32_t tot;
    (void)block_exclusive_u32(s, sh, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_B) k_scan_sums(uint32_t *tile_sum, uint32_t ntiles, const uint32_t *gate) {
    FY_GATE(gate);
    __shared__ uint32_t sh[SCAN_B / 64];
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < ntiles; b0 += SCAN_B) {
        const uint32_t i = b0 + threadIdx.x;
        const uint32_t v = i < ntiles ? tile_sum[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_exclusive_u32(v, sh, &tot);
        if (i < ntiles) tile_sum[i] = carry + ex;
        carry += tot;
    }
}

// out may alias in (each thread reads its elements before writing them)
__global__ void __launch_bounds__(SCAN_B) k_scan_apply(const uint32_t *in, uint32_t n, const uint32_t *tile_pre,
                                                       uint32_t *out, const uint32_t *gate) {
    FY_GATE(gate);
    __shared__ uint32_t sh[SCAN_B / 64];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_IPT;
    uint32_t v[SCAN_IPT], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_IPT; k++) { v[k] = base + k < n ? in[base + k] : 0u; s += v[k]; }
    uint32_t tot;
    uint32_t run = tile_pre[blockIdx.x] + block_exclusive_u32(s, sh, &tot);
#pragma unroll
    for (int k = 0; k < SCAN_IPT; k++) {
        if (base + k < n) out[base + k] = run;
        run += v[k];
    }
}

static void launch_scan(const uint32_t *in, uint32_t n, uint32_t *scan, uint32_t *out, const uint32_t *gate,
                        hipStream_t st) {
    const uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(SCAN_B), 0, st, in, n, scan, gate);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SCAN_B), 0, st, scan, ntiles, gate);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(SCAN_B), 0, st, in, n, scan, out, gate);
}

// scatter step indices into their target's bucket (order inside a bucket fixed later)
__global__ void __launch_bounds__(256) k_fy_scatter(const uint32_t *J, uint32_t n, const uint32_t *off,
                                                    uint32_t *cnt, uint32_t *bucket, const uint32_t *gate) {
    FY_GATE(gate);
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t j = J[i];
        const uint32_t k = atomicSub(&cnt[j], 1u) - 1u;
        bucket[off[j] + k] = i;
    }
}

// one thread per target j: sort its bucket, link successors, first writer fw(j)
__global__ void __launch_bounds__(256) k_fy_link(uint32_t n, const uint32_t *off, uint32_t *bucket,
                                                 uint32_t *succ, uint32_t *fw, const uint32_t *gate) {
    FY_GATE(gate);
    for (uint32_t j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) {
        const uint32_t b = off[j], e = j + 1 < n ? off[j + 1] : n;
        for (uint32_t a = b + 1; a < e; a++) {              // insertion sort (mean size 1)
            const uint32_t x = bucket[a];
            uint32_t q = a;
            while (q > b && bucket[q - 1] > x) { bucket[q] = bucket[q - 1]; q--; }
            bucket[q] = x;
        }
        for (uint32_t a = b; a < e; a++) succ[bucket[a]] = a + 1 < e ? bucket[a + 1] : FY_NONE;
        uint32_t f = FY_NONE;
        if (e > b) f = bucket[b] > j ? bucket[b] : (e > b + 1 ? bucket[b + 1] : FY_NONE);
        fw[j] = f;
    }
}

// perm[i] = v, and optionally the inverse inv[v] = i (where each index landed:
// the epoch's per-minibatch advantage statistics then stream over the rows in
// order instead of gathering them through perm, k_update.hip k_adv_stream)
__global__ void __launch_bounds__(256) k_fy_final(const uint32_t *J, uint32_t n, const uint32_t *succ,
                                                  const uint32_t *fw, uint32_t *perm, const uint32_t *skip,
                                                  uint32_t *inv) {
    if (skip && *skip) return;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t s = succ[i];
        uint32_t v;
        if (s == FY_NONE) {
            v = J[i];
        } else {
            v = s;
            for (uint32_t f = fw[v]; f != FY_NONE; f = fw[v]) v = f;   // strictly increasing: terminates
        }
        perm[i] = v;
        if (inv) inv[v] = i;
    }
}

// ================================================================ ranged ==
struct FyTab {
    const uint32_t *x, *cb;
    int nb, ncb;
};

// range of target j: the coarse index gives a lower bound, boundaries step it up
__device__ __forceinline__ uint32_t fyb_range(uint32_t j, const uint32_t *x, const uint32_t *cb) {
    uint32_t b = cb[j >> FYB_COARSE];
    while (x[b + 1] <= j) b++;
    return b;
}

__device__ __forceinline__ void fyb_load_tab(const FyTab &t, uint32_t *sx, uint32_t *scb) {
    for (int k = threadIdx.x; k <= t.nb; k += blockDim.x) sx[k] = t.x[k];
    for (int k = threadIdx.x; k < t.ncb; k += blockDim.x) scb[k] = t.cb[k];
}

// pass 1: per-block range histogram of a contiguous chunk of steps, range-major
// H[b][blk] so that one exclusive scan gives every (range, block) write offset
constexpr int FYB_U = 8;
__global__ void __launch_bounds__(FYB_THREADS) k_fyb_hist(const uint32_t *J, uint32_t n, uint32_t chunk, FyTab t,
                                                          uint32_t *H, uint32_t *flag) {
    extern __shared__ uint32_t fsm[];
    uint32_t *sx = fsm, *scb = sx + t.nb + 1, *hist = scb + t.ncb;
    fyb_load_tab(t, sx, scb);
    for (int k = threadIdx.x; k < t.nb; k += blockDim.x) hist[k] = 0u;
    if (blockIdx.x == 0 && threadIdx.x == 0) *flag = 0u;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
    // FYB_U targets loaded before their counts (the plain loop waited on each load in turn;
    // the counts do not depend on the order)
    uint32_t i = i0 + threadIdx.x;
    for (; i + (FYB_U - 1) * blockDim.x < i1; i += FYB_U * blockDim.x) {
        uint32_t jv[FYB_U];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) jv[u] = J[i + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) atomicAdd(&hist[fyb_range(jv[u], sx, scb)], 1u);
    }
    for (; i < i1; i += blockDim.x) atomicAdd(&hist[fyb_range(J[i], sx, scb)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < t.nb; k += blockDim.x) H[(size_t)k * gridDim.x + blockIdx.x] = hist[k];
}

// pass 2: (step, target) pairs into their range's slice (order inside a slice is
// fixed by the link pass)
__global__ void __launch_bounds__(FYB_THREADS) k_fyb_scatter(const uint32_t *J, uint32_t n, uint32_t chunk, FyTab t,
                                                             const uint32_t *H, uint2 *P) {
    extern __shared__ uint32_t fsm[];
    uint32_t *sx = fsm, *scb = sx + t.nb + 1, *pos = scb + t.ncb;
    fyb_load_tab(t, sx, scb);
    for (int k = threadIdx.x; k < t.nb; k += blockDim.x) pos[k] = H[(size_t)k * gridDim.x + blockIdx.x];
    __syncthreads();
    const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
    uint32_t i = i0 + threadIdx.x;                // (the slot order inside a range is free: see above)
    for (; i + (FYB_U - 1) * blockDim.x < i1; i += FYB_U * blockDim.x) {
        uint32_t jv[FYB_U];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) jv[u] = J[i + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < FYB_U; u++)
            P[atomicAdd(&pos[fyb_range(jv[u], sx, scb)], 1u)] = make_uint2(i + u * blockDim.x, jv[u]);
    }
    for (; i < i1; i += blockDim.x) {
        const uint32_t j = J[i];
        P[atomicAdd(&pos[fyb_range(j, sx, scb)], 1u)] = make_uint2(i, j);
    }
}

// passes 1 + 2 in one launch (r06; was k_fyb_hist, a three-launch scan of the [range][block]
// counts and k_fyb_scatter): the block's range histogram in LDS, then one global atomic per
// (block, range) reserves the block's slots in the range's fixed-capacity slice of P
// ([nb][FYB_CAP]; cursor[b] ends as range b's step count), then the chunk's steps are
// scattered into them (its J re-read, an L2 hit).  The slot order inside a range is free:
// k_fyb_link sorts it.  A range past FYB_CAP raises the flag (its excess is not written)
__global__ void __launch_bounds__(FYB_THREADS) k_fyb_bucket(const uint32_t *J, uint32_t n, uint32_t chunk, FyTab t,
                                                            uint32_t *cursor, uint2 *P, uint32_t *flag) {
    extern __shared__ uint32_t fsm[];
    uint32_t *sx = fsm, *scb = sx + t.nb + 1, *hist = scb + t.ncb;
    fyb_load_tab(t, sx, scb);
    for (int k = threadIdx.x; k < t.nb; k += blockDim.x) hist[k] = 0u;
    __syncthreads();
    const uint32_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
    uint32_t i = i0 + threadIdx.x;
    for (; i + (FYB_U - 1) * blockDim.x < i1; i += FYB_U * blockDim.x) {
        uint32_t jv[FYB_U];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) jv[u] = J[i + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) atomicAdd(&hist[fyb_range(jv[u], sx, scb)], 1u);
    }
    for (; i < i1; i += blockDim.x) atomicAdd(&hist[fyb_range(J[i], sx, scb)], 1u);
    __syncthreads();
    for (int k = threadIdx.x; k < t.nb; k += blockDim.x) {
        const uint32_t c = hist[k];
        uint32_t b0 = 0u;
        if (c) {
            b0 = atomicAdd(&cursor[k], c);
            if (b0 + c > (uint32_t)FYB_CAP) atomicOr(flag, 1u);
        }
        hist[k] = (uint32_t)k * FYB_CAP + b0;      // this block's first slot in range k
    }
    __syncthreads();
    i = i0 + threadIdx.x;
    for (; i + (FYB_U - 1) * blockDim.x < i1; i += FYB_U * blockDim.x) {
        uint32_t jv[FYB_U];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) jv[u] = J[i + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < FYB_U; u++) {
            const uint32_t rb = fyb_range(jv[u], sx, scb);
            const uint32_t slot = atomicAdd(&hist[rb], 1u);
            if (slot < (rb + 1u) * (uint32_t)FYB_CAP) P[slot] = make_uint2(i + u * blockDim.x, jv[u]);
        }
    }
    for (; i < i1; i += blockDim.x) {
        const uint32_t j = J[i], rb = fyb_range(j, sx, scb);
        const uint32_t slot = atomicAdd(&hist[rb], 1u);
        if (slot < (rb + 1u) * (uint32_t)FYB_CAP) P[slot] = make_uint2(i, j);
    }
}

// pass 3: one block per range — counting sort by target in LDS, each target's
// steps ordered by index, then succ / fw exactly as k_fy_link.  Ranges come as a
// [range][block] offset table H (e0 = H[b][0]) or, cursor != nullptr, as fixed slices
// P[b * FYB_CAP ...] of cursor[b] steps (cursor[b] reset to 0 for the next permutation)
__global__ void __launch_bounds__(FYB_LINK_THREADS) k_fyb_link(uint32_t n, FyTab t, const uint32_t *H, int nblk,
                                                               const uint2 *P, uint32_t *succ, uint32_t *fw,
                                                               uint32_t *flag, uint32_t *cursor) {
    __shared__ uint32_t ent_i[FYB_CAP];
    __shared__ uint16_t ent_t[FYB_CAP];
    __shared__ uint32_t tst[FYB_RMAX + 1];
    __shared__ uint32_t tcur[FYB_RMAX];
    __shared__ uint32_t srt[FYB_CAP];
    __shared__ uint32_t sh[FYB_LINK_THREADS / 64];
    const int b = blockIdx.x;
    uint32_t e0, cnt;
    if (cursor) {
        e0 = (uint32_t)b * FYB_CAP;
        cnt = cursor[b];
        __syncthreads();                      // every thread has read the count
        if (threadIdx.x == 0) cursor[b] = 0u;
    } else {
        e0 = H[(size_t)b * nblk];
        cnt = (b + 1 < t.nb ? H[(size_t)(b + 1) * nblk] : n) - e0;
    }
    const uint32_t lo = t.x[b], R = t.x[b + 1] - lo;
    if (cnt > (uint32_t)FYB_CAP) {          // far from uniform: the gated direct path takes over
        if (threadIdx.x == 0) atomicOr(flag, 1u);
        return;
    }
    for (uint32_t k = threadIdx.x; k < R; k += blockDim.x) tcur[k] = 0u;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) {
        const uint2 e = P[e0 + k];
        ent_i[k] = e.x;
        ent_t[k] = (uint16_t)(e.y - lo);
        atomicAdd(&tcur[e.y - lo], 1u);
    }
    __syncthreads();
    constexpr int PER = FYB_RMAX / FYB_LINK_THREADS;
    const uint32_t k0 = threadIdx.x * PER;
    uint32_t v[PER], s = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) { v[q] = k0 + q < R ? tcur[k0 + q] : 0u; s += v[q]; }
    uint32_t tot;
    uint32_t run = block_exclusive_u32(s, sh, &tot);
#pragma unroll
    for (int q = 0; q < PER; q++) {
        if (k0 + q < R) { tst[k0 + q] = run; tcur[k0 + q] = run; }
        run += v[q];
    }
    if (threadIdx.x == 0) tst[R] = cnt;
    __syncthreads();
    for (uint32_t k = threadIdx.x; k < cnt; k += blockDim.x) srt[atomicAdd(&tcur[ent_t[k]], 1u)] = ent_i[k];
    __syncthreads();
    for (uint32_t tt = threadIdx.x; tt < R; tt += blockDim.x) {
        const uint32_t a0 = tst[tt], a1 = tst[tt + 1], j = lo + tt;
        for (uint32_t a = a0 + 1; a < a1; a++) {            // insertion sort (mean size ~1)
            const uint32_t x = srt[a];
            uint32_t q = a;
            while (q > a0 && srt[q - 1] > x) { srt[q] = srt[q - 1]; q--; }
            srt[q] = x;
        }
        for (uint32_t a = a0; a < a1; a++) succ[srt[a]] = a + 1 < a1 ? srt[a + 1] : FY_NONE;
        uint32_t f = FY_NONE;
        if (a1 > a0) f = srt[a0] > j ? srt[a0] : (a1 > a0 + 1 ? srt[a0 + 1] : FY_NONE);
        fw[j] = f;
    }
}

// overflow fallback of the ranged path (a range held more steps than its LDS
// capacity: J far from uniform): the direct bucketing of k_fy_zero .. k_fy_final
// in ONE block, phase by phase (__syncthreads orders the block's global memory).
// Slow, exact, and launched unconditionally behind the flag, so the common case
// costs one empty launch instead of eight -- a block of FY_DIRECT_THREADS (r06: was 1024
// threads, which waited 72 us on average, up to 372, for a CU with room beside the
// update kernels, holding back the epoch's permutation event)
constexpr int FY_DIRECT_THREADS = 256;
__global__ void __launch_bounds__(FY_DIRECT_THREADS) k_fy_direct_block(const uint32_t *J, uint32_t n, uint32_t *scratch,
                                                                       uint32_t *perm, uint32_t *flag, uint32_t *inv) {
    if (*flag == 0u) return;
    __shared__ uint32_t sh[SCAN_B / 64];
    uint32_t *cnt = scratch, *bucket = scratch + (size_t)n, *succ = scratch + 2 * (size_t)n,
             *fw = scratch + 3 * (size_t)n, *off = perm;
    const uint32_t t = threadIdx.x, T = blockDim.x;
    for (uint32_t i = t; i < n; i += T) cnt[i] = 0u;
    __syncthreads();
    for (uint32_t i = t; i < n; i += T) atomicAdd(&cnt[J[i]], 1u);
    __syncthreads();
    uint32_t carry = 0;
    for (uint32_t b0 = 0; b0 < n; b0 += T * SCAN_IPT) {
        const uint32_t base = b0 + t * SCAN_IPT;
        uint32_t v[SCAN_IPT], sum = 0;
#pragma unroll
        for (int k = 0; k < SCAN_IPT; k++) { v[k] = base + k < n ? cnt[base + k] : 0u; sum += v[k]; }
        uint32_t tot;
        uint32_t run = carry + block_exclusive_u32(sum, sh, &tot);
#pragma unroll
        for (int k = 0; k < SCAN_IPT; k++) {
            if (base + k < n) off[base + k] = run;
            run += v[k];
        }
        carry += tot;
    }
    __syncthreads();
    for (uint32_t i = t; i < n; i += T) {
        const uint32_t j = J[i];
        bucket[off[j] + atomicSub(&cnt[j], 1u) - 1u] = i;
    }
    __syncthreads();
    for (uint32_t j = t; j < n; j += T) {
        const uint32_t b = off[j], e = j + 1 < n ? off[j + 1] : n;
        for (uint32_t a = b + 1; a < e; a++) {
            const uint32_t x = bucket[a];
            uint32_t q = a;
            while (q > b && bucket[q - 1] > x) { bucket[q] = bucket[q - 1]; q--; }
            bucket[q] = x;
        }
        for (uint32_t a = b; a < e; a++) succ[bucket[a]] = a + 1 < e ? bucket[a + 1] : FY_NONE;
        uint32_t f = FY_NONE;
        if (e > b) f = bucket[b] > j ? bucket[b] : (e > b + 1 ? bucket[b + 1] : FY_NONE);
        fw[j] = f;
    }
    __syncthreads();
    for (uint32_t i = t; i < n; i += T) {
        const uint32_t s = succ[i];
        uint32_t v = s;
        if (s == FY_NONE) v = J[i];
        else for (uint32_t f = fw[v]; f != FY_NONE; f = fw[v]) v = f;
        perm[i] = v;
        if (inv) inv[v] = i;
    }
    __syncthreads();
    if (t == 0) *flag = 0u;            // the ranged path's flag is 0 between permutations
}

static size_t fyb_lds(int nb, int ncb) { return sizeof(uint32_t) * (size_t)(2 * nb + 1 + ncb); }

// range boundaries: equal expected load FYB_LOAD, at most FYB_RMAX targets each
hipError_t fy_ranges_init(FyRanges &r, uint32_t n) {
    fy_ranges_free(r);
    r.n = n;
    if (n < FYB_MIN_N) return hipSuccess;
    const double nd = (double)n;
    auto load = [&](double x) { return x <= 0.0 ? 0.0 : x * (1.0 + std::log((nd + 0.5) / (x + 0.5))); };
    std::vector<uint32_t> x{0u};
    uint32_t cur = 0;
    while (cur < n) {
        const double goal = load(cur) + FYB_LOAD;
        uint64_t lo = (uint64_t)cur + 1, hi = std::min<uint64_t>((uint64_t)cur + FYB_RMAX, n);
        if (load((double)hi) <= goal) {
            lo = hi;
        } else {
            while (lo < hi) {
                const uint64_t mid = (lo + hi) / 2;
                if (load((double)mid) >= goal) hi = mid; else lo = mid + 1;
            }
        }
        cur = (uint32_t)lo;
        x.push_back(cur);
    }
    const int nb = (int)x.size() - 1;
    std::vector<uint32_t> cb(((size_t)n >> FYB_COARSE) + 1);
    size_t b = 0;
    for (size_t k = 0; k < cb.size(); k++) {
        const uint64_t j = (uint64_t)k << FYB_COARSE;
        while (b + 1 < (size_t)nb && x[b + 1] <= j) b++;
        cb[k] = (uint32_t)b;
    }
    // H [nb][FYB_BLOCKS] lives in the perm buffer; the tables must fit in LDS
    if ((size_t)nb * FYB_BLOCKS > n || fyb_lds(nb, (int)cb.size()) > FYB_LDS_MAX) return hipSuccess;
    hipError_t e = hipMalloc((void **)&r.x, sizeof(uint32_t) * x.size());
    if (e == hipSuccess) e = hipMalloc((void **)&r.cb, sizeof(uint32_t) * cb.size());
    // k_fyb_bucket's range slices, counts and overflow flag (zero: the invariant between
    // permutations that k_fyb_link and k_fy_direct_block restore)
    const size_t nbs = x.size() - 1;
    if (e == hipSuccess) e = hipMalloc((void **)&r.P, sizeof(uint2) * nbs * FYB_CAP);
    if (e == hipSuccess) e = hipMalloc((void **)&r.cursor, sizeof(uint32_t) * (nbs + 1));
    if (e == hipSuccess) e = hipMemset(r.cursor, 0, sizeof(uint32_t) * (nbs + 1));
    r.flag = r.cursor ? r.cursor + nbs : nullptr;
    if (e == hipSuccess) e = hipMemcpy(r.x, x.data(), sizeof(uint32_t) * x.size(), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(r.cb, cb.data(), sizeof(uint32_t) * cb.size(), hipMemcpyHostToDevice);
    if (e != hipSuccess) { fy_ranges_free(r); return e; }
    r.nb = nb;
    r.ncb = (int)cb.size();
    return hipSuccess;
}

void fy_ranges_free(FyRanges &r) {
    if (r.x) (void)hipFree(r.x);
    if (r.cb) (void)hipFree(r.cb);
    if (r.P) (void)hipFree(r.P);
    if (r.cursor) (void)hipFree(r.cursor);
    r.x = r.cb = r.cursor = r.flag = nullptr;
    r.P = nullptr;
    r.nb = r.ncb = 0;
}

// scratch: 4n u32 (counts/pairs, buckets/pairs, succ, fw); scan: n/8192 + 2 u32; perm: n u32
hipError_t fisher_yates_device(const uint32_t *d_J, uint32_t n, uint32_t *scratch, uint32_t *scan, uint32_t *perm,
                               hipStream_t st, const FyRanges *rg, uint32_t *inv) {
    if (n == 0) return hipSuccess;
    uint32_t *cnt = scratch, *bucket = scratch + (size_t)n, *succ = scratch + 2 * (size_t)n,
             *fw = scratch + 3 * (size_t)n;
    uint32_t *off = perm;                // the direct path's offsets live in perm until the final pass
    const int grid = 2048;
    if (rg && rg->nb > 0 && rg->n == n) {
        const FyTab t{rg->x, rg->cb, rg->nb, rg->ncb};
        uint32_t *flag = rg->flag;
        const uint32_t chunk = (n + FYB_BLOCKS - 1) / FYB_BLOCKS;
        const size_t lds = fyb_lds(t.nb, t.ncb);
        static const bool fused = !(getenv("BPPO_FY_FUSED") && atoi(getenv("BPPO_FY_FUSED")) == 0);
        if (fused) {
            hipLaunchKernelGGL(k_fyb_bucket, dim3(FYB_BLOCKS), dim3(FYB_THREADS), lds, st, d_J, n, chunk, t,
                               rg->cursor, rg->P, flag);
            hipLaunchKernelGGL(k_fyb_link, dim3(t.nb), dim3(FYB_LINK_THREADS), 0, st, n, t, (const uint32_t *)nullptr,
                               FYB_BLOCKS, (const uint2 *)rg->P, succ, fw, flag, rg->cursor);
        } else {      // r05's passes (A/B): histogram, scan of the [range][block] counts, scatter
            uint32_t *H = perm;
            hipLaunchKernelGGL(k_fyb_hist, dim3(FYB_BLOCKS), dim3(FYB_THREADS), lds, st, d_J, n, chunk, t, H, flag);
            launch_scan(H, (uint32_t)t.nb * FYB_BLOCKS, scan, H, nullptr, st);
            hipLaunchKernelGGL(k_fyb_scatter, dim3(FYB_BLOCKS), dim3(FYB_THREADS), lds, st, d_J, n, chunk, t,
                               (const uint32_t *)H, reinterpret_cast<uint2 *>(scratch));
            hipLaunchKernelGGL(k_fyb_link, dim3(t.nb), dim3(FYB_LINK_THREADS), 0, st, n, t, (const uint32_t *)H,
                               FYB_BLOCKS, reinterpret_cast<const uint2 *>(scratch), succ, fw, flag, (uint32_t *)nullptr);
        }
        // pass 4 (k_fy_final) runs unless a range overflowed; then the one-block
        // direct pass computes the permutation instead
        hipLaunchKernelGGL(k_fy_final, dim3(grid), dim3(256), 0, st, d_J, n, (const uint32_t *)succ,
                           (const uint32_t *)fw, perm, (const uint32_t *)flag, inv);
        hipLaunchKernelGGL(k_fy_direct_block, dim3(1), dim3(FY_DIRECT_THREADS), 0, st, d_J, n, scratch, perm, flag, inv);
        return hipGetLastError();
    }
    // direct path
    hipLaunchKernelGGL(k_fy_zero, dim3(grid), dim3(256), 0, st, cnt, n, nullptr);
    hipLaunchKernelGGL(k_fy_count, dim3(grid), dim3(256), 0, st, d_J, n, cnt, nullptr);
    launch_scan(cnt, n, scan, off, nullptr, st);
    hipLaunchKernelGGL(k_fy_scatter, dim3(grid), dim3(256), 0, st, d_J, n, (const uint32_t *)off, cnt, bucket, nullptr);
    hipLaunchKernelGGL(k_fy_link, dim3(grid), dim3(256), 0, st, n, (const uint32_t *)off, bucket, succ, fw, nullptr);
    hipLaunchKernelGGL(k_fy_final, dim3(grid), dim3(256), 0, st, d_J, n, succ, fw, perm, nullptr, inv);
    return hipGetLastError();
}

bppo_status launch_fisher_yates(bppo_ctx *c, const uint32_t *d_J, uint32_t n) {
    BPPO_HIP(c, fisher_yates_device(d_J, n, c->d_fy, c->d_scan, c->d_perm, c->stream, &c->fyr, nullptr));
    return BPPO_OK;
}

}  // namespace bppo

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
// (i = 0 is treated as a self-swap J[0] = 0).  So: bucket the steps by target
// (counting sort), order each bucket, read succ/fw off neighbours, and follow
// fw chains (mean length ~1, max ~20 at n = 2^23).  Bit-exact; no host swaps.
#include "bppo_internal.h"

namespace bppo {

constexpr uint32_t FY_NONE = 0xFFFFFFFFu;
constexpr int SCAN_B = 1024;           // threads per scan block
constexpr int SCAN_IPT = 8;            // elements per thread
constexpr int SCAN_TILE = SCAN_B * SCAN_IPT;

__global__ void __launch_bounds__(256) k_fy_count(const uint32_t *J, uint32_t n, uint32_t *cnt) {
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

__global__ void __launch_bounds__(SCAN_B) k_scan_tiles(const uint32_t *in, uint32_t n, uint32_t *tile_sum) {
    __shared__ uint32_t sh[SCAN_B / 64];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_IPT;
    uint32_t s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_IPT; k++) s += base + k < n ? in[base + k] : 0u;
    uint32_t tot;
    (void)block_exclusive_u32(s, sh, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(SCAN_B) k_scan_sums(uint32_t *tile_sum, uint32_t ntiles) {
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

__global__ void __launch_bounds__(SCAN_B) k_scan_apply(const uint32_t *in, uint32_t n, const uint32_t *tile_pre,
                                                       uint32_t *out) {
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

// scatter step indices into their target's bucket (order inside a bucket fixed later)
__global__ void __launch_bounds__(256) k_fy_scatter(const uint32_t *J, uint32_t n, const uint32_t *off,
                                                    uint32_t *cnt, uint32_t *bucket) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint32_t j = J[i];
        const uint32_t k = atomicSub(&cnt[j], 1u) - 1u;
        bucket[off[j] + k] = i;
    }
}

// one thread per target j: sort its bucket, link successors, first writer fw(j)
__global__ void __launch_bounds__(256) k_fy_link(uint32_t n, const uint32_t *off, uint32_t *bucket,
                                                 uint32_t *succ, uint32_t *fw) {
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

__global__ void __launch_bounds__(256) k_fy_final(const uint32_t *J, uint32_t n, const uint32_t *succ,
                                                  const uint32_t *fw, uint32_t *perm) {
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
    }
}

// scratch: 4n u32 (counts, buckets, succ, fw); scan: n/8192 + 2 u32; perm: n u32
hipError_t fisher_yates_device(const uint32_t *d_J, uint32_t n, uint32_t *scratch, uint32_t *scan, uint32_t *perm,
                               hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint32_t *cnt = scratch, *bucket = scratch + (size_t)n, *succ = scratch + 2 * (size_t)n,
             *fw = scratch + 3 * (size_t)n;
    uint32_t *off = perm;                // the offsets live in perm until the final pass overwrites it
    const uint32_t ntiles = (n + SCAN_TILE - 1) / SCAN_TILE;
    const int grid = 2048;
    hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t) * n, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_fy_count, dim3(grid), dim3(256), 0, st, d_J, n, cnt);
    hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(SCAN_B), 0, st, cnt, n, scan);
    hipLaunchKernelGGL(k_scan_sums, dim3(1), dim3(SCAN_B), 0, st, scan, ntiles);
    hipLaunchKernelGGL(k_scan_apply, dim3(ntiles), dim3(SCAN_B), 0, st, cnt, n, scan, off);
    hipLaunchKernelGGL(k_fy_scatter, dim3(grid), dim3(256), 0, st, d_J, n, off, cnt, bucket);
    hipLaunchKernelGGL(k_fy_link, dim3(grid), dim3(256), 0, st, n, off, bucket, succ, fw);
    hipLaunchKernelGGL(k_fy_final, dim3(grid), dim3(256), 0, st, d_J, n, succ, fw, perm);
    return hipGetLastError();
}

bppo_status launch_fisher_yates(bppo_ctx *c, const uint32_t *d_J, uint32_t n) {
    BPPO_HIP(c, fisher_yates_device(d_J, n, c->d_fy, c->d_scan, c->d_perm, c->stream));
    return BPPO_OK;
}

}  // namespace bppo

// k_gemm.hip — f32 MFMA GEMM engine for the wide actor-critic MLPs
// (Connect Four 86->512->512->{7,1}, Liar's Dice CTDE actor 270->256->256->49 and
// critic 390->512->512->512->1; mlp.rs:140-206, ctde.rs:132-183).
//
// v_mfma_f32_32x32x2_f32 computes, per output element, a k-ordered fmaf chain
// (one rounding per product, MI355X guide §3 "FP32-input MFMA"), so a forward
// GEMM that walks k in order, restarting the chain at every KC=256 block and
// summing the block results into C, reproduces matrixmultiply 0.3's sgemm
// (oracle/net.c or_linear) bit for bit: the rollout forward, the bootstrap and
// the update forward all go through gemm_fwd, so the first-minibatch PPO ratio
// is exactly 1 (ppo.rs:1452) and the sampled actions match the reference.
//
// Three operand forms, one kernel template:
//   FWD  Y = act(X W + b)           X [M][K] row-major, W [K][N] (Burn Linear)
//   DX   dX = (dZ W^T) * [H > 0]    dZ [M][K=out], W [N=in][K=out]
//   WG   dW = X^T dZ (+ db = 1^T dZ) split over row chunks, partial slabs
//        reduced in a fixed order (deterministic, no float atomics).
// Block = 4 waves; wave tile = TM x TN accumulators of 32x32; LDS holds one
// BK=32 stage of A (k-major, padded row) and B (k-major) double-buffered, the
// next stage prefetched into registers while the MFMAs of the current run.
#include "bppo_internal.h"
#include "bppo_gemm.h"
#include <algorithm>
#include <type_traits>

namespace bppo {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GBK = 32;      // k per LDS stage
constexpr int KC = 256;      // matrixmultiply sgemm k-block

template <int BM, int BN, int WM, int WN>
struct GemmShape {
    static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
    static constexpr int APAD = BM + 1;             // k-major A rows, +1: conflict-free transposing writes
    static constexpr int BPAD = BN + 1;
    static constexpr int A_ELEMS = GBK * BM / 256;  // per thread per stage
    static constexpr int B_ELEMS = GBK * BN / 256;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(TM >= 1 && TN >= 1, "wave tile >= 32x32");
};

// operand element (row r of the tile's M/N side, k) -> global address
//   KCONTIG: element at base[r * ld + k]  (row-major, k contiguous)
//   else:    element at base[k * ld + r]  (k-major, r contiguous)
template <int R, bool KCONTIG>
// A stage's loads are unconditional (clamped addresses) and an element outside the operand
// is zeroed when the stage is stored, after the MFMAs that hide the loads: a guarded load
// (`ok ? base[i] : 0`) was turned into a branch around the load with a wait at its end --
// every element of the next stage fetched one round trip after the other
struct TileLoader {
    static constexpr int E = GBK * R / 256;
    static_assert(E <= 32, "one mask bit per element");
    float v[E];
    uint32_t ok = 0;
    __device__ __forceinline__ void load(const float *__restrict__ base, int ld, int r0, int rmax, int k0,
                                         int kmax, int tid) {
        ok = 0;
#pragma unroll
        for (int e = 0; e < E; e++) {
            int r, k;
            if constexpr (KCONTIG) { k = tid & 31; r = (tid >> 5) + e * 8; }
            else { r = tid % R; k = tid / R + e * (256 / R); }
            const int gr = r0 + r, gk = k0 + k;
            const int cr = min(gr, rmax - 1), ck = min(gk, kmax - 1);
            v[e] = base[(size_t)(KCONTIG ? cr : ck) * ld + (KCONTIG ? ck : cr)];
            ok |= (gr < rmax && gk < kmax) ? (1u << e) : 0u;
        }
    }
    __device__ __forceinline__ void store(float *__restrict__ s, int tid) const {
#pragma unroll
        for (int e = 0; e < E; e++) {
            int r, k;
            if constexpr (KCONTIG) { k = tid & 31; r = (tid >> 5) + e * 8; }
            else { r = tid % R; k = tid / R + e * (256 / R); }
            const int m = (int)(ok << (31 - e)) >> 31;                    // bit e -> 0 / all ones
            s[k * (R + 1) + r] = __int_as_float(__float_as_int(v[e]) & m);
        }
    }
};

// Implicit-GEMM convolution operands on Connect Four's 6 x 7 board (cnn.rs:204-215,
// connect_four.rs:217 OBSERVATION_SHAPE): the A operand is never materialised, each
// element is gathered from the NHWC activation rows (or the raw observation rows of
// layer 0) when its LDS stage is filled.
//   kind 1  im2col rows: element (row = b*42 + hw, k = (ci*ks + kh)*ks + kw) =
//           src(b, h + kh - pad, w + kw - pad, ci) or 0 -- the FWD A operand and the
//           WG X operand (X^T dY = dW), in the reference's patch order, so the FWD
//           chains are bit-identical to the im2col form;
//   kind 2  transposed taps: element (row, k = (kh*ks + kw)*C + c) =
//           dY(b, h - kh + pad, w - kw + pad, c) or 0 -- the DX A operand, so
//           dX = A W_d^T is the input gradient directly (no dA matrix, no col2im).
struct ConvA {
    int kind = 0;
    int cin = 0, ks = 1, pad = 0;   // channels of the gathered planes; kernel size; same padding
    int cpad = 0;                   // kind 2: k's per tap (cin rounded up to GBK; the rest read 0)
    int obs = 0, ld = 0;            // kind 1 layer 0: src = observation rows, row stride ld
};
constexpr int CV_H = 6, CV_W = 7, CV_HW = CV_H * CV_W;

// per thread: one fixed patch / tap index, a run of rows step apart
template <int R, bool KCONTIG>
struct ConvLoader {
    static constexpr int E = GBK * R / 256;
    float v[E];
    __device__ __forceinline__ void load(const float *__restrict__ src, const ConvA &cv, int r0, int rmax, int k0,
                                         int kmax, int tid) {
        int fixed, row, step;
        if constexpr (KCONTIG) { fixed = k0 + (tid & 31); row = r0 + (tid >> 5); step = 8; }
        else { fixed = r0 + tid % R; row = k0 + tid / R; step = 256 / R; }
        const bool fok = fixed < (KCONTIG ? kmax : rmax);
        const int rowmax = KCONTIG ? rmax : kmax;
        int ci, dh, dw;
        if (cv.kind == 1) {
            const int kk2 = cv.ks * cv.ks;
            ci = fixed / kk2;
            const int t = fixed - ci * kk2, kh = t / cv.ks;
            dh = kh - cv.pad; dw = t - kh * cv.ks - cv.pad;
        } else {
            const int tap = fixed / cv.cpad, kh = tap / cv.ks;
            ci = fixed - tap * cv.cpad;
            dh = cv.pad - kh; dw = cv.pad - (tap - kh * cv.ks);
        }
        const bool cok = ci < cv.cin;   // kind 2: a tap's padding channels read 0
        int b = row / CV_HW, hw = row - b * CV_HW;
#pragma unroll
        for (int e = 0; e < E; e++) {
            const int h = hw / CV_W + dh, w = hw % CV_W + dw;
            float x = 0.0f;
            if (fok && cok && row < rowmax && h >= 0 && h < CV_H && w >= 0 && w < CV_W) {
                const int hw2 = h * CV_W + w;
                x = cv.obs ? src[(size_t)b * cv.ld + hw2 * cv.cin + ci] : src[((size_t)b * CV_HW + hw2) * cv.cin + ci];
            }
            v[e] = x;
            row += step; hw += step;
            if (hw >= CV_HW) { hw -= CV_HW; b++; }
        }
    }
    __device__ __forceinline__ void store(float *__restrict__ s, int tid) const {
#pragma unroll
        for (int e = 0; e < E; e++) {
            int r, k;
            if constexpr (KCONTIG) { k = tid & 31; r = (tid >> 5) + e * 8; }
            else { r = tid % R; k = tid / R + e * (256 / R); }
            s[k * (R + 1) + r] = v[e];
        }
    }
};

struct GemmArgs {
    ConvA cv;                    // A operand: implicit convolution form (kind != 0)
    const float *A; int lda;
    const float *B; int ldb;
    int M, N, K;                 // C is M x N, reduction K
    // FWD epilogue
    const float *bias; int act;  // act: 1 relu, 0 none (tanh: none here + k_tanh_inplace)
    float *out0; int ld0; int n0;   // cols [0, n0) -> out0[row*ld0 + col]
    float *out1; int ld1;           // cols [n0, N) -> out1[row*ld1 + col - n0]
    // DX epilogue: activation derivative from the layer output H [M][ldh]
    // (nullptr: none): dact 1 relu mask [H > 0], 2 tanh (1 - H^2)
    const float *H; int ldh; int dact;
    // DX, exact shared heads: + round(xa[row * ldxa] * xw[col]) after the chain (the value
    // head's contribution added as the oracle / autodiff does: a separate rounded product)
    const float *xa; int ldxa; const float *xw;
    // DX of a convolution (AK = 2): the chain restarts every kblk k's (one tap's Co channels)
    // and the finished taps are summed in tap order (the col2im gather's f32 adds); 0: off
    int kblk;
    // WG: partial slab [split][M][N] and column sums [split][N]; rows of the
    // reduction per split (float, or double for k_gemm_wg64)
    float *part; float *colsum; int k_per_split;
    int xcd;                     // XCD-aware tile order (tile_of)
    int avec, bvec;              // k_gemm_split: operand 16-B aligned with ld % 4 == 0 (float4 loads)
};

enum { GEMM_FWD = 0, GEMM_DX = 1, GEMM_WG = 2 };

// XCD-aware tile order.  The hardware deals blocks round-robin over the 8 XCDs (block b on
// XCD b % 8), each with its own L2.  Dealt in grid order, the N-tiles of one row tile (which
// read the same A rows) land on different XCDs and every XCD fetches those rows from HBM.
// Remapped, XCD j runs the logical tiles [j T/8, (j+1) T/8): consecutive tiles -- the N-tiles
// of a row tile, the tiles of one split -- share an L2.  g.xcd = 0: grid order.
struct Tile { int x, y, z; };
__device__ __forceinline__ Tile tile_of(int xcd) {
    const unsigned gx = gridDim.x, gy = gridDim.y;
    const unsigned total = gx * gy * gridDim.z;
    unsigned b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    if (xcd && total % 8 == 0) b = (b % 8) * (total / 8) + b / 8;
    return Tile{(int)(b % gx), (int)((b / gx) % gy), (int)(b / (gx * gy))};
}

// ---- epilogue of a wave's TM x TN 32x32 accumulator tiles at (mw, nw): C/D map
// col = lane & 31, row = (q & 3) + 8 (q >> 2) + 4 (lane >> 5)
template <int MODE, int TM, int TN>
__device__ __forceinline__ void gemm_epilogue(const GemmArgs &g, const f32x16 (&acc)[TM][TN], const Tile &tl, int mw,
                                              int nw, int lane) {
    const int col_l = lane & 31, rq = 4 * (lane >> 5);
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int col = nw + j * 32 + col_l;
            // DX: the tile's H (and xa) values loaded first from clamped addresses, used
            // below -- loaded behind the per-element guard they compiled to a branch and a
            // wait per element (64 round trips per wave for a 64 x 64 wave tile)
            // (the empty asm statements keep the loads here: without them the compiler sinks
            // each one into its element's guarded store again)
            float hvs[16], xas[16], xwc = 0.0f;
            if constexpr (MODE == GEMM_DX) {
                const int cc = min(col, g.N - 1);
                if (g.H) {
#pragma unroll
                    for (int q = 0; q < 16; q++)
                        hvs[q] = g.H[(size_t)min(mw + i * 32 + (q & 3) + 8 * (q >> 2) + rq, g.M - 1) * g.ldh + cc];
#pragma unroll
                    for (int q = 0; q < 16; q++) asm volatile("" : "+v"(hvs[q]));
                }
                if (g.xa) {
#pragma unroll
                    for (int q = 0; q < 16; q++)
                        xas[q] = g.xa[(size_t)min(mw + i * 32 + (q & 3) + 8 * (q >> 2) + rq, g.M - 1) * g.ldxa];
                    xwc = g.xw[cc];
#pragma unroll
                    for (int q = 0; q < 16; q++) asm volatile("" : "+v"(xas[q]));
                    asm volatile("" : "+v"(xwc));
                }
            }
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const int row = mw + i * 32 + (q & 3) + 8 * (q >> 2) + rq;
                if (row >= g.M || col >= g.N) continue;
                float v = acc[i][j][q];
                if constexpr (MODE == GEMM_FWD) {
                    v = __fadd_rn(v, g.bias[col]);
                    if (g.act == 1) v = v > 0.0f ? v : 0.0f;
                    if (col < g.n0) g.out0[(size_t)row * g.ld0 + col] = v;
                    else g.out1[(size_t)row * g.ld1 + (col - g.n0)] = v;
                } else if constexpr (MODE == GEMM_DX) {
                    if (g.xa) v = __fadd_rn(v, __fmul_rn(xas[q], xwc));
                    if (g.H) {
                        const float hv = hvs[q];
                        if (g.dact == 2) v = __fmul_rn(v, __fsub_rn(1.0f, __fmul_rn(hv, hv)));
                        else if (!(hv > 0.0f)) v = 0.0f;
                    }
                    g.out0[(size_t)row * g.ld0 + col] = v;
                } else {
                    g.part[((size_t)tl.z * g.M + row) * g.N + col] = v;
                }
            }
        }
}

template <int MODE, int BM, int BN, int WM, int WN, int AK>
__global__ void __launch_bounds__(256, 2) k_gemm(GemmArgs g) {
    using S = GemmShape<BM, BN, WM, WN>;
    constexpr int TM_ = S::TM, TN_ = S::TN;
    constexpr bool A_KC = MODE != GEMM_WG;        // FWD/DX: A row-major [M][K]; WG: A = X^T, X [K][M]
    constexpr bool B_KC = MODE == GEMM_DX;        // FWD: W [K][N]; DX: W [N][K]; WG: dZ [K][N]
    __shared__ float sA[2][GBK * S::APAD];
    __shared__ float sB[2][GBK * S::BPAD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const Tile tl = tile_of(g.xcd);
    const int m0 = tl.y * BM, n0 = tl.x * BN;
    int kbeg = 0, kend = g.K;
    if constexpr (MODE == GEMM_WG) {
        kbeg = tl.z * g.k_per_split;
        kend = min(g.K, kbeg + g.k_per_split);
    }
    // A: a plain operand, or (AK) the implicit convolution form g.cv
    typename std::conditional<AK != 0, ConvLoader<BM, A_KC>, TileLoader<BM, A_KC>>::type la;
    TileLoader<BN, B_KC> lb;
    auto load_a = [&](int k) {
        if constexpr (AK != 0) la.load(g.A, g.cv, m0, g.M, k, kend, tid);
        else la.load(g.A, g.lda, m0, g.M, k, kend, tid);
    };
    f32x16 acc[S::TM][S::TN], tot[S::TM][S::TN];
#pragma unroll
    for (int i = 0; i < S::TM; i++)
#pragma unroll
        for (int j = 0; j < S::TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) { acc[i][j][r] = 0.0f; tot[i][j][r] = 0.0f; }
    // bias-gradient column sums (WG, first row tile only): 256/BN threads per column
    float csum = 0.0f;
    const bool do_colsum = MODE == GEMM_WG && g.colsum != nullptr && tl.y == 0;

    load_a(kbeg);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, tid);
    la.store(sA[0], tid);
    lb.store(sB[0], tid);
    __syncthreads();
    int buf = 0;
    for (int k0 = kbeg; k0 < kend; k0 += GBK) {
        const bool more = k0 + GBK < kend;
        if (more) {
            load_a(k0 + GBK);
            lb.load(g.B, g.ldb, n0, g.N, k0 + GBK, kend, tid);
        }
        if (do_colsum) {
            const int c = tid % BN, part = tid / BN, np = 256 / BN;
#pragma unroll 4
            for (int k = part; k < GBK; k += np) csum += sB[buf][k * S::BPAD + c];
        }
        const float *a = sA[buf], *b = sB[buf];
        const int h = lane >> 5, r = lane & 31;
#pragma unroll
        for (int kk = 0; kk < GBK; kk += 2) {
            float af[S::TM], bf[S::TN];
#pragma unroll
            for (int i = 0; i < S::TM; i++) af[i] = a[(kk + h) * S::APAD + (wm * S::TM + i) * 32 + r];
#pragma unroll
            for (int j = 0; j < S::TN; j++) bf[j] = b[(kk + h) * S::BPAD + (wn * S::TN + j) * 32 + r];
#pragma unroll
            for (int i = 0; i < S::TM; i++)
#pragma unroll
                for (int j = 0; j < S::TN; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if constexpr (MODE == GEMM_DX && AK == 2) {
            // conv input gradient: taps are padded to kblk (a multiple of GBK) k's, so a tap
            // ends at a stage boundary: its chain is complete, add it to the tap sum
            if (g.kblk > 0 && ((k0 + GBK) % g.kblk) == 0) {
#pragma unroll
                for (int i = 0; i < S::TM; i++)
#pragma unroll
                    for (int j = 0; j < S::TN; j++)
#pragma unroll
                        for (int q = 0; q < 16; q++) {
                            tot[i][j][q] = __fadd_rn(tot[i][j][q], acc[i][j][q]);
                            acc[i][j][q] = 0.0f;
                        }
            }
        }
        if constexpr (MODE == GEMM_FWD) {
            // matrixmultiply KC block boundary: the chain restarts from 0 and the
            // finished block is summed into C (first block stored as is)
            if (((k0 + GBK) % KC) == 0 && more) {
#pragma unroll
                for (int i = 0; i < S::TM; i++)
#pragma unroll
                    for (int j = 0; j < S::TN; j++)
#pragma unroll
                        for (int q = 0; q < 16; q++) {
                            tot[i][j][q] = (k0 + GBK == KC) ? acc[i][j][q] : __fadd_rn(tot[i][j][q], acc[i][j][q]);
                            acc[i][j][q] = 0.0f;
                        }
            }
        }
        if (more) {
            __syncthreads();          // everyone done reading buf^1 (two stages ago)
            la.store(sA[buf ^ 1], tid);
            lb.store(sB[buf ^ 1], tid);
            __syncthreads();
            buf ^= 1;
        }
    }
    if constexpr (MODE == GEMM_FWD) {
        if (g.K > KC) {
#pragma unroll
            for (int i = 0; i < S::TM; i++)
#pragma unroll
                for (int j = 0; j < S::TN; j++)
#pragma unroll
                    for (int q = 0; q < 16; q++) acc[i][j][q] = __fadd_rn(tot[i][j][q], acc[i][j][q]);
        }
    }
    if constexpr (MODE == GEMM_DX && AK == 2) {
        if (g.kblk > 0) {        // every tap flushed (K is a multiple of kblk): the tap sum
#pragma unroll
            for (int i = 0; i < S::TM; i++)
#pragma unroll
                for (int j = 0; j < S::TN; j++)
#pragma unroll
                    for (int q = 0; q < 16; q++) acc[i][j][q] = __fadd_rn(tot[i][j][q], acc[i][j][q]);
        }
    }
    gemm_epilogue<MODE, TM_, TN_>(g, acc, tl, m0 + wm * S::TM * 32, n0 + wn * S::TN * 32, lane);
    if (do_colsum) {
        __shared__ float red[256];
        red[tid] = csum;
        __syncthreads();
        if (tid < BN) {
            float s = 0.0f;
            for (int p = 0; p < 256 / BN; p++) s += red[tid + p * BN];
            const int col = n0 + tid;
            if (col < g.N) g.colsum[(size_t)tl.z * g.N + col] = s;
        }
    }
}

// ---- split-bf16 contraction (every update minibatch after the first) -----------------
// The forward, input-gradient and weight-gradient GEMMs of the update's later minibatches
// need f32 ACCURACY, not the reference's rounding: their parameters already differ from
// the reference's in the last bits after the first Adam step (the first minibatch keeps
// the exact k_gemm chains: ratio exactly 1).  Each f32 operand is split exactly into three
// bf16 pieces x = x0 + x1 + x2 (8 significand bits each, round-to-nearest) when its LDS
// stage is filled -- once per block, not per wave -- and the six products of order <= 2
// (x2y0, x1y1, x0y2, x1y0, x0y1, x0y0, smallest first) accumulate in f32 on
// v_mfma_f32_32x32x16_bf16: |x1| <= 2^-8 |x|, |x2| <= 2^-16 |x|, so the dropped products
// are within (2^-23 + 2^-32) |xy| (tests/test_split_bf16.py), and 6 MFMAs of 32 cycles do
// the work of 8 f32 MFMAs of 64 cycles (2.7x the f32 MFMA rate; MI355X guide: 32x32x16
// bf16 = 16x the f32 rate per FLOP).
// LDS: the three piece images of A [BM][KP] and B [BN][KP] for one GBK = 32 stage, k
// contiguous (one ds_read_b128 per 8-k fragment), row stride KP = 40 bf16 (80 B: the 32
// rows of a fragment read hit distinct bank groups); one stage (60 KB at 128 x 128, two
// blocks per CU), the next stage's f32 values prefetched into registers under the MFMAs.
typedef __bf16 sbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 sbf16x2 __attribute__((ext_vector_type(2)));
constexpr int SKP = GBK + 8;

// three pieces of Q consecutive-k values -> LDS rows at s[p * plane + off].  (A pair-wise
// form -- one v_cvt_pk_bf16_f32 per piece pair, the halves read back from the packed word
// through an opaque asm -- ran the CfgC update 151-166 ms against 143 ms for this one:
// profiles/r05c/split_store_ab.txt)
typedef __bf16 sbf16x4 __attribute__((ext_vector_type(4)));
template <int Q>
__device__ __forceinline__ void split_store(const float *x, __bf16 *s, int plane, int off) {
    __bf16 p0[Q], p1[Q], p2[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) {
        const __bf16 a = (__bf16)x[j];
        const float r = x[j] - (float)a;
        const __bf16 b = (__bf16)r;
        p0[j] = a; p1[j] = b; p2[j] = (__bf16)(r - (float)b);
    }
    if constexpr (Q == 4) {
        *reinterpret_cast<sbf16x4 *>(s + off) = sbf16x4{p0[0], p0[1], p0[2], p0[3]};
        *reinterpret_cast<sbf16x4 *>(s + plane + off) = sbf16x4{p1[0], p1[1], p1[2], p1[3]};
        *reinterpret_cast<sbf16x4 *>(s + 2 * plane + off) = sbf16x4{p2[0], p2[1], p2[2], p2[3]};
    } else if constexpr (Q == 2) {
        *reinterpret_cast<sbf16x2 *>(s + off) = sbf16x2{p0[0], p0[1]};
        *reinterpret_cast<sbf16x2 *>(s + plane + off) = sbf16x2{p1[0], p1[1]};
        *reinterpret_cast<sbf16x2 *>(s + 2 * plane + off) = sbf16x2{p2[0], p2[1]};
    } else {
        s[off] = p0[0]; s[plane + off] = p1[0]; s[2 * plane + off] = p2[0];
    }
}

// four consecutive elements of a row of `base` from `idx` (bounded by `lim`): one float4
// when the operand is aligned (vec) and the quad is whole, else guarded scalars
__device__ __forceinline__ void load4(const float *__restrict__ base, size_t row_off, int idx, int lim, bool vec,
                                      bool row_ok, float (&v)[4]) {
    if (row_ok && vec && idx + 3 < lim) {
        const float4 q = *reinterpret_cast<const float4 *>(base + row_off + idx);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
#pragma unroll
        for (int u = 0; u < 4; u++) v[u] = (row_ok && idx + u < lim) ? base[row_off + idx + u] : 0.0f;
    }
}


// one operand's GBK x R stage.  KCONTIG (element (r, k) at base[r ld + k]): thread -> rows
// (tid >> 3) + 32 e, k quad (tid & 7) * 4.  k-major (element at base[k ld + r]): thread ->
// KQ consecutive k (KQ = 4, 2, 1 for R = 128, 64, 32) times an r quad, so each piece row
// segment it writes is KQ contiguous k's.
template <int R, bool KCONTIG>
struct SplitLoader {
    static constexpr int E = GBK * R / 256;            // elements per thread
    static constexpr int KQ = KCONTIG ? 4 : E / 4;     // consecutive k per piece write
    static constexpr int NKB = GBK / KQ;               // k-major: k blocks per r quad
    float v[E];
    __device__ __forceinline__ void load(const float *__restrict__ base, int ld, int r0, int rmax, int k0, int kmax,
                                         int tid, bool vec) {
        if constexpr (KCONTIG) {
#pragma unroll
            for (int e = 0; e < E / 4; e++) {
                const int r = r0 + (tid >> 3) + 32 * e, k = k0 + (tid & 7) * 4;
                float q[4];
                load4(base, (size_t)r * ld, k, kmax, vec, r < rmax, q);
#pragma unroll
                for (int u = 0; u < 4; u++) v[4 * e + u] = q[u];
            }
        } else {
            const int kb = (tid % NKB) * KQ, r4 = (tid / NKB) * 4;
#pragma unroll
            for (int j = 0; j < KQ; j++) {
                const int k = k0 + kb + j;
                float q[4];
                load4(base, (size_t)k * ld, r0 + r4, rmax, vec, k < kmax, q);
#pragma unroll
                for (int u = 0; u < 4; u++) v[4 * j + u] = q[u];
            }
        }
    }
    // pieces into s (three planes of R * SKP)
    __device__ __forceinline__ void store(__bf16 *s, int tid) const {
        constexpr int plane = R * SKP;
        if constexpr (KCONTIG) {
#pragma unroll
            for (int e = 0; e < E / 4; e++)
                split_store<4>(v + 4 * e, s, plane, ((tid >> 3) + 32 * e) * SKP + (tid & 7) * 4);
        } else {
            const int kb = (tid % NKB) * KQ, r4 = (tid / NKB) * 4;
#pragma unroll
            for (int u = 0; u < 4; u++) {
                float x[KQ];
#pragma unroll
                for (int j = 0; j < KQ; j++) x[j] = v[4 * j + u];
                split_store<KQ>(x, s, plane, (r4 + u) * SKP + kb);
            }
        }
    }
    // k-major: column sums of this thread's KQ k's per r (the bias gradient of WG's B)
    __device__ __forceinline__ void colsum(float (&cs)[4]) const {
        if constexpr (!KCONTIG) {
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int j = 0; j < KQ; j++) cs[u] += v[4 * j + u];
        }
    }
};

__device__ __forceinline__ void mfma6_split(f32x16 &acc, const sbf16x8 (&a)[3], const sbf16x8 (&b)[3]) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

template <int MODE, int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(256, 2) k_gemm_split(GemmArgs g) {
    using S = GemmShape<BM, BN, WM, WN>;
    constexpr bool A_KC = MODE != GEMM_WG;
    constexpr bool B_KC = MODE == GEMM_DX;
    __shared__ __attribute__((aligned(16))) __bf16 sA[3 * BM * SKP];
    __shared__ __attribute__((aligned(16))) __bf16 sB[3 * BN * SKP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const Tile tl = tile_of(g.xcd);
    const int m0 = tl.y * BM, n0 = tl.x * BN;
    int kbeg = 0, kend = g.K;
    if constexpr (MODE == GEMM_WG) {
        kbeg = tl.z * g.k_per_split;
        kend = min(g.K, kbeg + g.k_per_split);
    }
    SplitLoader<BM, A_KC> la;
    SplitLoader<BN, B_KC> lb;
    f32x16 acc[S::TM][S::TN];
#pragma unroll
    for (int i = 0; i < S::TM; i++)
#pragma unroll
        for (int j = 0; j < S::TN; j++)
#pragma unroll
            for (int r = 0; r < 16; r++) acc[i][j][r] = 0.0f;
    float cs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const bool do_colsum = MODE == GEMM_WG && g.colsum != nullptr && tl.y == 0;
    const int r = lane & 31, h = lane >> 5;

    la.load(g.A, g.lda, m0, g.M, kbeg, kend, tid, g.avec);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, tid, g.bvec);
    for (int k0 = kbeg; k0 < kend; k0 += GBK) {
        if (k0 != kbeg) __syncthreads();          // every wave done reading the previous stage
        la.store(sA, tid);
        lb.store(sB, tid);
        if (do_colsum) lb.colsum(cs);
        __syncthreads();
        if (k0 + GBK < kend) {                    // the next stage's values, in flight under the MFMAs
            la.load(g.A, g.lda, m0, g.M, k0 + GBK, kend, tid, g.avec);
            lb.load(g.B, g.ldb, n0, g.N, k0 + GBK, kend, tid, g.bvec);
        }
#pragma unroll
        for (int kk = 0; kk < GBK; kk += 16) {
            sbf16x8 af[S::TM][3], bf[S::TN][3];
#pragma unroll
            for (int i = 0; i < S::TM; i++)
#pragma unroll
                for (int p = 0; p < 3; p++)
                    af[i][p] = *reinterpret_cast<const sbf16x8 *>(sA + p * BM * SKP + ((wm * S::TM + i) * 32 + r) * SKP + kk + 8 * h);
#pragma unroll
            for (int j = 0; j < S::TN; j++)
#pragma unroll
                for (int p = 0; p < 3; p++)
                    bf[j][p] = *reinterpret_cast<const sbf16x8 *>(sB + p * BN * SKP + ((wn * S::TN + j) * 32 + r) * SKP + kk + 8 * h);
            // each 16-deep step's six products into a fresh partial, added to the running sum
            // with a round-to-nearest f32 add (the MFMA's own accumulation then spans 16 k's)
#pragma unroll
            for (int i = 0; i < S::TM; i++)
#pragma unroll
                for (int j = 0; j < S::TN; j++) {
                    f32x16 part;
#pragma unroll
                    for (int q = 0; q < 16; q++) part[q] = 0.0f;
                    mfma6_split(part, af[i], bf[j]);
#pragma unroll
                    for (int q = 0; q < 16; q++) acc[i][j][q] = __fadd_rn(acc[i][j][q], part[q]);
                }
        }
    }
    gemm_epilogue<MODE, S::TM, S::TN>(g, acc, tl, m0 + wm * S::TM * 32, n0 + wn * S::TN * 32, lane);
    if (do_colsum) {
        // the NKB threads of an r quad are consecutive lanes of one wave
        constexpr int NKB = SplitLoader<BN, false>::NKB;
#pragma unroll
        for (int u = 0; u < 4; u++)
#pragma unroll
            for (int o = 1; o < NKB; o <<= 1) cs[u] += __shfl_xor(cs[u], o, 64);
        if (tid % NKB == 0) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int col = n0 + (tid / NKB) * 4 + u;
                if (col < g.N) g.colsum[(size_t)tl.z * g.N + col] = cs[u];
            }
        }
    }
}

// ---- exact weight gradients: dW = X^T dZ on v_mfma_f64_16x16x4_f64 --------------
// The oracle (and autodiff in f64) sums x * dz over the rows in f64: every product of
// two f32 values is exact in f64, so the only rounding left is the f64 additions, and
// the f32 result equals the oracle's except in the ~2^-29-rare case of an f64 sum within
// its ordering error of an f32 rounding boundary.  The f32 MFMA accumulates in f32 over
// each split's rows (tens of thousands for a conv layer): its last-bit differences, fed
// through Adam, move the parameters off the oracle's by ~1 ulp, which the PPO loss then
// amplifies (tests/test_gpu_cnn.py).  Same LDS staging and loaders as k_gemm (WG form:
// A = X^T k-major, B = dZ k-major), f64 operands converted from the staged f32 values,
// 16x16 f64 tiles (f64 C/D map: col = lane & 15, row = (lane >> 4) + 4 reg), f64
// partial slabs [split][M][N] and f64 column sums, reduced in f64 and rounded once.
typedef double f64x4 __attribute__((ext_vector_type(4)));
template <int BM, int BN, int AK>
__global__ void __launch_bounds__(256, 2) k_gemm_wg64(GemmArgs g) {
    constexpr int WM = 2, WN = 2, TM = BM / WM / 16, TN = BN / WN / 16;
    constexpr int APAD = BM + 1, BPAD = BN + 1;
    static_assert(TM >= 1 && TN >= 1, "wave tile >= 16x16");
    __shared__ float sA[2][GBK * APAD];
    __shared__ float sB[2][GBK * BPAD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    const Tile tl = tile_of(g.xcd);
    const int m0 = tl.y * BM, n0 = tl.x * BN;
    const int kbeg = tl.z * g.k_per_split, kend = min(g.K, kbeg + g.k_per_split);
    typename std::conditional<AK != 0, ConvLoader<BM, false>, TileLoader<BM, false>>::type la;
    TileLoader<BN, false> lb;
    auto load_a = [&](int k) {
        if constexpr (AK != 0) la.load(g.A, g.cv, m0, g.M, k, kend, tid);
        else la.load(g.A, g.lda, m0, g.M, k, kend, tid);
    };
    f64x4 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
#pragma unroll
            for (int r = 0; r < 4; r++) acc[i][j][r] = 0.0;
    double csum = 0.0;
    const bool do_colsum = g.colsum != nullptr && tl.y == 0;
    load_a(kbeg);
    lb.load(g.B, g.ldb, n0, g.N, kbeg, kend, tid);
    la.store(sA[0], tid);
    lb.store(sB[0], tid);
    __syncthreads();
    int buf = 0;
    const int li = lane & 15, lk = lane >> 4;
    for (int k0 = kbeg; k0 < kend; k0 += GBK) {
        const bool more = k0 + GBK < kend;
        if (more) {
            load_a(k0 + GBK);
            lb.load(g.B, g.ldb, n0, g.N, k0 + GBK, kend, tid);
        }
        if (do_colsum) {
            const int c = tid % BN, part = tid / BN, np = 256 / BN;
#pragma unroll 4
            for (int k = part; k < GBK; k += np) csum += (double)sB[buf][k * BPAD + c];
        }
        const float *a = sA[buf], *b = sB[buf];
#pragma unroll
        for (int kk = 0; kk < GBK; kk += 4) {
            double af[TM], bf[TN];
#pragma unroll
            for (int i = 0; i < TM; i++) af[i] = (double)a[(kk + lk) * APAD + (wm * TM + i) * 16 + li];
#pragma unroll
            for (int j = 0; j < TN; j++) bf[j] = (double)b[(kk + lk) * BPAD + (wn * TN + j) * 16 + li];
#pragma unroll
            for (int i = 0; i < TM; i++)
#pragma unroll
                for (int j = 0; j < TN; j++)
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(af[i], bf[j], acc[i][j], 0, 0, 0);
        }
        if (more) {
            __syncthreads();
            la.store(sA[buf ^ 1], tid);
            lb.store(sB[buf ^ 1], tid);
            __syncthreads();
            buf ^= 1;
        }
    }
    double *part = reinterpret_cast<double *>(g.part);
#pragma unroll
    for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++) {
            const int col = n0 + (wn * TN + j) * 16 + li;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int row = m0 + (wm * TM + i) * 16 + lk + 4 * r;
                if (row < g.M && col < g.N) part[((size_t)tl.z * g.M + row) * g.N + col] = acc[i][j][r];
            }
        }
    if (do_colsum) {
        __shared__ double red[256];
        red[tid] = csum;
        __syncthreads();
        if (tid < BN) {
            double s = 0.0;
            for (int p = 0; p < 256 / BN; p++) s += red[tid + p * BN];
            const int col = n0 + tid;
            if (col < g.N) reinterpret_cast<double *>(g.colsum)[(size_t)tl.z * g.N + col] = s;
        }
    }
}

// ---- reference-exact weight gradients (bppo_set_minibatch_kernel 1) --------------------
// dW[k][o] = sum over the rows r IN ORDER of (double)X[r][k] * (double)dZ[r][o], one thread
// per (k, o), rounded to f32 once: the oracle's linear_bwd loop (oracle/net.c) bit for bit
// (each product of two f32 values is exact in f64, so the sequence of f64 additions is the
// whole arithmetic).  Latency-bound (one dependent f64 add per row per thread): a parity
// mode, for the sizes the tests run.  Threads of a wave take consecutive o (coalesced dZ
// reads, the X element shared); column sums (bias gradients) the same way.
struct SeqWg {
    ConvA cv;
    const float *X; int ldx;       // X [rows][Kin] (or the implicit im2col form cv)
    const float *dZ; int ldz;      // dZ [rows][N]
    int Kin, N, rows;
    float *dW0; int ldw0; int n0;  // cols [0, n0) -> dW0 [Kin][ldw0], [n0, N) -> dW1 [Kin][ldw1]
    float *dW1; int ldw1;
    float *db0, *db1;              // column sums likewise (may be null)
};
__device__ __forceinline__ float conv_x(const ConvA &cv, const float *src, int row, int k) {
    const int kk2 = cv.ks * cv.ks, ci = k / kk2, t = k - ci * kk2, kh = t / cv.ks;
    const int b = row / CV_HW, hw = row - b * CV_HW;
    const int h = hw / CV_W + kh - cv.pad, w = hw % CV_W + (t - kh * cv.ks) - cv.pad;
    if (h < 0 || h >= CV_H || w < 0 || w >= CV_W) return 0.0f;
    const int hw2 = h * CV_W + w;
    return cv.obs ? src[(size_t)b * cv.ld + hw2 * cv.cin + ci] : src[((size_t)b * CV_HW + hw2) * cv.cin + ci];
}
__global__ void __launch_bounds__(256) k_wg_seq(SeqWg a) {
    const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    const size_t nw = (size_t)a.Kin * a.N;
    if (t >= nw + (size_t)((a.db0 || a.db1) ? a.N : 0)) return;
    const bool bias = t >= nw;
    const int k = bias ? 0 : (int)(t / a.N), o = (int)(bias ? t - nw : t % a.N);
    double s = 0.0;
    if (bias) {
        for (int r = 0; r < a.rows; r++) s += (double)a.dZ[(size_t)r * a.ldz + o];
    } else if (a.cv.kind) {
        for (int r = 0; r < a.rows; r++) s += (double)conv_x(a.cv, a.X, r, k) * (double)a.dZ[(size_t)r * a.ldz + o];
    } else {
        for (int r = 0; r < a.rows; r++) s += (double)a.X[(size_t)r * a.ldx + k] * (double)a.dZ[(size_t)r * a.ldz + o];
    }
    if (bias) {
        float *d = o < a.n0 ? a.db0 : a.db1;
        if (d) d[o < a.n0 ? o : o - a.n0] = (float)s;
    } else if (o < a.n0) a.dW0[(size_t)k * a.ldw0 + o] = (float)s;
    else a.dW1[(size_t)k * a.ldw1 + (o - a.n0)] = (float)s;
}

// the f64 partials in split order, rounded to f32 once
// the partials' loads issued SPLIT_UNROLL at a time ahead of the (unchanged, k-ordered)
// adds: the plain loop waited on every load in turn (58 us per CfgC weight-gradient reduce
// of 128 splits, latency-bound)
constexpr int SPLIT_UNROLL = 16;
template <typename T>
__device__ __forceinline__ double split_sum(const T *__restrict__ part, int splits, size_t MN, size_t i) {
    double s = 0.0;
    int k = 0;
    for (; k + SPLIT_UNROLL <= splits; k += SPLIT_UNROLL) {
        T v[SPLIT_UNROLL];
#pragma unroll
        for (int u = 0; u < SPLIT_UNROLL; u++) v[u] = part[(size_t)(k + u) * MN + i];
#pragma unroll
        for (int u = 0; u < SPLIT_UNROLL; u++) s += (double)v[u];
    }
    for (; k < splits; k++) s += (double)part[(size_t)k * MN + i];
    return s;
}
__global__ void k_split_reduce64(const double *__restrict__ part, int splits, int M, int N, int n0,
                                 float *out0, int ld0, float *out1, int ld1) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= (size_t)M * N) return;
    const double s = split_sum(part, splits, (size_t)M * N, i);
    const int r = (int)(i / N), c = (int)(i % N);
    if (c < n0) out0[(size_t)r * ld0 + c] = (float)s;
    else out1[(size_t)r * ld1 + (c - n0)] = (float)s;
}

// fixed-order sum of the split partials: dst[r][c] = sum_s part[s][r][c] (f64),
// written to out0 for c < n0 and out1 (ld1) otherwise; scale applied at the end
__global__ void k_split_reduce(const float *__restrict__ part, int splits, int M, int N, int n0,
                               float *out0, int ld0, float *out1, int ld1) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= (size_t)M * N) return;
    const double s = split_sum(part, splits, (size_t)M * N, i);
    const int r = (int)(i / N), c = (int)(i % N);
    if (c < n0) out0[(size_t)r * ld0 + c] = (float)s;
    else out1[(size_t)r * ld1 + (c - n0)] = (float)s;
}

// tanh activation of a FWD output block [M][cols] (ld), in place: the
// elementwise pass after the GEMM (mlp.rs:187-191 -> glibc tanhf, restated
// bit-exactly in bppo_math.h).  HBM-bound: 8 B per element.
__global__ void __launch_bounds__(256) k_tanh_inplace(float *__restrict__ y, int M, int cols, int ld) {
    const size_t n = (size_t)M * cols;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const size_t r = i / cols, c = i % cols;
        float *p = y + r * ld + c;
        *p = bppo_math::tanhf_glibc_bf(*p);
    }
}
static hipError_t tanh_inplace(hipStream_t st, float *y, int M, int cols, int ld) {
    if (M <= 0 || cols <= 0) return hipSuccess;
    const size_t n = (size_t)M * cols;
    const unsigned blocks = (unsigned)std::min<size_t>((n + 255) / 256, 8192);
    hipLaunchKernelGGL(k_tanh_inplace, dim3(blocks), dim3(256), 0, st, y, M, cols, ld);
    return hipGetLastError();
}

// -------------------------------------------------------------- launchers --
// BPPO_GEMM_XCD=0: grid-order tiles (A/B of the XCD-aware order)
static int gemm_xcd() {
    static const int v = getenv("BPPO_GEMM_XCD") ? atoi(getenv("BPPO_GEMM_XCD")) : 1;
    return v;
}
template <int MODE, int BM, int BN, int WM, int WN, int AK>
static hipError_t launch(GemmArgs g, int splits, hipStream_t st) {
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, splits);
    g.xcd = gemm_xcd();
    hipLaunchKernelGGL((k_gemm<MODE, BM, BN, WM, WN, AK>), grid, dim3(256), 0, st, g);
    return hipGetLastError();
}

static bool vec_ok(const float *p, int ld) { return ((uintptr_t)p & 15) == 0 && (ld & 3) == 0; }
template <int MODE, int BM, int BN, int WM, int WN>
static hipError_t launch_split(GemmArgs g, int splits, hipStream_t st) {
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, splits);
    g.xcd = gemm_xcd();
    g.avec = vec_ok(g.A, g.lda); g.bvec = vec_ok(g.B, g.ldb);
    hipLaunchKernelGGL((k_gemm_split<MODE, BM, BN, WM, WN>), grid, dim3(256), 0, st, g);
    return hipGetLastError();
}
template <int MODE>
static hipError_t launch_split_by_width(const GemmArgs &g, int splits, hipStream_t st) {
    if (g.N <= 32) return launch_split<MODE, 128, 32, 4, 1>(g, splits, st);
    if (g.N <= 64) return launch_split<MODE, 128, 64, 4, 1>(g, splits, st);
    return launch_split<MODE, 128, 128, 2, 2>(g, splits, st);
}

template <int BM, int BN, int AK>
static hipError_t launch64(GemmArgs g, int splits, hipStream_t st) {
    dim3 grid((g.N + BN - 1) / BN, (g.M + BM - 1) / BM, splits);
    g.xcd = gemm_xcd();
    hipLaunchKernelGGL((k_gemm_wg64<BM, BN, AK>), grid, dim3(256), 0, st, g);
    return hipGetLastError();
}
// the same output tiling as launch_by_width, so gemm_wg_splits holds for both
template <int AK = 0>
static hipError_t launch64_by_width(const GemmArgs &g, int splits, hipStream_t st) {
    if (g.N <= 32) return launch64<128, 32, AK>(g, splits, st);
    if (g.N <= 64) return launch64<128, 64, AK>(g, splits, st);
    return launch64<128, 128, AK>(g, splits, st);
}

template <int MODE, int AK = 0>
static hipError_t launch_by_width(const GemmArgs &g, int splits, hipStream_t st) {
    if (g.N <= 32) return launch<MODE, 128, 32, 4, 1, AK>(g, splits, st);
    if (g.N <= 64) return launch<MODE, 128, 64, 4, 1, AK>(g, splits, st);
    return launch<MODE, 128, 128, 2, 2, AK>(g, splits, st);
}

hipError_t gemm_fwd(hipStream_t st, int M, int N, int K, const float *X, int ldx, const float *W,
                    int ldw, const float *bias, int act, float *out0, int ld0, int n0, float *out1,
                    int ld1, int split) {
    if (M <= 0 || N <= 0) return hipSuccess;
    GemmArgs g{};
    g.A = X; g.lda = ldx; g.B = W; g.ldb = ldw; g.M = M; g.N = N; g.K = K;
    g.bias = bias; g.act = act == 1 ? 1 : 0;
    g.out0 = out0; g.ld0 = ld0; g.n0 = out1 ? n0 : N; g.out1 = out1; g.ld1 = ld1;
    hipError_t e = split ? launch_split_by_width<GEMM_FWD>(g, 1, st) : launch_by_width<GEMM_FWD>(g, 1, st);
    if (e != hipSuccess || act != 2) return e;
    if ((e = tanh_inplace(st, out0, M, g.n0, ld0)) != hipSuccess) return e;
    return out1 ? tanh_inplace(st, out1, M, N - g.n0, ld1) : hipSuccess;
}

// conv layer forward (implicit im2col): Y [rows*42][Co] = relu(A(src) Wt + bias)
hipError_t gemm_conv_fwd(hipStream_t st, int rows, int Co, int Cin, int ks, const float *src, int obs_ld,
                         const float *Wt, const float *bias, float *out) {
    if (rows <= 0 || Co <= 0) return hipSuccess;
    GemmArgs g{};
    g.cv.kind = 1; g.cv.cin = Cin; g.cv.ks = ks; g.cv.pad = ks / 2; g.cv.obs = obs_ld > 0; g.cv.ld = obs_ld;
    g.A = src; g.B = Wt; g.ldb = Co; g.M = rows * CV_HW; g.N = Co; g.K = Cin * ks * ks;
    g.bias = bias; g.act = 1;
    g.out0 = out; g.ld0 = Co; g.n0 = Co;
    return launch_by_width<GEMM_FWD, 1>(g, 1, st);
}

// conv input gradient (transposed taps): dX [rows*42][Cin] = (A_t(dY) Wd^T) * [H > 0],
// Wd [Cin][ks*ks*cpad] with Wd[ci][(kh*ks + kw)*cpad + co] = weight[co][ci][kh][kw] (zero for
// co >= Co), cpad = gemm_conv_tap_pad(Co).  Each tap's chain over its channels is finished
// and added to the tap sum in (kh, kw) order -- the oracle's per-tap dA chains and col2im
// adds, bit for bit (the zero padding leaves a chain unchanged: fma(0, w, a) = a).
int gemm_conv_tap_pad(int Co) { return (Co + GBK - 1) / GBK * GBK; }
hipError_t gemm_conv_dx(hipStream_t st, int rows, int Cin, int Co, int ks, const float *dY, const float *Wd,
                        const float *H, float *out) {
    if (rows <= 0 || Cin <= 0) return hipSuccess;
    const int cpad = gemm_conv_tap_pad(Co);
    GemmArgs g{};
    g.cv.kind = 2; g.cv.cin = Co; g.cv.ks = ks; g.cv.pad = ks / 2; g.cv.cpad = cpad;
    g.A = dY; g.B = Wd; g.ldb = ks * ks * cpad; g.M = rows * CV_HW; g.N = Cin; g.K = ks * ks * cpad;
    g.H = H; g.ldh = Cin; g.dact = 1; g.out0 = out; g.ld0 = Cin; g.n0 = Cin;
    g.kblk = cpad;
    return launch_by_width<GEMM_DX, 2>(g, 1, st);
}

hipError_t gemm_dx(hipStream_t st, int M, int N, int K, const float *dZ, int ldz, const float *W,
                   int ldw, const float *H, int ldh, int act, float *out, int ldo, const float *xa, int ldxa,
                   const float *xw, int split) {
    if (M <= 0 || N <= 0) return hipSuccess;
    GemmArgs g{};
    g.A = dZ; g.lda = ldz; g.B = W; g.ldb = ldw; g.M = M; g.N = N; g.K = K;
    g.H = H; g.ldh = ldh; g.dact = act == 2 ? 2 : 1; g.out0 = out; g.ld0 = ldo; g.n0 = N;
    g.xa = xa; g.ldxa = ldxa; g.xw = xw;
    return split ? launch_split_by_width<GEMM_DX>(g, 1, st) : launch_by_width<GEMM_DX>(g, 1, st);
}

int gemm_wg_splits(int Kin, int N, int rows) {
    const int tiles = ((Kin + 127) / 128) * ((N + (N <= 32 ? 31 : N <= 64 ? 63 : 127)) / (N <= 32 ? 32 : N <= 64 ? 64 : 128));
    // ~2048 blocks (BPPO_WG_BLOCKS: another target, for A/B runs of the slab traffic)
    static const int target = getenv("BPPO_WG_BLOCKS") ? std::max(1, atoi(getenv("BPPO_WG_BLOCKS"))) : 2048;
    int s = (target + tiles - 1) / tiles;
    const int max_by_rows = (rows + 1023) / 1024;        // >= 1024 rows per split
    if (s > max_by_rows) s = max_by_rows;
    if (s > GEMM_MAX_SPLITS) s = GEMM_MAX_SPLITS;
    if (s < 1) s = 1;
    return s;
}

static hipError_t wgrad(hipStream_t st, const ConvA &cv, int Kin, int N, int rows, const float *X, int ldx,
                        const float *dZ, int ldz, float *part, float *colsum, float *dW0, int ldw0, int n0,
                        float *dW1, int ldw1, float *db0, float *db1, int splits, int exact);

hipError_t gemm_wgrad(hipStream_t st, int Kin, int N, int rows, const float *X, int ldx, const float *dZ,
                      int ldz, float *part, float *colsum, float *dW0, int ldw0, int n0, float *dW1, int ldw1,
                      float *db0, float *db1, int splits, int exact) {
    return wgrad(st, ConvA{}, Kin, N, rows, X, ldx, dZ, ldz, part, colsum, dW0, ldw0, n0, dW1, ldw1, db0, db1, splits,
                 exact);
}

// conv weight gradient (implicit im2col X): dWt [Cin*ks*ks][Co] = X(src)^T dY over rows*42 positions
hipError_t gemm_conv_wgrad(hipStream_t st, int rows, int Co, int Cin, int ks, const float *src, int obs_ld,
                           const float *dY, float *part, float *colsum, float *dWt, float *db, int splits, int exact) {
    ConvA cv;
    cv.kind = 1; cv.cin = Cin; cv.ks = ks; cv.pad = ks / 2; cv.obs = obs_ld > 0; cv.ld = obs_ld;
    return wgrad(st, cv, Cin * ks * ks, Co, rows * CV_HW, src, 0, dY, Co, part, colsum, dWt, Co, Co, nullptr, 0, db,
                 nullptr, splits, exact);
}

static hipError_t wgrad(hipStream_t st, const ConvA &cv, int Kin, int N, int rows, const float *X, int ldx,
                        const float *dZ, int ldz, float *part, float *colsum, float *dW0, int ldw0, int n0,
                        float *dW1, int ldw1, float *db0, float *db1, int splits, int exact) {
    if (Kin <= 0 || N <= 0) return hipSuccess;
    if (exact == 2) {        // reference-exact: row-ordered f64 sums, one thread per entry
        SeqWg a{};
        a.cv = cv; a.X = X; a.ldx = ldx; a.dZ = dZ; a.ldz = ldz; a.Kin = Kin; a.N = N; a.rows = rows;
        a.dW0 = dW0; a.ldw0 = ldw0; a.n0 = dW1 ? n0 : N; a.dW1 = dW1; a.ldw1 = ldw1; a.db0 = db0; a.db1 = db1;
        const size_t nt = (size_t)Kin * N + ((db0 || db1) ? N : 0);
        hipLaunchKernelGGL(k_wg_seq, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, a);
        return hipGetLastError();
    }
    GemmArgs g{};
    g.cv = cv;
    g.A = X; g.lda = ldx; g.B = dZ; g.ldb = ldz; g.M = Kin; g.N = N; g.K = rows;
    g.part = part; g.colsum = (db0 || db1) ? colsum : nullptr;
    g.k_per_split = ((rows + splits - 1) / splits + GBK - 1) / GBK * GBK;
    const int sp = (rows + g.k_per_split - 1) / g.k_per_split;
    hipError_t e;
    if (exact < 0 && cv.kind == 0) e = launch_split_by_width<GEMM_WG>(g, sp, st);
    else if (exact > 0) e = cv.kind ? launch64_by_width<1>(g, sp, st) : launch64_by_width<0>(g, sp, st);
    else e = cv.kind ? launch_by_width<GEMM_WG, 1>(g, sp, st) : launch_by_width<GEMM_WG>(g, sp, st);
    if (e != hipSuccess) return e;
    if (exact < 0) exact = 0;                 // f32 partials either way
    const size_t MN = (size_t)Kin * N;
    const int nn0 = dW1 ? n0 : N;
    if (exact)
        hipLaunchKernelGGL(k_split_reduce64, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st,
                           (const double *)part, sp, Kin, N, nn0, dW0, ldw0, dW1, ldw1);
    else
        hipLaunchKernelGGL(k_split_reduce, dim3((unsigned)((MN + 255) / 256)), dim3(256), 0, st, part, sp, Kin, N,
                           nn0, dW0, ldw0, dW1, ldw1);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if (db0 || db1) {
        // bias gradient: colsum [sp][N] -> db0 (cols < n0) / db1
        if (exact)
            hipLaunchKernelGGL(k_split_reduce64, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st,
                               (const double *)colsum, sp, 1, N, db1 ? n0 : N, db0, 0, db1, 0);
        else
            hipLaunchKernelGGL(k_split_reduce, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, st, colsum, sp, 1, N,
                               db1 ? n0 : N, db0, 0, db1, 0);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace bppo

// ------------------------------------------------------------ parity hook ---
// bppo_debug_gemm: host buffers in/out; mode 0 FWD (bias, act 0 none / 1 relu /
// 2 tanh), 1 DX (H optional: act 2 tanh derivative, else relu mask), 2 WG
// (out = [Kin][N] weight grad, out2 = [N] bias grad), 3 WG with f64 sums (k_gemm_wg64),
// 4 WG with row-ordered f64 sums (k_wg_seq), 5 / 6 / 7: FWD / DX / WG on the split-bf16
// contraction (k_gemm_split).
extern "C" bppo_status bppo_debug_gemm(int32_t mode, int32_t M, int32_t N, int32_t K, const float *A,
                                       const float *B, const float *bias_or_H, int32_t act, float *out,
                                       float *out2) {
    using namespace bppo;
    if (!A || !B || !out || M <= 0 || N <= 0 || K <= 0 || mode < 0 || mode > 7) return BPPO_ERR_ARG;
    int exact = 0, split = 0;
    if (mode >= 5) {                   // split-bf16
        split = 1;
        mode -= 5;
        if (mode == 2) exact = -1;
    } else if (mode >= 3) {            // 3: f64 MFMA sums, 4: row-ordered f64 sums
        exact = mode - 2;
        mode = 2;
    }
    float *dA = nullptr, *dB = nullptr, *dX = nullptr, *dO = nullptr, *dO2 = nullptr, *dP = nullptr, *dC = nullptr;
    size_t nA = mode == 2 ? (size_t)K * M : (size_t)M * K;   // WG: X [rows=K][Kin=M]
    size_t nB = mode == 1 ? (size_t)N * K : (size_t)K * N;
    size_t nX = mode == 0 ? (size_t)N : (mode == 1 ? (size_t)M * N : 0);
    bppo_status s = BPPO_ERR_HIP;
    const int splits = mode == 2 ? gemm_wg_splits(M, N, K) : 1;
    do {
        if (hipMalloc((void **)&dA, nA * 4) != hipSuccess || hipMalloc((void **)&dB, nB * 4) != hipSuccess) break;
        if (hipMalloc((void **)&dO, (size_t)M * N * 4) != hipSuccess) break;
        if (hipMemcpy(dA, A, nA * 4, hipMemcpyHostToDevice) != hipSuccess) break;
        if (hipMemcpy(dB, B, nB * 4, hipMemcpyHostToDevice) != hipSuccess) break;
        if (nX && bias_or_H) {
            if (hipMalloc((void **)&dX, nX * 4) != hipSuccess) break;
            if (hipMemcpy(dX, bias_or_H, nX * 4, hipMemcpyHostToDevice) != hipSuccess) break;
        }
        hipError_t e;
        if (mode == 0) {
            if (!dX) break;
            e = gemm_fwd(nullptr, M, N, K, dA, K, dB, N, dX, act, dO, N, N, nullptr, 0, split);
        } else if (mode == 1) {
            e = gemm_dx(nullptr, M, N, K, dA, K, dB, K, dX, N, act, dO, N, nullptr, 0, nullptr, split);
        } else {
            if (hipMalloc((void **)&dO2, (size_t)N * 4) != hipSuccess) break;
            if (hipMalloc((void **)&dP, (size_t)splits * M * N * 8) != hipSuccess) break;
            if (hipMalloc((void **)&dC, (size_t)splits * N * 8) != hipSuccess) break;
            e = gemm_wgrad(nullptr, M, N, K, dA, M, dB, N, dP, dC, dO, N, N, nullptr, 0, dO2, nullptr, splits, exact);
        }
        if (e != hipSuccess || hipDeviceSynchronize() != hipSuccess) break;
        if (hipMemcpy(out, dO, (size_t)M * N * 4, hipMemcpyDeviceToHost) != hipSuccess) break;
        if (mode == 2 && out2 && hipMemcpy(out2, dO2, (size_t)N * 4, hipMemcpyDeviceToHost) != hipSuccess) break;
        s = BPPO_OK;
    } while (0);
    (void)hipFree(dA); (void)hipFree(dB); (void)hipFree(dX); (void)hipFree(dO); (void)hipFree(dO2);
    (void)hipFree(dP); (void)hipFree(dC);
    return s;
}

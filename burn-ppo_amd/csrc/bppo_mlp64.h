// bppo_mlp64.h — shared pieces of the MFMA kernels for the CfgB network
// (5 -> 64 -> 64 -> {2, 1}, relu; configs/cartpole.toml): parameter staging in
// LDS with conflict-free row strides, the per-wave transpose buffers, and the
// v_mfma_f32_32x32x2_f32 C/D layout helpers.
#pragma once
#include "bppo_device.h"
#include "bppo_math.h"

namespace bppo {
namespace mmb {
constexpr int H = 64, RS = 65, TR = 32;          // hidden width, LDS row stride, rows per wave tile
struct Params {
    // glibc expf / logf tables (bppo_math.h) in LDS: the loss's five expf and
    // one logf per row read them at LDS latency instead of from the L2
    uint64_t exp2tab[32];
    double linvc[16], llogc[16];
    float W0[6 * H];      // [d][k], d = 5 is a zero pad row (K 5 -> 6)
    float b0[H];
    float W1[H * RS];     // [k][o], row stride 65: conflict-free for both operand reads
    float b1[H];
    float Wp[H * 2];
    float bp[2];
    float Wv[H];
    float bv[2];
    float2 PV[2][H];      // {Wp[2k + h], Wv[k]}: the minibatch heads' (logit h, value) chain pair
    __device__ __forceinline__ float expf(float x) const { return bppo_math::expf_glibc_tab(x, exp2tab); }
    __device__ __forceinline__ float logf(float x) const { return bppo_math::logf_glibc_tab(x, linvc, llogc); }
};
struct Wave {
    float X[TR * 9];      // [row][d]
    float T[TR * RS];     // transpose staging: H1 -> H2 -> dZ2, [row][col]
    float dl[TR * 4];     // dL/d(logit0, logit1, value) per row
};
constexpr int WAVES = 8;
constexpr size_t LDS = sizeof(Params) + WAVES * sizeof(Wave);

// per-wave LDS of the minibatch kernel: H1 and H2 -> dZ2 both stay in LDS
// (neither is held in registers through the backward); X at stride 5
// (conflict-free: 5c mod 64 is distinct over 32 lanes)
struct WaveB {
    float X[TR * 5];
    float T1[TR * RS];    // H1 [row][k]
    float T2[TR * RS];    // H2, then dZ2 in place [row][o]
    float dl[TR * 4];
};
constexpr size_t LDSB = sizeof(Params) + WAVES * sizeof(WaveB);
static_assert(LDSB <= 160 * 1024, "minibatch kernel LDS over the gfx950 limit");

// whole block: flat Burn-order params -> LDS layout
__device__ __forceinline__ void load_params(Params &S, const float *__restrict__ P) {
    constexpr CpOffsets O = cp_offsets<64, 2>();
    for (int i = threadIdx.x; i < 6 * H; i += blockDim.x) S.W0[i] = i < 5 * H ? P[O.w0 + i] : 0.0f;
    for (int i = threadIdx.x; i < H * H; i += blockDim.x) S.W1[(i / H) * RS + (i % H)] = P[O.w1 + i];
    for (int i = threadIdx.x; i < H; i += blockDim.x) {
        S.b0[i] = P[O.b0 + i]; S.b1[i] = P[O.b1 + i]; S.Wv[i] = P[O.wv + i];
        S.Wp[2 * i] = P[O.wp + 2 * i]; S.Wp[2 * i + 1] = P[O.wp + 2 * i + 1];
        S.PV[0][i] = make_float2(P[O.wp + 2 * i], P[O.wv + i]);
        S.PV[1][i] = make_float2(P[O.wp + 2 * i + 1], P[O.wv + i]);
    }
    if (threadIdx.x < 32) S.exp2tab[threadIdx.x] = bppo_math::kExp2fTab[threadIdx.x];
    if (threadIdx.x < 16) {
        S.linvc[threadIdx.x] = bppo_math::kLogfInvc[threadIdx.x];
        S.llogc[threadIdx.x] = bppo_math::kLogfLogc[threadIdx.x];
    }
    if (threadIdx.x < 2) S.bp[threadIdx.x] = P[O.bp + threadIdx.x];
    if (threadIdx.x == 0) S.bv[0] = P[O.bv];
}

// C/D row of accumulator register q for lane half h
__device__ __forceinline__ int cd_row(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }
}  // namespace mmb

// LDS hand-off between the lanes of ONE wave: wait for this wave's LDS
// operations only (lgkmcnt), not for its outstanding global loads (a wavefront
// release fence would also drain vmcnt and stall the prefetched gathers)
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

typedef float f32x16_t __attribute__((ext_vector_type(16)));
}  // namespace bppo

// bppo_gemm.h — launchers of the f32 MFMA GEMM engine (k_gemm.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace bppo {

constexpr int GEMM_MAX_SPLITS = 1024;   // narrow conv weight gradients (Kin x Co = 72 x 8) need ~4 blocks per CU

// Y = act(X W + b): X [M][K] (ldx), W [K][N] (ldw), bias [N]; columns [0, n0)
// go to out0 (ld0), [n0, N) to out1 (ld1) when out1 != nullptr.  Bit-exact
// with matrixmultiply's KC=256 k-ordered fma chains (see k_gemm.hip).
// act: 0 none, 1 relu, 2 tanh (glibc tanhf, bit-exact).
// split != 0: the split-bf16 contraction (k_gemm_split: f32 accuracy, not the chains)
hipError_t gemm_fwd(hipStream_t st, int M, int N, int K, const float *X, int ldx, const float *W,
                    int ldw, const float *bias, int act, float *out0, int ld0, int n0, float *out1,
                    int ld1, int split = 0);
// out = (dZ W^T) * act'(H) given the layer OUTPUT H (may be null: no factor):
// act 2 tanh -> (1 - H^2), otherwise relu -> [H > 0].  dZ [M][K] (ldz), W [N][K] (ldw).
// Each element is the k-ordered fmaf chain from 0 (the oracle's linear_bwd dx).  xa / xw
// (may be null): + round(xa[row * ldxa] * xw[col]) after the chain, before act' -- a
// one-column head's input gradient added as its own rounded product (a shared trunk's
// value head beside the policy head's chain)
hipError_t gemm_dx(hipStream_t st, int M, int N, int K, const float *dZ, int ldz, const float *W,
                   int ldw, const float *H, int ldh, int act, float *out, int ldo, const float *xa = nullptr,
                   int ldxa = 0, const float *xw = nullptr, int split = 0);
// dW = X^T dZ over `rows` rows: X [rows][Kin] (ldx), dZ [rows][N] (ldz).
// Columns [0, n0) -> dW0 [Kin][ldw0], [n0, N) -> dW1 [Kin][ldw1] (when dW1);
// bias gradient (column sums of dZ) -> db0 / db1 likewise (either may be null).
// part: [splits][Kin][N] scratch, colsum: [splits][N] scratch (sized for doubles when exact).
// exact 0: f32 MFMA chains per split, f64 reduce; 1: f64 products and sums (k_gemm_wg64),
// the f32 result equal to the oracle's f64 sum's rounding but for rare ordering ties;
// 2: row-ordered f64 sums (k_wg_seq), the oracle's arithmetic exactly (latency-bound);
// -1: the split-bf16 contraction (k_gemm_split) per split, f64 reduce.
hipError_t gemm_wgrad(hipStream_t st, int Kin, int N, int rows, const float *X, int ldx, const float *dZ,
                      int ldz, float *part, float *colsum, float *dW0, int ldw0, int n0, float *dW1, int ldw1,
                      float *db0, float *db1, int splits, int exact = 0);
int gemm_wg_splits(int Kin, int N, int rows);

// Implicit-GEMM convolutions on Connect Four's 6 x 7 board (k_gemm.hip ConvA): NHWC
// activation rows [rows*42][C]; layer 0 reads the observation rows (obs_ld > 0: row
// stride, channels-last (h*7 + w)*Cin + ci, cnn.rs:252-262).
//   fwd   Y = relu(im2col(src) Wt + bias), Wt [Cin*ks*ks][Co] -- bit-identical to the
//         materialised im2col GEMM (same k order and KC blocks)
//   wgrad dWt = im2col(src)^T dY, db = column sums of dY (split-K, fixed-order reduce)
//   dx    dX = (taps(dY) Wd^T) * [H > 0], Wd [Cin][ks*ks*cpad]: one chain per tap (Co
//         channels, zero-padded to cpad), the taps summed in (kh, kw) order -- the
//         oracle's col2im gather
hipError_t gemm_conv_fwd(hipStream_t st, int rows, int Co, int Cin, int ks, const float *src, int obs_ld,
                         const float *Wt, const float *bias, float *out);
hipError_t gemm_conv_wgrad(hipStream_t st, int rows, int Co, int Cin, int ks, const float *src, int obs_ld,
                           const float *dY, float *part, float *colsum, float *dWt, float *db, int splits,
                           int exact = 0);
hipError_t gemm_conv_dx(hipStream_t st, int rows, int Cin, int Co, int ks, const float *dY, const float *Wd,
                        const float *H, float *out);
int gemm_conv_tap_pad(int Co);   // k's per tap of gemm_conv_dx's Wd (Co rounded up to 32)

}  // namespace bppo

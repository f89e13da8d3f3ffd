// cnn.hip — the CNN actor-critic trunk (network/cnn.rs:24-330) for Connect Four
// as implicit-GEMM convolutions on the f32 MFMA engine (k_gemm.hip ConvA): the
// patches are gathered from the NHWC activations while the GEMM's LDS stages are
// filled, so no im2col matrix exists in HBM (a 64-channel layer's would be
// rows*42 x 576 floats: 25 GB for a 262,144-row minibatch).
//
//   spatial   obs[:, :H*W*C] read as [B, H, W, C] then permuted to NCHW
//             (cnn.rs:252-262) — the observation itself is plane-major
//             (connect_four.rs:186-206), so element (c, h, w) of the conv input is
//             obs[(h*W + w)*C + c], exactly as the reference's reshape sees it;
//   conv      stride 1, same padding (k/2), bias, relu (cnn.rs:204-215):
//             Y[b*HW + hw][co] = relu(sum_k A[b*HW + hw][k] Wt[k][co] + bias[co]),
//             k = (ci, kh, kw) in Burn's weight order [Cout][Cin][kh][kw], the
//             KC = 256 fma chains of every Linear (bit-identical to the oracle's
//             materialised im2col GEMM: same elements, same order);
//   flatten   [B, C, H, W] -> [B, C*H*W] (NCHW, cnn.rs:216-218), then cat extra
//             features (cnn.rs:307-311) -> F [B][fdim], the first FC layer's input;
//   backward  dWt = A^T dY (implicit A, fixed-order split-K), db = column sums; the
//             input gradient as ONE transposed-conv GEMM dX = taps(dY) Wd^T times
//             relu'(input), Wd [Cin][(kh, kw, co)] (no dA matrix, no col2im pass).
#include "bppo_internal.h"
#include "bppo_gemm.h"
#include <algorithm>

namespace bppo {

#define CHIP(c, expr)                                                       \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);              \
    } while (0)

// F[b][c*HW + hw] = Y[b*HW + hw][c];  F[b][HW*Cl + j] = x[b*ldx + HW*C0 + j]
__global__ void __launch_bounds__(256) k_cnn_flatten(int B, int HW, int Cl, int C0, int E,
                                                      const float *__restrict__ Y, const float *__restrict__ x,
                                                      int ldx, float *__restrict__ F) {
    const int fd = HW * Cl + E;
    const size_t total = (size_t)B * fd;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const size_t b = i / fd;
        const int j = (int)(i % fd);
        F[i] = j < HW * Cl ? Y[(b * HW + j % HW) * Cl + j / HW] : x[b * ldx + (size_t)HW * C0 + (j - HW * Cl)];
    }
}

// dY[b*HW + hw][c] = dF[b][c*HW + hw]  (relu' already applied by the FC layer's DX epilogue)
__global__ void __launch_bounds__(256) k_cnn_unflatten(int B, int HW, int Cl, int fd, const float *__restrict__ dF,
                                                        float *__restrict__ dY) {
    const size_t total = (size_t)B * HW * Cl;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % Cl);
        const size_t row = i / Cl;
        dY[i] = dF[(row / HW) * fd + (size_t)c * HW + row % HW];
    }
}

// Burn conv weight [Cout][K] <-> GEMM operand [K][Cout]
__global__ void k_cnn_transpose(int R, int Cc, const float *__restrict__ src, float *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R * Cc) return;
    const int r = i / Cc, cc = i % Cc;
    dst[(size_t)cc * R + r] = src[i];
}

// Burn conv weight [Co][Cin][kk] -> the transposed-conv operand Wd[ci][t*cpad + co], the
// padding channels co in [Co, cpad) zero
__global__ void k_cnn_pack_dx(int Co, int Cin, int kk, int cpad, const float *__restrict__ w, float *__restrict__ wd) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cpad * Cin * kk) return;
    const int co = i / (Cin * kk), r = i % (Cin * kk), ci = r / kk, t = r % kk;
    wd[(size_t)ci * kk * cpad + t * cpad + co] = co < Co ? w[i] : 0.0f;
}

static dim3 grid_for(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 65536)); }

bppo_status cnn_alloc(bppo_ctx *c) {
    const NetLayout &n = c->net;
    const size_t HW = (size_t)n.H * n.W, R = (size_t)c->rows_max * HW;
    size_t kmax = 0, cmax = 0, wt = 0, wd = 0;
    c->cnn_stacks = n.critic_fc0 > n.critic_first ? 2 : 1;
    for (int s = 0; s < c->cnn_stacks; s++) {
        for (int l = 0; l < n.n_conv; l++) {
            kmax = std::max(kmax, (size_t)n.in[l]);
            cmax = std::max(cmax, (size_t)std::max(n.out[l], n.conv_cin[l]));
            c->cnn_wt_off[s][l] = wt;
            wt += (size_t)n.in[l] * n.out[l];
            c->cnn_wd_off[s][l] = wd;
            wd += (size_t)n.in[l] * gemm_conv_tap_pad(n.out[l]);   // Cin*kk*cpad
            CHIP(c, hipMalloc((void **)&c->d_cnn_y[s][l], R * n.out[l] * 4));
        }
        CHIP(c, hipMalloc((void **)&c->d_cnn_f[s], (size_t)c->rows_max * n.fdim * 4));
    }
    const size_t dy = std::max(R * cmax, (size_t)c->rows_max * n.fdim);
    CHIP(c, hipMalloc((void **)&c->d_cnn_dy[0], dy * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_dy[1], dy * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_wt, wt * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_wd, wd * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_owt, wt * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_dwt, kmax * cmax * 4));
    return BPPO_OK;
}

void cnn_free(bppo_ctx *c) {
    for (int s = 0; s < 2; s++) {
        for (float *q : c->d_cnn_y[s]) if (q) (void)hipFree(q);
        if (c->d_cnn_f[s]) (void)hipFree(c->d_cnn_f[s]);
    }
    void *p[] = {c->d_cnn_dy[0], c->d_cnn_dy[1], c->d_cnn_wt, c->d_cnn_wd, c->d_cnn_owt, c->d_cnn_dwt};
    for (void *q : p) if (q) (void)hipFree(q);
}

// the conv weights of `params` as GEMM operands (after every params change): Wt
// [K][Cout] for the forward, and (wd != nullptr) Wd [Cin][kk*Cout] for the input
// gradient of layers >= 1
bppo_status cnn_pack(bppo_ctx *c, const float *params, float *wt, float *wd) {
    const NetLayout &n = c->net;
    const int kk = n.ksize * n.ksize;
    for (int s = 0; s < c->cnn_stacks; s++)
        for (int l = 0; l < n.n_conv; l++) {
            const int R = n.out[l], Cc = n.in[l], lg = n.conv_base(s) + l;   // [Cout][K] -> [K][Cout]
            hipLaunchKernelGGL(k_cnn_transpose, dim3((R * Cc + 255) / 256), dim3(256), 0, c->stream, R, Cc,
                               params + n.w[lg], wt + c->cnn_wt_off[s][l]);
            if (wd && l > 0) {
                const int cpad = gemm_conv_tap_pad(R);
                hipLaunchKernelGGL(k_cnn_pack_dx, dim3((cpad * Cc + 255) / 256), dim3(256), 0, c->stream, R,
                                   n.conv_cin[l], kk, cpad, params + n.w[lg], wd + c->cnn_wd_off[s][l]);
            }
        }
    CHIP(c, hipGetLastError());
    return BPPO_OK;
}

// conv stack s + flatten of `rows` observation rows (x, ld ldx) -> d_cnn_f[s] [rows][fdim]
bppo_status cnn_features(bppo_ctx *c, int s, int rows, const float *x, int ldx, const float *params, const float *wt) {
    const NetLayout &n = c->net;
    const int HW = n.H * n.W, l0 = n.conv_base(s);
    for (int l = 0; l < n.n_conv; l++)
        CHIP(c, gemm_conv_fwd(c->stream, rows, n.out[l], n.conv_cin[l], n.ksize, l ? c->d_cnn_y[s][l - 1] : x,
                              l ? 0 : ldx, wt + c->cnn_wt_off[s][l], params + n.b[l0 + l], c->d_cnn_y[s][l]));
    const int Cl = n.out[n.n_conv - 1];
    hipLaunchKernelGGL(k_cnn_flatten, grid_for((size_t)rows * n.fdim), dim3(256), 0, c->stream, rows, HW, Cl, n.C, n.E,
                       (const float *)c->d_cnn_y[s][n.n_conv - 1], x, ldx, c->d_cnn_f[s]);
    CHIP(c, hipGetLastError());
    return BPPO_OK;
}

// dF = dL/dF [rows][fdim] (relu' of the last conv already applied) -> conv weight
// and bias gradients of stack s into grad (Burn layout); the activations of the last
// cnn_features call of that stack on the same rows are reused
bppo_status cnn_backward(bppo_ctx *c, int s, int rows, const float *x, int ldx, float *dF, float *grad, int exact) {
    const NetLayout &n = c->net;
    const int HW = n.H * n.W, M = rows * HW, last = n.n_conv - 1, l0 = n.conv_base(s);
    float *dy = c->d_cnn_dy[0], *dy2 = c->d_cnn_dy[1];
    if (dF == dy) std::swap(dy, dy2);
    hipLaunchKernelGGL(k_cnn_unflatten, grid_for((size_t)M * n.out[last]), dim3(256), 0, c->stream, rows, HW,
                       n.out[last], n.fdim, (const float *)dF, dy);
    CHIP(c, hipGetLastError());
    for (int l = last; l >= 0; l--) {
        const int K = n.in[l], Co = n.out[l];
        const float *src = l ? c->d_cnn_y[s][l - 1] : x;
        const int sp = gemm_wg_splits(K, Co, M);
        CHIP(c, gemm_conv_wgrad(c->stream, rows, Co, n.conv_cin[l], n.ksize, src, l ? 0 : ldx, dy, c->d_part,
                                c->d_colsum, c->d_cnn_dwt, grad + n.b[l0 + l], sp, exact));
        hipLaunchKernelGGL(k_cnn_transpose, dim3((K * Co + 255) / 256), dim3(256), 0, c->stream, K, Co,
                           (const float *)c->d_cnn_dwt, grad + n.w[l0 + l]);
        CHIP(c, hipGetLastError());
        if (l == 0) break;
        // the input gradient straight into the previous layer's NHWC rows, relu' applied
        CHIP(c, gemm_conv_dx(c->stream, rows, n.conv_cin[l], Co, n.ksize, dy, c->d_cnn_wd + c->cnn_wd_off[s][l],
                             c->d_cnn_y[s][l - 1], dy2));
        std::swap(dy, dy2);
    }
    return BPPO_OK;
}

}  // namespace bppo

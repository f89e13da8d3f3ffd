// cnn.hip — the CNN actor-critic trunk (network/cnn.rs:24-330) for Connect Four
// on the f32 MFMA GEMM engine, as implicit-GEMM convolutions staged through an
// im2col buffer in HBM (288 GB per GPU: the whole minibatch's im2col fits, so a
// conv layer is ONE engine GEMM, not a loop of small ones).
//
//   spatial   obs[:, :H*W*C] read as [B, H, W, C] then permuted to NCHW
//             (cnn.rs:252-262) — the observation itself is plane-major
//             (connect_four.rs:186-206), so element (c, h, w) of the conv input is
//             obs[(h*W + w)*C + c], exactly as the reference's reshape sees it;
//   conv      stride 1, same padding (k/2), bias, relu (cnn.rs:204-215):
//             Y[b*HW + hw][co] = relu(sum_k A[b*HW + hw][k] Wt[k][co] + bias[co]),
//             k = (ci, kh, kw) in Burn's weight order [Cout][Cin][kh][kw], through
//             gemm_fwd (matrixmultiply's KC = 256 fma chains, like every Linear);
//   flatten   [B, C, H, W] -> [B, C*H*W] (NCHW, cnn.rs:216-218), then cat extra
//             features (cnn.rs:307-311) -> F [B][fdim], the first FC layer's input;
//   backward  dWt = im2col^T dY (gemm_wgrad, fixed-order split-K), db = column
//             sums, dA = dY Wt^T (gemm_dx), then col2im as a GATHER (each input
//             element sums its <= k*k taps in (kh, kw) order: deterministic, no
//             atomics) times relu'(input).
// Activations are NHWC rows ([b*HW + hw][channel]), so each conv is a plain
// row-major GEMM and its output feeds the next im2col directly.
// split_networks (cnn.rs:116-135, 264-302): a second conv stack (s = 1, layers
// [critic_first, critic_fc0)) on the same spatial input feeds the critic's FC layers;
// every function below takes the stack index s.
#include "bppo_internal.h"
#include "bppo_gemm.h"
#include <algorithm>

namespace bppo {

#define CHIP(c, expr)                                                       \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);              \
    } while (0)

struct ConvGeo { int B, H, W, Cin, ks, pad; };

// im2col: A[b*HW + hw][(ci*ks + kh)*ks + kw].  src(b, hw', ci): from the raw
// observation rows (layer 0, the reference's channels-last reshape) or from the
// previous layer's NHWC output
template <bool FROM_OBS>
__global__ void __launch_bounds__(256) k_cnn_im2col(ConvGeo g, const float *__restrict__ src, int ld,
                                                     float *__restrict__ A) {
    const int K = g.Cin * g.ks * g.ks, HW = g.H * g.W;
    const size_t total = (size_t)g.B * HW * K;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int k = (int)(i % K);
        const size_t row = i / K;
        const int hw = (int)(row % HW);
        const size_t b = row / HW;
        const int ci = k / (g.ks * g.ks), kk = k % (g.ks * g.ks), kh = kk / g.ks, kw = kk % g.ks;
        const int h = hw / g.W + kh - g.pad, w = hw % g.W + kw - g.pad;
        float v = 0.0f;
        if (h >= 0 && h < g.H && w >= 0 && w < g.W) {
            const int hw2 = h * g.W + w;
            v = FROM_OBS ? src[b * ld + (size_t)hw2 * g.Cin + ci] : src[(b * HW + hw2) * g.Cin + ci];
        }
        A[i] = v;
    }
}

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

// col2im gather: dX[b*HW + hw][ci] = [Y > 0] * sum over (kh, kw) ascending of
// dA[b*HW + hw_out][(ci*ks + kh)*ks + kw], hw_out = (h - kh + pad, w - kw + pad)
__global__ void __launch_bounds__(256) k_cnn_col2im(ConvGeo g, const float *__restrict__ dA,
                                                     const float *__restrict__ Y, float *__restrict__ dX) {
    const int K = g.Cin * g.ks * g.ks, HW = g.H * g.W;
    const size_t total = (size_t)g.B * HW * g.Cin;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
        const int ci = (int)(i % g.Cin);
        const size_t row = i / g.Cin;
        const int hw = (int)(row % HW);
        const size_t b = row / HW;
        const int h = hw / g.W, w = hw % g.W;
        float s = 0.0f;
        for (int kh = 0; kh < g.ks; kh++)
            for (int kw = 0; kw < g.ks; kw++) {
                const int ho = h - kh + g.pad, wo = w - kw + g.pad;
                if (ho < 0 || ho >= g.H || wo < 0 || wo >= g.W) continue;
                s = __fadd_rn(s, dA[(b * HW + ho * g.W + wo) * K + (ci * g.ks + kh) * g.ks + kw]);
            }
        dX[i] = Y[i] > 0.0f ? s : 0.0f;
    }
}

// Burn conv weight [Cout][K] <-> GEMM operand [K][Cout]
__global__ void k_cnn_transpose(int R, int Cc, const float *__restrict__ src, float *__restrict__ dst) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= R * Cc) return;
    const int r = i / Cc, cc = i % Cc;
    dst[(size_t)cc * R + r] = src[i];
}

static dim3 grid_for(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 65536)); }

static ConvGeo geo(const NetLayout &n, int l, int B) {
    return ConvGeo{B, n.H, n.W, n.conv_cin[l], n.ksize, n.ksize / 2};
}

bppo_status cnn_alloc(bppo_ctx *c) {
    const NetLayout &n = c->net;
    const size_t HW = (size_t)n.H * n.W, R = (size_t)c->rows_max * HW;
    size_t kmax = 0, cmax = 0, wt = 0;
    c->cnn_stacks = n.critic_fc0 > n.critic_first ? 2 : 1;
    for (int s = 0; s < c->cnn_stacks; s++) {
        for (int l = 0; l < n.n_conv; l++) {
            kmax = std::max(kmax, (size_t)n.in[l]);
            cmax = std::max(cmax, (size_t)std::max(n.out[l], n.conv_cin[l]));
            c->cnn_wt_off[s][l] = wt;
            wt += (size_t)n.in[l] * n.out[l];
            CHIP(c, hipMalloc((void **)&c->d_cnn_y[s][l], R * n.out[l] * 4));
        }
        CHIP(c, hipMalloc((void **)&c->d_cnn_f[s], (size_t)c->rows_max * n.fdim * 4));
    }
    const size_t dy = std::max(R * cmax, (size_t)c->rows_max * n.fdim);
    CHIP(c, hipMalloc((void **)&c->d_cnn_a, R * kmax * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_dy[0], dy * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_dy[1], dy * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_wt, wt * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_owt, wt * 4));
    CHIP(c, hipMalloc((void **)&c->d_cnn_dwt, kmax * cmax * 4));
    return BPPO_OK;
}

void cnn_free(bppo_ctx *c) {
    for (int s = 0; s < 2; s++) {
        for (float *q : c->d_cnn_y[s]) if (q) (void)hipFree(q);
        if (c->d_cnn_f[s]) (void)hipFree(c->d_cnn_f[s]);
    }
    void *p[] = {c->d_cnn_a, c->d_cnn_dy[0], c->d_cnn_dy[1], c->d_cnn_wt, c->d_cnn_owt, c->d_cnn_dwt};
    for (void *q : p) if (q) (void)hipFree(q);
}

// the conv weights of `params` as GEMM operands [K][Cout] (after every params change)
bppo_status cnn_pack(bppo_ctx *c, const float *params, float *wt) {
    const NetLayout &n = c->net;
    for (int s = 0; s < c->cnn_stacks; s++)
        for (int l = 0; l < n.n_conv; l++) {
            const int R = n.out[l], Cc = n.in[l], lg = n.conv_base(s) + l;   // [Cout][K] -> [K][Cout]
            hipLaunchKernelGGL(k_cnn_transpose, dim3((R * Cc + 255) / 256), dim3(256), 0, c->stream, R, Cc,
                               params + n.w[lg], wt + c->cnn_wt_off[s][l]);
        }
    CHIP(c, hipGetLastError());
    return BPPO_OK;
}

// conv stack s + flatten of `rows` observation rows (x, ld ldx) -> d_cnn_f[s] [rows][fdim]
bppo_status cnn_features(bppo_ctx *c, int s, int rows, const float *x, int ldx, const float *params, const float *wt) {
    const NetLayout &n = c->net;
    const int HW = n.H * n.W, l0 = n.conv_base(s);
    for (int l = 0; l < n.n_conv; l++) {
        const ConvGeo g = geo(n, l, rows);
        const size_t tot = (size_t)rows * HW * n.in[l];
        if (l == 0) hipLaunchKernelGGL(k_cnn_im2col<true>, grid_for(tot), dim3(256), 0, c->stream, g, x, ldx, c->d_cnn_a);
        else hipLaunchKernelGGL(k_cnn_im2col<false>, grid_for(tot), dim3(256), 0, c->stream, g,
                                (const float *)c->d_cnn_y[s][l - 1], 0, c->d_cnn_a);
        CHIP(c, hipGetLastError());
        CHIP(c, gemm_fwd(c->stream, rows * HW, n.out[l], n.in[l], c->d_cnn_a, n.in[l], wt + c->cnn_wt_off[s][l],
                         n.out[l], params + n.b[l0 + l], 1, c->d_cnn_y[s][l], n.out[l], n.out[l], nullptr, 0));
    }
    const int Cl = n.out[n.n_conv - 1];
    hipLaunchKernelGGL(k_cnn_flatten, grid_for((size_t)rows * n.fdim), dim3(256), 0, c->stream, rows, HW, Cl, n.C, n.E,
                       (const float *)c->d_cnn_y[s][n.n_conv - 1], x, ldx, c->d_cnn_f[s]);
    CHIP(c, hipGetLastError());
    return BPPO_OK;
}

// dF = dL/dF [rows][fdim] (relu' of the last conv already applied) -> conv weight
// and bias gradients of stack s into grad (Burn layout); the activations of the last
// cnn_features call of that stack on the same rows are reused
bppo_status cnn_backward(bppo_ctx *c, int s, int rows, const float *x, int ldx, float *dF, float *grad) {
    const NetLayout &n = c->net;
    const int HW = n.H * n.W, M = rows * HW, last = n.n_conv - 1, l0 = n.conv_base(s);
    float *dy = c->d_cnn_dy[0], *dy2 = c->d_cnn_dy[1];
    if (dF == dy) std::swap(dy, dy2);
    hipLaunchKernelGGL(k_cnn_unflatten, grid_for((size_t)M * n.out[last]), dim3(256), 0, c->stream, rows, HW,
                       n.out[last], n.fdim, (const float *)dF, dy);
    CHIP(c, hipGetLastError());
    for (int l = last; l >= 0; l--) {
        const ConvGeo g = geo(n, l, rows);
        const int K = n.in[l], Co = n.out[l];
        const size_t tot = (size_t)M * K;
        if (l == 0) hipLaunchKernelGGL(k_cnn_im2col<true>, grid_for(tot), dim3(256), 0, c->stream, g, x, ldx, c->d_cnn_a);
        else hipLaunchKernelGGL(k_cnn_im2col<false>, grid_for(tot), dim3(256), 0, c->stream, g,
                                (const float *)c->d_cnn_y[s][l - 1], 0, c->d_cnn_a);
        CHIP(c, hipGetLastError());
        const int sp = gemm_wg_splits(K, Co, M);
        CHIP(c, gemm_wgrad(c->stream, K, Co, M, c->d_cnn_a, K, dy, Co, c->d_part, c->d_colsum, c->d_cnn_dwt, Co, Co,
                           nullptr, 0, grad + n.b[l0 + l], nullptr, sp));
        hipLaunchKernelGGL(k_cnn_transpose, dim3((K * Co + 255) / 256), dim3(256), 0, c->stream, K, Co,
                           (const float *)c->d_cnn_dwt, grad + n.w[l0 + l]);
        CHIP(c, hipGetLastError());
        if (l == 0) break;
        // dA = dY Wt^T (im2col layout), then col2im into the previous layer's output
        CHIP(c, gemm_dx(c->stream, M, K, Co, dy, Co, c->d_cnn_wt + c->cnn_wt_off[s][l], Co, nullptr, 0, 0, c->d_cnn_a,
                        K));
        hipLaunchKernelGGL(k_cnn_col2im, grid_for((size_t)M * n.conv_cin[l]), dim3(256), 0, c->stream, g,
                           (const float *)c->d_cnn_a, (const float *)c->d_cnn_y[s][l - 1], dy2);
        CHIP(c, hipGetLastError());
        std::swap(dy, dy2);
    }
    return BPPO_OK;
}

}  // namespace bppo

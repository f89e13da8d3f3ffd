// How does v_mfma_f32_32x32x16_bf16 round its f32 accumulation?  One wave; every output
// element D[i][j] = C[i][j] + sum_k A[i][k] B[k][j] with A[i][k] = 1 for the k's under test
// and B[k][j] = the test products, C = c.  Compared with round-to-nearest-even of the exact
// sum (f64 on the host) and with truncation toward zero.  Diagnosis only.
//   hipcc --offload-arch=gfx950 -O2 -o scripts/probes/mfma_round_probe scripts/probes/mfma_round_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstring>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Case { float c; float p[4]; };

__global__ void run(const Case *cs, int n, float *out) {
    const int lane = threadIdx.x;
    for (int t = 0; t < n; t++) {
        bf16x8 a, b;
        for (int j = 0; j < 8; j++) { a[j] = (__bf16)0.0f; b[j] = (__bf16)0.0f; }
        // k = 8 (lane / 32) + j: the test products sit at k = 0..3 (lanes 0-31, j = 0..3)
        if (lane < 32)
            for (int j = 0; j < 4; j++) { a[j] = (__bf16)1.0f; b[j] = (__bf16)cs[t].p[j]; }
        f32x16 acc;
        for (int q = 0; q < 16; q++) acc[q] = cs[t].c;
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
        if (lane == 0) out[t] = acc[0];
    }
}

static float rne(double x) { return (float)x; }
static float trunc0(double x) {
    float f = (float)x;
    if (std::fabs((double)f) > std::fabs(x)) f = std::nextafter(f, 0.0f);
    return f;
}

int main() {
    const float u = ldexpf(1.0f, -24);
    Case h[] = {
        {1.0f, {1.25f * u, 0, 0, 0}},                  // 1 + 1.25 ulp/2: RNE up, truncation 1
        {1.0f, {u, 0.25f * u, 0, 0}},                  // the same sum from two products
        {1.0f, {0.75f * u, 0.75f * u, 0, 0}},          // 1.5 half-ulps from two products
        {1.0f, {-1.25f * 0.5f * u, 0, 0, 0}},          // below 1: half-ulp there is 2^-25
        {1.0f, {0.5f * u, 0.5f * u, 0.5f * u, 0}},     // 3 x half-ulp
        {0.0f, {1.0f, ldexpf(1.0f, -25), 0, 0}},       // product sum alone
        {0.0f, {1.0f, ldexpf(1.0f, -24) * 1.5f, 0, 0}},
        {1.0f, {ldexpf(1.0f, -26), ldexpf(1.0f, -26), ldexpf(1.0f, -26), ldexpf(1.0f, -26)}},  // 4 x quarter ulp
        {3.0f, {-1.0f, -1.0f, u, 0}},                  // cancellation, then a tiny term
    };
    const int n = sizeof(h) / sizeof(h[0]);
    Case *d; float *o;
    hipMalloc(&d, sizeof(h)); hipMalloc(&o, n * 4);
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, d, n, o);
    float r[64];
    if (hipMemcpy(r, o, n * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("failed\n"); return 1; }
    for (int t = 0; t < n; t++) {
        double ex = h[t].c;
        for (int j = 0; j < 4; j++) ex += (double)(float)(__bf16)h[t].p[j];
        printf("case %d: mfma %.10g  rne %.10g  trunc %.10g  -> %s\n", t, r[t], rne(ex), trunc0(ex),
               r[t] == rne(ex) ? (r[t] == trunc0(ex) ? "rne=trunc" : "RNE") : (r[t] == trunc0(ex) ? "TRUNC" : "other"));
    }
    return 0;
}

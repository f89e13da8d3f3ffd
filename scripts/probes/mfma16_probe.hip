// Layout and rounding probe for v_mfma_f32_16x16x4_f32 on gfx950.
//  1. layout: A lane l = 1000 + l, B lane l = l (one-hot style sums decoded on the host)
//     -> checks the assumed mapping A[m][k] = lane (m + 16 k), B[k][n] = lane (n + 16 k),
//        D register j of lane l = D[4 (l / 16) + j][l % 16];
//  2. rounding: random operands; D must equal, bit for bit, the k-ordered fma chain
//     acc = fma(a_k, b_k, acc), k = 0..3, from the initial C (chained over 16 steps).
// Build: hipcc -O3 --offload-arch=gfx950 -w mfma16_probe.hip -o mfma16_probe.bin
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void k_probe(const float *A, const float *B, float *D, int steps) {
    const int l = threadIdx.x;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < steps; s++)
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[s * 64 + l], B[s * 64 + l], acc, 0, 0, 0);
    for (int j = 0; j < 4; j++) D[l * 4 + j] = acc[j];
}

int main() {
    const int steps = 16;
    float hA[64 * steps], hB[64 * steps], hD[256];
    float *dA, *dB, *dD;
    hipMalloc(&dA, sizeof hA); hipMalloc(&dB, sizeof hB); hipMalloc(&dD, sizeof hD);
    // 1. layout: B one-hot per (k, n) candidate: set B lane (n + 16 k) = 1 only for one lane
    int bad = 0;
    for (int kk = 0; kk < 4; kk++)
        for (int n = 0; n < 16; n++) {
            for (int l = 0; l < 64; l++) { hA[l] = (float)(l + 1); hB[l] = (l == n + 16 * kk) ? 1.f : 0.f; }
            hipMemcpy(dA, hA, 64 * 4, hipMemcpyHostToDevice);
            hipMemcpy(dB, hB, 64 * 4, hipMemcpyHostToDevice);
            hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, 1);
            hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
            // expected: D[m][n] = A[m][kk] = lane m + 16 kk -> value m + 16 kk + 1, other columns 0
            for (int l = 0; l < 64; l++)
                for (int j = 0; j < 4; j++) {
                    const int m = 4 * (l / 16) + j, col = l % 16;
                    const float want = col == n ? (float)(m + 16 * kk + 1) : 0.f;
                    if (hD[l * 4 + j] != want) bad++;
                }
        }
    printf("layout mismatches: %d\n", bad);
    // 2. rounding: the k-ordered fma chain, chained over `steps` instructions
    srand(7);
    for (int i = 0; i < 64 * steps; i++) {
        hA[i] = (float)((rand() / (double)RAND_MAX - 0.5) * pow(2.0, rand() % 20 - 10));
        hB[i] = (float)((rand() / (double)RAND_MAX - 0.5) * pow(2.0, rand() % 20 - 10));
    }
    hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, dA, dB, dD, steps);
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int chain_bad = 0, tree_bad = 0;
    for (int m = 0; m < 16; m++)
        for (int n = 0; n < 16; n++) {
            float acc = 0.f, acc2 = 0.f;
            for (int s = 0; s < steps; s++) {
                for (int k = 0; k < 4; k++) acc = fmaf(hA[s * 64 + m + 16 * k], hB[s * 64 + n + 16 * k], acc);
                float t = 0.f;   // alternative: the 4 products summed first, then added
                for (int k = 0; k < 4; k++) t += hA[s * 64 + m + 16 * k] * hB[s * 64 + n + 16 * k];
                acc2 += t;
            }
            const int l = n + 16 * (m / 4), j = m % 4;
            uint32_t g, c, c2;
            memcpy(&g, &hD[l * 4 + j], 4); memcpy(&c, &acc, 4); memcpy(&c2, &acc2, 4);
            chain_bad += g != c;
            tree_bad += g != c2;
        }
    printf("k-ordered fma chain mismatches: %d / 256, sum-then-add mismatches: %d / 256\n", chain_bad, tree_bad);
    return 0;
}

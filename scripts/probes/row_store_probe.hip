// Store-pattern probe for the packed 64-byte update rows (8.39 M rows = 537 MB):
// what a kernel pays to write part or all of each row, by access pattern.
//   A  8 B  per row (float2 at float 8), lane = 4 consecutive rows (k_gae_1p_seg r02)
//   B  32 B per row (second sector), lane = 4 consecutive rows
//   C  64 B per row, lane = 4 consecutive rows (16 float4 stores per lane, 256 B stride)
//   D  64 B per row, wave-contiguous: store k of a wave writes bytes [1 KB k, 1 KB (k+1))
//   E  16 B per row (first float4), lane = row (the rollout's pattern)
// plus a read-only stream of 20 B per row (the GAE inputs) for scale.
// Build: hipcc -O3 --offload-arch=gfx950 row_store_probe.hip -o row_store_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t NROWS = 8388608;

__global__ void kA(float4 *rows, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    float2 *o = reinterpret_cast<float2 *>(rows + 4 * (4 * g) + 2);
    o[0] = make_float2(1.f, 2.f); o[8] = make_float2(1.f, 2.f); o[16] = make_float2(1.f, 2.f); o[24] = make_float2(1.f, 2.f);
}
__global__ void kB(float4 *rows, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    float4 *o = rows + 4 * (4 * g) + 2;
    const float4 a = make_float4(1.f, 2.f, 0.f, 0.f), z = make_float4(0.f, 0.f, 0.f, 0.f);
    o[0] = a; o[1] = z; o[4] = a; o[5] = z; o[8] = a; o[9] = z; o[12] = a; o[13] = z;
}
__global__ void kC(float4 *rows, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    float4 *o = rows + 16 * g;
#pragma unroll
    for (int k = 0; k < 16; k++) o[k] = make_float4((float)k, 1.f, 2.f, 3.f);
}
__global__ void kD(float4 *rows, size_t n4) {
    // each wave owns 64 lanes x 4 rows = 256 rows = 16 KB; store k covers 1 KB contiguous
    const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x & 63;
    if (wave * 64 >= n4) return;
    float4 *base = rows + wave * 64 * 16;
#pragma unroll
    for (int k = 0; k < 16; k++) base[k * 64 + lane] = make_float4((float)k, 1.f, 2.f, 3.f);
}
__global__ void kE(float4 *rows, size_t n) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n) return;
    rows[4 * g] = make_float4(1.f, 2.f, 3.f, 4.f);
}
// F: 32 B per row, lane = row, two float4 stores at +0 / +16 (32 B stride across lanes)
__global__ void kF(float4 *rows, size_t n) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n) return;
    rows[2 * g] = make_float4(1.f, 2.f, 3.f, 4.f);
    rows[2 * g + 1] = make_float4(5.f, 6.f, 7.f, 8.f);
}
// G: 32 B per row, the wave's 64 rows (2 KB) as float4 #lane and #64 + lane
__global__ void kG(float4 *rows, size_t n) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n) return;
    const size_t w0 = g & ~(size_t)63;
    const int lane = threadIdx.x & 63;
    rows[2 * w0 + lane] = make_float4(1.f, 2.f, 3.f, 4.f);
    rows[2 * w0 + 64 + lane] = make_float4(5.f, 6.f, 7.f, 8.f);
}
// H: 8 B per row, lane = 4 consecutive rows: two float4 stores (32 B stride across lanes)
__global__ void kH(float4 *pairs, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    pairs[2 * g] = make_float4(1.f, 2.f, 3.f, 4.f);
    pairs[2 * g + 1] = make_float4(5.f, 6.f, 7.f, 8.f);
}
// I: 8 B per row, wave-contiguous float4 #lane and #64 + lane
__global__ void kI(float4 *pairs, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    const size_t w0 = g & ~(size_t)63;
    const int lane = threadIdx.x & 63;
    pairs[2 * w0 + lane] = make_float4(1.f, 2.f, 3.f, 4.f);
    pairs[2 * w0 + 64 + lane] = make_float4(5.f, 6.f, 7.f, 8.f);
}
__global__ void kR(const float4 *a, const float4 *b, const float4 *c, float4 *out, size_t n4) {
    size_t g = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (g >= n4) return;
    const float4 x = a[g], y = b[g], z = c[g];
    out[g] = make_float4(x.x + y.x + z.x, x.y + y.y + z.y, x.z + y.z + z.z, x.w + y.w + z.w);
}

int main() {
    float4 *rows, *a, *b, *c, *o;
    hipMalloc(&rows, NROWS * 64);
    hipMalloc(&a, NROWS * 4); hipMalloc(&b, NROWS * 4); hipMalloc(&c, NROWS * 4); hipMalloc(&o, NROWS * 4);
    hipMemset(rows, 0, NROWS * 64);
    hipMemset(a, 0, NROWS * 4); hipMemset(b, 0, NROWS * 4); hipMemset(c, 0, NROWS * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const size_t n4 = NROWS / 4;
    auto run = [&](const char *name, auto launch, double bytes) {
        for (int i = 0; i < 3; i++) launch();
        hipEventRecord(e0);
        const int reps = 20;
        for (int i = 0; i < reps; i++) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-44s %8.1f us  %7.1f GB/s of useful bytes\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    };
    run("A 8 B/row, 4 rows per lane", [&] { hipLaunchKernelGGL(kA, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 8.0);
    run("B 32 B/row (sector), 4 rows per lane", [&] { hipLaunchKernelGGL(kB, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 32.0);
    run("C 64 B/row, 4 rows per lane", [&] { hipLaunchKernelGGL(kC, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 64.0);
    run("D 64 B/row, wave-contiguous 1 KB stores", [&] { hipLaunchKernelGGL(kD, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 64.0);
    run("E 16 B/row, lane = row", [&] { hipLaunchKernelGGL(kE, dim3((NROWS + 255) / 256), dim3(256), 0, 0, rows, NROWS); },
        NROWS * 16.0);
    run("F 32 B/row, lane = row (2 x float4, 32 B stride)", [&] { hipLaunchKernelGGL(kF, dim3((NROWS + 255) / 256), dim3(256), 0, 0, rows, NROWS); },
        NROWS * 32.0);
    run("G 32 B/row, wave-contiguous", [&] { hipLaunchKernelGGL(kG, dim3((NROWS + 255) / 256), dim3(256), 0, 0, rows, NROWS); },
        NROWS * 32.0);
    run("H 8 B/row, 4 rows per lane (32 B stride)", [&] { hipLaunchKernelGGL(kH, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 8.0);
    run("I 8 B/row, wave-contiguous", [&] { hipLaunchKernelGGL(kI, dim3((n4 + 255) / 256), dim3(256), 0, 0, rows, n4); },
        NROWS * 8.0);
    run("R read 3 x 4 B + write 4 B per row, coalesced", [&] { hipLaunchKernelGGL(kR, dim3((n4 + 255) / 256), dim3(256), 0, 0, a, b, c, o, n4); },
        NROWS * 16.0);
    return 0;
}

// Are the device's f32 division / square root correctly rounded, as the host's (and the
// oracle's Adam step) are?  Each op on 2^24 random operands on the GPU against the host.
//   hipcc --offload-arch=gfx950 -O2 -ffp-contract=off -fno-fast-math -o scripts/probes/fp_rounding_probe scripts/probes/fp_rounding_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void ops(const float *a, const float *b, const double *d, int n, float *o_div, float *o_sqrt,
                    float *o_sqrtd, float *o_sqrtf, float *o_divop) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    o_div[i] = __fdiv_rn(a[i], b[i]);
    o_sqrt[i] = __fsqrt_rn(fabsf(a[i]));
    o_sqrtd[i] = (float)sqrt(d[i]);
    o_sqrtf[i] = sqrtf(fabsf(a[i]));
    o_divop[i] = a[i] / b[i];
}

static uint32_t bits(float x) { uint32_t u; memcpy(&u, &x, 4); return u; }

int main() {
    const int n = 1 << 24;
    std::vector<float> a(n), b(n);
    std::vector<double> d(n);
    uint64_t s = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; };
    for (int i = 0; i < n; i++) {
        // magnitudes spread over the range Adam sees (1e-12 .. 1e2)
        const double ea = -12.0 + 14.0 * (double)(rnd() >> 11) / 9007199254740992.0;
        const double eb = -12.0 + 14.0 * (double)(rnd() >> 11) / 9007199254740992.0;
        a[i] = (float)(((rnd() & 1) ? 1.0 : -1.0) * pow(10.0, ea));
        b[i] = (float)(pow(10.0, eb));
        d[i] = (double)(rnd() >> 11) * pow(2.0, -50.0);
    }
    float *da, *db, *o1, *o2, *o3, *o4, *o5;
    double *dd;
    hipMalloc(&da, n * 4); hipMalloc(&db, n * 4); hipMalloc(&dd, n * 8);
    hipMalloc(&o1, n * 4); hipMalloc(&o2, n * 4); hipMalloc(&o3, n * 4); hipMalloc(&o4, n * 4); hipMalloc(&o5, n * 4);
    hipMemcpy(da, a.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(db, b.data(), n * 4, hipMemcpyHostToDevice);
    hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(ops, dim3((n + 255) / 256), dim3(256), 0, 0, da, db, dd, n, o1, o2, o3, o4, o5);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
    std::vector<float> r1(n), r2(n), r3(n), r4(n), r5(n);
    hipMemcpy(r1.data(), o1, n * 4, hipMemcpyDeviceToHost); hipMemcpy(r2.data(), o2, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r3.data(), o3, n * 4, hipMemcpyDeviceToHost); hipMemcpy(r4.data(), o4, n * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r5.data(), o5, n * 4, hipMemcpyDeviceToHost);
    long m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0;
    int shown = 0;
    for (int i = 0; i < n; i++) {
        const float q = a[i] / b[i], sq = sqrtf(fabsf(a[i])), sd = (float)sqrt(d[i]);
        if (bits(r1[i]) != bits(q)) { m1++; if (shown++ < 4) printf("  div %.9g / %.9g: dev %.9g host %.9g\n", a[i], b[i], r1[i], q); }
        if (bits(r2[i]) != bits(sq)) m2++;
        if (bits(r3[i]) != bits(sd)) m3++;
        if (bits(r4[i]) != bits(sq)) m4++;
        if (bits(r5[i]) != bits(q)) m5++;
    }
    printf("of %d: __fdiv_rn %ld differ, __fsqrt_rn %ld, (float)sqrt(double) %ld, sqrtf %ld, a / b %ld\n", n, m1, m2, m3,
           m4, m5);
    return 0;
}

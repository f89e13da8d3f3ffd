// bppo_math.h — bit-exact restatement of the platform libm transcendentals the
// reference's Rust code calls (f32::ln -> logf, f32::sin/cos -> sinf/cosf).
//
// The reference runs on glibc 2.35 (x86-64, FMA ifunc variants): logf is
// sysdeps/ieee754/flt-32/e_logf.c and sinf/cosf are s_sinf.c / s_cosf.c with
// sincosf.h (ARM optimized-routines algorithms, double-precision evaluation,
// compiled with -mfma so a*b+c contracts to fma).  Call sites:
//   utils.rs:25         gumbel = -ln(-ln(u))
//   cartpole.rs:51-52   theta.cos(), theta.sin()
// The constant tables below are the data that glibc's libm.so.6 carries
// (__logf_data, __sincosf_table, __inv_pio4).  Origin and licence: these tables
// (and the tanhf/expm1f constants further down, from fdlibm via glibc) are third-
// party data from the GNU C Library 2.35, licensed LGPL-2.1-or-later (the logf /
// sincosf tables originate in ARM's optimized-routines, MIT / Apache-2.0 with LLVM
// exception); they are reproduced as data, needed for bit-exact transcendentals.
// tests/test_libm_restatement.py
// checks every Gumbel input and every float |x| < 1 against the real glibc on
// the host, and the GPU tests check device == host on the same inputs, so the
// device kernels reproduce the reference bit for bit.
//
// Shared verbatim between host C++ and HIP device code; every operation is an
// explicit IEEE double op or fma (build with -ffp-contract=off).
#pragma once
#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#define BPPO_HD __host__ __device__ __forceinline__
#else
#define BPPO_HD static inline
#endif

namespace bppo_math {

BPPO_HD uint32_t asuint(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
BPPO_HD float asfloat(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// Constant tables: namespace-scope so runtime-indexed reads stay in constant
// memory on the device (function-local arrays would be copied to scratch).
#if defined(__HIP_DEVICE_COMPILE__)
#define BPPO_TABLE static __constant__ const
#else
#define BPPO_TABLE static const
#endif
BPPO_TABLE double kLogfInvc[16] = {
        0x1.661ec79f8f3bep+0, 0x1.571ed4aaf883dp+0, 0x1.49539f0f010bp+0,  0x1.3c995b0b80385p+0,
        0x1.30d190c8864a5p+0, 0x1.25e227b0b8eap+0,  0x1.1bb4a4a1a343fp+0, 0x1.12358f08ae5bap+0,
        0x1.0953f419900a7p+0, 0x1.0p+0,             0x1.e608cfd9a47acp-1, 0x1.ca4b31f026aap-1,
        0x1.b2036576afce6p-1, 0x1.9c2d163a1aa2dp-1, 0x1.886e6037841edp-1, 0x1.767dcf5534862p-1};
BPPO_TABLE double kLogfLogc[16] = {
        -0x1.57bf7808caadep-2, -0x1.2bef0a7c06ddbp-2, -0x1.01eae7f513a67p-2, -0x1.b31d8a68224e9p-3,
        -0x1.6574f0ac07758p-3, -0x1.1aa2bc79c81p-3,   -0x1.a4e76ce8c0e5ep-4, -0x1.1973c5a611cccp-4,
        -0x1.252f438e10c1ep-5, 0x0.0p+0,              0x1.aa5aa5df25984p-5,  0x1.c5e53aa362eb4p-4,
        0x1.526e57720db08p-3,  0x1.bc2860d22477p-3,   0x1.1058bc8a07ee1p-2,  0x1.4043057b6ee09p-2};
BPPO_TABLE uint32_t kInvPio4[24] = {
        0xa2u,       0xa2f9u,     0xa2f983u,   0xa2f9836eu, 0xf9836e4eu, 0x836e4e44u,
        0x6e4e4415u, 0x4e441529u, 0x441529fcu, 0x1529fc27u, 0x29fc2757u, 0xfc2757d1u,
        0x2757d1f5u, 0x57d1f534u, 0xd1f534ddu, 0xf534ddc0u, 0x34ddc0dbu, 0xddc0db62u,
        0xc0db6295u, 0xdb629599u, 0x6295993cu, 0x95993c43u, 0x993c4390u, 0x3c439041u};
BPPO_TABLE uint64_t kExp2fTab[32] = {
        0x3ff0000000000000ULL, 0x3fefd9b0d3158574ULL, 0x3fefb5586cf9890fULL, 0x3fef9301d0125b51ULL,
        0x3fef72b83c7d517bULL, 0x3fef54873168b9aaULL, 0x3fef387a6e756238ULL, 0x3fef1e9df51fdee1ULL,
        0x3fef06fe0a31b715ULL, 0x3feef1a7373aa9cbULL, 0x3feedea64c123422ULL, 0x3feece086061892dULL,
        0x3feebfdad5362a27ULL, 0x3feeb42b569d4f82ULL, 0x3feeab07dd485429ULL, 0x3feea47eb03a5585ULL,
        0x3feea09e667f3bcdULL, 0x3fee9f75e8ec5f74ULL, 0x3feea11473eb0187ULL, 0x3feea589994cce13ULL,
        0x3feeace5422aa0dbULL, 0x3feeb737b0cdc5e5ULL, 0x3feec49182a3f090ULL, 0x3feed503b23e255dULL,
        0x3feee89f995ad3adULL, 0x3feeff76f2fb5e47ULL, 0x3fef199bdd85529cULL, 0x3fef3720dcef9069ULL,
        0x3fef5818dcfba487ULL, 0x3fef7c97337b9b5fULL, 0x3fefa4afa2a490daULL, 0x3fefd0765b6e4540ULL};

// ------------------------------------------------------------------ logf ----
// (the _tab forms take the tables from a caller-chosen copy, e.g. in LDS)
BPPO_HD float logf_glibc_tab(float x, const double *invc_t, const double *logc_t) {
    // __logf_data (LOGF_TABLE_BITS = 4): {invc, logc}
            const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2,
                 A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix = asuint(x);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        if (ix * 2 == 0) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);
        ix = asuint(x * 0x1p23f);
        ix -= 23u << 23;
    }
    uint32_t tmp = ix - 0x3f330000u;
    int i = (int)((tmp >> (23 - 4)) % 16);
    int k = (int32_t)tmp >> 23;
    uint32_t iz = ix - (tmp & (0x1ffu << 23));
    double invc = invc_t[i], logc = logc_t[i];
    double z = (double)asfloat(iz);
    double r = fma(z, invc, -1.0);
    double y0 = fma((double)k, Ln2, logc);
    double r2 = r * r;
    double y = fma(A1, r, A2);
    y = fma(A0, r2, y);
    y = fma(y, r2, y0 + r);
    return (float)y;
}
BPPO_HD float logf_glibc(float x) { return logf_glibc_tab(x, kLogfInvc, kLogfLogc); }

// ---------------------------------------------------------- sinf / cosf ----
struct sincos_t {
    double sign[4], hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};

BPPO_HD sincos_t sincos_table(int which) {
    // __sincosf_table[0] / [1] (table 1 negates the cosine coefficients)
    const double g = which ? -1.0 : 1.0;
    sincos_t t = {{1.0, -1.0, -1.0, 1.0}, 0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0,
                  g * 0x1.0p+0, g * -0x1.ffffffd0c621cp-2, -0x1.555545995a603p-3,
                  g * 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7, g * -0x1.6c087e89a359dp-10,
                  -0x1.994eb3774cf24p-13, g * 0x1.99343027bf8c3p-16};
    return t;
}

BPPO_HD uint32_t abstop12(float x) { return (asuint(x) >> 20) & 0x7ff; }

BPPO_HD float sinf_poly(double x, double x2, const sincos_t &p, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = fma(x2, p.s3, p.s2);
        double x7 = x3 * x2;
        double s = fma(x3, p.s1, x);
        return (float)fma(x7, s1, s);
    } else {
        double x4 = x2 * x2;
        double c2 = fma(x2, p.c4, p.c3);
        double c1 = fma(x2, p.c1, p.c0);
        double x6 = x4 * x2;
        double c = fma(x4, p.c2, c1);
        return (float)fma(x6, c2, c);
    }
}

BPPO_HD double reduce_fast(double x, const sincos_t &p, int *np) {
    double r = x * p.hpi_inv;
    int32_t n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
    return fma(-(double)n, p.hpi, x);
}

BPPO_HD double reduce_large(uint32_t xi, int *np) {
    // __inv_pio4: bits of 4/pi, each entry the previous shifted by 8 bits
        const double pi63 = 0x1.921fb54442d18p-62;
    const uint32_t *arr = &kInvPio4[(xi >> 26) & 15];
    int shift = (xi >> 23) & 7;
    uint64_t n, res0, res1, res2;
    xi = (xi & 0xffffff) | 0x800000;
    xi <<= shift;
    res0 = xi * arr[0];
    res1 = (uint64_t)xi * arr[4];
    res2 = (uint64_t)xi * arr[8];
    res0 = (res2 >> 32) | (res0 << 32);
    res0 += res1;
    n = (res0 + (1ULL << 61)) >> 62;
    res0 -= n << 62;
    double x = (double)(int64_t)res0;
    *np = (int)n;
    return x * pi63;
}

BPPO_HD float sinf_glibc(float y) {
    double x = y;
    int n;
    if (abstop12(y) < 0x3f4u) {            // abstop12(pio4)
        double s = x * x;
        if (abstop12(y) < 0x398u) return y;  // abstop12(0x1p-12f)
        return sinf_poly(x, s, sincos_table(0), 0);
    } else if (abstop12(y) < 0x42fu) {     // abstop12(120.0f)
        sincos_t p = sincos_table(0);
        x = reduce_fast(x, p, &n);
        double s = ((n + 1) & 2) ? -1.0 : 1.0;   // sign[4] = {1,-1,-1,1}
        if (n & 2) p = sincos_table(1);
        return sinf_poly(x * s, x * x, p, n);
    } else if (abstop12(y) < 0x7f8u) {
        uint32_t xi = asuint(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        sincos_t p = sincos_table(0);
        double s = ((n + sign + 1) & 2) ? -1.0 : 1.0;
        if ((n + sign) & 2) p = sincos_table(1);
        return sinf_poly(x * s, x * x, p, n);
    }
    return (y - y) / (y - y);
}

BPPO_HD float cosf_glibc(float y) {
    double x = y;
    int n;
    if (abstop12(y) < 0x3f4u) {
        double x2 = x * x;
        if (abstop12(y) < 0x398u) return 1.0f;
        return sinf_poly(x, x2, sincos_table(0), 1);
    } else if (abstop12(y) < 0x42fu) {
        sincos_t p = sincos_table(0);
        x = reduce_fast(x, p, &n);
        double s = ((n + 1) & 2) ? -1.0 : 1.0;   // sign[4] = {1,-1,-1,1}
        if (n & 2) p = sincos_table(1);
        return sinf_poly(x * s, x * x, p, n ^ 1);
    } else if (abstop12(y) < 0x7f8u) {
        uint32_t xi = asuint(y);
        int sign = xi >> 31;
        x = reduce_large(xi, &n);
        sincos_t p = sincos_table(0);
        double s = ((n + sign + 1) & 2) ? -1.0 : 1.0;
        if ((n + sign) & 2) p = sincos_table(1);
        return sinf_poly(x * s, x * x, p, n ^ 1);
    }
    return (y - y) / (y - y);
}


// ------------------------------------------------------------------ expf ----
// e_expf.c with __exp2f_data (EXP2F_TABLE_BITS = 5): used by log_softmax /
// entropy / ratio = exp(log_ratio) (utils.rs:43-57, ppo.rs:1452).
BPPO_HD uint64_t asuint64(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
BPPO_HD double asdouble(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

BPPO_HD float expf_glibc_tab(float x, const uint64_t *tab) {
        const double SHIFT = 0x1.8p+52, InvLn2N = 0x1.71547652b82fep+5;
    const double C0 = 0x1.c6af84b912394p-20, C1 = 0x1.ebfce50fac4f3p-13, C2 = 0x1.62e42ff0c52d6p-6;
    double xd = (double)x;
    uint32_t abstop = (asuint(x) >> 20) & 0x7ff;
    if (abstop >= 0x42bu) {                       // top12(88.0f)
        if (asuint(x) == asuint(-INFINITY)) return 0.0f;
        if (abstop >= 0x7f8u) return x + x;
        if (x > 0x1.62e42ep6f) return INFINITY;
        if (x < -0x1.9fe368p6f) return 0.0f;
    }
    double z = InvLn2N * xd;
    double kd = z + SHIFT;
    uint64_t ki = asuint64(kd);
    kd -= SHIFT;
    double r = fma(InvLn2N, xd, -kd);   // glibc's -mfma build contracts z - kd
    uint64_t t = tab[ki % 32];
    t += ki << (52 - 5);
    double s = asdouble(t);
    double zz = fma(C0, r, C1);
    double r2 = r * r;
    double y = fma(C2, r, 1.0);
    y = fma(zz, r2, y);
    y = y * s;
    return (float)y;
}

BPPO_HD float expf_glibc(float x) { return expf_glibc_tab(x, kExp2fTab); }

// ---------------------------------------------------------------- tanhf ---
// The tanh activation (mlp.rs:187-191, Burn ndarray -> f32::tanh -> tanhf).
// glibc 2.35 tanhf/expm1f are the fdlibm single-precision routines
// (sysdeps/ieee754/flt-32/s_tanhf.c, s_expm1f.c) with no FMA ifunc variant: pure
// float arithmetic, every product and sum rounded on its own.  Restated from the
// published fdlibm algorithm; a one-off run over all 2^32 non-NaN floats found
// zero mismatches against this image's glibc, and
// tests/test_libm_restatement.py re-checks dense and random samples.
// expm1f for the arguments tanhf passes (finite, |x| < 44); the overflow branch
// is kept for completeness.
BPPO_HD float expm1f_glibc(float x) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f, invln2 = 1.4426950216e+00f;
    const float Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f, Q3 = -7.9365076090e-05f,
                Q4 = 4.0082177293e-06f, Q5 = -2.0109921195e-07f;
    uint32_t hx = asuint(x);
    const uint32_t neg = hx >> 31;
    hx &= 0x7fffffffu;
    if (hx >= 0x4195b844u) {                        // |x| >= 27 ln2
        if (hx >= 0x42b17218u) {                    // |x| >= 88.72
            if (hx > 0x7f800000u) return x + x;
            if (hx == 0x7f800000u) return neg ? -1.0f : x;
            if (x > 8.8721679688e+01f) return INFINITY;
        }
        if (neg) return 1.0e-30f - 1.0f;            // -1 (inexact)
    }
    float hi, lo, c = 0.0f, t;
    int32_t k;
    if (hx > 0x3eb17218u) {                         // |x| > ln2 / 2: reduce by k ln2
        if (hx < 0x3F851592u) {                     // and |x| < 1.5 ln2
            if (!neg) { hi = x - ln2_hi; lo = ln2_lo; k = 1; }
            else { hi = x + ln2_hi; lo = -ln2_lo; k = -1; }
        } else {
            k = (int32_t)(invln2 * x + (neg ? -0.5f : 0.5f));
            t = (float)k;
            hi = x - t * ln2_hi;                    // exact
            lo = t * ln2_lo;
        }
        x = hi - lo;
        c = (hi - x) - lo;
    } else if (hx < 0x33000000u) {                  // |x| < 2^-25
        return x;
    } else {
        k = 0;
    }
    const float hfx = 0.5f * x, hxs = x * hfx;
    const float r1 = 1.0f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    t = 3.0f - r1 * hfx;
    float e = hxs * ((r1 - t) / (6.0f - x * t));
    if (k == 0) return x - (x * e - hxs);
    e = (x * (e - c) - c);
    e -= hxs;
    if (k == -1) return 0.5f * (x - e) - 0.5f;
    if (k == 1) return x < -0.25f ? -2.0f * (e - (x + 0.5f)) : 1.0f + 2.0f * (x - e);
    float y;
    if (k <= -2 || k > 56) {                        // exp(x) - 1 ~ exp(x)
        y = 1.0f - (e - x);
        y = asfloat(asuint(y) + ((uint32_t)k << 23));
        return y - 1.0f;
    }
    if (k < 23) {
        t = asfloat(0x3f800000u - (0x1000000u >> k));   // 1 - 2^-k
        y = t - (e - x);
    } else {
        t = asfloat((uint32_t)(0x7f - k) << 23);         // 2^-k
        y = x - (e + t);
        y += 1.0f;
    }
    return asfloat(asuint(y) + ((uint32_t)k << 23));
}

BPPO_HD float tanhf_glibc(float x) {
    const uint32_t jx = asuint(x), ix = jx & 0x7fffffffu;
    if (ix >= 0x7f800000u) return (jx >> 31) ? 1.0f / x - 1.0f : 1.0f / x + 1.0f;   // +-inf, NaN
    float z;
    if (ix < 0x41b00000u) {                          // |x| < 22
        if (ix == 0) return x;
        if (ix < 0x24000000u) return x * (1.0f + x); // |x| < 2^-55
        if (ix >= 0x3f800000u) {                     // |x| >= 1
            const float t = expm1f_glibc(2.0f * fabsf(x));
            z = 1.0f - 2.0f / (t + 2.0f);
        } else {
            const float t = expm1f_glibc(-2.0f * fabsf(x));
            z = -t / (t + 2.0f);
        }
    } else {
        z = 1.0f - 1.0e-30f;                         // +-1 (inexact)
    }
    return (jx >> 31) ? -z : z;
}

// The same arithmetic as tanhf_glibc with every branch turned into a select
// (each candidate is computed exactly as its branch would compute it), for
// straight-line use inside fully unrolled per-unit loops on the device.  The
// expm1f argument a = +-2|x| lies in (-2, 44): only the reductions k = 0, -1
// and the general k path occur, and the result paths k <= -2 / k > 56,
// 2 <= k < 23 and k >= 23.
BPPO_HD float tanhf_glibc_bf(float x) {
    const float ln2_hi = 6.9313812256e-01f, ln2_lo = 9.0580006145e-06f, invln2 = 1.4426950216e+00f;
    const float Q1 = -3.3333335072e-02f, Q2 = 1.5873016091e-03f, Q3 = -7.9365076090e-05f,
                Q4 = 4.0082177293e-06f, Q5 = -2.0109921195e-07f;
    const uint32_t jx = asuint(x), ix = jx & 0x7fffffffu;
    const float ax = asfloat(ix);
    const bool big = ix >= 0x3f800000u;
    const float a = big ? 2.0f * ax : -2.0f * ax;           // expm1f argument
    const uint32_t ha = asuint(a) & 0x7fffffffu;
    const bool aneg = !big;
    // argument reduction
    const bool red = ha > 0x3eb17218u, near1 = ha < 0x3F851592u;
    const int32_t kg = (int32_t)(invln2 * a + (aneg ? -0.5f : 0.5f));
    const float tg = (float)kg;
    const float hi = near1 ? (aneg ? a + ln2_hi : a - ln2_hi) : a - tg * ln2_hi;
    const float lo = near1 ? (aneg ? -ln2_lo : ln2_lo) : tg * ln2_lo;
    const int32_t k = red ? (near1 ? (aneg ? -1 : 1) : kg) : 0;
    const float xr_red = hi - lo;
    const float xr = red ? xr_red : a;
    const float c = red ? (hi - xr_red) - lo : 0.0f;
    // primary range
    const float hfx = 0.5f * xr, hxs = xr * hfx;
    const float r1 = 1.0f + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
    const float t = 3.0f - r1 * hfx;
    const float e0 = hxs * ((r1 - t) / (6.0f - xr * t));
    const float res_k0 = xr - (xr * e0 - hxs);
    float e = (xr * (e0 - c) - c);
    e -= hxs;
    const float res_m1 = 0.5f * (xr - e) - 0.5f;
    const uint32_t ksh = (uint32_t)k << 23;
    const float ya = 1.0f - (e - xr);
    const float res_a = asfloat(asuint(ya) + ksh) - 1.0f;                 // k <= -2 or k > 56
    const int32_t kb = k < 1 ? 1 : (k > 24 ? 24 : k);                    // keep the shifts in range
    const float yb = asfloat(0x3f800000u - (0x1000000u >> kb)) - (e - xr);
    const float res_b = asfloat(asuint(yb) + ksh);                         // 2 <= k < 23
    const int32_t kc = k > 126 ? 126 : (k < 0 ? 0 : k);
    float yc = xr - (e + asfloat((uint32_t)(0x7f - kc) << 23));
    yc += 1.0f;
    const float res_c = asfloat(asuint(yc) + ksh);                         // k >= 23
    float tm = k < 23 ? res_b : res_c;
    tm = (k <= -2 || k > 56) ? res_a : tm;
    tm = k == -1 ? res_m1 : tm;
    tm = k == 0 ? res_k0 : tm;
    tm = ha < 0x33000000u ? a : tm;                                        // |a| < 2^-25
    // tanh from expm1
    const float q = (big ? 2.0f : -tm) / (tm + 2.0f);
    float z = big ? 1.0f - q : q;
    z = ix >= 0x41b00000u ? 1.0f - 1.0e-30f : z;                          // |x| >= 22
    z = (jx >> 31) ? -z : z;
    z = ix < 0x24000000u ? x * (1.0f + x) : z;                             // |x| < 2^-55 (and +-0)
    // +-inf already gives +-1 above; NaN -> quiet NaN (glibc: 1/x +- 1)
    z = ix > 0x7f800000u ? x + x : z;
    return z;
}

}  // namespace bppo_math

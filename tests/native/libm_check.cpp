// Host harness for tests/test_libm_restatement.py: compares the product's
// bppo_math.h restatement with the platform glibc on given inputs.
#include "bppo_math.h"
#include <cmath>
#include <cstddef>
extern "C" {
size_t mismatch_logf(const float *x, size_t n, float *ref, float *got) {
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        ref[i] = logf(x[i]); got[i] = bppo_math::logf_glibc(x[i]);
        bad += bppo_math::asuint(ref[i]) != bppo_math::asuint(got[i]);
    }
    return bad;
}
size_t mismatch_expf(const float *x, size_t n, float *ref, float *got) {
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        ref[i] = expf(x[i]); got[i] = bppo_math::expf_glibc(x[i]);
        bad += bppo_math::asuint(ref[i]) != bppo_math::asuint(got[i]);
    }
    return bad;
}
size_t mismatch_sincos(const float *x, size_t n, float *rs, float *gs, float *rc, float *gc) {
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        rs[i] = sinf(x[i]); gs[i] = bppo_math::sinf_glibc(x[i]);
        rc[i] = cosf(x[i]); gc[i] = bppo_math::cosf_glibc(x[i]);
        bad += (bppo_math::asuint(rs[i]) != bppo_math::asuint(gs[i])) +
               (bppo_math::asuint(rc[i]) != bppo_math::asuint(gc[i]));
    }
    return bad;
}
size_t mismatch_tanhf(const float *x, size_t n, float *ref, float *got) {
    size_t bad = 0;
    for (size_t i = 0; i < n; i++) {
        ref[i] = tanhf(x[i]); got[i] = bppo_math::tanhf_glibc(x[i]);
        bad += bppo_math::asuint(ref[i]) != bppo_math::asuint(got[i]);
        bad += bppo_math::asuint(ref[i]) != bppo_math::asuint(bppo_math::tanhf_glibc_bf(x[i]));   // device form
    }
    return bad;
}
// every Gumbel draw of utils.rs:20-25: u = gen_range(1e-10f32..1.0) from word w,
// g = -ln(-ln(u)); k = w >> 9 indexes all 2^23 distinct u.
size_t mismatch_gumbel_all(void) {
    size_t bad = 0;
    for (uint32_t k = 0; k < (1u << 23); k++) {
        float v = bppo_math::asfloat(k | 0x3F800000u) - 1.0f;
        float u = v * 1.0f + 1e-10f;
        float a = -logf(-logf(u));
        float b = -bppo_math::logf_glibc(-bppo_math::logf_glibc(u));
        bad += bppo_math::asuint(a) != bppo_math::asuint(b);
    }
    return bad;
}
}

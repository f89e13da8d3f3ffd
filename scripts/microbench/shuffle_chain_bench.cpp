// Micro-benchmark of the rand 0.8.5 Fisher-Yates draw chain (gen_range(0..i+1)
// with UniformInt<u32> zone rejection) — the host-serial part of ppo_update's
// shuffle.  Variants are checked against the plain loop.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include <chrono>
#include <random>
#include <immintrin.h>
using u32 = uint32_t; using u64 = uint64_t;
static inline u32 zone_of(u32 r) { return (r << __builtin_clz(r)) - 1u; }

size_t v_branchy(const u32 *w, u32 n, u32 *J) {
    size_t used = 0;
    for (u32 i = n - 1; i >= 1; i--) {
        u32 range = i + 1, zone = zone_of(range);
        for (;;) { u64 m = (u64)w[used++] * range; if ((u32)m <= zone) { J[i] = (u32)(m >> 32); break; } }
    }
    return used;
}
size_t v_branchless(const u32 *w, u32 n, u32 *J) {
    u32 i = n - 1; size_t p = 0;
    while (i >= 1) { u32 range = i + 1; u32 zone = zone_of(range); u64 m = (u64)w[p++] * range;
        J[i] = (u32)(m >> 32); i -= ((u32)m <= zone); }
    return p;
}
// band loop: lz constant inside [lowr, 2 lowr); zone updated incrementally
size_t v_band(const u32 *w, u32 n, u32 *J) {
    u32 r = n; size_t p = 0;
    while (r >= 2) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2) {
            u64 m = (u64)w[p++] * r;
            J[r - 1] = (u32)(m >> 32);
            u32 acc = (u32)m <= z;
            r -= acc; z -= acc ? s : 0;
        }
    }
    return p;
}
// two words per step; the second word's candidate products derived by subtraction
size_t v_spec2(const u32 *w, u32 n, u32 *J) {
    u32 r = n; size_t p = 0;
    while (r >= 2) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr + 2) {
            const u32 wa = w[p], wb = w[p + 1];
            const u64 ma = (u64)wa * r, mb = (u64)wb * r;
            const u32 acca = (u32)ma <= z;
            J[r - 1] = (u32)(ma >> 32);
            const u64 mb1 = mb - wb;                     // wb * (r-1)
            const u64 mbs = acca ? mb1 : mb;
            const u32 zb = z - (acca ? s : 0);
            const u32 accb = (u32)mbs <= zb;
            J[r - 1 - acca] = (u32)(mbs >> 32);
            const u32 acc = acca + accb;
            r -= acc; z -= acc * s; p += 2;
        }
        while (r >= lowr && r >= 2) {
            u64 m = (u64)w[p++] * r; J[r - 1] = (u32)(m >> 32);
            u32 acc = (u32)m <= z; r -= acc; z -= acc ? s : 0;
        }
    }
    return p;
}
// four words per step; 10-bit acceptance pattern resolved by table
struct Tab4 { uint8_t nacc[1024]; uint8_t accmask[1024]; };
static Tab4 make_tab4() {
    Tab4 t;
    for (int idx = 0; idx < 1024; idx++) {
        // bits: A0 | B0 B1 | C0 C1 C2 | D0 D1 D2 D3  (word q, offset j = rejections so far)
        int off[4] = {0, 1, 3, 6};
        int j = 0, acc = 0, am = 0;
        for (int q = 0; q < 4; q++) {
            int bit = (idx >> (off[q] + j)) & 1;
            if (bit) { am |= 1 << q; acc++; } else j++;
        }
        t.nacc[idx] = (uint8_t)acc; t.accmask[idx] = (uint8_t)am;
    }
    return t;
}
static const Tab4 TAB4 = make_tab4();
size_t v_spec4(const u32 *w, u32 n, u32 *J) {
    u32 r = n; size_t p = 0;
    while (r >= 2) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr + 4) {
            const u32 w0 = w[p], w1 = w[p + 1], w2 = w[p + 2], w3 = w[p + 3];
            // lo of w_q * (r - q + j), zone z - (q - j) s
            const u32 l0 = w0 * r, l1 = w1 * r, l2 = w2 * r, l3 = w3 * r;
            u32 idx = (u32)(l0 <= z);
            idx |= (u32)(l1 - w1 <= z - s) << 1;      // B, j=0 : range r-1
            idx |= (u32)(l1 <= z) << 2;               // B, j=1 : range r
            idx |= (u32)(l2 - 2 * w2 <= z - 2 * s) << 3;
            idx |= (u32)(l2 - w2 <= z - s) << 4;
            idx |= (u32)(l2 <= z) << 5;
            idx |= (u32)(l3 - 3 * w3 <= z - 3 * s) << 6;
            idx |= (u32)(l3 - 2 * w3 <= z - 2 * s) << 7;
            idx |= (u32)(l3 - w3 <= z - s) << 8;
            idx |= (u32)(l3 <= z) << 9;
            const u32 am = TAB4.accmask[idx], acc = TAB4.nacc[idx];
            // emit accepted words: m-th accepted gets range r - m
            u32 rr = r;
            const u32 ws[4] = {w0, w1, w2, w3};
#pragma GCC unroll 4
            for (int q = 0; q < 4; q++) {
                const u64 m = (u64)ws[q] * rr;
                J[rr - 1] = (u32)(m >> 32);           // rejected words are overwritten by the next accept
                rr -= (am >> q) & 1;
            }
            r -= acc; z -= acc * s; p += 4;
        }
        while (r >= lowr && r >= 2) {
            u64 m = (u64)w[p++] * r; J[r - 1] = (u32)(m >> 32);
            u32 acc = (u32)m <= z; r -= acc; z -= acc ? s : 0;
        }
    }
    return p;
}
// decision chain only (no J): lower bound for any emission strategy
size_t v_decide_only(const u32 *w, u32 n, u32 *J) {
    u32 r = n; size_t p = 0;
    while (r >= 2) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2) { u32 acc = (u32)(w[p++] * r) <= z; r -= acc; z -= acc ? s : 0; }
    }
    J[1] = (u32)p;
    return p;
}

#if defined(__AVX512F__) && defined(__AVX512VL__) && defined(__AVX512BW__)
// 16 words per block, acceptance masks for 8 rejection offsets, branchless resolution
size_t v_avx512(const u32 *w, u32 n, u32 *J) {
    u32 r = n; size_t p = 0;
    const __m512i kidx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i rev = _mm512_setr_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    while (r >= 2) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        while (r >= lowr + 24) {
            const u32 z = (r << lz) - 1u;
            const __m512i wv = _mm512_loadu_si512((const void *)(w + p));
            const __m512i rk = _mm512_sub_epi32(_mm512_set1_epi32((int)r), kidx);
            __m512i lo = _mm512_mullo_epi32(wv, rk);
            __m512i zz = _mm512_sub_epi32(_mm512_set1_epi32((int)z), _mm512_slli_epi32(kidx, lz));
            const __m512i sv = _mm512_set1_epi32((int)s);
            u64 M[8];
#pragma GCC unroll 8
            for (int j = 0; j < 8; j++) {
                M[j] = (u64)_mm512_cmple_epu32_mask(lo, zz);
                lo = _mm512_add_epi32(lo, wv); zz = _mm512_add_epi32(zz, sv);
            }
            // walk: k = first unprocessed word; rejection j lands at the first 0 of M[j] at >= k
            u64 k = 0, rejmask = 0;
#pragma GCC unroll 8
            for (int j = 0; j < 8; j++) {
                const u64 rej = ((~M[j]) & 0xFFFFull & (~0ull << k)) | (1ull << 16);
                const u64 kz = (u64)__builtin_ctzll(rej);
                rejmask |= 1ull << kz;
                k = kz + 1;
            }
            // after 8 rejections the block stops at k (<= 16); k = 17 means fewer than 8 rejections
            const u32 stop = k > 16 ? 16u : (u32)k;
            const u32 valid = (u32)((1u << stop) - 1u);
            const u32 am = (~(u32)rejmask) & valid;
            const u32 acc = (u32)__builtin_popcount(am);
            const __m512i wc = _mm512_maskz_compress_epi32((__mmask16)am, wv);
            const __m512i rng = _mm512_sub_epi32(_mm512_set1_epi32((int)r), kidx);   // r - m
            const __m512i pe = _mm512_mul_epu32(wc, rng);
            const __m512i po = _mm512_mul_epu32(_mm512_srli_epi64(wc, 32), _mm512_srli_epi64(rng, 32));
            const __m512i hi = _mm512_mask_blend_epi32((__mmask16)0xAAAA, _mm512_srli_epi64(pe, 32), po);
            const __m512i hr = _mm512_permutexvar_epi32(rev, hi);
            const __mmask16 sm = (__mmask16)(0xFFFFu & ~((1u << (16 - acc)) - 1u));
            _mm512_mask_storeu_epi32((void *)(J + r - 16), sm, hr);
            r -= acc; p += stop;
        }
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2) {
            u64 m = (u64)w[p++] * r; J[r - 1] = (u32)(m >> 32);
            u32 acc = (u32)m <= z; r -= acc; z -= acc ? s : 0;
        }
    }
    return p;
}
#endif

typedef size_t (*walk_fn)(const u32 *, u32, u32 *);
int main() {
    const u32 n = 1u << 23;
    std::vector<u32> w((size_t)n * 2);
    std::mt19937 g(1);
    for (auto &x : w) x = g();
    std::vector<u32> ref(n, 0), J(n, 0);
    size_t uref = v_branchy(w.data(), n, ref.data());
    struct { const char *name; walk_fn f; bool check; } vs[] = {
        {"branchy", v_branchy, true}, {"branchless", v_branchless, true}, {"band", v_band, true},
        {"spec2", v_spec2, true}, {"spec4", v_spec4, true}, {"decide_only", v_decide_only, false},
#if defined(__AVX512F__) && defined(__AVX512VL__) && defined(__AVX512BW__)
        {"avx512", v_avx512, true},
#endif
    };
    for (auto &v : vs) {
        double best = 1e30; size_t used = 0;
        for (int rep = 0; rep < 3; rep++) {
            std::fill(J.begin(), J.end(), 0);
            auto t0 = std::chrono::steady_clock::now();
            used = v.f(w.data(), n, J.data());
            auto t1 = std::chrono::steady_clock::now();
            best = std::min(best, std::chrono::duration<double, std::milli>(t1 - t0).count());
        }
        bool ok = used == uref && (!v.check || J == ref);
        printf("%-12s %8.2f ms  %.3f ns/word  %s\n", v.name, best, best * 1e6 / (double)uref, ok ? "OK" : "MISMATCH");
    }
    return 0;
}

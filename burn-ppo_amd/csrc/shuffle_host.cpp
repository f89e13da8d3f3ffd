// shuffle_host.cpp — see shuffle_host.h.
//
// The chain is sequential: draw i's word position depends on every earlier
// rejection.  Its latency per word is what bounds ppo_update's shuffle, so the
// walker works in bands of equal leading-zero count (the zone then moves by a
// constant 2^lz per accepted draw) and, with AVX-512, tests 16 words against 8
// candidate rejection counts at once and resolves the path with bit scans.
#include "shuffle_host.h"

#include <immintrin.h>
#include <cstdlib>
#include <string.h>

namespace bppo_host {

typedef uint32_t u32;
typedef uint64_t u64;

// ------------------------------------------------------------------ ChaCha --
static inline u32 rotl(u32 v, int n) { return (v << n) | (v >> (32 - n)); }

static void chacha12_block_scalar(const u32 key[8], u64 ctr, u64 stream, u32 out[16]) {
    u32 x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, key[0], key[1], key[2], key[3],
                 key[4], key[5], key[6], key[7], (u32)ctr, (u32)(ctr >> 32), (u32)stream,
                 (u32)(stream >> 32)};
    u32 s[16];
    memcpy(s, x, sizeof s);
#define QR(a, b, c, d)                              \
    x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);     \
    x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);     \
    x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);      \
    x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    for (int r = 0; r < 6; r++) {
        QR(0, 4, 8, 12) QR(1, 5, 9, 13) QR(2, 6, 10, 14) QR(3, 7, 11, 15)
        QR(0, 5, 10, 15) QR(1, 6, 11, 12) QR(2, 7, 8, 13) QR(3, 4, 9, 14)
    }
#undef QR
    for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

// 8 consecutive blocks (counters ctr .. ctr+7) -> 128 words in stream order
__attribute__((target("avx2"))) static void chacha12_8blocks_avx2(const u32 key[8], u64 ctr, u64 stream,
                                                                  u32 *out) {
    __m256i x[16], s[16];
    x[0] = _mm256_set1_epi32(0x61707865); x[1] = _mm256_set1_epi32(0x3320646e);
    x[2] = _mm256_set1_epi32(0x79622d32); x[3] = _mm256_set1_epi32(0x6b206574);
    for (int i = 0; i < 8; i++) x[4 + i] = _mm256_set1_epi32((int)key[i]);
    // 64-bit counters ctr+l split into low / high words (carry handled per lane)
    u32 lo[8], hi[8];
    for (int l = 0; l < 8; l++) { u64 c = ctr + (u64)l; lo[l] = (u32)c; hi[l] = (u32)(c >> 32); }
    x[12] = _mm256_loadu_si256((const __m256i *)lo);
    x[13] = _mm256_loadu_si256((const __m256i *)hi);
    x[14] = _mm256_set1_epi32((int)(u32)stream);
    x[15] = _mm256_set1_epi32((int)(u32)(stream >> 32));
    for (int i = 0; i < 16; i++) s[i] = x[i];
    const __m256i r16 = _mm256_setr_epi8(2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13,
                                         2, 3, 0, 1, 6, 7, 4, 5, 10, 11, 8, 9, 14, 15, 12, 13);
    const __m256i r8 = _mm256_setr_epi8(3, 0, 1, 2, 7, 4, 5, 6, 11, 8, 9, 10, 15, 12, 13, 14,
                                        3, 0, 1, 2, 7, 4, 5, 6, 11, 8, 9, 10, 15, 12, 13, 14);
#define ROTV(v, n) _mm256_or_si256(_mm256_slli_epi32(v, n), _mm256_srli_epi32(v, 32 - n))
#define QRV(a, b, c, d)                                                                   \
    x[a] = _mm256_add_epi32(x[a], x[b]); x[d] = _mm256_shuffle_epi8(_mm256_xor_si256(x[d], x[a]), r16); \
    x[c] = _mm256_add_epi32(x[c], x[d]); x[b] = ROTV(_mm256_xor_si256(x[b], x[c]), 12);              \
    x[a] = _mm256_add_epi32(x[a], x[b]); x[d] = _mm256_shuffle_epi8(_mm256_xor_si256(x[d], x[a]), r8);  \
    x[c] = _mm256_add_epi32(x[c], x[d]); x[b] = ROTV(_mm256_xor_si256(x[b], x[c]), 7);
    for (int r = 0; r < 6; r++) {
        QRV(0, 4, 8, 12) QRV(1, 5, 9, 13) QRV(2, 6, 10, 14) QRV(3, 7, 11, 15)
        QRV(0, 5, 10, 15) QRV(1, 6, 11, 12) QRV(2, 7, 8, 13) QRV(3, 4, 9, 14)
    }
#undef QRV
#undef ROTV
    for (int i = 0; i < 16; i++) x[i] = _mm256_add_epi32(x[i], s[i]);
    // transpose: lane l of x[i] is word i of block l
    alignas(32) u32 t[16][8];
    for (int i = 0; i < 16; i++) _mm256_store_si256((__m256i *)t[i], x[i]);
    for (int l = 0; l < 8; l++)
        for (int i = 0; i < 16; i++) out[l * 16 + i] = t[i][l];
}

// 16 consecutive blocks -> 256 words (AVX-512: native rotates)
__attribute__((target("avx512f"))) static void chacha12_16blocks_avx512(const u32 key[8], u64 ctr, u64 stream,
                                                                       u32 *out) {
    __m512i x[16], s[16];
    x[0] = _mm512_set1_epi32(0x61707865); x[1] = _mm512_set1_epi32(0x3320646e);
    x[2] = _mm512_set1_epi32(0x79622d32); x[3] = _mm512_set1_epi32(0x6b206574);
    for (int i = 0; i < 8; i++) x[4 + i] = _mm512_set1_epi32((int)key[i]);
    u32 lo[16], hi[16];
    for (int l = 0; l < 16; l++) { u64 c = ctr + (u64)l; lo[l] = (u32)c; hi[l] = (u32)(c >> 32); }
    x[12] = _mm512_loadu_si512((const void *)lo);
    x[13] = _mm512_loadu_si512((const void *)hi);
    x[14] = _mm512_set1_epi32((int)(u32)stream);
    x[15] = _mm512_set1_epi32((int)(u32)(stream >> 32));
    for (int i = 0; i < 16; i++) s[i] = x[i];
#define QRZ(a, b, c, d)                                                                     \
    x[a] = _mm512_add_epi32(x[a], x[b]); x[d] = _mm512_rol_epi32(_mm512_xor_si512(x[d], x[a]), 16); \
    x[c] = _mm512_add_epi32(x[c], x[d]); x[b] = _mm512_rol_epi32(_mm512_xor_si512(x[b], x[c]), 12); \
    x[a] = _mm512_add_epi32(x[a], x[b]); x[d] = _mm512_rol_epi32(_mm512_xor_si512(x[d], x[a]), 8);  \
    x[c] = _mm512_add_epi32(x[c], x[d]); x[b] = _mm512_rol_epi32(_mm512_xor_si512(x[b], x[c]), 7);
    for (int r = 0; r < 6; r++) {
        QRZ(0, 4, 8, 12) QRZ(1, 5, 9, 13) QRZ(2, 6, 10, 14) QRZ(3, 7, 11, 15)
        QRZ(0, 5, 10, 15) QRZ(1, 6, 11, 12) QRZ(2, 7, 8, 13) QRZ(3, 4, 9, 14)
    }
#undef QRZ
    alignas(64) u32 t[16][16];
    for (int i = 0; i < 16; i++) _mm512_store_si512((void *)t[i], _mm512_add_epi32(x[i], s[i]));
    for (int l = 0; l < 16; l++)
        for (int i = 0; i < 16; i++) out[l * 16 + i] = t[i][l];
}

static bool have_avx512() {
    static int v = -1;
    if (v < 0) { __builtin_cpu_init(); v = __builtin_cpu_supports("avx512f") ? 1 : 0; }
    return v == 1;
}

static bool have_avx2() {
    static int v = -1;
    if (v < 0) { __builtin_cpu_init(); v = __builtin_cpu_supports("avx2") ? 1 : 0; }
    return v == 1;
}

void chacha12_words(const u32 key[8], u64 stream, u64 pos, u32 *out, size_t n) {
    size_t o = 0;
    u32 blk[128];
    // leading partial block
    if (pos & 15) {
        chacha12_block_scalar(key, pos >> 4, stream, blk);
        for (u64 w = pos & 15; w < 16 && o < n; w++) out[o++] = blk[w];
    }
    u64 b = (pos + o) >> 4;
    if (have_avx512()) {
        while (n - o >= 256) {
            chacha12_16blocks_avx512(key, b, stream, out + o);
            o += 256; b += 16;
        }
    }
    const bool v8 = have_avx2();
    while (n - o >= 128 && v8) {
        chacha12_8blocks_avx2(key, b, stream, out + o);
        o += 128; b += 8;
    }
    while (o < n) {
        chacha12_block_scalar(key, b, stream, blk);
        for (int w = 0; w < 16 && o < n; w++) out[o++] = blk[w];
        b++;
    }
}

// ------------------------------------------------------------------- walk --
// band [lowr, 2*lowr): every range there has the same leading-zero count lz
static inline size_t walk_scalar(const u32 *w, size_t nw, u32 *rp, u32 *J) {
    u32 r = *rp;
    size_t p = 0;
    while (r >= 2 && p < nw) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2 && p < nw) {
            const u64 m = (u64)w[p++] * r;
            J[r - 1] = (u32)(m >> 32);           // a rejected draw's slot is rewritten by the accept
            const u32 acc = (u32)m <= z;
            r -= acc;
            z -= acc ? s : 0u;
        }
    }
    *rp = r;
    return p;
}

__attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt")))
static size_t walk_avx512(const u32 *w, size_t nw, u32 *rp, u32 *J) {
    u32 r = *rp;
    size_t p = 0;
    const __m512i kidx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i rev = _mm512_setr_epi32(15, 14, 13, 12, 11, 10, 9, 8, 7, 6, 5, 4, 3, 2, 1, 0);
    while (r >= 2 && p < nw) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        // 16-word blocks while the whole block stays inside the band and the buffer
        while (r >= lowr + 24 && p + 16 <= nw) {
            const u32 z = (r << lz) - 1u;
            const __m512i wv = _mm512_loadu_si512((const void *)(w + p));
            const __m512i rk = _mm512_sub_epi32(_mm512_set1_epi32((int)r), kidx);
            __m512i lo = _mm512_mullo_epi32(wv, rk);                   // lo(w_k (r - k))
            __m512i zz = _mm512_sub_epi32(_mm512_set1_epi32((int)z), _mm512_slli_epi32(kidx, lz));
            const __m512i sv = _mm512_set1_epi32((int)s);
            u64 M[8];                                                  // bit k: word k accepted after j rejections
            for (int j = 0; j < 8; j++) {
                M[j] = (u64)_mm512_cmple_epu32_mask(lo, zz);
                lo = _mm512_add_epi32(lo, wv);
                zz = _mm512_add_epi32(zz, sv);
            }
            u64 k = 0, rejmask = 0;
            for (int j = 0; j < 8; j++) {                              // j-th rejection: first 0 of M[j] at >= k
                const u64 rej = ((~M[j]) & 0xFFFFull & (~0ull << k)) | (1ull << 16);
                const u64 kz = (u64)__builtin_ctzll(rej);
                rejmask |= 1ull << kz;
                k = kz + 1;
            }
            const u32 stop = k > 16 ? 16u : (u32)k;                    // 8th rejection ends the block early
            const u32 valid = (u32)((1u << stop) - 1u);
            const u32 am = (~(u32)rejmask) & valid;
            const u32 acc = (u32)__builtin_popcount(am);
            // m-th accepted word draws with range r - m
            const __m512i wc = _mm512_maskz_compress_epi32((__mmask16)am, wv);
            const __m512i pe = _mm512_mul_epu32(wc, rk);
            const __m512i po = _mm512_mul_epu32(_mm512_srli_epi64(wc, 32), _mm512_srli_epi64(rk, 32));
            const __m512i hi = _mm512_mask_blend_epi32((__mmask16)0xAAAA, _mm512_srli_epi64(pe, 32), po);
            const __m512i hr = _mm512_permutexvar_epi32(rev, hi);
            const __mmask16 sm = (__mmask16)(0xFFFFu & ~((1u << (16 - acc)) - 1u));
            _mm512_mask_storeu_epi32((void *)(J + r - 16), sm, hr);
            r -= acc;
            p += stop;
        }
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2 && p < nw) {
            const u64 m = (u64)w[p++] * r;
            J[r - 1] = (u32)(m >> 32);
            const u32 a = (u32)m <= z;
            r -= a;
            z -= a ? s : 0u;
            if (r >= lowr + 24 && p + 16 <= nw) break;   // back to blocks
        }
    }
    *rp = r;
    return p;
}

// the same chain without the J stores: only the range r advances (speculative
// and true walks record checkpoint states; the GPU rebuilds J from them)
static inline size_t walk_scalar_nj(const u32 *w, size_t nw, u32 *rp) {
    u32 r = *rp;
    size_t p = 0;
    while (r >= 2 && p < nw) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2 && p < nw) {
            const u32 lo = w[p++] * r;
            const u32 acc = lo <= z;
            r -= acc;
            z -= acc ? s : 0u;
        }
    }
    *rp = r;
    return p;
}

// 32 words per block, NH hypotheses m = rejections so far (r_j = r - j + m).
// M[m] = acceptance of every word under hypothesis m.  The resolution keeps the
// mask L of positions consumed so far: the next rejection under hypothesis m is
// the lowest bit of Z_m = ~M[m] above L, so L' = blsmsk(Z_m & ~L) — two 1-cycle
// ops per step.  Bits >= 32 of Z are set (virtual rejections past the block),
// so after the NH steps P = popcount(L) gives the block exactly:
//   consumed = min(P, 32), accepted = P - NH
// (NH rejections inside the block: P = last one + 1; fewer: P = 32 + the
// virtual ones).  9 rejections are expected per 32 words; NH = 10 (measured
// fastest on the EPYC 9575F: 0.48 ns/word vs 0.57 at NH = 16) ends the blocks
// with more rejections early, at their 10th.
template <int NH>
__attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt")))
static size_t walk_avx512_nj_t(const u32 *w, size_t nw, u32 *rp) {
    u32 r = *rp;
    size_t p = 0;
    const __m512i kidx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i kidx16 = _mm512_add_epi32(kidx, _mm512_set1_epi32(16));
    while (r >= 2 && p < nw) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        const __m512i sv = _mm512_set1_epi32((int)s);
        const __m512i kz = _mm512_slli_epi32(kidx, lz), kz16 = _mm512_slli_epi32(kidx16, lz);
        while (r >= lowr + 48 && p + 32 <= nw) {
            const u32 z = (r << lz) - 1u;
            const __m512i w0 = _mm512_loadu_si512((const void *)(w + p));
            const __m512i w1 = _mm512_loadu_si512((const void *)(w + p + 16));
            const __m512i rv = _mm512_set1_epi32((int)r), zv = _mm512_set1_epi32((int)z);
            __m512i lo0 = _mm512_mullo_epi32(w0, _mm512_sub_epi32(rv, kidx));
            __m512i lo1 = _mm512_mullo_epi32(w1, _mm512_sub_epi32(rv, kidx16));
            __m512i zz0 = _mm512_sub_epi32(zv, kz), zz1 = _mm512_sub_epi32(zv, kz16);
            u64 Z[NH];
            for (int j = 0; j < NH; j++) {
                const __mmask32 m = _mm512_kunpackw(_mm512_cmple_epu32_mask(lo1, zz1), _mm512_cmple_epu32_mask(lo0, zz0));
                Z[j] = (u64)(u32)~_cvtmask32_u32(m) | 0xFFFFFFFF00000000ull;
                lo0 = _mm512_add_epi32(lo0, w0); lo1 = _mm512_add_epi32(lo1, w1);
                zz0 = _mm512_add_epi32(zz0, sv); zz1 = _mm512_add_epi32(zz1, sv);
            }
            u64 L = 0;
            for (int j = 0; j < NH; j++) L = _blsmsk_u64(Z[j] & ~L);
            const u32 P = (u32)__builtin_popcountll(L);
            r -= P - NH;
            p += P < 32 ? P : 32;
        }
        u32 z = (r << lz) - 1u;
        while (r >= lowr && r >= 2 && p < nw) {
            const u32 lo = w[p++] * r;
            const u32 a = lo <= z;
            r -= a;
            z -= a ? s : 0u;
            if (r >= lowr + 48 && p + 32 <= nw) break;
        }
    }
    *rp = r;
    return p;
}
static size_t walk_avx512_nj(const u32 *w, size_t nw, u32 *rp) { return walk_avx512_nj_t<10>(w, nw, rp); }

// one 32-word block of walk_avx512_nj_t (the caller checked r >= lowr + 48 and
// 32 words left): returns the words consumed, advances r
template <int NH>
__attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt"), always_inline))
static inline u32 block32(const u32 *w, u32 &r) {
    const int lz = __builtin_clz(r);
    const u32 z = (r << lz) - 1u;
    const __m512i kidx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i kidx16 = _mm512_add_epi32(kidx, _mm512_set1_epi32(16));
    const __m512i sv = _mm512_set1_epi32((int)(1u << lz));
    const __m512i w0 = _mm512_loadu_si512((const void *)w);
    const __m512i w1 = _mm512_loadu_si512((const void *)(w + 16));
    const __m512i rv = _mm512_set1_epi32((int)r), zv = _mm512_set1_epi32((int)z);
    __m512i lo0 = _mm512_mullo_epi32(w0, _mm512_sub_epi32(rv, kidx));
    __m512i lo1 = _mm512_mullo_epi32(w1, _mm512_sub_epi32(rv, kidx16));
    __m512i zz0 = _mm512_sub_epi32(zv, _mm512_slli_epi32(kidx, lz));
    __m512i zz1 = _mm512_sub_epi32(zv, _mm512_slli_epi32(kidx16, lz));
    u64 Z[NH];
    for (int j = 0; j < NH; j++) {
        const __mmask32 m = _mm512_kunpackw(_mm512_cmple_epu32_mask(lo1, zz1), _mm512_cmple_epu32_mask(lo0, zz0));
        Z[j] = (u64)(u32)~_cvtmask32_u32(m) | 0xFFFFFFFF00000000ull;
        lo0 = _mm512_add_epi32(lo0, w0); lo1 = _mm512_add_epi32(lo1, w1);
        zz0 = _mm512_add_epi32(zz0, sv); zz1 = _mm512_add_epi32(zz1, sv);
    }
    u64 L = 0;
    for (int j = 0; j < NH; j++) L = _blsmsk_u64(Z[j] & ~L);
    const u32 P = (u32)__builtin_popcountll(L);
    r -= P - NH;
    return P < 32 ? P : 32;
}

static inline bool block_ok(u32 r, size_t p, size_t nw) {
    const u32 lowr = 1u << (31 - __builtin_clz(r));
    return r >= lowr + 48 && p + 32 <= nw;
}

// single draws until a full in-band block fits again (or the words / the chain end)
static inline void steps_until_block(const u32 *w, size_t nw, size_t &p, u32 &r) {
    while (r >= 2 && p < nw) {
        if (r >= 2 && block_ok(r, p, nw)) return;
        const int lz = __builtin_clz(r);
        const u32 lo = w[p++] * r;
        r -= lo <= (r << lz) - 1u;
    }
}

// two independent chains, one block of each per iteration: the out-of-order core
// overlaps their dependency chains (0.24-0.30 ns per word per chain measured on the
// box with scripts/microbench/walk2_bench.cpp, vs 0.42-0.44 for one chain)
__attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt")))
static void walk2_avx512_nj(const u32 *wa, size_t na, u32 *rap, size_t *ua, const u32 *wb, size_t nb, u32 *rbp,
                            size_t *ub) {
    u32 ra = *rap, rb = *rbp;
    size_t pa = 0, pb = 0;
    for (;;) {
        while (block_ok(ra, pa, na) && block_ok(rb, pb, nb)) {
            pa += block32<10>(wa + pa, ra);
            pb += block32<10>(wb + pb, rb);
        }
        steps_until_block(wa, na, pa, ra);
        steps_until_block(wb, nb, pb, rb);
        const bool da = ra < 2 || pa >= na || !block_ok(ra, pa, na);
        const bool db = rb < 2 || pb >= nb || !block_ok(rb, pb, nb);
        if (da || db) break;        // one chain has reached its end or the end of its words
    }
    *rap = ra; *rbp = rb; *ua = pa; *ub = pb;
}

static int isa_level() {
    static int v = -1;
    if (v < 0) {
        __builtin_cpu_init();
        v = (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw") &&
             __builtin_cpu_supports("avx512vl") && __builtin_cpu_supports("avx512dq")) ? 2 : 1;
    }
    return v;
}

int chain_walk_isa() { return isa_level(); }

size_t chain_walk_nj(const u32 *w, size_t nw, u32 *r) {
    if (isa_level() == 2) return walk_avx512_nj(w, nw, r);
    return walk_scalar_nj(w, nw, r);
}

void chain_walk2_nj(const u32 *wa, size_t na, u32 *ra, size_t *ua, const u32 *wb, size_t nb, u32 *rb, size_t *ub) {
    if (isa_level() == 2) return walk2_avx512_nj(wa, na, ra, ua, wb, nb, rb, ub);
    *ua = walk_scalar_nj(wa, na, ra);
    *ub = walk_scalar_nj(wb, nb, rb);
}

size_t chain_walk(const u32 *w, size_t nw, u32 *r, u32 *J) {
    if (isa_level() == 2) return walk_avx512(w, nw, r, J);
    return walk_scalar(w, nw, r, J);
}

}  // namespace bppo_host

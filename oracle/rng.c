/*
 * rng.c — restatement of the RNG stack burn-ppo uses (TEST INFRASTRUCTURE ONLY).
 *
 * Reference call sites: main.rs:189 (StdRng::seed_from_u64(config.seed)),
 * main.rs:1964 / cartpole.rs:92-95 (per-env StdRng::seed_from_u64(seed + i)),
 * utils.rs:20 (gen_range(1e-10f32..1.0)), cartpole.rs:275-278
 * (gen_range(-0.05..0.05)), liars_dice.rs:194 (gen_range(1..=6) as u8),
 * ppo.rs:1816 (indices.shuffle(rng)), checkpoint.rs:390-400 (fill_bytes 32 B).
 *
 * Restated (not vendored, verify): rand 0.8.5, rand_core 0.6.4, rand_chacha
 * 0.3.1 (Cargo.lock:4962-5004).  The ChaCha core is pinned against OpenSSL's
 * chacha20 (tests/golden/chacha20_openssl.json, made by
 * tests/golden/make_chacha_fixture.js) and the RFC 8439 block vector.
 */
#include <string.h>
#include "oracle.h"

#define ROTL(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d)                \
    a += b; d ^= a; d = ROTL(d, 16);  \
    c += d; b ^= c; b = ROTL(b, 12);  \
    a += b; d ^= a; d = ROTL(d, 8);   \
    c += d; b ^= c; b = ROTL(b, 7);

/* rand_chacha guts.rs refill_wide: constants, key, 64-bit counter, stream. */
void or_chacha_block(const uint32_t key[8], uint64_t counter, uint64_t stream, int rounds,
                     uint32_t out[16]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
    for (int i = 0; i < 8; i++) s[4 + i] = key[i];
    s[12] = (uint32_t)counter; s[13] = (uint32_t)(counter >> 32);
    s[14] = (uint32_t)stream;  s[15] = (uint32_t)(stream >> 32);
    memcpy(x, s, sizeof s);
    for (int r = 0; r < rounds; r += 2) {
        QR(x[0], x[4], x[8], x[12]); QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]); QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]); QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]); QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

/* rand_core 0.6.4 SeedableRng::seed_from_u64: PCG32 fills the 32-byte seed. */
void or_rng_seed_key(uint64_t state, uint32_t key_out[8]) {
    const uint64_t MUL = 6364136223846793005ULL, INC = 11634580027462260723ULL;
    for (int i = 0; i < 8; i++) {
        state = state * MUL + INC;
        uint32_t xorshifted = (uint32_t)(((state >> 18) ^ state) >> 27);
        uint32_t rot = (uint32_t)(state >> 59);
        key_out[i] = (xorshifted >> rot) | (xorshifted << ((32 - rot) & 31));
    }
}

void or_rng_from_key(or_rng *r, const uint32_t key[8], int rounds) {
    memcpy(r->key, key, sizeof r->key);
    r->stream = 0;
    r->word_pos = 0;
    r->cached_block = UINT64_MAX;
    r->rounds = rounds;
}

void or_rng_seed_u64(or_rng *r, uint64_t seed) {
    uint32_t k[8];
    or_rng_seed_key(seed, k);
    or_rng_from_key(r, k, 12);
}

/* rand_core BlockRng::next_u32: consecutive keystream words. */
uint32_t or_rng_next_u32(or_rng *r) {
    uint64_t blk = r->word_pos >> 4;
    if (blk != r->cached_block) {
        or_chacha_block(r->key, blk, r->stream, r->rounds, r->block);
        r->cached_block = blk;
    }
    return r->block[r->word_pos++ & 15];
}

/* BlockRng::next_u64: low word first, including the buffer-edge case. */
uint64_t or_rng_next_u64(or_rng *r) {
    uint64_t lo = or_rng_next_u32(r);
    uint64_t hi = or_rng_next_u32(r);
    return (hi << 32) | lo;
}

/* BlockRng::fill_bytes via fill_via_u32_chunks: ceil(n/4) words, LE bytes. */
void or_rng_fill_bytes(or_rng *r, uint8_t *dst, size_t n) {
    size_t i = 0;
    while (i < n) {
        uint32_t w = or_rng_next_u32(r);
        for (int b = 0; b < 4 && i < n; b++, i++) dst[i] = (uint8_t)(w >> (8 * b));
    }
}

/* rand 0.8.5 UniformFloat<f32>::sample_single (range [low, high)). */
float or_gen_range_f32(or_rng *r, float low, float high) {
    float scale = high - low;
    for (;;) {
        uint32_t bits = (or_rng_next_u32(r) >> 9) | 0x3F800000u;
        float v12;
        memcpy(&v12, &bits, 4);
        float v01 = v12 - 1.0f;
        float res = v01 * scale + low;   /* two roundings: no contraction */
        if (res < high) return res;
    }
}

/* rand 0.8.5 UniformInt<u32>::sample_single -> sample_single_inclusive(low, high-1):
 * widening multiply, zone = (range << leading_zeros(range)) - 1. */
uint32_t or_gen_range_u32(or_rng *r, uint32_t low, uint32_t high) {
    uint32_t range = high - 1 - low + 1;
    if (range == 0) return or_rng_next_u32(r);
    uint32_t zone = (range << __builtin_clz(range)) - 1u;
    for (;;) {
        uint64_t m = (uint64_t)or_rng_next_u32(r) * (uint64_t)range;
        uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
        if (lo <= zone) return low + hi;
    }
}

/* rand 0.8.5 UniformInt<u64>::sample_single ([low, high)), the form
 * `gen_range(0..n)` takes for usize on 64-bit targets (opponent_pool.rs:109):
 * next_u64 (two words, low first), 64x64 -> 128 widening multiply, zone
 * (range << lz(range)) - 1.  Restated, verify. */
uint64_t or_gen_range_u64(or_rng *r, uint64_t low, uint64_t high) {
    uint64_t range = high - 1 - low + 1;
    if (range == 0) return or_rng_next_u64(r);
    uint64_t zone = (range << __builtin_clzll(range)) - 1u;
    for (;;) {
        unsigned __int128 m = (unsigned __int128)or_rng_next_u64(r) * range;
        uint64_t lo = (uint64_t)m, hi = (uint64_t)(m >> 64);
        if (lo <= zone) return low + hi;
    }
}

/* UniformInt<u8>::sample_single_inclusive: u32 arithmetic, modulus zone. */
uint8_t or_gen_range_u8_incl(or_rng *r, uint8_t low, uint8_t high) {
    uint32_t range = (uint32_t)(uint8_t)(high - low) + 1u;
    uint32_t ints_to_reject = (UINT32_MAX - range + 1u) % range;
    uint32_t zone = UINT32_MAX - ints_to_reject;
    for (;;) {
        uint64_t m = (uint64_t)or_rng_next_u32(r) * (uint64_t)range;
        uint32_t lo = (uint32_t)m, hi = (uint32_t)(m >> 32);
        if (lo <= zone) return (uint8_t)(low + hi);
    }
}

/* rand 0.8.5 SliceRandom::shuffle: for i in (1..len).rev() swap(i, gen_index(i+1)). */
void or_shuffle_u32(or_rng *r, uint32_t *v, size_t n) {
    if (n < 2) return;
    for (size_t i = n - 1; i >= 1; i--) {
        uint32_t j = or_gen_range_u32(r, 0, (uint32_t)(i + 1));
        uint32_t t = v[i]; v[i] = v[j]; v[j] = t;
    }
}

/* the swap targets of or_shuffle_u32 (J[i] = gen_range(0..i+1), i = n-1..1; J[0] = 0)
 * and the sequential swap pass that turns them into the permutation */
void or_shuffle_targets(or_rng *r, uint32_t *J, size_t n) {
    if (n == 0) return;
    J[0] = 0;
    for (size_t i = n - 1; i >= 1; i--) J[i] = or_gen_range_u32(r, 0, (uint32_t)(i + 1));
}

void or_apply_swaps(const uint32_t *J, uint32_t *v, size_t n) {
    for (size_t i = n; i-- > 1;) {
        uint32_t j = J[i], t = v[i];
        v[i] = v[j]; v[j] = t;
    }
}

void or_rng_words(uint64_t seed, uint64_t skip, uint32_t *out, size_t n) {
    or_rng r;
    or_rng_seed_u64(&r, seed);
    r.word_pos = skip;
    for (size_t i = 0; i < n; i++) out[i] = or_rng_next_u32(&r);
}

void or_rng_words_key(const uint32_t key[8], int rounds, uint64_t skip, uint32_t *out, size_t n) {
    or_rng r;
    or_rng_from_key(&r, key, rounds);
    r.word_pos = skip;
    for (size_t i = 0; i < n; i++) out[i] = or_rng_next_u32(&r);
}

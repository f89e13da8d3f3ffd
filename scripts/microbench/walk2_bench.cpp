// walk2_bench.cpp — is the host shuffle walker latency-bound?  Compares one
// chain walked alone with two independent chains walked in one thread, their
// 32-word blocks interleaved (the same block math as shuffle_host.cpp
// walk_avx512_nj_t, NH = 10), and checks both against the engine's walker.
//   g++ -O3 -march=native -std=c++17 -I../../burn-ppo_amd/csrc walk2_bench.cpp \
//       ../../burn-ppo_amd/csrc/shuffle_host.cpp -o walk2_bench
#include <immintrin.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <ctime>
#include <cstdlib>
#include <thread>
#include <vector>
#include "shuffle_host.h"

typedef uint32_t u32;
typedef uint64_t u64;
static const int NH = 10;

struct Ch { const u32 *w; size_t nw, p; u32 r; };

// one 32-word block of chain c if it is inside a band and the buffer; returns
// false when the chain needs the scalar tail (band edge, end of buffer)
__attribute__((target("avx512f,avx512bw,avx512vl,avx512dq,bmi,bmi2,popcnt")))
static inline bool block(Ch &c) {
    const u32 r = c.r;
    if (r < 2) return false;
    const int lz = __builtin_clz(r);
    const u32 lowr = 1u << (31 - lz), s = 1u << lz;
    if (!(r >= lowr + 48 && c.p + 32 <= c.nw)) return false;
    const __m512i kidx = _mm512_setr_epi32(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15);
    const __m512i kidx16 = _mm512_add_epi32(kidx, _mm512_set1_epi32(16));
    const __m512i sv = _mm512_set1_epi32((int)s);
    const u32 z = (r << lz) - 1u;
    const __m512i w0 = _mm512_loadu_si512((const void *)(c.w + c.p));
    const __m512i w1 = _mm512_loadu_si512((const void *)(c.w + c.p + 16));
    const __m512i rv = _mm512_set1_epi32((int)r), zv = _mm512_set1_epi32((int)z);
    __m512i lo0 = _mm512_mullo_epi32(w0, _mm512_sub_epi32(rv, kidx));
    __m512i lo1 = _mm512_mullo_epi32(w1, _mm512_sub_epi32(rv, kidx16));
    __m512i zz0 = _mm512_sub_epi32(zv, _mm512_slli_epi32(kidx, lz)), zz1 = _mm512_sub_epi32(zv, _mm512_slli_epi32(kidx16, lz));
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
    c.r = r - (P - NH);
    c.p += P < 32 ? P : 32;
    return true;
}
static inline void tail(Ch &c) {        // scalar steps until a block fits again
    u32 r = c.r;
    while (r >= 2 && c.p < c.nw) {
        const int lz = __builtin_clz(r);
        const u32 lowr = 1u << (31 - lz), s = 1u << lz;
        u32 z = (r << lz) - 1u;
        bool brk = false;
        while (r >= lowr && r >= 2 && c.p < c.nw) {
            const u32 lo = c.w[c.p++] * r;
            const u32 a = lo <= z;
            r -= a;
            z -= a ? s : 0u;
            if (r >= lowr + 48 && c.p + 32 <= c.nw) { brk = true; break; }
        }
        if (brk) break;
    }
    c.r = r;
}
static void walk1(Ch &a) {
    while (a.r >= 2 && a.p < a.nw)
        if (!block(a)) tail(a);
}
static void walk2(Ch &a, Ch &b) {
    for (;;) {
        const bool la = a.r >= 2 && a.p < a.nw, lb = b.r >= 2 && b.p < b.nw;
        if (!la && !lb) break;
        if (la && lb) {
            const bool ba = block(a), bb = block(b);
            if (!ba) tail(a);
            if (!bb) tail(b);
        } else if (la) { if (!block(a)) tail(a); }
        else { if (!block(b)) tail(b); }
    }
}

// self-made words: ChaCha12 pieces of 1024 words into an L1-resident buffer,
// (a) made then walked, (b) the next piece made in the same loop iteration as
// the current piece is walked (out-of-order overlap of the two)
static size_t walk_selfgen(const u32 key[8], u64 stream, u64 pos, u32 *r, bool overlap) {
    alignas(64) static thread_local u32 buf[2][1024 + 32];
    const u64 p0 = pos;
    int cur = 0;
    bppo_host::chacha12_words(key, stream, pos, buf[cur], 1024);
    while (*r >= 2) {
        if (overlap) bppo_host::chacha12_words(key, stream, pos + 1024, buf[cur ^ 1], 1024);
        Ch c{buf[cur], 1024, 0, *r};
        walk1(c);
        *r = c.r;
        if (c.p < 1024) { pos += c.p; break; }
        pos += 1024;
        cur ^= 1;
        if (!overlap) bppo_host::chacha12_words(key, stream, pos, buf[cur], 1024);
    }
    return (size_t)(pos - p0);
}

// T threads each walking one chain at once over shared read-only words: does
// the per-thread rate hold as the host's cores fill?
static void scaling(const std::vector<u32> &wa, size_t pa) {
    const char *tl = getenv("WALK_THREADS");
    std::vector<int> Ts = tl ? std::vector<int>{atoi(tl)} : std::vector<int>{1, 2, 4, 8, 12, 16};
    const int reps = getenv("WALK_REPS") ? atoi(getenv("WALK_REPS")) : 1;
    for (int rep = 0; rep < reps; rep++)
    for (int T : Ts) {
        std::vector<std::thread> th;
        std::vector<double> ns(T), cpu(T);
        for (int t = 0; t < T; t++)
            th.emplace_back([&, t]() {
                Ch a{wa.data() + 64 * t, wa.size() - 64 * t, 0, 8388608u};
                timespec c0, c1;
                clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
                auto t0 = std::chrono::steady_clock::now();
                walk1(a);
                ns[t] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / a.p * 1e9;
                clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
                cpu[t] = ((c1.tv_sec - c0.tv_sec) * 1e9 + (c1.tv_nsec - c0.tv_nsec)) / a.p;
            });
        for (auto &x : th) x.join();
        double mx = 0, sm = 0, sc = 0;
        for (int t = 0; t < T; t++) { mx = std::max(mx, ns[t]); sm += ns[t]; sc += cpu[t]; }
        printf("threads %2d: wall mean %.3f max %.3f | cpu mean %.3f ns/word per thread\n", T, sm / T, mx, sc / T);
    }
    (void)pa;
}

int main() {
    const u32 n = 8388608;
    const size_t W = 12000000;
    std::vector<u32> wa(W), wb(W);
    u32 key[8] = {9, 8, 7, 6, 5, 4, 3, 2};
    bppo_host::chacha12_words(key, 3, 0, wa.data(), W);
    bppo_host::chacha12_words(key, 4, 0, wb.data(), W);
    u32 ra = n, rb = n;
    const size_t pa = bppo_host::chain_walk_nj(wa.data(), W, &ra), pb = bppo_host::chain_walk_nj(wb.data(), W, &rb);
    for (int rep = 0; rep < 3; rep++) {
        Ch a{wa.data(), W, 0, n}, b{wb.data(), W, 0, n};
        auto t0 = std::chrono::steady_clock::now();
        walk1(a);
        auto t1 = std::chrono::steady_clock::now();
        Ch a2{wa.data(), W, 0, n}, b2{wb.data(), W, 0, n};
        walk2(a2, b2);
        auto t2 = std::chrono::steady_clock::now();
        const double d1 = std::chrono::duration<double>(t1 - t0).count(), d2 = std::chrono::duration<double>(t2 - t1).count();
        printf("one chain %.3f ns/word | two interleaved %.3f ns/word (per word of both) | ok %d %d %d\n",
               d1 / a.p * 1e9, d2 / (a2.p + b2.p) * 1e9, a.p == pa && a.r == ra, a2.p == pa && a2.r == ra,
               b2.p == pb && b2.r == rb);
    }
    scaling(wa, pa);
    if (getenv("WALK_THREADS")) return 0;
    for (int rep = 0; rep < 2; rep++) {
        for (int ov = 0; ov < 2; ov++) {
            u32 r = n;
            auto t0 = std::chrono::steady_clock::now();
            const size_t used = walk_selfgen(key, 3, 0, &r, ov != 0);
            const double d = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            printf("self-made words (%s): %.3f ns/word | ok %d\n", ov ? "next piece made beside the walk" : "make then walk",
                   d / used * 1e9, used == pa && r == ra);
        }
    }
    return 0;
}

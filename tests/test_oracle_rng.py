"""Oracle RNG stack (oracle/rng.c) pinned against the ChaCha KATs.

rand_chacha's stream is the plain ChaCha keystream, so the core is pinned by
OpenSSL's chacha20 (fixture made by tests/golden/make_chacha_fixture.js) and by
the RFC 8439 section 2.3.2 block vector.  seed_from_u64 / gen_range / shuffle
are restated from rand_core 0.6.4 / rand 0.8.5 (not vendored: parity unpinned
beyond these properties)."""
import ctypes as C
import json
import os

import numpy as np

import oracle_ffi as O

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_chacha20_matches_openssl():
    fx = json.load(open(os.path.join(GOLD, "chacha20_openssl.json")))
    for case in fx["cases"]:
        words = np.array(case["words"], np.uint32)
        for b in range(len(words) // 16):
            got = O.chacha_block(case["key_words"], case["counter"] + b, 0, rounds=20)
            assert np.array_equal(got, words[16 * b:16 * b + 16]), case["counter"]


def test_chacha20_rfc8439_block():
    key = np.frombuffer(bytes(range(32)), np.uint32)
    counter = 1 | (0x09000000 << 32)      # state word 12 = 1, word 13 = nonce[0]
    stream = 0x4A000000                   # words 14-15 = nonce[1], nonce[2]
    got = O.chacha_block(key, counter, stream, rounds=20).tobytes().hex()
    assert got == ("10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
                   "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_stdrng_stream_is_chacha12_keystream():
    key = O.seed_key(42)
    w = O.stdrng_words(42, 80)
    for b in range(5):
        assert np.array_equal(w[16 * b:16 * b + 16], O.chacha_block(key, b, 0, rounds=12))
    # word addressability: skipping k words == drawing k words
    assert np.array_equal(O.stdrng_words(42, 30, skip=50), w[50:80])


def test_seed_from_u64_pcg32_expansion():
    # rand_core 0.6.4 seed_from_u64: PCG32 (MUL 6364136223846793005, INC 11634580027462260723)
    def pcg32(state):
        out = []
        M = (1 << 64) - 1
        for _ in range(8):
            state = (state * 6364136223846793005 + 11634580027462260723) & M
            xs = (((state >> 18) ^ state) >> 27) & 0xFFFFFFFF
            rot = state >> 59
            out.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & 0xFFFFFFFF)
        return out
    for seed in (0, 1, 42, 43, 2**63 - 1):
        assert list(O.seed_key(seed)) == pcg32(seed)


def test_next_u64_and_fill_bytes_consume_consecutive_words():
    L = O.lib()
    r = O.new_rng(7)
    w = O.stdrng_words(7, 80)
    r.word_pos = 63                       # straddle a BlockRng buffer edge
    x = L.or_rng_next_u64(C.byref(r))
    assert x == (int(w[64]) << 32) | int(w[63])
    buf = np.zeros(32, np.uint8)
    L.or_rng_fill_bytes(C.byref(r), buf, 32)   # checkpoint.rs:390-400 draws 32 bytes = 8 words
    assert r.word_pos == 73
    assert np.array_equal(buf.view(np.uint32), w[65:73])


def test_gen_range_f32_gumbel_uses_one_word_and_stays_in_range():
    L = O.lib()
    r = O.new_rng(3)
    w = O.stdrng_words(3, 5000)
    for i in range(5000):
        u = L.or_gen_range_f32(C.byref(r), np.float32(1e-10), np.float32(1.0))
        v = np.array([(int(w[i]) >> 9) | 0x3F800000], np.uint32).view(np.float32)[0] - np.float32(1)
        assert u == np.float32(v * np.float32(1.0) + np.float32(1e-10))
        assert 0.0 < u < 1.0
    assert r.word_pos == 5000


def test_gen_range_u32_zone_and_rejection():
    L = O.lib()
    # range = 2^23 has zone = 2^31 - 1: exactly the words with bit 31 of lo clear accepted
    n = 1 << 23
    r = O.new_rng(11)
    w = O.stdrng_words(11, 400)
    pos = 0
    for _ in range(100):
        got = L.or_gen_range_u32(C.byref(r), 0, n)
        while True:
            m = int(w[pos]) * n
            pos += 1
            if (m & 0xFFFFFFFF) <= (n << 8) - 1:
                break
        assert got == m >> 32
        assert r.word_pos == pos


def test_gen_range_u8_dice_distribution():
    L = O.lib()
    r = O.new_rng(5)
    vals = [L.or_gen_range_u8_incl(C.byref(r), 1, 6) for _ in range(6000)]
    assert set(vals) == {1, 2, 3, 4, 5, 6}
    assert all(900 < vals.count(k) < 1100 for k in range(1, 7))


def test_shuffle_is_permutation_and_fisher_yates_order():
    L = O.lib()
    n = 1000
    a = np.arange(n, dtype=np.uint32)
    r = O.new_rng(9)
    L.or_shuffle_u32(C.byref(r), a, n)
    assert sorted(a.tolist()) == list(range(n))
    # replay: for i in (1..n).rev() swap(i, gen_range(0..i+1))
    b = list(range(n))
    r2 = O.new_rng(9)
    for i in range(n - 1, 0, -1):
        j = L.or_gen_range_u32(C.byref(r2), 0, i + 1)
        b[i], b[j] = b[j], b[i]
    assert a.tolist() == b

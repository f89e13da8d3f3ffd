// shuffle_host.h — host-side pieces of rand 0.8.5's SliceRandom::shuffle on
// StdRng (ChaCha12), the one inherently sequential part of ppo_update
// (ppo.rs:1816).  Plain C++ (compiled with g++; no HIP types).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace bppo_host {

// ChaCha12 words at absolute stream positions [pos, pos+n) (rand_chacha 0.3.1
// layout: 64-bit block counter in words 12-13, stream in 14-15).  SIMD across
// blocks (AVX-512: 16 blocks per step, AVX2: 8); single-threaded.
void chacha12_words(const uint32_t key[8], uint64_t stream, uint64_t pos, uint32_t *out, size_t n);

// The Fisher-Yates draw chain: for i = n-1 .. 1, J[i] = gen_range(0..i+1) with
// UniformInt<u32>'s zone rejection (rand 0.8.5 uniform.rs sample_single_inclusive:
// zone = (range << lz(range)) - 1, accept the word v iff lo(v * range) <= zone,
// result hi(v * range)).  *r is the current range (= i + 1; starts at n).
// Consumes words from w[0 .. nw) and stops when *r < 2 or the buffer is used
// up; returns the number of words consumed.  Runtime dispatch: AVX-512 blocks of
// 16 words where the CPU has it, else the scalar band loop.
size_t chain_walk(const uint32_t *w, size_t nw, uint32_t *r, uint32_t *J);

// chain_walk without writing J (the range r advances exactly the same way)
size_t chain_walk_nj(const uint32_t *w, size_t nw, uint32_t *r);

// two independent chains at once (their blocks interleaved in one loop): walks both
// until EITHER has used all its words or reached r < 2; *ua / *ub = the words each
// consumed (the other chain stops at a block boundary, its state exact).  Same
// chains as chain_walk_nj over the same words.
void chain_walk2_nj(const uint32_t *wa, size_t na, uint32_t *ra, size_t *ua,
                    const uint32_t *wb, size_t nb, uint32_t *rb, size_t *ub);

// 2 = AVX-512 walker, 1 = scalar
int chain_walk_isa();

}  // namespace bppo_host

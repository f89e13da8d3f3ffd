// shuffle_engine.hip — the host side of ppo_update's per-epoch shuffle
// (ppo.rs:1816 `indices.shuffle(rng)`, rand 0.8.5 SliceRandom::shuffle):
//
//   words      : the ChaCha12 words of the main StdRng stream for one update's
//                shuffles: made on the host by producer threads into pinned
//                memory in chunks, in the order the walkers reach them, and
//                independently on the GPU (device copy for the J expansion);
//   true walk  : the sequential rejection chain -> J[i] = gen_range(0..i+1),
//                i = n-1..1 (shuffle_host.cpp), epoch by epoch;
//   speculation: epoch e >= 1 starts where epoch e-1 ends, known only after
//                walking it, and the next update's first epoch starts `gap`
//                words (the rollout's T*N*A Gumbel draws) after this update's
//                last one.  K walkers start at every such boundary at once, at
//                guesses spread around the expected position, recording the
//                remaining range r at every SHUF_CK-th word position.  The true
//                walk of an epoch runs from the real boundary only until, at a
//                checkpoint, its r equals a speculative walk's r at the same
//                position: from there the two walks are the same walk, so the
//                epoch's end and J[0 .. r) come from the speculative one.  With
//                no meeting the true walk finishes the epoch itself.  The walks
//                for the next update's first epoch ("carry" set) run during this
//                update's job, on this job's word buffer (double-buffered).
//   copy stream: each epoch's J to HBM; an event per epoch lets the compute
//                stream wait for exactly that epoch.
//
// Results are identical to the single sequential walk (the RNG word positions
// and every J[i]); only the wall time changes.  The engine runs one update
// ahead: the next update's shuffles start at end + T*N*A (the rollout's Gumbel
// draws use exactly one word per (env, action)).  A different start (KL early
// stop, rng_set) cancels and restarts.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <pthread.h>
#include <x86intrin.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>
#include "bppo_internal.h"
#include "shuffle_host.h"

namespace bppo {

static bool shuf_debug() {
    static int v = -1;
    if (v < 0) v = getenv("BPPO_SHUFFLE_DEBUG") ? 1 : 0;
    return v == 1;
}
static double shuf_t_ms() {   // debug timestamps: ms since the first call
    static const auto t0 = std::chrono::steady_clock::now();
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}
#define SHUF_LOG(...)                                        \
    do {                                                     \
        if (shuf_debug()) { fprintf(stderr, "%9.3f ", shuf_t_ms()); fprintf(stderr, __VA_ARGS__); fflush(stderr); } \
    } while (0)

// ChaCha12 words [base, base + len) (base a multiple of 16): one block per thread
__global__ void k_chacha_words(Key8 key, uint64_t stream, uint64_t base, uint64_t len, uint32_t *out) {
    const uint64_t b = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
    if (b * 16 >= len) return;
    uint32_t blk[16];
    chacha12_block(key, (base >> 4) + b, stream, blk);
    uint4 *o = reinterpret_cast<uint4 *>(out + b * 16);
    o[0] = make_uint4(blk[0], blk[1], blk[2], blk[3]);
    o[1] = make_uint4(blk[4], blk[5], blk[6], blk[7]);
    o[2] = make_uint4(blk[8], blk[9], blk[10], blk[11]);
    o[3] = make_uint4(blk[12], blk[13], blk[14], blk[15]);
}

// J from walk segments.  Segments are consecutive pieces of the epoch's chain
// (segment i covers words [pos0, pos1) from range r0, <= SHUF_CK words), ONE WAVE per
// segment, 64 words per step: lane j holds word j of the step and tests it under
// hypotheses h = 0 .. XJ_H-1 ("h rejections among the words before it": range
// r - j + h), each test a compare whose lane mask is the hypothesis' rejection ballot
// (lo(w (r - j + h)) and the zone advance by w and 2^lz per hypothesis: one mul per
// word, then adds).  The step's true rejections are then a scalar find-first chain over
// the ballots: the first rejection under h = 0, the next one under h = 1 past it, ...;
// a step with XJ_H rejections ends at the last one.  Every accepted lane j then knows
// its range r_j = r - j + (rejections below j) and stores J[r_j - 1] = hi(w r_j) --
// consecutive lanes, consecutive (descending) J entries.  A step whose ranges would
// leave the lz band (a power of two crossed, or the epoch's last words) walks on lane
// 0 word by word.  Each range is accepted exactly once in the epoch, so segments never
// write the same J.  (r01-r03h: one LANE per segment walking sequentially -- few
// long-lived waves that held CUs against the update kernels: 5.7 ms of side-stream
// busy time per CfgB update, overlapping 71 of 112 minibatch launches.)
struct WordRegions {
    const uint32_t *ptr[4];
    uint64_t base[4], len[4];
    int n;
};
constexpr int XJ_WAVES = 4;           // waves (segments) per block
constexpr int XJ_H = 16;              // rejection hypotheses per 64-word step

// word q (absolute stream position) of the job's device word regions, else ChaCha12
__device__ __forceinline__ uint32_t xj_word(const Key8 &key, uint64_t stream, const WordRegions &wr, uint64_t q) {
    for (int k = 0; k < wr.n; k++)
        if (q >= wr.base[k] && q < wr.base[k] + wr.len[k]) return wr.ptr[k][q - wr.base[k]];
    uint32_t blk[16];
    chacha12_block(key, q >> 4, stream, blk);
    uint32_t v = blk[0];
#pragma unroll
    for (int i = 1; i < 16; i++) v = (int)(q & 15) == i ? blk[i] : v;
    return v;
}

__global__ void __launch_bounds__(64 * XJ_WAVES) k_expand_J(Key8 key, uint64_t stream, const ShuffleEngine::Seg *segs,
                                                          int ns, WordRegions wr, uint32_t *J) {
    const int lane = threadIdx.x & 63;
    const int si = blockIdx.x * XJ_WAVES + (threadIdx.x >> 6);
    if (si == 0 && lane == 0) J[0] = 0;
    if (si >= ns) return;
    const ShuffleEngine::Seg g = segs[si];
    uint32_t r = g.r0;
    uint64_t q = g.pos0;
    uint32_t avail = q < g.pos1 ? (uint32_t)min((uint64_t)64, g.pos1 - q) : 0u;
    uint32_t w = lane < (int)avail ? xj_word(key, stream, wr, q + lane) : 0u;
    while (q < g.pos1 && r >= 2) {
        // the next step's words in flight under this one (r06), assuming it consumes all 64
        // (it does unless XJ_H rejections end it early or the segment ends)
        const uint64_t qn = q + 64;
        const uint32_t availn = qn < g.pos1 ? (uint32_t)min((uint64_t)64, g.pos1 - qn) : 0u;
        const uint32_t wn = lane < (int)availn ? xj_word(key, stream, wr, qn + lane) : 0u;
        const int lz = __clz(r);
        const uint32_t lowr = 1u << (31 - lz);
        if (r >= lowr + 64 && r >= 66) {
            // ---- hypothesis ballots: lane j, hypothesis h tests range r - j + h
            const uint32_t s = 1u << lz;
            const uint32_t rj = r - (uint32_t)lane;
            uint32_t lo = w * rj, z = (rj << lz) - 1u;
            const uint64_t valid = avail >= 64 ? ~0ull : ((1ull << avail) - 1ull);
            uint64_t rejm = 0;                 // the step's true rejections
            uint32_t b = avail;                // words the step consumes
            uint32_t nrej = 0;
            uint64_t from = 0;                 // bits below `from` are resolved
            bool open = true;
#pragma unroll
            for (int h = 0; h < XJ_H; h++) {
                const uint64_t acc = __ballot(lo <= z);
                lo += w;
                z += s;
                if (open) {
                    const uint64_t rem = ~acc & valid & ~from;
                    if (rem == 0) { open = false; continue; }   // every remaining word accepted
                    const int jh = __builtin_ctzll(rem);
                    rejm |= 1ull << jh;
                    nrej++;
                    from = jh == 63 ? ~0ull : ((2ull << jh) - 1ull);
                    if (h == XJ_H - 1) b = (uint32_t)jh + 1;        // XJ_H rejections: the step ends there
                }
            }
            // ---- accepted lanes below b store their draw
            const uint32_t below = (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(rejm >> 32),
                                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)rejm, 0u));
            if ((uint32_t)lane < b && !((rejm >> lane) & 1ull)) {
                const uint32_t rr = r - (uint32_t)lane + below;
                J[rr - 1] = __umulhi(w, rr);
            }
            r -= b - nrej;
            q += b;
        } else {
            // ---- band edge or the epoch's last words: lane 0 walks word by word
            uint32_t rr = r, used = 0;
            if (lane == 0) {
                int lz1 = __clz(rr);
                uint32_t lowr1 = 1u << (31 - lz1), sh = 1u << lz1, z = (rr << lz1) - 1u;
                for (uint32_t j = 0; j < avail && rr >= 2; j++) {
                    const uint32_t wj = xj_word(key, stream, wr, q + j);
                    const uint64_t m = (uint64_t)wj * rr;
                    used = j + 1;
                    if ((uint32_t)m <= z) {
                        J[rr - 1] = (uint32_t)(m >> 32);
                        rr--;
                        z -= sh;
                        if (rr < lowr1 && rr >= 1) { lz1 = __clz(rr); lowr1 = 1u << (31 - lz1); sh = 1u << lz1; z = (rr << lz1) - 1u; }
                    }
                }
            }
            r = __shfl(rr, 0, 64);
            q += __shfl(used, 0, 64);
        }
        if (q == qn) {
            w = wn;
            avail = availn;
        } else if (q < g.pos1) {
            avail = (uint32_t)min((uint64_t)64, g.pos1 - q);
            w = lane < (int)avail ? xj_word(key, stream, wr, q + lane) : 0u;
        }
    }
}

// A job's J expansions on the copy stream wait for the end of the update the caller enqueued
// last (its ev_upd) when BPPO_XJ_GATE is set: 1 every epoch, 2 epochs after the first.  No
// deadlock: an update waits only for its own job's epochs, and the caller records its ev_upd
// after enqueuing every epoch it runs, i.e. after those expansions were launched
void ShuffleEngine::xj_gate_wait(int e) {
    static const int mode = getenv("BPPO_XJ_GATE") ? atoi(getenv("BPPO_XJ_GATE")) : 0;
    if (gate && (mode == 1 || (mode == 2 && e > 0))) hip_note(hipStreamWaitEvent(copy, gate, 0), "hipStreamWaitEvent");
}

// expected words per shuffle of n and its std dev: draw with range R accepts with
// probability a = (R << lz(R)) / 2^32 (uniform.rs zone), geometric word count
static void shuffle_word_stats(uint32_t n, double &mean, double &sd) {
    double m = 0.0, v = 0.0;
    for (uint32_t R = n; R >= 2; R--) {
        const double a = (double)(R << __builtin_clz(R)) / 4294967296.0;
        m += 1.0 / a;
        v += (1.0 - a) / (a * a);
    }
    mean = m;
    sd = std::sqrt(v);
}

// The host copy of the words is read only by the host walkers (the GPU makes its
// own), so it is plain memory on 2 MB pages, not pinned 4 KB pages: a walker
// streams ~8 GB/s of words, and on 4 KB pages the hardware prefetcher restarts at
// every page (= every 1024-word checkpoint piece).  Touched here so the producers
// never fault.
static uint32_t *host_words_alloc(uint64_t words) {
    const size_t bytes = (size_t)words * 4;
    const size_t huge = (size_t)2 << 20, sz = (bytes + huge - 1) / huge * huge;
    void *p = mmap(nullptr, sz, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p == MAP_FAILED) return nullptr;
    (void)madvise(p, sz, MADV_HUGEPAGE);
    memset(p, 0, sz);
    return static_cast<uint32_t *>(p);
}
static void host_words_free(uint32_t *h, uint64_t words) {
    const size_t huge = (size_t)2 << 20, bytes = (size_t)words * 4;
    (void)munmap(h, (bytes + huge - 1) / huge * huge);
}

bppo_status ShuffleEngine::init(int device, const Key8 &k, uint64_t strm, uint32_t n_, int epochs_, uint64_t gap_,
                                std::string &err, bool windows) {
    dev = device; n = n_; epochs = epochs_; key = k; stream = strm; gap = gap_;
    if (epochs > SHUF_MAX_EPOCHS) { err = "num_epochs > 32 not supported by the shuffle engine"; return BPPO_ERR_UNSUPPORTED; }
    shuffle_word_stats(n, Ew, sigma);
    win = windows ? shuffle_window(n) : 0;
    // K walkers per epoch boundary: epochs 1..E-1 of a job plus the next job's
    // first epoch (two alternating carry sets).  K = 6 measured best for CfgB on a
    // 16-CPU share (K = 2/4/5/6: 281/284/311/316 M env-steps/s): more starting
    // points meet the true walk sooner even oversubscribed.
    // (BPPO_SHUFFLE_SPEC overrides; 0 = sequential walk only)
    // BPPO_HOST_THREADS: this rank's CPU budget (bench.py: the CPUs this process may
    // use / ranks on the node), so 8 ranks of one node do not oversubscribe it.
    // K and the word producers scale with it; 16 CPUs (one GPU's share) -> K = 6.
    host_cpus = 16;
    if (const char *e = getenv("BPPO_HOST_THREADS")) host_cpus = std::max(1, atoi(e));
    K = std::max(1, std::min(6, (6 * host_cpus + 8) / 16));
    if (const char *e = getenv("BPPO_SHUFFLE_SPEC")) K = std::max(0, atoi(e));
    // C leading epochs of the next job are speculated during this job (their walks
    // get a whole job of head start; later epochs' walks start with their job)
    C = std::min(2, std::max(epochs, 1));
    // frontier scheduling (depth D): the walks of a boundary start only when the
    // boundary D epochs before it is known exactly, so they guess around an exact
    // position with one-sigma-times-sqrt(D) spread, and only ~2 groups walk at once
    // (the job-start policy ran every boundary's group at once, sqrt(e) wide, and
    // oversubscribed a 16-CPU share).  Needs the next job's first D + 1 epochs as
    // carry groups.  BPPO_SHUFFLE_FRONTIER=0: the job-start policy.
    // Default depth 2 with >= 8 CPUs (r04: the walk binds at depth 1 — epoch e+2's walks
    // start when e resolves, so two resolved epochs take at least one epoch's walk, ~5.2 ms;
    // depth 2 gives the walks of e+3 that head start.  A/B on two boxes, 3 + 2 runs each:
    // 12.41-12.57 vs 12.42-13.75 ms/update, shuffle_wait ~0 vs 0.7-5 ms,
    // profiles/r04_windows/frontier_ab.txt); depth 1 below 8 CPUs (more CPU per update)
    fr_depth = getenv("BPPO_SHUFFLE_FRONTIER") ? atoi(getenv("BPPO_SHUFFLE_FRONTIER")) : (host_cpus >= 8 ? 2 : 1);
    if (fr_depth > 0 && epochs >= 3 && K > 0) {
        C = std::min(fr_depth + 1, epochs - 1);
        fr_depth = C - 1;
        // one-sigma anchors: K = 5 over +-2 sigma misses ~1 in 40 boundaries and
        // meets after ~2 M words (scripts/microbench/comb_sim.cpp); fewer walks
        // leave the true walk and the met chains their CPUs
        if (!getenv("BPPO_SHUFFLE_SPEC")) K = std::max(1, std::min(fr_depth >= 2 ? 4 : 5, (5 * host_cpus + 8) / 16));
    } else {
        fr_depth = 0;
    }
    // shuffle_windows: every epoch's start is known when the job starts, so each epoch is
    // one exact walk (slot e), all walked at once; nothing to speculate or carry
    if (win) { K = 1; C = 0; fr_depth = 0; }
    // and the epochs' walks go in pairs, two chains interleaved per thread (half the
    // walking CPU of one chain per thread: the walker is latency-bound)
    // (only when the rank has fewer CPUs than epochs: with one CPU per epoch each walk
    // runs alone, 0.45 instead of 0.54 ns per word of wall time; BPPO_SHUFFLE_PAIR=0/1 forces)
    keep_guess = !(getenv("BPPO_SHUFFLE_KEEP_GUESS") && atoi(getenv("BPPO_SHUFFLE_KEEP_GUESS")) == 0);
    pair = win && host_cpus < epochs;
    if (const char *e = getenv("BPPO_SHUFFLE_PAIR")) pair = win && atoi(e) != 0;
    win_producers = win && getenv("BPPO_SHUFFLE_WIN_PRODUCERS") && atoi(getenv("BPPO_SHUFFLE_WIN_PRODUCERS")) == 1;
    // opt-in (BPPO_SHUFFLE_GPU_WORDS=1): the job's words, made on the GPU for the J
    // expansion a whole job ahead, are copied (hipMemcpyAsync D2H) to the walks' pinned
    // host buffer, so the walks make no words themselves: 2-CPU walk 14.0 -> 8.3 ms and
    // 40.8 -> 35.6 ms of CPU per update, but on this image HIP runs those copies as blit
    // kernels (__amd_rocclr_copyBuffer, 462 launches in the r04ai trace) that take CUs
    // from the update: 13.8 -> 16.1 ms/update (profiles/r04_windows/windows_ab.txt).  An
    // SDMA path (hsa_amd_memory_async_copy, r03n: 10-50 GB/s by box) is the way to keep
    // the CPU saving without the CU cost.  (r04k's first form, kernels writing host memory
    // over PCIe, stretched the rollout 1.2 -> 4.0 ms.)
    win_gpu_words = win && !win_producers && getenv("BPPO_SHUFFLE_GPU_WORDS") &&
                    atoi(getenv("BPPO_SHUFFLE_GPU_WORDS")) == 1;
    // exact continuations need the last epoch in the in-job groups
    const bool cont_on = !win && epochs - 1 >= C;
    K = std::min(K, SHUF_MAX_SPEC / (std::max(epochs - C, 0) + 2 * C + (cont_on ? 2 : 0)));
    ncur = K * std::max(epochs - C, 0);
    nspec = ncur + 2 * C * K;
    if (cont_on && K > 0) {
        cont0 = nspec;
        nspec += 2 * K;
    }
    const size_t bytes = sizeof(uint32_t) * (size_t)n * epochs;
    maxseg = (int)((Ew + 48.0 * sigma) / SHUF_CK) + 16;
    const size_t sbytes = sizeof(Seg) * (size_t)maxseg * epochs;
    for (int s = 0; s < 2; s++) {
        if (hipHostMalloc((void **)&seg_host[s], sbytes, hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void **)&d_seg[s], sbytes) != hipSuccess ||
            hipMalloc((void **)&d_J[s], bytes) != hipSuccess) {
            err = "shuffle buffers: allocation failed";
            return BPPO_ERR_HIP;
        }
        for (int e = 0; e < epochs; e++)
            if (hipEventCreateWithFlags(&ev[s][e], hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
                err = "shuffle events: creation failed";
                return BPPO_ERR_HIP;
            }
    }
    for (int s = 0; s < 2; s++)
        if (hipEventCreateWithFlags(&consumed[s], hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
            err = "shuffle events: creation failed";
            return BPPO_ERR_HIP;
        }
    if (win && getenv("BPPO_SHUFFLE_GPU_WORDS") && atoi(getenv("BPPO_SHUFFLE_GPU_WORDS")) == 1 &&
        (hipStreamCreateWithFlags(&d2h, hipStreamNonBlocking) != hipSuccess ||
         hipEventCreateWithFlags(&words_made, hipEventDisableTiming) != hipSuccess)) {
        err = "shuffle word copies: stream creation failed";
        return BPPO_ERR_HIP;
    }
    if (make_side_stream(dev, &copy) != hipSuccess) {   // lowest priority
        err = "shuffle copy stream: creation failed";
        return BPPO_ERR_HIP;
    }
    // word buffers: the job's epochs plus the carry region, 12 sigma of slack each
    auto chunks = [](double w) { return ((uint64_t)std::max(w, 1.0) + SHUF_CHUNK - 1) / SHUF_CHUNK * SHUF_CHUNK; };
    const double sE = sigma * std::sqrt((double)std::max(epochs, 1));
    const uint64_t cap0 = chunks(epochs * Ew + 12.0 * sE + 4.0 * SHUF_CK) + SHUF_CHUNK;
    const double sC = sigma * std::sqrt((double)(epochs + C));
    const uint64_t cap1 = K && !win ? chunks(C * Ew + 8.0 * sC + 12.0 * sigma + 8.0 * SHUF_CK) + SHUF_CHUNK : 0;
    // windowed: one region per epoch of its expected words + 10 sigma (a longer walk makes
    // the rest of its words itself)
    const uint64_t capw = (uint64_t)epochs * chunks(Ew + 10.0 * sigma + 4.0 * SHUF_CK);
    for (int b = 0; b < 2; b++) {
        WordBuf &w = wb[b];
        w.cap = win ? capw : cap0 + cap1;
        if (hipMalloc((void **)&w.d, w.cap * 4) != hipSuccess ||
            !(w.h = host_words_alloc(w.cap))) {
            err = "shuffle word buffers: allocation failed";
            return BPPO_ERR_HIP;
        }
        if (win_gpu_words) {
            // the walks' word buffer, pinned so the SDMA engines can copy the GPU's words
            // into it (made on the GPU anyway for the J expansion); only queried
            const size_t huge = (size_t)2 << 20, sz = ((size_t)w.cap * 4 + huge - 1) / huge * huge;
            if (hipHostRegister(w.h, sz, hipHostRegisterDefault) != hipSuccess) {
                (void)hipGetLastError();
                w.gpu = false;           // the walks make their own words
            } else {
                w.hd = w.h;              // registered (unregister at shutdown)
                w.gpu = true;
            }
        }
        const size_t nch = w.cap / SHUF_CHUNK;
        w.ev.assign(nch, nullptr);
        w.ok.reset(new std::atomic<int>[nch]);
        for (size_t c = 0; c < nch; c++) {
            w.ok[c] = 0;
            if (hipEventCreateWithFlags(&w.ev[c], w.gpu ? hipEventDisableTiming
                                                         : hipEventDisableTiming | hipEventBlockingSync) != hipSuccess) {
                err = "shuffle chunk events: creation failed";
                return BPPO_ERR_HIP;
            }
        }
    }
    const uint64_t nck = (uint64_t)((Ew + 24.0 * sigma) / SHUF_CK) + 4;
    for (int i = 0; i < nspec; i++) spec[i].ck.assign(nck, 0xFFFFFFFFu);
    for (int i = 0; i < nspec; i++) workers.emplace_back([this, i]() { worker(i); });
    const int ngen = win && !win_producers ? 0 : std::max(1, std::min(4, host_cpus / 4));
    for (int i = 0; i < ngen; i++) gens.emplace_back([this]() { generator(); });
    th = std::thread([this]() { run(); });
    return BPPO_OK;
}

int ShuffleEngine::ensure(uint64_t start) {
    std::unique_lock<std::mutex> lk(mu);
    for (int sl = 0; sl < 2; sl++)
        if (slot_valid[sl] && slot_start[sl] == start) {
            consumer = sl;
            lk.unlock();
            cv.notify_all();
            return sl;
        }
    // a start the engine did not predict (KL early stop, rng_set): drop everything
    if (running >= 0 || pending >= 0) {
        cancel = true;
        pending = -1;
        cv.notify_all();
        cv.wait(lk, [&] { return running < 0; });
        cancel = false;
    }
    chain_from = -1;
    slot_valid[0] = slot_valid[1] = false;
    const int sl = last_slot ^ 1;
    last_slot = sl;
    slot_start[sl] = start;
    slot_valid[sl] = true;
    ready[sl] = 0;
    pending = sl;
    consumer = sl;
    lk.unlock();
    cv.notify_all();
    return sl;
}

void ShuffleEngine::wait_epoch(int slot, int e) {
    std::unique_lock<std::mutex> lk(mu);
    const bool had = ready[slot] > e;
    cv.wait(lk, [&] { return ready[slot] > e || !slot_valid[slot]; });
    SHUF_LOG("[shuf] consumer epoch %d %s\n", e, had ? "ready" : "waited");
}

bool ShuffleEngine::epoch_ready(int slot, int e) {
    std::lock_guard<std::mutex> lk(mu);
    return slot_valid[slot] && ready[slot] > e;
}

hipError_t ShuffleEngine::release(int slot, hipStream_t st) {
    const hipError_t e = hipEventRecord(consumed[slot], st);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(mu);
    consumed_used[slot] = true;
    return hipSuccess;
}

void ShuffleEngine::hip_note(hipError_t e, const char *what) {
    if (e == hipSuccess) return;
    (void)hipGetLastError();                         // this thread's slot: reported here
    std::lock_guard<std::mutex> lk(hip_mu);
    if (hip_bad.load(std::memory_order_relaxed)) return;
    hip_msg = std::string("shuffle engine: ") + what + ": " + hipGetErrorString(e);
    hip_bad.store(true, std::memory_order_release);
}

bool ShuffleEngine::failed(std::string &msg) const {
    if (!hip_bad.load(std::memory_order_acquire)) return false;
    msg = hip_msg;
    return true;
}

// words [pos, pos + len) of word buffer b (one checkpoint piece: never crosses a
// chunk); outside its regions (not at the usual sizes) they are made here

const uint32_t *ShuffleEngine::words(int b, uint64_t pos, uint64_t len, std::vector<uint32_t> &scratch, bool true_walk) {
    if (true_walk && alt_b >= 0 && pos >= alt_reg.base && pos + len <= alt_reg.base + alt_reg.len) {
        // the previous job's carry region (its chunks' flags are not reset before this job
        // ends: the buffer is re-made only by the next job, after this walk)
        WordBuf &a = wb[alt_b];
        const uint64_t o = alt_reg.off + (pos - alt_reg.base);
        if (a.ok[(size_t)(o / SHUF_CHUNK)].load(std::memory_order_acquire)) return a.h + o;
    }
    WordBuf &w = wb[b];
    for (int g = 0; g < w.nreg; g++) {
        const WordBuf::Region &R = w.reg[g];
        if (pos >= R.base && pos + len <= R.base + R.len) {
            const uint64_t o = R.off + (pos - R.base);
            const size_t c = (size_t)(o / SHUF_CHUNK);
            // a chunk the producers have not reached yet: the walk makes this piece
            // itself (ChaCha12, ~0.3 ns/word) rather than waiting for them
            if (w.ok[c].load(std::memory_order_acquire)) return w.h + o;
            if (w.gpu && event_query(w.ev[c]) == hipSuccess) {   // written by the GPU
                w.ok[c].store(1, std::memory_order_release);
                return w.h + o;
            }
            break;
        }
    }
    scratch.resize(len);
    bppo_host::chacha12_words(key.k, stream, pos, scratch.data(), len);
    return scratch.data();
}

// walk from pos up to the next checkpoint boundary (or the end of the shuffle)
// (the diagnostic counters are per walk thread and folded into the engine's
// atomics once per walk / epoch: shared counters per piece would ping-pong one
// cache line between every walker's core)
uint64_t ShuffleEngine::walk_piece(int b, uint64_t pos, uint32_t *r, std::vector<uint32_t> &scratch, WalkStats &st,
                                   bool true_walk) {
    const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
    const uint64_t t0 = __rdtsc();
    const uint32_t *w = words(b, pos, q - pos, scratch, true_walk);
    const uint64_t t1 = __rdtsc();
    const uint64_t used = bppo_host::chain_walk_nj(w, (size_t)(q - pos), r);
    st.tsc_words += t1 - t0;
    st.tsc_walk += __rdtsc() - t1;
    st.words += used;
    return pos + used;
}
void ShuffleEngine::flush(WalkStats &st, std::atomic<uint64_t> &words_ctr) {
    words_ctr.fetch_add(st.words, std::memory_order_relaxed);
    tsc_walk.fetch_add(st.tsc_walk, std::memory_order_relaxed);
    tsc_words.fetch_add(st.tsc_words, std::memory_order_relaxed);
    st = WalkStats{};
}

void ShuffleEngine::launch_walk(int i, uint64_t start, int wbuf) {
    SpecWalk &s = spec[i];
    s.start = start;
    s.ck_base = start / SHUF_CK * SHUF_CK;
    s.wbuf = wbuf;
    s.end = 0;
    std::fill(s.ck.begin(), s.ck.end(), 0xFFFFFFFFu);
    s.progress.store(-1, std::memory_order_relaxed);
    s.stop.store(false, std::memory_order_relaxed);
    s.merged_to.store(-1, std::memory_order_relaxed);
    s.merge_q = 0;
    s.done.store(0, std::memory_order_release);
    s.running = true;
    s.job = seq;
    s.gen++;
}

void ShuffleEngine::stop_walks(int lo, int hi) {
    std::unique_lock<std::mutex> lk(mu);
    for (int i = lo; i < hi; i++) spec[i].stop.store(true, std::memory_order_relaxed);
    cv.notify_all();
    cv.wait(lk, [&] {
        if (quit) return true;
        for (int i = lo; i < hi; i++) if (spec[i].running) return false;
        return true;
    });
}

// Walks of one boundary start at increasing guesses and never cross (a walk
// started earlier has the smaller or equal range at every position), so once two
// neighbours hold the same range at a checkpoint they are one walk: the right one
// stops and records which walk carries on from there.  peek() follows those links.
int ShuffleEngine::peek(int i, uint64_t q, uint32_t *r) {
    for (;;) {
        SpecWalk &t = spec[i];
        if (q <= t.start) return -1;
        const int mt = t.merged_to.load(std::memory_order_acquire);
        if (mt >= 0 && q >= t.merge_q) { i = mt; continue; }
        const int64_t c = (int64_t)((q - t.ck_base) / SHUF_CK);
        if (c >= (int64_t)t.ck.size()) return -1;
        if (t.progress.load(std::memory_order_acquire) >= c) { *r = t.ck[c]; return 1; }
        if (t.done.load(std::memory_order_acquire) && t.merged_to.load(std::memory_order_acquire) < 0) return -1;
        return 0;
    }
}

void ShuffleEngine::worker(int i) {
    (void)pthread_setname_np(pthread_self(), "bppo-spec");   // per-thread CPU accounting (bench.py)
    (void)hipSetDevice(dev);
    // CPU priority by when a walk is needed: epoch 1's walks first, then epoch
    // 2's, ..., the next job's carry set last (16 CPUs run ~K (E + 1) walks; the
    // scheduler otherwise shares them evenly and delays the walk needed first)
    {
        // frontier scheduling keeps few walks alive at once: one niceness (1) for all;
        // so do windowed jobs, whose epochs are all needed within the same update (a
        // graded niceness, up to 19, starved the later epochs' walks on a node where
        // other ranks' threads run at normal priority)
        const int g = i < ncur ? i / std::max(K, 1) : std::max(epochs - C, 0);
        const int nv = (fr_depth > 0 || win) ? 1 : 3 * g;
        if (nv > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), std::min(19, nv));
    }
    std::vector<uint32_t> scratch;
    WalkStats wst;
    uint64_t seen = 0;
    SpecWalk &s = spec[i];
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || s.gen != seen; });
            if (quit) { s.running = false; cv.notify_all(); return; }
            seen = s.gen;
        }
        if (pair && i < nspec - (nspec & 1)) {
            if (i & 1) continue;        // walked by worker i - 1, interleaved with its own
            walk_pair(i, wst);
            continue;
        }
        uint64_t pos = s.start;
        uint32_t r = n;
        while (r >= 2 && !s.stop.load(std::memory_order_relaxed)) {
            const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
            pos = walk_piece(s.wbuf, pos, &r, scratch, wst);
            if (pos == q) {
                const int64_t c = (int64_t)((q - s.ck_base) / SHUF_CK);
                if (c < (int64_t)s.ck.size()) {
                    s.ck[c] = r;
                    s.progress.store(c, std::memory_order_release);
                }
                uint32_t rl;
                if (i % K != 0 && peek(i - 1, q, &rl) == 1 && rl == r) {   // coalesced with the left neighbour
                    s.merge_q = q;
                    s.merged_to.store(i - 1, std::memory_order_release);
                    break;
                }
            }
        }
        s.end = pos;
        flush(wst, spec_words);
        {
            std::lock_guard<std::mutex> lk(mu);
            s.done.store(1, std::memory_order_release);
            s.running = false;
            // a walk of this job's last epoch that finished the epoch on its own: its
            // exact continuation into the next job's first epoch
            if (cont_dst0 >= 0 && s.job == cont_seq && i >= cont_src0 && i < cont_src0 + K && r < 2 &&
                !s.stop.load(std::memory_order_relaxed) && s.merged_to.load(std::memory_order_relaxed) < 0 &&
                !quit && !cancel.load(std::memory_order_relaxed))
                launch_walk(cont_dst0 + (i - cont_src0), pos + gap, cont_wb);
        }
        cv.notify_all();
    }
}

// windowed jobs: walks i and i + 1 (two epochs, known starts, nothing to merge with)
// in one thread, their 32-word blocks interleaved (chain_walk2_nj); checkpoints as
// in worker().  A walk that ends is marked done at once, the other goes on alone.
// (r06 tried the speculative walks of chained jobs in pairs too, with worker()'s merge
// and continuation rules: 116-119 instead of 137-148 ms of CPU per update, but each chain
// at ~0.54 instead of 0.45 ns per word, and the walk per update 12.1-13.2 instead of
// 10.4-10.9 ms: profiles/r06d/.  Not kept.)
void ShuffleEngine::walk_pair(int i, WalkStats &st) {
    struct Chain {
        SpecWalk *s;
        uint64_t pos;
        uint32_t r;
        const uint32_t *w;
        size_t left;
        std::vector<uint32_t> scratch;
        bool live;
    } ch[2];
    {
        std::unique_lock<std::mutex> lk(mu);   // the partner's launch is under the same lock
        cv.wait(lk, [&] { return quit || spec[i + 1].running; });
        if (quit) return;
    }
    auto refill = [&](Chain &c) {
        const uint64_t q = (c.pos / SHUF_CK + 1) * SHUF_CK;
        const uint64_t t0 = __rdtsc();
        c.w = words(c.s->wbuf, c.pos, q - c.pos, c.scratch);
        st.tsc_words += __rdtsc() - t0;
        c.left = (size_t)(q - c.pos);
    };
    auto finish = [&](Chain &c) {
        c.live = false;
        c.s->end = c.pos;
        std::lock_guard<std::mutex> lk(mu);
        c.s->done.store(1, std::memory_order_release);
        c.s->running = false;
    };
    auto advance = [&](Chain &c, size_t used) {
        c.w += used;
        c.left -= used;
        c.pos += used;
        st.words += used;
        if (c.r < 2) { finish(c); cv.notify_all(); return; }
        // a stop is taken only at a checkpoint, as in worker(): a stopped walk's end is then
        // its last recorded checkpoint, never a position inside a piece
        if (c.left == 0) {                       // at a checkpoint
            const int64_t k = (int64_t)((c.pos - c.s->ck_base) / SHUF_CK);
            if (k < (int64_t)c.s->ck.size()) {
                c.s->ck[k] = c.r;
                c.s->progress.store(k, std::memory_order_release);
            }
            if (c.s->stop.load(std::memory_order_relaxed)) { finish(c); cv.notify_all(); return; }
            refill(c);
        }
    };
    for (int k = 0; k < 2; k++) {
        Chain &c = ch[k];
        c.s = &spec[i + k];
        c.pos = c.s->start;
        c.r = n;
        c.live = n >= 2;
        if (c.live) refill(c);
        else finish(c);
    }
    while (ch[0].live && ch[1].live) {
        size_t u0 = 0, u1 = 0;
        const uint64_t t0 = __rdtsc();
        bppo_host::chain_walk2_nj(ch[0].w, ch[0].left, &ch[0].r, &u0, ch[1].w, ch[1].left, &ch[1].r, &u1);
        st.tsc_walk += __rdtsc() - t0;
        advance(ch[0], u0);
        advance(ch[1], u1);
    }
    for (int k = 0; k < 2; k++) {
        Chain &c = ch[k];
        while (c.live) {
            const uint64_t t0 = __rdtsc();
            const size_t u = bppo_host::chain_walk_nj(c.w, c.left, &c.r);
            st.tsc_walk += __rdtsc() - t0;
            advance(c, u);
        }
    }
    flush(st, spec_words);
    cv.notify_all();
}

void ShuffleEngine::generator() {
    (void)pthread_setname_np(pthread_self(), "bppo-words");
    uint64_t seen = 0;
    for (;;) {
        WordBuf *W;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || gen_job != seen; });
            if (quit) return;
            seen = gen_job;
            W = gen_buf;
            gen_active++;
        }
        for (;;) {
            const size_t k = gen_next.fetch_add(1, std::memory_order_relaxed);
            if (k >= gen_order.size()) break;
            const auto pc = gen_order[k];
            bppo_host::chacha12_words(key.k, stream, pc.first, W->h + pc.second * SHUF_CHUNK, SHUF_CHUNK);
            W->ok[pc.second].store(1, std::memory_order_release);
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            gen_active--;
        }
        cv.notify_all();
    }
}

void ShuffleEngine::run() {
    (void)pthread_setname_np(pthread_self(), "bppo-true");
    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);   // its short sleeps behind a met chain: 1 us slack, not 50
    (void)hipSetDevice(dev);
    std::vector<uint32_t> scratch;
    for (;;) {
        uint64_t start;
        int slot;
        bool wait_consumed = false;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || pending >= 0 || (chain_from >= 0 && consumer == chain_from); });
            if (quit) return;
            if (pending < 0) {
                // chain: the caller consumes the job just resolved, so the other slot is
                // free on the host; its GPU readers are ordered by the `consumed` event
                slot = chain_from ^ 1;
                chain_from = -1;
                last_slot = slot;
                slot_start[slot] = chain_start;
                slot_valid[slot] = true;
                ready[slot] = 0;
            } else {
                slot = pending;
                pending = -1;
            }
            running = slot;
            start = slot_start[slot];
            wait_consumed = consumed_used[slot];
        }
        if (wait_consumed) hip_note(hipStreamWaitEvent(copy, consumed[slot], 0), "hipStreamWaitEvent");
        seq++;
        if (win) {
            const bool ok = run_windowed(slot, start);
            if (!ok) stop_walks(0, nspec);
            {
                std::lock_guard<std::mutex> lk(mu);
                running = -1;
                if (!ok) {
                    slot_valid[slot] = false;
                } else {
                    chain_from = slot;                     // the next job: known since this one started
                    chain_start = job_end(slot) + gap;
                }
            }
            cv.notify_all();
            continue;
        }
        const int b = (int)(seq & 1);                 // word buffer and carry set of this job
        const int cs = 1 - b;                         // carry set the previous job launched for us
        const int cur0 = 0, cur1 = ncur;
        const int cn0 = ncur + b * C * K, cn1 = cn0 + C * K;   // carry group launched now (next job)
        const int cp0 = ncur + cs * C * K;                     // carry group for this job's epochs 0..C-1
        SHUF_LOG("[shuf] job %llu start=%llu slot=%d carry=%d\n", (unsigned long long)seq, (unsigned long long)start,
                 slot, (int)carry_valid[cs]);
        // walks of two jobs ago still on this buffer / carry slots have stopped
        stop_walks(cn0, cn1);
        const int ccn0 = cont0 ? cont0 + b * K : 0, ccp0 = cont0 ? cont0 + cs * K : 0;
        if (cont0) {
            stop_walks(ccn0, ccn0 + K);
            std::lock_guard<std::mutex> lk(mu);
            for (int i = ccn0; i < ccn0 + K; i++) {          // not launched yet: peek() says never
                spec[i].start = ~0ull;
                spec[i].merged_to.store(-1, std::memory_order_relaxed);
            }
            cont_src0 = cur0 + (epochs - 1 - C) * K;
            cont_dst0 = ccn0;
            cont_wb = b;
            cont_seq = seq;
            cont_valid[b] = K > 0;
        }
        // ---- words: this job's epochs, then the region of the next job's first epoch
        WordBuf &W = wb[b];
        const double sE = sigma * std::sqrt((double)std::max(epochs, 1));
        {
            auto chunks = [](double w) { return ((uint64_t)std::max(w, 1.0) + SHUF_CHUNK - 1) / SHUF_CHUNK * SHUF_CHUNK; };
            // the previous job's carry region (buffer b ^ 1, its region 1) was made for this
            // job's first epochs: when it holds this start, region 0 begins where it ends and
            // the true walk reads those words from it (made once per update, not twice: r06,
            // ~35 M producer words per CfgB update).  Any region's words are the stream's
            // words at those positions, so a mispredicted start is only a smaller overlap.
            const uint64_t s0 = start / SHUF_CK * SHUF_CK;
            const uint64_t end0 = s0 + chunks((double)(start - s0) + epochs * Ew + 10.0 * sE + 4.0 * SHUF_CK);
            const WordBuf &Pv = wb[b ^ 1];
            alt_b = -1;
            uint64_t base0 = s0;
            static const bool reuse = !(getenv("BPPO_SHUFFLE_CARRY_REUSE") && atoi(getenv("BPPO_SHUFFLE_CARRY_REUSE")) == 0);
            if (reuse && seq > 1 && Pv.nreg == 2 && Pv.reg[1].len > 0 && Pv.reg[1].base <= s0 &&
                Pv.reg[1].base + Pv.reg[1].len > s0 && Pv.reg[1].base + Pv.reg[1].len < end0) {
                alt_b = b ^ 1;
                alt_reg = Pv.reg[1];
                base0 = alt_reg.base + alt_reg.len;
            }
            W.nreg = 1;
            W.reg[0].base = base0;
            W.reg[0].off = 0;
            W.reg[0].len = std::min(W.cap, chunks((double)(end0 - base0)));   // whole chunks (their ok flags)
            if (K > 0) {
                const double sC = sigma * std::sqrt((double)(epochs + C));
                const double lo = (double)start + epochs * Ew + (double)gap - 4.0 * sC - 4.0 * SHUF_CK;
                uint64_t b1 = (uint64_t)std::max(lo, 0.0) / SHUF_CK * SHUF_CK;
                b1 = std::max(b1, W.reg[0].base + W.reg[0].len);
                const uint64_t len1 = std::min(W.cap - W.reg[0].len, chunks(C * Ew + 8.0 * sC + 12.0 * sigma + 8.0 * SHUF_CK));
                if (len1 > 0) {
                    W.reg[1].base = b1; W.reg[1].off = W.reg[0].len; W.reg[1].len = len1;
                    W.nreg = 2;
                }
            }
        }
        std::vector<std::pair<double, size_t>> order;
        for (int g = 0; g < W.nreg; g++) {
            const WordBuf::Region &R = W.reg[g];
            hipLaunchKernelGGL(k_chacha_words, dim3((unsigned)((R.len / 16 + 255) / 256)), dim3(256), 0, copy, key,
                               stream, R.base, R.len, W.d + R.off);
            hip_note(hipGetLastError(), "k_chacha_words launch");
            for (uint64_t o = 0; o < R.len; o += SHUF_CHUNK) {
                const size_t c = (size_t)((R.off + o) / SHUF_CHUNK);
                W.ok[c] = 0;
                const double p = (double)(R.base + o);
                const double org = g == 0 ? (double)start : (double)start + epochs * Ew + (double)gap;
                const double key_t = std::fmod(std::max(0.0, p - org + 4.0 * sE), std::max(Ew, 1.0));
                order.push_back({key_t, c});
            }
        }
        std::sort(order.begin(), order.end());
        {
            // the host copy of the words: made by the producer threads in need order
            // (the previous job's list is finished: producers run far ahead of walks)
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return gen_active == 0 || quit; });
            gen_order.clear();
            for (auto &oc : order) {
                const size_t c = oc.second;
                const WordBuf::Region *R = nullptr;
                for (int g = 0; g < W.nreg; g++)
                    if (c * SHUF_CHUNK >= W.reg[g].off && c * SHUF_CHUNK < W.reg[g].off + W.reg[g].len) R = &W.reg[g];
                if (R) gen_order.push_back({R->base + (c * SHUF_CHUNK - R->off), c});
            }
            gen_buf = &W;
            gen_next.store(0, std::memory_order_relaxed);
            gen_job++;
        }
        cv.notify_all();
        // ---- speculative walks: epochs 1 .. E-1 of this job, and the next job's first epoch
        // K guesses evenly over centre +- spread*sd
        const double spread = 2.0;
        auto guess = [&](double centre, double sd, int k) {
            return (uint64_t)std::max((double)start, std::floor(centre + ((k + 0.5) / K - 0.5) * 2.0 * spread * sd));
        };
        if (fr_depth > 0) {
            // frontier: this job's in-job groups and the next job's carry groups are
            // launched as boundaries resolve (below); until then peek() says never
            std::lock_guard<std::mutex> lk(mu);
            for (int i = cur0; i < cur1; i++) { spec[i].start = ~0ull; spec[i].merged_to.store(-1, std::memory_order_relaxed); }
            for (int i = cn0; i < cn1; i++) { spec[i].start = ~0ull; spec[i].merged_to.store(-1, std::memory_order_relaxed); }
            carry_valid[b] = K > 0;
        } else {
            std::lock_guard<std::mutex> lk(mu);
            for (int e = C; e < epochs; e++)
                for (int k = 0; k < K; k++)
                    launch_walk(cur0 + (e - C) * K + k, guess((double)start + e * Ew, sigma * std::sqrt((double)e), k), b);
            for (int c = 0; c < C; c++)
                for (int k = 0; k < K; k++)
                    launch_walk(cn0 + c * K + k, guess((double)start + (epochs + c) * Ew + (double)gap,
                                                       sigma * std::sqrt((double)(epochs + c)), k), b);
            carry_valid[b] = K > 0;
        }
        cv.notify_all();
        // ---- true walks (checkpoint states only; J is rebuilt on the GPU)
        uint64_t pos = start;
        bool cancelled = false;
        WalkStats tst;
        std::vector<std::pair<uint64_t, uint32_t>> tck;
        for (int e = 0; e < epochs && !cancelled; e++) {
            auto t0 = std::chrono::steady_clock::now();
            if (ev_used[slot][e]) hip_note(hipEventSynchronize(ev[slot][e]), "hipEventSynchronize");   // previous upload of this buffer
            uint32_t r = n;
            int met = -1, walked = 0;
            int s0 = 0, s1 = 0;                        // candidate speculative walks for this epoch
            if (e < C) { if (carry_valid[cs]) { s0 = cp0 + e * K; s1 = s0 + K; } }
            else { s0 = cur0 + (e - C) * K; s1 = s0 + K; }
            int c0 = 0, c1 = 0;                        // the previous job's exact continuations (epoch 0)
            if (e == 0 && cont0 && cont_valid[cs]) { c0 = ccp0; c1 = ccp0 + K; }
            tck.clear();
            tck.push_back({pos, r});
            // The true walk never waits on a speculative walk: at each checkpoint it
            // compares only with the candidates already past it (one that lags would
            // gain nothing).  After a meet it keeps walking itself and leapfrogs to the
            // met chain's recorded states whenever that chain is ahead, so the epoch
            // closes at the earlier of its own walk and the chain's end.
            int fin = -1;                              // chain walk whose end closes the epoch
            uint64_t endp = 0, chain_front = 0;
            // candidates on our chain at checkpoint q (range rq); keep (or switch to) the
            // one furthest ahead — an exact continuation meets at once but started late,
            // a guessed walk of the same chain may have a long head start
            auto frontier = [&](int i) -> uint64_t {
                for (int mt; (mt = spec[i].merged_to.load(std::memory_order_acquire)) >= 0;) i = mt;
                const int64_t pr = spec[i].progress.load(std::memory_order_acquire);
                return pr < 0 ? 0 : spec[i].ck_base + (uint64_t)pr * SHUF_CK;
            };
            auto try_switch = [&](uint64_t q, uint32_t rq) -> bool {
                int best = met;
                uint64_t bf = met >= 0 ? frontier(met) : 0;
                for (int g = 0; g < 2; g++)
                    for (int i = g ? s0 : c0; i < (g ? s1 : c1); i++) {
                        uint32_t rs = 0;
                        if (i == met || peek(i, q, &rs) != 1 || rs != rq) continue;
                        const uint64_t f = frontier(i);
                        if (best < 0 || f > bf) { best = i; bf = f; }
                    }
                if (best == met) return false;
                met = best;
                // from here on the epoch's chain lives only in the met walk and the walks
                // it has merged into (merges go leftwards): every other walk of this
                // boundary is stopped and frees its CPU — except, while the met walk is an
                // exact continuation, the guessed walks (g = 1): one of them may carry the
                // same chain further once they coalesce, and the leapfrog below keeps
                // checking them.  (Should the chain's head later merge into a neighbour
                // stopped here, that neighbour's recorded states stay valid and the true
                // walk walks on from its end -- slower, never wrong.)
                const bool on_cont = met >= c0 && met < c1;
                bool keep[SHUF_MAX_SPEC] = {};
                for (int i = met; i >= 0; i = spec[i].merged_to.load(std::memory_order_acquire)) keep[i] = true;
                for (int g = 0; g < 2; g++)
                    for (int i = g ? s0 : c0; i < (g ? s1 : c1); i++)
                        if (!keep[i] && !(on_cont && g == 1 && keep_guess))
                            spec[i].stop.store(true, std::memory_order_relaxed);
                return true;
            };
            while (r >= 2) {
                if (met >= 0) {
                    if (cancel.load(std::memory_order_relaxed) || quit) { cancelled = true; break; }
                    int f = met;                       // the chain's current last walk
                    for (int mt; (mt = spec[f].merged_to.load(std::memory_order_acquire)) >= 0;) f = mt;
                    const bool chain_done = spec[f].done.load(std::memory_order_acquire) != 0 &&
                                            spec[f].merged_to.load(std::memory_order_acquire) < 0;
                    uint32_t rr = 0;
                    const bool recheck = keep_guess && s1 > s0 && met >= c0 && met < c1;
                    for (uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK; r >= 2 && peek(met, q, &rr) == 1; q += SHUF_CK) {
                        tck.push_back({q, rr});
                        pos = q;
                        r = rr;
                        // following an exact continuation: a guessed walk of this boundary
                        // that has coalesced with the chain is further ahead -- jump to it
                        if (recheck && try_switch(q, rr)) break;
                    }
                    if (r < 2) break;
                    if (chain_done && spec[f].end > pos && spec[f].end - pos <= SHUF_CK) {
                        fin = f;
                        endp = spec[f].end;
                        break;
                    }
                    // frontier: the met chain's walker started a boundary earlier and is
                    // ahead on this same chain; our own piece would only duplicate it, so
                    // sleep while it advances and walk only if it stalls
                    if (fr_depth > 0 && !chain_done && pos > chain_front) {
                        chain_front = pos;
                        std::this_thread::sleep_for(std::chrono::microseconds(10));
                        continue;
                    }
                }
                const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
                pos = walk_piece(b, pos, &r, scratch, tst, true);
                if (cancel.load(std::memory_order_relaxed)) { cancelled = true; break; }
                if (pos != q || r < 2) continue;
                tck.push_back({q, r});
                if (s0 == s1 && c0 == c1) continue;
                if (met < 0) walked++;
                try_switch(q, r);
            }
            flush(tst, true_words);
            if (cancelled) break;
            Seg *S = seg_host[slot] + (size_t)e * maxseg;
            int ns = 0;
            bool overflow = false;
            auto add = [&](uint64_t p0, uint64_t p1, uint32_t r0) {
                if (p1 <= p0 || r0 < 2) return;
                if (ns >= maxseg) { overflow = true; return; }
                S[ns++] = Seg{p0, p1, r0, 0};
            };
            for (size_t i = 0; i + 1 < tck.size(); i++) add(tck[i].first, tck[i + 1].first, tck[i].second);
            if (fin >= 0) pos = endp;                  // the chain's last piece closes the epoch
            add(tck.back().first, pos, tck.back().second);
            coalesced[slot][e] = met >= 0 ? walked : -1;
            // The next boundary is now known exactly (x).  Walks of one boundary never
            // cross, so only the two started nearest x on either side can ever meet the
            // true walk (any farther one meets it only through them); a walk started at
            // x itself is the true chain.  Stop the rest and give their CPUs to those.
            auto prune = [&](int g0, int g1, uint64_t x) {
                int lo = -1, hi = -1, exact = -1;
                for (int i = g0; i < g1; i++) {
                    const uint64_t st = spec[i].start;
                    if (st == ~0ull) continue;
                    if (st == x) exact = i;
                    if (st <= x && (lo < 0 || st > spec[lo].start)) lo = i;
                    if (st > x && (hi < 0 || st < spec[hi].start)) hi = i;
                }
                // keep those walks and the walks their chains continue in (merge links)
                bool keep[SHUF_MAX_SPEC] = {};
                for (int k0 : {exact >= 0 ? exact : lo, exact >= 0 ? -1 : hi})
                    for (int i = k0; i >= 0; i = spec[i].merged_to.load(std::memory_order_acquire)) keep[i] = true;
                for (int i = g0; i < g1; i++)
                    if (!keep[i]) spec[i].stop.store(true, std::memory_order_relaxed);
                return exact;
            };
            if (K > 0 && !cancelled) {
                std::lock_guard<std::mutex> lk(mu);
                if (e + 1 < epochs) {
                    if (e + 1 < C) { if (carry_valid[cs]) prune(cp0 + (e + 1) * K, cp0 + (e + 2) * K, pos); }
                    else prune(cur0 + (e + 1 - C) * K, cur0 + (e + 2 - C) * K, pos);
                } else {
                    // the next job's first epoch.  An exact continuation is the true
                    // chain, but it started only when a walk of this epoch finished; the
                    // guessed walks started when the boundary fr_depth epochs earlier
                    // resolved, so the two nearest x may be far ahead on the same chain
                    // once they coalesce with it: keep them beside the continuation (the
                    // true walk follows whichever is ahead).  keep_guess = 0: r02's rule
                    // (an exact continuation stops every guessed walk).
                    const uint64_t x = pos + gap;
                    const int ex = cont0 ? prune(ccn0, ccn0 + K, x) : -1;
                    if (ex >= 0 && !keep_guess) for (int i = cn0; i < cn0 + K; i++) spec[i].stop.store(true, std::memory_order_relaxed);
                    else prune(cn0, cn0 + K, x);
                }
            }
            // frontier: the boundary fr_depth epochs past this one now has an exact
            // anchor (this epoch's end, + gap across the job boundary)
            if (fr_depth > 0 && !cancelled) {
                std::lock_guard<std::mutex> lk(mu);
                const int t = e + 1 + fr_depth;
                int g0 = -1;
                if (t < epochs) g0 = cur0 + (t - C) * K;
                else if (t - epochs < C) g0 = cn0 + (t - epochs) * K;
                if (g0 >= 0) {
                    const double centre = (double)pos + fr_depth * Ew + (t >= epochs ? (double)gap : 0.0);
                    const double sd = sigma * std::sqrt((double)fr_depth);
                    for (int k = 0; k < K; k++) launch_walk(g0 + k, guess(centre, sd, k), b);
                }
                cv.notify_all();
            }
            if (overflow) {   // never at sane sizes: fall back to the sequential walk of the epoch
                std::vector<uint32_t> Jh(n);
                const uint64_t e0 = shuffle_walk_host(key, stream, tck.front().first, n, Jh.data());
                hip_note(hipMemcpyAsync(d_J[slot] + (size_t)e * n, Jh.data(), 4ull * n, hipMemcpyHostToDevice, copy), "hipMemcpyAsync");
                hip_note(hipStreamSynchronize(copy), "hipStreamSynchronize");
                pos = e0;
            } else {
                WordRegions wr{};
                for (int bb = 0; bb < 2; bb++)
                    for (int g = 0; g < wb[bb].nreg; g++) {
                        wr.ptr[wr.n] = wb[bb].d + wb[bb].reg[g].off;
                        wr.base[wr.n] = wb[bb].reg[g].base;
                        wr.len[wr.n] = wb[bb].reg[g].len;
                        wr.n++;
                    }
                Seg *dS = d_seg[slot] + (size_t)e * maxseg;
                hip_note(hipMemcpyAsync(dS, S, sizeof(Seg) * (size_t)std::max(ns, 1), hipMemcpyHostToDevice, copy), "hipMemcpyAsync");
                xj_gate_wait(e);
                hipLaunchKernelGGL(k_expand_J, dim3((unsigned)((std::max(ns, 1) + XJ_WAVES - 1) / XJ_WAVES)),
                                   dim3(64 * XJ_WAVES), 0, copy, key, stream, (const Seg *)dS, ns, wr,
                                   d_J[slot] + (size_t)e * n);
                hip_note(hipGetLastError(), "k_expand_J launch");
            }
            end_pos[slot][e] = pos;
            hip_note(hipEventRecord(ev[slot][e], copy), "hipEventRecord");
            ev_used[slot][e] = true;
            walk_ms[slot][e] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            SHUF_LOG("[shuf] epoch %d end=%llu met=%d segs=%d (%.2f ms)\n", e, (unsigned long long)pos,
                     coalesced[slot][e], ns, walk_ms[slot][e]);
            {
                std::lock_guard<std::mutex> lk(mu);
                ready[slot] = e + 1;
            }
            cv.notify_all();
            if (K > 0) stop_walks(s0, s1);        // this epoch's walks have served
            if (c1 > c0) { stop_walks(c0, c1); cont_valid[cs] = false; }
            if (e == C - 1) carry_valid[cs] = false;
        }
        SHUF_LOG("[shuf] job done cancelled=%d\n", (int)cancelled);
        // this job's in-update walks are done with; the carry set keeps running for
        // the next job (all of it is dropped on a cancel)
        stop_walks(cur0, cur1);
        if (cancelled) {
            stop_walks(0, nspec);
            carry_valid[0] = carry_valid[1] = false;
            cont_valid[0] = cont_valid[1] = false;
        }
        {
            std::lock_guard<std::mutex> lk(mu);
            running = -1;
            if (cancelled) {
                slot_valid[slot] = false;
            } else {
                chain_from = slot;                     // next job: gap words after this one's end
                chain_start = end_pos[slot][epochs - 1] + gap;
            }
        }
        cv.notify_all();
    }
}

// shuffle_windows: the job's epochs start at start + e * win, all known now, so each is
// walked exactly and completely by its own walker (slot e), all at once; the epochs
// resolve in order as their walks finish.  J is rebuilt on the GPU from the walk's
// checkpoint states, as for the chained walks.
bool ShuffleEngine::run_windowed(int slot, uint64_t start) {
    const int b = (int)(seq & 1);
    WordBuf &W = wb[b];
    auto chunks = [](double w) { return ((uint64_t)std::max(w, 1.0) + SHUF_CHUNK - 1) / SHUF_CHUNK * SHUF_CHUNK; };
    const uint64_t rlen = std::min(W.cap / (uint64_t)epochs, chunks(Ew + 10.0 * sigma + 4.0 * SHUF_CK));
    // one job's regions (epoch e at s0 + e * win) and its chunks in the order the walks
    // reach them (every epoch's words interleaved)
    auto regions = [&](WordBuf &B, uint64_t s0, std::vector<size_t> &order) {
        std::vector<std::pair<double, size_t>> ord;
        B.nreg = epochs;
        for (int e = 0; e < epochs; e++) {
            WordBuf::Region &R = B.reg[e];
            R.base = (s0 + (uint64_t)e * win) / SHUF_CK * SHUF_CK;
            R.off = (uint64_t)e * rlen;
            R.len = rlen;
            for (uint64_t o = 0; o < R.len; o += SHUF_CHUNK) {
                const size_t c = (size_t)((R.off + o) / SHUF_CHUNK);
                B.ok[c] = 0;
                ord.push_back({(double)o + 0.25 * e, c});
            }
        }
        std::sort(ord.begin(), ord.end());
        order.clear();
        for (auto &oc : ord) order.push_back(oc.second);
    };
    // the job's words on the GPU (the J expansion reads them) and, with GPU-made host
    // words, copied to the walks' pinned host buffer chunk by chunk on the SDMA engines
    auto make_words = [&](WordBuf &B, uint64_t s0, std::vector<size_t> &order) {
        regions(B, s0, order);
        for (int e = 0; e < epochs; e++)
            hipLaunchKernelGGL(k_chacha_words, dim3((unsigned)((B.reg[e].len / 16 + 255) / 256)), dim3(256), 0, copy,
                               key, stream, B.reg[e].base, B.reg[e].len, B.d + B.reg[e].off);
        hip_note(hipGetLastError(), "k_chacha_words launch");
        if (B.gpu) {
            hip_note(hipEventRecord(words_made, copy), "hipEventRecord");
            hip_note(hipStreamWaitEvent(d2h, words_made, 0), "hipStreamWaitEvent");
            for (size_t c : order) {
                const uint64_t o = c * SHUF_CHUNK;
                hip_note(hipMemcpyAsync(B.h + o, B.d + o, SHUF_CHUNK * 4, hipMemcpyDeviceToHost, d2h), "hipMemcpyAsync");
                hip_note(hipEventRecord(B.ev[c], d2h), "hipEventRecord");
            }
        }
        B.made_for = s0;
    };
    std::vector<size_t> order, next_order;
    if (!(W.gpu && W.made_for == start)) make_words(W, start, order);   // not made a job ahead (first job, moved start)
    else regions(W, start, order);                                      // (made a job ago: same regions)
    // the next job's words now, a whole job ahead of its walks (its start is known:
    // this job's fixed span plus the next rollout's words)
    if (W.gpu) make_words(wb[b ^ 1], start + (uint64_t)epochs * win + gap, next_order);
    {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return gen_active == 0 || quit; });
        gen_order.clear();
        // every word of a windowed job is on a true chain and read by exactly one walk:
        // the walks make their own pieces (no producer threads making the same words
        // twice when the walks outrun them; BPPO_SHUFFLE_WIN_PRODUCERS=1 restores them)
        if (win_producers)
            for (size_t c : order) {
                const WordBuf::Region &R = W.reg[c * SHUF_CHUNK / rlen];
                gen_order.push_back({R.base + (c * SHUF_CHUNK - R.off), c});
            }
        gen_buf = &W;
        gen_next.store(0, std::memory_order_relaxed);
        gen_job++;
        for (int e = 0; e < epochs; e++) launch_walk(e, start + (uint64_t)e * win, b);
    }
    cv.notify_all();
    for (int e = 0; e < epochs; e++) {
        const auto t0 = std::chrono::steady_clock::now();
        if (ev_used[slot][e]) hip_note(hipEventSynchronize(ev[slot][e]), "hipEventSynchronize");   // previous upload of this buffer
        SpecWalk &w = spec[e];
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || cancel.load(std::memory_order_relaxed) ||
                                     (!w.running && w.done.load(std::memory_order_acquire)); });
            if (quit || cancel.load(std::memory_order_relaxed)) return false;
        }
        const uint64_t p0 = start + (uint64_t)e * win, pend = w.end;   // (its words count as spec_words)
        Seg *S = seg_host[slot] + (size_t)e * maxseg;
        int ns = 0;
        bool overflow = false;
        auto add = [&](uint64_t a, uint64_t z, uint32_t r0) {
            if (z <= a || r0 < 2) return;
            if (ns >= maxseg) { overflow = true; return; }
            S[ns++] = Seg{a, z, r0, 0};
        };
        // [p0, first checkpoint) from the full range, then one segment per checkpoint
        uint64_t q = w.ck_base + SHUF_CK;
        add(p0, std::min(q, pend), n);
        for (size_t c = 1; q < pend; c++, q += SHUF_CK) {
            if (c >= w.ck.size()) { overflow = true; break; }   // longer than any recorded walk
            add(q, std::min(q + SHUF_CK, pend), w.ck[c]);
        }
        if (overflow) {   // never at sane sizes: the sequential walk of the epoch
            std::vector<uint32_t> Jh(n);
            (void)shuffle_walk_host(key, stream, p0, n, Jh.data());
            hip_note(hipMemcpyAsync(d_J[slot] + (size_t)e * n, Jh.data(), 4ull * n, hipMemcpyHostToDevice, copy), "hipMemcpyAsync");
            hip_note(hipStreamSynchronize(copy), "hipStreamSynchronize");
        } else {
            WordRegions wr{};
            wr.ptr[0] = W.d + W.reg[e].off; wr.base[0] = W.reg[e].base; wr.len[0] = W.reg[e].len; wr.n = 1;
            Seg *dS = d_seg[slot] + (size_t)e * maxseg;
            hip_note(hipMemcpyAsync(dS, S, sizeof(Seg) * (size_t)std::max(ns, 1), hipMemcpyHostToDevice, copy), "hipMemcpyAsync");
            xj_gate_wait(e);
            hipLaunchKernelGGL(k_expand_J, dim3((unsigned)((std::max(ns, 1) + XJ_WAVES - 1) / XJ_WAVES)),
                               dim3(64 * XJ_WAVES), 0, copy, key, stream, (const Seg *)dS, ns, wr,
                               d_J[slot] + (size_t)e * n);
            hip_note(hipGetLastError(), "k_expand_J launch");
        }
        end_pos[slot][e] = pend;
        coalesced[slot][e] = -1;
        hip_note(hipEventRecord(ev[slot][e], copy), "hipEventRecord");
        ev_used[slot][e] = true;
        walk_ms[slot][e] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        {
            std::lock_guard<std::mutex> lk(mu);
            ready[slot] = e + 1;
        }
        cv.notify_all();
    }
    return true;
}

void ShuffleEngine::shutdown() {
    if (th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
            cancel = true;
            for (int i = 0; i < nspec; i++) spec[i].stop = true;
        }
        cv.notify_all();
        th.join();
        for (auto &w : workers) w.join();
        workers.clear();
        for (auto &g : gens) g.join();
        gens.clear();
    }
    if (copy) { (void)hipStreamSynchronize(copy); (void)hipStreamDestroy(copy); copy = nullptr; }
    if (d2h) { (void)hipStreamSynchronize(d2h); (void)hipStreamDestroy(d2h); d2h = nullptr; }
    if (words_made) { (void)hipEventDestroy(words_made); words_made = nullptr; }
    for (int s = 0; s < 2; s++) {
        if (consumed[s]) { (void)hipEventDestroy(consumed[s]); consumed[s] = nullptr; }
        for (int e = 0; e < epochs; e++) if (ev[s][e]) { (void)hipEventDestroy(ev[s][e]); ev[s][e] = nullptr; }
        if (seg_host[s]) { (void)hipHostFree(seg_host[s]); seg_host[s] = nullptr; }
        if (d_seg[s]) { (void)hipFree(d_seg[s]); d_seg[s] = nullptr; }
        if (d_J[s]) { (void)hipFree(d_J[s]); d_J[s] = nullptr; }
    }
    for (int b = 0; b < 2; b++) {
        for (auto &e : wb[b].ev) if (e) (void)hipEventDestroy(e);
        wb[b].ev.clear();
        if (wb[b].d) { (void)hipFree(wb[b].d); wb[b].d = nullptr; }
        if (wb[b].h && wb[b].hd) (void)hipHostUnregister(wb[b].h);
        wb[b].hd = nullptr;
        if (wb[b].h) { host_words_free(wb[b].h, wb[b].cap); wb[b].h = nullptr; }
    }
}

// side streams (J expansion, Fisher-Yates): lowest priority; BPPO_SIDE_PRIO=normal (A/B)
// creates them at the default priority
hipError_t make_side_stream(int device, hipStream_t *st) {
    (void)device;
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    static const bool normal = getenv("BPPO_SIDE_PRIO") && std::string(getenv("BPPO_SIDE_PRIO")) == "normal";
    if (normal) return hipStreamCreateWithFlags(st, hipStreamNonBlocking);
    return hipStreamCreateWithPriority(st, hipStreamNonBlocking, lo);
}

// single-shot host walk (parity hook): J for one shuffle of n from word position pos
uint64_t shuffle_walk_host(const Key8 &key, uint64_t stream, uint64_t pos, uint32_t n, uint32_t *J) {
    const size_t C = (size_t)1 << 18;
    std::vector<uint32_t> w(C);
    uint32_t r = n;
    while (r >= 2) {
        bppo_host::chacha12_words(key.k, stream, pos, w.data(), C);
        pos += bppo_host::chain_walk(w.data(), C, &r, J);
    }
    if (n) J[0] = 0;
    return pos;
}

}  // namespace bppo

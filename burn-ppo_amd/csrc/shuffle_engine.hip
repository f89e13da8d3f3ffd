// shuffle_engine.hip — the host side of ppo_update's per-epoch shuffle
// (ppo.rs:1816 `indices.shuffle(rng)`, rand 0.8.5 SliceRandom::shuffle):
//
//   words      : the ChaCha12 words of the main StdRng stream for one update's
//                shuffles, made by a GPU kernel and copied to pinned host
//                memory in chunks (ordered by when the walkers reach them);
//   true walk  : the sequential rejection chain -> J[i] = gen_range(0..i+1),
//                i = n-1..1 (shuffle_host.cpp), epoch by epoch;
//   speculation: epoch e >= 1 starts where epoch e-1 ends, known only after
//                walking it.  K walkers start every epoch e >= 1 at once, at
//                guesses spread around the expected boundary, recording the
//                remaining range r at every SHUF_CK-th word position.  The true
//                walk of epoch e runs from the real boundary only until, at a
//                checkpoint, its r equals a speculative walk's r at the same
//                position: from there the two walks are the same walk, so the
//                epoch's end and J[0 .. r) come from the speculative one.  With
//                no meeting the true walk finishes the epoch itself.
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
#include "bppo_internal.h"
#include "shuffle_host.h"

namespace bppo {

static bool shuf_debug() {
    static int v = -1;
    if (v < 0) v = getenv("BPPO_SHUFFLE_DEBUG") ? 1 : 0;
    return v == 1;
}
#define SHUF_LOG(...)                                        \
    do {                                                     \
        if (shuf_debug()) { fprintf(stderr, __VA_ARGS__); fflush(stderr); } \
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

bppo_status ShuffleEngine::init(int device, const Key8 &k, uint64_t strm, uint32_t n_, int epochs_,
                                std::string &err) {
    dev = device; n = n_; epochs = epochs_; key = k; stream = strm;
    if (epochs > SHUF_MAX_EPOCHS) { err = "num_epochs > 32 not supported by the shuffle engine"; return BPPO_ERR_UNSUPPORTED; }
    shuffle_word_stats(n, Ew, sigma);
    // speculative walks per epoch (BPPO_SHUFFLE_SPEC, default: about 12 walker threads in all)
    K = epochs > 1 ? std::max(1, std::min(4, 12 / (epochs - 1))) : 0;
    if (const char *e = getenv("BPPO_SHUFFLE_SPEC")) K = std::max(0, std::min(SHUF_MAX_SPEC, atoi(e)));
    nspec = std::min(SHUF_MAX_SPEC, K * std::max(0, epochs - 1));
    K = epochs > 1 ? nspec / (epochs - 1) : 0;
    nspec = K * std::max(0, epochs - 1);
    const size_t bytes = sizeof(uint32_t) * (size_t)n * epochs;
    for (int s = 0; s < 2; s++) {
        if (hipHostMalloc((void **)&J_host[s], bytes, hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void **)&d_J[s], bytes) != hipSuccess) {
            err = "shuffle buffers: allocation failed";
            return BPPO_ERR_HIP;
        }
        for (int e = 0; e < epochs; e++)
            if (hipEventCreateWithFlags(&ev[s][e], hipEventDisableTiming) != hipSuccess) {
                err = "shuffle events: creation failed";
                return BPPO_ERR_HIP;
            }
    }
    if (hipStreamCreateWithFlags(&copy, hipStreamNonBlocking) != hipSuccess) {
        err = "shuffle copy stream: creation failed";
        return BPPO_ERR_HIP;
    }
    // word buffer: all epochs plus 12 sigma of slack, whole chunks
    const double need = epochs * Ew + 12.0 * sigma * std::sqrt((double)epochs) + 4.0 * SHUF_CK + 64.0;
    wcap = ((uint64_t)need + SHUF_CHUNK - 1) / SHUF_CHUNK * SHUF_CHUNK + SHUF_CHUNK;
    if (hipMalloc((void **)&d_words, wcap * 4) != hipSuccess ||
        hipHostMalloc((void **)&h_words, wcap * 4, hipHostMallocDefault) != hipSuccess) {
        err = "shuffle word buffers: allocation failed";
        return BPPO_ERR_HIP;
    }
    const size_t nch = wcap / SHUF_CHUNK;
    chunk_ev.assign(nch, nullptr);
    chunk_ok.reset(new std::atomic<int>[nch]);
    for (size_t c = 0; c < nch; c++) {
        chunk_ok[c] = 0;
        if (hipEventCreateWithFlags(&chunk_ev[c], hipEventDisableTiming) != hipSuccess) {
            err = "shuffle chunk events: creation failed";
            return BPPO_ERR_HIP;
        }
    }
    const uint64_t nck = wcap / SHUF_CK + 2;
    for (int i = 0; i < nspec; i++) {
        if (hipHostMalloc((void **)&spec[i].J, sizeof(uint32_t) * (size_t)n, hipHostMallocDefault) != hipSuccess) {
            err = "shuffle speculative buffers: allocation failed";
            return BPPO_ERR_HIP;
        }
        spec[i].ck.assign(nck, 0xFFFFFFFFu);
        spec[i].done = 1;
    }
    for (int i = 0; i < nspec; i++) workers.emplace_back([this, i]() { worker(i); });
    th = std::thread([this]() { run(); });
    return BPPO_OK;
}

int ShuffleEngine::ensure(uint64_t start) {
    std::unique_lock<std::mutex> lk(mu);
    if (job_valid && job_start == start) return job_slot;
    if (job_running || job_pending) {
        cancel = true;
        cv.notify_all();
        cv.wait(lk, [&] { return !job_running && !job_pending; });
        cancel = false;
    }
    job_slot ^= 1;
    job_start = start;
    job_pending = true;
    job_valid = true;
    ready[job_slot] = 0;
    lk.unlock();
    cv.notify_all();
    return job_slot;
}

void ShuffleEngine::wait_epoch(int slot, int e) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return ready[slot] > e; });
}

// words [pos, pos + len) of the current job (one checkpoint piece: never crosses
// a chunk); outside the GPU-made range (never at the usual sizes) they are made here
const uint32_t *ShuffleEngine::words(uint64_t pos, uint64_t len, std::vector<uint32_t> &scratch) {
    if (pos >= wbase && pos + len <= wbase + wlen) {
        const size_t c = (size_t)((pos - wbase) / SHUF_CHUNK);
        if (!chunk_ok[c].load(std::memory_order_acquire)) {
            (void)hipEventSynchronize(chunk_ev[c]);
            chunk_ok[c].store(1, std::memory_order_release);
        }
        return h_words + (pos - wbase);
    }
    scratch.resize(len);
    bppo_host::chacha12_words(key.k, stream, pos, scratch.data(), len);
    return scratch.data();
}

// walk from pos up to the next checkpoint boundary (or the end of the shuffle)
uint64_t ShuffleEngine::walk_piece(uint64_t pos, uint32_t *r, uint32_t *J, std::vector<uint32_t> &scratch) {
    const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
    const uint32_t *w = words(pos, q - pos, scratch);
    return pos + bppo_host::chain_walk(w, (size_t)(q - pos), r, J);
}

void ShuffleEngine::worker(int i) {
    (void)hipSetDevice(dev);
    std::vector<uint32_t> scratch;
    uint64_t seen = 0;
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || gen != seen; });
            if (quit) return;
            seen = gen;
        }
        SpecWalk &s = spec[i];
        uint64_t pos = s.start;
        uint32_t r = n;
        while (r >= 2 && !cancel.load(std::memory_order_relaxed)) {
            const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
            pos = walk_piece(pos, &r, s.J, scratch);
            if (pos == q) {
                const int64_t c = (int64_t)((q - wbase) / SHUF_CK);
                if (c < (int64_t)s.ck.size()) {
                    s.ck[c] = r;
                    s.progress.store(c, std::memory_order_release);
                }
            }
        }
        if (n) s.J[0] = 0;
        s.end = pos;
        {
            std::lock_guard<std::mutex> lk(mu);
            s.done.store(1, std::memory_order_release);
            busy--;
        }
        cv.notify_all();
    }
}

void ShuffleEngine::run() {
    (void)hipSetDevice(dev);
    std::vector<uint32_t> scratch;
    for (;;) {
        uint64_t start;
        int slot;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return quit || job_pending; });
            if (quit) return;
            job_pending = false;
            job_running = true;
            start = job_start;
            slot = job_slot;
        }
        SHUF_LOG("[shuf] job start=%llu slot=%d\n", (unsigned long long)start, slot);
        // uploads still reading the speculative J buffers / host words have finished
        (void)hipStreamSynchronize(copy);
        // ---- words of the whole job, made on the GPU, copied in need order
        wbase = start / SHUF_CK * SHUF_CK;
        {
            const double need = (double)(start - wbase) + epochs * Ew +
                                10.0 * sigma * std::sqrt((double)std::max(epochs, 1)) + 4.0 * SHUF_CK;
            wlen = std::min(wcap, ((uint64_t)need + SHUF_CHUNK - 1) / SHUF_CHUNK * SHUF_CHUNK);
        }
        const size_t nch = (size_t)(wlen / SHUF_CHUNK);
        hipLaunchKernelGGL(k_chacha_words, dim3((unsigned)((wlen / 16 + 255) / 256)), dim3(256), 0, copy, key,
                           stream, wbase, wlen, d_words);
        std::vector<std::pair<double, size_t>> order(nch);
        for (size_t c = 0; c < nch; c++) {
            chunk_ok[c] = 0;
            const double off = std::max(0.0, (double)(wbase + c * SHUF_CHUNK) - (double)start);
            order[c] = {std::fmod(off, std::max(Ew, 1.0)), c};
        }
        std::sort(order.begin(), order.end());
        for (auto &oc : order) {
            const size_t c = oc.second;
            (void)hipMemcpyAsync(h_words + c * SHUF_CHUNK, d_words + c * SHUF_CHUNK, SHUF_CHUNK * 4,
                                 hipMemcpyDeviceToHost, copy);
            (void)hipEventRecord(chunk_ev[c], copy);
        }
        // ---- speculative walks of epochs 1 .. E-1
        {
            std::lock_guard<std::mutex> lk(mu);
            for (int e = 1; e < epochs; e++)
                for (int k = 0; k < K; k++) {
                    SpecWalk &s = spec[(e - 1) * K + k];
                    const double spread = 3.0 * sigma * std::sqrt((double)e);
                    const double guess = (double)start + e * Ew + ((k + 0.5) / K - 0.5) * spread;
                    s.start = (uint64_t)std::max((double)start, std::floor(guess));
                    s.epoch = e;
                    s.end = 0;
                    s.progress.store(-1, std::memory_order_relaxed);
                    s.done.store(0, std::memory_order_relaxed);
                    std::fill(s.ck.begin(), s.ck.end(), 0xFFFFFFFFu);
                }
            busy = nspec;
            gen++;
        }
        cv.notify_all();
        // ---- true walks
        uint64_t pos = start;
        bool cancelled = false;
        for (int e = 0; e < epochs && !cancelled; e++) {
            auto t0 = std::chrono::steady_clock::now();
            if (ev_used[slot][e]) (void)hipEventSynchronize(ev[slot][e]);   // previous upload of this buffer
            uint32_t *J = J_host[slot] + (size_t)e * n;
            uint32_t r = n;
            int met = -1;
            int walked = 0;
            while (r >= 2) {
                const uint64_t q = (pos / SHUF_CK + 1) * SHUF_CK;
                pos = walk_piece(pos, &r, J, scratch);
                if (cancel.load(std::memory_order_relaxed)) { cancelled = true; break; }
                if (pos != q || r < 2 || e == 0 || K == 0) continue;
                walked++;
                const int64_t c = (int64_t)((q - wbase) / SHUF_CK);
                for (int k = 0; k < K && met < 0; k++) {
                    SpecWalk &s = spec[(e - 1) * K + k];
                    if (s.start > q || c >= (int64_t)s.ck.size()) continue;
                    // wait until that walk has passed q (or finished before it)
                    while (s.progress.load(std::memory_order_acquire) < c && !s.done.load(std::memory_order_acquire) &&
                           !cancel.load(std::memory_order_relaxed))
                        std::this_thread::yield();
                    if (s.progress.load(std::memory_order_acquire) >= c && s.ck[c] == r) met = (e - 1) * K + k;
                }
                if (met >= 0) break;
            }
            if (cancelled) break;
            uint32_t *dJ = d_J[slot] + (size_t)e * n;
            if (met >= 0) {
                SpecWalk &s = spec[met];
                while (!s.done.load(std::memory_order_acquire) && !cancel.load(std::memory_order_relaxed))
                    std::this_thread::yield();
                if (!s.done.load(std::memory_order_acquire)) { cancelled = true; break; }
                pos = s.end;
                // J[r .. n) from the true walk, J[0 .. r) from the speculative walk
                (void)hipMemcpyAsync(dJ + r, J + r, sizeof(uint32_t) * (size_t)(n - r), hipMemcpyHostToDevice, copy);
                (void)hipMemcpyAsync(dJ, s.J, sizeof(uint32_t) * (size_t)r, hipMemcpyHostToDevice, copy);
                coalesced[slot][e] = walked;
            } else {
                if (n) J[0] = 0;
                (void)hipMemcpyAsync(dJ, J, sizeof(uint32_t) * n, hipMemcpyHostToDevice, copy);
                coalesced[slot][e] = -1;
            }
            end_pos[slot][e] = pos;
            (void)hipEventRecord(ev[slot][e], copy);
            ev_used[slot][e] = true;
            walk_ms[slot][e] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            SHUF_LOG("[shuf] epoch %d end=%llu met=%d (%.2f ms)\n", e, (unsigned long long)pos, coalesced[slot][e],
                     walk_ms[slot][e]);
            {
                std::lock_guard<std::mutex> lk(mu);
                ready[slot] = e + 1;
            }
            cv.notify_all();
        }
        SHUF_LOG("[shuf] job done cancelled=%d, stopping walkers\n", (int)cancelled);
        // leftover speculative walks matter only until their epoch is resolved:
        // stop them and wait, so the next job can reuse their buffers
        {
            std::unique_lock<std::mutex> lk(mu);
            cancel = true;
            cv.notify_all();
            // (at shutdown, workers that never picked up this job just exit)
            cv.wait(lk, [&] { return busy == 0 || quit; });
            cancel = false;
            job_running = false;
            if (cancelled) job_valid = false;
        }
        cv.notify_all();
    }
}

void ShuffleEngine::shutdown() {
    if (th.joinable()) {
        {
            std::lock_guard<std::mutex> lk(mu);
            quit = true;
            cancel = true;
        }
        cv.notify_all();
        th.join();
        for (auto &w : workers) w.join();
        workers.clear();
    }
    if (copy) { (void)hipStreamSynchronize(copy); (void)hipStreamDestroy(copy); copy = nullptr; }
    for (int s = 0; s < 2; s++) {
        for (int e = 0; e < epochs; e++) if (ev[s][e]) { (void)hipEventDestroy(ev[s][e]); ev[s][e] = nullptr; }
        if (J_host[s]) { (void)hipHostFree(J_host[s]); J_host[s] = nullptr; }
        if (d_J[s]) { (void)hipFree(d_J[s]); d_J[s] = nullptr; }
    }
    for (auto &e : chunk_ev) if (e) (void)hipEventDestroy(e);
    chunk_ev.clear();
    for (int i = 0; i < SHUF_MAX_SPEC; i++) if (spec[i].J) { (void)hipHostFree(spec[i].J); spec[i].J = nullptr; }
    if (d_words) { (void)hipFree(d_words); d_words = nullptr; }
    if (h_words) { (void)hipHostFree(h_words); h_words = nullptr; }
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

// shuffle_engine.hip — the host side of ppo_update's per-epoch shuffle
// (ppo.rs:1816 `indices.shuffle(rng)`, rand 0.8.5 SliceRandom::shuffle):
//
//   producers  : ChaCha12 words of the main StdRng stream, chunk by chunk,
//                ahead of the walker (WordRing);
//   walker     : the sequential rejection chain -> J[i] = gen_range(0..i+1)
//                for i = n-1..1 (shuffle_host.cpp), one epoch at a time;
//   copy stream: each finished epoch's J to HBM; an event per epoch lets the
//                compute stream wait for exactly that epoch.
//
// The walker is one update ahead: once an update's last shuffle is drawn, the
// next update's shuffles start at end + T*N*A (the rollout's Gumbel draws use
// exactly one word per (env, action)), so their chain overlaps the next
// rollout.  A different start (KL early stop, rng_set) cancels and restarts.
#include <algorithm>
#include <chrono>
#include <cstring>
#include "bppo_internal.h"
#include "shuffle_host.h"

namespace bppo {

// ------------------------------------------------------------ word ring ----
void WordRing::start(const Key8 &k, uint64_t strm, int nthreads) {
    key = k;
    stream = strm;
    buf = (uint32_t *)malloc(sizeof(uint32_t) * C * R);
    for (int i = 0; i < R; i++) chunk_id[i] = -1;
    next = floor = 0;
    for (int t = 0; t < nthreads; t++) {
        producers.emplace_back([this]() {
            for (;;) {
                int64_t k2;
                uint64_t g;
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return quit || next < floor + R; });
                    if (quit) return;
                    k2 = next++;
                    g = gen;
                    inflight++;
                }
                uint32_t *dst = buf + (size_t)(k2 % R) * C;
                bppo_host::chacha12_words(key.k, stream, (uint64_t)k2 * C, dst, C);
                {
                    std::lock_guard<std::mutex> lk(mu);
                    if (g == gen) chunk_id[k2 % R] = k2;
                    inflight--;
                }
                cv.notify_all();
            }
        });
    }
}

void WordRing::reset(int64_t first_chunk) {
    std::unique_lock<std::mutex> lk(mu);
    gen++;
    cv.wait(lk, [&] { return inflight == 0; });
    for (int i = 0; i < R; i++) chunk_id[i] = -1;
    next = floor = first_chunk;
    lk.unlock();
    cv.notify_all();
}

const uint32_t *WordRing::get(int64_t chunk) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return quit || chunk_id[chunk % R] == chunk; });
    return buf + (size_t)(chunk % R) * C;
}

void WordRing::release_below(int64_t chunk) {
    {
        std::lock_guard<std::mutex> lk(mu);
        if (chunk > floor) floor = chunk;
    }
    cv.notify_all();
}

void WordRing::stop() {
    {
        std::lock_guard<std::mutex> lk(mu);
        quit = true;
    }
    cv.notify_all();
    for (auto &t : producers) t.join();
    producers.clear();
    free(buf);
    buf = nullptr;
}

// --------------------------------------------------------------- engine ----
bppo_status ShuffleEngine::init(int device, const Key8 &key, uint64_t stream, uint32_t n_, int epochs_,
                                std::string &err) {
    dev = device;
    n = n_;
    epochs = epochs_;
    if (epochs > SHUF_MAX_EPOCHS) { err = "num_epochs > 32 not supported"; return BPPO_ERR_ARG; }
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
    words.start(key, stream, 2);
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

void ShuffleEngine::run() {
    (void)hipSetDevice(dev);
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
        const int64_t C = (int64_t)WordRing::C;
        words.reset((int64_t)(start / (uint64_t)C));
        uint64_t pos = start;
        bool cancelled = false;
        for (int e = 0; e < epochs && !cancelled; e++) {
            auto t0 = std::chrono::steady_clock::now();
            if (ev_used[slot][e]) (void)hipEventSynchronize(ev[slot][e]);   // previous upload of this buffer
            uint32_t *J = J_host[slot] + (size_t)e * n;
            uint32_t r = n;
            while (r >= 2) {
                const int64_t ch = (int64_t)(pos / (uint64_t)C);
                const uint32_t *w = words.get(ch);
                const size_t off = (size_t)(pos - (uint64_t)ch * (uint64_t)C);
                pos += bppo_host::chain_walk(w + off, (size_t)C - off, &r, J);
                if ((pos / (uint64_t)C) != (uint64_t)ch) words.release_below((int64_t)(pos / (uint64_t)C));
                {
                    std::lock_guard<std::mutex> lk(mu);
                    if (cancel) { cancelled = true; break; }
                }
            }
            if (cancelled) break;
            J[0] = 0;
            end_pos[slot][e] = pos;
            (void)hipMemcpyAsync(d_J[slot] + (size_t)e * n, J, sizeof(uint32_t) * n, hipMemcpyHostToDevice,
                                 copy);
            (void)hipEventRecord(ev[slot][e], copy);
            ev_used[slot][e] = true;
            walk_ms[slot][e] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
            {
                std::lock_guard<std::mutex> lk(mu);
                ready[slot] = e + 1;
            }
            cv.notify_all();
        }
        {
            std::lock_guard<std::mutex> lk(mu);
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
        words.stop();
    }
    if (copy) { (void)hipStreamSynchronize(copy); (void)hipStreamDestroy(copy); copy = nullptr; }
    for (int s = 0; s < 2; s++) {
        for (int e = 0; e < epochs; e++) if (ev[s][e]) { (void)hipEventDestroy(ev[s][e]); ev[s][e] = nullptr; }
        if (J_host[s]) { (void)hipHostFree(J_host[s]); J_host[s] = nullptr; }
        if (d_J[s]) { (void)hipFree(d_J[s]); d_J[s] = nullptr; }
    }
}

// single-shot host walk (parity hook): J for one shuffle of n from word position pos
uint64_t shuffle_walk_host(const Key8 &key, uint64_t stream, uint64_t pos, uint32_t n, uint32_t *J) {
    const size_t C = WordRing::C;
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

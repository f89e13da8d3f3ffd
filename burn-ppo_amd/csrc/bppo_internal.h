// bppo_internal.h — context layout and kernel launchers shared by the HIP
// translation units of libbppo.so.  Not part of the public C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string>
#include <vector>
#include <thread>
#include <mutex>
#include <condition_variable>
#include <atomic>
#include <memory>
#include "../../include/bppo.h"
#include "bppo_device.h"

namespace bppo {

// ---------------------------------------------------------------- layout ----
struct NetLayout {
    static constexpr int MAX_LAYERS = 16;   // checked by ctx_init before make_layout
    int n_layers = 0;             // linear layers in record order
    int in[MAX_LAYERS], out[MAX_LAYERS];
    size_t w[MAX_LAYERS], b[MAX_LAYERS];
    int n_actor_hidden = 0;       // hidden layers of the actor / shared backbone
    int policy = 0, value = 0;    // layer indices of the heads
    int critic_first = -1;        // critic layers [critic_first, value) (CTDE, split_networks)
    int critic_fc0 = -1;          // its first FC layer (split CNN: after the critic's own conv stack)
    int ctde = 0, relu = 1;       // ctde: two trunks (CTDE, or split_networks with the critic on obs)
    int rec[MAX_LAYERS];          // Burn record position of layer l (split_networks: actor, critic, heads)
    size_t n_params = 0;
    // CNN (network/cnn.rs): layers [0, n_conv) are the conv layers (in = Cin k k,
    // out = Cout; weight [Cout][Cin][k][k] then bias in Burn record order), then the
    // FC layers [n_conv, n_actor_hidden), policy, value; split_networks (cnn.rs:116-135)
    // adds the critic's conv stack [critic_first, critic_fc0) and FC layers [critic_fc0, value)
    int n_conv = 0, ksize = 3, H = 0, W = 0, C = 0, E = 0, fdim = 0;
    int conv_cin[4] = {0, 0, 0, 0};
    // first layer of conv stack s (0: actor / shared, 1: the split critic's)
    int conv_base(int s) const { return s ? critic_first : 0; }
    bool is_conv(int l) const {
        return n_conv && (l < n_conv || (critic_fc0 > critic_first && l >= critic_first && l < critic_fc0));
    }
};
NetLayout make_layout(const bppo_config &c, int obs_dim, int priv_dim, int act_dim);

// episode record written by the rollout kernel
constexpr int EP_SUMMARY_BLOCKS = 128;   // k_ep_summary grid (partial sums per block)
constexpr int WIDE_SPLIT_MIN_ROWS = 32768;   // wide_minibatch: the split-bf16 GEMMs from this minibatch size on
constexpr int RPOOL_K = 16;              // CfgB rollout: reset states drawn ahead per env (k_reset_pool)
constexpr int TM_SLOTS = 10;             // phase timer event pairs (enum TM_* below)
constexpr int ROLL_HOST_WORDS = 2 + 2 * EP_SUMMARY_BLOCKS;     // pinned doubles per rollout slot
constexpr int ADV_STREAM_BLOCKS = 512, ADV_STREAM_MAXM = 16;   // k_adv_stream grid, most minibatches
// metric slots after the gradient, d_grad[np + k]: GRAD_METRIC_SLOTS (= WM_COUNT, bppo_wide.h)
// travel with the gradient through the W > 1 SUM all-reduce; value_error_max (slot
// GRAD_VEMAX) cannot be summed, so its reduction also writes a rank-local copy to slot
// GRAD_VEMAX_LOCAL, past the all-reduced range, and the metric row reads that copy
constexpr int GRAD_METRIC_SLOTS = 14, GRAD_VEMAX = 9, GRAD_VEMAX_LOCAL = GRAD_METRIC_SLOTS;

struct EpisodeRec {
    float total_reward[BPPO_MAX_PLAYERS];
    int32_t length, env_index, step, pad;
};

// Welford state (count, mean, M2) — Chan merge is the associative combine
struct Welford { double n, mean, m2; };

// -------------------------------------------------------------- shuffle -----
// rand 0.8.5 SliceRandom::shuffle (ppo.rs:1816) on the main StdRng.  The draw
// chain (every draw may reject, so each draw's word position depends on all
// earlier ones) is walked on host threads (shuffle_host.cpp) over ChaCha12 words
// made on the GPU; each epoch's swap targets J[i] go to HBM on a copy stream and
// the GPU turns them into the permutation (k_shuffle.hip).  Epoch e >= 1 starts
// where epoch e-1 ends, which is known only after walking it, so K speculative
// walks per epoch start at once near the expected boundary; the true walk of
// epoch e runs from the real boundary only until its state (word position,
// remaining range) meets one of them, after which both are the same walk.
constexpr int SHUF_MAX_EPOCHS = 32;
constexpr int SHUF_MAX_SPEC = 64;
constexpr uint64_t SHUF_CK = 1024;               // checkpoint spacing (words) = GPU J segment length
constexpr uint64_t SHUF_CHUNK = (uint64_t)1 << 20; // words per GPU->host copy
// shuffle_windows (bppo_config): epoch e of an update draws from word position
// S + e * shuffle_window(n) of the main stream, S the update's first shuffle word, and
// the next rollout starts at S + epochs * shuffle_window(n).  A shuffle of n uses ~1.39 n
// words (2 n at most but for a ~2^-(10^5) tail), so the window is 2 n + 2^20.
__host__ __device__ constexpr uint64_t shuffle_window(uint64_t n) { return 2 * n + ((uint64_t)1 << 20); }

struct SpecWalk {
    uint64_t start = 0, end = 0, ck_base = 0;     // checkpoint c is word position ck_base + c*CK
    int wbuf = 0;                                 // word buffer it reads
    std::vector<uint32_t> ck;                     // remaining range at checkpoint c
    std::atomic<int64_t> progress{-1};            // last checkpoint index written
    std::atomic<int> done{1};
    std::atomic<bool> stop{false};
    std::atomic<int> merged_to{-1};               // left neighbour it coalesced with (then stopped)
    uint64_t merge_q = 0;                         // word position of that checkpoint (set before merged_to)
    uint64_t gen = 0;                             // assignment counter (the worker follows it)
    uint64_t job = 0;                             // engine job (seq) that launched it
    bool running = false;                         // guarded by the engine mutex
};

struct WordBuf {                                  // ChaCha12 words made on the GPU for one job
    uint32_t *d = nullptr, *h = nullptr;
    uint64_t cap = 0;                             // words
    struct Region { uint64_t base = 0, len = 0, off = 0; } reg[SHUF_MAX_EPOCHS];
    int nreg = 0;
    std::vector<hipEvent_t> ev;                   // per SHUF_CHUNK chunk of h
    std::unique_ptr<std::atomic<int>[]> ok;
    uint32_t *hd = nullptr;                       // windowed GPU words: h is registered (pinned)
    bool gpu = false;                             // windowed: chunks of h are copied from d (ev[c] completes)
    uint64_t made_for = ~0ull;                    // job start whose words d (and h's copies) hold
};

// target-range table of the ranged Fisher-Yates bucketing (k_shuffle.hip)
struct FyRanges {
    uint32_t *x = nullptr;            // device [nb + 1] range boundaries
    uint32_t *cb = nullptr;           // device [ncb] first range of each 2^11-target block
    uint32_t *cursor = nullptr;       // device [nb] steps per range (k_fyb_bucket; reset by k_fyb_link)
    uint2 *P = nullptr;               // device [nb][FYB_CAP] (step, target) slots of each range
    uint32_t *flag = nullptr;         // device: a range overflowed (0 between permutations)
    int nb = 0, ncb = 0;              // nb = 0: direct bucketing only
    uint32_t n = 0;
};

// one epoch's minibatch split (ppo.rs:1830-1836: minibatch m has base + (m < rem)
// rows) and the block chunking of its per-minibatch advantage statistics: block b
// owns shuffled positions [b C, (b + 1) C), C no larger than the smallest
// minibatch, so a block touches at most two minibatches (k_update.hip)
struct EpochSplit { uint32_t B, base, rem, M; };
__device__ __forceinline__ uint32_t mb_of(uint32_t i, const EpochSplit &s) {
    const uint32_t big = s.rem * (s.base + 1);
    return i < big ? i / (s.base + 1) : s.rem + (i - big) / s.base;
}
struct ShuffleEngine {
    int dev = 0;
    uint32_t n = 0;
    int epochs = 0;
    Key8 key{};
    uint64_t stream = 0;
    uint64_t gap = 0;                             // words between an update's last shuffle and the next update's first
    uint64_t win = 0;                             // shuffle_windows: epoch e starts at job start + e * win (0: chained)
    bool keep_guess = true;                       // keep the nearest guessed walks beside an exact continuation
    bool pair = false;                            // windowed: worker 2m walks epochs 2m and 2m+1 interleaved
    bool win_producers = false;                   // windowed: host word producers (default: the walks make their words)
    bool win_gpu_words = false;                   // windowed: the job's GPU words are copied to the host (SDMA)
    hipStream_t d2h = nullptr;                    // those copies
    hipEvent_t words_made = nullptr;
    double Ew = 0.0, sigma = 0.0;                 // expected words per shuffle, its std dev
    int K = 0;                                    // speculative walks per epoch boundary
    int host_cpus = 16;                           // CPU budget of this rank (BPPO_HOST_THREADS)
    WordBuf wb[2];                                // double-buffered by job parity
    // walker slots: [0, ncur) K per epoch C..E-1 of the current job; then two
    // (by job parity) carry groups of C*K for the next job's epochs 0..C-1
    // carry sets of K for the next job's first epoch (alternating by job parity)
    SpecWalk spec[SHUF_MAX_SPEC];
    int nspec = 0, ncur = 0;
    int C = 1;                                    // leading epochs of the next job speculated during this one
    int fr_depth = 0;                             // frontier scheduling depth (0: all groups at job start)
    // exact continuations: when a walk of this job's last epoch finishes that epoch
    // at word x, a walk of the next job's first epoch starts at x + gap — exactly
    // where the next job starts whenever the true walk met that chain.  Two sets of
    // K slots (by job parity) after the carry groups.
    int cont0 = 0;                                // first continuation slot (0: none)
    bool cont_valid[2] = {false, false};
    int cont_src0 = -1, cont_dst0 = -1, cont_wb = 0;   // this job's last-epoch group -> its set (mu)
    uint64_t cont_seq = 0;
    std::vector<std::thread> workers;
    // host word producers: the job's ChaCha12 words into the pinned word buffer,
    // chunk by chunk in the order the walks need them (no device -> host copies)
    std::vector<std::thread> gens;
    std::vector<std::pair<uint64_t, size_t>> gen_order;   // (word position, chunk) of the current job
    WordBuf *gen_buf = nullptr;
    std::atomic<size_t> gen_next{0};
    uint64_t gen_job = 0;
    int gen_active = 0;                           // producers inside a job's list (mu)
    void generator();
    uint64_t seq = 0;                             // jobs started
    bool carry_valid[2] = {false, false};
    // job control: a job = one update's shuffles in a J slot.  The engine chains
    // the next job (start = last end + gap) as soon as one is resolved, at most
    // one job ahead of the job the caller consumes.
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    bool quit = false;
    bool slot_valid[2] = {false, false};          // slot holds (or is computing) the job for slot_start
    uint64_t slot_start[2] = {0, 0};
    int pending = -1, running = -1;               // slot queued / being computed
    int consumer = -1;                            // slot the caller last asked for
    int chain_from = -1;                          // resolved slot whose successor may be chained
    uint64_t chain_start = 0;
    int last_slot = 1;
    hipEvent_t consumed[2] = {nullptr, nullptr};  // recorded by the caller after its last read of d_J[slot]
    bool consumed_used[2] = {false, false};
    std::atomic<bool> cancel{false};
    int ready[2] = {0, 0};                        // epochs of the slot's job already on the device
    uint64_t end_pos[2][SHUF_MAX_EPOCHS];
    // each epoch's walk as segments (start position, start range, end position),
    // one per checkpoint interval; the GPU rebuilds J from them (k_expand_J)
    struct Seg { uint64_t pos0, pos1; uint32_t r0, pad; };
    int maxseg = 0;
    Seg *seg_host[2] = {nullptr, nullptr};        // pinned [epochs][maxseg]
    Seg *d_seg[2] = {nullptr, nullptr};
    uint32_t *d_J[2] = {nullptr, nullptr};        // device [epochs][n]
    hipEvent_t ev[2][SHUF_MAX_EPOCHS] = {};
    bool ev_used[2][SHUF_MAX_EPOCHS] = {};
    hipStream_t copy = nullptr;
    // the caller's end-of-update event (bppo_ctx::ev_upd): with BPPO_XJ_GATE the J expansions
    // wait for the update enqueued last, so a job the walks finished early is not expanded
    // beside that update's minibatches (1: every epoch, 2: epochs after the first)
    hipEvent_t gate = nullptr;
    double walk_ms[2][SHUF_MAX_EPOCHS] = {};
    int coalesced[2][SHUF_MAX_EPOCHS] = {};       // checkpoints walked before meeting a speculative walk (-1: none)
    std::atomic<uint64_t> spec_words{0}, true_words{0};   // words walked since the caller last read them
    std::atomic<uint64_t> tsc_walk{0}, tsc_words{0};      // TSC ticks walking / getting words (all walks)
    bppo_status init(int device, const Key8 &key, uint64_t stream, uint32_t n_, int epochs_, uint64_t gap_,
                     std::string &err, bool windows = false);
    bool run_windowed(int slot, uint64_t start);   // one job of independent epoch walks (false: cancelled)
    void xj_gate_wait(int e);                      // BPPO_XJ_GATE: copy waits on `gate` before epoch e's expansion
    uint64_t job_end(int slot) const { return win ? slot_start[slot] + (uint64_t)epochs * win : end_pos[slot][epochs - 1]; }
    // a HIP call of the engine's own thread that failed (its uploads, J expansions, events):
    // the first one is kept and the caller's next wait on the engine reports it
    std::atomic<bool> hip_bad{false};
    std::mutex hip_mu;
    std::string hip_msg;                          // (hip_mu) written once, before hip_bad is set
    void hip_note(hipError_t e, const char *what);
    bool failed(std::string &msg) const;          // -> true and the message after a failure
    int ensure(uint64_t start);               // job for this start (reused if already running/done) -> slot
    hipError_t release(int slot, hipStream_t st);   // the caller is done enqueuing reads of d_J[slot] on st
    void wait_epoch(int slot, int e);
    bool epoch_ready(int slot, int e);        // non-blocking wait_epoch
    void shutdown();
    void run();
    void worker(int i);
    void launch_walk(int i, uint64_t start, int wbuf);   // mu held
    void stop_walks(int lo, int hi);                     // stop and wait (mu not held)
    const uint32_t *words(int b, uint64_t pos, uint64_t len, std::vector<uint32_t> &scratch, bool true_walk = false);
    // the true walk's second word source (run thread only): the previous job's carry region,
    // which holds this job's first epochs (made once, not again in this job's region 0)
    int alt_b = -1;
    WordBuf::Region alt_reg;
    struct WalkStats { uint64_t words = 0, tsc_walk = 0, tsc_words = 0; };
    void walk_pair(int i, WalkStats &st);
    uint64_t walk_piece(int b, uint64_t pos, uint32_t *r, std::vector<uint32_t> &scratch, WalkStats &st,
                        bool true_walk = false);
    void flush(WalkStats &st, std::atomic<uint64_t> &words_ctr);
    int peek(int i, uint64_t q, uint32_t *r);     // walk i's range at checkpoint q: 1 known, 0 not yet, -1 never
};
uint64_t shuffle_walk_host(const Key8 &key, uint64_t stream, uint64_t pos, uint32_t n, uint32_t *J);
// a low-priority side stream (shuffle copy stream, Fisher-Yates stream)
hipError_t make_side_stream(int device, hipStream_t *st);

struct Timers {
    hipEvent_t a = nullptr, b = nullptr;
};

}  // namespace bppo

struct bppo_ctx {
    bppo_config cfg;
    int dev = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    int N = 0, T = 0, D = 0, A = 0, P = 1, G = 0;
    int Pa = 1;                       // players actually seated (Skull: player_count; else P)
    bppo::NetLayout net;
    // parameters + Adam
    float *d_params = nullptr, *d_m1 = nullptr, *d_m2 = nullptr;
    std::vector<int32_t> adam_t;
    float *d_grad = nullptr;          // [n_params + metric slots]
    double *d_grad64 = nullptr;
    float *d_slab = nullptr;          // per-wave partial gradients
    size_t slab_rows = 0;
    int slab_used = 0;                // waves that wrote a row in the last minibatch launch
    int relu_mfma = 1;                // CfgB net (64x2 relu): the MFMA minibatch kernel
    int mb_kernel = 0;                // bppo_set_minibatch_kernel: 0 exact first / split rest, 1 exact, 2 split
    float *dbg_params = nullptr;      // bppo_debug_record_params: host [dbg_params_max][n_params]
    int dbg_params_max = 0;
    // env state (CartPole SoA)
    float *d_cp = nullptr;            // x, x_dot, theta, theta_dot  [4][N]
    int32_t *d_steps = nullptr;
    uint64_t *d_env_pos = nullptr;
    float *d_ep_ret = nullptr;        // [N*P]
    int32_t *d_ep_len = nullptr;
    uint64_t env_step = 0;            // the envs' current_step (Environment::set_step, env.rs:329-333)
    // reward_shaping_coef Schedule (schedule.rs:29) as (value, step) milestones
    std::vector<double> shaping_v;
    std::vector<uint64_t> shaping_s;
    // rollout buffer [T][N][...]
    float *d_obs = nullptr, *d_rew = nullptr, *d_rew_raw = nullptr, *d_done = nullptr;
    float *d_val = nullptr, *d_logp = nullptr, *d_adv = nullptr, *d_ret = nullptr;
    int32_t *d_act = nullptr;
    double *d_X = nullptr;            // rolling returns per (t,e) for the return-normalizer scan
    float *d_gumbel = nullptr;        // CfgB MFMA rollout: Gumbel noise [T][N][2], made ahead of it
    float4 *d_rpool = nullptr;        // CfgB MFMA rollout: each env's next RPOOL_K reset states [K][N], made ahead of it
    uint64_t *d_rpos = nullptr;       //   and the stream position after each [K][N]
    // normalizers
    double *d_on = nullptr;           // [3][D]: mean, M2, (count in slot) ; host mirror below
    std::vector<double> on_mean, on_m2;
    double on_count = 0;
    double *d_obs_part = nullptr;     // per-env Welford partials [N][2*D]
    double *d_rn_returns = nullptr;   // [N*P]
    double *d_rn_stats = nullptr;     // {mean, M2, count}
    bppo::Welford *d_scan_agg = nullptr;
    // bootstrap
    float *d_last_v = nullptr;
    // episodes
    bppo::EpisodeRec *d_eps = nullptr;
    int32_t *d_ep_count = nullptr;
    int32_t eps_cap = 0;
    double *d_ep_sum = nullptr;          // [EP_SUMMARY_BLOCKS][2] partial sums (return, length)
    int32_t *d_err = nullptr;
    // main RNG
    bppo::Key8 rng_key{};
    uint64_t rng_pos = 0;
    // shuffle
    bppo::ShuffleEngine shuf;
    uint32_t *d_perm = nullptr;       // shuffled indices of the current epoch (may point into d_perm_ep)
    uint32_t *d_perm_base = nullptr;  // allocation behind d_perm for the opponent-pool path
    // the engine's epochs are permuted on fy_stream as soon as their J is on the
    // device — from the rollout on, so the permutations run beside the rollout
    // and the return-normaliser / GAE kernels instead of between minibatches
    uint32_t *d_perm_ep = nullptr;    // [epochs][TN] one permutation per epoch
    uint32_t *d_inv_ep = nullptr;     // [epochs][TN] their inverses (row -> shuffled position)
    double *d_advpart = nullptr;      // k_adv_stream block partials
    hipStream_t fy_stream = nullptr;
    bool fy_shared = false;           // BPPO_FY_ON_COPY=1 (A/B): fy_stream IS the engine's copy stream
    hipEvent_t fy_ev[bppo::SHUF_MAX_EPOCHS] = {};
    // CfgB 64-lane rollout: its Gumbel words and reset pool made on prep_stream as soon as the
    // previous env-state writer (ev_env: the last rollout / reset / vecenv step) finished, i.e.
    // beside the previous update's minibatches, not between them and the rollout (r06)
    hipStream_t prep_stream = nullptr;
    hipEvent_t ev_env = nullptr, ev_prep = nullptr;
    int fy_slot = -1, fy_done = 0;    // engine slot whose epochs [0, fy_done) are enqueued on fy_stream
    uint32_t *d_fy = nullptr;         // Fisher-Yates scratch [4][TN]: count/offset, bucket, succ, fw
    uint32_t *d_scan = nullptr;       // scan block sums
    bppo::FyRanges fyr;               // target ranges of the ranged Fisher-Yates bucketing
    int shuf_slot = -1;               // engine slot holding this update's J
    // scratch
    double *d_red = nullptr;          // reduction scratch
    double *h_red = nullptr;          // pinned mirror
    double *hd_red = nullptr;         // h_red's device address (BPPO_ZERO_COPY=1: kernels write their
                                      // few host-bound results there instead of a D2H copy)
    float *h_rows = nullptr;          // pinned: the update's metric rows
    float *d_mb_stats = nullptr;      // advantage [mean, std, min, max] of each minibatch of the epoch [M][4]
    float *d_mb_cur = nullptr;        // the current minibatch's row of d_mb_stats
    float *d_rows = nullptr;          // per-minibatch metric rows of one update [E*M][WM_COUNT + 4]
    std::vector<float> last_rows;     // the last update's rows, host copy (bppo_buffer_get "minibatch_rows")
    // CfgB net: the update's minibatch rows packed in two arrays, so every store of the
    // rollout and of GAE covers whole 32-byte sectors of consecutive rows: d_rowA [B][2]
    // float4 = [obs 0..3][obs 4, action, log-prob, value] (32 B, the rollout writes it),
    // d_rowB [B] float2 = [advantage, return] (8 B, GAE writes it); k_pack_rows otherwise
    float4 *d_rowA = nullptr;
    float2 *d_rowB = nullptr;
    // all-reduce hook
    bppo_allreduce_fn allreduce = nullptr;
    void *allreduce_user = nullptr;
    int world = 1;
    int rank = -1;                    // bppo_set_rank: this context's slot in W > 1 all-gathers (unset: -1)
    float *d_pa_gather = nullptr;     // PopArt at W > 1: [world][9] floats (3 doubles, 3 floats each)
    int allreduce_async = 0;          // callback enqueues on the stream (no host sync per minibatch)
    // ---- multi-player ("wide") path: Connect Four / Liar's Dice (wide_api.hip)
    int wide = 0;                     // env_kind != CartPole
    int L = 0;                        // rollout row length G + D: [priv | obs]
    int rows_max = 0;                 // max(N, largest minibatch): rows of the activation buffers
    void *d_wstate = nullptr;         // per-env state structs [N]
    float *d_xc = nullptr;            // rollout rows [T][N][L]
    float *d_obs_raw = nullptr;       // normalize_obs: raw obs rows [T][N][D] for the stats update
    // opponent pool (ppo.rs:537-1063): K opponent models, envs [0, n_opp) play them
    int opp_K = 0, n_opp = 0;
    float *d_opp_params = nullptr;    // [K][n_params]
    double *d_opp_on = nullptr;       // [K][2D + 1] obs normalizer per model
    std::vector<int> opp_has_norm;
    int32_t *d_lpos = nullptr, *d_p2o = nullptr, *d_curopp = nullptr;   // [n_opp], [n_opp][P], [P - 1]
    int32_t *d_group = nullptr, *d_gpos = nullptr;                        // per step [N]
    float *d_valid = nullptr;         // learner-turn flags [T][N]
    uint64_t *d_rngpos = nullptr;     // main RNG word position during an opponent rollout
    float *d_oraw = nullptr, *d_oxc = nullptr, *d_ologits = nullptr;     // [N][L], [N][L], [N][A]
    uint32_t *d_vidx = nullptr, *d_Jopp = nullptr;                         // [T N]
    uint32_t *d_nvalid = nullptr;
    uint32_t n_valid = 0;
    int32_t *d_gbase = nullptr, *h_gbase = nullptr;   // per step: draw-order base of each mover group
    double *d_obsw_part = nullptr;    // normalize_obs: per-chunk partial stats [256][D][3]
    size_t obsw_part_n = 0;
    uint8_t *d_mask = nullptr;        // action masks [T][N][A] (0/1)
    int32_t *d_players = nullptr;     // acting player [T][N]
    float *d_allr = nullptr;          // all_rewards [T][N][P]
    float *d_lvpp = nullptr;          // last_value_per_player [N][P]
    float *d_hbuf = nullptr;          // hidden activations, layer l at hoff[l], [rows][out[l]]
    size_t hoff[16] = {};
    float *d_logits = nullptr, *d_values = nullptr;  // forward outputs [rows][A], [rows]
    float *d_xcg = nullptr;           // gathered minibatch rows [mb][L]
    float *d_dout = nullptr;          // dL/d[logits | value] [mb][A+1]
    float *d_dz[2] = {nullptr, nullptr};            // backward ping-pong [mb][Wmax]
    float *d_heads = nullptr, *d_heads_b = nullptr; // packed shared-trunk heads [W][A+1], [A+1]
    float *d_part = nullptr, *d_colsum = nullptr;   // split-K weight-grad scratch
    double *d_mpart = nullptr;        // loss-metric partials
    // CNN actor-critic (cnn.hip): conv outputs (post-relu, NHWC rows) per conv layer,
    // im2col scratch, the flattened NCHW features + extra [rows][fdim], backward
    // scratch, conv weights packed [k k Cin][Cout] (GEMM operand) and their gradient
    // -- per conv stack s (0: actor / shared, 1: the split_networks critic)
    float *d_cnn_y[2][4] = {};
    float *d_cnn_f[2] = {nullptr, nullptr};
    float *d_cnn_dy[2] = {nullptr, nullptr};
    float *d_cnn_wt = nullptr, *d_cnn_wd = nullptr, *d_cnn_owt = nullptr, *d_cnn_dwt = nullptr;
    size_t cnn_wt_off[2][4] = {};
    size_t cnn_wd_off[2][4] = {};     // the input-gradient operands (taps padded, gemm_conv_tap_pad)
    int cnn_stacks = 1;
    // PopArt value normalization (popart.hip, normalization.rs:262-366): running
    // statistics on the host, normalized update buffers, the update's views
    double pa_mean = 0.0, pa_m2 = 0.0, pa_count = 0.0, pa_eps = 1e-4;
    float pa_rescale_mag = 0.0f;
    double pa_tsum = 0.0, pa_tsq = 0.0, pa_tcount = 0.0;
    float *d_ret_n = nullptr, *d_val_n = nullptr;
    double *d_pa_part = nullptr;
    const float *u_ret = nullptr, *u_val = nullptr;   // returns / old values the minibatches read
    float *d_bxc = nullptr;           // bootstrap / VecEnv scratch rows [N][L]
    uint8_t *d_bmask = nullptr;
    int32_t *d_bplayers = nullptr;
    int32_t *d_act_in = nullptr;      // VecEnv::step actions [N]
    float *d_scr_r = nullptr;         // VecEnv::step rewards [N][P]
    uint8_t *d_scr_d = nullptr;       // VecEnv::step dones [N]
    // timing
    hipEvent_t ev[bppo::TM_SLOTS][2] = {};
    hipEvent_t ev_block = nullptr;    // blocking-sync event for host waits on the stream
    float last_ms[8] = {0};
    double last_walk_ms = 0.0, last_wait_ms = 0.0;
    double sync_wait_ms = 0.0, last_host_ms = 0.0, last_sync_ms = 0.0;   // bppo_train_step host split
    double wait_est_us = 0.0;         // recent per-update waits (wait_event: one coarse sleep first)
    // the fused CartPole minibatch kernel alone (no slab reduction), every launch of the
    // last update: bppo_last_kernel_ms "minibatch_kernel" (mean), "_min", "_max"
    static constexpr int MB_EV = 64;
    hipEvent_t mb_ev[MB_EV][2] = {};
    int mb_ev_n = 0;
    int mb_launch = 0;                // minibatch kernel launches of this update (mb_ev sampling)
    float mb_k_mean = 0.0f, mb_k_min = 0.0f, mb_k_max = 0.0f;
    bool mb_ev_split[MB_EV] = {};     // launch i ran k_minibatch_split (else the exact k_minibatch_mfma)
    float mb_k_split = 0.0f, mb_k_exact = 0.0f;   // mean of each kind's launches (0: none)
    double last_spec_mwords = 0.0, last_true_mwords = 0.0;   // host walk work since the previous update
    double last_walk_cpu_ms = 0.0, last_words_cpu_ms = 0.0;   // thread time in chain_walk / in words()
    int last_met = 0;
    int collected = 0, gae_done = 0;
    // bppo_train_steps pipelining
    hipEvent_t ev_upd = nullptr;      // end of an update's work (its host wait)
    int coll_slot = 1;                // pinned / timer slot of the last enqueued rollout
    uint64_t rollout_rng_pos[2] = {0, 0};
    bool prefetch_next = false, prefetched = false;
    // packed update rows written by the MFMA rollout (obs, action, log-prob, value) and
    // the GAE pass (advantage, return): k_pack_rows is skipped when both did
    bool rows_from_rollout = false, rows_packed = false;
    uint64_t prefetch_env_step = 0;
    // explained variance (bppo_set_explained_variance_mode): 0 = f64 sums on the device
    // (k_ev); 1 = the reference's f32 sequential sums (ppo.rs:1268-1294) on a host thread,
    // from D2H copies of the buffers made on ev_stream beside the update
    int ev_mode = 0;
    hipStream_t ev_stream = nullptr;
    hipEvent_t ev_gae = nullptr, ev_copied = nullptr;
    float *h_ev_v = nullptr, *h_ev_r = nullptr, *h_ev_valid = nullptr;
    std::thread ev_thread;
    float ev_ref = 0.0f;
};

namespace bppo {
// kernel-phase timer slots
enum { TM_ROLLOUT = 0, TM_GAE = 1, TM_UPDATE = 2, TM_FWDBWD = 3, TM_RETNORM = 4, TM_SHUFFLE = 5,
       TM_ADAM = 6, TM_BOOT = 7 };
// the rollout / return-normaliser events of the other rollout slot (bppo_train_steps
// enqueues a rollout while the previous one's events are still to be read)
enum { TM_ROLLOUT_B = 8, TM_RETNORM_B = 9 };

// launchers (k_rollout.hip)
bppo_status launch_cartpole_reset(bppo_ctx *c);
bppo_status launch_cartpole_rollout(bppo_ctx *c, uint64_t base_pos, const double *mean,
                                    const double *sd, int norm_on);
bppo_status launch_cartpole_vecenv_step(bppo_ctx *c, const int32_t *d_actions, float *d_rew,
                                        uint8_t *d_done, float *d_obs_out);
bppo_status launch_cartpole_observe(bppo_ctx *c, float *d_obs_out);
bppo_status launch_obs_norm_merge(bppo_ctx *c);
bppo_status launch_episode_summary(bppo_ctx *c, double *host_slot);
// BPPO_ZERO_COPY=1 (A/B): the episode summary and the explained-variance sums written into
// pinned host memory by their kernels instead of copied after them
inline bool zero_copy() {
    static const bool z = getenv("BPPO_ZERO_COPY") && atoi(getenv("BPPO_ZERO_COPY")) == 1;
    return z;
}
bppo_status launch_obs_norm_rows(bppo_ctx *c, int rows, float *x, int ld, float *raw);
bppo_status launch_obs_norm_rows_on(bppo_ctx *c, int rows, float *x, int ld, float *raw, const double *on);
bppo_status launch_bootstrap(bppo_ctx *c, const double *mean, const double *sd, int norm_on);
bppo_status launch_forward_rows(bppo_ctx *c, const float *d_obs, int B, float *d_logits,
                                float *d_values);
// (k_gae.hip)
// (no context: the launch's HIP status goes to *herr when given)
bppo_status launch_gae_1p(const float *r, const float *d, const float *v, const float *lv, int T,
                          int N, float gamma, float lambda, float *adv, float *ret, hipStream_t s,
                          float2 *pairs = nullptr, bool *pairs_done = nullptr, hipError_t *herr = nullptr);
bppo_status launch_gae_mp(const float *ar, const int32_t *pl, const float *d, const float *v,
                          const float *lvpp, int T, int N, int P, float gamma, float lambda,
                          float *adv, float *ret, hipStream_t s, hipError_t *herr = nullptr);
bppo_status launch_return_norm(bppo_ctx *c);
// (k_update.hip)
bppo_status launch_fisher_yates(bppo_ctx *c, const uint32_t *d_J, uint32_t n);
hipError_t fisher_yates_device(const uint32_t *d_J, uint32_t n, uint32_t *scratch, uint32_t *scan, uint32_t *perm,
                               hipStream_t st, const FyRanges *rg, uint32_t *inv = nullptr);
hipError_t fy_ranges_init(FyRanges &r, uint32_t n);
void fy_ranges_free(FyRanges &r);
bppo_status launch_epoch_adv_stats(bppo_ctx *c, uint32_t B, int M, const uint32_t *inv = nullptr);
bppo_status launch_minibatch(bppo_ctx *c, uint32_t start, uint32_t n, float ent_coef, bool exact);
bppo_status launch_adam(bppo_ctx *c, float lr, const float *c1, const float *c2, float *metric_dst = nullptr,
                        int nm = 0);
bppo_status launch_metric_row(bppo_ctx *c, float *dst, int nm);
bppo_status launch_pack_rows(bppo_ctx *c);
bppo_status launch_explained_variance(bppo_ctx *c, const float *valid);
void explained_variance_sums(bppo_ctx *c, double *out4);   // after the stream wait
// (wide_api.hip) multi-player path
bppo_status wide_init(bppo_ctx *c);
void wide_free(bppo_ctx *c);
bppo_status wide_reset(bppo_ctx *c);
bppo_status wide_pack(bppo_ctx *c);
bppo_status wide_forward(bppo_ctx *c, int rows, const float *xc, int ldxc, float *logits, float *values,
                         int split = 0);   // split: the update GEMMs on k_gemm_split (wide_minibatch)
bppo_status wide_forward_actor(bppo_ctx *c, int rows, const float *xc, int ldxc, const float *params, float *logits);
// CNN trunk (cnn.hip): conv stack + flatten of `rows` obs rows -> d_cnn_f; backward
// of the conv stack from dF (dL/d features, [rows][fdim]) into the gradient
bppo_status cnn_alloc(bppo_ctx *c);
void cnn_free(bppo_ctx *c);
bppo_status cnn_pack(bppo_ctx *c, const float *params, float *wt, float *wd);
bppo_status cnn_features(bppo_ctx *c, int s, int rows, const float *x, int ldx, const float *params, const float *wt);
bppo_status cnn_backward(bppo_ctx *c, int s, int rows, const float *x, int ldx, float *dF, float *grad, int exact);
// how the wide path sums its weight gradients (gemm_wgrad's `exact`) where it does not run the
// split-bf16 contraction: 0 f32 split-K MFMA chains (mode 2); 1 f64 products and sums on the
// f64 MFMA (k_gemm_wg64), the default (mode 0): f32 chains over a minibatch's rows leave the
// parameters ~1 ulp off the oracle's after each Adam step, which the PPO loss amplifies (a
// 64-channel conv layer's B*42 positions from minibatch 12 on, r04; the Liar's Dice MLP's
// 1024-row minibatches at minibatch 26 of 32, profiles/r05c/wide_scale_probe.json), f64 sums
// round to the oracle's f32 but for rare ties; 2 the oracle's row-ordered f64 sums (k_wg_seq,
// bppo_set_minibatch_kernel 1: the reference-exact parity mode)
inline int wide_exact_grad(const bppo_ctx *c) {
    if (c->mb_kernel == 1) return 2;
    return c->mb_kernel == 0 ? 1 : 0;
}
// opponent pool (opponents.hip)
bool opp_active(const bppo_ctx *c);
bppo_status opp_alloc(bppo_ctx *c);
void opp_free(bppo_ctx *c);
bppo_status opp_rollout_begin(bppo_ctx *c, uint64_t base);
bppo_status opp_step_group(bppo_ctx *c, int t);
bppo_status opp_step_forwards(bppo_ctx *c);
bppo_status opp_step_seats(bppo_ctx *c, int t);
bppo_status opp_rollout_end(bppo_ctx *c);
bppo_status opp_compact_valid(bppo_ctx *c);
bppo_status opp_map_perm(bppo_ctx *c, uint32_t n);
bppo_status wide_collect(bppo_ctx *c, uint64_t base);
bppo_status wide_bootstrap_gae(bppo_ctx *c);
bppo_status wide_minibatch(bppo_ctx *c, uint32_t start, uint32_t n, double ent_coef, bool first);
bppo_status wide_observe_host(bppo_ctx *c, float *obs, int32_t *players, uint8_t *masks, float *priv);
bppo_status wide_step_host(bppo_ctx *c, const int32_t *actions, float *obs, float *rewards, uint8_t *dones,
                           int32_t *n_eps);
bppo_status wide_forward_host(bppo_ctx *c, const float *obs, const float *priv, int B, float *logits,
                              float *values);
bppo_status wide_buffer_get(bppo_ctx *c, const char *name, void *host, size_t bytes, bool *handled);
// PopArt (popart.hip)
double popart_std(const bppo_ctx *c);

// Schedule::get (schedule.rs:54-78): piecewise-linear over (value, step) milestones,
// first value before the first milestone, last value after the last, 0 when empty
inline double schedule_get(const std::vector<double> &v, const std::vector<uint64_t> &s, uint64_t step) {
    const size_t n = v.size();
    if (n == 0) return 0.0;
    if (n == 1 || step <= s[0]) return v[0];
    for (size_t i = 0; i + 1 < n; i++)
        if (step >= s[i] && step < s[i + 1]) {
            const double t = (double)(step - s[i]) / (double)(s[i + 1] - s[i]);
            return v[i] + (v[i + 1] - v[i]) * t;
        }
    return v[n - 1];
}
// the shaping bonus the envs add this step: reward_shaping_coef.get(current_step) as f32
inline float shaping_coef(const bppo_ctx *c) { return (float)schedule_get(c->shaping_v, c->shaping_s, c->env_step); }
bppo_status popart_alloc(bppo_ctx *c);
void popart_free(bppo_ctx *c);
bppo_status popart_denorm(bppo_ctx *c, float *v, size_t n);
bppo_status popart_update_begin(bppo_ctx *c, const float *valid);
bppo_status popart_target_stats(bppo_ctx *c, int full_epochs, size_t rows_done, const float *valid);
// libm device check
bppo_status launch_libm(int which, const float *d_x, float *d_y, size_t n);

inline bppo_status hip_fail(bppo_ctx *c, hipError_t e, const char *what) {
    if (c) c->err = std::string(what) + ": " + hipGetErrorString(e);
    return BPPO_ERR_HIP;
}
// A kernel launch's status is read with hipGetLastError, which returns the last error
// of ANY earlier HIP call on this thread that nobody cleared.  So every call whose
// status is handled where it is made clears the slot there (event_query / event_ms
// below: "not ready" is an answer, not a failure), every other call on the enqueue
// path is checked, and each launch helper names its kernel in the message.
// (r04: a pipelined run reported "gae launch failed" for an earlier call's status;
// DESIGN.md section 5b names it.)
inline bppo_status launch_check(bppo_ctx *c, const char *kernel) {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? BPPO_OK : hip_fail(c, e, kernel);
}
inline hipError_t event_query(hipEvent_t ev) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipSuccess) (void)hipGetLastError();
    return e;
}
inline bool event_ms(hipEvent_t a, hipEvent_t b, float *ms) {
    const hipError_t e = hipEventElapsedTime(ms, a, b);
    if (e != hipSuccess) (void)hipGetLastError();
    return e == hipSuccess;
}
}  // namespace bppo

#define TRY(x)                                 \
    do {                                       \
        bppo_status _s = (x);                  \
        if (_s != BPPO_OK) return _s;          \
    } while (0)

#define BPPO_HIP(c, expr)                                                   \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) return bppo::hip_fail((c), _e, #expr);        \
    } while (0)

// bppo_api.hip — the C-ABI (include/bppo.h): context lifecycle, the
// host-side orchestration of one update (collect_rollouts -> bootstrap + GAE ->
// ppo_update, main.rs:724-963), the rand-0.8 shuffle chain thread, parity hooks.
#include <algorithm>
#include <pthread.h>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <sys/prctl.h>
#include <x86intrin.h>
#include "bppo_internal.h"
#include "shuffle_host.h"
#include "bppo_wide.h"

using namespace bppo;

namespace bppo {
// TSC ticks per millisecond, measured once against steady_clock (shuffle engine
// diagnostics)
static double tsc_per_ms() {
    static double v = 0.0;
    if (v == 0.0) {
        const auto t0 = std::chrono::steady_clock::now();
        const uint64_t c0 = __rdtsc();
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
        const uint64_t c1 = __rdtsc();
        v = (double)(c1 - c0) / std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    return v;
}


NetLayout make_layout(const bppo_config &c, int obs_dim, int priv_dim, int act_dim) {
    NetLayout L;
    // split_networks (mlp.rs:100-130): a second trunk of num_hidden x hidden_size on obs,
    // i.e. the CTDE structure with no privileged input (ctde.rs ignores the flag)
    const bool split = c.split_networks && !c.ctde;
    L.ctde = c.ctde || split; L.relu = c.relu;
    auto add = [&](int in, int out) {
        int i = L.n_layers++;
        L.in[i] = in; L.out[i] = out;
        return i;
    };
    int in = obs_dim;
    if (c.cnn) {
        // cnn.rs:66-150: conv stack on the (H, W, C) spatial part, FC layers on
        // [flattened conv output | extra features], heads of cnn_fc_hidden_size
        L.H = 6; L.W = 7; L.C = 2;                     // connect_four.rs:217 OBSERVATION_SHAPE
        L.E = obs_dim - L.H * L.W * L.C;
        L.ksize = c.kernel_size;
        int cin = L.C;
        for (int l = 0; l < c.num_conv_layers; l++) {
            const int co = c.conv_channels[l < 4 ? l : 3];
            L.conv_cin[l] = cin;
            add(cin * L.ksize * L.ksize, co);
            cin = co;
        }
        L.n_conv = c.num_conv_layers;
        L.fdim = L.H * L.W * cin + L.E;
        in = L.fdim;
        for (int l = 0; l < c.cnn_num_fc_layers; l++) { add(in, c.cnn_fc_hidden_size); in = c.cnn_fc_hidden_size; }
        L.n_actor_hidden = L.n_conv + c.cnn_num_fc_layers;
    } else {
        for (int l = 0; l < c.num_hidden; l++) { add(in, c.hidden_size); in = c.hidden_size; }
        L.n_actor_hidden = c.num_hidden;
    }
    L.policy = add(in, act_dim);
    if (L.ctde && c.cnn) {
        // split CNN (cnn.rs:116-135): the critic's own conv stack (same shapes) and FC layers
        L.critic_first = L.n_layers;
        for (int l = 0; l < L.n_conv; l++) add(L.in[l], L.out[l]);
        L.critic_fc0 = L.n_layers;
        int cin = L.fdim;
        for (int l = 0; l < c.cnn_num_fc_layers; l++) { add(cin, c.cnn_fc_hidden_size); cin = c.cnn_fc_hidden_size; }
        L.value = add(cin, 1);
    } else if (L.ctde) {
        int cin = split ? obs_dim : priv_dim + obs_dim;
        const int nc = split ? c.num_hidden : c.critic_num_hidden, wc = split ? c.hidden_size : c.critic_hidden_size;
        L.critic_first = L.critic_fc0 = L.n_layers;
        for (int l = 0; l < nc; l++) { add(cin, wc); cin = wc; }
        L.value = add(cin, 1);
    } else {
        L.value = add(in, 1);
    }
    // offsets in Burn record order: the layer order above, except split_networks'
    // record (mlp.rs:47-62) puts the critic layers before the policy head
    int order[16], no = 0;
    for (int l = 0; l < L.n_layers; l++)
        if (!split || l < L.n_actor_hidden || (l >= L.critic_first && l < L.value)) order[no++] = l;
    if (split) { order[no++] = L.policy; order[no++] = L.value; }
    size_t off = 0;
    for (int r = 0; r < L.n_layers; r++) {
        const int l = order[r];
        L.rec[l] = r;
        L.w[l] = off; off += (size_t)L.in[l] * L.out[l];
        L.b[l] = off; off += L.out[l];
    }
    L.n_params = off;
    return L;
}

// ----------------------------------------------------------- libm check ----
__global__ void k_libm(int which, const float *x, float *y, size_t n) {
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float v = x[i];
    switch (which) {
    case 0: y[i] = bppo_math::logf_glibc(v); break;
    case 1: y[i] = bppo_math::sinf_glibc(v); break;
    case 2: y[i] = bppo_math::cosf_glibc(v); break;
    case 3: y[i] = -bppo_math::logf_glibc(-bppo_math::logf_glibc(v)); break;
    case 5: y[i] = bppo_math::tanhf_glibc_bf(v); break;   // the form the MLP kernels use
    default: y[i] = bppo_math::expf_glibc(v); break;
    }
}

bppo_status launch_libm(int which, const float *d_x, float *d_y, size_t n) {
    hipLaunchKernelGGL(k_libm, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, which, d_x, d_y, n);
    return hipGetLastError() == hipSuccess ? BPPO_OK : BPPO_ERR_HIP;
}

}  // namespace bppo

// ======================================================================= ABI
static float powi_f32(float a, int b) {   // compiler-rt __powisf2 (Rust f32::powi)
    int recip = b < 0;
    float r = 1.0f;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0f / r : r;
}

template <class T>
static bppo_status dalloc(bppo_ctx *c, T **p, size_t n) {
    *p = nullptr;
    if (n == 0) return BPPO_OK;
    BPPO_HIP(c, hipMalloc((void **)p, n * sizeof(T)));
    BPPO_HIP(c, hipMemsetAsync(*p, 0, n * sizeof(T), c->stream));
    return BPPO_OK;
}

extern "C" size_t bppo_config_size(void) { return sizeof(bppo_config); }
extern "C" size_t bppo_update_metrics_size(void) { return sizeof(bppo_update_metrics); }
extern "C" size_t bppo_episode_size(void) { return sizeof(bppo_episode); }
extern "C" size_t bppo_rollout_info_size(void) { return sizeof(bppo_rollout_info); }

extern "C" const char *bppo_version(void) { return "bppo-mi355x 0.1 (gfx950)"; }

extern "C" const char *bppo_last_error(const bppo_ctx *c) { return c ? c->err.c_str() : "null ctx"; }

// wait for the context stream on a blocking-sync event: the host thread sleeps
// instead of polling (polling eats the CPU quota the shuffle walkers run on)
// (hipEventSynchronize on a blocking-sync event still spun here: measured ~1 CPU per
// process for the whole update; a sleeping poll at 20 us with 1 us timer slack frees it)
// The per-update wait of bppo_train_steps (~12 ms on CfgB) repeats from one update to
// the next, so it starts with ONE coarse sleep of 70 % of the recent waits and only
// then polls at 20 us: every poll is a wake-up plus an event query, and polling the
// whole wait cost the driving thread ~1 CPU per rank (14 ms of CPU per 13.9 ms update
// in r03h), CPU the shuffle walkers of an 8-rank node need.
static hipError_t wait_event(bppo_ctx *c, hipEvent_t ev) {   // sleeping poll (see sync_stream)
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e = event_query(ev);
    if (e == hipErrorNotReady) {
        if (c->wait_est_us > 200.0)
            std::this_thread::sleep_for(std::chrono::microseconds((long)(0.7 * c->wait_est_us)));
        while ((e = event_query(ev)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    c->wait_est_us = c->wait_est_us > 0.0 ? 0.5 * c->wait_est_us + 500.0 * ms : 1000.0 * ms;
    c->sync_wait_ms += ms;
    return e;
}

static hipError_t sync_stream(bppo_ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    if (!c->ev_block) e = hipStreamSynchronize(c->stream);
    else {
        static thread_local bool slack = false;
        if (!slack) { (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0); slack = true; }
        e = hipEventRecord(c->ev_block, c->stream);
        while (e == hipSuccess && (e = event_query(c->ev_block)) == hipErrorNotReady) {
            std::this_thread::sleep_for(std::chrono::microseconds(20));
            e = hipSuccess;
        }
    }
    c->sync_wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return e;
}

static bool cartpole_fused_net(const bppo_config &c) {
    return !c.split_networks && !c.cnn && !c.ctde && (c.hidden_size == 16 || c.hidden_size == 32 || c.hidden_size == 64) &&
           (c.num_hidden == 1 || c.num_hidden == 2);
}

static bppo_status ctx_init(bppo_ctx *c, const bppo_config *cfg, int dev, void *stream) {
    c->cfg = *cfg;
    c->dev = dev;
    // the configuration is validated before the first HIP call
    if (cfg->num_envs <= 0 || cfg->num_steps <= 0 || cfg->num_epochs <= 0 || cfg->num_minibatches <= 0) {
        c->err = "num_envs, num_steps, num_epochs, num_minibatches must be positive";
        return BPPO_ERR_ARG;
    }
    c->N = cfg->num_envs; c->T = cfg->num_steps;
    switch (cfg->env_kind) {
    case BPPO_ENV_CARTPOLE: c->D = 5; c->A = 2; c->P = 1; c->G = 0; break;
    case BPPO_ENV_CONNECT_FOUR: c->D = 86; c->A = 7; c->P = 2; c->G = 0; break;
    case BPPO_ENV_LIARS_DICE: c->D = 270; c->A = 49; c->P = 4; c->G = cfg->ctde ? 120 : 0; break;
    case BPPO_ENV_SKULL: c->D = 135; c->A = 33; c->P = 6; c->G = cfg->ctde ? 200 : 0; break;   // skull.rs:1046-1060
    default: c->err = "unknown env_kind"; return BPPO_ERR_ARG;
    }
    c->Pa = c->P;
    if (cfg->env_kind == BPPO_ENV_SKULL) {
        c->Pa = cfg->player_count ? cfg->player_count : 4;          // PlayerCountMode::default (config.rs:667-671)
        if (c->Pa < 2 || c->Pa > 6) { c->err = "Skull supports 2-6 players"; return BPPO_ERR_ARG; }   // skull.rs:159-162
    }
    // the fused CartPole kernels (k_rollout.hip, k_update.hip) cover the shared-trunk
    // MLPs of {16, 32, 64} x {1, 2}; every other CartPole net (mlp.rs:76-132 accepts any
    // width and depth; split_networks) runs on the GEMM engine path like the other envs
    c->wide = cfg->env_kind != BPPO_ENV_CARTPOLE || !cartpole_fused_net(*cfg);
    if (c->wide && !cfg->ctde) c->G = 0;
    // num_hidden = 0 would feed obs into heads of hidden_size inputs (mlp.rs:121-125), a
    // shape panic in the reference unless obs_dim == hidden_size
    if (!cfg->cnn && (cfg->hidden_size < 1 || cfg->num_hidden < 1 ||
                      (cfg->ctde && (cfg->critic_hidden_size < 1 || cfg->critic_num_hidden < 1)))) {
        c->err = "hidden_size / num_hidden (critic_*) must be positive";
        return BPPO_ERR_ARG;
    }
    if (!(cfg->reward_shaping_coef >= 0.0)) { c->err = "reward_shaping_coef must be >= 0"; return BPPO_ERR_ARG; }   // config.rs:1514-1519
    if (cfg->cnn) {
        // cnn.rs:73-74 "CNN requires OBSERVATION_SHAPE" (only Connect Four has one)
        if (cfg->env_kind != BPPO_ENV_CONNECT_FOUR || cfg->ctde) { c->err = "CNN requires OBSERVATION_SHAPE (Connect Four)"; return BPPO_ERR_ARG; }
        if (cfg->num_conv_layers < 1 || cfg->num_conv_layers > 4 || cfg->kernel_size < 1 || cfg->kernel_size > 7 ||
            !(cfg->kernel_size & 1) || cfg->cnn_num_fc_layers < 1 || cfg->cnn_fc_hidden_size < 1) {
            c->err = "CNN: 1-4 conv layers, odd kernel_size <= 7 (same padding), >= 1 FC layer";
            return BPPO_ERR_UNSUPPORTED;
        }
        for (int l = 0; l < cfg->num_conv_layers; l++)
            if (cfg->conv_channels[l < 4 ? l : 3] < 1) { c->err = "conv_channels must be positive"; return BPPO_ERR_ARG; }
    }
    // NetLayout holds at most 16 layers (its per-layer tables, Adam's 32 tensors):
    // MLP (split_networks doubles the trunk), CTDE actor + critic, CNN conv + FC stacks
    {
        const int split = cfg->split_networks && !cfg->ctde ? 2 : 1;
        const int layers = cfg->cnn ? split * (cfg->num_conv_layers + cfg->cnn_num_fc_layers) + 2
                         : cfg->ctde ? cfg->num_hidden + cfg->critic_num_hidden + 2
                                     : split * cfg->num_hidden + 2;
        if (layers > NetLayout::MAX_LAYERS) {
            c->err = "network: at most 16 layers in all (hidden / conv / FC layers + heads)";
            return BPPO_ERR_UNSUPPORTED;
        }
    }
    BPPO_HIP(c, hipSetDevice(dev));
    if (stream) { c->stream = (hipStream_t)stream; c->own_stream = false; }
    else {
        // the hot path's stream at the highest priority: the shuffle engine's copy-stream
        // kernels (J expansion) only take CUs the update kernels leave free
        int lo = 0, hi = 0;
        BPPO_HIP(c, hipDeviceGetStreamPriorityRange(&lo, &hi));
        BPPO_HIP(c, hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi));
        c->own_stream = true;
    }
    c->net = make_layout(*cfg, c->D, c->G, c->A);
    const size_t np = c->net.n_params;
    const size_t TN = (size_t)c->T * c->N;
    c->adam_t.assign(2 * c->net.n_layers, 0);
    TRY(dalloc(c, &c->d_params, np));
    TRY(dalloc(c, &c->d_m1, np));
    TRY(dalloc(c, &c->d_m2, np));
    TRY(dalloc(c, &c->d_grad, np + 64));
    c->slab_rows = 256 * 8;   // one 8-wave (MFMA) or 4-wave block per CU, persistent over the minibatch
    c->relu_mfma = cfg->relu ? 1 : 0;
    if (!c->wide) TRY(dalloc(c, &c->d_slab, c->slab_rows * (np + 64)));
    TRY(dalloc(c, &c->d_cp, (size_t)4 * c->N));
    TRY(dalloc(c, &c->d_steps, (size_t)c->N));
    TRY(dalloc(c, &c->d_env_pos, (size_t)c->N));
    TRY(dalloc(c, &c->d_ep_ret, (size_t)c->N * c->P));
    TRY(dalloc(c, &c->d_ep_len, (size_t)c->N));
    if (!c->wide) TRY(dalloc(c, &c->d_obs, TN * c->D));
    TRY(dalloc(c, &c->d_rew, TN));
    TRY(dalloc(c, &c->d_rew_raw, TN));
    TRY(dalloc(c, &c->d_done, TN));
    TRY(dalloc(c, &c->d_val, TN));
    TRY(dalloc(c, &c->d_logp, TN));
    TRY(dalloc(c, &c->d_adv, TN));
    TRY(dalloc(c, &c->d_ret, TN));
    TRY(dalloc(c, &c->d_act, TN));
    if (!c->wide || cfg->normalize_returns) TRY(dalloc(c, &c->d_X, TN));
    if (!c->wide && cfg->hidden_size == 64 && cfg->num_hidden == 2 && cfg->relu)
    {
        TRY(dalloc(c, &c->d_gumbel, TN * 2));
        TRY(dalloc(c, &c->d_rpool, (size_t)RPOOL_K * c->N));
        TRY(dalloc(c, &c->d_rpos, (size_t)RPOOL_K * c->N));
    }
    TRY(dalloc(c, &c->d_on, (size_t)2 * c->D + 1));
    if (!c->wide) TRY(dalloc(c, &c->d_obs_part, (size_t)c->N * 2 * c->D));
    if (!c->wide) {   // VecEnv::step / get_observations scratch (freed by wide_free with the rest)
        TRY(dalloc(c, &c->d_act_in, (size_t)c->N));
        TRY(dalloc(c, &c->d_scr_r, (size_t)c->N));
        TRY(dalloc(c, &c->d_bxc, (size_t)c->N * c->D));
        BPPO_HIP(c, hipMalloc((void **)&c->d_scr_d, (size_t)c->N));
    }
    TRY(dalloc(c, &c->d_rn_returns, (size_t)c->N * c->P));
    TRY(dalloc(c, &c->d_rn_stats, 4));
    TRY(dalloc(c, &c->d_scan_agg, (TN + 4095) / 4096 + 1));
    TRY(dalloc(c, &c->d_last_v, (size_t)c->N));
    // room for every episode a rollout can complete (one per env-step): the episode
    // summary then sums all of them (a smaller cap kept whichever episodes claimed
    // slots first); CartPole's integer returns sum exactly in f64, so its mean does not
    // depend on the order the waves claimed their record slots
    c->eps_cap = (int)std::min<size_t>((size_t)c->T * c->N + 4096, (size_t)INT32_MAX / 2);
    TRY(dalloc(c, &c->d_eps, (size_t)c->eps_cap));
    TRY(dalloc(c, &c->d_ep_count, 1));
    TRY(dalloc(c, &c->d_ep_sum, ROLL_HOST_WORDS));   // [count, err] + the partial sums: one host slot's layout
    TRY(dalloc(c, &c->d_err, 1));
    TRY(dalloc(c, &c->d_perm_base, TN));
    c->d_perm = c->d_perm_base;
    TRY(dalloc(c, &c->d_perm_ep, TN * (size_t)cfg->num_epochs));
    TRY(dalloc(c, &c->d_inv_ep, TN * (size_t)cfg->num_epochs));
    TRY(dalloc(c, &c->d_advpart, (size_t)ADV_STREAM_BLOCKS * ADV_STREAM_MAXM * 4));
    {
        // BPPO_FY_ON_COPY=1 (A/B): the permutations on the shuffle engine's copy stream (one
        // side stream instead of two; set after the engine's init below)
        c->fy_shared = getenv("BPPO_FY_ON_COPY") && atoi(getenv("BPPO_FY_ON_COPY")) == 1;
        if (!c->fy_shared) BPPO_HIP(c, make_side_stream(dev, &c->fy_stream));
        for (int e = 0; e < cfg->num_epochs && e < SHUF_MAX_EPOCHS; e++)
            BPPO_HIP(c, hipEventCreateWithFlags(&c->fy_ev[e], hipEventDisableTiming));
        // the prep stream only when it is used (BPPO_PREP_SIDE=1): with this third low-priority
        // stream created (even idle) every device-bound run took 13.1-13.6 instead of
        // 10.9-11.2 ms per update, the phases outside the minibatch kernels 15-25 % slower;
        // GPU_MAX_HW_QUEUES=8 did not remove it (profiles/r06y/, r06z/)
        if (getenv("BPPO_PREP_SIDE") && atoi(getenv("BPPO_PREP_SIDE")) == 1) {
            BPPO_HIP(c, make_side_stream(dev, &c->prep_stream));
            BPPO_HIP(c, hipEventCreateWithFlags(&c->ev_prep, hipEventDisableTiming));
        }
        BPPO_HIP(c, hipEventCreateWithFlags(&c->ev_env, hipEventDisableTiming));
    }
    TRY(dalloc(c, &c->d_fy, 4 * TN));
    TRY(dalloc(c, &c->d_scan, TN / 8192 + 2));
    BPPO_HIP(c, fy_ranges_init(c->fyr, (uint32_t)TN));
    TRY(dalloc(c, &c->d_red, 4 * 1024 + 64));
    TRY(dalloc(c, &c->d_mb_stats, (size_t)4 * std::max(cfg->num_minibatches, 2)));
    c->d_mb_cur = c->d_mb_stats;
    TRY(dalloc(c, &c->d_rows, (size_t)cfg->num_epochs * cfg->num_minibatches * (WM_COUNT + 4)));
    BPPO_HIP(c, hipHostMalloc((void **)&c->h_rows,
                              sizeof(float) * (size_t)cfg->num_epochs * cfg->num_minibatches * (WM_COUNT + 4),
                              hipHostMallocDefault));
    if (!c->wide && cfg->hidden_size == 64 && cfg->num_hidden == 2 && cfg->relu && c->D == 5)
    {
        BPPO_HIP(c, hipMalloc((void **)&c->d_rowA, sizeof(float4) * 2 * TN));
        BPPO_HIP(c, hipMalloc((void **)&c->d_rowB, sizeof(float2) * TN));
    }
    BPPO_HIP(c, hipHostMalloc((void **)&c->h_red, sizeof(double) * (4 * 1024 + 64 + 2 * ROLL_HOST_WORDS),
                              hipHostMallocDefault));   // + two slots of the rollout's flags and episode partials
    BPPO_HIP(c, hipHostGetDevicePointer((void **)&c->hd_red, c->h_red, 0));
    BPPO_HIP(c, hipEventCreateWithFlags(&c->ev_upd, hipEventDisableTiming));
    BPPO_HIP(c, hipEventRecord(c->ev_upd, c->stream));      // recorded once, so every wait on it is defined
    BPPO_HIP(c, hipEventCreateWithFlags(&c->ev_block, hipEventDisableTiming | hipEventBlockingSync));
    for (int i = 0; i < TM_SLOTS; i++) {
        BPPO_HIP(c, hipEventCreate(&c->ev[i][0]));
        BPPO_HIP(c, hipEventCreate(&c->ev[i][1]));
    }
    for (int i = 0; i < bppo_ctx::MB_EV; i++) {
        BPPO_HIP(c, hipEventCreate(&c->mb_ev[i][0]));
        BPPO_HIP(c, hipEventCreate(&c->mb_ev[i][1]));
    }
    c->rng_key = seed_key(cfg->seed);
    c->rng_pos = 0;
    c->shuf.gate = c->ev_upd;     // before init: the engine thread starts in it
    TRY(c->shuf.init(dev, c->rng_key, cfg->rng_stream, (uint32_t)TN, cfg->num_epochs, TN * (uint64_t)c->A, c->err,
                     cfg->shuffle_windows != 0));
    if (c->fy_shared) c->fy_stream = c->shuf.copy;
    c->on_mean.assign(c->D, 0.0); c->on_m2.assign(c->D, 0.0); c->on_count = 0;
    c->u_ret = c->d_ret; c->u_val = c->d_val;
    c->shaping_v.assign(1, cfg->reward_shaping_coef); c->shaping_s.assign(1, 0);   // Schedule::constant
    if (cfg->normalize_values) TRY(popart_alloc(c));
    if (c->wide) {
        TRY(wide_init(c));
        TRY(wide_reset(c));
        TRY(wide_pack(c));
    } else {
        TRY(launch_cartpole_reset(c));
    }
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_create(const bppo_config *cfg, int hip_device, void *hip_stream,
                                   bppo_ctx **out) {
    if (!cfg || !out) return BPPO_ERR_ARG;
    bppo_ctx *c = new bppo_ctx();
    bppo_status s = ctx_init(c, cfg, hip_device, hip_stream);
    *out = c;   // returned even on failure so bppo_last_error can explain; caller destroys
    return s;
}

extern "C" void bppo_destroy(bppo_ctx *c) {
    if (!c) return;
    if (c->ev_thread.joinable()) c->ev_thread.join();
    if (c->ev_stream) { (void)hipStreamSynchronize(c->ev_stream); (void)hipStreamDestroy(c->ev_stream); }
    if (c->ev_gae) (void)hipEventDestroy(c->ev_gae);
    if (c->ev_copied) (void)hipEventDestroy(c->ev_copied);
    for (float *h : {c->h_ev_v, c->h_ev_r, c->h_ev_valid}) if (h) (void)hipHostFree(h);
    if (c->fy_stream) (void)hipStreamSynchronize(c->fy_stream);   // reads the engine's J buffers
    if (c->prep_stream) (void)hipStreamSynchronize(c->prep_stream);
    c->shuf.shutdown();
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    wide_free(c);
    popart_free(c);
    void *ptrs[] = {c->d_params, c->d_m1, c->d_m2, c->d_grad, c->d_slab, c->d_cp, c->d_steps,
                    c->d_env_pos, c->d_ep_ret, c->d_ep_len, c->d_obs, c->d_rew, c->d_rew_raw,
                    c->d_done, c->d_val, c->d_logp, c->d_adv, c->d_ret, c->d_act, c->d_X, c->d_on,
                    c->d_obs_part, c->d_rn_returns, c->d_rn_stats, c->d_scan_agg, c->d_last_v,
                    c->d_eps, c->d_ep_count, c->d_ep_sum, c->d_err, c->d_perm_base, c->d_perm_ep, c->d_inv_ep, c->d_advpart, c->d_fy, c->d_scan,
                    c->d_red, c->d_mb_stats, c->d_gumbel, c->d_rpool, c->d_rpos, c->d_rows, c->d_rowA, c->d_rowB};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    fy_ranges_free(c->fyr);
    if (c->h_red) (void)hipHostFree(c->h_red);
    if (c->h_rows) (void)hipHostFree(c->h_rows);
    if (c->ev_block) (void)hipEventDestroy(c->ev_block);
    if (c->ev_upd) (void)hipEventDestroy(c->ev_upd);
    for (int i = 0; i < TM_SLOTS; i++) {
        if (c->ev[i][0]) (void)hipEventDestroy(c->ev[i][0]);
        if (c->ev[i][1]) (void)hipEventDestroy(c->ev[i][1]);
    }
    for (auto &pr : c->mb_ev)
        for (hipEvent_t e : pr) if (e) (void)hipEventDestroy(e);
    if (c->fy_stream && !c->fy_shared) { (void)hipStreamSynchronize(c->fy_stream); (void)hipStreamDestroy(c->fy_stream); }
    for (hipEvent_t e : c->fy_ev) if (e) (void)hipEventDestroy(e);
    if (c->prep_stream) (void)hipStreamDestroy(c->prep_stream);
    for (hipEvent_t e : {c->ev_env, c->ev_prep}) if (e) (void)hipEventDestroy(e);
    if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" size_t bppo_num_params(const bppo_ctx *c) { return c ? c->net.n_params : 0; }

// a rollout bppo_train_steps enqueued ahead (and left pending by an error) was drawn
// with the state these setters replace: drop it (the envs and the RNG stay where it
// left them; the next bppo_collect_rollouts draws a new one)
static void drop_prefetch(bppo_ctx *c) {
    if (!c->prefetched) return;
    c->prefetched = false;
    c->collected = 0;
    c->gae_done = 0;
}

extern "C" bppo_status bppo_params_set(bppo_ctx *c, const float *h, size_t n) {
    if (!c || !h || n != c->net.n_params) { if (c) c->err = "params_set: size mismatch"; return BPPO_ERR_ARG; }
    drop_prefetch(c);
    BPPO_HIP(c, hipMemcpyAsync(c->d_params, h, n * 4, hipMemcpyHostToDevice, c->stream));
    if (c->wide) TRY(wide_pack(c));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_params_get(bppo_ctx *c, float *h, size_t n) {
    if (!c || !h || n != c->net.n_params) { if (c) c->err = "params_get: size mismatch"; return BPPO_ERR_ARG; }
    BPPO_HIP(c, hipMemcpyAsync(h, c->d_params, n * 4, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_forward(bppo_ctx *c, const float *obs, const float *priv, int32_t B,
                                    float *logits, float *values) {
    if (!c || !obs || B <= 0) return BPPO_ERR_ARG;
    if (c->wide) return wide_forward_host(c, obs, priv, B, logits, values);
    // scratch freed on every return path (an inference call, not the rollout path)
    struct Scratch { float *p[3] = {nullptr, nullptr, nullptr}; ~Scratch() { for (float *q : p) (void)hipFree(q); } } t;
    BPPO_HIP(c, hipMalloc((void **)&t.p[0], sizeof(float) * (size_t)B * c->D));
    BPPO_HIP(c, hipMalloc((void **)&t.p[1], sizeof(float) * (size_t)B * c->A));
    BPPO_HIP(c, hipMalloc((void **)&t.p[2], sizeof(float) * (size_t)B));
    float *d_o = t.p[0], *d_l = t.p[1], *d_v = t.p[2];
    BPPO_HIP(c, hipMemcpyAsync(d_o, obs, sizeof(float) * (size_t)B * c->D, hipMemcpyHostToDevice, c->stream));
    bppo_status s = launch_forward_rows(c, d_o, B, d_l, d_v);
    if (s == BPPO_OK) {
        if (logits) BPPO_HIP(c, hipMemcpyAsync(logits, d_l, sizeof(float) * (size_t)B * c->A, hipMemcpyDeviceToHost, c->stream));
        if (values) BPPO_HIP(c, hipMemcpyAsync(values, d_v, sizeof(float) * (size_t)B, hipMemcpyDeviceToHost, c->stream));
    }
    // drain before the scratch is freed, whatever happened above
    const bppo_status ss = sync_stream(c) == hipSuccess ? BPPO_OK : BPPO_ERR_HIP;
    return s != BPPO_OK ? s : ss;
}

extern "C" bppo_status bppo_rng_get(bppo_ctx *c, uint64_t *p) {
    if (!c || !p) return BPPO_ERR_ARG;
    *p = c->rng_pos;
    return BPPO_OK;
}
extern "C" bppo_status bppo_rng_set(bppo_ctx *c, uint64_t p) {
    if (!c) return BPPO_ERR_ARG;
    drop_prefetch(c);
    c->shuf_slot = -1;
    c->fy_slot = -1; c->fy_done = 0;     // permutations made ahead belong to the old start
    c->rng_pos = p;
    return BPPO_OK;
}

// checkpoint.rs:390-400 save_rng_state: rng.fill_bytes(&mut [u8; 32]) — rand_core
// 0.6 BlockRng::fill_bytes takes ceil(n / 4) whole words, little-endian
extern "C" bppo_status bppo_rng_fill_bytes(bppo_ctx *c, uint8_t *dst, size_t n) {
    if (!c || (!dst && n)) return BPPO_ERR_ARG;
    const size_t nw = (n + 3) / 4;
    uint32_t blk[16];
    uint64_t cached = ~0ull;
    for (size_t i = 0; i < nw; i++) {
        const uint64_t pos = c->rng_pos + i;
        if ((pos >> 4) != cached) { chacha12_block(c->rng_key, pos >> 4, c->cfg.rng_stream, blk); cached = pos >> 4; }
        const uint32_t w = blk[pos & 15];
        for (int b = 0; b < 4 && 4 * i + b < n; b++) dst[4 * i + b] = (uint8_t)(w >> (8 * b));
    }
    c->rng_pos += nw;
    c->shuf_slot = -1;
    c->fy_slot = -1; c->fy_done = 0;
    return BPPO_OK;
}

// checkpoint.rs:405-426 load_rng_state: StdRng::from_seed(seed) — the 32 seed bytes
// are the ChaCha12 key (8 little-endian words), block counter 0.  The shuffle
// engine precomputes words of the old key, so it is restarted on the new one.
extern "C" bppo_status bppo_rng_from_seed(bppo_ctx *c, const uint8_t *seed) {
    if (!c || !seed) return BPPO_ERR_ARG;
    drop_prefetch(c);
    Key8 k;
    for (int i = 0; i < 8; i++)
        k.k[i] = (uint32_t)seed[4 * i] | ((uint32_t)seed[4 * i + 1] << 8) | ((uint32_t)seed[4 * i + 2] << 16) |
                 ((uint32_t)seed[4 * i + 3] << 24);
    BPPO_HIP(c, sync_stream(c));
    BPPO_HIP(c, hipStreamSynchronize(c->fy_stream));   // its permutations read the engine's J
    c->fy_slot = -1; c->fy_done = 0;
    c->shuf.shutdown();
    c->shuf.~ShuffleEngine();
    new (&c->shuf) ShuffleEngine();
    c->rng_key = k;
    c->rng_pos = 0;
    c->shuf_slot = -1;
    const size_t TN = (size_t)c->T * c->N;
    c->shuf.gate = c->ev_upd;
    TRY(c->shuf.init(c->dev, c->rng_key, c->cfg.rng_stream, (uint32_t)TN, c->cfg.num_epochs, TN * (uint64_t)c->A, c->err,
                     c->cfg.shuffle_windows != 0));
    if (c->fy_shared) c->fy_stream = c->shuf.copy;
    return BPPO_OK;
}

extern "C" bppo_status bppo_rng_key_get(bppo_ctx *c, uint32_t *key) {
    if (!c || !key) return BPPO_ERR_ARG;
    for (int i = 0; i < 8; i++) key[i] = c->rng_key.k[i];
    return BPPO_OK;
}

// Adam state (burn-optim AdamState: moment_1, moment_2, time per parameter tensor):
// m1/m2 flat like the parameters, steps [2 * layers] in record order (W, b per Linear)
extern "C" bppo_status bppo_optimizer_get(bppo_ctx *c, float *m1, float *m2, int32_t *steps, size_t n) {
    if (!c || n != c->net.n_params) { if (c) c->err = "optimizer_get: size mismatch"; return BPPO_ERR_ARG; }
    if (m1) BPPO_HIP(c, hipMemcpyAsync(m1, c->d_m1, n * 4, hipMemcpyDeviceToHost, c->stream));
    if (m2) BPPO_HIP(c, hipMemcpyAsync(m2, c->d_m2, n * 4, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    // adam_t is indexed by layer (2 l, 2 l + 1); steps[] is in record order
    if (steps)
        for (int l = 0; l < c->net.n_layers; l++)
            for (int k = 0; k < 2; k++) steps[2 * c->net.rec[l] + k] = c->adam_t[2 * l + k];
    return BPPO_OK;
}

extern "C" bppo_status bppo_optimizer_set(bppo_ctx *c, const float *m1, const float *m2, const int32_t *steps,
                                          size_t n) {
    // (a rollout enqueued ahead does not read the Adam moments: it stays valid)
    if (!c || !m1 || !m2 || !steps || n != c->net.n_params) {
        if (c) c->err = "optimizer_set: size mismatch";
        return BPPO_ERR_ARG;
    }
    BPPO_HIP(c, hipMemcpyAsync(c->d_m1, m1, n * 4, hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, hipMemcpyAsync(c->d_m2, m2, n * 4, hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, sync_stream(c));
    for (int l = 0; l < c->net.n_layers; l++)
        for (int k = 0; k < 2; k++) c->adam_t[2 * l + k] = steps[2 * c->net.rec[l] + k];
    return BPPO_OK;
}

extern "C" size_t bppo_num_param_tensors(const bppo_ctx *c) { return c ? c->adam_t.size() : 0; }

extern "C" bppo_status bppo_vecenv_reset(bppo_ctx *c) {
    if (!c) return BPPO_ERR_ARG;
    drop_prefetch(c);
    TRY(c->wide ? wide_reset(c) : launch_cartpole_reset(c));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_vecenv_observe(bppo_ctx *c, float *obs, int32_t *players, uint8_t *masks,
                                           float *priv) {
    (void)priv; (void)masks;
    if (!c) return BPPO_ERR_ARG;
    if (c->wide) return wide_observe_host(c, obs, players, masks, priv);
    if (obs) {
        TRY(launch_cartpole_observe(c, c->d_bxc));
        BPPO_HIP(c, hipMemcpyAsync(obs, c->d_bxc, sizeof(float) * (size_t)c->N * c->D, hipMemcpyDeviceToHost, c->stream));
        BPPO_HIP(c, sync_stream(c));
    }
    if (players) std::fill(players, players + c->N, 0);
    return BPPO_OK;
}

extern "C" bppo_status bppo_vecenv_step(bppo_ctx *c, const int32_t *actions, float *obs, float *rewards,
                                        uint8_t *dones, bppo_episode *eps, int32_t cap, int32_t *n_eps) {
    if (!c || !actions) return BPPO_ERR_ARG;
    const int N = c->N;
    if (c->wide) {
        BPPO_HIP(c, hipMemsetAsync(c->d_ep_count, 0, 4, c->stream));
        int32_t cnt = 0;
        TRY(wide_step_host(c, actions, obs, rewards, dones, &cnt));
        if (n_eps) *n_eps = cnt;
        if (eps && cap > 0 && cnt > 0) {
            std::vector<EpisodeRec> recs(std::min(cnt, c->eps_cap));
            BPPO_HIP(c, hipMemcpy(recs.data(), c->d_eps, sizeof(EpisodeRec) * recs.size(), hipMemcpyDeviceToHost));
            std::sort(recs.begin(), recs.end(), [](const EpisodeRec &a, const EpisodeRec &b) {
                return a.env_index < b.env_index; });
            for (int i = 0; i < (int)recs.size() && i < cap; i++) {
                std::memcpy(eps[i].total_reward, recs[i].total_reward, sizeof(float) * BPPO_MAX_PLAYERS);
                eps[i].length = recs[i].length; eps[i].env_index = recs[i].env_index;
                eps[i].step = recs[i].step; eps[i].pad = 0;
            }
        }
        return BPPO_OK;
    }
    // persistent scratch (ctx_init): no allocator round-trip per step
    int32_t *d_a = c->d_act_in; float *d_r = c->d_scr_r, *d_o = c->d_bxc; uint8_t *d_d = c->d_scr_d;
    BPPO_HIP(c, hipMemcpyAsync(d_a, actions, sizeof(int32_t) * N, hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, hipMemsetAsync(c->d_ep_count, 0, 4, c->stream));
    TRY(launch_cartpole_vecenv_step(c, d_a, d_r, d_d, d_o));
    if (rewards) BPPO_HIP(c, hipMemcpyAsync(rewards, d_r, sizeof(float) * N, hipMemcpyDeviceToHost, c->stream));
    if (dones) BPPO_HIP(c, hipMemcpyAsync(dones, d_d, N, hipMemcpyDeviceToHost, c->stream));
    if (obs) BPPO_HIP(c, hipMemcpyAsync(obs, d_o, sizeof(float) * (size_t)N * c->D, hipMemcpyDeviceToHost, c->stream));
    int32_t cnt = 0;
    BPPO_HIP(c, hipMemcpyAsync(&cnt, c->d_ep_count, 4, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    if (n_eps) *n_eps = cnt;
    if (eps && cap > 0 && cnt > 0) {
        std::vector<EpisodeRec> recs(std::min(cnt, c->eps_cap));
        BPPO_HIP(c, hipMemcpy(recs.data(), c->d_eps, sizeof(EpisodeRec) * recs.size(), hipMemcpyDeviceToHost));
        std::sort(recs.begin(), recs.end(), [](const EpisodeRec &a, const EpisodeRec &b) {
            return a.env_index < b.env_index; });
        for (int i = 0; i < (int)recs.size() && i < cap; i++) {
            std::memcpy(eps[i].total_reward, recs[i].total_reward, sizeof(float) * BPPO_MAX_PLAYERS);
            eps[i].length = recs[i].length; eps[i].env_index = recs[i].env_index;
            eps[i].step = recs[i].step; eps[i].pad = 0;
        }
    }
    return BPPO_OK;
}

// Environment::set_step (env.rs:329-333): the step every schedulable env parameter
// (Liar's Dice reward shaping, liars_dice.rs:535, 635) is evaluated at
extern "C" bppo_status bppo_vecenv_set_step(bppo_ctx *c, uint64_t s) {
    if (!c) return BPPO_ERR_ARG;
    c->env_step = s;
    return BPPO_OK;
}

// reward_shaping_coef as a Schedule (config.rs:761-762; schedule.rs:29): milestones
// (values[i], steps[i]) in the caller's order (the reference sorts at parse time,
// schedule.rs:144, 268).  n = 0 is the empty schedule (get = 0.0).  Initial value
// must be >= 0 (config.rs:1514-1519).
extern "C" bppo_status bppo_set_reward_shaping_schedule(bppo_ctx *c, const double *values, const uint64_t *steps,
                                                        int32_t n) {
    if (!c || n < 0 || (n > 0 && (!values || !steps))) return BPPO_ERR_ARG;
    std::vector<double> v(values, values + n);
    std::vector<uint64_t> s(steps, steps + n);
    if (bppo::schedule_get(v, s, 0) < 0.0) { c->err = "reward_shaping_coef must be >= 0"; return BPPO_ERR_ARG; }
    c->shaping_v = std::move(v); c->shaping_s = std::move(s);
    return BPPO_OK;
}

extern "C" bppo_status bppo_obs_norm_get(bppo_ctx *c, double *mean, double *m2, double *count) {
    if (!c) return BPPO_ERR_ARG;
    std::vector<double> h(2 * c->D + 1);
    BPPO_HIP(c, hipMemcpyAsync(h.data(), c->d_on, sizeof(double) * h.size(), hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    if (mean) std::memcpy(mean, h.data(), sizeof(double) * c->D);
    if (m2) std::memcpy(m2, h.data() + c->D, sizeof(double) * c->D);
    if (count) *count = h[2 * c->D];
    return BPPO_OK;
}

extern "C" bppo_status bppo_obs_norm_set(bppo_ctx *c, const double *mean, const double *m2, double count) {
    if (!c || !mean || !m2) return BPPO_ERR_ARG;
    drop_prefetch(c);
    std::vector<double> h(2 * c->D + 1);
    std::memcpy(h.data(), mean, sizeof(double) * c->D);
    std::memcpy(h.data() + c->D, m2, sizeof(double) * c->D);
    h[2 * c->D] = count;
    BPPO_HIP(c, hipMemcpyAsync(c->d_on, h.data(), sizeof(double) * h.size(), hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_ret_norm_get(bppo_ctx *c, double *mvc, double *returns) {
    if (!c) return BPPO_ERR_ARG;
    if (mvc) BPPO_HIP(c, hipMemcpyAsync(mvc, c->d_rn_stats, sizeof(double) * 3, hipMemcpyDeviceToHost, c->stream));
    if (returns) BPPO_HIP(c, hipMemcpyAsync(returns, c->d_rn_returns, sizeof(double) * (size_t)c->N * c->P, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_ret_norm_set(bppo_ctx *c, const double *mvc, const double *returns) {
    if (!c) return BPPO_ERR_ARG;
    drop_prefetch(c);
    if (mvc) BPPO_HIP(c, hipMemcpyAsync(c->d_rn_stats, mvc, sizeof(double) * 3, hipMemcpyHostToDevice, c->stream));
    if (returns) BPPO_HIP(c, hipMemcpyAsync(c->d_rn_returns, returns, sizeof(double) * (size_t)c->N * c->P, hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" bppo_status bppo_popart_get(bppo_ctx *c, double *st) {
    if (!c || !st) return BPPO_ERR_ARG;
    st[0] = c->pa_mean; st[1] = c->pa_m2; st[2] = c->pa_count; st[3] = c->pa_eps;
    return BPPO_OK;
}

extern "C" bppo_status bppo_popart_set(bppo_ctx *c, const double *st) {
    if (!c || !st) return BPPO_ERR_ARG;
    drop_prefetch(c);
    c->pa_mean = st[0]; c->pa_m2 = st[1]; c->pa_count = st[2]; c->pa_eps = st[3];
    return BPPO_OK;
}

static bppo_status tm_begin(bppo_ctx *c, int slot) {
    BPPO_HIP(c, hipEventRecord(c->ev[slot][0], c->stream));
    return BPPO_OK;
}
static bppo_status tm_end(bppo_ctx *c, int slot) {
    BPPO_HIP(c, hipEventRecord(c->ev[slot][1], c->stream));
    return BPPO_OK;
}
static void tm_read(bppo_ctx *c, int slot) {
    float ms = 0;
    if (event_ms(c->ev[slot][0], c->ev[slot][1], &ms)) c->last_ms[slot] = ms;
}

// Fisher-Yates of every epoch of the engine's job in `slot` whose J is already on
// the device (the host engine has resolved it), in epoch order on fy_stream,
// each into its own permutation buffer (ppo.rs:1816 indices.shuffle; the
// permutation of epoch e depends only on that epoch's RNG words)
static bppo_status fy_enqueue_ready(bppo_ctx *c, int slot) {
    const size_t B = (size_t)c->T * c->N;
    if (slot != c->fy_slot) {
        // a new update's permutations overwrite perm/inv, which the previous update's
        // minibatches may still be reading when its successor's rollout is enqueued
        // behind it (bppo_train_steps): wait for the end of that update
        c->fy_slot = slot; c->fy_done = 0;
        BPPO_HIP(c, hipStreamWaitEvent(c->fy_stream, c->ev_upd, 0));
    }
    if (c->shuf.failed(c->err)) return BPPO_ERR_HIP;
    while (c->fy_done < c->cfg.num_epochs && c->shuf.epoch_ready(slot, c->fy_done)) {
        const int e = c->fy_done;
        // the engine thread may have recorded a HIP failure (J upload, expansion, event) and
        // then marked this epoch ready: its J is not to be permuted
        if (c->shuf.failed(c->err)) return BPPO_ERR_HIP;
        BPPO_HIP(c, hipStreamWaitEvent(c->fy_stream, c->shuf.ev[slot][e], 0));
        if (e > 0) BPPO_HIP(c, hipStreamWaitEvent(c->fy_stream, c->fy_ev[e - 1], 0));   // shared scratch
        BPPO_HIP(c, hipEventRecord(c->ev[TM_SHUFFLE][0], c->fy_stream));
        BPPO_HIP(c, fisher_yates_device(c->shuf.d_J[slot] + (size_t)e * B, (uint32_t)B, c->d_fy, c->d_scan,
                                        c->d_perm_ep + (size_t)e * B, c->fy_stream, &c->fyr,
                                        c->d_inv_ep + (size_t)e * B));
        BPPO_HIP(c, hipEventRecord(c->ev[TM_SHUFFLE][1], c->fy_stream));
        BPPO_HIP(c, hipEventRecord(c->fy_ev[e], c->fy_stream));
        c->fy_done++;
    }
    return BPPO_OK;
}

// collect_rollouts (ppo.rs:213-500), enqueue half: everything up to the episode
// summary and the device flags' copies into pinned host words (no host wait)
// the rollout's device flags and episode partials land in one of two pinned slots, so
// a rollout enqueued behind an update (bppo_train_steps) does not overwrite the
// previous rollout's before they are read
static double *roll_host(bppo_ctx *c, int slot) { return c->h_red + 4 * 1024 + 64 + (size_t)slot * ROLL_HOST_WORDS; }

static bppo_status collect_enqueue(bppo_ctx *c, bool summary) {
    const size_t TN = (size_t)c->T * c->N;
    c->coll_slot ^= 1;
    const int tro = c->coll_slot ? TM_ROLLOUT_B : TM_ROLLOUT, trn = c->coll_slot ? TM_RETNORM_B : TM_RETNORM;
    // the episode counter and error flags start at 0: zeroed here for the wide envs, by the
    // CartPole launcher (in its Gumbel kernel where that runs on the update stream)
    if (c->wide) {
        BPPO_HIP(c, hipMemsetAsync(c->d_ep_count, 0, 4, c->stream));
        BPPO_HIP(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
    }
    const uint64_t base = c->rng_pos;
    TRY(tm_begin(c, tro));
    if (c->wide) TRY(wide_collect(c, base));
    else {
        TRY(launch_cartpole_rollout(c, base, nullptr, nullptr, c->cfg.normalize_obs));
        TRY(popart_denorm(c, c->d_val, TN));            // ppo.rs:355-359 (multi-player: in the sampler)
    }
    TRY(tm_end(c, tro));
    // self-play: the update's shuffles start right after this rollout's Gumbel words,
    // so the epochs the engine has resolved are permuted now, beside the rollout
    // (beside the rollout is where they cost least: it leaves VGPRs and LDS free on every
    // CU, while the minibatch kernels fill them -- profiles/r03j_mb_overlap.txt)
    if (!opp_active(c)) {
        c->shuf_slot = c->shuf.ensure(base + TN * (uint64_t)c->A);
        TRY(fy_enqueue_ready(c, c->shuf_slot));
    }
    if (opp_active(c)) {
        // opponent pool: seat reshuffles drew a data-dependent number of words
        TRY(opp_rollout_end(c));
    } else {
        c->rng_pos = base + TN * (uint64_t)c->A;   // one word per (env, action) per step
        // this update's shuffles start here; the engine usually began them already
        c->shuf_slot = c->shuf.ensure(c->rng_pos);
    }
    if (c->cfg.normalize_obs) TRY(launch_obs_norm_merge(c));       // ppo.rs:495-497
    TRY(tm_begin(c, trn));
    if (c->cfg.normalize_returns) TRY(launch_return_norm(c));      // ppo.rs:390-408
    else if (!c->wide) BPPO_HIP(c, hipMemcpyAsync(c->d_rew, c->d_rew_raw, TN * 4, hipMemcpyDeviceToDevice, c->stream));
    TRY(tm_end(c, trn));
    int32_t *hv = reinterpret_cast<int32_t *>(roll_host(c, c->coll_slot));     // pinned
    if (summary) {
        // the summary kernel writes the episode count, the error flags and its partial sums in
        // the host slot's layout: into d_ep_sum and ONE copy (r05: three), or with
        // BPPO_ZERO_COPY=1 straight into the pinned slot (A/B: slower, gaps after the kernels
        // that write host memory -- profiles/r06t/)
        if (zero_copy()) {
            TRY(launch_episode_summary(c, c->hd_red + (roll_host(c, c->coll_slot) - c->h_red)));
        } else {
            TRY(launch_episode_summary(c, c->d_ep_sum));
            BPPO_HIP(c, hipMemcpyAsync(hv, c->d_ep_sum, sizeof(double) * ROLL_HOST_WORDS, hipMemcpyDeviceToHost, c->stream));
        }
    } else {
        BPPO_HIP(c, hipMemcpyAsync(&hv[0], c->d_ep_count, 4, hipMemcpyDeviceToHost, c->stream));
        BPPO_HIP(c, hipMemcpyAsync(&hv[1], c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    }
    c->collected = 1; c->gae_done = 0;
    c->rollout_rng_pos[c->coll_slot] = c->rng_pos;   // RNG position after the rollout (info; the update moves it on)
    return BPPO_OK;
}

// finish half, after the stream has drained past collect_enqueue: device error
// flags -> status, episode summary -> info
static bppo_status collect_finish(bppo_ctx *c, bppo_rollout_info *info, int slot) {
    float ms = 0;
    const int tro = slot ? TM_ROLLOUT_B : TM_ROLLOUT, trn = slot ? TM_RETNORM_B : TM_RETNORM;
    if (event_ms(c->ev[tro][0], c->ev[tro][1], &ms)) c->last_ms[TM_ROLLOUT] = ms;
    if (event_ms(c->ev[trn][0], c->ev[trn][1], &ms)) c->last_ms[TM_RETNORM] = ms;
    const int32_t *hv = reinterpret_cast<const int32_t *>(roll_host(c, slot));
    const double *part = roll_host(c, slot) + 2;
    // device error bits: 1 non-finite log-prob, 2 empty action mask, 4 opponent seat
    // table names a model outside [0, n_models)
    if (hv[1] & 2) { c->err = "Empty action mask: an env has no valid action"; return BPPO_ERR_EMPTY_MASK; }
    if (hv[1] & 1) { c->err = "NaN/Inf in log probs — model producing corrupt logits"; return BPPO_ERR_NONFINITE; }
    if (hv[1] & 4) { c->err = "opponent pool: pos_to_opp names a model index outside [0, n_models)"; return BPPO_ERR_ARG; }
    if (hv[1] & 8) { c->err = "Invalid action: outside the env's action mask"; return BPPO_ERR_ARG; }   // skull.rs:1116-1128
    if (hv[1]) { c->err = "collect_rollouts: unknown device error flag"; return BPPO_ERR_HIP; }
    if (info) {
        info->episodes = hv[0];
        info->rng_word_pos = c->rollout_rng_pos[slot];
        info->mean_return = 0; info->mean_length = 0;
        const int n = std::min(hv[0], c->eps_cap);
        if (n > 0) {
            double sr = 0, sl = 0;
            for (int b = 0; b < EP_SUMMARY_BLOCKS; b++) { sr += part[2 * b]; sl += part[2 * b + 1]; }
            info->mean_return = (float)(sr / n); info->mean_length = (float)(sl / n);
        }
    }
    return BPPO_OK;
}

extern "C" bppo_status bppo_collect_rollouts(bppo_ctx *c, bppo_rollout_info *info) {
    if (!c) return BPPO_ERR_ARG;
    // a rollout bppo_train_steps enqueued ahead (it returned an error before using it)
    // IS the next rollout: the RNG and the envs have moved past it already
    if (c->prefetched) c->prefetched = false;
    else TRY(collect_enqueue(c, info != nullptr));
    BPPO_HIP(c, sync_stream(c));
    return collect_finish(c, info, c->coll_slot);
}

extern "C" bppo_status bppo_rollout_episodes(bppo_ctx *c, bppo_episode *eps, int32_t cap, int32_t *n) {
    if (!c) return BPPO_ERR_ARG;
    int32_t cnt = 0;
    BPPO_HIP(c, hipMemcpyAsync(&cnt, c->d_ep_count, 4, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    int m = std::min(cnt, c->eps_cap);
    std::vector<EpisodeRec> recs(m);
    if (m) {
        BPPO_HIP(c, hipMemcpyAsync(recs.data(), c->d_eps, sizeof(EpisodeRec) * m, hipMemcpyDeviceToHost, c->stream));
        BPPO_HIP(c, sync_stream(c));
    }
    // reference order: by step, then env index (env.rs:470-483 collects in env order per step)
    std::sort(recs.begin(), recs.end(), [](const EpisodeRec &a, const EpisodeRec &b) {
        return a.step != b.step ? a.step < b.step : a.env_index < b.env_index; });
    for (int i = 0; i < m && i < cap; i++) {
        std::memcpy(eps[i].total_reward, recs[i].total_reward, sizeof(float) * BPPO_MAX_PLAYERS);
        eps[i].length = recs[i].length; eps[i].env_index = recs[i].env_index;
        eps[i].step = recs[i].step; eps[i].pad = 0;
    }
    if (n) *n = cnt;
    return BPPO_OK;
}

// bootstrap + GAE (main.rs:877-947)
// enqueue half (the CartPole path has no host read in it)
static bppo_status gae_enqueue(bppo_ctx *c) {
    c->prefetched = false;        // a pending rollout is consumed here (e.g. after a bppo_train_steps error)
    if (c->wide) {
        TRY(tm_begin(c, TM_GAE));
        TRY(wide_bootstrap_gae(c));
        TRY(tm_end(c, TM_GAE));
        c->gae_done = 1;
        return BPPO_OK;
    }
    TRY(tm_begin(c, TM_BOOT));
    TRY(launch_bootstrap(c, nullptr, nullptr, c->cfg.normalize_obs));
    TRY(popart_denorm(c, c->d_last_v, (size_t)c->N));   // main.rs:898-907
    TRY(tm_end(c, TM_BOOT));
    TRY(tm_begin(c, TM_GAE));
    bool packed = false;
    hipError_t he = hipSuccess;
    bppo_status s = launch_gae_1p(c->d_rew, c->d_done, c->d_val, c->d_last_v, c->T, c->N,
                                  (float)c->cfg.gamma, (float)c->cfg.gae_lambda, c->d_adv, c->d_ret,
                                  c->stream, c->rows_from_rollout ? c->d_rowB : nullptr, &packed, &he);
    c->rows_packed = packed;
    if (s != BPPO_OK) return he != hipSuccess ? hip_fail(c, he, "k_gae_1p launch") : s;
    TRY(tm_end(c, TM_GAE));
    c->gae_done = 1;
    return BPPO_OK;
}

extern "C" bppo_status bppo_compute_gae(bppo_ctx *c) {
    if (!c || !c->collected) { if (c) c->err = "compute_gae before collect_rollouts"; return BPPO_ERR_ARG; }
    TRY(gae_enqueue(c));
    BPPO_HIP(c, sync_stream(c));
    if (!c->wide) tm_read(c, TM_BOOT);
    tm_read(c, TM_GAE);
    return BPPO_OK;
}

// ppo.rs:1268-1294 compute_explained_variance as the reference computes it: f32
// iterator sums in order (each chain sequential; the two independent chains of a
// round are interleaved only for instruction-level parallelism), population
// variances, no fma contraction ((r - mean).powi(2) is a multiply, then the add)
static float ev_reference_f32(const float *v, const float *r, const float *valid, size_t n_all) {
#pragma clang fp contract(off)
    size_t n_ = 0;
    float s_r = 0.0f, s_res = 0.0f;
    for (size_t i = 0; i < n_all; i++) {
        if (valid && !(valid[i] > 0.5f)) continue;     // opponent pool: learner rows (ppo.rs:2047-2056)
        s_r += r[i];
        s_res += r[i] - v[i];
        n_++;
    }
    const float n = (float)n_;
    if (n < 2.0f) return 0.0f;
    const float mr = s_r / n, mres = s_res / n;
    float q_r = 0.0f, q_res = 0.0f;
    for (size_t i = 0; i < n_all; i++) {
        if (valid && !(valid[i] > 0.5f)) continue;
        const float d = r[i] - mr;
        q_r += d * d;
        const float e = (r[i] - v[i]) - mres;
        q_res += e * e;
    }
    const float vr = q_r / n;
    if (vr < 1e-8f) return 0.0f;
    return 1.0f - (q_res / n) / vr;
}

extern "C" bppo_status bppo_set_explained_variance_mode(bppo_ctx *c, int32_t mode) {
    if (!c || mode < 0 || mode > 1) return BPPO_ERR_ARG;
    if (mode == 1 && !c->h_ev_v) {
        // every resource into a local first: committed together, or all released
        const size_t TN = (size_t)c->T * c->N;
        hipStream_t st = nullptr;
        hipEvent_t e_gae = nullptr, e_cp = nullptr;
        float *hv = nullptr, *hr = nullptr, *hm = nullptr;
        hipError_t e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&e_gae, hipEventDisableTiming);
        if (e == hipSuccess) e = hipEventCreateWithFlags(&e_cp, hipEventDisableTiming | hipEventBlockingSync);
        if (e == hipSuccess) e = hipHostMalloc((void **)&hv, TN * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void **)&hr, TN * 4, hipHostMallocDefault);
        if (e == hipSuccess) e = hipHostMalloc((void **)&hm, TN * 4, hipHostMallocDefault);
        if (e != hipSuccess) {
            for (float *h : {hv, hr, hm}) if (h) (void)hipHostFree(h);
            if (e_cp) (void)hipEventDestroy(e_cp);
            if (e_gae) (void)hipEventDestroy(e_gae);
            if (st) (void)hipStreamDestroy(st);
            return hip_fail(c, e, "explained-variance reference mode: allocation");
        }
        c->ev_stream = st; c->ev_gae = e_gae; c->ev_copied = e_cp;
        c->h_ev_r = hr; c->h_ev_valid = hm;
        c->h_ev_v = hv;                    // last: marks the set complete
    }
    c->ev_mode = mode;
    return BPPO_OK;
}

extern "C" bppo_status bppo_debug_record_params(bppo_ctx *c, float *host, int32_t max_minibatches) {
    if (!c || max_minibatches < 0) return BPPO_ERR_ARG;
    c->dbg_params = max_minibatches > 0 ? host : nullptr;
    c->dbg_params_max = host ? max_minibatches : 0;
    return BPPO_OK;
}

extern "C" bppo_status bppo_set_minibatch_kernel(bppo_ctx *c, int32_t mode) {
    if (!c || mode < 0 || mode > 2) return BPPO_ERR_ARG;
    c->mb_kernel = mode;
    return BPPO_OK;
}

// mode 1: copy the buffers the metric reads (stream order: after GAE, before anything
// later rewrites them) and sum them on a host thread while the update runs
static bppo_status ev_reference_begin(bppo_ctx *c, const float *d_valid) {
    const size_t TN = (size_t)c->T * c->N;
    // a thread left by an update that returned early still reads the pinned buffers
    // (or waits on ev_copied): it ends before they are refilled or the event re-recorded
    if (c->ev_thread.joinable()) c->ev_thread.join();
    BPPO_HIP(c, hipEventRecord(c->ev_gae, c->stream));
    BPPO_HIP(c, hipStreamWaitEvent(c->ev_stream, c->ev_gae, 0));
    BPPO_HIP(c, hipMemcpyAsync(c->h_ev_v, c->d_val, TN * 4, hipMemcpyDeviceToHost, c->ev_stream));
    BPPO_HIP(c, hipMemcpyAsync(c->h_ev_r, c->d_ret, TN * 4, hipMemcpyDeviceToHost, c->ev_stream));
    if (d_valid) BPPO_HIP(c, hipMemcpyAsync(c->h_ev_valid, d_valid, TN * 4, hipMemcpyDeviceToHost, c->ev_stream));
    BPPO_HIP(c, hipEventRecord(c->ev_copied, c->ev_stream));
    const bool vf = d_valid != nullptr;
    c->ev_thread = std::thread([c, TN, vf]() {
        (void)pthread_setname_np(pthread_self(), "bppo-ev");
        (void)hipEventSynchronize(c->ev_copied);
        c->ev_ref = ev_reference_f32(c->h_ev_v, c->h_ev_r, vf ? c->h_ev_valid : nullptr, TN);
    });
    return BPPO_OK;
}

// ppo_update (ppo.rs:1661-2112)
extern "C" bppo_status bppo_ppo_update(bppo_ctx *c, double lr, double ent_coef, bppo_update_metrics *m) {
    if (!c || !c->gae_done) { if (c) c->err = "ppo_update before compute_gae"; return BPPO_ERR_ARG; }
    // opponent pool: train on the learner rows only (ppo.rs:1696-1720); their count
    // varies per update, so each epoch's swap targets come from the sequential
    // host walk instead of the speculating shuffle engine
    const bool opp = opp_active(c);
    if (opp) {
        // the opponent path permutes on this stream with the shared scratch, into the
        // context's own buffer, after anything still queued on fy_stream
        if (c->fy_done > 0) BPPO_HIP(c, hipStreamWaitEvent(c->stream, c->fy_ev[c->fy_done - 1], 0));
        c->fy_slot = -1; c->fy_done = 0;
        c->d_perm = c->d_perm_base;
        TRY(opp_compact_valid(c));
    }
    if (!opp && c->shuf_slot < 0) c->shuf_slot = c->shuf.ensure(c->rng_pos);
    const int slot = c->shuf_slot;
    const size_t B = opp ? (size_t)c->n_valid : (size_t)c->T * c->N;
    std::vector<uint32_t> Jh(opp ? std::max<size_t>(B, 1) * c->cfg.num_epochs : 0);
    uint64_t opp_pos = c->rng_pos;
    const int M = c->cfg.num_minibatches;
    const size_t base_mb = B / M, rem = B % M;
    const int np = (int)c->net.n_params;
    const int NM = WM_COUNT;
    std::vector<float> rows;          // per minibatch: NM metric sums + 4 adv stats
    int epochs_run = 0;
    bool stop = false;
    double wait_ms = 0.0;
    TRY(tm_begin(c, TM_UPDATE));
    // mode 1 copies d_val / d_ret on ev_stream beside the update: on every return from here
    // the context stream waits for those copies, so the next rollout cannot overwrite the
    // buffers under them (the normal path enqueues the wait itself below)
    struct EvCopyGuard {
        bppo_ctx *c; bool armed = false;
        ~EvCopyGuard() { if (armed) (void)hipStreamWaitEvent(c->stream, c->ev_copied, 0); }
    } ev_guard{c};
    if (c->ev_mode == 1) { TRY(ev_reference_begin(c, opp ? c->d_valid : nullptr)); ev_guard.armed = true; }
    TRY(popart_update_begin(c, opp ? c->d_valid : nullptr));   // ppo.rs:1787-1808
    if (c->d_rowA && !c->rows_packed) TRY(launch_pack_rows(c));
    c->rows_packed = false;
    float fw_ms = 0, sh_ms = 0;
    // without a KL early stop or a host all-reduce nothing in the loop needs the
    // metrics on the host: the minibatches are enqueued back to back and the rows
    // are read once after the last one (no per-minibatch stream drain)
    const bool deferred = c->cfg.target_kl < 0 && !(c->allreduce && c->world > 1 && !c->allreduce_async);
    int nrow = 0;
    // the deferred path times the update's last minibatch that runs: sizes do not grow with
    // the slot index, so it is slot M-1 unless B < M (then rem-1; none when B == 0); lockstep
    // slots (W > 1) all run
    const int last_run_mb = (base_mb > 0 || (c->allreduce && c->world > 1)) ? M - 1 : (int)rem - 1;
    bool fw_recorded = false;
    bool first_mb = true;                 // the update's first minibatch: the rollout's parameters
    size_t rows_done = 0;                 // rows of the KL-stopped epoch's minibatches that ran
    for (int ep = 0; ep < c->cfg.num_epochs && !stop; ep++) {
        epochs_run++;
        hipEvent_t s0 = c->ev[TM_SHUFFLE][0], s1 = c->ev[TM_SHUFFLE][1];
        if (opp) {
            uint32_t *J = Jh.data() + (size_t)ep * B;
            auto w0 = std::chrono::steady_clock::now();
            opp_pos = shuffle_walk_host(c->rng_key, c->cfg.rng_stream, opp_pos, (uint32_t)B, J);   // ppo.rs:1816
            wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
            BPPO_HIP(c, hipMemcpyAsync(c->d_Jopp, J, sizeof(uint32_t) * B, hipMemcpyHostToDevice, c->stream));
            BPPO_HIP(c, hipEventRecord(s0, c->stream));
            if (B) TRY(launch_fisher_yates(c, c->d_Jopp, (uint32_t)B));
            if (B) TRY(opp_map_perm(c, (uint32_t)B));
            BPPO_HIP(c, hipEventRecord(s1, c->stream));
        } else {
            if (slot != c->fy_slot || ep >= c->fy_done) {
                auto w0 = std::chrono::steady_clock::now();
                c->shuf.wait_epoch(slot, ep);
                wait_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
            }
            TRY(fy_enqueue_ready(c, slot));          // this epoch and any other resolved since
            BPPO_HIP(c, hipStreamWaitEvent(c->stream, c->fy_ev[ep], 0));
            c->d_perm = c->d_perm_ep + (size_t)ep * B;
        }
        // no learner rows (opponent pool): the reference shuffles an empty index
        // list (no RNG words) and skips every minibatch (ppo.rs:1815-1831).  W > 1: the
        // ranks' learner-row counts differ, so every rank runs all M minibatch slots of
        // every epoch in lockstep (one all-reduce each); a rank whose slot is empty adds a
        // zero gradient and zero metric partials (oracle/ppo.c or_trainers_update)
        const bool lockstep = c->allreduce && c->world > 1;
        if (B == 0 && !lockstep) continue;
        if (B) TRY(launch_epoch_adv_stats(c, (uint32_t)B, M, opp ? nullptr : c->d_inv_ep + (size_t)ep * B));
        size_t start = 0;
        for (int mb = 0; mb < M; mb++) {
            const size_t sz = base_mb + ((size_t)mb < rem ? 1 : 0);
            if (sz == 0 && !lockstep) continue;
            // the "minibatch" phase time is the last minibatch's (read after the update in the
            // deferred path): only that one is bracketed there -- each timestamp marker on the
            // stream costs a few us of idle compute stream
            const bool fw_timed = !deferred || (ep == c->cfg.num_epochs - 1 && mb == last_run_mb);
            if (fw_timed) BPPO_HIP(c, hipEventRecord(c->ev[TM_FWDBWD][0], c->stream));
            c->d_mb_cur = c->d_mb_stats + 4 * mb;
            // Adam's bias corrections for this step (burn-optim: per tensor, f32 powers)
            float c1[64], c2[64];
            for (int t = 0; t < 2 * c->net.n_layers; t++) {
                int ti = ++c->adam_t[t];
                c1[t] = 1.0f - powi_f32(0.9f, ti);
                c2[t] = 1.0f - powi_f32(0.999f, ti);
            }
            float *metric_dst = c->d_rows + (size_t)nrow * (NM + 4);
            const bool multi = c->allreduce && c->world > 1;
            if (sz == 0) {                 // lockstep slot without rows on this rank
                BPPO_HIP(c, hipMemsetAsync(c->d_grad, 0, sizeof(float) * ((size_t)np + 64), c->stream));   // + tail
                BPPO_HIP(c, hipMemsetAsync(c->d_mb_cur, 0, sizeof(float) * 4, c->stream));
                // value_error_max of no rows: -inf, as the oracle's (the metric row reads the
                // rank-local copy; the summed slot GRAD_VEMAX is not read)
                static const float ninf = -INFINITY;
                BPPO_HIP(c, hipMemcpyAsync(c->d_grad + np + GRAD_VEMAX_LOCAL, &ninf, sizeof(float),
                                           hipMemcpyHostToDevice, c->stream));
            } else if (c->wide) {
                if (c->dbg_params && nrow < c->dbg_params_max)   // parity hook: this minibatch's parameters
                    BPPO_HIP(c, hipMemcpyAsync(c->dbg_params + (size_t)nrow * np, c->d_params, sizeof(float) * np,
                                               hipMemcpyDeviceToHost, c->stream));
                TRY(wide_minibatch(c, (uint32_t)start, (uint32_t)sz, ent_coef, first_mb));
            } else {
                if (c->dbg_params && nrow < c->dbg_params_max)
                    BPPO_HIP(c, hipMemcpyAsync(c->dbg_params + (size_t)nrow * np, c->d_params, sizeof(float) * np,
                                               hipMemcpyDeviceToHost, c->stream));
                TRY(launch_minibatch(c, (uint32_t)start, (uint32_t)sz, (float)ent_coef, first_mb));
            }
            if (fw_timed) { BPPO_HIP(c, hipEventRecord(c->ev[TM_FWDBWD][1], c->stream)); fw_recorded = true; }
            first_mb = false;
            if (multi) {
                if (!c->allreduce_async) BPPO_HIP(c, sync_stream(c));
                if (c->allreduce(c->d_grad, (size_t)np + NM, c->allreduce_user) != 0) {
                    c->err = "all-reduce callback failed";
                    return BPPO_ERR_COMM;
                }
            }
            // clip + Adam; the metric row (grad[np .. np+NM) and adv stats) into the
            // update's device rows
            TRY(launch_adam(c, (float)lr, c1, c2, metric_dst, NM));
            if (c->wide) TRY(wide_pack(c));
            nrow++;
            if (!deferred) {
                std::vector<float> row(NM + 4);
                BPPO_HIP(c, hipMemcpyAsync(row.data(), c->d_rows + (size_t)(nrow - 1) * (NM + 4), sizeof(float) * (NM + 4),
                                           hipMemcpyDeviceToHost, c->stream));
                BPPO_HIP(c, sync_stream(c));
                float ms = 0;
                if (event_ms(c->ev[TM_FWDBWD][0], c->ev[TM_FWDBWD][1], &ms)) fw_ms = ms;
                if (mb == 0 && event_ms(s0, s1, &ms)) sh_ms = ms;
                rows.insert(rows.end(), row.begin(), row.end());
            }
            if (!deferred && c->cfg.target_kl >= 0) {
                const float *row = &rows[rows.size() - (NM + 4)];
                const float n = row[10] > 0 ? row[10] : 1.0f;
                if (row[3] / n > (float)c->cfg.target_kl) { stop = true; rows_done = start + sz; break; }   // ppo.rs:2019-2023
            }
            start += sz;
        }
    }
    if (deferred && nrow > 0) {
        rows.resize((size_t)nrow * (NM + 4));
        // into pinned memory: a pageable destination makes the copy synchronous and the
        // host thread spins in it for the whole update (a CPU the shuffle walkers need);
        // read after the one stream wait below, behind the explained-variance pass
        BPPO_HIP(c, hipMemcpyAsync(c->h_rows, c->d_rows, sizeof(float) * rows.size(), hipMemcpyDeviceToHost, c->stream));
    }
    TRY(tm_end(c, TM_UPDATE));
    c->last_wait_ms = wait_ms;
    c->last_walk_ms = 0.0;
    c->last_met = 0;
    if (opp) {
        c->rng_pos = opp_pos;                               // the epochs walked (early stop: started ones)
        c->last_walk_ms = wait_ms;
        BPPO_HIP(c, hipStreamSynchronize(c->stream));      // Jh's copies done
    } else {
        // only started epochs consumed words (reference); windowed: the update's fixed span
        c->rng_pos = c->shuf.win ? c->shuf.job_end(slot) : c->shuf.end_pos[slot][epochs_run - 1];
        for (int e = 0; e < epochs_run; e++) {
            c->last_walk_ms += c->shuf.walk_ms[slot][e];
            c->last_met += c->shuf.coalesced[slot][e] >= 0 && e > 0;
        }
        c->last_spec_mwords = (double)c->shuf.spec_words.exchange(0) * 1e-6;
        c->last_true_mwords = (double)c->shuf.true_words.exchange(0) * 1e-6;
        c->last_walk_cpu_ms = (double)c->shuf.tsc_walk.exchange(0) / tsc_per_ms();
        c->last_words_cpu_ms = (double)c->shuf.tsc_words.exchange(0) / tsc_per_ms();
        c->shuf_slot = -1;
        // this update's reads of the J slot are enqueued (fy_stream's too: epochs
        // permuted ahead but not run after a KL early stop); the next update's
        // shuffles begin after its rollout's T*N*A Gumbel words (usually chained already)
        if (c->fy_slot == slot && c->fy_done > 0)
            BPPO_HIP(c, hipStreamWaitEvent(c->stream, c->fy_ev[c->fy_done - 1], 0));
        c->fy_slot = -1;
        c->fy_done = 0;
        BPPO_HIP(c, c->shuf.release(slot, c->stream));
        c->shuf.ensure(c->rng_pos + (uint64_t)c->T * c->N * (uint64_t)c->A);
    }
    TRY(popart_target_stats(c, stop ? epochs_run - 1 : epochs_run, rows_done, opp ? c->d_valid : nullptr));
    TRY(launch_explained_variance(c, opp ? c->d_valid : nullptr));
    // mode 1: nothing after this update (the next rollout) overwrites the copied buffers early
    if (ev_guard.armed) { ev_guard.armed = false; BPPO_HIP(c, hipStreamWaitEvent(c->stream, c->ev_copied, 0)); }
    BPPO_HIP(c, hipEventRecord(c->ev_upd, c->stream));      // end of this update's work
    if (c->prefetch_next) {
        // bppo_train_steps: the next rollout goes in behind this update (it needs only the
        // updated parameters and the RNG position after this update's shuffles, both in
        // stream / host order now); the host then waits for this update alone
        c->prefetch_next = false;
        c->env_step = c->prefetch_env_step;
        TRY(collect_enqueue(c, true));
        c->prefetched = true;
        BPPO_HIP(c, wait_event(c, c->ev_upd));
    } else {
        BPPO_HIP(c, sync_stream(c));
    }
    if (deferred && nrow > 0) {
        std::memcpy(rows.data(), c->h_rows, sizeof(float) * rows.size());
        float ms = 0;
        if (fw_recorded && event_ms(c->ev[TM_FWDBWD][0], c->ev[TM_FWDBWD][1], &ms)) fw_ms = ms;   // else 0
        if (event_ms(c->ev[TM_SHUFFLE][0], c->ev[TM_SHUFFLE][1], &ms)) sh_ms = ms;
    }
    double ev4[4];
    explained_variance_sums(c, ev4);
    if (c->ev_thread.joinable()) c->ev_thread.join();     // mode 1: the reference's f32 sums
    tm_read(c, TM_UPDATE);
    if (c->mb_ev_n > 0) {                     // every minibatch kernel launch of this update
        double sum = 0.0, ks[2] = {0.0, 0.0};
        float lo = INFINITY, hi = 0.0f;
        int n = 0, kn[2] = {0, 0};
        for (int i = 0; i < c->mb_ev_n; i++) {
            float ms = 0.0f;
            if (!event_ms(c->mb_ev[i][0], c->mb_ev[i][1], &ms)) continue;
            sum += ms; lo = std::min(lo, ms); hi = std::max(hi, ms); n++;
            ks[c->mb_ev_split[i]] += ms; kn[c->mb_ev_split[i]]++;
        }
        if (n) { c->mb_k_mean = (float)(sum / n); c->mb_k_min = lo; c->mb_k_max = hi; }
        c->mb_k_exact = kn[0] ? (float)(ks[0] / kn[0]) : 0.0f;
        c->mb_k_split = kn[1] ? (float)(ks[1] / kn[1]) : 0.0f;
        c->mb_ev_n = 0;
    }
    c->mb_launch = 0;
    c->last_ms[TM_FWDBWD] = fw_ms;
    c->last_ms[TM_SHUFFLE] = sh_ms;
    c->last_rows = rows;
    if (m) {
        std::memset(m, 0, sizeof *m);
        const int nup = (int)(rows.size() / (NM + 4));
        float tp = 0, tv = 0, th = 0, tk = 0, tc = 0, tl = 0, tvm = 0, trm = 0, tam = 0, tas = 0;
        float tamin = INFINITY, tamax = -INFINITY, tvem = 0, tves = 0, tvemax = -INFINITY;
        float tav = 0, tevp = 0;
        for (int u = 0; u < nup; u++) {
            const float *r = &rows[(size_t)u * (NM + 4)];
            const float n = r[10] > 0 ? r[10] : 1.0f;
            const float pl = r[0] / n, vl = 0.5f * (r[1] / n), h = r[2] / n;
            tp += pl; tv += vl; th += h; tk += r[3] / n; tc += r[4] / n;
            tl += pl + vl * (float)c->cfg.value_coef + (-h) * (float)ent_coef;
            tvm += r[5] / n; trm += r[6] / n;
            const float vem = r[7] / n;
            tvem += vem;
            const double var = n > 1 ? ((double)r[8] - (double)n * vem * vem) / (double)(n - 1) : 0.0;
            tves += sqrtf((float)std::max(var, 0.0));
            tvemax = std::max(tvemax, r[9]);
            tav += r[WM_VALID] / n;
            tevp += r[WM_NCHOICE] > 0 ? r[WM_HV] / r[WM_NCHOICE] : 0.0f;
            tam += r[NM]; tas += r[NM + 1];
            tamin = std::min(tamin, r[NM + 2]); tamax = std::max(tamax, r[NM + 3]);
        }
        // averaged over the minibatches run; none run -> 0/0 = NaN as in ppo.rs:2071-2090
        const float n = (float)nup;
        m->policy_loss = tp / n; m->value_loss = tv / n; m->entropy = th / n;
        m->entropy_scaled = m->entropy / logf((float)c->A);
        m->approx_kl = tk / n; m->clip_fraction = tc / n; m->total_loss = tl / n;
        m->value_mean = tvm / n; m->returns_mean = trm / n;
        m->adv_mean_raw = tam / n; m->adv_std_raw = tas / n; m->adv_min_raw = tamin; m->adv_max_raw = tamax;
        m->value_error_mean = tvem / n; m->value_error_std = tves / n; m->value_error_max = tvemax;
        const double Bn = (double)B;
        const double mr = ev4[0] / Bn, vr = ev4[1] / Bn - mr * mr;
        const double mres = ev4[2] / Bn, vres = ev4[3] / Bn - mres * mres;
        // ppo.rs:1268-1294 (fewer than 2 rows or Var(R) < 1e-8 -> 0)
        m->explained_variance = (B < 2 || vr < 1e-8) ? 0.0f : (float)(1.0 - vres / vr);
        if (c->ev_mode == 1) m->explained_variance = c->ev_ref;
        // ppo.rs:1549-1565: only envs with action masks report these (None -> 0)
        if (c->cfg.env_kind != BPPO_ENV_CARTPOLE) { m->avg_valid_actions = tav / n; m->entropy_valid_pct = tevp / n; }
        m->num_updates = nup; m->epochs_run = epochs_run;
        // PopArt metrics (ppo.rs:2061-2068): None -> NaN
        m->value_norm_target_mean = m->value_norm_target_std = NAN;
        m->value_norm_rescale_mag = c->pa_rescale_mag;
        if (c->cfg.normalize_values && c->pa_tcount > 0) {
            const double mean = c->pa_tsum / c->pa_tcount, var = c->pa_tsq / c->pa_tcount - mean * mean;
            m->value_norm_target_mean = (float)mean;
            m->value_norm_target_std = (float)std::sqrt(std::max(var, 0.0));
        }
    }
    c->collected = 0; c->gae_done = 0;
    return BPPO_OK;
}

// One iteration of main.rs:860-947 + ppo_update in one call: the rollout, the
// bootstrap/GAE and the update are enqueued back to back with no host wait
// between them (bppo_collect_rollouts and bppo_compute_gae each drain the stream
// for their results).  The rollout's device error flags are read after the update:
// a non-finite log-prob or an empty mask returns its status then, with the update
// already applied (the reference panics before updating; either way the run ends).
extern "C" bppo_status bppo_train_step(bppo_ctx *c, double lr, double ent_coef, bppo_rollout_info *info,
                                       bppo_update_metrics *m) {
    if (!c) return BPPO_ERR_ARG;
    const auto t0 = std::chrono::steady_clock::now();
    c->sync_wait_ms = 0.0;
    if (c->prefetched) c->prefetched = false;     // enqueued ahead by bppo_train_steps (see bppo_collect_rollouts)
    else TRY(collect_enqueue(c, info != nullptr));
    TRY(gae_enqueue(c));
    const bppo_status us = bppo_ppo_update(c, lr, ent_coef, m);   // drains the stream at its end
    if (us == BPPO_OK) { if (!c->wide) tm_read(c, TM_BOOT); tm_read(c, TM_GAE); }
    const bppo_status cs = collect_finish(c, info, c->coll_slot);
    // host time in the call outside stream waits: enqueue work + engine waits
    c->last_host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() -
                      c->sync_wait_ms;
    c->last_sync_ms = c->sync_wait_ms;
    return cs != BPPO_OK ? cs : us;
}

// n iterations of bppo_train_step in one call, software-pipelined: each update's
// last stream wait covers that update only, with the next iteration's rollout
// already enqueued behind it, so the GPU never idles between iterations (the
// host tail of one update, the caller and the next enqueue ran in that gap).
// Results are those of n sequential bppo_train_step calls with lr[k], ent[k] and
// the env step global_step0 + k*T*N; nothing is left pending when it returns.
// phase_keys/phase_sums (optional): bppo_last_kernel_ms of each key summed over the n.
extern "C" bppo_status bppo_train_steps(bppo_ctx *c, int32_t n, const double *lr, const double *ent_coef,
                                        uint64_t global_step0, bppo_rollout_info *infos, bppo_update_metrics *ms,
                                        const char *const *phase_keys, int32_t nkeys, float *phase_sums) {
    if (!c || n < 0 || !lr || !ent_coef || (nkeys > 0 && (!phase_keys || !phase_sums))) return BPPO_ERR_ARG;
    for (int k = 0; k < nkeys; k++) phase_sums[k] = 0.0f;
    const uint64_t TN = (uint64_t)c->T * c->N * (uint64_t)c->world;   // the job's env steps per iteration
    for (int32_t k = 0; k < n; k++) {
        const auto t0 = std::chrono::steady_clock::now();
        c->sync_wait_ms = 0.0;
        if (!c->prefetched) { c->env_step = global_step0 + (uint64_t)k * TN; TRY(collect_enqueue(c, true)); }
        c->prefetched = false;
        const int slot = c->coll_slot;
        TRY(gae_enqueue(c));
        c->prefetch_next = k + 1 < n;
        c->prefetch_env_step = global_step0 + (uint64_t)(k + 1) * TN;
        const bppo_status us = bppo_ppo_update(c, lr[k], ent_coef[k], ms ? &ms[k] : nullptr);
        c->prefetch_next = false;
        // on an error the next iteration's rollout may already be enqueued (ppo_update
        // enqueues it before its wait): drain the stream so nothing is pending on
        // return; that rollout stays the context's next one (prefetched), which
        // bppo_collect_rollouts / bppo_train_step(s) then use instead of drawing another
        if (us != BPPO_OK) { (void)sync_stream(c); c->collected = c->prefetched ? 1 : 0; return us; }
        if (!c->wide) tm_read(c, TM_BOOT);
        tm_read(c, TM_GAE);
        const bppo_status cs = collect_finish(c, infos ? &infos[k] : nullptr, slot);
        if (cs != BPPO_OK) { (void)sync_stream(c); c->collected = c->prefetched ? 1 : 0; return cs; }
        c->last_host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() -
                          c->sync_wait_ms;
        c->last_sync_ms = c->sync_wait_ms;
        for (int q = 0; q < nkeys; q++) {
            float v = 0.0f;
            if (bppo_last_kernel_ms(c, phase_keys[q], &v) == BPPO_OK) phase_sums[q] += v;
        }
    }
    return BPPO_OK;
}

// W > 1.  PopArt's statistics are all-gathered (popart.hip): its
// scratch is sized for the world here
static bppo_status check_world(bppo_ctx *c, int32_t world) {
    if (world > 1 && c->cfg.normalize_values) {
        if (c->d_pa_gather) { BPPO_HIP(c, hipFree(c->d_pa_gather)); c->d_pa_gather = nullptr; }
        BPPO_HIP(c, hipMalloc((void **)&c->d_pa_gather, sizeof(float) * 9 * (size_t)world));
    }
    return BPPO_OK;
}

extern "C" bppo_status bppo_set_rank(bppo_ctx *c, int32_t rank) {
    if (!c || rank < 0) return BPPO_ERR_ARG;
    c->rank = rank;
    return BPPO_OK;
}

extern "C" bppo_status bppo_set_allreduce(bppo_ctx *c, bppo_allreduce_fn fn, void *user, int32_t world) {
    if (!c || world < 1) return BPPO_ERR_ARG;
    TRY(check_world(c, world));
    c->allreduce = fn; c->allreduce_user = user; c->world = world; c->allreduce_async = 0;
    return BPPO_OK;
}

extern "C" bppo_status bppo_set_allreduce_async(bppo_ctx *c, bppo_allreduce_fn fn, void *user, int32_t world) {
    if (!c || world < 1) return BPPO_ERR_ARG;
    TRY(check_world(c, world));
    c->allreduce = fn; c->allreduce_user = user; c->world = world; c->allreduce_async = 1;
    return BPPO_OK;
}

extern "C" bppo_status bppo_get_stream(bppo_ctx *c, void **stream) {
    if (!c || !stream) return BPPO_ERR_ARG;
    *stream = (void *)c->stream;
    return BPPO_OK;
}

struct BufDesc { void *ptr; size_t bytes; };
static BufDesc find_buf(bppo_ctx *c, const char *name) {
    const size_t TN = (size_t)c->T * c->N;
    if (!strcmp(name, "obs")) return {c->d_obs, TN * c->D * 4};
    if (!strcmp(name, "actions")) return {c->d_act, TN * 4};
    if (!strcmp(name, "rewards")) return {c->d_rew, TN * 4};
    if (!strcmp(name, "raw_rewards")) return {c->d_rew_raw, TN * 4};
    if (!strcmp(name, "valid")) return {c->d_valid, c->d_valid ? TN * 4 : 0};
    if (!strcmp(name, "dones")) return {c->d_done, TN * 4};
    if (!strcmp(name, "values")) return {c->d_val, TN * 4};
    if (!strcmp(name, "log_probs")) return {c->d_logp, TN * 4};
    if (!strcmp(name, "advantages")) return {c->d_adv, TN * 4};
    if (!strcmp(name, "returns")) return {c->d_ret, TN * 4};
    if (!strcmp(name, "all_rewards")) return {c->d_rew, TN * 4};
    if (!strcmp(name, "perm")) return {c->d_perm, TN * 4};
    if (!strncmp(name, "perm_ep:", 8)) {          // epoch e's permutation of the last update
        const int e = atoi(name + 8);
        if (e < 0 || e >= c->cfg.num_epochs || !c->d_perm_ep) return {nullptr, 0};
        return {c->d_perm_ep + (size_t)e * TN, TN * 4};
    }
    if (!strcmp(name, "last_values")) return {c->d_last_v, (size_t)c->N * 4};
    if (!strcmp(name, "grad")) return {c->d_grad, c->net.n_params * 4};
    return {nullptr, 0};
}

extern "C" bppo_status bppo_buffer_get(bppo_ctx *c, const char *name, void *host, size_t bytes) {
    if (!c || !name || !host) return BPPO_ERR_ARG;
    if (c->wide) {
        bool handled = false;
        bppo_status s = wide_buffer_get(c, name, host, bytes, &handled);
        if (handled) return s;
    }
    BufDesc b = find_buf(c, name);
    if (!b.ptr || bytes < b.bytes) { c->err = std::string("buffer_get: unknown buffer or too small: ") + name; return BPPO_ERR_ARG; }
    BPPO_HIP(c, hipMemcpyAsync(host, b.ptr, b.bytes, hipMemcpyDeviceToHost, c->stream));
    BPPO_HIP(c, sync_stream(c));
    return BPPO_OK;
}

extern "C" int32_t bppo_minibatch_rows(bppo_ctx *c, float *out, int32_t max_rows, int32_t *row_width) {
    if (!c) return -1;
    const int32_t w = WM_COUNT + 4;
    const int32_t n = (int32_t)(c->last_rows.size() / (size_t)w);
    if (row_width) *row_width = w;
    if (out && max_rows > 0)
        std::memcpy(out, c->last_rows.data(), sizeof(float) * (size_t)std::min(n, max_rows) * (size_t)w);
    return n;
}

extern "C" bppo_status bppo_buffer_set(bppo_ctx *c, const char *name, const void *host, size_t bytes) {
    if (!c || !name || !host) return BPPO_ERR_ARG;
    BufDesc b = find_buf(c, name);
    if (!b.ptr || bytes != b.bytes) { c->err = std::string("buffer_set: unknown buffer or size mismatch: ") + name; return BPPO_ERR_ARG; }
    BPPO_HIP(c, hipMemcpyAsync(b.ptr, host, b.bytes, hipMemcpyHostToDevice, c->stream));
    BPPO_HIP(c, sync_stream(c));
    if (!strcmp(name, "advantages") || !strcmp(name, "returns")) c->gae_done = c->collected = 1;
    c->rows_packed = c->rows_from_rollout = false;   // the update re-packs its rows from the buffers
    return BPPO_OK;
}

extern "C" bppo_status bppo_gae_device(const float *r, const float *d, const float *v, const float *lv,
                                       int32_t T, int32_t N, float gamma, float lambda, float *adv,
                                       float *ret, void *stream) {
    if (!r || !d || !v || !lv || !adv || !ret || T < 0 || N < 0) return BPPO_ERR_ARG;
    return launch_gae_1p(r, d, v, lv, T, N, gamma, lambda, adv, ret, (hipStream_t)stream);
}

extern "C" bppo_status bppo_gae_rows_device(const float *r, const float *d, const float *v, const float *lv,
                                            int32_t T, int32_t N, float gamma, float lambda, float *adv,
                                            float *ret, float *rows, void *stream) {
    if (!r || !d || !v || !lv || !adv || !ret || !rows || T < 0 || N < 0) return BPPO_ERR_ARG;
    // only the segmented kernel writes the pairs: refuse other shapes before launching anything
    if (N % 4 != 0 || T > 128 ||
        ((uintptr_t)r | (uintptr_t)d | (uintptr_t)v | (uintptr_t)lv | (uintptr_t)adv | (uintptr_t)ret | (uintptr_t)rows) % 16)
        return BPPO_ERR_UNSUPPORTED;
    bool packed = false;
    const bppo_status s = launch_gae_1p(r, d, v, lv, T, N, gamma, lambda, adv, ret, (hipStream_t)stream,
                                        reinterpret_cast<float2 *>(rows), &packed);
    return s != BPPO_OK ? s : packed ? BPPO_OK : BPPO_ERR_UNSUPPORTED;
}

extern "C" bppo_status bppo_gae_mp_device(const float *ar, const int32_t *pl, const float *d,
                                          const float *v, const float *lvpp, int32_t T, int32_t N,
                                          int32_t P, float gamma, float lambda, float *adv, float *ret,
                                          void *stream) {
    if (!ar || !pl || !d || !v || !lvpp || !adv || !ret || T < 0 || N < 0 || P < 1 || P > BPPO_MAX_PLAYERS)
        return BPPO_ERR_ARG;
    return launch_gae_mp(ar, pl, d, v, lvpp, T, N, P, gamma, lambda, adv, ret, (hipStream_t)stream);
}

extern "C" bppo_status bppo_last_kernel_ms(bppo_ctx *c, const char *k, float *ms) {
    if (!c || !k || !ms) return BPPO_ERR_ARG;
    static const char *names[8] = {"rollout", "gae", "update", "minibatch", "return_norm", "shuffle",
                                   "adam", "bootstrap"};
    for (int i = 0; i < 8; i++)
        if (!strcmp(k, names[i])) { *ms = c->last_ms[i]; return BPPO_OK; }
    // host side of the shuffle: draw-chain walk of the last update's epochs, and the
    // time ppo_update blocked waiting for it
    if (!strcmp(k, "shuffle_walk")) { *ms = (float)c->last_walk_ms; return BPPO_OK; }
    if (!strcmp(k, "minibatch_kernel")) { *ms = c->mb_k_mean; return BPPO_OK; }   // all launches of the last update
    if (!strcmp(k, "minibatch_kernel_min")) { *ms = c->mb_k_min; return BPPO_OK; }
    if (!strcmp(k, "minibatch_kernel_max")) { *ms = c->mb_k_max; return BPPO_OK; }
    if (!strcmp(k, "minibatch_kernel_split")) { *ms = c->mb_k_split; return BPPO_OK; }   // k_minibatch_split launches
    if (!strcmp(k, "minibatch_kernel_exact")) { *ms = c->mb_k_exact; return BPPO_OK; }   // k_minibatch_mfma launches
    if (!strcmp(k, "shuffle_wait")) { *ms = (float)c->last_wait_ms; return BPPO_OK; }
    if (!strcmp(k, "host_enqueue")) { *ms = (float)c->last_host_ms; return BPPO_OK; }   // bppo_train_step outside stream waits
    if (!strcmp(k, "host_sync_wait")) { *ms = (float)c->last_sync_ms; return BPPO_OK; }
    if (!strcmp(k, "shuffle_walk_tsc_ms")) { *ms = (float)c->last_walk_cpu_ms; return BPPO_OK; }    // all walks, in chain_walk
    if (!strcmp(k, "shuffle_words_tsc_ms")) { *ms = (float)c->last_words_cpu_ms; return BPPO_OK; }  // all walks, getting words
    if (!strcmp(k, "shuffle_spec_mwords")) { *ms = (float)c->last_spec_mwords; return BPPO_OK; }   // speculative walk words (M)
    if (!strcmp(k, "shuffle_true_mwords")) { *ms = (float)c->last_true_mwords; return BPPO_OK; }   // true walk words (M)
    if (!strcmp(k, "shuffle_met")) { *ms = (float)c->last_met; return BPPO_OK; }   // epochs resolved by speculation
    return BPPO_ERR_ARG;
}

extern "C" bppo_status bppo_debug_libm(int32_t which, int32_t device, const float *x, float *y, size_t n) {
    if (!x || !y) return BPPO_ERR_ARG;
    if (!device) {
        for (size_t i = 0; i < n; i++) {
            float v = x[i];
            switch (which) {
            case 0: y[i] = bppo_math::logf_glibc(v); break;
            case 1: y[i] = bppo_math::sinf_glibc(v); break;
            case 2: y[i] = bppo_math::cosf_glibc(v); break;
            case 3: y[i] = -bppo_math::logf_glibc(-bppo_math::logf_glibc(v)); break;
            case 5: y[i] = bppo_math::tanhf_glibc(v); break;
            default: y[i] = bppo_math::expf_glibc(v); break;
            }
        }
        return BPPO_OK;
    }
    float *dx = nullptr, *dy = nullptr;
    if (hipMalloc((void **)&dx, n * 4) != hipSuccess || hipMalloc((void **)&dy, n * 4) != hipSuccess) return BPPO_ERR_HIP;
    bppo_status s = BPPO_ERR_HIP;
    if (hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice) == hipSuccess &&
        launch_libm(which, dx, dy, n) == BPPO_OK && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(y, dy, n * 4, hipMemcpyDeviceToHost) == hipSuccess)
        s = BPPO_OK;
    (void)hipFree(dx); (void)hipFree(dy);
    return s;
}

// shuffle parity hooks: the host draw chain alone, and the device Fisher-Yates
// on caller-given swap targets
extern "C" bppo_status bppo_debug_shuffle_chain(uint64_t seed, uint64_t stream, uint64_t word_pos, uint32_t n,
                                                uint32_t *J, uint64_t *end_pos) {
    if (!J && n) return BPPO_ERR_ARG;
    const Key8 key = seed_key(seed);
    const uint64_t e = shuffle_walk_host(key, stream, word_pos, n, J);
    if (end_pos) *end_pos = e;
    return BPPO_OK;
}

extern "C" bppo_status bppo_debug_chain_walk2(uint64_t seed, uint64_t stream, uint64_t pos_a, uint64_t pos_b,
                                              uint32_t n, uint32_t piece, uint64_t *end_a, uint64_t *end_b) {
    if (!end_a || !end_b || piece < 1) return BPPO_ERR_ARG;
    const Key8 key = seed_key(seed);
    struct Ch { uint64_t pos; uint32_t r; std::vector<uint32_t> w; size_t off, left; } ch[2];
    ch[0].pos = pos_a; ch[1].pos = pos_b;
    auto refill = [&](Ch &c) {
        const uint64_t q = (c.pos / piece + 1) * piece;
        c.w.resize(q - c.pos);
        bppo_host::chacha12_words(key.k, stream, c.pos, c.w.data(), c.w.size());
        c.off = 0;
        c.left = c.w.size();
    };
    for (Ch &c : ch) { c.r = n; refill(c); }
    auto live = [](const Ch &c) { return c.r >= 2; };
    auto advance = [&](Ch &c, size_t u) {
        c.off += u; c.left -= u; c.pos += u;
        if (live(c) && c.left == 0) refill(c);
    };
    while (live(ch[0]) && live(ch[1])) {
        size_t u0 = 0, u1 = 0;
        bppo_host::chain_walk2_nj(ch[0].w.data() + ch[0].off, ch[0].left, &ch[0].r, &u0,
                                  ch[1].w.data() + ch[1].off, ch[1].left, &ch[1].r, &u1);
        advance(ch[0], u0);
        advance(ch[1], u1);
    }
    for (Ch &c : ch)
        while (live(c)) advance(c, bppo_host::chain_walk_nj(c.w.data() + c.off, c.left, &c.r));
    *end_a = ch[0].pos;
    *end_b = ch[1].pos;
    return BPPO_OK;
}

// the full shuffle engine (GPU-made words, speculative walks) for `jobs`
// consecutive updates of `epochs` shuffles of n, the first starting at word
// position start and each next one `gap` words after the previous update's last
// shuffle (the rollout's draws): J [jobs][epochs][n] as rebuilt in HBM, end
// positions [jobs][epochs], and per epoch the checkpoints the true walk needed
// before it met a speculative walk (-1: walked the whole epoch)
extern "C" bppo_status bppo_debug_shuffle_engine(uint64_t seed, uint64_t stream, uint64_t start, uint32_t n,
                                                 int32_t epochs, uint64_t gap, int32_t jobs, int32_t windows,
                                                 uint32_t *J, uint64_t *ends, int32_t *met) {
    if (!J || !ends || n < 2 || epochs < 1 || epochs > SHUF_MAX_EPOCHS || jobs < 1) return BPPO_ERR_ARG;
    ShuffleEngine *e = new ShuffleEngine();
    std::string err;
    bppo_status s = e->init(0, seed_key(seed), stream, n, epochs, gap, err, windows != 0);
    uint64_t pos = start;
    for (int j = 0; j < jobs && s == BPPO_OK; j++) {
        const int slot = e->ensure(pos);
        for (int k = 0; k < epochs; k++) e->wait_epoch(slot, k);
        const size_t o = (size_t)j * epochs;
        if (hipStreamSynchronize(e->copy) != hipSuccess ||
            hipMemcpy(J + o * n, e->d_J[slot], sizeof(uint32_t) * (size_t)n * epochs, hipMemcpyDeviceToHost) != hipSuccess)
            s = BPPO_ERR_HIP;
        for (int k = 0; k < epochs; k++) {
            ends[o + k] = e->end_pos[slot][k];
            if (met) met[o + k] = e->coalesced[slot][k];
        }
        pos = e->job_end(slot) + gap;
    }
    e->shutdown();
    delete e;
    return s;
}

extern "C" bppo_status bppo_debug_fisher_yates(int32_t device, const uint32_t *J, uint32_t n, uint32_t *perm) {
    if (!J || !perm) return BPPO_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return BPPO_ERR_HIP;
    uint32_t *dJ = nullptr, *dP = nullptr, *dS = nullptr, *dC = nullptr;
    FyRanges rg;
    bppo_status s = BPPO_ERR_HIP;
    if (hipMalloc((void **)&dJ, 4ull * n + 4) == hipSuccess && hipMalloc((void **)&dP, 4ull * n + 4) == hipSuccess &&
        hipMalloc((void **)&dS, 16ull * n + 16) == hipSuccess && hipMalloc((void **)&dC, 4ull * (n / 8192 + 2)) == hipSuccess &&
        hipMemcpy(dJ, J, 4ull * n, hipMemcpyHostToDevice) == hipSuccess &&
        fy_ranges_init(rg, n) == hipSuccess &&
        fisher_yates_device(dJ, n, dS, dC, dP, nullptr, &rg) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
        hipMemcpy(perm, dP, 4ull * n, hipMemcpyDeviceToHost) == hipSuccess)
        s = BPPO_OK;
    (void)hipFree(dJ); (void)hipFree(dP); (void)hipFree(dS); (void)hipFree(dC);
    fy_ranges_free(rg);
    return s;
}

// apply_action_mask + sample_categorical + log_prob_categorical (utils.rs:10-45,
// 96-135) on host rows through the device sampler the multi-player rollout uses
// (k_sample_masked): Gumbel words of StdRng(seed) stream `stream` from word_pos,
// row-major [row][action]; masks may be NULL (all valid)
extern "C" bppo_status bppo_debug_sample(int32_t A, int32_t B, const float *logits, const uint8_t *masks,
                                         uint64_t seed, uint64_t stream, uint64_t word_pos, int32_t *actions,
                                         float *log_probs) {
    if (!logits || !actions || B <= 0 || (A != 2 && A != 7 && A != 49)) return BPPO_ERR_ARG;
    const size_t nA = (size_t)B * A;
    float *d_l = nullptr, *d_v = nullptr, *d_lp = nullptr, *d_val = nullptr, *d_lv = nullptr;
    uint8_t *d_m = nullptr;
    int32_t *d_p = nullptr, *d_a = nullptr, *d_e = nullptr;
    bppo_status s = BPPO_ERR_HIP;
    std::vector<uint8_t> ones;
    if (!masks) { ones.assign(nA, 1); masks = ones.data(); }
    int32_t err = 0;
    if (hipMalloc((void **)&d_l, nA * 4) == hipSuccess && hipMalloc((void **)&d_m, nA) == hipSuccess &&
        hipMalloc((void **)&d_v, 4ull * B) == hipSuccess && hipMalloc((void **)&d_lp, 4ull * B) == hipSuccess &&
        hipMalloc((void **)&d_val, 4ull * B) == hipSuccess && hipMalloc((void **)&d_lv, 4ull * B) == hipSuccess &&
        hipMalloc((void **)&d_p, 4ull * B) == hipSuccess && hipMalloc((void **)&d_a, 4ull * B) == hipSuccess &&
        hipMalloc((void **)&d_e, 4) == hipSuccess && hipMemset(d_v, 0, 4ull * B) == hipSuccess &&
        hipMemset(d_p, 0, 4ull * B) == hipSuccess && hipMemset(d_e, 0, 4) == hipSuccess &&
        hipMemcpy(d_l, logits, nA * 4, hipMemcpyHostToDevice) == hipSuccess &&
        hipMemcpy(d_m, masks, nA, hipMemcpyHostToDevice) == hipSuccess) {
        SampleArgs g;
        g.N = B; g.P = 1; g.logits = d_l; g.values = d_v; g.mask = d_m; g.players = d_p;
        g.key = seed_key(seed); g.stream = stream; g.base = word_pos;
        g.act = d_a; g.logp = d_lp; g.val = d_val; g.lvpp = d_lv; g.err = d_e;
        if (wide_sample(A, nullptr, g) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
            hipMemcpy(actions, d_a, 4ull * B, hipMemcpyDeviceToHost) == hipSuccess &&
            (!log_probs || hipMemcpy(log_probs, d_lp, 4ull * B, hipMemcpyDeviceToHost) == hipSuccess) &&
            hipMemcpy(&err, d_e, 4, hipMemcpyDeviceToHost) == hipSuccess)
            s = (err & 2) ? BPPO_ERR_EMPTY_MASK : (err & 1) ? BPPO_ERR_NONFINITE : BPPO_OK;
    }
    void *ptrs[] = {d_l, d_m, d_v, d_lp, d_val, d_lv, d_p, d_a, d_e};
    for (void *q : ptrs) if (q) (void)hipFree(q);
    return s;
}

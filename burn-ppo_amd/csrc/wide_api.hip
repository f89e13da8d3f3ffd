// wide_api.hip — orchestration of the multi-player path (Connect Four,
// Liar's Dice; MLP or CTDE actor-critic) on one HIP stream:
//
//   collect_rollouts (ppo.rs:213-500): per step  observe -> actor/critic GEMMs
//     -> masked Gumbel sample -> env step, everything resident in HBM
//   bootstrap + compute_gae_multiplayer (main.rs:877-947, ppo.rs:1140-1264)
//   ppo_update minibatch (ppo.rs:1833-1984): gather -> forward GEMMs (saved
//     activations) -> masked loss -> backward GEMMs -> flat gradient
//
// The rollout row of step t / env e is [priv (G) | obs (D)], so the CTDE critic
// input cat[priv, obs] (ctde.rs:160-183) and the actor input obs are two views
// of one buffer with row stride L = G + D.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>
#include "bppo_internal.h"
#include "bppo_gemm.h"
#include "bppo_wide.h"

namespace bppo {

#define WHIP(c, expr)                                                       \
    do {                                                                    \
        hipError_t _e = (expr);                                             \
        if (_e != hipSuccess) return hip_fail((c), _e, #expr);              \
    } while (0)

template <class T>
static bppo_status walloc(bppo_ctx *c, T **p, size_t n) {
    *p = nullptr;
    if (n == 0) return BPPO_OK;
    WHIP(c, hipMalloc((void **)p, n * sizeof(T)));
    WHIP(c, hipMemsetAsync(*p, 0, n * sizeof(T), c->stream));
    return BPPO_OK;
}
#define WTRY(x)                                \
    do {                                       \
        bppo_status _s = (x);                  \
        if (_s != BPPO_OK) return _s;          \
    } while (0)

// fully connected hidden layers (their activations live in d_hbuf); CNN conv
// layers [0, n_conv) keep theirs in d_cnn_y (cnn.hip)
static bool is_hidden(const NetLayout &n, int l) {
    return (l >= n.n_conv && l < n.n_actor_hidden) || (n.ctde && l >= n.critic_fc0 && l < n.value);
}

bppo_status wide_init(bppo_ctx *c) {
    const bppo_config &cfg = c->cfg;
    if (cfg.ctde && cfg.env_kind != BPPO_ENV_LIARS_DICE && cfg.env_kind != BPPO_ENV_SKULL) {
        c->err = "CTDE needs privileged obs";
        return BPPO_ERR_ARG;
    }
    if (!cfg.ctde) c->G = 0;
    c->L = c->G + c->D;
    const NetLayout &n = c->net;
    const size_t TN = (size_t)c->T * c->N;
    const int mb_max = (int)(TN / cfg.num_minibatches + (TN % cfg.num_minibatches ? 1 : 0));
    c->rows_max = std::max(c->N, mb_max);
    size_t off = 0;
    int wmax = 0;
    for (int l = 0; l < n.n_layers; l++)
        if (is_hidden(n, l)) { c->hoff[l] = off; off += (size_t)c->rows_max * n.out[l]; wmax = std::max(wmax, n.out[l]); }
    WTRY(walloc(c, (char **)&c->d_wstate, (size_t)c->N * wide_state_bytes(cfg.env_kind)));
    WTRY(walloc(c, &c->d_xc, TN * c->L));
    WTRY(walloc(c, &c->d_mask, TN * c->A));
    WTRY(walloc(c, &c->d_players, TN));
    WTRY(walloc(c, &c->d_allr, TN * c->P));
    WTRY(walloc(c, &c->d_lvpp, (size_t)c->N * c->P));
    WTRY(walloc(c, &c->d_hbuf, off));
    WTRY(walloc(c, &c->d_logits, (size_t)c->rows_max * c->A));
    WTRY(walloc(c, &c->d_values, (size_t)c->rows_max));
    WTRY(walloc(c, &c->d_xcg, (size_t)mb_max * c->L));
    WTRY(walloc(c, &c->d_dout, (size_t)mb_max * (c->A + 1)));
    WTRY(walloc(c, &c->d_dz[0], (size_t)mb_max * wmax));
    WTRY(walloc(c, &c->d_dz[1], (size_t)mb_max * wmax));
    if (!n.ctde) {
        WTRY(walloc(c, &c->d_heads, (size_t)n.in[n.policy] * (c->A + 1)));
        WTRY(walloc(c, &c->d_heads_b, (size_t)(c->A + 1)));
    }
    // split-K scratch: the largest splits x Kin x N over the weight-gradient GEMMs
    size_t part = 0, cs = 0;
    for (int l = 0; l < n.n_layers; l++) {
        int N = n.out[l];
        if (!n.ctde && l == n.policy) N = c->A + 1;
        if (!n.ctde && l == n.value) continue;
        const int Kin = (!n.ctde && l == n.policy) ? n.in[l] : n.in[l];
        const int rows_l = n.is_conv(l) ? mb_max * n.H * n.W : mb_max;   // conv GEMMs: one row per position
        const int s = gemm_wg_splits(Kin, N, rows_l);
        part = std::max(part, (size_t)s * Kin * N);
        cs = std::max(cs, (size_t)s * N);
    }
    // sized for the f64 partials of the exact weight gradients (k_gemm_wg64)
    WTRY(walloc(c, &c->d_part, 2 * part));
    WTRY(walloc(c, &c->d_colsum, 2 * cs));
    WTRY(walloc(c, &c->d_mpart, (size_t)1024 * WM_COUNT));
    WTRY(walloc(c, &c->d_bxc, (size_t)c->N * c->L));
    WTRY(walloc(c, &c->d_bmask, (size_t)c->N * c->A));
    WTRY(walloc(c, &c->d_bplayers, (size_t)c->N));
    WTRY(walloc(c, &c->d_act_in, (size_t)c->N));
    WTRY(walloc(c, &c->d_scr_r, (size_t)c->N * c->P));
    WTRY(walloc(c, &c->d_scr_d, (size_t)c->N));
    if (n.n_conv) WTRY(cnn_alloc(c));
    if (cfg.normalize_obs) {
        WTRY(walloc(c, &c->d_obs_raw, TN * c->D));
        c->obsw_part_n = (size_t)256 * c->D * 3;
        WTRY(walloc(c, &c->d_obsw_part, c->obsw_part_n));
    }
    return BPPO_OK;
}

void wide_free(bppo_ctx *c) {
    void *ptrs[] = {c->d_wstate, c->d_xc, c->d_mask, c->d_players, c->d_allr, c->d_lvpp, c->d_hbuf,
                    c->d_logits, c->d_values, c->d_xcg, c->d_dout, c->d_dz[0], c->d_dz[1], c->d_heads,
                    c->d_heads_b, c->d_part, c->d_colsum, c->d_mpart, c->d_bxc, c->d_bmask, c->d_bplayers,
                    c->d_act_in, c->d_scr_r, c->d_scr_d, c->d_obs_raw, c->d_obsw_part};
    for (void *p : ptrs) if (p) (void)hipFree(p);
    cnn_free(c);
    opp_free(c);
}

bppo_status wide_reset(bppo_ctx *c) {
    WHIP(c, wide_env_reset(c->cfg.env_kind, c->stream, c->N, c->cfg.env_seed_base, c->Pa, c->d_wstate, c->d_env_pos,
                           c->d_ep_ret, c->d_ep_len));
    return BPPO_OK;
}

// shared-trunk heads packed as one [W][A+1] GEMM operand (after every params change)
bppo_status wide_pack(bppo_ctx *c) {
    const NetLayout &n = c->net;
    if (n.n_conv) WTRY(cnn_pack(c, c->d_params, c->d_cnn_wt, c->d_cnn_wd));
    if (n.ctde) return BPPO_OK;
    WHIP(c, wide_pack_heads(c->stream, c->d_params, n.in[n.policy], c->A, n.w[n.policy], n.b[n.policy],
                            n.w[n.value], n.b[n.value], c->d_heads, c->d_heads_b));
    return BPPO_OK;
}

// forward (mlp.rs:140-206 / ctde.rs:132-183) of `rows` rows [priv | obs] (ld ldxc);
// hidden activations stay in d_hbuf for the backward
bppo_status wide_forward(bppo_ctx *c, int rows, const float *xc, int ldxc, float *logits, float *values, int split) {
    const NetLayout &n = c->net;
    const float *P = c->d_params;
    const float *x = xc + c->G;
    int ldx = ldxc;
    if (n.n_conv) {                                  // CNN trunk (cnn.rs:241-330) -> features [rows][fdim]
        WTRY(cnn_features(c, 0, rows, x, ldx, P, c->d_cnn_wt));
        x = c->d_cnn_f[0]; ldx = n.fdim;
    }
    for (int l = n.n_conv; l < n.n_actor_hidden; l++) {
        float *h = c->d_hbuf + c->hoff[l];
        WHIP(c, gemm_fwd(c->stream, rows, n.out[l], n.in[l], x, ldx, P + n.w[l], n.out[l], P + n.b[l], c->cfg.relu ? 1 : 2, h,
                         n.out[l], n.out[l], nullptr, 0, split));
        x = h; ldx = n.out[l];
    }
    const int K = n.in[n.policy];
    if (!n.ctde) {
        WHIP(c, gemm_fwd(c->stream, rows, c->A + 1, K, x, ldx, c->d_heads, c->A + 1, c->d_heads_b, 0, logits, c->A,
                         c->A, values, 1, split));
        return BPPO_OK;
    }
    WHIP(c, gemm_fwd(c->stream, rows, c->A, K, x, ldx, P + n.w[n.policy], c->A, P + n.b[n.policy], 0, logits,
                     c->A, c->A, nullptr, 0, split));
    const float *xq = xc;
    int ldq = ldxc;
    if (n.n_conv) {                                  // split CNN critic: its own conv stack (cnn.rs:284-296)
        WTRY(cnn_features(c, 1, rows, xc + c->G, ldxc, P, c->d_cnn_wt));
        xq = c->d_cnn_f[1]; ldq = n.fdim;
    }
    for (int l = n.critic_fc0; l < n.value; l++) {
        float *h = c->d_hbuf + c->hoff[l];
        WHIP(c, gemm_fwd(c->stream, rows, n.out[l], n.in[l], xq, ldq, P + n.w[l], n.out[l], P + n.b[l], c->cfg.relu ? 1 : 2, h,
                         n.out[l], n.out[l], nullptr, 0, split));
        xq = h; ldq = n.out[l];
    }
    WHIP(c, gemm_fwd(c->stream, rows, 1, n.in[n.value], xq, ldq, P + n.w[n.value], 1, P + n.b[n.value], 0, values,
                     1, 1, nullptr, 0, split));
    return BPPO_OK;
}

// actor logits only, with caller-given parameters (an opponent model,
// ppo.rs:827-843: forward_actor for CTDE, the shared trunk + policy head for MLP)
bppo_status wide_forward_actor(bppo_ctx *c, int rows, const float *xc, int ldxc, const float *P, float *logits) {
    const NetLayout &n = c->net;
    const float *x = xc + c->G;
    int ldx = ldxc;
    if (n.n_conv) {
        WTRY(cnn_pack(c, P, c->d_cnn_owt, nullptr));
        WTRY(cnn_features(c, 0, rows, x, ldx, P, c->d_cnn_owt));
        x = c->d_cnn_f[0]; ldx = n.fdim;
    }
    for (int l = n.n_conv; l < n.n_actor_hidden; l++) {
        float *h = c->d_hbuf + c->hoff[l];
        WHIP(c, gemm_fwd(c->stream, rows, n.out[l], n.in[l], x, ldx, P + n.w[l], n.out[l], P + n.b[l],
                         c->cfg.relu ? 1 : 2, h, n.out[l], n.out[l], nullptr, 0));
        x = h; ldx = n.out[l];
    }
    WHIP(c, gemm_fwd(c->stream, rows, c->A, n.in[n.policy], x, ldx, P + n.w[n.policy], c->A, P + n.b[n.policy], 0,
                     logits, c->A, c->A, nullptr, 0));
    return BPPO_OK;
}

// collect_rollouts (ppo.rs:213-500), self-play path; with an opponent pool
// (opponents.hip) collect_rollouts_with_opponents (ppo.rs:537-1063).  Observation normalizer:
// each step's obs columns normalized in place with the lagged stats (raw copy
// kept, stats updated after the rollout); return normalizer: the env writes
// the raw acting rewards, launch_return_norm normalizes them after the rollout
bppo_status wide_collect(bppo_ctx *c, uint64_t base) {
    const int N = c->N, A = c->A, P = c->P, L = c->L;
    const bool opp = opp_active(c);
    WHIP(c, hipMemsetAsync(c->d_lvpp, 0, sizeof(float) * (size_t)N * P, c->stream));
    if (opp) WTRY(opp_rollout_begin(c, base));
    for (int t = 0; t < c->T; t++) {
        const size_t r0 = (size_t)t * N;
        float *xc = c->d_xc + r0 * L;
        WHIP(c, wide_env_observe(c->cfg.env_kind, c->G > 0, c->stream, N, c->d_wstate, xc, c->d_mask + r0 * A,
                                 c->d_players + r0));
        if (opp) WTRY(opp_step_group(c, t));
        if (c->cfg.normalize_obs) WTRY(launch_obs_norm_rows(c, N, xc + c->G, L, c->d_obs_raw + r0 * c->D));
        WTRY(wide_forward(c, N, xc, L, c->d_logits, c->d_values));
        if (opp) WTRY(opp_step_forwards(c));
        SampleArgs s;
        s.N = N; s.P = P; s.logits = c->d_logits; s.values = c->d_values; s.mask = c->d_mask + r0 * A;
        s.players = c->d_players + r0; s.key = c->rng_key; s.stream = c->cfg.rng_stream;
        s.base = base + r0 * (uint64_t)A;
        s.act = c->d_act + r0; s.logp = c->d_logp + r0; s.val = c->d_val + r0; s.lvpp = c->d_lvpp; s.err = c->d_err;
        if (opp) { s.group = c->d_group; s.gpos = c->d_gpos; s.dbase = c->d_rngpos; }
        if (c->cfg.normalize_values && c->pa_count >= 2.0) { s.pa_on = 1; s.pa_mean = c->pa_mean; s.pa_std = popart_std(c); }
        WHIP(c, wide_sample(A, c->stream, s));
        WideStepArgs w;
        w.N = N; w.t = t; w.state = c->d_wstate; w.env_pos = c->d_env_pos; w.seed_base = c->cfg.env_seed_base;
        w.actions = c->d_act + r0; w.shaping = shaping_coef(c);
        w.all_r = c->d_allr + r0 * P; w.rew_act = (c->cfg.normalize_returns ? c->d_rew_raw : c->d_rew) + r0; w.done_f = c->d_done + r0; w.done_u8 = nullptr;
        w.ep_ret = c->d_ep_ret; w.ep_len = c->d_ep_len; w.eps = c->d_eps; w.ep_count = c->d_ep_count;
        w.eps_cap = c->eps_cap; w.err = c->d_err;
        WHIP(c, wide_env_step(c->cfg.env_kind, c->stream, w));
        if (opp) WTRY(opp_step_seats(c, t));
    }
    return BPPO_OK;
}

// main.rs:877-947: bootstrap value of the post-rollout state for the player to
// move, then compute_gae_multiplayer
bppo_status wide_bootstrap_gae(bppo_ctx *c) {
    const int N = c->N;
    WHIP(c, wide_env_observe(c->cfg.env_kind, c->G > 0, c->stream, N, c->d_wstate, c->d_bxc, c->d_bmask, c->d_bplayers));
    if (c->cfg.normalize_obs) WTRY(launch_obs_norm_rows(c, N, c->d_bxc + c->G, c->L, nullptr));   // updated stats
    WTRY(wide_forward(c, N, c->d_bxc, c->L, c->d_logits, c->d_values));
    WTRY(popart_denorm(c, c->d_values, (size_t)N));    // main.rs:898-907
    WHIP(c, wide_boot_lvpp(c->stream, N, c->P, c->d_values, c->d_bplayers, c->d_lvpp));
    WHIP(c, hipMemcpyAsync(c->d_last_v, c->d_values, sizeof(float) * N, hipMemcpyDeviceToDevice, c->stream));
    hipError_t he = hipSuccess;
    if (c->P == 1) {   // CartPole on this path: main.rs:928-946 dispatches single-player to compute_gae
        bppo_status s1 = launch_gae_1p(c->d_rew, c->d_done, c->d_val, c->d_last_v, c->T, N, (float)c->cfg.gamma,
                                       (float)c->cfg.gae_lambda, c->d_adv, c->d_ret, c->stream, nullptr, nullptr, &he);
        if (s1 != BPPO_OK) return he != hipSuccess ? hip_fail(c, he, "k_gae_1p launch") : s1;
        return s1;
    }
    bppo_status s = launch_gae_mp(c->d_allr, c->d_players, c->d_done, c->d_val, c->d_lvpp, c->T, N, c->P,
                                  (float)c->cfg.gamma, (float)c->cfg.gae_lambda, c->d_adv, c->d_ret, c->stream, &he);
    if (s != BPPO_OK) {
        if (he != hipSuccess) return hip_fail(c, he, "k_gae_mp launch");
        c->err = "multiplayer GAE: unsupported player count";
    }
    return s;
}

// one minibatch of ppo_update: gather, forward, loss, backward -> d_grad[0, np),
// metrics -> d_grad[np, np + WM_COUNT)
bppo_status wide_minibatch(bppo_ctx *c, uint32_t start, uint32_t mb, double ent_coef, bool first) {
    const NetLayout &n = c->net;
    const int hact = c->cfg.relu ? 1 : 2;   // hidden activation derivative in the DX epilogues
    const int A = c->A, L = c->L, rows = (int)mb;
    const float *P = c->d_params;
    float *G = c->d_grad;
    // the split-bf16 contraction (k_gemm_split) for the MLP GEMMs of every minibatch after the
    // update's first (mode 0) or of all of them (bppo_set_minibatch_kernel 2); the first keeps
    // the exact forward chains (ratio exactly 1) -- as the CfgB update's k_minibatch_split --
    // and runs its backward split like the others (`bsplit` below).  Mode 0
    // splits only minibatches of WIDE_SPLIT_MIN_ROWS rows or more: below that the GEMMs are
    // launch- and latency-bound (no time to win), while the split forward's last-bit
    // differences -- a ReLU pre-activation that close to zero switches its unit for that row
    // -- are amplified by Adam over many tiny minibatches (a 72-row Liar's Dice CTDE update
    // drifts 1e-3 from the oracle by minibatch 3 with the split, 0 with the exact chains:
    // profiles/r05c/popart_split_probe.log)
    static const bool exact_all = getenv("BPPO_MB_EXACT_ALL") != nullptr;
    const bool big = rows >= WIDE_SPLIT_MIN_ROWS;
    const int split = n.n_conv == 0 && (c->mb_kernel == 2 || (c->mb_kernel == 0 && !first && !exact_all && big)) ? 1 : 0;
    // the backward (input and weight gradients) needs f32 accuracy only -- the ratio is
    // the forward's -- so the update's first minibatch runs its backward split too
    const int bsplit = n.n_conv == 0 && (c->mb_kernel == 2 || (c->mb_kernel == 0 && !exact_all && big)) ? 1 : 0;
    // weight-gradient sums: f64 (or row-ordered, mode 1) for the small minibatches; from
    // WIDE_SPLIT_MIN_ROWS rows the f32 split-K chains (the update's first minibatch, and the
    // CNN's) -- the f64 MFMA runs them ~4x slower (CfgC 142 -> 151 ms per update, CfgD 482 ->
    // 517 ms, profiles/r05c/r05t_wide_*.log) and the minibatches after the first run the
    // split-bf16 contraction anyway
    const int exact = bsplit ? -1 : (big && c->mb_kernel == 0 ? 0 : wide_exact_grad(c));
    WHIP(c, wide_gather(c->stream, c->d_perm, start, mb, c->d_xc, L, c->d_xcg));
    WTRY(wide_forward(c, rows, c->d_xcg, L, c->d_logits, c->d_values, split));
    LossArgs g;
    g.perm = c->d_perm; g.start = start; g.n = mb; g.act = c->d_act; g.logp = c->d_logp; g.adv = c->d_adv;
    g.ret = c->u_ret; g.val = c->u_val; g.mask = c->d_mask; g.logits = c->d_logits; g.values = c->d_values;
    g.mb_stats = c->d_mb_cur; g.dout = c->d_dout; g.part = c->d_mpart;
    g.lo = (float)(1.0 - c->cfg.clip_epsilon); g.hi = (float)(1.0 + c->cfg.clip_epsilon);
    g.ceps = (float)c->cfg.clip_epsilon; g.inv_mb = (float)(1.0 / (double)mb); g.ent_coef = (float)ent_coef;
    g.value_coef = (float)c->cfg.value_coef; g.clip_value = c->cfg.clip_value;
    g.inv_mb_d = 1.0 / (double)mb; g.ent_coef_d = ent_coef; g.value_coef_d = c->cfg.value_coef;
    const int blocks = std::max(1, std::min(1024, (int)((mb + 255) / 256)));
    WHIP(c, wide_loss(A, c->stream, g, blocks, G + n.n_params));
    float *dz = c->d_dz[0], *dz2 = c->d_dz[1];
    auto wgrad = [&](int Kin, int N, const float *X, int ldx, const float *dZ, int ldz, float *dW0, int ldw0,
                     int n0, float *dW1, int ldw1, float *db0, float *db1) -> bppo_status {
        const int sp = gemm_wg_splits(Kin, N, rows);
        WHIP(c, gemm_wgrad(c->stream, Kin, N, rows, X, ldx, dZ, ldz, c->d_part, c->d_colsum, dW0, ldw0, n0, dW1,
                           ldw1, db0, db1, sp, exact));
        return BPPO_OK;
    };
    // walk hidden layers [first, last] down, dz holds dL/dz of layer `last`

    auto hidden_chain = [&](int first, int last, const float *x0, int ldx0) -> bppo_status {
        for (int l = last; l >= first; l--) {
            const float *X = l > first ? c->d_hbuf + c->hoff[l - 1] : x0;
            const int ldx = l > first ? n.out[l - 1] : ldx0;
            WTRY(wgrad(n.in[l], n.out[l], X, ldx, dz, n.out[l], G + n.w[l], n.out[l], n.out[l], nullptr, 0,
                       G + n.b[l], nullptr));
            if (l > first) {
                WHIP(c, gemm_dx(c->stream, rows, n.in[l], n.out[l], dz, n.out[l], P + n.w[l], n.out[l],
                                c->d_hbuf + c->hoff[l - 1], n.out[l - 1], hact, dz2, n.in[l], nullptr, 0, nullptr,
                                bsplit));
                std::swap(dz, dz2);
            }
        }
        return BPPO_OK;
    };
    // CNN stack s: FC layers [f0, last] down to the features, dF = dz W^T * [F > 0] (the
    // conv part of F is relu output), then the conv stack
    auto cnn_trunk_backward = [&](int s, int f0, int last) -> bppo_status {
        WTRY(hidden_chain(f0, last, c->d_cnn_f[s], n.fdim));
        float *dF = c->d_cnn_dy[0];
        WHIP(c, gemm_dx(c->stream, rows, n.fdim, n.out[f0], dz, n.out[f0], P + n.w[f0], n.out[f0], c->d_cnn_f[s],
                        n.fdim, 1, dF, n.fdim));
        return cnn_backward(c, s, rows, c->d_xcg + c->G, L, dF, G, exact);
    };
    const int la = n.n_actor_hidden - 1;
    const float *Ha = c->d_hbuf + c->hoff[la];
    const int Wa = n.out[la];
    if (!n.ctde) {
        // heads: dW = H^T [dlogits | dv] split into policy / value tensors
        WTRY(wgrad(Wa, A + 1, Ha, Wa, c->d_dout, A + 1, G + n.w[n.policy], A, A, G + n.w[n.value], 1,
                   G + n.b[n.policy], G + n.b[n.value]));
        // the trunk's input gradient: the policy head's chain over its A outputs, then the value
        // head's product added as its own rounded term (the two heads are two Linear modules)
        WHIP(c, gemm_dx(c->stream, rows, Wa, A, c->d_dout, A + 1, c->d_heads, A + 1, Ha, Wa, hact, dz, Wa,
                        c->d_dout + A, A + 1, P + n.w[n.value], bsplit));
        if (!n.n_conv) {
            WTRY(hidden_chain(0, la, c->d_xcg + c->G, L));
            return BPPO_OK;
        }
        // CNN: FC layers down to the features, dF = dz W^T * [F > 0] (the conv
        // part of F is relu output), then the conv stack
        WTRY(cnn_trunk_backward(0, n.n_conv, la));
        return BPPO_OK;
    }
    // CTDE actor
    WTRY(wgrad(Wa, A, Ha, Wa, c->d_dout, A + 1, G + n.w[n.policy], A, A, nullptr, 0, G + n.b[n.policy], nullptr));
    WHIP(c, gemm_dx(c->stream, rows, Wa, A, c->d_dout, A + 1, P + n.w[n.policy], A, Ha, Wa, hact, dz, Wa, nullptr, 0,
                    nullptr, bsplit));
    if (n.n_conv) WTRY(cnn_trunk_backward(0, n.n_conv, la));   // split CNN actor
    else WTRY(hidden_chain(0, la, c->d_xcg + c->G, L));
    // CTDE critic
    const int lc = n.value - 1;
    const float *Hc = c->d_hbuf + c->hoff[lc];
    const int Wc = n.out[lc];
    dz = c->d_dz[0]; dz2 = c->d_dz[1];
    WTRY(wgrad(Wc, 1, Hc, Wc, c->d_dout + A, A + 1, G + n.w[n.value], 1, 1, nullptr, 0, G + n.b[n.value], nullptr));
    WHIP(c, gemm_dx(c->stream, rows, Wc, 1, c->d_dout + A, A + 1, P + n.w[n.value], 1, Hc, Wc, hact, dz, Wc, nullptr,
                    0, nullptr, bsplit));
    if (n.n_conv) return cnn_trunk_backward(1, n.critic_fc0, lc);   // split CNN critic
    WTRY(hidden_chain(n.critic_first, lc, c->d_xcg, L));
    return BPPO_OK;
}

// ---------------------------------------------------------- host surfaces --
// VecEnv::get_observations / get_current_players / get_action_masks / get_privileged_obs
bppo_status wide_observe_host(bppo_ctx *c, float *obs, int32_t *players, uint8_t *masks, float *priv) {
    const int N = c->N, L = c->L;
    WHIP(c, wide_env_observe(c->cfg.env_kind, c->G > 0, c->stream, N, c->d_wstate, c->d_bxc, c->d_bmask, c->d_bplayers));
    std::vector<float> rows((size_t)N * L);
    WHIP(c, hipMemcpyAsync(rows.data(), c->d_bxc, rows.size() * 4, hipMemcpyDeviceToHost, c->stream));
    if (players) WHIP(c, hipMemcpyAsync(players, c->d_bplayers, 4 * (size_t)N, hipMemcpyDeviceToHost, c->stream));
    if (masks) WHIP(c, hipMemcpyAsync(masks, c->d_bmask, (size_t)N * c->A, hipMemcpyDeviceToHost, c->stream));
    WHIP(c, hipStreamSynchronize(c->stream));
    for (int e = 0; e < N; e++) {
        if (obs) std::memcpy(obs + (size_t)e * c->D, rows.data() + (size_t)e * L + c->G, 4 * (size_t)c->D);
        if (priv && c->G) std::memcpy(priv + (size_t)e * c->G, rows.data() + (size_t)e * L, 4 * (size_t)c->G);
    }
    return BPPO_OK;
}

bppo_status wide_step_host(bppo_ctx *c, const int32_t *actions, float *obs, float *rewards, uint8_t *dones,
                           int32_t *n_eps) {
    const int N = c->N, P = c->P;
    WHIP(c, hipMemcpyAsync(c->d_act_in, actions, 4 * (size_t)N, hipMemcpyHostToDevice, c->stream));
    WHIP(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
    WideStepArgs w;
    w.N = N; w.t = 0; w.state = c->d_wstate; w.env_pos = c->d_env_pos; w.seed_base = c->cfg.env_seed_base;
    w.actions = c->d_act_in; w.shaping = shaping_coef(c);
    w.all_r = c->d_scr_r; w.rew_act = nullptr; w.done_f = nullptr; w.done_u8 = c->d_scr_d;
    w.ep_ret = c->d_ep_ret; w.ep_len = c->d_ep_len; w.eps = c->d_eps; w.ep_count = c->d_ep_count;
    w.eps_cap = c->eps_cap; w.err = c->d_err;
    WHIP(c, wide_env_step(c->cfg.env_kind, c->stream, w));
    if (rewards) WHIP(c, hipMemcpyAsync(rewards, c->d_scr_r, 4 * (size_t)N * P, hipMemcpyDeviceToHost, c->stream));
    if (dones) WHIP(c, hipMemcpyAsync(dones, c->d_scr_d, (size_t)N, hipMemcpyDeviceToHost, c->stream));
    int32_t cnt = 0, err = 0;
    WHIP(c, hipMemcpyAsync(&cnt, c->d_ep_count, 4, hipMemcpyDeviceToHost, c->stream));
    WHIP(c, hipMemcpyAsync(&err, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    WHIP(c, hipStreamSynchronize(c->stream));
    if (n_eps) *n_eps = cnt;
    if (err & 8) { c->err = "Invalid action: outside the env's action mask"; return BPPO_ERR_ARG; }   // skull.rs:1116-1128
    if (obs) WTRY(wide_observe_host(c, obs, nullptr, nullptr, nullptr));
    return BPPO_OK;
}

// ActorCriticNetwork::forward on host rows (obs [B][D], priv [B][G] for CTDE)
bppo_status wide_forward_host(bppo_ctx *c, const float *obs, const float *priv, int B, float *logits,
                              float *values) {
    if (c->G && !priv) { c->err = "CTDE forward needs privileged obs"; return BPPO_ERR_ARG; }
    const int L = c->L, chunk = c->rows_max;
    std::vector<float> rows((size_t)std::min(B, chunk) * L);
    float *d_rows = nullptr;
    WHIP(c, hipMalloc((void **)&d_rows, rows.size() * 4));
    bppo_status st = BPPO_OK;
    for (int r0 = 0; r0 < B && st == BPPO_OK; r0 += chunk) {
        const int nr = std::min(chunk, B - r0);
        for (int r = 0; r < nr; r++) {
            if (c->G) std::memcpy(rows.data() + (size_t)r * L, priv + (size_t)(r0 + r) * c->G, 4 * (size_t)c->G);
            std::memcpy(rows.data() + (size_t)r * L + c->G, obs + (size_t)(r0 + r) * c->D, 4 * (size_t)c->D);
        }
        if (hipMemcpyAsync(d_rows, rows.data(), (size_t)nr * L * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess) {
            st = BPPO_ERR_HIP; break;
        }
        st = wide_forward(c, nr, d_rows, L, c->d_logits, c->d_values);
        if (st != BPPO_OK) break;
        if (logits && hipMemcpyAsync(logits + (size_t)r0 * c->A, c->d_logits, (size_t)nr * c->A * 4,
                                     hipMemcpyDeviceToHost, c->stream) != hipSuccess) { st = BPPO_ERR_HIP; break; }
        if (values && hipMemcpyAsync(values + r0, c->d_values, (size_t)nr * 4, hipMemcpyDeviceToHost,
                                     c->stream) != hipSuccess) { st = BPPO_ERR_HIP; break; }
        if (hipStreamSynchronize(c->stream) != hipSuccess) { st = BPPO_ERR_HIP; break; }
    }
    (void)hipFree(d_rows);
    if (st == BPPO_ERR_HIP && c->err.empty()) c->err = "wide forward: HIP failure";
    return st;
}

// RolloutBuffer exports of the wide layout: obs/priv are column views of the
// [priv | obs] rows, masks are stored u8 and exported as the reference's f32 0/1
bppo_status wide_buffer_get(bppo_ctx *c, const char *name, void *host, size_t bytes, bool *handled) {
    const size_t TN = (size_t)c->T * c->N;
    *handled = true;
    auto need = [&](size_t b) -> bool {
        if (bytes < b) { c->err = std::string("buffer_get: too small: ") + name; return false; }
        return true;
    };
    if (!strcmp(name, "obs") || !strcmp(name, "priv")) {
        const bool is_obs = !strcmp(name, "obs");
        const int w = is_obs ? c->D : c->G, off = is_obs ? c->G : 0;
        if (w == 0) { c->err = "buffer_get: no privileged obs"; return BPPO_ERR_ARG; }
        if (!need(TN * w * 4)) return BPPO_ERR_ARG;
        std::vector<float> rows(TN * c->L);
        WHIP(c, hipMemcpyAsync(rows.data(), c->d_xc, rows.size() * 4, hipMemcpyDeviceToHost, c->stream));
        WHIP(c, hipStreamSynchronize(c->stream));
        float *o = (float *)host;
        for (size_t r = 0; r < TN; r++) std::memcpy(o + r * w, rows.data() + r * c->L + off, 4 * (size_t)w);
        return BPPO_OK;
    }
    if (!strcmp(name, "masks")) {
        if (!need(TN * c->A * 4)) return BPPO_ERR_ARG;
        std::vector<uint8_t> m(TN * c->A);
        WHIP(c, hipMemcpyAsync(m.data(), c->d_mask, m.size(), hipMemcpyDeviceToHost, c->stream));
        WHIP(c, hipStreamSynchronize(c->stream));
        float *o = (float *)host;
        for (size_t i = 0; i < m.size(); i++) o[i] = m[i] ? 1.0f : 0.0f;
        return BPPO_OK;
    }
    if (!strncmp(name, "hidden:", 7)) {
        // test hook: hidden layer l's activations of the last forward -- the last minibatch's
        // rows in gather (perm) order, [rows_max][out[l]] (tests/test_gpu_gemm_split.py reads
        // the device's ReLU decisions from them)
        const int l = atoi(name + 7);
        if (l < 0 || l >= c->net.n_layers || !is_hidden(c->net, l)) { c->err = "buffer_get: not a hidden layer"; return BPPO_ERR_ARG; }
        const size_t b = (size_t)c->rows_max * c->net.out[l] * 4;
        if (!need(b)) return BPPO_ERR_ARG;
        WHIP(c, hipMemcpyAsync(host, c->d_hbuf + c->hoff[l], b, hipMemcpyDeviceToHost, c->stream));
        WHIP(c, hipStreamSynchronize(c->stream));
        return BPPO_OK;
    }
    struct { const char *n; const void *p; size_t b; } tab[] = {
        {"players", c->d_players, TN * 4},
        {"all_rewards", c->d_allr, TN * c->P * 4},
        {"last_v_pp", c->d_lvpp, (size_t)c->N * c->P * 4},
    };
    for (auto &t : tab)
        if (!strcmp(name, t.n)) {
            if (!need(t.b)) return BPPO_ERR_ARG;
            WHIP(c, hipMemcpyAsync(host, t.p, t.b, hipMemcpyDeviceToHost, c->stream));
            WHIP(c, hipStreamSynchronize(c->stream));
            return BPPO_OK;
        }
    *handled = false;
    return BPPO_OK;
}

}  // namespace bppo

// bppo_wide.h — argument blocks and launchers of the multi-player path
// (k_wide.hip) and its orchestration (wide_api.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "bppo_device.h"

namespace bppo {

struct EpisodeRec;

struct WideStepArgs {
    int N, t;
    void *state;
    uint64_t *env_pos;
    uint64_t seed_base;
    const int32_t *actions;
    float shaping;
    float *all_r;        // [N][P] (may be null)
    float *rew_act;      // [N] reward of the acting player (may be null)
    float *done_f;       // [N] (may be null)
    uint8_t *done_u8;    // [N] (may be null)
    float *ep_ret;       // [N][P]
    int32_t *ep_len;
    EpisodeRec *eps;
    int32_t *ep_count;
    int eps_cap;
    int32_t *err;        // bit 3: an action outside the env's mask (Skull panics, skull.rs:1113-1128)
};

struct SampleArgs {
    int N, P;
    const float *logits, *values;
    const uint8_t *mask;
    const int32_t *players;
    Key8 key;
    uint64_t stream, base;
    int32_t *act;
    float *logp, *val, *lvpp;
    int32_t *err;        // bit 0: non-finite log-prob, bit 1: empty mask
    // opponent pool: row group (0 learner, 1 + model) and its position in the
    // step's draw order; the step's first word position from device memory
    const int32_t *group = nullptr, *gpos = nullptr;
    const uint64_t *dbase = nullptr;
    // PopArt (ppo.rs:355-359): stored values denormalized, v * std + mean in f64
    int pa_on = 0;
    double pa_mean = 0.0, pa_std = 1.0;
};

// metric slots written after the gradient (d_grad[np + k]); the first 11 are
// shared with the CartPole kernel (k_update.hip M_*)
enum { WM_PL = 0, WM_VL, WM_H, WM_KL, WM_CF, WM_V, WM_R, WM_VE, WM_VE2, WM_VEMAX, WM_N, WM_VALID, WM_HV,
       WM_NCHOICE, WM_COUNT };

struct LossArgs {
    const uint32_t *perm;
    uint32_t start, n;
    const int32_t *act;
    const float *logp, *adv, *ret, *val;
    const uint8_t *mask;
    const float *logits, *values;   // minibatch forward [n][A], [n]
    const float *mb_stats;
    float *dout;                    // [n][A+1]
    double *part;                   // [blocks][WM_COUNT]
    float lo, hi, ceps, inv_mb, ent_coef, value_coef;
    // the gradient of the loss in f64, rounded once (the oracle's hand-written autodiff:
    // inv = 1 / mb, entropy / value coefficients as the config's f64 values)
    double inv_mb_d, ent_coef_d, value_coef_d;
    int clip_value;
};

// players: Skull's num_players (new_with_players, main.rs:2008-2014)
hipError_t wide_env_reset(int kind, hipStream_t st, int N, uint64_t seed_base, int players, void *state,
                          uint64_t *env_pos, float *ep_ret, int32_t *ep_len);
// rows [priv | obs] when with_priv (CTDE), [obs] otherwise
hipError_t wide_env_observe(int kind, int with_priv, hipStream_t st, int N, const void *state, float *xc,
                            uint8_t *mask, int32_t *players);
hipError_t wide_env_step(int kind, hipStream_t st, const WideStepArgs &a);
hipError_t wide_sample(int A, hipStream_t st, const SampleArgs &g);
hipError_t wide_boot_lvpp(hipStream_t st, int N, int P, const float *values, const int32_t *players, float *lvpp);
hipError_t wide_gather(hipStream_t st, const uint32_t *perm, uint32_t start, uint32_t n, const float *src, int L,
                       float *dst);
hipError_t wide_pack_heads(hipStream_t st, const float *params, int K, int A, size_t wp, size_t bp, size_t wv,
                           size_t bv, float *W, float *b);
hipError_t wide_loss(int A, hipStream_t st, const LossArgs &g, int blocks, float *metrics_out);
size_t wide_state_bytes(int kind);

}  // namespace bppo

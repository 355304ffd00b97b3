// snk_dqn.hpp — DQNModel handle internals shared by snk_dqn.hip / snk_trainer.hip
#pragma once
#include "snk_qnet.hpp"

namespace snk {
struct DeepNet;   // the configs[2] bf16 net (snk_deep.hip)
}

struct snk_dqn_s {
    snk::QLayout L{};
    float lr = 5e-4f, rho = 0.9f, eps = 1e-8f;
    float *theta_q = nullptr, *theta_t = nullptr, *acc = nullptr, *grad = nullptr, *tmp = nullptr;
    float *wt_q = nullptr, *wt_t = nullptr;   // forward weight images of q_net / t_net
    uint16_t *wtb_q = nullptr, *wtb_t = nullptr;   // their exact bf16 split planes (x6 forward); null = fp32 MFMA
    int32_t *perm = nullptr;        // packed index -> Flux.destructure index
    snk::QWork act, tgt, trn;       // workspaces: acting (n_envs), target net, training batch
    float *slab = nullptr;
    int64_t slab_cap = 0;
    int64_t slab_gen = 0;           // bumped on every slab reallocation
    double *loss_dev = nullptr;
    uint8_t *meta = nullptr;
    int64_t meta_cap = 0;
    // per-sample Jacobian / Gram workspace (snk_laplace.hip)
    snk::QWork jw;
    float *jbuf = nullptr;
    int64_t jbuf_floats = 0, jn_cap = 0;
    uint16_t *jplanes = nullptr;    // h3 Gram: jbuf rows as scaled fp16 parts [n][ldh/32][h 32 | l 32]
    int32_t *jexp = nullptr;        //   and their per-row power-of-two exponents
    int64_t jplanes_halves = 0, jexp_cap = 0;
    uint16_t *dplanes = nullptr;    // the Dense-section Gram operands a3 | dz1 | h1 as h3 segments
    int32_t *dexp = nullptr;        //   (h3_seg_rows_kernel) and their exponents [3][dexp_cap]
    int64_t dplanes_halves = 0, dexp_cap = 0;
    float *gpart = nullptr;         // the K-split Gram's fp32 partial tiles (syrk_h3k_kernel)
    int64_t gpart_floats = 0;
    int64_t *jidx = nullptr;
    uint8_t *jact = nullptr;
    // snk_dqn_create_deep: the deeper bf16 net; L then holds its head offsets and P only
    snk::DeepNet *deep = nullptr;
};

namespace snk {
const EnvDev &env_dev(snk_env h);
const ReplayDev &replay_dev(snk_replay h);
int32_t replay_batch(snk_replay h);
void replay_launch_sample(const ReplayDev &d, int32_t batch, uint64_t seed, uint64_t draw,
                          const int64_t *draw_dev, int64_t *idx, int32_t *b_dev, hipStream_t s,
                          int64_t pending = 0);
BoardSrc src_env(const EnvDev &E);
BoardSrc src_replay(const ReplayDev &R, const int64_t *idx, int chan0);
BoardSrc src_float(const QLayout &L, const float *x);
struct LossOpts {
    GradSlabs *defer = nullptr;      // leave K-split slabs and Dense2 to grad_update_launch
    bool loss_mean = true;           // reduce the per-sample losses into h->loss_dev here
};
void dqn_loss_grad(snk_dqn_s *h, const BoardSrc &s_src, const BoardSrc &sn_src, const HeadArgs &meta, int64_t B,
                   double gamma, hipStream_t s, const LossOpts &o = LossOpts{});
// RMSProp + forward image (+ target copy when *counter % rate == 0) of an already finished gradient
UpdateTarget dqn_update_target(snk_dqn_s *h, const int64_t *counter, int64_t rate);
void dqn_sync_target_launch(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s);
void dqn_permute(snk_dqn_s *h, const float *src, float *dst, bool to_packed, hipStream_t s);
// q_net parameters changed: rebuild its forward weight image
void dqn_q_changed(snk_dqn_s *h, hipStream_t s);
// ---- the deeper bf16 net (snk_deep.hip), dispatched to when h->deep is set
void deep_create(snk_dqn_s *h, int bs, int C, uint64_t seed);
void deep_free(snk_dqn_s *h);
int64_t deep_ws_gen(const snk_dqn_s *h);
void deep_q_changed(snk_dqn_s *h, hipStream_t s);
void deep_t_changed(snk_dqn_s *h, hipStream_t s);
void deep_sync_target(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s);
// workspaces for an acting batch of S_act and / or a training batch of B (0: none)
void deep_prepare(snk_dqn_s *h, int64_t S_act, int64_t B);
// forward + head of q_net / t_net over S samples; returns the device Q [S][3]
const float *deep_forward(snk_dqn_s *h, int32_t which, const BoardSrc &src, int64_t S, HeadMode mode,
                          const HeadArgs &ha, hipStream_t s);
void deep_loss_grad(snk_dqn_s *h, const BoardSrc &s_src, const BoardSrc &sn_src, const HeadArgs &meta, int64_t B,
                    double gamma, hipStream_t s, bool loss_mean);
const double *deep_batch_losses(snk_dqn_s *h);
// RMSProp on the finished gradient, weight images, update_target_net! when *counter % rate == 0
void deep_apply(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s);

// generation of every buffer a captured trainer graph points into
inline int64_t dqn_ws_gen(const snk_dqn_s *h) {
    return h->act.gen + h->tgt.gen + h->trn.gen + h->slab_gen + deep_ws_gen(h);
}
}  // namespace snk

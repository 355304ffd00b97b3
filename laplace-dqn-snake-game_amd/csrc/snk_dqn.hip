// snk_dqn.hip — DQNModel handle (structs.jl:120-147): q_net, t_net and the
// RMSProp state, plus the C-ABI for forward, epsilon_greedy, the DQN update
// (utils.jl:442-466) and update_target_net! (utils.jl:174-177).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "snk_dqn.hpp"

namespace snk {

__global__ void permute_kernel(const float *__restrict__ src, float *__restrict__ dst, const int32_t *__restrict__ perm,
                               int64_t P, int to_packed) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
        if (to_packed)
            dst[i] = src[perm[i]];
        else
            dst[perm[i]] = src[i];
    }
}

__global__ void copy_if_due_kernel(const float *__restrict__ src, float *__restrict__ dst, int64_t P,
                                   const int64_t *__restrict__ counter, int64_t rate) {
    // update_target_net! when nb % target_update_rate == 0 (utils.jl:469-472)
    if (counter && (*counter % rate) != 0) return;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

__global__ void batch_meta_kernel(const int32_t *__restrict__ actions1, const uint8_t *__restrict__ mask3,
                                  int64_t B, uint8_t *__restrict__ act0, uint8_t *__restrict__ maskbits) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    act0[b] = (uint8_t)(actions1[b] - 1);
    maskbits[b] = (uint8_t)((mask3[3 * b] ? 1 : 0) | (mask3[3 * b + 1] ? 2 : 0) | (mask3[3 * b + 2] ? 4 : 0));
}

void dqn_permute(snk_dqn_s *h, const float *src, float *dst, bool to_packed, hipStream_t s) {
    permute_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->L.P, 256), 2048), 256, 0, s>>>(src, dst, h->perm,
                                                                                          h->L.P, to_packed);
    launch_check("permute_kernel");
}

void dqn_sync_target_launch(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s) {
    if (h->deep) {
        deep_sync_target(h, counter, rate, s);
        return;
    }
    copy_if_due_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->L.P, 256), 2048), 256, 0, s>>>(
        h->theta_q, h->theta_t, h->L.P, counter, rate);
    launch_check("copy_if_due_kernel");
    copy_if_due_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->L.T, 256), 2048), 256, 0, s>>>(
        h->wt_q, h->wt_t, h->L.T, counter, rate);
    launch_check("copy_if_due_kernel");
    if (h->wtb_q) {   // 3*T bf16 = 1.5*T words (T is even)
        copy_if_due_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->L.T, 256), 2048), 256, 0, s>>>(
            reinterpret_cast<const float *>(h->wtb_q), reinterpret_cast<float *>(h->wtb_t), 3 * h->L.T / 2, counter,
            rate);
        launch_check("copy_if_due_kernel");
    }
}

void dqn_q_changed(snk_dqn_s *h, hipStream_t s) {
    if (h->deep)
        deep_q_changed(h, s);
    else
        transpose_fwd_launch(h->L, h->theta_q, h->wt_q, h->wtb_q, s);
}

static const float *which_wt(snk_dqn_s *h, int32_t which) {
    return which == SNK_NET_TARGET ? h->wt_t : h->wt_q;
}
static const uint16_t *which_wtb(snk_dqn_s *h, int32_t which) {
    return which == SNK_NET_TARGET ? h->wtb_t : h->wtb_q;
}

BoardSrc src_env(const EnvDev &E) {
    BoardSrc b;
    b.base = E.frames;
    b.tptr = &E.ctl->t;
    b.pitch = E.pitch;
    b.slot_stride = E.n * (int64_t)E.pitch;
    b.C = E.C;
    b.ncell = E.bs * E.bs;
    return b;
}
BoardSrc src_replay(const ReplayDev &R, const int64_t *idx, int chan0) {
    BoardSrc b;
    b.base = R.frames;
    b.idx = idx;
    b.pitch = R.pitch;
    b.C = R.C;
    b.replay_nf = R.C + 1;
    b.ncell = R.bs * R.bs;
    b.chan0 = chan0;
    return b;
}
BoardSrc src_float(const QLayout &L, const float *x) {
    BoardSrc b;
    b.fbase = x;
    b.C = L.C;
    b.ncell = L.ncell;
    return b;
}

// One DQN loss + gradient on B transitions of a replay (or explicit batch):
// target forward on s', online forward on s with the Huber head, backward.
void dqn_loss_grad(snk_dqn_s *h, const BoardSrc &s_src, const BoardSrc &sn_src, const HeadArgs &meta, int64_t B,
                   double gamma, hipStream_t s, const LossOpts &o) {
    if (h->deep) {   // the deeper bf16 net finishes its gradient itself (o.defer unused)
        deep_loss_grad(h, s_src, sn_src, meta, B, gamma, s, o.loss_mean);
        if (o.defer) *o.defer = GradSlabs{};
        return;
    }
    qwork_ensure(h->tgt, h->L, B, false);
    qwork_ensure(h->trn, h->L, B, true);
    const int64_t need = qnet_backward_slab_floats(h->L, B);
    if (need > h->slab_cap) {
        SNK_HIP(hipStreamSynchronize(s));
        dfree(h->slab);
        h->slab = dalloc<float>(need);
        h->slab_cap = need;
        ++h->slab_gen;
    }
    HeadArgs ta = meta;
    ta.gamma = gamma;
    ta.target = h->trn.target;
    ta.B = B;
    // t_net(s') and q_net(s) share every layer launch; the loss head needs the target first
    HeadArgs la = ta;
    la.loss = h->trn.loss;
    la.dq = h->trn.dq;
    la.dz1 = h->trn.dz1;
    const FwdNet nets[2] = {FwdNet{h->theta_t, h->wt_t, h->wtb_t, sn_src, &h->tgt},
                            FwdNet{h->theta_q, h->wt_q, h->wtb_q, s_src, &h->trn}};
    const int ks = qnet_forward_update_pair(h->L, nets, B, s, &la);
    if (ks > 0) qnet_head_pair(h->L, h->theta_t, h->tgt, h->theta_q, h->trn, B, la, s, ks);
    if (o.loss_mean) loss_mean_launch(h->trn.loss, B, h->loss_dev, s);
    BwdOpts bo;
    bo.defer = o.defer;
    bo.dz1_ready = true;
    qnet_backward(h->L, h->theta_q, s_src, B, h->trn, h->grad, h->slab, h->slab_cap, s, bo);
}

UpdateTarget dqn_update_target(snk_dqn_s *h, const int64_t *counter, int64_t rate) {
    UpdateTarget u;
    u.theta = h->theta_q;
    u.acc = h->acc;
    u.wt = h->wt_q;
    u.theta_t = h->theta_t;
    u.wt_t = h->wt_t;
    u.wtb = h->wtb_q;
    u.wtb_t = h->wtb_t;
    u.counter = counter;
    u.rate = rate;
    u.lr = h->lr;
    u.rho = h->rho;
    u.eps = h->eps;
    return u;
}

}  // namespace snk

using namespace snk;

// glorot_uniform (Flux default init for Conv and Dense), zero biases, from a
// counter RNG (the reference draws from Julia's unseeded global RNG).
static void glorot_init(const QLayout &L, uint64_t seed, std::vector<float> &flux) {
    flux.assign(L.P, 0.0f);
    uint64_t ctr = 0;
    auto fill = [&](int64_t off, int64_t n, double fan_in, double fan_out) {
        const double lim = std::sqrt(6.0 / (fan_in + fan_out));
        for (int64_t i = 0; i < n; ++i) {
            const double u = (double)(splitmix64(seed ^ splitmix64(++ctr)) >> 11) * (1.0 / 9007199254740992.0);
            flux[off + i] = (float)((2.0 * u - 1.0) * lim);
        }
    };
    fill(L.off_w1, 9 * L.C * 16, 9.0 * L.C, 9.0 * 16);
    fill(L.off_w2, 9 * 16 * 32, 9.0 * 16, 9.0 * 32);
    fill(L.off_w3, 36 * 32 * 64, 36.0 * 32, 36.0 * 64);
    fill(L.off_d1w, (int64_t)L.K1 * 64, L.K1, 64);
    fill(L.off_d2w, 3 * 64, 64, 3);
}

extern "C" int snk_dqn_create(snk_dqn *out, int32_t bs, int32_t C, float lr, float rho, float eps, uint64_t seed) {
    return guard([&] {
        SNK_CHECK(out, SNK_ERR_INVALID, "out is NULL");
        SNK_CHECK(bs >= 6 && bs <= 20 && (C == 1 || C == 2), SNK_ERR_INVALID, "bad DQNModel geometry");
        auto *h = new snk_dqn_s();
        h->L = make_layout(bs, C);
        h->lr = lr;
        h->rho = rho;
        h->eps = eps;
        const int64_t P = h->L.P;
        h->theta_q = dalloc<float>(P);
        h->theta_t = dalloc<float>(P);
        h->acc = dalloc<float>(P);
        h->grad = dalloc<float>(P);
        h->tmp = dalloc<float>(P);
        h->perm = dalloc<int32_t>(P);
        h->loss_dev = dalloc<double>(1);
        std::vector<int32_t> perm(P);
        packed_to_flux_index(h->L, perm.data());
        std::vector<float> flux;
        glorot_init(h->L, seed, flux);
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(h->perm, perm.data(), P * 4, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(h->tmp, flux.data(), P * 4, hipMemcpyHostToDevice, s));
        h->wt_q = dalloc<float>(h->L.T);
        h->wt_t = dalloc<float>(h->L.T);
        // forward GEMMs on the exact bf16x6 split (default) or plain fp32 MFMA (SNK_ARITH_CONV_FP32)
        if (!arith(SNK_ARITH_CONV_FP32)) {
            h->wtb_q = dalloc<uint16_t>(3 * h->L.T);
            h->wtb_t = dalloc<uint16_t>(3 * h->L.T);
        }
        dqn_permute(h, h->tmp, h->theta_q, true, s);
        dqn_q_changed(h, s);
        dqn_sync_target_launch(h, nullptr, 1, s);   // t_net = deepcopy(q_net) (structs.jl:136)
        SNK_HIP(hipMemsetAsync(h->acc, 0, P * 4, s));
        SNK_HIP(hipMemsetAsync(h->grad, 0, P * 4, s));
        SNK_HIP(hipMemsetAsync(h->loss_dev, 0, 8, s));
        SNK_HIP(hipStreamSynchronize(s));
        *out = h;
    });
}

extern "C" int snk_dqn_destroy(snk_dqn h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        deep_free(h);
        qwork_free(h->act);
        qwork_free(h->tgt);
        qwork_free(h->trn);
        qwork_free(h->jw);
        for (void *p : {(void *)h->jbuf, (void *)h->jplanes, (void *)h->jexp, (void *)h->dplanes, (void *)h->dexp, (void *)h->gpart, (void *)h->jidx, (void *)h->jact, (void *)h->theta_q, (void *)h->theta_t,
                        (void *)h->acc, (void *)h->grad, (void *)h->tmp,
                        (void *)h->perm, (void *)h->slab, (void *)h->loss_dev, (void *)h->meta, (void *)h->wt_q,
                        (void *)h->wt_t, (void *)h->wtb_q, (void *)h->wtb_t})
            dfree(p);
        delete h;
    });
}

extern "C" int snk_dqn_nparams(snk_dqn h, int64_t *P) {
    return guard([&] {
        SNK_CHECK(h && P, SNK_ERR_INVALID, "NULL argument");
        *P = h->L.P;
    });
}

static float *which_buf(snk_dqn h, int32_t which) {
    switch (which) {
        case SNK_NET_Q: return h->theta_q;
        case SNK_NET_TARGET: return h->theta_t;
        case SNK_NET_OPT_STATE: return h->acc;
        case SNK_NET_GRAD: return h->grad;
    }
    SNK_CHECK(false, SNK_ERR_INVALID, "bad net selector %d", which);
    return nullptr;
}

extern "C" int snk_dqn_set_params(snk_dqn h, int32_t which, const float *flux_host) {
    return guard([&] {
        SNK_CHECK(h && flux_host, SNK_ERR_INVALID, "NULL argument");
        float *dst = which_buf(h, which);
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(h->tmp, flux_host, h->L.P * 4, hipMemcpyHostToDevice, s));
        dqn_permute(h, h->tmp, dst, true, s);
        if (which == SNK_NET_Q) dqn_q_changed(h, s);
        if (which == SNK_NET_TARGET) {
            if (h->deep)
                deep_t_changed(h, s);
            else
                transpose_fwd_launch(h->L, h->theta_t, h->wt_t, h->wtb_t, s);
        }
        SNK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int snk_dqn_get_params(snk_dqn h, int32_t which, float *flux_host) {
    return guard([&] {
        SNK_CHECK(h && flux_host, SNK_ERR_INVALID, "NULL argument");
        const float *src = which_buf(h, which);
        hipStream_t s = stream();
        dqn_permute(h, src, h->tmp, false, s);
        SNK_HIP(hipMemcpyAsync(flux_host, h->tmp, h->L.P * 4, hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int snk_dqn_buffer_ptr(snk_dqn h, int32_t which, float **packed_dev) {
    return guard([&] {
        SNK_CHECK(h && packed_dev, SNK_ERR_INVALID, "NULL argument");
        *packed_dev = which_buf(h, which);
    });
}

extern "C" int snk_dqn_sync_target(snk_dqn h) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        dqn_sync_target_launch(h, nullptr, 1, stream());
    });
}

extern "C" int snk_dqn_forward(snk_dqn h, int32_t which, const float *x_dev, int64_t B, float *q_dev) {
    return guard([&] {
        SNK_CHECK(h && x_dev && q_dev && B > 0, SNK_ERR_INVALID, "bad forward arguments");
        SNK_CHECK(which == SNK_NET_Q || which == SNK_NET_TARGET, SNK_ERR_INVALID, "forward needs q or target net");
        hipStream_t s = stream();
        if (h->deep) {
            const float *q = deep_forward(h, which, src_float(h->L, x_dev), B, HEAD_Q, HeadArgs{}, s);
            SNK_HIP(hipMemcpyAsync(q_dev, q, B * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
            return;
        }
        qwork_ensure(h->act, h->L, B, false);
        qnet_forward(h->L, which_buf(h, which), which_wt(h, which), src_float(h->L, x_dev), B, h->act, HEAD_Q,
                     HeadArgs{}, s, -1, which_wtb(h, which));
        SNK_HIP(hipMemcpyAsync(q_dev, h->act.q, B * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
    });
}

extern "C" int snk_dqn_forward_env(snk_dqn h, int32_t which, snk_env env, float *q_dev) {
    return guard([&] {
        SNK_CHECK(h && env && q_dev, SNK_ERR_INVALID, "NULL argument");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(E.bs == h->L.bs && E.C == h->L.C, SNK_ERR_INVALID, "env/model geometry mismatch");
        hipStream_t s = stream();
        if (h->deep) {
            const float *q = deep_forward(h, which, src_env(E), E.n, HEAD_Q, HeadArgs{}, s);
            SNK_HIP(hipMemcpyAsync(q_dev, q, E.n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
            return;
        }
        qwork_ensure(h->act, h->L, E.n, false);
        qnet_forward(h->L, which_buf(h, which), which_wt(h, which), src_env(E), E.n, h->act, HEAD_Q, HeadArgs{}, s,
                     -1, which_wtb(h, which));
        SNK_HIP(hipMemcpyAsync(q_dev, h->act.q, E.n * 3 * sizeof(float), hipMemcpyDeviceToDevice, s));
    });
}

extern "C" int snk_dqn_act(snk_dqn h, snk_env env, float epsilon, uint64_t seed, uint8_t *act_dev) {
    return guard([&] {
        SNK_CHECK(h && env && act_dev, SNK_ERR_INVALID, "NULL argument");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(E.bs == h->L.bs && E.C == h->L.C, SNK_ERR_INVALID, "env/model geometry mismatch");
        hipStream_t s = stream();
        HeadArgs ha;
        ha.act = act_dev;
        ha.epsilon = epsilon;
        ha.seed = seed;
        ha.tptr = &E.ctl->t;
        if (h->deep) {
            deep_forward(h, SNK_NET_Q, src_env(E), E.n, HEAD_ACT, ha, s);
            return;
        }
        qwork_ensure(h->act, h->L, E.n, false);
        qnet_forward(h->L, h->theta_q, h->wt_q, src_env(E), E.n, h->act, HEAD_ACT, ha, s, -1, h->wtb_q);
    });
}

extern "C" int snk_dqn_time_act_layers(snk_dqn h, snk_env env, int32_t reps, double *ms_out) {
    return guard([&] {
        SNK_CHECK(h && env && ms_out && reps > 0, SNK_ERR_INVALID, "bad time_act_layers arguments");
        SNK_CHECK(!h->deep, SNK_ERR_INVALID, "deep net: use snk_dqn_time_deep_layers");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(E.bs == h->L.bs && E.C == h->L.C, SNK_ERR_INVALID, "env/model geometry mismatch");
        hipStream_t s = stream();
        qwork_ensure(h->act, h->L, E.n, false);
        if (h->meta_cap < E.n) {
            SNK_HIP(hipStreamSynchronize(s));
            dfree(h->meta);
            h->meta = dalloc<uint8_t>(2 * E.n);
            h->meta_cap = E.n;
        }
        HeadArgs ha;
        ha.act = h->meta;
        ha.epsilon = 0.05f;
        ha.tptr = &E.ctl->t;
        qnet_forward(h->L, h->theta_q, h->wt_q, src_env(E), E.n, h->act, HEAD_ACT, ha, s, -1, h->wtb_q);
        hipEvent_t a, b;
        SNK_HIP(hipEventCreate(&a));
        SNK_HIP(hipEventCreate(&b));
        // conv2 + conv3 fused (conv_h3f_kernel): ms_out[1] = 0, ms_out[2] = the fused kernel
        const bool f23 = qnet_fused23(h->L, h->theta_q, h->wt_q, h->wtb_q, E.n, h->act);
        for (int layer = 0; layer < 5; ++layer) {
            if (f23 && layer == 1) {
                ms_out[1] = 0.0;
                continue;
            }
            const int only = f23 && layer == 2 ? QNET_ONLY_CONV23 : layer;
            SNK_HIP(hipEventRecord(a, s));
            for (int r = 0; r < reps; ++r)
                qnet_forward(h->L, h->theta_q, h->wt_q, src_env(E), E.n, h->act, HEAD_ACT, ha, s, only, h->wtb_q);
            SNK_HIP(hipEventRecord(b, s));
            SNK_HIP(hipEventSynchronize(b));
            float ms = 0.0f;
            SNK_HIP(hipEventElapsedTime(&ms, a, b));
            ms_out[layer] = (double)ms / reps;
        }
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
    });
}

extern "C" int snk_dqn_last_q(snk_dqn h, float *q_host, int64_t n) {
    return guard([&] {
        SNK_CHECK(h && q_host && n >= 0 && n <= h->act.cap && !h->deep, SNK_ERR_INVALID, "bad last_q arguments");
        SNK_HIP(hipMemcpyAsync(q_host, h->act.q, n * 3 * sizeof(float), hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_dqn_train_activations(snk_dqn h, int32_t layer, float *host, int64_t n) {
    return guard([&] {
        SNK_CHECK(h && host && n >= 0 && layer >= 0 && layer <= 3, SNK_ERR_INVALID, "bad train_activations arguments");
        SNK_CHECK(!h->deep, SNK_ERR_INVALID, "deep net: train_activations is not supported");
        const QWork &w = h->trn;
        SNK_CHECK(w.cap > 0, SNK_ERR_STATE, "no training forward has run");
        const float *src[4] = {w.a1, w.a2, w.a3, w.h1};
        const int64_t per[4] = {(int64_t)h->L.ncell * 16, (int64_t)h->L.ncell * 32, h->L.K1, 64};
        SNK_CHECK(n <= w.cap * per[layer], SNK_ERR_INVALID, "n exceeds the training workspace");
        SNK_HIP(hipMemcpyAsync(host, src[layer], n * sizeof(float), hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

static void finish_loss(snk_dqn h, double *loss_host) {
    if (!loss_host) return;
    SNK_HIP(hipMemcpyAsync(loss_host, h->loss_dev, sizeof(double), hipMemcpyDeviceToHost, stream()));
    SNK_HIP(hipStreamSynchronize(stream()));
}

extern "C" int snk_dqn_loss_grad(snk_dqn h, snk_replay rb, const int64_t *idx_dev, int64_t B, double gamma,
                                 double *loss_host) {
    return guard([&] {
        SNK_CHECK(h && rb && idx_dev && B > 0, SNK_ERR_INVALID, "bad loss_grad arguments");
        const ReplayDev &R = replay_dev(rb);
        SNK_CHECK(R.bs == h->L.bs && R.C == h->L.C, SNK_ERR_INVALID, "replay/model geometry mismatch");
        HeadArgs m;
        m.idx = idx_dev;
        m.rew = R.reward;
        m.done = R.done;
        m.mask = R.mask;
        m.act_idx = R.act;
        dqn_loss_grad(h, src_replay(R, idx_dev, 0), src_replay(R, idx_dev, 1), m, B, gamma, stream());
        finish_loss(h, loss_host);
    });
}

extern "C" int snk_dqn_loss_grad_batch(snk_dqn h, const float *states, const int32_t *actions, const float *rewards,
                                       const float *next_states, const uint8_t *dones, const uint8_t *mask3,
                                       int64_t B, double gamma, double *loss_host) {
    return guard([&] {
        SNK_CHECK(h && states && actions && rewards && next_states && dones && mask3 && B > 0, SNK_ERR_INVALID,
                  "bad loss_grad_batch arguments");
        hipStream_t s = stream();
        if (B > h->meta_cap) {
            SNK_HIP(hipStreamSynchronize(s));
            dfree(h->meta);
            h->meta = dalloc<uint8_t>(2 * B);
            h->meta_cap = B;
        }
        batch_meta_kernel<<<ceil_div(B, 256), 256, 0, s>>>(actions, mask3, B, h->meta, h->meta + B);
        launch_check("batch_meta_kernel");
        HeadArgs m;
        m.rew = rewards;
        m.done = dones;
        m.mask = h->meta + B;
        m.act_idx = h->meta;
        dqn_loss_grad(h, src_float(h->L, states), src_float(h->L, next_states), m, B, gamma, s);
        finish_loss(h, loss_host);
    });
}

extern "C" int snk_dqn_apply_grad(snk_dqn h) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        if (h->deep) {
            deep_apply(h, nullptr, 1, stream());
            return;
        }
        const UpdateTarget u = dqn_update_target(h, nullptr, 1);   // RMSProp + forward image, one pass
        grad_update_launch(h->L, nullptr, h->grad, &u, stream());
    });
}

extern "C" int snk_dqn_update(snk_dqn h, snk_replay rb, const int64_t *idx_dev, int64_t B, double gamma,
                              double *loss_host) {
    int st = snk_dqn_loss_grad(h, rb, idx_dev, B, gamma, nullptr);
    if (st != SNK_OK) return st;
    st = snk_dqn_apply_grad(h);
    if (st != SNK_OK) return st;
    return guard([&] { finish_loss(h, loss_host); });
}

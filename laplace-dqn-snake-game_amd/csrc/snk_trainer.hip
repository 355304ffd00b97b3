// snk_trainer.hip — the batched train! loop (utils.jl:420-494) on the device.
//
// One iteration = one lockstep step of every env:
//   epsilon_greedy over all envs (Q forward + head)  (utils.jl:153-172)
//   step! + virtual_step + store!                    (utils.jl:100-132, 267-277)
//   episode statistics of finished games             (utils.jl:478)
//   `updates_per_iter` DQN updates: sample, TD target, Huber, backward,
//   RMSProp, update_target_net! at nb % rate == 0, epsilon decay
//                                                    (utils.jl:442-481)
// Every counter the loop needs (env step, replay count, update count,
// epsilon) lives in device memory, so an iteration is a fixed launch sequence
// that is captured once into a hipGraph and replayed.
#include <algorithm>
#include <cmath>
#include <vector>

#include "snk_dqn.hpp"

namespace snk {

struct alignas(16) TrainStats {
    int64_t episodes;      // finished episodes
    int64_t score_sum;
    int64_t updates;       // updates run by this trainer
    int64_t nb;            // the reference's batch counter: update_target_net! when nb % rate == 0
                           // (train!: nb = 0, 1, ... utils.jl:431-469; compute_D: from 1, compute_D.jl:56-134)
    int64_t env_steps;
    double reward_sum;     // sum of finished episode rewards
    double last_loss;
    float reward_max;
    int32_t score_max;
    float epsilon;         // tr.epsilon (utils.jl:480)
    int32_t pad;
};

// the post-update bookkeeping as its own launch (the deeper net's update path)
__global__ __launch_bounds__(256) void post_update_kernel(PostUpdate p) { post_update_block(p); }

void comm_allreduce_mean(snk_comm h, float *buf, int64_t n, hipStream_t s);
void comm_broadcast(snk_comm h, float *buf, int64_t n, int root, hipStream_t s);
int comm_size(snk_comm h);

}  // namespace snk

using namespace snk;

struct snk_trainer_s {
    snk_comm comm = nullptr;
    snk_env env = nullptr;
    snk_dqn dqn = nullptr;
    snk_replay rb = nullptr;
    snk_trainer_cfg_t cfg{};
    TrainStats *stats = nullptr;
    uint8_t *act = nullptr;
    int64_t *idx = nullptr;
    double *loss_log = nullptr;
    int64_t log_cap = 0;
    uint32_t *ticket = nullptr;   // grad_update_kernel's arrival counter (post-update fold)
    int32_t B = 64;
    // [learn][n]: n iterations back to back in one graph (iterations only communicate
    // through device counters, so a longer graph is the same launch sequence with the
    // per-graph launch gap and the first iteration's weight-max scan paid once per graph):
    // n = `unroll`, and n = the remainder of a run that is not a multiple of it (one graph
    // for the tail instead of one single-iteration graph per leftover iteration; the
    // TAILS most recently used tail lengths stay cached per learn mode, see snk_trainer_run)
    static constexpr int MAXG = 64, TAILS = 3;
    hipGraph_t graph[2][MAXG + 1] = {};
    hipGraphExec_t exec[2][MAXG + 1] = {};
    int64_t used[2][MAXG + 1] = {};   // last use (use_clock) of each cached graph
    int64_t use_clock = 0;
    int unroll = 8;
    int64_t ws_gen = 0;   // dqn workspace generation the graphs were captured against
    // snk_trainer_set_trace: every update's finished gradient is also copied to
    // trace + slot * P, slot = (position of the update in the launch sequence) % trace_slots
    float *trace = nullptr;
    int64_t trace_slots = 0;
    // snk_trainer_set_act_trace: every iteration's actions (n bytes) and act-forward
    // Q values (n x 3 floats, optional) are copied to act_trace / q_trace + slot * n (x 3),
    // slot = (iteration within the launch sequence) % act_trace_slots
    uint8_t *act_trace = nullptr;
    float *q_trace = nullptr;
    int64_t act_trace_slots = 0;
    void drop_graphs() {
        for (int g = 0; g < 2; ++g)
            for (int i = 0; i <= MAXG; ++i) {
                if (exec[g][i]) (void)hipGraphExecDestroy(exec[g][i]);
                if (graph[g][i]) (void)hipGraphDestroy(graph[g][i]);
                exec[g][i] = nullptr;
                graph[g][i] = nullptr;
            }
    }
};

// One iteration's launch sequence (capturable: no host sync, no allocation),
// with n_upd DQN updates after the env step. The first update's replay draw
// counts the n transitions this step stores.
// chain: the previous iteration of this launch sequence (same learn / n_upd) ran
// just before, so its last grad_update wrote the conv3 weight-max partials of
// the image the act forward reads (no scan); next_chain: the next one will.
// split / next_split: as chain / next_chain for the split weight images of the act forward
// (grad_update writes them, the act forward skips w3_split_kernel); a captured graph's first
// iteration and every unroll-th eager iteration re-split with fresh exponents, so eager runs and
// graph replays compute the same bits
static void trainer_iteration(snk_trainer_s *h, bool learn, int n_upd, hipStream_t s, int it = 0, bool chain = false,
                              bool next_chain = false, bool split = false, bool next_split = false) {
    const EnvDev &E = env_dev(h->env);
    const ReplayDev &R = replay_dev(h->rb);
    snk_dqn_s *q = h->dqn;
    const bool upd = learn && n_upd > 0;
    const uint64_t sseed = h->cfg.seed ^ 0x5A4D504C45ULL;
    chain = chain && upd && !q->deep;
    next_chain = next_chain && upd && !q->deep;
    split = split && chain && arith(SNK_ARITH_SPLIT_CHAIN);
    next_split = next_split && next_chain && arith(SNK_ARITH_SPLIT_CHAIN);
    // the first update's sample (counting the n transitions this step stores) rides in a
    // spare workgroup of a launch of the act forward (batch <= 64): the weight-max scan or the
    // fused conv kernel (small net), the head (deep net)
    const bool ride = upd && h->B <= 64;
    if (chain) q->act.wmax_fresh = 1;
    if (split) q->act.split_fresh = 1;
    // a fresh split followed by chained ones: bound the weights' movement until the next fresh
    // split (at most `unroll` iterations of n_upd RMSProp steps) for its exponents
    q->act.split_grow = next_split ? (float)(2.0 * h->unroll * n_upd * (double)q->lr / std::sqrt(1.0 - (double)q->rho))
                                   : 0.0f;
    HeadArgs ha;
    SampleRider rider;
    if (ride) {
        rider.count = R.count; rider.cap = R.cap; rider.pending = E.n; rider.batch = h->B; rider.seed = sseed;
        rider.draw_dev = &h->stats->updates; rider.out = h->idx;
        if (q->deep) ha.rider = rider;
    } else if (upd) {
        replay_launch_sample(R, h->B, sseed, 0, &h->stats->updates, h->idx, nullptr, s, E.n);
    }
    ha.act = h->act;
    ha.seed = h->cfg.seed;
    ha.tptr = &E.ctl->t;
    ha.eps_dev = &h->stats->epsilon;
    const float *qact = q->act.q;
    // the act head inside env_step_kernel (small lockstep batches): the act forward stops at
    // Dense1's slabs and the step computes each env's Q-values and action first (bit-identical
    // to head_kernel<HEAD_ACT>; SNK_ARITH_ENV_HEAD = 0: the separate head launch)
    const bool env_head = !q->deep && arith(SNK_ARITH_ENV_HEAD) && env_act_head_ok(E, qnet_act_slab_count(q->L, E.n));
    EnvActHead eh;
    if (q->deep) {
        qact = deep_forward(q, SNK_NET_Q, src_env(E), E.n, HEAD_ACT, ha, s);
    } else if (env_head) {
        eh.ks = qnet_forward_act_slabs(q->L, q->theta_q, q->wt_q, src_env(E), E.n, q->act, s, q->wtb_q,
                                       ride ? &rider : nullptr);
        eh.slab = q->act.slab;
        eh.b1 = q->theta_q + q->L.off_d1b;
        eh.w2 = q->theta_q + q->L.off_d2w;
        eh.b2 = q->theta_q + q->L.off_d2b;
        eh.h1 = q->act.h1;
        eh.q = q->act.q;
        eh.act_out = h->act;
        eh.seed = ha.seed;
        eh.eps_dev = ha.eps_dev;
    } else {
        qnet_forward(q->L, q->theta_q, q->wt_q, src_env(E), E.n, q->act, HEAD_ACT, ha, s, -1, q->wtb_q,
                     ride ? &rider : nullptr);
    }
    // step! + virtual_step + store! + the episode statistics, one launch
    const EpisodeAcc acc{&h->stats->episodes, &h->stats->score_sum, &h->stats->env_steps, &h->stats->reward_sum,
                         &h->stats->reward_max, &h->stats->score_max};
    auto trace = [&]() {
        if (!h->act_trace) return;
        const int64_t slot = (int64_t)it % h->act_trace_slots;
        SNK_HIP(hipMemcpyAsync(h->act_trace + slot * E.n, h->act, (size_t)E.n, hipMemcpyDeviceToDevice, s));
        if (h->q_trace)
            SNK_HIP(hipMemcpyAsync(h->q_trace + slot * E.n * 3, qact, (size_t)E.n * 3 * sizeof(float),
                                   hipMemcpyDeviceToDevice, s));
    };
    if (!env_head) trace();
    env_launch_step(E, h->act, SNK_ACT_INDEX, &R, s, &acc, env_head ? &eh : nullptr);
    if (env_head) trace();   // the actions and Q-values the step computed
    if (!upd) return;
    for (int u = 0; u < n_upd; ++u) {
        // update u > 0 of the non-deep net: drawn by update u-1's grad_update_kernel (PostUpdate::next)
        if (u > 0 && q->deep) replay_launch_sample(R, h->B, sseed, 0, &h->stats->updates, h->idx, nullptr, s);
        HeadArgs m;
        m.idx = h->idx;
        m.rew = R.reward;
        m.done = R.done;
        m.mask = R.mask;
        m.act_idx = R.act;
        GradSlabs pend;
        LossOpts lo;
        lo.defer = &pend;
        lo.loss_mean = false;
        dqn_loss_grad(q, src_replay(R, h->idx, 0), src_replay(R, h->idx, 1), m, h->B, h->cfg.gamma, s, lo);
        PostUpdate post{q->deep ? deep_batch_losses(q) : q->trn.loss, h->B, q->loss_dev, &h->stats->last_loss,
                        h->loss_log, h->log_cap, &h->stats->updates, &h->stats->nb, &h->stats->epsilon,
                        h->cfg.decay, h->cfg.epsilon_end, h->ticket, SampleRider{}};
        const bool last = u + 1 == n_upd;
        if (!q->deep && !last) {   // the next update's replay draw (utils.jl:442), count unchanged
            post.next.count = R.count; post.next.cap = R.cap; post.next.pending = 0; post.next.batch = h->B;
            post.next.seed = sseed; post.next.out = h->idx;
        }
        if (q->deep) {   // the deeper bf16 net: finished gradient, [mean over ranks], RMSProp + images + target
            if (h->comm) comm_allreduce_mean(h->comm, q->grad, q->L.P, s);
            deep_apply(q, &h->stats->nb, h->cfg.target_update_rate, s);
            post_update_kernel<<<1, 256, 0, s>>>(post);
            launch_check("post_update_kernel");
        } else {
            // one pass: finish the gradient, RMSProp, forward image, update_target_net! when
            // nb % rate == 0, and (last block to arrive) the post-update bookkeeping
            UpdateTarget ut = dqn_update_target(q, &h->stats->nb, h->cfg.target_update_rate);
            if (last && next_chain) ut.wmax_out = q->act.wmax_part;   // for the next iteration's act forward
            if (last && next_split) {   // ... and its split images (w3_split_kernel's exponents)
                ut.s_w3h = q->act.w3h;
                ut.s_w2h = q->act.w2h;
                ut.s_w1h = q->act.w1h;
                ut.s_w3e = q->act.w3e;
                ut.s_w1e = q->act.w1e;
            }
            if (h->comm) {   // data-parallel replicas: mean gradient before the step
                grad_update_launch(q->L, &pend, q->grad, nullptr, s);
                comm_allreduce_mean(h->comm, q->grad, q->L.P, s);
                grad_update_launch(q->L, nullptr, q->grad, &ut, s, &post);
            } else {
                grad_update_launch(q->L, &pend, q->grad, &ut, s, &post);
            }
            if (ut.wmax_out) {
                q->act.wmax_n = GU_WMAX_BLOCKS;
                q->act.wmax_img = q->wt_q + q->L.off_t3;
            }
        }
        if (h->trace) {
            const int64_t slot = ((int64_t)it * n_upd + u) % h->trace_slots;
            SNK_HIP(hipMemcpyAsync(h->trace + slot * q->L.P, q->grad, q->L.P * sizeof(float),
                                   hipMemcpyDeviceToDevice, s));
        }
    }
}

static_assert(sizeof(snk_trainer_cfg_t) == 64 && sizeof(snk_trainer_stats_t) == 80, "ABI sizes in snakehip.h");

extern "C" int snk_abi_sizes(int64_t *cfg_size, int64_t *stats_size) {
    return guard([&] {
        SNK_CHECK(cfg_size && stats_size, SNK_ERR_INVALID, "NULL argument");
        *cfg_size = (int64_t)sizeof(snk_trainer_cfg_t);
        *stats_size = (int64_t)sizeof(snk_trainer_stats_t);
    });
}

extern "C" int snk_trainer_create(snk_trainer *out, snk_env env, snk_dqn dqn, snk_replay rb,
                                  const snk_trainer_cfg_t *cfg) {
    return guard([&] {
        SNK_CHECK(out && env && dqn && rb && cfg, SNK_ERR_INVALID, "NULL argument");
        SNK_CHECK(cfg->struct_size == (int32_t)sizeof(snk_trainer_cfg_t), SNK_ERR_INVALID,
                  "snk_trainer_cfg_t.struct_size = %d, the library's struct has %d bytes (binding out of date)",
                  cfg->struct_size, (int)sizeof(snk_trainer_cfg_t));
        const EnvDev &E = env_dev(env);
        const ReplayDev &R = replay_dev(rb);
        SNK_CHECK(E.autoreset, SNK_ERR_STATE, "the batched trainer needs auto-reset envs");
        SNK_CHECK(E.bs == dqn->L.bs && E.C == dqn->L.C && R.bs == E.bs && R.C == E.C, SNK_ERR_INVALID,
                  "env / model / replay geometry mismatch");
        SNK_CHECK(cfg->updates_per_iter >= 0 && cfg->target_update_rate > 0, SNK_ERR_INVALID, "bad trainer config");
        auto *h = new snk_trainer_s();
        h->env = env;
        h->dqn = dqn;
        h->rb = rb;
        h->cfg = *cfg;
        h->B = replay_batch(rb);
        h->log_cap = cfg->loss_log_capacity > 0 ? cfg->loss_log_capacity : 1;
        hipStream_t s = stream();
        h->stats = dalloc<TrainStats>(1);
        h->act = dalloc<uint8_t>(E.n);
        h->idx = dalloc<int64_t>(h->B);
        h->loss_log = dalloc<double>(h->log_cap);
        h->ticket = dalloc<uint32_t>(9 * 32);
        SNK_HIP(hipMemsetAsync(h->ticket, 0, 9 * 32 * sizeof(uint32_t), s));
        // iterations per captured graph: they only communicate through device
        // counters, so a longer graph is the same launch sequence with the
        // graph launch gap paid once per `unroll` (measured 12.34 M env-steps/s
        // at 8 against 12.28 M at 1)
        SNK_CHECK(cfg->graph_unroll <= snk_trainer_s::MAXG, SNK_ERR_INVALID,
                  "graph_unroll %d: at most %d iterations per captured graph", cfg->graph_unroll,
                  snk_trainer_s::MAXG);
        h->unroll = cfg->graph_unroll > 0 ? cfg->graph_unroll : 8;
        TrainStats st{};
        st.epsilon = cfg->epsilon;
        st.reward_max = -INFINITY;
        SNK_HIP(hipMemcpyAsync(h->stats, &st, sizeof st, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemsetAsync(h->loss_log, 0, h->log_cap * sizeof(double), s));
        SNK_HIP(hipMemsetAsync(h->act, 0, E.n, s));
        SNK_HIP(hipMemsetAsync(h->idx, 0, h->B * sizeof(int64_t), s));
        // every workspace the iteration touches is allocated now (graph capture)
        if (dqn->deep) {
            deep_prepare(dqn, E.n, h->B);
        } else {
            qwork_ensure(dqn->act, dqn->L, E.n, false);
            qwork_ensure(dqn->tgt, dqn->L, h->B, false);
            qwork_ensure(dqn->trn, dqn->L, h->B, true);
        }
        const int64_t need = dqn->deep ? 0 : qnet_backward_slab_floats(dqn->L, h->B);
        if (need > dqn->slab_cap) {
            dfree(dqn->slab);
            dqn->slab = dalloc<float>(need);
            dqn->slab_cap = need;
            ++dqn->slab_gen;
        }
        SNK_HIP(hipStreamSynchronize(s));
        h->ws_gen = dqn_ws_gen(dqn);
        *out = h;
    });
}

extern "C" int snk_trainer_destroy(snk_trainer h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        h->drop_graphs();
        for (void *p : {(void *)h->stats, (void *)h->act, (void *)h->idx, (void *)h->loss_log, (void *)h->ticket})
            dfree(p);
        delete h;
    });
}

// the trainer's buffers (allocated at create) may have been reallocated since
// a graph was captured: a model call with a larger batch grows the shared dqn
// workspaces. Re-size what the iteration touches and drop stale graphs.
static void trainer_refresh(snk_trainer_s *h) {
    snk_dqn_s *q = h->dqn;
    if (q->deep) {
        deep_prepare(q, env_dev(h->env).n, h->B);
    } else {
        qwork_ensure(q->act, q->L, env_dev(h->env).n, false);
        qwork_ensure(q->tgt, q->L, h->B, false);
        qwork_ensure(q->trn, q->L, h->B, true);
    }
    const int64_t gen = dqn_ws_gen(q);
    if (gen != h->ws_gen) {
        SNK_HIP(hipStreamSynchronize(stream()));
        h->drop_graphs();
        h->ws_gen = gen;
    }
}

static void trainer_check_replay(snk_trainer_s *h) {
    int64_t len = 0;
    if (snk_replay_length(h->rb, &len) != SNK_OK) throw Error{SNK_ERR_HIP};
    SNK_CHECK(len >= h->B, SNK_ERR_STATE, "replay holds %lld < batch_size %d transitions (fill it first)",
              (long long)len, h->B);
}

extern "C" int snk_trainer_run(snk_trainer h, int64_t iters, int32_t learn, int32_t use_graph) {
    return guard([&] {
        SNK_CHECK(h && iters >= 0, SNK_ERR_INVALID, "bad trainer_run arguments");
        hipStream_t s = stream();
        const int upi = h->cfg.updates_per_iter;
        if (learn && upi > 0) trainer_check_replay(h);
        trainer_refresh(h);
        const int g = learn ? 1 : 0;
        const int U = h->unroll;
        auto capture = [&](int n) {   // the n-iteration graph, captured once
            h->used[g][n] = ++h->use_clock;
            if (h->exec[g][n]) return h->exec[g][n];
            if (n != U) {   // a new tail length: keep the TAILS - 1 most recently used other tails
                int cached = 0, lru = 0;
                for (int m = 1; m <= snk_trainer_s::MAXG; ++m) {
                    if (m == U || m == n || !h->exec[g][m]) continue;
                    ++cached;
                    if (!lru || h->used[g][m] < h->used[g][lru]) lru = m;
                }
                if (cached >= snk_trainer_s::TAILS) {   // evict the least recently used one (each holds m iterations)
                    SNK_HIP(hipStreamSynchronize(s));
                    (void)hipGraphExecDestroy(h->exec[g][lru]);
                    (void)hipGraphDestroy(h->graph[g][lru]);
                    h->exec[g][lru] = nullptr;
                    h->graph[g][lru] = nullptr;
                }
            }
            SNK_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
            try {
                for (int i = 0; i < n; ++i) trainer_iteration(h, learn != 0, upi, s, i, i > 0, i + 1 < n, i > 0, i + 1 < n);
            } catch (...) {
                hipGraph_t dummy;
                (void)hipStreamEndCapture(s, &dummy);
                throw;
            }
            SNK_HIP(hipStreamEndCapture(s, &h->graph[g][n]));
            SNK_HIP(hipGraphInstantiate(&h->exec[g][n], h->graph[g][n], nullptr, nullptr, 0));
            return h->exec[g][n];
        };
        if (!use_graph) {
            for (int64_t i = 0; i < iters; ++i)
                trainer_iteration(h, learn != 0, upi, s, (int)(i % (1 << 20)), i > 0, i + 1 < iters, i % U != 0,
                                  i + 1 < iters && (i + 1) % U != 0);
            return;
        }
        if (U <= 1) {
            hipGraphExec_t e = capture(1);
            for (int64_t i = 0; i < iters; ++i) SNK_HIP(hipGraphLaunch(e, s));
            return;
        }
        int64_t i = 0;
        if (iters >= U) {
            hipGraphExec_t e = capture(U);
            for (; i + U <= iters; i += U) SNK_HIP(hipGraphLaunch(e, s));
        }
        if (i < iters) SNK_HIP(hipGraphLaunch(capture((int)(iters - i)), s));   // the tail: one graph (< U iterations)
    });
}

extern "C" int snk_trainer_run_partial(snk_trainer h, int32_t n_updates) {
    return guard([&] {
        SNK_CHECK(h && n_updates >= 0 && n_updates <= h->cfg.updates_per_iter, SNK_ERR_INVALID,
                  "run_partial: 0 <= n_updates <= updates_per_iter");
        if (n_updates > 0) trainer_check_replay(h);
        trainer_refresh(h);
        trainer_iteration(h, true, n_updates, stream());
    });
}

extern "C" int snk_trainer_set_trace(snk_trainer h, float *grad_ring_dev, int64_t slots) {
    return guard([&] {
        SNK_CHECK(h && (grad_ring_dev == nullptr || slots > 0), SNK_ERR_INVALID, "bad set_trace arguments");
        SNK_HIP(hipStreamSynchronize(stream()));
        h->trace = grad_ring_dev;
        h->trace_slots = grad_ring_dev ? slots : 0;
        h->drop_graphs();   // re-captured with (or without) the copies
    });
}

extern "C" int snk_trainer_set_act_trace(snk_trainer h, uint8_t *act_ring_dev, float *q_ring_dev, int64_t slots) {
    return guard([&] {
        SNK_CHECK(h && (act_ring_dev == nullptr || slots > 0) && (q_ring_dev == nullptr || act_ring_dev),
                  SNK_ERR_INVALID, "bad set_act_trace arguments");
        SNK_HIP(hipStreamSynchronize(stream()));
        h->act_trace = act_ring_dev;
        h->q_trace = act_ring_dev ? q_ring_dev : nullptr;
        h->act_trace_slots = act_ring_dev ? slots : 0;
        h->drop_graphs();   // re-captured with (or without) the copies
    });
}

extern "C" int snk_trainer_set_nb(snk_trainer h, int64_t nb) {
    return guard([&] {
        SNK_CHECK(h && nb >= 0, SNK_ERR_INVALID, "bad set_nb arguments");
        SNK_HIP(hipMemcpyAsync(&h->stats->nb, &nb, sizeof nb, hipMemcpyHostToDevice, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_trainer_set_comm(snk_trainer h, snk_comm comm) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        hipStream_t s = stream();
        snk_dqn_s *q = h->dqn;
        if (comm) {
            // replicas start from rank 0's q_net; t_net = q_net; fresh RMSProp state
            comm_broadcast(comm, q->theta_q, q->L.P, 0, s);
            dqn_q_changed(q, s);
            dqn_sync_target_launch(q, nullptr, 1, s);
            SNK_HIP(hipMemsetAsync(q->acc, 0, q->L.P * sizeof(float), s));
        }
        SNK_HIP(hipStreamSynchronize(s));
        h->comm = comm;   // NULL: detach (updates local again)
        h->drop_graphs();  // captured graphs predate the collective
    });
}

extern "C" int snk_trainer_stats(snk_trainer h, snk_trainer_stats_t *out) {
    return guard([&] {
        SNK_CHECK(h && out, SNK_ERR_INVALID, "NULL argument");
        SNK_CHECK(out->struct_size == (int32_t)sizeof(snk_trainer_stats_t), SNK_ERR_INVALID,
                  "snk_trainer_stats_t.struct_size = %d, the library's struct has %d bytes (binding out of date)",
                  out->struct_size, (int)sizeof(snk_trainer_stats_t));
        TrainStats st;
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(&st, h->stats, sizeof st, hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
        out->episodes = st.episodes;
        out->score_sum = st.score_sum;
        out->updates = st.updates;
        out->nb = st.nb;
        out->env_steps = st.env_steps;
        out->reward_sum = st.reward_sum;
        out->last_loss = st.last_loss;
        out->reward_max = st.reward_max;
        out->score_max = st.score_max;
        out->epsilon = st.epsilon;
    });
}

extern "C" int snk_trainer_losses(snk_trainer h, double *host, int64_t n) {
    return guard([&] {
        SNK_CHECK(h && host && n >= 0 && n <= h->log_cap, SNK_ERR_INVALID, "bad losses arguments");
        SNK_HIP(hipMemcpyAsync(host, h->loss_log, n * sizeof(double), hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_trainer_time_act_kernel(snk_trainer h, int32_t iters, double *ms_out) {
    return guard([&] {
        SNK_CHECK(h && iters > 0 && ms_out, SNK_ERR_INVALID, "bad time_act_kernel arguments");
        const int upi = h->cfg.updates_per_iter;
        if (upi > 0) trainer_check_replay(h);
        trainer_refresh(h);
        hipStream_t s = stream();
        // each timed eager iteration is queued behind one replay of the learning graph (U
        // iterations) with no host wait in between, so the GPU runs it as busy and as warm as the
        // graph loop (timed one by one with a host wait each, the kernel ran up to 15 % longer: the
        // clocks fall in the idle gaps); the events are recorded by the kernel's own dispatch
        // (h3f_timing_hook, hipExtLaunchKernelGGL)
        std::vector<hipEvent_t> ev(2 * (size_t)iters, nullptr);
        auto release = [&]() {
            h3f_timing_hook(nullptr, nullptr);
            for (hipEvent_t e : ev)
                if (e) (void)hipEventDestroy(e);
        };
        try {
            for (hipEvent_t &e : ev) SNK_HIP(hipEventCreate(&e));
            const bool graph = upi > 0 && h->unroll > 1;
            auto replay = [&]() {   // one learning-graph replay (its error message stays set)
                const int st = snk_trainer_run(h, h->unroll, 1, 1);
                if (st != SNK_OK) throw Error{st};
            };
            if (graph) replay();
            for (int i = 0; i < iters; ++i) {
                hipEvent_t a = ev[2 * i], b = ev[2 * i + 1];
                SNK_HIP(hipEventRecord(a, s));   // complete even if the kernel is absent
                SNK_HIP(hipEventRecord(b, s));
                h3f_timing_hook(a, b);
                trainer_iteration(h, true, upi, s);
                h3f_timing_hook(nullptr, nullptr);
                if (graph && i + 1 < iters) replay();
            }
            SNK_HIP(hipStreamSynchronize(s));
            std::vector<double> ms;
            for (int i = 0; i < iters; ++i) {
                float t = 0.0f;
                SNK_HIP(hipEventElapsedTime(&t, ev[2 * i], ev[2 * i + 1]));
                if (t > 0.0f) ms.push_back(t);
            }
            std::sort(ms.begin(), ms.end());
            const size_t n = ms.size();
            *ms_out = n == 0 ? 0.0 : n % 2 ? ms[n / 2] : 0.5 * (ms[n / 2 - 1] + ms[n / 2]);
        } catch (...) {
            release();
            throw;
        }
        release();
    });
}

extern "C" int snk_trainer_act_ptr(snk_trainer h, uint8_t **act_dev) {
    return guard([&] {
        SNK_CHECK(h && act_dev, SNK_ERR_INVALID, "NULL argument");
        *act_dev = h->act;
    });
}

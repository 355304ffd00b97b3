// snk_replay.hip — ReplayBuffer on the device (structs.jl:104-116).
//
// A ring of `capacity` transition slots. Slot k holds the n_frames+1 boards
// b_{t-C}..b_t (int8, 16-byte pitched) from which both s = (b_{t-C}..b_{t-1})
// and s' = (b_{t-C+1}..b_t) are read (utils.jl:141-149 frame semantics), plus
// SoA metadata. store! (utils.jl:267-277) writes slot count % capacity, which
// is exactly the reference's push-then-overwrite-from-position-1 order.
// sample (utils.jl:280-287) draws min(batch_size, length) distinct slots
// (Floyd's algorithm, device-side, counter-based RNG). stack_exp
// (utils.jl:343-383) is the gather kernel below; the DQN update reads slots
// directly by index and never materialises it.
#include <vector>

#include "snk_internal.hpp"

namespace snk {

// stack_exp: one thread per (sample, cell); metadata by thread (b, 0).
__global__ void replay_gather_kernel(ReplayDev R, const int64_t *__restrict__ idx, int64_t B,
                                     float *__restrict__ states, int32_t *__restrict__ actions,
                                     float *__restrict__ rewards, float *__restrict__ next_states,
                                     uint8_t *__restrict__ dones, uint8_t *__restrict__ mask,
                                     uint8_t *__restrict__ dirs) {
    const int ncell = R.bs * R.bs, C = R.C;
    const int64_t total = B * (int64_t)C * ncell;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / ((int64_t)C * ncell);
        const int r = (int)(i - b * C * ncell);
        const int f = r / ncell, c = r - f * ncell;
        const int64_t slot = idx[b];
        const int8_t *fr = R.frames + slot * (int64_t)(C + 1) * R.pitch;
        if (states) states[i] = (float)fr[f * R.pitch + c];
        if (next_states) next_states[i] = (float)fr[(f + 1) * R.pitch + c];
        if (r == 0) {
            if (actions) actions[b] = R.act[slot] == 255 ? 0 : (int32_t)R.act[slot] + 1;  // 1-based
            if (rewards) rewards[b] = R.reward[slot];
            if (dones) dones[b] = R.done[slot];
            if (mask)
                for (int k = 0; k < 3; ++k) mask[3 * b + k] = (R.mask[slot] >> k) & 1;
            if (dirs) dirs[b] = R.dirs[slot];
        }
    }
}

// Floyd's algorithm: a uniformly random B-subset of [0, len). Step n draws
// t_n uniform in [0, len-B+n] and keeps t_n unless already chosen, else
// len-B+n. The B candidates are drawn in parallel (one thread each); one
// thread then runs the short serial pass against an open-addressing set in LDS.
__global__ __launch_bounds__(256) void replay_sample_kernel(const int64_t *__restrict__ count, int64_t cap,
                                                            int32_t batch, uint64_t seed, uint64_t draw,
                                                            const int64_t *__restrict__ draw_dev,
                                                            int64_t *__restrict__ out, int32_t *__restrict__ b_out,
                                                            int64_t pending) {
    constexpr int HS = 8192;   // >= 2 * max batch (4096)
    __shared__ int64_t set[HS];
    __shared__ int64_t cand[4096];
    if (draw_dev) draw = (uint64_t)*draw_dev;
    const int64_t len = min(*count + pending, cap);   // pending: transitions stored before the draw is used
    const int B = (int)min((int64_t)batch, len);
    int hs = 128;
    while (hs < 2 * B) hs <<= 1;
    for (int i = threadIdx.x; i < hs; i += blockDim.x) set[i] = -1;
    for (int n = threadIdx.x; n < B; n += blockDim.x) {
        const uint64_t jp1 = (uint64_t)(len - B + n + 1);
        cand[n] = (int64_t)__umul64hi(rng_hash(seed, draw, (uint64_t)n), jp1);   // [0, len-B+n]
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        if (b_out) *b_out = B;
        for (int n = 0; n < B; ++n) {
            const int64_t t = cand[n];
            int p = (int)(splitmix64((uint64_t)t) & (uint64_t)(hs - 1));
            bool found = false;
            for (int64_t v; (v = set[p]) >= 0; p = (p + 1) & (hs - 1))
                if (v == t) { found = true; break; }
            const int64_t v = found ? len - B + n : t;
            if (found) {
                p = (int)(splitmix64((uint64_t)v) & (uint64_t)(hs - 1));
                while (set[p] >= 0) p = (p + 1) & (hs - 1);
            }
            set[p] = v;
            out[n] = v;
        }
    }
}

// The same draw for B <= 64 in one wave: lane n holds candidate t_n; the serial
// pass broadcasts t_n and asks all earlier lanes at once (ballot) whether it
// was already chosen. Same output as the LDS-set version.
__global__ __launch_bounds__(64) void replay_sample_wave_kernel(SampleRider r) { sample_wave(r); }

__global__ void replay_store_kernel(ReplayDev R, int64_t B, const int8_t *__restrict__ frames,
                                    const uint8_t *__restrict__ act, const float *__restrict__ rew,
                                    const uint8_t *__restrict__ done, const uint8_t *__restrict__ mask,
                                    const uint8_t *__restrict__ dirs) {
    const int ncell = R.bs * R.bs, nf = R.C + 1;
    const int64_t base = *R.count;
    const int64_t total = B * (int64_t)nf * ncell;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t b = i / ((int64_t)nf * ncell);
        const int r = (int)(i - b * nf * ncell);
        const int f = r / ncell, c = r - f * ncell;
        const int64_t slot = (base + b) % R.cap;
        R.frames[slot * nf * R.pitch + f * R.pitch + c] = frames[i];
        if (r == 0) {
            R.act[slot] = act[b];
            R.reward[slot] = rew[b];
            R.done[slot] = done[b];
            R.mask[slot] = mask[b];
            R.dirs[slot] = dirs[b];
        }
    }
}

__global__ void replay_advance_kernel(int64_t *count, int64_t B) {
    if (threadIdx.x == 0) *count += B;
}

}  // namespace snk

using namespace snk;

struct snk_replay_s {
    ReplayDev d{};
    int32_t batch_size = 64;
    uint8_t *staging = nullptr;
    size_t staging_bytes = 0;
};

namespace snk {
const EnvDev &env_dev(snk_env h);
const ReplayDev &replay_dev(snk_replay h) { return h->d; }
int32_t replay_batch(snk_replay h) { return h->batch_size; }
}  // namespace snk

extern "C" int snk_replay_create(snk_replay *out, int64_t cap, int32_t bs, int32_t C, int32_t batch) {
    return guard([&] {
        SNK_CHECK(out, SNK_ERR_INVALID, "out is NULL");
        SNK_CHECK(cap > 0 && bs >= 6 && bs <= 20 && (C == 1 || C == 2), SNK_ERR_INVALID,
                  "bad replay geometry");
        // structs.jl:113
        SNK_CHECK(batch > 0 && batch <= cap, SNK_ERR_STATE,
                  "batch_size cannot be greater than the capacity of the buffer.");
        SNK_CHECK(batch <= 4096, SNK_ERR_INVALID, "batch_size > 4096 unsupported");
        auto *h = new snk_replay_s();
        ReplayDev &d = h->d;
        d.cap = cap;
        d.bs = bs;
        d.C = C;
        d.pitch = frame_pitch(bs);
        d.frames = dalloc<int8_t>((size_t)cap * (C + 1) * d.pitch);
        d.reward = dalloc<float>(cap);
        d.act = dalloc<uint8_t>(cap);
        d.done = dalloc<uint8_t>(cap);
        d.mask = dalloc<uint8_t>(cap);
        d.dirs = dalloc<uint8_t>(cap);
        d.count = dalloc<int64_t>(1);
        h->batch_size = batch;
        hipStream_t s = stream();
        SNK_HIP(hipMemsetAsync(d.count, 0, sizeof(int64_t), s));
        SNK_HIP(hipMemsetAsync(d.frames, 0, (size_t)cap * (C + 1) * d.pitch, s));
        SNK_HIP(hipStreamSynchronize(s));
        *out = h;
    });
}

extern "C" int snk_replay_destroy(snk_replay h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        for (void *p : {(void *)h->d.frames, (void *)h->d.reward, (void *)h->d.act, (void *)h->d.done,
                        (void *)h->d.mask, (void *)h->d.dirs, (void *)h->d.count, (void *)h->staging})
            dfree(p);
        delete h;
    });
}

extern "C" int snk_env_step_store(snk_env env, const uint8_t *act_dev, int32_t act_mode, snk_replay rb) {
    return guard([&] {
        SNK_CHECK(env && rb && act_dev, SNK_ERR_INVALID, "NULL argument");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(E.autoreset, SNK_ERR_STATE, "fused store needs auto-reset envs");
        SNK_CHECK(E.bs == rb->d.bs && E.C == rb->d.C, SNK_ERR_INVALID, "env/replay geometry mismatch");
        hipStream_t s = stream();
        env_launch_step(E, act_dev, act_mode, &rb->d, s);
    });
}

extern "C" int snk_env_time_step(snk_env env, snk_replay rb, const uint8_t *act_dev, int32_t reps, double *ms_out) {
    return guard([&] {
        SNK_CHECK(env && act_dev && ms_out && reps > 0, SNK_ERR_INVALID, "bad time_step arguments");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(!rb || E.autoreset, SNK_ERR_STATE, "fused store needs auto-reset envs");
        hipStream_t s = stream();
        hipEvent_t a, b;
        SNK_HIP(hipEventCreate(&a));
        SNK_HIP(hipEventCreate(&b));
        // back-to-back launches between one event pair: the steady-state time per step
        // (kernel + launch boundary), as the trainer's graph runs it
        env_launch_step(E, act_dev, SNK_ACT_INDEX, rb ? &rb->d : nullptr, s);   // warm
        SNK_HIP(hipEventRecord(a, s));
        for (int r = 0; r < reps; ++r) env_launch_step(E, act_dev, SNK_ACT_INDEX, rb ? &rb->d : nullptr, s);
        SNK_HIP(hipEventRecord(b, s));
        SNK_HIP(hipEventSynchronize(b));
        float ms = 0.0f;
        SNK_HIP(hipEventElapsedTime(&ms, a, b));
        const double total = ms;
        *ms_out = total / reps;
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
    });
}

extern "C" int snk_replay_store(snk_replay h, int64_t B, const int8_t *frames, const uint8_t *act,
                                const float *rew, const uint8_t *done, const uint8_t *mask,
                                const uint8_t *dirs) {
    return guard([&] {
        SNK_CHECK(h && B >= 0 && frames && act && rew && done && mask && dirs, SNK_ERR_INVALID,
                  "NULL argument");
        if (B == 0) return;
        const ReplayDev &d = h->d;
        const size_t nfb = (size_t)B * (d.C + 1) * d.bs * d.bs;
        const size_t need = nfb + (size_t)B * (5 + 4) + 64;
        hipStream_t s = stream();
        if (need > h->staging_bytes) {
            SNK_HIP(hipStreamSynchronize(s));
            dfree(h->staging);
            h->staging = dalloc<uint8_t>(need);
            h->staging_bytes = need;
        }
        uint8_t *p = h->staging;
        int8_t *df = (int8_t *)p;
        float *drew = (float *)(p + ((nfb + 15) & ~size_t(15)));
        uint8_t *dact = (uint8_t *)(drew + B);
        uint8_t *ddone = dact + B, *dmask = ddone + B, *ddirs = dmask + B;
        SNK_HIP(hipMemcpyAsync(df, frames, nfb, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(drew, rew, B * 4, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(dact, act, B, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(ddone, done, B, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(dmask, mask, B, hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(ddirs, dirs, B, hipMemcpyHostToDevice, s));
        const int64_t total = (int64_t)nfb;
        replay_store_kernel<<<std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0, s>>>(
            d, B, df, dact, drew, ddone, dmask, ddirs);
        launch_check("replay_store_kernel");
        replay_advance_kernel<<<1, 64, 0, s>>>(d.count, B);
        launch_check("replay_advance_kernel");
        SNK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int snk_replay_position(snk_replay h, int64_t *count) {
    return guard([&] {
        SNK_CHECK(h && count, SNK_ERR_INVALID, "NULL argument");
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(count, h->d.count, sizeof(int64_t), hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int snk_replay_length(snk_replay h, int64_t *len) {
    return guard([&] {
        SNK_CHECK(h && len, SNK_ERR_INVALID, "NULL argument");
        int64_t c = 0;
        if (snk_replay_position(h, &c) != SNK_OK) throw Error{SNK_ERR_HIP};
        *len = std::min(c, h->d.cap);
    });
}

extern "C" int snk_replay_empty(snk_replay h) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        SNK_HIP(hipMemsetAsync(h->d.count, 0, sizeof(int64_t), stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

namespace snk {
void replay_launch_sample(const ReplayDev &d, int32_t batch, uint64_t seed, uint64_t draw,
                          const int64_t *draw_dev, int64_t *idx, int32_t *b_dev, hipStream_t s, int64_t pending) {
    if (batch <= 64) {
        SampleRider r;
        r.count = d.count; r.cap = d.cap; r.pending = pending; r.batch = batch; r.seed = seed; r.draw = draw;
        r.draw_dev = draw_dev; r.out = idx; r.b_out = b_dev;
        replay_sample_wave_kernel<<<1, 64, 0, s>>>(r);
    }
    else
        replay_sample_kernel<<<1, 256, 0, s>>>(d.count, d.cap, batch, seed, draw, draw_dev, idx, b_dev, pending);
    launch_check("replay_sample_kernel");
}
}  // namespace snk

extern "C" int snk_replay_sample(snk_replay h, uint64_t seed, uint64_t draw, int64_t *idx_dev,
                                 int32_t *B_out) {
    return guard([&] {
        SNK_CHECK(h && idx_dev, SNK_ERR_INVALID, "NULL argument");
        int64_t len = 0;
        if (snk_replay_length(h, &len) != SNK_OK) throw Error{SNK_ERR_HIP};
        SNK_CHECK(len > 0, SNK_ERR_STATE, "cannot sample an empty buffer");
        replay_launch_sample(h->d, h->batch_size, seed, draw, nullptr, idx_dev, nullptr, stream(), 0);
        if (B_out) *B_out = (int32_t)std::min<int64_t>(h->batch_size, len);
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_replay_gather(snk_replay h, const int64_t *idx, int64_t B, float *states,
                                 int32_t *actions, float *rewards, float *next_states, uint8_t *dones,
                                 uint8_t *mask, uint8_t *dirs) {
    return guard([&] {
        SNK_CHECK(h && idx && B > 0, SNK_ERR_INVALID, "bad gather arguments");
        const int64_t total = B * (int64_t)h->d.C * h->d.bs * h->d.bs;
        hipStream_t s = stream();
        replay_gather_kernel<<<std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0, s>>>(
            h->d, idx, B, states, actions, rewards, next_states, dones, mask, dirs);
        launch_check("replay_gather_kernel");
    });
}

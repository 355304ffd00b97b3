// snk_env.hip — batched Snake environment on gfx950.
//
// One fused kernel per lockstep step of n envs implements step!
// (utils.jl:100-109: move_wrapper! -> grow_maybe! -> sample_food! /
// remove_tail! -> check_collision -> update_board!) plus virtual_step's
// suicidal mask (utils.jl:112-132), auto-reset (utils.jl:199 `SnakeGame()`)
// and, optionally, store! of the transition into the replay ring
// (utils.jl:267-277).
//
// Mapping: a workgroup is ONE wave of 64 lanes that owns 64 envs.
//   Phase A  the wave streams the 64 current boards (16-byte pieces,
//            consecutive lanes -> consecutive bytes) HBM -> LDS;
//   Phase B  lane e runs env e's scalar logic against its LDS board: O(1)
//            collision test (board[new_head] lookup replaces the reference's
//            O(L) count over the body), food-list probe, in-place edits of
//            the <= 3 cells that change, next-state suicidal mask;
//   Phase C  the wave streams the new boards LDS -> HBM frame ring, and the
//            b_{t-C}..b_t frames into the replay slot.
// Per env-step HBM traffic is 2*pitch + 32 B of state/outputs (+ (C+1)*pitch
// when storing): the board is touched once in each direction.
#include <algorithm>
#include <vector>

#include "snk_internal.hpp"

namespace snk {

__device__ __forceinline__ int food_search(const int8_t *b, const int16_t *food, int n_food,
                                           uint64_t used) {
    // utils.jl:25-34: first list entry (in list order) whose cell is empty
    for (int k = 0; k < n_food; ++k)
        if (!((used >> k) & 1ull) && b[food[k]] == 0) return k;
    return -1;
}
__device__ __forceinline__ bool has_empty(const int8_t *b, int ncell) {
    for (int c = 0; c < ncell; ++c)
        if (b[c] == 0) return true;
    return false;
}

template <int PITCH>
__global__ __launch_bounds__(64) void env_step_kernel(EnvDev E, const uint8_t *__restrict__ act,
                                                      int act_mode, ReplayDev R, int store) {
    __shared__ __attribute__((aligned(16))) int8_t sb[64 * PITCH];
    __shared__ uint8_t s_flag[64];  // bit0 stepped, bit1 reset
    constexpr int NCH = PITCH / 16;
    const int lane = threadIdx.x;
    const int64_t e0 = (int64_t)blockIdx.x * 64;
    const int ne = (int)min((int64_t)64, E.n - e0);
    const int64_t t = E.ctl->t;
    const int cur = (int)(t % 3), nxt = (int)((t + 1) % 3), prv = (int)((t + 2) % 3);
    const int64_t rc = store ? *R.count : 0;

    // ---- Phase A: current boards HBM -> LDS ------------------------------
    for (int idx = lane; idx < ne * NCH; idx += 64) {
        const int e = idx / NCH, c = idx - e * NCH;
        const int4 v = *reinterpret_cast<const int4 *>(E.frames + ((e0 + e) * 3 + cur) * PITCH + c * 16);
        *reinterpret_cast<int4 *>(sb + e * PITCH + c * 16) = v;
    }
    __syncthreads();

    // ---- Phase B: per-env logic (lane = env) ------------------------------
    uint8_t flag = 0;
    if (lane < ne) {
        const int64_t e = e0 + lane;
        const int bs = E.bs, cap = E.ring_cap;
        int8_t *b = sb + lane * PITCH;
        EnvState st = E.state[e];
        const int prev = st.flags & 3;
        if (!(st.flags & 4)) {
            flag = 1;
            const int a = act[e];
            const int dir = act_mode == SNK_ACT_INDEX ? avail_action(prev, a % 3) : (a & 3);
            uint16_t *ring = E.ring + e * cap;
            const int head_cell = ring[st.head];
            int tail_idx = st.head + st.len - 1;
            if (tail_idx >= cap) tail_idx -= cap;
            const int tail_cell = ring[tail_idx];
            // grow_maybe! (utils.jl:66-81)
            const int nh = head_cell + dir_delta(bs, dir);
            const int old = b[nh];
            const bool eat = old == 2;
            float reward = eat ? 1.0f : -0.01f;
            uint64_t used = st.food_used;
            int food_cell = -1;
            bool fault = false;
            int score = st.score;
            if (eat) {
                score += 1;
                const int k = food_search(b, E.food, E.n_food, used);  // pre-update board
                if (k >= 0) {
                    used |= 1ull << k;
                    food_cell = E.food[k];
                } else if (has_empty(b, bs * bs)) {
                    fault = true;  // utils.jl:37 BoundsError in the reference
                }
            }
            // check_collision (utils.jl:55-58) after the tail pop; truncation
            // utils.jl:88 with length(board_history) = n_frames + steps - 1
            const bool body = old == 1 && !(!eat && nh == tail_cell);
            const int steps = st.steps + 1;
            const bool lost = old == -1 || body || dir == (prev ^ 1) || (E.C + steps - 1 > E.max_hist);
            if (lost) reward = -1.0f;
            // update_board! (utils.jl:43-52) as cell edits
            if (!eat) b[tail_cell] = 0;
            b[nh] = 1;
            if (food_cell >= 0) b[food_cell] = 2;
            const int nhead = st.head == 0 ? cap - 1 : st.head - 1;
            ring[nhead] = (uint16_t)nh;
            const int nlen = st.len + (eat ? 1 : 0);
            const int ntail_idx = eat ? tail_idx : (tail_idx == 0 ? cap - 1 : tail_idx - 1);
            const int ntail_cell = eat ? tail_cell : ring[ntail_idx];
            // virtual_step (utils.jl:112-132): would each next action lose?
            uint8_t mask = 7;
            if (!lost) {
                mask = 0;
                const bool trunc2 = E.C + steps > E.max_hist;
                for (int k2 = 0; k2 < 3; ++k2) {
                    const int nh2 = nh + dir_delta(bs, avail_action(dir, k2));
                    const int v = b[nh2];
                    const bool veat = v == 2;
                    const bool vbody = v == 1 && !(!veat && nh2 == ntail_cell);
                    if (v == -1 || vbody || trunc2) mask |= (uint8_t)(1 << k2);
                    if (veat && food_search(b, E.food, E.n_food, used) < 0 && has_empty(b, bs * bs))
                        fault = true;  // the virtual step's sample_food! would throw too
                }
            }
            const float epr = E.ep_reward[e] + reward;
            const uint8_t dirs = (uint8_t)(prev | (dir << 2) | ((lost ? 1 : 0) << 4));
            E.out_reward[e] = reward;
            E.out_done[e] = lost;
            E.out_mask[e] = mask;
            E.out_dirs[e] = dirs;
            E.out_ep_reward[e] = epr;
            E.out_score[e] = (uint8_t)score;
            if (fault) atomicAdd(E.fault_count, 1u);
            if (store) {
                const int64_t slot = (rc + e) % R.cap;
                R.reward[slot] = reward;
                R.act[slot] = (uint8_t)(act_mode == SNK_ACT_INDEX ? a % 3 : avail_index(prev, dir));
                R.done[slot] = lost;
                R.mask[slot] = mask;
                R.dirs[slot] = dirs;
            }
            if (lost && E.autoreset) {
                flag |= 2;
                EnvState ns{};
                ns.head = 0;
                ns.len = 2;
                ring[0] = (uint16_t)((bs - 3) + bs);  // structs.jl:47 (bs-2, 2)
                ring[1] = (uint16_t)((bs - 2) + bs);  //              (bs-1, 2)
                E.state[e] = ns;
                E.ep_reward[e] = 0.0f;
            } else {
                EnvState ns;
                ns.food_used = used;
                ns.head = (uint16_t)nhead;
                ns.len = (uint16_t)nlen;
                ns.steps = (uint16_t)steps;
                ns.flags = (uint8_t)(dir | (lost ? 4 : 0) | ((fault || (st.flags & 8)) ? 8 : 0));
                ns.score = (uint8_t)score;
                E.state[e] = ns;
                E.ep_reward[e] = epr;
            }
        } else {
            // lost and not auto-reset: the game is over, nothing moves
            E.out_reward[e] = 0.0f;
            E.out_done[e] = 1;
            E.out_mask[e] = 7;
            E.out_dirs[e] = (uint8_t)(prev | (prev << 2) | (1 << 4));
            E.out_ep_reward[e] = E.ep_reward[e];
            E.out_score[e] = st.score;
        }
        s_flag[lane] = flag;
    }
    __syncthreads();

    // ---- Phase C: LDS -> frame ring (+ replay slot) -----------------------
    for (int idx = lane; idx < ne * NCH; idx += 64) {
        const int e = idx / NCH, c = idx - e * NCH;
        const int64_t ge = e0 + e;
        const uint8_t f = s_flag[e];
        const int4 vnew = *reinterpret_cast<const int4 *>(sb + e * PITCH + c * 16);
        int8_t *fr = E.frames + ge * 3 * PITCH + c * 16;
        if (store && (f & 1)) {
            const int64_t slot = (rc + ge) % R.cap;
            int8_t *rf = R.frames + slot * (int64_t)(R.C + 1) * PITCH + c * 16;
            const int4 vcur = *reinterpret_cast<const int4 *>(fr + cur * PITCH);
            if (R.C == 2) {
                const int4 vprv = *reinterpret_cast<const int4 *>(fr + prv * PITCH);
                *reinterpret_cast<int4 *>(rf) = vprv;
                *reinterpret_cast<int4 *>(rf + PITCH) = vcur;
                *reinterpret_cast<int4 *>(rf + 2 * PITCH) = vnew;
            } else {
                *reinterpret_cast<int4 *>(rf) = vcur;
                *reinterpret_cast<int4 *>(rf + PITCH) = vnew;
            }
        }
        if (f & 2) {
            // auto-reset: next state is (b0, b0) (structs.jl:53 n_frames copies)
            const int4 v0 = *reinterpret_cast<const int4 *>(E.init_board + c * 16);
            *reinterpret_cast<int4 *>(fr + nxt * PITCH) = v0;
            if (E.C == 2) *reinterpret_cast<int4 *>(fr + cur * PITCH) = v0;
        } else {
            *reinterpret_cast<int4 *>(fr + nxt * PITCH) = vnew;
        }
    }
}

__global__ void env_advance_kernel(Ctl *ctl, int64_t *replay_count, int64_t n) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        ctl->t += 1;
        if (replay_count) *replay_count += n;
    }
}

// reset! for masked envs: SnakeGame() board in all 3 frame slots
__global__ void env_reset_kernel(EnvDev E, const uint8_t *__restrict__ mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E.n || (mask && !mask[e])) return;
    int8_t *fr = E.frames + e * 3 * E.pitch;
    for (int s = 0; s < 3; ++s)
        for (int c = 0; c < E.pitch; c += 16)
            *reinterpret_cast<int4 *>(fr + s * E.pitch + c) = *reinterpret_cast<const int4 *>(E.init_board + c);
    uint16_t *ring = E.ring + e * E.ring_cap;
    ring[0] = (uint16_t)((E.bs - 3) + E.bs);
    ring[1] = (uint16_t)((E.bs - 2) + E.bs);
    EnvState ns{};
    ns.head = 0;
    ns.len = 2;
    E.state[e] = ns;
    E.ep_reward[e] = 0.0f;
}

// assemble_state! / game.board gather: out [n][nf][bs*bs], frames oldest first
__global__ void env_gather_kernel(EnvDev E, int nf, int8_t *__restrict__ out) {
    const int ncell = E.bs * E.bs;
    const int64_t total = E.n * (int64_t)nf * ncell;
    const int64_t t = E.ctl->t;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = i / ((int64_t)nf * ncell);
        const int r = (int)(i - e * nf * ncell);
        const int f = r / ncell, c = r - f * ncell;
        const int slot = (int)((t + 3 - (nf - 1 - f)) % 3);
        out[i] = E.frames[(e * 3 + slot) * E.pitch + c];
    }
}

__global__ void env_synth_kernel(EnvDev E, uint64_t seed, uint8_t *__restrict__ act) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E.n) return;
    act[e] = (uint8_t)((rng_hash(seed, (uint64_t)e, (uint64_t)E.ctl->t) >> 32) % 3);
}

void env_launch_step(const EnvDev &E, const uint8_t *act, int act_mode, const ReplayDev *R,
                     hipStream_t s) {
    ReplayDev r{};
    if (R) r = *R;
    const int grid = ceil_div(E.n, 64);
    const int store = R ? 1 : 0;
    switch (E.pitch) {
        case 48: env_step_kernel<48><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 64: env_step_kernel<64><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 96: env_step_kernel<96><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 112: env_step_kernel<112><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 128: env_step_kernel<128><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 144: env_step_kernel<144><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 176: env_step_kernel<176><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 208: env_step_kernel<208><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 240: env_step_kernel<240><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 256: env_step_kernel<256><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 304: env_step_kernel<304><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 336: env_step_kernel<336><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 368: env_step_kernel<368><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        case 400: env_step_kernel<400><<<grid, 64, 0, s>>>(E, act, act_mode, r, store); break;
        default: SNK_CHECK(false, SNK_ERR_INVALID, "unsupported board pitch %d", E.pitch);
    }
    launch_check("env_step_kernel");
}

void env_launch_advance(const EnvDev &E, const ReplayDev *R, hipStream_t s) {
    env_advance_kernel<<<1, 64, 0, s>>>(E.ctl, R ? R->count : nullptr, E.n);
    launch_check("env_advance_kernel");
}

}  // namespace snk

// =========================================================================
// C ABI
// =========================================================================
using namespace snk;

struct snk_env_s {
    EnvDev d{};
    int8_t *init_board = nullptr;
    int16_t *food = nullptr;
    uint8_t *scratch = nullptr;   // [n] staging for host masks
    int8_t *gather = nullptr;     // [n][C][ncell]
    int32_t n_food_host = 0;
};

extern "C" int snk_env_create(snk_env *out, int64_t n, int32_t bs, int32_t C, uint32_t food_seed,
                              int32_t max_hist, int32_t autoreset) {
    return guard([&] {
        SNK_CHECK(out, SNK_ERR_INVALID, "out is NULL");
        SNK_CHECK(n > 0, SNK_ERR_INVALID, "n_envs must be > 0");
        SNK_CHECK(bs >= 6 && bs <= 20, SNK_ERR_INVALID, "board_size %d outside [6, 20]", bs);
        SNK_CHECK(C == 1 || C == 2, SNK_ERR_INVALID, "n_frames must be 1 or 2 (got %d)", C);
        SNK_CHECK(max_hist >= 1 && max_hist < 60000, SNK_ERR_INVALID, "max_hist out of range");
        auto *h = new snk_env_s();
        EnvDev &d = h->d;
        d.n = n;
        d.bs = bs;
        d.C = C;
        d.pitch = frame_pitch(bs);
        d.max_hist = max_hist;
        d.autoreset = autoreset ? 1 : 0;
        d.ring_cap = bs * bs;
        d.n_food = 50;
        const int ncell = bs * bs;
        // structs.jl:70 food list (host Xoshiro restatement), 50 entries
        int32_t cells[64];
        if (snk_food_list(bs, food_seed, d.n_food, cells) != SNK_OK) throw Error{SNK_ERR_INTERNAL};
        int16_t food16[64];
        for (int k = 0; k < d.n_food; ++k) food16[k] = (int16_t)cells[k];
        // structs.jl:34-51 SnakeGame() board
        std::vector<int8_t> b0(d.pitch, 0);
        for (int j = 0; j < bs; ++j)
            for (int i = 0; i < bs; ++i)
                b0[i + j * bs] = (i == 0 || i == bs - 1 || j == 0 || j == bs - 1) ? -1 : 0;
        b0[3 + 4 * bs] = 2;
        b0[(bs - 3) + bs] = 1;
        b0[(bs - 2) + bs] = 1;
        (void)ncell;
        hipStream_t s = stream();
        h->food = dalloc<int16_t>(64);
        h->init_board = dalloc<int8_t>(d.pitch);
        SNK_HIP(hipMemcpyAsync(h->food, food16, sizeof(food16), hipMemcpyHostToDevice, s));
        SNK_HIP(hipMemcpyAsync(h->init_board, b0.data(), d.pitch, hipMemcpyHostToDevice, s));
        d.food = h->food;
        d.init_board = h->init_board;
        d.frames = dalloc<int8_t>((size_t)n * 3 * d.pitch);
        d.ring = dalloc<uint16_t>((size_t)n * d.ring_cap);
        d.state = dalloc<EnvState>(n);
        d.ep_reward = dalloc<float>(n);
        d.out_reward = dalloc<float>(n);
        d.out_done = dalloc<uint8_t>(n);
        d.out_mask = dalloc<uint8_t>(n);
        d.out_dirs = dalloc<uint8_t>(n);
        d.out_ep_reward = dalloc<float>(n);
        d.out_score = dalloc<uint8_t>(n);
        d.fault_count = dalloc<uint32_t>(1);
        d.ctl = dalloc<Ctl>(1);
        h->scratch = dalloc<uint8_t>(n);
        h->gather = dalloc<int8_t>((size_t)n * C * d.ring_cap);
        SNK_HIP(hipMemsetAsync(d.fault_count, 0, sizeof(uint32_t), s));
        SNK_HIP(hipMemsetAsync(d.ctl, 0, sizeof(Ctl), s));
        SNK_HIP(hipMemsetAsync(d.out_reward, 0, n * sizeof(float), s));
        SNK_HIP(hipMemsetAsync(d.out_done, 0, n, s));
        SNK_HIP(hipMemsetAsync(d.out_mask, 0, n, s));
        SNK_HIP(hipMemsetAsync(d.out_dirs, 0, n, s));
        SNK_HIP(hipMemsetAsync(d.out_ep_reward, 0, n * sizeof(float), s));
        SNK_HIP(hipMemsetAsync(d.out_score, 0, n, s));
        env_reset_kernel<<<ceil_div(n, 256), 256, 0, s>>>(d, nullptr);
        launch_check("env_reset_kernel");
        SNK_HIP(hipStreamSynchronize(s));
        *out = h;
    });
}

extern "C" int snk_env_destroy(snk_env h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        EnvDev &d = h->d;
        for (void *p : {(void *)d.frames, (void *)d.ring, (void *)d.state, (void *)d.ep_reward,
                        (void *)d.out_reward, (void *)d.out_done, (void *)d.out_mask, (void *)d.out_dirs,
                        (void *)d.out_ep_reward, (void *)d.out_score, (void *)d.fault_count, (void *)d.ctl,
                        (void *)h->init_board, (void *)h->food, (void *)h->scratch, (void *)h->gather})
            dfree(p);
        delete h;
    });
}

extern "C" int snk_env_reset(snk_env h, const uint8_t *mask_host) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "env is NULL");
        hipStream_t s = stream();
        const uint8_t *m = nullptr;
        if (mask_host) {
            SNK_HIP(hipMemcpyAsync(h->scratch, mask_host, h->d.n, hipMemcpyHostToDevice, s));
            m = h->scratch;
        }
        env_reset_kernel<<<ceil_div(h->d.n, 256), 256, 0, s>>>(h->d, m);
        launch_check("env_reset_kernel");
        SNK_HIP(hipStreamSynchronize(s));
    });
}

extern "C" int snk_env_step(snk_env h, const uint8_t *act_dev, int32_t act_mode) {
    return guard([&] {
        SNK_CHECK(h && act_dev, SNK_ERR_INVALID, "env/act is NULL");
        SNK_CHECK(act_mode == SNK_ACT_INDEX || act_mode == SNK_ACT_DIRECTION, SNK_ERR_INVALID,
                  "bad act_mode %d", act_mode);
        hipStream_t s = stream();
        env_launch_step(h->d, act_dev, act_mode, nullptr, s);
        env_launch_advance(h->d, nullptr, s);
    });
}

extern "C" int snk_env_outputs(snk_env h, float **reward, uint8_t **done, uint8_t **mask,
                               uint8_t **dirs, float **ep_reward, uint8_t **score) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "env is NULL");
        if (reward) *reward = h->d.out_reward;
        if (done) *done = h->d.out_done;
        if (mask) *mask = h->d.out_mask;
        if (dirs) *dirs = h->d.out_dirs;
        if (ep_reward) *ep_reward = h->d.out_ep_reward;
        if (score) *score = h->d.out_score;
    });
}

static void env_gather(snk_env h, int nf, int8_t *host) {
    hipStream_t s = stream();
    const int64_t total = h->d.n * nf * (int64_t)h->d.bs * h->d.bs;
    env_gather_kernel<<<std::min<int64_t>(ceil_div(total, 256), 4096), 256, 0, s>>>(h->d, nf, h->gather);
    launch_check("env_gather_kernel");
    SNK_HIP(hipMemcpyAsync(host, h->gather, total, hipMemcpyDeviceToHost, s));
    SNK_HIP(hipStreamSynchronize(s));
}

extern "C" int snk_env_get_boards(snk_env h, int8_t *boards_host) {
    return guard([&] {
        SNK_CHECK(h && boards_host, SNK_ERR_INVALID, "NULL argument");
        env_gather(h, 1, boards_host);
    });
}

extern "C" int snk_env_get_states(snk_env h, int8_t *states_host) {
    return guard([&] {
        SNK_CHECK(h && states_host, SNK_ERR_INVALID, "NULL argument");
        env_gather(h, h->d.C, states_host);
    });
}

extern "C" int snk_env_get_scalars(snk_env h, int32_t *score, int32_t *len, int32_t *steps,
                                   int32_t *prev_dir, uint8_t *lost, float *ep_reward) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "env is NULL");
        const int64_t n = h->d.n;
        std::vector<EnvState> st(n);
        std::vector<float> er(n);
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(st.data(), h->d.state, n * sizeof(EnvState), hipMemcpyDeviceToHost, s));
        SNK_HIP(hipMemcpyAsync(er.data(), h->d.ep_reward, n * sizeof(float), hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
        for (int64_t e = 0; e < n; ++e) {
            if (score) score[e] = st[e].score;
            if (len) len[e] = st[e].len;
            if (steps) steps[e] = st[e].steps;
            if (prev_dir) prev_dir[e] = st[e].flags & 3;
            if (lost) lost[e] = (st[e].flags >> 2) & 1;
            if (ep_reward) ep_reward[e] = er[e];
        }
    });
}

extern "C" int snk_env_get_snake(snk_env h, int64_t e, int32_t *cells_host, int32_t *len_out) {
    return guard([&] {
        SNK_CHECK(h && e >= 0 && e < h->d.n, SNK_ERR_INVALID, "bad env index");
        EnvState st;
        std::vector<uint16_t> ring(h->d.ring_cap);
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(&st, h->d.state + e, sizeof st, hipMemcpyDeviceToHost, s));
        SNK_HIP(hipMemcpyAsync(ring.data(), h->d.ring + e * h->d.ring_cap, ring.size() * 2,
                               hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
        if (len_out) *len_out = st.len;
        if (cells_host)
            for (int k = 0; k < st.len; ++k) cells_host[k] = ring[(st.head + k) % h->d.ring_cap];
    });
}

extern "C" int snk_env_check_faults(snk_env h, int64_t *count_out) {
    int st = guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "env is NULL");
        uint32_t c = 0;
        hipStream_t s = stream();
        SNK_HIP(hipMemcpyAsync(&c, h->d.fault_count, sizeof c, hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
        if (count_out) *count_out = c;
        SNK_CHECK(c == 0, SNK_ERR_FOOD_EXHAUSTED,
                  "%u env-steps found the food list exhausted (reference: BoundsError at utils.jl:37)", c);
    });
    return st;
}

extern "C" int snk_env_synth_actions(snk_env h, uint64_t seed, uint8_t *act_dev) {
    return guard([&] {
        SNK_CHECK(h && act_dev, SNK_ERR_INVALID, "NULL argument");
        env_synth_kernel<<<ceil_div(h->d.n, 256), 256, 0, stream()>>>(h->d, seed, act_dev);
        launch_check("env_synth_kernel");
    });
}

extern "C" int snk_env_info(snk_env h, int64_t *n, int32_t *bs, int32_t *C, int64_t *t) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "env is NULL");
        if (n) *n = h->d.n;
        if (bs) *bs = h->d.bs;
        if (C) *C = h->d.C;
        if (t) {
            Ctl c;
            hipStream_t s = stream();
            SNK_HIP(hipMemcpyAsync(&c, h->d.ctl, sizeof c, hipMemcpyDeviceToHost, s));
            SNK_HIP(hipStreamSynchronize(s));
            *t = c.t;
        }
    });
}

// internal accessor for the other translation units
namespace snk {
const EnvDev &env_dev(snk_env h) { return h->d; }
}

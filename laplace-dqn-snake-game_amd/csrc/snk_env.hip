// snk_env.hip — batched Snake environment on gfx950.
//
// One fused kernel per lockstep step of n envs implements step!
// (utils.jl:100-109: move_wrapper! -> grow_maybe! -> sample_food! /
// remove_tail! -> check_collision -> update_board!) plus virtual_step's
// suicidal mask (utils.jl:112-132), auto-reset (utils.jl:199 `SnakeGame()`),
// optionally store! of the transition into the replay ring (utils.jl:267-277)
// and the trainer's episode statistics (utils.jl:478).
//
// Mapping: a workgroup of 2 waves owns 64 envs (NE).
//   Phase A  all 128 threads stream the 64 current boards (16-byte pieces,
//            consecutive threads -> consecutive bytes) HBM -> registers, where
//            they stay until phase C; LDS gets a 2-bit copy (value + 1 per cell).
//            Wave 0 first issues its lanes' state / action / episode-reward loads
//            so their latency hides under the board stream;
//   Phase B  wave 0, lane e = env e, runs the scalar logic against the packed
//            UNMODIFIED board: O(1) collision (board[new_head] replaces the
//            reference's O(L) body scan), food-list probe, next-state suicidal
//            mask. The <= 3 changed cells (tail -> 0, head -> 1, food -> 2) are
//            recorded as patches, and the logic reads the new board through them;
//   Phase C  every thread patches its register pieces and writes the new boards
//            to the frame ring and, when storing, b_{t-C}..b_t into the replay
//            slot (b_{t-1} read from HBM in the same pass).
// The boards live in registers (13 pieces per thread at 20x20), so LDS (a 6.4 KB
// packed copy) does not cap the envs in flight: 4-5 waves per SIMD = 512-640 envs
// per CU. Per env-step HBM traffic is 2 * pitch + 45 B (+ (C + 1) * pitch written
// and (C - 1) * pitch read when storing): every board byte is touched once in each
// direction; the body ring is touched once (one entry read, one written).
// The last workgroup to arrive (agent-scope ticket) advances the step counter
// and the replay count, and reduces the per-workgroup episode partials in
// workgroup order (deterministic), so a step is ONE launch.
#include <algorithm>
#include <vector>

#include "snk_internal.hpp"

namespace snk {

// envs per workgroup: 64, or 32 for batches up to ENV_NE_SMALL_MAX envs (4096 envs in 64
// workgroups left 3/4 of the CUs idle on a latency-bound step; 128 workgroups finish sooner)
constexpr int ENV_NE = 64, ENV_NT = 128, ENV_NE_SMALL = 32;
constexpr int64_t ENV_NE_SMALL_MAX = 16384;
// Profiling builds only (make clocks): per-workgroup phase timestamps (100 MHz realtime
// counter) into a debug buffer, read back by snk_env_debug_clocks.
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_env_clk;
#define ENV_CLK(slot) \
    do { if (threadIdx.x == 0 && g_env_clk) g_env_clk[(int64_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define ENV_CLK1(slot) \
    do { if (threadIdx.x == 64 && g_env_clk) g_env_clk[(int64_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define ENV_CLK(slot) do { } while (0)
#define ENV_CLK1(slot) do { } while (0)
#endif
typedef int i32x4 __attribute__((ext_vector_type(4)));   // native vector: register arrays stay in VGPRs

// utils.jl:25-34: first list entry (in list order) whose cell is empty
template <class Cell>
__device__ __forceinline__ int food_search(const Cell &cell, const int16_t *food, int n_food, uint64_t used) {
    for (int k = 0; k < n_food; ++k)
        if (!((used >> k) & 1ull) && cell(food[k]) == 0) return k;
    return -1;
}
template <class Cell>
__device__ __forceinline__ bool has_empty(const Cell &cell, int ncell) {
    for (int c = 0; c < ncell; ++c)
        if (cell(c) == 0) return true;
    return false;
}

// the 16 board bytes [base, base + 16) with patch p (cell pc[p], value p) applied, p ascending
__device__ __forceinline__ i32x4 patch16(i32x4 v, int base, const int16_t *pc) {
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const int off = pc[p] - base;
        if ((unsigned)off < 16u) {
            const int w = off >> 2, sh = (off & 3) * 8;
            const int keep = ~(0xff << sh), val = p << sh;
            v[0] = w == 0 ? (v[0] & keep) | val : v[0];
            v[1] = w == 1 ? (v[1] & keep) | val : v[1];
            v[2] = w == 2 ? (v[2] & keep) | val : v[2];
            v[3] = w == 3 ? (v[3] & keep) | val : v[3];
        }
    }
    return v;
}

__device__ __forceinline__ void st_sc1(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t wave_sum_i64(int64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max_f32(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_max_i32(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

// board cell c from the packed LDS copy (2-bit codes, value + 1: -1 wall .. 2 food)
__device__ __forceinline__ int cell_at(const uint32_t *bp, int c) {
    return (int)((bp[c >> 4] >> ((c & 15) * 2)) & 3u) - 1;
}
// 16 board bytes -> 16 2-bit codes (byte + 1, carry-free per byte)
__device__ __forceinline__ uint32_t pack16(const i32x4 v) {
    uint32_t out = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t x = (uint32_t)v[w];
        const uint32_t inc = (((x & 0x7f7f7f7fu) + 0x01010101u) ^ (x & 0x80808080u)) & 0x03030303u;
        const uint32_t cmp = (inc | (inc >> 6) | (inc >> 12) | (inc >> 18)) & 0xffu;
        out |= cmp << (8 * w);
    }
    return out;
}

// The act head of env e (head_kernel<HEAD_ACT>'s arithmetic to the bit), thread t = 0..3 of
// the env's quad of adjacent lanes: the thread owns Dense1 outputs o = 4t + i + 16m (i, m =
// 0..3; float4 loads of each slab row); h = bias + slabs in slab order, relu; Dense2's sum in
// wave_sum's butterfly order over o (xor 32, 16, 8, 4, 2, 1): 32 and 16 pair outputs the thread
// owns, 8 and 4 pair thread t with t ^ 2 and t ^ 1 (DPP quad permutes; both partners form the
// same commutative sums), 2 and 1 are local again. Writes h1, q, the action (act_out and the
// workgroup's LDS slot).
typedef float envf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float quad_xor(float v, int x) {
    const int o = x == 1 ? __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false)    // [1,0,3,2]
                         : __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false);   // [2,3,0,1]
    return __builtin_bit_cast(float, o);
}
__device__ __forceinline__ void env_act_head(const EnvActHead &H, int64_t n, int64_t e, int t, bool valid, int64_t step,
                                             uint8_t *s_slot) {
    constexpr int KMAX = 8;
    const int64_t es = valid ? e : 0;
    // epsilon first: loaded behind the early returns below it was one more memory round trip
    // after the Q values, on the step's critical path
    const float eps = H.eps_dev ? *H.eps_dev : H.epsilon;
    envf4 z[KMAX][4];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
        if (k < H.ks)
#pragma unroll
            for (int m = 0; m < 4; ++m)
                z[k][m] = *reinterpret_cast<const envf4 *>(H.slab + ((int64_t)k * n + es) * 64 + 16 * m + 4 * t);
    envf4 h[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        h[m] = *reinterpret_cast<const envf4 *>(H.b1 + 16 * m + 4 * t);
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (k < H.ks) h[m] += z[k][m];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[m][i] = h[m][i] > 0.0f ? h[m][i] : 0.0f;
    }
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float v[4];   // (p[o] + p[o + 32]) + (p[o + 16] + p[o + 48]), o = 4t + i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float p[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) p[m] = H.w2[a * 64 + 16 * m + 4 * t + i] * h[m][i];
            v[i] = (p[0] + p[2]) + (p[1] + p[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + quad_xor(v[i], 2);   // o ^ 8: thread t ^ 2
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + quad_xor(v[i], 1);   // o ^ 4: thread t ^ 1
        q[a] = H.b2[a] + ((v[0] + v[2]) + (v[1] + v[3]));                 // o ^ 2, o ^ 1
    }
    if (!valid) return;
#pragma unroll
    for (int m = 0; m < 4; ++m) *reinterpret_cast<envf4 *>(H.h1 + e * 64 + 16 * m + 4 * t) = h[m];
    if (t != 0) return;
    H.q[e * 3 + 0] = q[0];
    H.q[e * 3 + 1] = q[1];
    H.q[e * 3 + 2] = q[2];
    // utils.jl:161-169: Float32(rand()) < epsilon ? rand(av) : av[argmax(Q)] (head_kernel's draw)
    const float u = rng_uniform(rng_hash(H.seed, (uint64_t)e, (uint64_t)step));
    int act;
    if (u < eps) {
        act = (int)((rng_hash(H.seed ^ 0xA5A5A5A5A5A5A5A5ULL, (uint64_t)e, (uint64_t)step) >> 32) % 3);
    } else {
        act = 0;   // argmax: first maximum
        if (q[1] > q[act]) act = 1;
        if (q[2] > q[act]) act = 2;
    }
    H.act_out[e] = (uint8_t)act;
    *s_slot = (uint8_t)act;
}

// Boards stay in the registers of the thread that loaded them (NPT 16-byte pieces per
// thread, 13 at 20x20); LDS holds only a 2-bit copy for the logic lanes (100 B per env at
// 20x20), so LDS no longer caps the envs in flight: 2-wave workgroups, 5 per SIMD.
template <int PITCH>
constexpr int env_waves_per_simd() { return PITCH > 304 ? 4 : 5; }   // the register budget of NPT pieces

// HEAD: the act head runs here first (EnvActHead; four threads per env: NE * 4 == ENV_NT);
// the occupancy bound is dropped (these grids fill a quarter of the SIMDs at most)
template <int PITCH, int NE = ENV_NE, bool HEAD = false>
__global__ __launch_bounds__(ENV_NT, HEAD ? 1 : env_waves_per_simd<PITCH>()) void env_step_kernel(
    EnvDev E, const uint8_t *__restrict__ act, int act_mode, ReplayDev R, int store, EpisodeAcc acc, int with_acc,
    EnvActHead H) {
    constexpr int NCH = PITCH / 16, NPT = (NE * NCH + ENV_NT - 1) / ENV_NT;
    __shared__ uint32_t sbp[NE * NCH];                              // packed boards
    __shared__ __attribute__((aligned(8))) int16_t s_pc[NE * 4];   // patch cells (tail, head, food), -1 = none
    __shared__ uint8_t s_flag[NE];                                  // bit0 stepped, bit1 reset
    __shared__ int16_t s_food[64];
    __shared__ float s_epr[NE];   // finished episodes: reward (NaN = not finished), score
    __shared__ uint8_t s_score[NE];
    __shared__ uint8_t s_act[NE];   // HEAD: the actions
    ENV_CLK(0);
    const int tid = threadIdx.x;
    const bool w0 = tid < 64;
    const int lane = tid & 63;
    const int64_t e0 = (int64_t)blockIdx.x * NE;
    const int ne = (int)min((int64_t)NE, E.n - e0);
    const int64_t t = E.ctl->t;
    const int cur = (int)(t % 3), nxt = (int)((t + 1) % 3), prv = (int)((t + 2) % 3);
    const int64_t rc = store ? *R.count : 0;
    const int bs = E.bs, cap = E.ring_cap;

    // ---- wave 0: per-env loads first (state, action, episode reward) ----
    const bool live = w0 && lane < ne;
    const int64_t e = e0 + lane;
    EnvState st{};
    int a = 0, head_cell = 0, tail_cell = 0, tail_next = 0, tail_idx = 0;
    float epr0 = 0.0f;
    if (live) {
        st = E.state[e];
        if (!HEAD) a = act[e];
        epr0 = E.ep_reward[e];
        head_cell = (int)st.head_cell;
        tail_cell = (int)st.tail_cell;
        tail_next = (int)st.tail_next;   // the new tail unless the snake eats
    }
    if (w0 && lane < E.n_food) s_food[lane] = E.food[lane];
    ENV_CLK(1);

    // ---- Phase A: current boards HBM -> registers (+ packed copy in LDS) ----
    // slot-major ring: the workgroup's 64 boards of a slot are one contiguous 64 * PITCH run
    const int8_t *fcur = E.frames + ((int64_t)cur * E.n + e0) * PITCH;
    int8_t *fnxt = E.frames + ((int64_t)nxt * E.n + e0) * PITCH;
    const int8_t *fprv = E.frames + ((int64_t)prv * E.n + e0) * PITCH;
    i32x4 vcur[NPT];
#pragma clang loop unroll(full)
    for (int k = 0; k < NPT; ++k) {
        const int idx = tid + k * ENV_NT;
        if (idx < ne * NCH) vcur[k] = *reinterpret_cast<const i32x4 *>(fcur + idx * 16);
    }
    if constexpr (HEAD) {   // with the board loads in flight; the barrier below publishes s_act
        static_assert(NE * 4 == ENV_NT, "four threads per env");
        const int el = tid >> 2;
        env_act_head(H, E.n, e0 + el, tid & 3, el < ne, t, s_act + el);
    }
#pragma clang loop unroll(full)
    for (int k = 0; k < NPT; ++k) {
        const int idx = tid + k * ENV_NT;
        if (idx < ne * NCH) sbp[idx] = pack16(vcur[k]);
    }
    __syncthreads();
    ENV_CLK(2);

    // ---- Phase B: per-env logic (wave 0, lane = env) ----------------------
    bool done_out = false;
    float epr_out = 0.0f;
    int score_out = 0;
    if (live) {
        if (HEAD) a = s_act[lane];
        uint8_t flag = 0;
        int16_t pc[3] = {-1, -1, -1};
        const uint32_t *bp = sbp + lane * NCH;
        const int prev = st.flags & 3;
        if (!(st.flags & 4)) {
            flag = 1;
            const int dir = act_mode == SNK_ACT_INDEX ? avail_action(prev, a % 3) : (a & 3);
            uint16_t *ring = E.ring + e * cap;
            // the cell after the new tail (next step's tail_next), read now, used at the end
            tail_idx = (int)st.head + (int)st.len - 1;
            if (tail_idx >= cap) tail_idx -= cap;
            const int ring2 = ring[tail_idx >= 2 ? tail_idx - 2 : tail_idx - 2 + cap];
            // grow_maybe! (utils.jl:66-81)
            const int nh = head_cell + dir_delta(bs, dir);
            const int old = cell_at(bp, nh);
            const bool eat = old == 2;
            float reward = eat ? 1.0f : -0.01f;
            uint64_t used = st.food_used;
            int food_cell = -1;
            bool fault = false;
            int score = st.score;
            auto cell_old = [&](int c) { return cell_at(bp, c); };
            if (eat) {
                score += 1;
                const int k = food_search(cell_old, s_food, E.n_food, used);   // pre-update board
                if (k >= 0) {
                    used |= 1ull << k;
                    food_cell = s_food[k];
                } else if (has_empty(cell_old, bs * bs)) {
                    fault = true;   // utils.jl:37 BoundsError in the reference
                }
            }
            // check_collision (utils.jl:55-58) after the tail pop; truncation
            // utils.jl:88 with length(board_history) = n_frames + steps - 1
            const bool body = old == 1 && !(!eat && nh == tail_cell);
            const int steps = st.steps + 1;
            const bool lost = old == -1 || body || dir == (prev ^ 1) || (E.C + steps - 1 > E.max_hist);
            if (lost) reward = -1.0f;
            // update_board! (utils.jl:43-52) as patches, applied in this order
            pc[0] = eat ? -1 : (int16_t)tail_cell;
            pc[1] = (int16_t)nh;
            pc[2] = (int16_t)food_cell;
            auto cell_new = [&](int c) {
                return c == food_cell ? 2 : c == nh ? 1 : (!eat && c == tail_cell) ? 0 : cell_at(bp, c);
            };
            const int nhead = st.head == 0 ? cap - 1 : st.head - 1;
            ring[nhead] = (uint16_t)nh;
            const int nlen = st.len + (eat ? 1 : 0);
            const int ntail_cell = eat ? tail_cell : tail_next;
            // virtual_step (utils.jl:112-132): would each next action lose?
            uint8_t mask = 7;
            if (!lost) {
                mask = 0;
                const bool trunc2 = E.C + steps > E.max_hist;
                for (int k2 = 0; k2 < 3; ++k2) {
                    const int nh2 = nh + dir_delta(bs, avail_action(dir, k2));
                    const int v = cell_new(nh2);
                    const bool veat = v == 2;
                    const bool vbody = v == 1 && !(!veat && nh2 == ntail_cell);
                    if (v == -1 || vbody || trunc2) mask |= (uint8_t)(1 << k2);
                    if (veat && food_search(cell_new, s_food, E.n_food, used) < 0 && has_empty(cell_new, bs * bs))
                        fault = true;   // the virtual step's sample_food! would throw too
                }
            }
            const float epr = epr0 + reward;
            const uint8_t dirs = (uint8_t)(prev | (dir << 2) | ((lost ? 1 : 0) << 4));
            E.out_reward[e] = reward;
            E.out_done[e] = lost;
            E.out_mask[e] = mask;
            E.out_dirs[e] = dirs;
            E.out_ep_reward[e] = epr;
            E.out_score[e] = (uint8_t)score;
            done_out = lost;
            epr_out = epr;
            score_out = score;
            if (fault) atomicAdd(E.fault_count, 1u);
            // store! in env order (utils.jl:267-277): with more envs than capacity, only the
            // last cap transitions of the step survive it, so only they are written (the
            // overwritten ones would otherwise race on their slots)
            if (store && E.n - e <= R.cap) {
                const int64_t slot = (rc + e) % R.cap;
                R.reward[slot] = reward;
                R.act[slot] = (uint8_t)(act_mode == SNK_ACT_INDEX ? a % 3 : avail_index(prev, dir));
                R.done[slot] = lost;
                R.mask[slot] = mask;
                R.dirs[slot] = dirs;
            }
            if (lost && E.autoreset) {
                flag |= 2;
                const EnvState ns = EnvState::fresh(bs);
                ring[0] = (uint16_t)((bs - 3) + bs);   // structs.jl:47 (bs-2, 2)
                ring[1] = (uint16_t)((bs - 2) + bs);   //              (bs-1, 2)
                E.state[e] = ns;
                E.ep_reward[e] = 0.0f;
            } else {
                EnvState ns{};
                ns.food_used = used;
                ns.head = (uint16_t)nhead;
                ns.len = (uint16_t)nlen;
                ns.steps = (uint16_t)steps;
                ns.flags = (uint8_t)(dir | (lost ? 4 : 0) | ((fault || (st.flags & 8)) ? 8 : 0));
                ns.score = (uint8_t)score;
                ns.head_cell = (uint64_t)nh;
                ns.tail_cell = (uint64_t)ntail_cell;
                ns.tail_next = (uint64_t)(eat ? tail_next : nlen == 2 ? nh : ring2);
                E.state[e] = ns;
                E.ep_reward[e] = epr;
            }
        } else {
            // lost and not auto-reset: the game is over, nothing moves
            E.out_reward[e] = 0.0f;
            E.out_done[e] = 1;
            E.out_mask[e] = 7;
            E.out_dirs[e] = (uint8_t)(prev | (prev << 2) | (1 << 4));
            E.out_ep_reward[e] = epr0;
            E.out_score[e] = st.score;
            done_out = true;
            epr_out = epr0;
            score_out = st.score;
        }
        s_flag[lane] = flag;
        s_epr[lane] = done_out ? epr_out : __builtin_nanf("");
        s_score[lane] = (uint8_t)score_out;
        s_pc[lane * 4 + 0] = pc[0];
        s_pc[lane * 4 + 1] = pc[1];
        s_pc[lane * 4 + 2] = pc[2];
    }
    __syncthreads();

    ENV_CLK(3);
    // ---- arrival (wave 1, which stored nothing yet): partials (write-through), ticket ----
    // Every wave read ctl / R.count before the first barrier. Only the partial stores are
    // drained before the ticket; the last arriver reduces after its share of phase C.
    bool is_last = false;
    if (tid >= 64 && tid < 128) {
        if (with_acc) {
            const bool d = lane < ne && !__builtin_isnan(s_epr[lane]);
            const float er = d ? s_epr[lane] : 0.0f;
            const int sc = d ? s_score[lane] : 0;
            const int64_t cnt = wave_sum_i64(d ? 1 : 0);
            const int64_t ssum = wave_sum_i64(sc);
            const double rsum = wave_sum_f64((double)er);
            const float rmax = wave_max_f32(d ? er : -INFINITY);
            const int smax = wave_max_i32(sc);
            if (lane < 4) {
                const uint64_t word = lane == 0 ? (uint64_t)cnt
                                    : lane == 1 ? (uint64_t)ssum
                                    : lane == 2 ? (uint64_t)__double_as_longlong(rsum)
                                                : ((uint64_t)(uint32_t)__float_as_uint(rmax) |
                                                   ((uint64_t)(uint32_t)smax << 32));
                st_sc1(E.part + (int64_t)blockIdx.x * 4 + lane, word);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // with statistics: ONE counter (the partials' hand-off: release by the drained sc1
        // stores above, acquire by the last arriver's sc1 loads). Without: shard k =
        // blockIdx % 8 counts its workgroups, the last of a shard adds to the top counter
        // (8 shards: no single word serialises 4096 arrivals)
        const int nwg = (int)gridDim.x;
        uint32_t last = 0;
        if (lane == 0) {
            if (with_acc) {
                last = __hip_atomic_fetch_add(E.ticket + 8 * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                       (uint32_t)(nwg - 1);
            } else {
                const int k = (int)(blockIdx.x & 7);
                const uint32_t size_k = (uint32_t)((nwg - k + 7) >> 3);
                if (__hip_atomic_fetch_add(E.ticket + k * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    size_k - 1) {
                    __hip_atomic_store(E.ticket + k * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    last = __hip_atomic_fetch_add(E.ticket + 8 * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                           (uint32_t)(min(nwg, 8) - 1);
                }
            }
        }
        is_last = __shfl(last, 0, 64) != 0;
        ENV_CLK1(4);
    }

    // ---- Phase C: patched boards -> frame ring (+ replay slot) -----------
    // in groups of PG pieces per thread: the b_{t-1} loads of a group go out together
    constexpr int PG = 2;
    const bool rd_prv = store && R.C == 2;
#pragma clang loop unroll(full)
    for (int k0 = 0; k0 < NPT; k0 += PG) {
        i32x4 vp[PG];
        if (rd_prv) {
#pragma clang loop unroll(full)
            for (int k = 0; k < PG; ++k) {
                const int idx = tid + (k0 + k) * ENV_NT;
                if (k0 + k < NPT && idx < ne * NCH) {
                    vp[k] = *reinterpret_cast<const i32x4 *>(fprv + idx * 16);
                }
            }
        }
#pragma clang loop unroll(full)
        for (int k = 0; k < PG; ++k) {
            const int idx = tid + (k0 + k) * ENV_NT;
            if (k0 + k < NPT && idx < ne * NCH) {
                const int el = idx / NCH, c = idx - el * NCH;
                const int64_t ge = e0 + el;
                const uint8_t f = s_flag[el];
                const i32x4 vc = vcur[k0 + k];
                const i32x4 vnew = (f & 1) ? patch16(vc, c * 16, s_pc + el * 4) : vc;
                if (store && (f & 1) && E.n - ge <= R.cap) {
                    const int64_t slot = (rc + ge) % R.cap;
                    int8_t *rf = R.frames + slot * (int64_t)(R.C + 1) * PITCH + c * 16;
                    if (rd_prv) {
                        *reinterpret_cast<i32x4 *>(rf) = vp[k];
                        *reinterpret_cast<i32x4 *>(rf + PITCH) = vc;
                        *reinterpret_cast<i32x4 *>(rf + 2 * PITCH) = vnew;
                    } else {
                        *reinterpret_cast<i32x4 *>(rf) = vc;
                        *reinterpret_cast<i32x4 *>(rf + PITCH) = vnew;
                    }
                }
                if (f & 2) {
                    // auto-reset: next state is (b0, b0) (structs.jl:53 n_frames copies)
                    const i32x4 v0 = *reinterpret_cast<const i32x4 *>(E.init_board + c * 16);
                    *reinterpret_cast<i32x4 *>(fnxt + idx * 16) = v0;
                    if (E.C == 2) *reinterpret_cast<i32x4 *>(E.frames + ((int64_t)cur * E.n + e0) * PITCH + idx * 16) = v0;
                } else {
                    *reinterpret_cast<i32x4 *>(fnxt + idx * 16) = vnew;
                }
            }
        }
    }

#ifdef SNK_ENV_CLOCKS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ENV_CLK(5);
    ENV_CLK1(6);
#endif
    if (!is_last) return;
    if (with_acc) {
        int64_t cnt = 0, ssum = 0;
        double rsum = 0.0;
        float rmax = -INFINITY;
        int smax = 0;
        for (int g0 = 0; g0 < (int)gridDim.x; g0 += 64) {
            const int g = g0 + lane;
            int64_t c1 = 0, s1 = 0;
            double r1 = 0.0;
            float m1 = -INFINITY;
            int sm1 = 0;
            if (g < (int)gridDim.x) {
                const uint64_t *p = E.part + (int64_t)g * 4;
                c1 = (int64_t)ld_sc1(p);
                s1 = (int64_t)ld_sc1(p + 1);
                r1 = __longlong_as_double((long long)ld_sc1(p + 2));
                const uint64_t w3 = ld_sc1(p + 3);
                m1 = __uint_as_float((uint32_t)w3);
                sm1 = (int)(uint32_t)(w3 >> 32);
            }
            cnt += wave_sum_i64(c1);
            ssum += wave_sum_i64(s1);
            rsum += wave_sum_f64(r1);
            rmax = fmaxf(rmax, wave_max_f32(m1));
            smax = max(smax, wave_max_i32(sm1));
        }
        if (lane == 0) {
            *acc.episodes += cnt;
            *acc.reward_sum += rsum;
            *acc.score_sum += ssum;
            if (cnt > 0) {
                *acc.reward_max = fmaxf(*acc.reward_max, rmax);
                *acc.score_max = max(*acc.score_max, smax);
            }
            *acc.env_steps += E.n;
        }
    }
    if (lane == 0) {
        E.ctl->t = t + 1;
        if (store) *R.count = rc + E.n;
        __hip_atomic_store(E.ticket + 8 * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// reset! for masked envs: SnakeGame() board in all 3 frame slots
__global__ void env_reset_kernel(EnvDev E, const uint8_t *__restrict__ mask) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E.n || (mask && !mask[e])) return;
    for (int s = 0; s < 3; ++s) {
        int8_t *fr = E.frames + ((int64_t)s * E.n + e) * E.pitch;
        for (int c = 0; c < E.pitch; c += 16)
            *reinterpret_cast<int4 *>(fr + c) = *reinterpret_cast<const int4 *>(E.init_board + c);
    }
    uint16_t *ring = E.ring + e * E.ring_cap;
    ring[0] = (uint16_t)((E.bs - 3) + E.bs);
    ring[1] = (uint16_t)((E.bs - 2) + E.bs);
    E.state[e] = EnvState::fresh(E.bs);
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
        out[i] = E.frames[((int64_t)slot * E.n + e) * E.pitch + c];
    }
}

__global__ void env_synth_kernel(EnvDev E, uint64_t seed, uint8_t *__restrict__ act) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= E.n) return;
    act[e] = (uint8_t)((rng_hash(seed, (uint64_t)e, (uint64_t)E.ctl->t) >> 32) % 3);
}

template <int P>
static void env_step_launch_p(bool small, bool head, int grid, hipStream_t s, const EnvDev &E, const uint8_t *act,
                              int act_mode, const ReplayDev &r, int store, const EpisodeAcc &ea, int wa,
                              const EnvActHead &H) {
    if constexpr (P <= 256) {
        if (small && head) {
            env_step_kernel<P, ENV_NE_SMALL, true><<<grid, ENV_NT, 0, s>>>(E, act, act_mode, r, store, ea, wa, H);
            return;
        }
        if (small) {
            env_step_kernel<P, ENV_NE_SMALL><<<grid, ENV_NT, 0, s>>>(E, act, act_mode, r, store, ea, wa, H);
            return;
        }
    }
    env_step_kernel<P, ENV_NE><<<grid, ENV_NT, 0, s>>>(E, act, act_mode, r, store, ea, wa, H);
}

bool env_act_head_ok(const EnvDev &E, int ks) {
    return E.n <= ENV_NE_SMALL_MAX && E.pitch <= 256 && ks >= 1 && ks <= 8;
}

void env_launch_step(const EnvDev &E, const uint8_t *act, int act_mode, const ReplayDev *R, hipStream_t s,
                     const EpisodeAcc *acc, const EnvActHead *head) {
    ReplayDev r{};
    if (R) r = *R;
    EpisodeAcc ea{};
    if (acc) ea = *acc;
    const int wa = acc ? 1 : 0;
    const bool small = E.n <= ENV_NE_SMALL_MAX && E.pitch <= 256;
    const int grid = (int)ceil_div(E.n, small ? ENV_NE_SMALL : ENV_NE);
    const int store = R ? 1 : 0;
    EnvActHead H{};
    if (head) {
        SNK_CHECK(env_act_head_ok(E, head->ks) && act_mode == SNK_ACT_INDEX && head->act_out == act && head->slab &&
                      head->b1 && head->w2 && head->b2 && head->h1 && head->q,
                  SNK_ERR_INTERNAL, "env step: fused act head");
        H = *head;
    }
#define SNK_ENV_CASE(P) \
    case P: env_step_launch_p<P>(small, head != nullptr, grid, s, E, act, act_mode, r, store, ea, wa, H); break;
    switch (E.pitch) {
        SNK_ENV_CASE(48) SNK_ENV_CASE(64) SNK_ENV_CASE(96) SNK_ENV_CASE(112) SNK_ENV_CASE(128)
        SNK_ENV_CASE(144) SNK_ENV_CASE(176) SNK_ENV_CASE(208) SNK_ENV_CASE(240) SNK_ENV_CASE(256)
        SNK_ENV_CASE(304) SNK_ENV_CASE(336) SNK_ENV_CASE(368) SNK_ENV_CASE(400)
        default: SNK_CHECK(false, SNK_ERR_INVALID, "unsupported board pitch %d", E.pitch);
    }
#undef SNK_ENV_CASE
    launch_check("env_step_kernel");
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
        d.ticket = dalloc<uint32_t>(9 * 32);
        d.part = dalloc<uint64_t>((size_t)ceil_div(n, ENV_NE_SMALL) * 4);
        SNK_HIP(hipMemsetAsync(d.ticket, 0, 9 * 32 * sizeof(uint32_t), s));
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
                        (void *)d.ticket, (void *)d.part,
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

#ifdef SNK_ENV_CLOCKS
// profiling builds: out[g][8] = the phase stamps of the LAST step launch (call after it)
extern "C" int snk_env_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 8);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 8 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_env_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
#endif

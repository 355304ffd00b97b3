// snk_internal.hpp — device-side data layout of libsnakehip.
//
// HBM layout (all SoA, sized for 288 GB HBM3E):
//   env frames  int8  [3][n][pitch]   ring of the last 3 boards, slot-major (a slot of
//                                     all envs is one contiguous stream)
//   env ring    u16   [n][bs*bs]      snake body ring (head index moves down)
//   env state   16 B  [n]             EnvState below (one 128-bit load/store)
//   replay      int8  [cap][C+1][pitch] + SoA metadata [cap]
// Boards are Julia column-major (cell = i + j*bs, 0-based), so a frame is the
// same bytes as the reference's board Matrix{Int} narrowed to Int8.
#pragma once
#include "snk_common.hpp"

namespace snk {

enum Dir : int { DIR_U = 0, DIR_D = 1, DIR_L = 2, DIR_R = 3 };  // utils.jl:8 order

struct alignas(16) EnvState {
    // word 0
    uint64_t food_used : 50;  // consumed entries of the shared food list (n_food = 50)
    uint64_t head_cell : 9;   // board cell of the head   (= ring[head]; bs <= 20: cell < 400)
    uint64_t flags : 4;       // bits 0-1 prev_dir, bit 2 lost, bit 3 faulted
    uint64_t pad0 : 1;
    // word 1
    uint64_t head : 9;        // ring index of the head (pushfirst! decrements)
    uint64_t len : 9;         // snake length (<= bs^2)
    uint64_t steps : 16;      // real steps of the current episode (max_hist < 60000)
    uint64_t score : 8;
    uint64_t tail_cell : 9;   // board cell of the tail (= ring[head + len - 1])
    uint64_t tail_next : 9;   // the cell the tail moves to (= ring[head + len - 2])
    uint64_t pad1 : 4;
    // head, tail and next-tail cells ride in the state: a step issues its one body-ring
    // read (the tail's next-but-one, for the NEXT step) after the state has arrived and
    // consumes it only when it writes the new state
    __host__ __device__ static EnvState fresh(int bs) {   // structs.jl:47 snake (bs-2, 2), (bs-1, 2)
        EnvState s{};
        s.head = 0;
        s.len = 2;
        s.head_cell = (uint64_t)((bs - 3) + bs);
        s.tail_cell = (uint64_t)((bs - 2) + bs);
        s.tail_next = s.head_cell;
        return s;
    }
};
static_assert(sizeof(EnvState) == 16, "EnvState must be 16 bytes");

// Step/replay control words kept on the device so a captured hipGraph can
// advance them without host involvement.
struct alignas(16) Ctl {
    int64_t t;             // global env step counter: current board in slot t % 3
    int64_t replay_count;  // transitions ever stored (slot = count % cap)
    int64_t updates;       // DQN updates done (target sync / epsilon schedule)
    int64_t iter;          // trainer iterations
};

struct EnvDev {
    int64_t n;
    int bs, C, pitch, max_hist, autoreset, n_food, ring_cap;
    int8_t *frames;       // [3][n][pitch]: slot (t % 3) of env e at (slot * n + e) * pitch
    uint16_t *ring;       // [n][ring_cap]
    EnvState *state;      // [n]
    float *ep_reward;     // [n] running episode reward (utils.jl:207)
    // outputs of the last step
    float *out_reward;    // [n]
    uint8_t *out_done;    // [n]
    uint8_t *out_mask;    // [n] 3 suicidal bits of the next state (virtual_step)
    uint8_t *out_dirs;    // [n] prev_dir | dir<<2 | lost<<4
    float *out_ep_reward; // [n] episode reward including this step
    uint8_t *out_score;   // [n] score after this step (before auto-reset)
    const int16_t *food;  // [n_food] shared Xoshiro(42) food list (cells)
    const int8_t *init_board;  // [pitch] SnakeGame() board b0
    uint32_t *fault_count;
    Ctl *ctl;
    uint32_t *ticket;     // arrival counters of the step kernel's workgroups, 0 between launches:
                          // [k * 32] shard k = blockIdx % 8, [8 * 32] the top / single counter
    uint64_t *part;       // [ceil(n / 64)][4] per-workgroup episode statistics (EpisodeAcc)
};

// Trainer statistics the step kernel folds in (episode_stats, utils.jl:478): the
// last workgroup to finish reduces the per-workgroup partials in workgroup order.
struct EpisodeAcc {
    int64_t *episodes, *score_sum, *env_steps;
    double *reward_sum;
    float *reward_max;
    int32_t *score_max;
};

struct ReplayDev {
    int64_t cap;
    int bs, C, pitch;
    int8_t *frames;   // [cap][C+1][pitch]: b_{t-C} .. b_t
    float *reward;    // [cap]
    uint8_t *act;     // [cap] action index into available_actions (255 = not available)
    uint8_t *done;    // [cap]
    uint8_t *mask;    // [cap] suicidal bits
    uint8_t *dirs;    // [cap] prev_dir | dir<<2 | lost<<4
    int64_t *count;   // device: transitions ever stored (slot = count % cap)
};

__host__ __device__ inline int dir_delta(int bs, int d) {
    return d == DIR_U ? -1 : d == DIR_D ? 1 : d == DIR_L ? -bs : bs;
}
// utils.jl:7-10: the i-th surviving action of [U, D, L, R] after removing
// the reverse of prev_dir.
__host__ __device__ inline int avail_action(int prev_dir, int idx) {
    int rev = prev_dir ^ 1;
    return idx + (idx >= rev ? 1 : 0);
}
__host__ __device__ inline int avail_index(int prev_dir, int dir) {
    int rev = prev_dir ^ 1;
    if (dir == rev) return 255;
    return dir - (dir > rev ? 1 : 0);
}

// sample(rpb) (utils.jl:280-287) for a batch of <= 64: Floyd's algorithm on the counter
// stream, one wave (lane n draws t_n; a ballot finds an earlier equal pick)
struct SampleRider {
    const int64_t *count = nullptr;   // transitions stored so far (device)
    int64_t cap = 0, pending = 0;     // pending: transitions the coming step stores
    int32_t batch = 0;
    uint64_t seed = 0, draw = 0;
    const int64_t *draw_dev = nullptr;
    int64_t *out = nullptr;           // [batch] slots; nullptr: no rider
    int32_t *b_out = nullptr;
};
__device__ inline void sample_wave(const SampleRider &r) {
    const int lane = threadIdx.x & 63;
    const uint64_t draw = r.draw_dev ? (uint64_t)*r.draw_dev : r.draw;
    const int64_t len = min(*r.count + r.pending, r.cap);
    const int B = (int)min((int64_t)r.batch, len);
    const int64_t t = lane < B ? (int64_t)__umul64hi(rng_hash(r.seed, draw, (uint64_t)lane), (uint64_t)(len - B + lane + 1))
                               : -1;
    int64_t v = -2;
    for (int n = 0; n < B; ++n) {   // n is wave-uniform: v_readlane, not an LDS permute
        const int64_t tn = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)t >> 32), n) << 32) |
                                     (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)t, n));
        const bool hit = __ballot(lane < n && v == tn) != 0;
        if (lane == n) v = hit ? len - B + n : tn;
    }
    if (lane < B) r.out[lane] = v;
    if (lane == 0 && r.b_out) *r.b_out = B;
}
// Launch helpers implemented in the .hip files. One launch is a whole lockstep
// step: its last workgroup also advances ctl->t (and the replay count when
// storing) and, with acc, folds the finished episodes into the trainer stats.
// head (the trainer's act step, small lockstep batches): the act head of the act forward runs
// in the step kernel (head_kernel<HEAD_ACT>'s arithmetic to the bit) and writes act itself
struct EnvActHead {
    const float *slab = nullptr;   // the act forward's Dense1 slabs [ks][n][64]
    int ks = 0;
    const float *b1 = nullptr, *w2 = nullptr, *b2 = nullptr;   // Dense1 bias, Dense2 weights [3][64], bias
    float *h1 = nullptr, *q = nullptr;                        // outputs [n][64], [n][3]
    uint8_t *act_out = nullptr;                               // the actions (the step's act argument)
    uint64_t seed = 0;
    const float *eps_dev = nullptr;
    float epsilon = 0.0f;
};
// whether env_launch_step can run the act head for this env batch (and ks slabs)
bool env_act_head_ok(const EnvDev &E, int ks);
void env_launch_step(const EnvDev &E, const uint8_t *act, int act_mode, const ReplayDev *R,
                     hipStream_t s, const EpisodeAcc *acc = nullptr, const EnvActHead *head = nullptr);

}  // namespace snk

// snk_internal.hpp — device-side data layout of libsnakehip.
//
// HBM layout (all SoA, sized for 288 GB HBM3E):
//   env frames  int8  [n][3][pitch]   ring of the last 3 boards per env
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
    uint64_t food_used;  // consumed entries of the shared food list (<= 64)
    uint16_t head;       // ring index of the head (pushfirst! decrements)
    uint16_t len;        // snake length
    uint16_t steps;      // real steps of the current episode
    uint8_t flags;       // bits 0-1 prev_dir, bit 2 lost, bit 3 faulted
    uint8_t score;
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
    int8_t *frames;       // [n][3][pitch]
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

// Launch helpers implemented in the .hip files
void env_launch_step(const EnvDev &E, const uint8_t *act, int act_mode, const ReplayDev *R,
                     hipStream_t s);
void env_launch_advance(const EnvDev &E, const ReplayDev *R, hipStream_t s);

}  // namespace snk

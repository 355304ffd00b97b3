/*
 * snakehip.h — C ABI of libsnakehip, the MI355X (gfx950) hot path of
 * lucagiorgetti/Laplace-DQN-Snake-game.
 *
 * Drop-in boundary: the reference is Julia with no FFI; its "API" is a set of
 * generic functions over mutable structs. Each entry point
 * below names the reference function it replaces (file:line). A Julia host
 * binds them with `ccall`; tests bind them with ctypes.
 *
 * Conventions
 *  - Every function returns int status (SNK_OK = 0); on failure a
 *    thread-local message is available from snk_last_error().
 *  - Pointers named *_dev are device pointers (snk_malloc, or any HIP device
 *    allocation of this process); pointers named *_host are host memory.
 *  - Boards are Julia column-major: cell = (i-1) + (j-1)*board_size for the
 *    reference's 1-based board[i, j]; values -1 wall, 0 empty, 1 snake, 2 food.
 *  - Directions use the order of utils.jl:8: 0=U(-1,0) 1=D(1,0) 2=L(0,-1)
 *    3=R(0,1). An "action index" is the position in available_actions().
 *  - Work is enqueued on the library stream (snk_set_stream); functions that
 *    return data to host memory synchronise that stream.
 */
#ifndef SNAKEHIP_H
#define SNAKEHIP_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SNK_OK 0
#define SNK_ERR_INVALID 1          /* bad argument */
#define SNK_ERR_FOOD_EXHAUSTED 2   /* utils.jl:37 board[0] = 2 -> BoundsError */
#define SNK_ERR_HIP 3              /* HIP runtime error */
#define SNK_ERR_NOMEM 4
#define SNK_ERR_STATE 5            /* e.g. structs.jl:154 batch_size > capacity */
#define SNK_ERR_INTERNAL 6

#define SNK_ACT_INDEX 0            /* actions are indices into available_actions */
#define SNK_ACT_DIRECTION 1        /* actions are absolute directions (play_snake.jl) */

/* ---------------------------------------------------------------- runtime */
const char *snk_last_error(void);
int snk_version(int32_t *version_out);
int snk_device_count(int32_t *n_out);
int snk_set_device(int32_t device);
/* hipStream_t to enqueue on; NULL restores the library's own stream */
int snk_set_stream(void *hip_stream);
int snk_synchronize(void);
int snk_malloc(void **dev_out, int64_t bytes);
int snk_free(void *dev);
int snk_memcpy_h2d(void *dst_dev, const void *src_host, int64_t bytes);
int snk_memcpy_d2h(void *dst_host, const void *src_dev, int64_t bytes);
int snk_memset(void *dev, int32_t value, int64_t bytes);

/* structs.jl:111 — the 50-entry food list drawn from Xoshiro(seed):
 * (rand(rng, 2:bs-1), rand(rng, 2:bs-1)) per entry, returned as cells. */
int snk_food_list(int32_t board_size, uint32_t seed, int32_t n, int32_t *cells_host);

/* ---------------------------------------------------------------- env
 * A batch of n independent SnakeGame()s stepped in lockstep
 * (structs.jl:47-141 SnakeGame; utils.jl:7-149 env methods). */
typedef struct snk_env_s *snk_env;

/* SnakeGame(board_size, n_frames, discount, Xoshiro(food_seed)) for n envs.
 * max_hist: utils.jl:88 `length(board_history) > 500` truncation (500).
 * autoreset: 1 = a lost env restarts as SnakeGame() on its next step. */
int snk_env_create(snk_env *out, int64_t n_envs, int32_t board_size, int32_t n_frames,
                   uint32_t food_seed, int32_t max_hist, int32_t autoreset);
int snk_env_destroy(snk_env env);
/* reset! — re-create SnakeGame() for envs with mask_host[e] != 0 (NULL = all) */
int snk_env_reset(snk_env env, const uint8_t *mask_host);
/* step! (utils.jl:100-109) fused with virtual_step (utils.jl:112-132) for every
 * env. act_dev: [n] uint8 action index (SNK_ACT_INDEX) or direction
 * (SNK_ACT_DIRECTION). Results stay on the device (snk_env_outputs). */
int snk_env_step(snk_env env, const uint8_t *act_dev, int32_t act_mode);
/* Device pointers of the last step's outputs, each [n]:
 *   reward f32, done u8, mask u8 (bit k: k-th next available action suicidal),
 *   dirs u8 (prev_dir | dir<<2 | lost<<4), ep_reward f32 (episode reward
 *   including this step), score u8 (score after this step). */
int snk_env_outputs(snk_env env, float **reward, uint8_t **done, uint8_t **mask, uint8_t **dirs,
                    float **ep_reward, uint8_t **score);
/* game.board for every env: boards_host [n][bs*bs] int8 */
int snk_env_get_boards(snk_env env, int8_t *boards_host);
/* assemble_state! (utils.jl:135-139): states_host [n][n_frames][bs*bs] int8, oldest first */
int snk_env_get_states(snk_env env, int8_t *states_host);
/* per-env scalars: score, snake length, steps of the episode, prev_dir, lost */
int snk_env_get_scalars(snk_env env, int32_t *score, int32_t *len, int32_t *steps,
                        int32_t *prev_dir, uint8_t *lost, float *ep_reward);
/* snake body (snake[1] = head) of env e, cells_host [>= len] */
int snk_env_get_snake(snk_env env, int64_t e, int32_t *cells_host, int32_t *len_out);
/* number of env-steps whose food sampling hit utils.jl:37 (list exhausted);
 * returns SNK_ERR_FOOD_EXHAUSTED when > 0 */
int snk_env_check_faults(snk_env env, int64_t *count_out);
/* synthetic action indices hash(seed, env, step) % 3 (bench/test workloads) */
int snk_env_synth_actions(snk_env env, uint64_t seed, uint8_t *act_dev);
int snk_env_info(snk_env env, int64_t *n, int32_t *board_size, int32_t *n_frames, int64_t *t);

/* ---------------------------------------------------------------- replay
 * ReplayBuffer (structs.jl:145-157) with store! (utils.jl:267-277),
 * sample (utils.jl:280-287) and stack_exp (utils.jl:343-383). Each slot holds
 * the n_frames+1 boards b_{t-C}..b_t of one transition plus its metadata. */
typedef struct snk_replay_s *snk_replay;

int snk_replay_create(snk_replay *out, int64_t capacity, int32_t board_size, int32_t n_frames,
                      int32_t batch_size);
int snk_replay_destroy(snk_replay rb);
/* env step + store in one fused kernel (the hot path) */
int snk_env_step_store(snk_env env, const uint8_t *act_dev, int32_t act_mode, snk_replay rb);
/* store! of B explicit transitions (host arrays). frames_host [B][C+1][bs*bs]
 * b_{t-C}..b_t; act = index into available_actions at action time. */
int snk_replay_store(snk_replay rb, int64_t B, const int8_t *frames_host, const uint8_t *act_host,
                     const float *reward_host, const uint8_t *done_host, const uint8_t *mask_host,
                     const uint8_t *dirs_host);
int snk_replay_length(snk_replay rb, int64_t *len_out);   /* Base.length */
int snk_replay_position(snk_replay rb, int64_t *count_out);
int snk_replay_empty(snk_replay rb);                       /* empty_buffer! */
/* sample without replacement: B = min(batch_size, length) distinct indices */
int snk_replay_sample(snk_replay rb, uint64_t seed, uint64_t draw, int64_t *idx_dev, int32_t *B_out);
/* stack_exp: Float32 states/next_states (bs,bs,C,B) Julia memory, 1-based
 * action indices like utils.jl:363, rewards, dones, suicidal mask [B][3]. */
int snk_replay_gather(snk_replay rb, const int64_t *idx_dev, int64_t B, float *states_dev,
                      int32_t *actions_dev, float *rewards_dev, float *next_states_dev,
                      uint8_t *dones_dev, uint8_t *mask_dev, uint8_t *dirs_dev);

#ifdef __cplusplus
}
#endif
#endif

/*
 * snake_oracle.h — CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference Julia code of
 * lucagiorgetti/Laplace-DQN-Snake-game, used ONLY as the checker by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg. Nothing in the
 * product path (laplace-dqn-snake-game_amd/) links, loads or calls this.
 *
 * Pinning:
 *   - Xoshiro(42) food list + RNG state: pinned bit-exact against
 *     /root/reference/trainers/very_long_training1.bson (fixture
 *     tests/golden/bson_vanilla.json).
 *   - step!/collision/food path: pinned against both best-game GIFs
 *     (fixtures tests/golden/gif_*.npz) — every frame reproduced.
 *   - Q-net forward: pinned through the argmax KAT (129/129 greedy actions of
 *     the vanilla GIF with the BSON weights).
 *   - backward / RMSProp / Welford / Gram: parity UNPINNED against the
 *     reference (Flux/Zygote/Optimisers are not runnable here and the
 *     reference ships no fixture for them); checked by finite differences.
 *
 * Conventions: boards are Julia column-major, 0-based cell c = (i-1)+(j-1)*bs
 * for the reference's 1-based board[i, j] (i = row, 1 = top). Directions are
 * coded in the order of utils.jl:8: 0=U(-1,0) 1=D(1,0) 2=L(0,-1) 3=R(0,1).
 */
#ifndef SNAKE_ORACLE_H
#define SNAKE_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_MAX_CELLS 400   /* bs <= 20 */
#define ORC_MAX_FOOD 64

/* ---- Julia Random.Xoshiro restatement ---------------------------------- */
void orc_julia_xoshiro_seed(uint32_t seed, uint64_t state5[5]);
uint64_t orc_xoshiro_next(uint64_t st[4]);
int64_t orc_rand_range(uint64_t st[4], int64_t a, int64_t b);
/* structs.jl:70 — n pairs (rand(rng,2:bs-1), rand(rng,2:bs-1)); cells out */
void orc_food_list(int bs, uint32_t seed, int n, int32_t *cells, uint64_t st_after[4]);

/* ---- env (structs.jl:33-99, utils.jl:7-149) ---------------------------- */
typedef struct orc_game {
    int32_t bs, n_frames, max_hist;
    int32_t len;            /* snake length */
    int32_t prev_dir, dir;
    int32_t score, lost, steps, fault;
    int32_t hist_len;       /* length(game.board_history) */
    float reward, episode_reward;
    int32_t n_food;
    int32_t food[ORC_MAX_FOOD];
    int16_t snake[ORC_MAX_CELLS + 2];    /* snake[0] = head */
    int8_t hist[3][ORC_MAX_CELLS];       /* [0]=b_t (board) [1]=b_{t-1} [2]=b_{t-2} */
} orc_game;

int orc_game_sizeof(void);
void orc_game_init(orc_game *g, int bs, int n_frames, int max_hist,
                   const int32_t *food, int n_food);
int orc_available_actions(int prev_dir, int32_t out[3]);
/* step!(game, action) with an absolute direction; returns 0, or 2 when the
 * reference would throw BoundsError in sample_food! (utils.jl:37) */
int orc_step(orc_game *g, int dir);
/* virtual_step (utils.jl:112-132): suicidal flags for the 3 next actions */
void orc_virtual_mask(const orc_game *g, uint8_t mask[3]);

/* Batched driver: N independent games, lockstep, auto-reset after done.
 * One call = one env step of every game with action INDICES act[e] in 0..2
 * (index into available_actions(prev_dir), utils.jl:7-10).
 * Per env outputs: reward, done, suicidal mask (3 bytes), dir taken, prev_dir
 * at action time, and the n_frames+1 frames b_{t-C}..b_t (oldest first). */
typedef struct orc_batch orc_batch;
orc_batch *orc_batch_create(int n, int bs, int n_frames, int max_hist,
                            const int32_t *food, int n_food);
void orc_batch_destroy(orc_batch *b);
int orc_batch_step(orc_batch *b, const uint8_t *act, float *reward, uint8_t *done,
                   uint8_t *mask3, uint8_t *dir_taken, uint8_t *prev_dir,
                   int8_t *frames /* [n][C+1][bs*bs] or NULL */);
void orc_batch_boards(const orc_batch *b, int8_t *boards /* [n][bs*bs] */);
void orc_batch_scalars(const orc_batch *b, int32_t *score, int32_t *len,
                       int32_t *steps, int32_t *prev_dir, float *ep_reward);
/* current Q-net input state (C frames, oldest first) of every env */
void orc_batch_states(const orc_batch *b, int8_t *states /* [n][C][bs*bs] */);

/* counter RNG shared by product and oracle for synthetic actions */
uint64_t orc_splitmix64(uint64_t x);
uint32_t orc_synth_action(uint64_t seed, uint64_t env, uint64_t step);

/* ---- Q-net (structs.jl:127-139), Flux destructure param order ------------ */
int64_t orc_qnet_nparams(int bs, int C);
/* x: [B][C][bs][bs] Julia (bs,bs,C,B) memory, q: [B][3] */
void orc_qnet_forward(int bs, int C, const float *params, int B, const double *x, double *q);
/* grad += sum_b sum_a dq[b][a] * dq[b][a]/dtheta  (grad zeroed by caller) */
void orc_qnet_backward(int bs, int C, const float *params, int B, const double *x,
                       const double *dq, double *grad);
/* utils.jl:448-466 one DQN loss+grad (TD target promoted to Float64) */
double orc_dqn_loss_grad(int bs, int C, const float *q_params, const float *t_params, int B,
                         const double *s, const int32_t *a_idx, const float *r,
                         const double *s_next, const uint8_t *done, const uint8_t *mask3,
                         double gamma, double *grad, double *target_out);
/* kink-aware variants (test infrastructure): relu decisions per sample
 * [B][orc_qnet_relu_count] = a1 | a2 | a3 (channel-major) | h1; relu_in NULL =
 * the reference's z > 0; relu_out / margin_out (z / sum|terms|) may be NULL */
int64_t orc_qnet_relu_count(int bs, int C);
void orc_qnet_backward_ex(int bs, int C, const float *params, int B, const double *x, const double *dq,
                          double *grad, const uint8_t *relu_in, uint8_t *relu_out, double *margin_out);
double orc_dqn_loss_grad_ex(int bs, int C, const float *q_params, const float *t_params, int B,
                            const double *s, const int32_t *a_idx, const float *r,
                            const double *s_next, const uint8_t *done, const uint8_t *mask3,
                            double gamma, double *grad, double *target_out,
                            const uint8_t *relu_in, uint8_t *relu_out, double *margin_out);
/* ---- deeper bf16 Q-net (BASELINE configs[2], builder-defined; see the .c) -- */
int64_t orc_deep_nparams(int bs, int C);
void orc_deep_forward(int bs, int C, const float *params, int B, const double *x, double *q);
void orc_deep_backward(int bs, int C, const float *params, int B, const double *x, const double *dq,
                       double *grad);
double orc_deep_loss_grad(int bs, int C, const float *q_params, const float *t_params, int B,
                          const double *s, const int32_t *a_idx, const float *r, const double *s_next,
                          const uint8_t *done, const uint8_t *mask3, double gamma, double *grad,
                          double *target_out);
/* Optimisers.RMSProp apply! in Float32 (utils.jl:429,466) */
void orc_rmsprop(int64_t P, float *theta, float *acc, const float *grad,
                 float eta, float rho, float eps);

/* ---- Laplace (compute_D.jl:9-31,67-81; plot_traj.jl:10-16) -------------- */
/* D: P x K column-major (K columns of length P). Welford over columns in
 * Float64, then D .-= mean. mean/var out (var = m2 / max(n-1,1)). */
void orc_welford_center(int64_t P, int K, double *D, double *mean, double *var);
/* G = D' * D  (K x K, column-major) */
void orc_gram(int64_t P, int K, const double *D, double *G);

#ifdef __cplusplus
}
#endif
#endif

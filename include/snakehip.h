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
#define SNK_ERR_STATE 5            /* e.g. structs.jl:113 batch_size > capacity */
#define SNK_ERR_INTERNAL 6

#define SNK_ACT_INDEX 0            /* actions are indices into available_actions */
#define SNK_ACT_DIRECTION 1        /* actions are absolute directions (play_snake.jl) */

/* ---------------------------------------------------------------- runtime */
const char *snk_last_error(void);
int snk_version(int32_t *version_out);
/* sha256 (hex) of the sources this library was linked from: the csrc .hip and .hpp files, this
   header and csrc/Makefile, as `sha256sum <sorted files> | sha256sum` in csrc/ (build provenance) */
const char *snk_build_source_sha256(void);
int snk_device_count(int32_t *n_out);
int snk_set_device(int32_t device);
/* hipStream_t to enqueue on; NULL restores the library's own stream */
int snk_set_stream(void *hip_stream);
int snk_synchronize(void);
/* GEMM arithmetic selection, process-wide (no reference counterpart: the
 * reference computes in Flux fp32). Every knob defaults to the production
 * path; tests switch one to compare the production kernel against an
 * alternative of the same error class. Read when a kernel is launched (a
 * captured trainer graph keeps what it was captured with); SNK_ARITH_CONV_FP32
 * is read when a model is created. value: 0 or 1. */
#define SNK_ARITH_X6S 0          /* 1: conv3 x6 forward on conv_x6s (4 samples in LDS); 0: x6m16 */
#define SNK_ARITH_H3S 1          /* 1: act-forward conv3 on the fp16 h3 split; 0: bf16 x6 */
#define SNK_ARITH_DH3 2          /* 1: act-forward Dense1 on dense_h3_kernel; 0: x6 GEMM */
#define SNK_ARITH_H3C2 3         /* 1: conv2 fused into the h3 act forward (conv_h3f); 0: conv3 only */
#define SNK_ARITH_CONV_FP32 4    /* 1: models created from now on use native f32 MFMA (no split) */
#define SNK_ARITH_SYRK_H3_32 5   /* 1: Jacobian Gram on the round-2 32x32x16 kernel; 0: syrk_h3q */
#define SNK_ARITH_UPD_HEAD 6     /* 1: the update's heads run in upd_fwd_kernel's tail; 0: head_pair_kernel (same bits) */
#define SNK_ARITH_ENV_HEAD 7     /* 1: the trainer's act head runs in env_step_kernel; 0: head_kernel (same bits) */
#define SNK_ARITH_SPLIT_CHAIN 8  /* 1: the trainer's grad_update writes the next act forward's split weights; 0: w3_split every act */
#define SNK_ARITH_SYRK_KSPLIT 9  /* 1: Jacobian Gram on 256x256 tiles, K split into fp32 chunks summed in fp64; 0: SNK_ARITH_SYRK_H3_32's kernel */
#define SNK_ARITH_COUNT 10
int snk_set_arith(int32_t knob, int32_t value);
int snk_get_arith(int32_t knob, int32_t *value_out);
int snk_malloc(void **dev_out, int64_t bytes);
int snk_free(void *dev);
int snk_memcpy_h2d(void *dst_dev, const void *src_host, int64_t bytes);
int snk_memcpy_d2h(void *dst_host, const void *src_dev, int64_t bytes);
int snk_memset(void *dev, int32_t value, int64_t bytes);

/* structs.jl:70 — the 50-entry food list drawn from Xoshiro(seed):
 * (rand(rng, 2:bs-1), rand(rng, 2:bs-1)) per entry, returned as cells. */
int snk_food_list(int32_t board_size, uint32_t seed, int32_t n, int32_t *cells_host);

/* ---------------------------------------------------------------- env
 * A batch of n independent SnakeGame()s stepped in lockstep
 * (structs.jl:33-99 SnakeGame; utils.jl:7-149 env methods). */
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
 * ReplayBuffer (structs.jl:104-116) with store! (utils.jl:267-277),
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

/* ---------------------------------------------------------------- DQNModel
 * DQNModel (structs.jl:120-147): q_net, t_net = deepcopy(q_net) and the
 * RMSProp(lr) state. Parameters cross the ABI in Flux.destructure order
 * (per layer weight then bias, each column-major; Conv = true convolution). */
typedef struct snk_dqn_s *snk_dqn;

#define SNK_NET_Q 0          /* q_net */
#define SNK_NET_TARGET 1     /* t_net */
#define SNK_NET_OPT_STATE 2  /* RMSProp accumulator (Optimisers `quad`) */
#define SNK_NET_GRAD 3       /* gradient of the last loss */

/* DQNModel(board_size, 3; lr) with Flux's glorot_uniform init drawn from a
 * counter RNG seeded by init_seed; RMSProp(lr, rho, eps) = (5e-4, 0.9, 1e-8). */
int snk_dqn_create(snk_dqn *out, int32_t board_size, int32_t n_frames, float lr, float rho, float eps,
                   uint64_t init_seed);
/* BASELINE.json configs[2]: the deeper conv Q-net in bf16 (builder-defined; the
 * reference has none). It extends structs.jl:127-139 by one more 3x3 convolution
 * and wider channels:
 *   Conv(3,3,C=>32,relu;pad=1) Conv(3,3,32=>32,relu;pad=1) Conv(3,3,32=>64,relu;pad=1)
 *   Conv(6,6,64=>64,relu) flatten Dense((bs-5)^2*64=>64,relu) Dense(64=>3)
 * with conv / Dense1 weights and every conv activation in bf16, fp32 sums,
 * fp32 master weights, RMSProp and head. board_size 10, 12 or 20.
 * The handle answers every DQNModel and trainer entry point below, and
 * snk_laplace_snapshot / snk_laplace_sample_params; snk_jacobian,
 * snk_jacobian_gram(_shard), snk_laplace_sampling, snk_dqn_time_act_layers and
 * snk_dqn_last_q refuse it (SNK_ERR_INVALID). */
int snk_dqn_create_deep(snk_dqn *out, int32_t board_size, int32_t n_frames, float lr, float rho, float eps,
                        uint64_t init_seed);
/* measurement: average ms per launch of each stage of the deep net's
 * epsilon_greedy forward over env's batch (HIP events on the library stream),
 * ms_out[6]: [0] L0 + L1 + L2 (one fused bf16 MFMA launch, deep_front_kernel),
 * [1] = [2] = 0 (inside [0]), [3] L3 (deep_conv3_kernel), [4] Dense1, [5] head */
int snk_dqn_time_deep_layers(snk_dqn m, snk_env env, int32_t reps, double *ms_out);
int snk_dqn_destroy(snk_dqn m);
int snk_dqn_nparams(snk_dqn m, int64_t *P_out);
/* Flux.destructure / restructure: which = SNK_NET_* */
int snk_dqn_set_params(snk_dqn m, int32_t which, const float *flux_host);
int snk_dqn_get_params(snk_dqn m, int32_t which, float *flux_host);
/* device buffer (packed layout) of a SNK_NET_* vector; for
 * data-parallel gradient all-reduce and target broadcast */
int snk_dqn_buffer_ptr(snk_dqn m, int32_t which, float **packed_dev);
/* update_target_net! (utils.jl:174-177) */
int snk_dqn_sync_target(snk_dqn m);
/* m(x): x_dev Float32 (bs,bs,C,B) Julia memory -> q_dev (3,B) */
int snk_dqn_forward(snk_dqn m, int32_t which, const float *x_dev, int64_t B, float *q_dev);
/* Q of every env's assemble_state! -> q_dev [n][3] */
int snk_dqn_forward_env(snk_dqn m, int32_t which, snk_env env, float *q_dev);
/* epsilon_greedy (utils.jl:153-172) for every env: act_dev [n] action index */
int snk_dqn_act(snk_dqn m, snk_env env, float epsilon, uint64_t seed, uint8_t *act_dev);
/* measurement: average ms per launch of each stage of the epsilon_greedy
 * forward over env's batch, ms_out[5] = conv1, conv2, conv3, dense1, head
 * (HIP events on the library stream); when the forward fuses conv1 and conv2
 * into conv3 (conv_h3f_kernel) ms_out[0] is the conv3 weight-max scan,
 * ms_out[1] = 0 and ms_out[2] is the fused kernel */
int snk_dqn_time_act_layers(snk_dqn m, snk_env env, int32_t reps, double *ms_out);
/* measurement: average ms of the fused step(+store) kernel over reps real steps */
int snk_env_time_step(snk_env env, snk_replay rb_or_null, const uint8_t *act_dev, int32_t reps, double *ms_out);
/* Q of the last forward_env/act call, host [n][3] */
int snk_dqn_last_q(snk_dqn m, float *q_host, int64_t n);
/* test hook: the relu outputs of q_net in the last training forward (loss_grad,
 * update, or the trainer's last update): layer 0 a1 [B][bs*bs][16], 1 a2
 * [B][bs*bs][32], 2 a3 [B][(bs-5)^2][64], 3 h1 [B][64]; position = i + j*side
 * for board[i, j]. n floats from the start. */
int snk_dqn_train_activations(snk_dqn m, int32_t layer, float *host, int64_t n);
/* utils.jl:448-464: TD target on t_net (Float64, suicidal mask -> -100),
 * Huber loss (delta 1, mean) and its gradient into SNK_NET_GRAD, for the
 * replay slots idx_dev[B]. loss_host may be NULL (no synchronisation). */
int snk_dqn_loss_grad(snk_dqn m, snk_replay rb, const int64_t *idx_dev, int64_t B, double gamma,
                      double *loss_host);
/* the same for explicit stack_exp tensors (actions 1-based, mask [B][3]) */
int snk_dqn_loss_grad_batch(snk_dqn m, const float *states_dev, const int32_t *actions_dev,
                            const float *rewards_dev, const float *next_states_dev, const uint8_t *dones_dev,
                            const uint8_t *mask_dev, int64_t B, double gamma, double *loss_host);
/* Flux.update!(opt_state, q_net, grads) with the SNK_NET_GRAD buffer (utils.jl:466) */
int snk_dqn_apply_grad(snk_dqn m);
/* loss_grad + apply_grad */
int snk_dqn_update(snk_dqn m, snk_replay rb, const int64_t *idx_dev, int64_t B, double gamma,
                   double *loss_host);

/* ---------------------------------------------------------------- trainer
 * The batched train! loop (utils.jl:420-494) over a batch of envs. */
typedef struct snk_trainer_s *snk_trainer;
/* ABI guard: the caller sets struct_size = sizeof(the struct) as its first
 * field; the library refuses (SNK_ERR_INVALID) any other size, so a host
 * binding whose struct layout drifts from this header fails loudly instead of
 * being read past its end. snk_abi_sizes reports the sizes it expects. */
typedef struct {
    int32_t struct_size;        /* = sizeof(snk_trainer_cfg_t) = 64 */
    float epsilon;              /* structs.jl:165 epsilon = 1.0 */
    float epsilon_end;          /* 0.05 */
    float decay;                /* 1e-6, subtracted per update (utils.jl:480) */
    int32_t updates_per_iter;   /* DQN updates per lockstep env step */
    int64_t target_update_rate; /* 1000 (utils.jl:469) */
    double gamma;               /* 0.97 (utils.jl:451) */
    uint64_t seed;              /* counter-RNG seed for actions and sampling */
    int64_t loss_log_capacity;  /* ring of per-update losses (tr.losses) */
    int32_t graph_unroll;       /* lockstep iterations per captured hipGraph (0 = 8, at most 64) */
} snk_trainer_cfg_t;
typedef struct {
    int32_t struct_size;        /* = sizeof(snk_trainer_stats_t) = 80, set by the caller */
    int64_t episodes, score_sum, updates, nb, env_steps;
    double reward_sum, last_loss;
    float reward_max;
    int32_t score_max;
    float epsilon;
} snk_trainer_stats_t;

/* sizeof(snk_trainer_cfg_t), sizeof(snk_trainer_stats_t) as compiled into the library */
int snk_abi_sizes(int64_t *trainer_cfg_size, int64_t *trainer_stats_size);
/* Trainer(; ...) (structs.jl:164-174) over a batch of games, a model and a replay buffer */
int snk_trainer_create(snk_trainer *out, snk_env env, snk_dqn m, snk_replay rb, const snk_trainer_cfg_t *cfg);
int snk_trainer_destroy(snk_trainer t);
/* iters lockstep iterations; learn = 0 is fill_buffer! (utils.jl:389-402);
 * use_graph = 1 replays one captured hipGraph per iteration */
int snk_trainer_run(snk_trainer t, int64_t iters, int32_t learn, int32_t use_graph);
/* one lockstep iteration with n_updates <= updates_per_iter updates (the last,
 * partial iteration of train! when n_batches + 1 is not a multiple) */
int snk_trainer_run_partial(snk_trainer t, int32_t n_updates);
/* the reference's batch counter nb: update_target_net! runs after an update
 * when nb % target_update_rate == 0, then nb += 1. train! starts at 0
 * (utils.jl:431,469), compute_D at 1 (compute_D.jl:56,134). Default 0. */
int snk_trainer_set_nb(snk_trainer t, int64_t nb);
/* test/trace hook: after every update the finished gradient (P floats, packed layout
 * of snk_dqn_buffer_ptr) is also copied to grad_ring_dev + slot * P, where
 * slot = (i x updates_per_iter + u) % slots for update u of iteration i, and i counts
 * the iterations of ONE launch sequence: within a captured graph (a graph replay
 * restarts at i = 0: graphs of graph_unroll iterations, then one graph of the
 * remaining iterations; only the latest remainder length stays cached) or within an eager snk_trainer_run call (i = 0, 1, ... mod 2^20).
 * A ring of graph_unroll x updates_per_iter slots therefore maps one graph replay
 * slot for slot. One device-to-device copy per update, appended to the same graphs
 * (which are re-captured). NULL turns it off. */
int snk_trainer_set_trace(snk_trainer t, float *grad_ring_dev, int64_t slots);
/* test/trace hook: after every iteration's act forward its actions (n_envs bytes,
 * action indices) are copied to act_ring_dev + slot * n_envs and, if q_ring_dev is
 * not NULL, its Q values (n_envs x 3 floats, [env][action]) to q_ring_dev +
 * slot * 3 n_envs, slot = i % slots with i as in snk_trainer_set_trace. NULL turns
 * it off. */
int snk_trainer_set_act_trace(snk_trainer t, uint8_t *act_ring_dev, float *q_ring_dev, int64_t slots);
int snk_trainer_stats(snk_trainer t, snk_trainer_stats_t *out);
/* tr.losses: loss of update u at host[u % loss_log_capacity] */
int snk_trainer_losses(snk_trainer t, double *host, int64_t n);
int snk_trainer_act_ptr(snk_trainer t, uint8_t **act_dev);
/* measurement: `iters` real (learning) trainer iterations, eager, each queued behind one
 * replay of the learning graph (no host wait between them), with HIP events recorded by the
 * dispatch of the act forward's fused conv kernel (conv_h3f_kernel) on the library stream:
 * *ms_out = its median duration inside the training loop (0 when this trainer's act forward
 * does not run it). The graph replays are real training steps too. */
int snk_trainer_time_act_kernel(snk_trainer t, int32_t iters, double *ms_out);

/* ---------------------------------------------------------------- multi-GPU
 * Data-parallel replicas (new: the reference is single-process). One process
 * per GPU; RCCL over xGMI. The 128-byte unique id is created on rank 0 and
 * shipped to the other ranks by the host (torch.distributed store/gloo). */
typedef struct snk_comm_s *snk_comm;
int snk_comm_unique_id(uint8_t *id128_host);
int snk_comm_create(snk_comm *out, int32_t nranks, int32_t rank, const uint8_t *id128_host);
int snk_comm_destroy(snk_comm c);
int snk_comm_allreduce_mean(snk_comm c, float *buf_dev, int64_t n);
int snk_comm_broadcast(snk_comm c, float *buf_dev, int64_t n, int32_t root);
/* what RCCL itself reports for the communicator (ncclCommCount / ncclCommUserRank), not the
 * arguments it was created with: the bench records it so a scaling run proves its rank count */
int snk_comm_info(snk_comm c, int32_t *nranks_out, int32_t *rank_out);
/* the trainer all-reduces (mean) the gradient of every update across the
 * communicator; broadcasts rank 0's q_net first. c = NULL detaches (updates
 * are local again; nothing is broadcast) */
int snk_trainer_set_comm(snk_trainer t, snk_comm c);

/* ---------------------------------------------------------------- Laplace D
 * compute_D.jl:33-142: the deviation matrix D (P x K, Float64, Julia
 * column-major: column pos = one Float64.(destructure(q_net)) snapshot,
 * contiguous), its Welford mean/var (compute_D.jl:9-31, duplicated at
 * la_utils.jl:14-36) and the Gram G = D'D (K x K) whose eigenvalues / (K-1)
 * are the spectrum plot_traj.jl:10-16 takes from svd(D). */
typedef struct snk_laplace_s *snk_laplace;
#define SNK_LAP_D 0      /* double [K][P] (= Julia P x K column-major) */
#define SNK_LAP_MEAN 1   /* double [P] */
#define SNK_LAP_VAR 2    /* double [P]  m2 / max(K-1, 1) */
#define SNK_LAP_GRAM 3   /* double [K][K] */
#define SNK_LAP_D32 4    /* float [K][ld32] fp32 copy of the centred D (MFMA operand) */
int snk_laplace_create(snk_laplace *out, int64_t n_params, int32_t K);
int snk_laplace_destroy(snk_laplace h);
/* compute_D.jl:67-71  deviation_matrix[:, pos] = Float64.(theta) (pos 0-based) */
int snk_laplace_snapshot(snk_laplace h, snk_dqn m, int32_t pos);
/* load / read one column (host doubles, P of them) */
int snk_laplace_set_column(snk_laplace h, int32_t pos, const double *col_host);
int snk_laplace_get(snk_laplace h, int32_t which, void *host, int64_t bytes);
int snk_laplace_buffer_ptr(snk_laplace h, int32_t which, void **dev_out, int64_t *ld_out);
/* compute_D.jl:74-81: fit! every column in order (Welford, Float64), then
 * deviation_matrix .-= mean; also refreshes the fp32 copy */
int snk_laplace_fit_center(snk_laplace h);
/* G = D'D (K x K): fp32 MFMA over the centred D, fp64 accumulation across
 * 1024-long k blocks and across the K-splits; ms_out (optional) = kernel ms */
int snk_laplace_gram(snk_laplace h, float *ms_out);

/* Per-sample Jacobians of the Q-net over replay slots (north_star "D = J'J";
 * the reference has no Jacobian): row s is
 * dQ(state of slot s)[a_s] / dtheta with a_s the stored action index, i.e.
 * the direction of the per-sample gradient of the Huber TD loss
 * (utils.jl:453-464). J_dev: float [n][n_params] in Flux.destructure order.
 * slots_dev: int64 [n] replay slots, NULL = slots 0..n-1. */
int snk_jacobian(snk_dqn m, snk_replay rb, const int64_t *slots_dev, int64_t n, float *J_dev);
/* G = J J' (n x n, float, full symmetric) over replay slots 0..n-1 without
 * materialising the Dense sections of J (rank-1 per sample:
 * G = Gc + (A3 A3' + 1) o (Z Z') + [a_i = a_j] o (H H' + 1), Gc the conv
 * sections' Gram on MFMA). ms_out (optional, 4 floats): forward + data
 * gradients, per-sample conv Jacobians, conv Gram, dense terms + mirror. */
int snk_jacobian_gram(snk_dqn m, snk_replay rb, int64_t n, float *G_dev, float *ms_out);

/* D(50k) across ranks: the n x n Gram's 128 x 128 lower-triangle
 * tiles are split into nranks contiguous runs of the XCD-aware tile order; each
 * rank computes every Jacobian row (cheap) and only its own tiles (+ their
 * mirror) into G_dev, leaving the rest untouched. ms_out as snk_jacobian_gram. */
int snk_jacobian_gram_shard(snk_dqn m, snk_replay rb, int64_t n, int32_t rank, int32_t nranks, float *G_dev,
                            float *ms_out);
/* the tiles of shard rank / nranks: count, and (optional) their top-left
 * (row, col) element pairs, tiles_host [2 * count] (host only, no device) */
int snk_gram_tiles(int64_t n, int32_t rank, int32_t nranks, int32_t *tiles_host, int64_t *count_out);
/* every rank's shard tiles onto root's G_dev (point-to-point over RCCL: each
 * rank packs its tiles and sends them on its own link; root unpacks and
 * mirrors). Collective: every rank of c calls it after its shard. */
int snk_jacobian_gram_gather(snk_comm c, int64_t n, float *G_dev, int32_t root);

/* ---------------------------------------------------------------- Laplace sampling
 * la_utils.jl:83-118. D, mean and var are the handle's (after
 * snk_laplace_fit_center: the centred deviation matrix and its Welford
 * statistics, la_utils.jl:161-167). Model n's weights:
 *   w = mean + 1/sqrt(2) * sqrt(|var|) .* z1 + 1/sqrt(2(K-1)) * D * z2   (fp64, term by term)
 * with z1 (P, Flux index) and z2 (K) from the counter-based normal stream
 * z(seed, n, stream 1|2, i) (the reference draws from the unseeded global RNG).
 */
/* the stream itself (tests): out_host[q] = z(seed, model, which, i0 + q) */
int snk_laplace_normals(uint64_t seed, int64_t model, int32_t which, int64_t i0, int64_t n, double *out_host);
/* sample_model (la_utils.jl:83-95): model n's weights in Flux.destructure order (Float32) */
int snk_laplace_sample_params(snk_laplace h, snk_dqn m, uint64_t seed, int64_t model, float *flux_host);
/* laplace_sampling! (la_utils.jl:97-118) with epsilon 0: tr_reward = greedy episode
 * reward of m's q_net; models 0..n_models-1 each play one greedy episode (lockstep,
 * `chunk` models at a time, 0 = up to 4096); the transitions of every model with
 * reward > tr_reward are appended to rb in (model, step) order.
 * rewards_host / lengths_host (optional, n_models): each model's episode. */
int snk_laplace_sampling(snk_laplace h, snk_dqn m, snk_replay rb, int64_t n_models, uint64_t seed, int64_t chunk,
                         float *tr_reward_out, int64_t *n_better_out, float *rewards_host, int32_t *lengths_host);

#ifdef __cplusplus
}
#endif
#endif

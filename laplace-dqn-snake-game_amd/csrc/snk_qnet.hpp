// snk_qnet.hpp — the DQNModel Q-net on the device (structs.jl:127-139).
//
//   Conv(3x3, C=>16, relu, pad 1) -> Conv(3x3, 16=>32, relu, pad 1)
//   -> Conv(6x6, 32=>64, relu) -> flatten -> Dense(64*(bs-5)^2 => 64, relu)
//   -> Dense(64 => 3)
//
// Parameters live on the device in a PACKED order (a per-section permutation
// of Flux.destructure's order, same section sizes and offsets): each conv
// weight is the GEMM matrix W[k][co] with k = (kk*Cin + ci), kk = du + KS*dv
// the input offset of a TRUE convolution (Flux flips the kernel:
// W[kk][ci][co] = w_flux[KS-1-du, KS-1-dv, ci, co]), immediately followed by
// its bias (so a weight-gradient GEMM with an extra all-ones row writes
// weight and bias gradients as one contiguous block); Dense1 is
// W[p*64 + c][o] matching the device activation layout [s][p][c].
// Activations: [sample][position p = i + j*H (column-major)][channel].
#pragma once
#include "snk_conv.hpp"
#include "snk_gemm.hpp"
#include "snk_internal.hpp"

namespace snk {

struct QLayout {
    int bs, C, ncell, Wo, K1;   // K1 = Wo*Wo*64 (Dense1 fan-in)
    int64_t off_w1, off_b1, off_w2, off_b2, off_w3, off_b3, off_d1w, off_d1b, off_d2w, off_d2b, P;
    // forward weight image [kk][out][in] of conv2, conv3, Dense1 (size T)
    int64_t off_t2, off_t3, off_td, T;
};
QLayout make_layout(int bs, int C);
// flux index of every packed index (host)
void packed_to_flux_index(const QLayout &L, int32_t *perm);
// theta -> forward weight image (after every change of theta)
// wtb (optional): the exact bf16 split planes of the image (3*T uint16) for the x6 kernels
void transpose_fwd_launch(const QLayout &L, const float *theta, float *wt, uint16_t *wtb, hipStream_t s);

// Source of the Q-net input planes: env frame ring, replay slots, or a
// float tensor in Julia (bs,bs,C,B) memory.
struct BoardSrc {
    const int8_t *base = nullptr;
    const float *fbase = nullptr;
    const int64_t *idx = nullptr;   // replay slot per sample
    const int64_t *tptr = nullptr;  // env frame-ring step counter
    int pitch = 0, C = 1, ncell = 0, chan0 = 0, replay_nf = 0;
    int64_t slot_stride = 0;        // env frame ring: bytes between frame slots (n * pitch)
    __device__ __forceinline__ float load(int64_t s, int c, int cell) const {
        if (fbase) return fbase[(s * C + c) * ncell + cell];
        return (float)plane(s, c)[cell];
    }
    // int8 plane of (sample, channel); nullptr in float mode. The env frame ring is
    // slot-major ([3][n][pitch], slot_stride = n * pitch): slot = (t + 3 - (C - 1 - c)) % 3
    __device__ __forceinline__ const int8_t *plane(int64_t s, int c) const {
        if (fbase) return nullptr;
        if (idx) return base + idx[s] * (int64_t)replay_nf * pitch + (int64_t)(c + chan0) * pitch;
        const int slot = (int)((*tptr + 3 - (C - 1 - c)) % 3);
        return base + slot * slot_stride + s * (int64_t)pitch;
    }
};

// Device workspace for one batch geometry
struct QWork {
    int64_t cap = 0, slab_floats = 0, cslab_floats = 0;
    float *a1 = nullptr, *a2 = nullptr, *a3 = nullptr, *slab = nullptr, *h1 = nullptr, *q = nullptr;
    float *cslab = nullptr;   // partial sums of kk-split convolutions
    uint16_t *a2b = nullptr;  // x6 forward: a2 as bf16 planes [S*ncell][3][32]
    uint16_t *a1b = nullptr;  // x6 forward: a1 as bf16 planes [S*ncell][3][16]
    // training only
    float *dq = nullptr, *dz1 = nullptr, *dz3 = nullptr, *dz2 = nullptr, *dzc1 = nullptr;
    float *x0 = nullptr;      // input planes as floats, written by the training forward's conv1
    int x0_valid = 0;         // set by the forward that wrote x0 (the unfused conv1 path)
    float *wmax_part = nullptr;      // h3 conv3: per-block partial max |w| of the conv3 weight image
    int wmax_n = 0;                  //   valid partials (conv1_fwd_kernel / wmax_scan_kernel wrote them)
    const float *wmax_img = nullptr; //   of this image
    int wmax_fresh = 0;              //   set by the trainer: the partials were written by the grad_update that
                                     //   last changed the image (the next full forward skips its scan; reset there)
    int split_fresh = 0;             // set by the trainer: w3h / w2h / w1h were written by the grad_update that
                                     //   last changed the image (UpdateTarget::s_*): the next act forward skips
                                     //   w3_split_kernel (reset there)
    float split_grow = 0.0f;         // set by the trainer: a bound on how far any weight can move before the
                                     //   next fresh split (the chained RMSProp steps x lr / sqrt(1 - rho), x2):
                                     //   w3_split_kernel caps its exponents so the chained splits cannot overflow
    uint16_t *w3h = nullptr;         // h3 conv3 weights pre-split for conv_h3f_kernel's LDS-DMA staging:
    int *w3e = nullptr;              //   [36 kk][512 16-byte chunks] in the B buffers' swizzled order, and their exponent
    uint16_t *w2h = nullptr;         //   (w3e[1]: conv2's) and conv2's weights pre-split into the B2 image bytes
    uint16_t *w1h = nullptr;         // Dense1's image pre-split for dense_h3_kernel ([Wo^2][2][64][64] halves),
    int *w1e = nullptr;              //   one exponent per (position, output)
    float *a3max = nullptr;          // per-sample max of a3 (conv_h3f_kernel's epilogue), Dense1's h3 row scale
    int dh3_ready = 0;               // a3, a3max, w1h / w1e are those of the last conv_h3f + w3_split forward
                                     //   (a Dense1-only call, e.g. the per-layer timing, may then use dense_h3)
    double *target = nullptr, *loss = nullptr;
    uint32_t *h3f_ticket = nullptr;  // persistent conv_h3f_kernel's group counter (zero between launches)
    uint32_t *upd_ticket = nullptr;  // training: per-sample arrivals of the update forward's four workgroups
                                     //   (upd_fwd_kernel phase 5), 0 between launches
    int has_train = 0;
    int64_t gen = 0;          // bumped on every reallocation (captured graphs hold the old pointers)
};

void qwork_ensure(QWork &w, const QLayout &L, int64_t S, bool train);
void qwork_free(QWork &w);

// Head epilogues
enum HeadMode { HEAD_Q = 0, HEAD_ACT = 1, HEAD_TARGET = 2, HEAD_LOSS = 3 };
struct HeadArgs {
    // ACT
    uint8_t *act = nullptr;
    float epsilon = 0.0f;
    uint64_t seed = 0;
    const int64_t *tptr = nullptr;
    const float *eps_dev = nullptr;   // if set, epsilon read from the device
    // TARGET / LOSS (replay metadata by slot)
    const int64_t *idx = nullptr;
    const float *rew = nullptr;
    const uint8_t *done = nullptr;
    const uint8_t *mask = nullptr;
    const uint8_t *act_idx = nullptr;
    double gamma = 0.97;
    double *target = nullptr;
    double *loss = nullptr;
    float *dq = nullptr;
    float *dz1 = nullptr;   // LOSS: also write Dense2's data gradient (the backward's first step)
    int64_t B = 0;
    // ACT: an extra workgroup runs this replay draw (the trainer's next update sample)
    SampleRider rider;
};

// forward: q[S][3] into w.q (and w.h1); mode-specific epilogue
// only = -1: the whole chain; 0..4: just conv1 / conv2 / conv3 / dense1 / head
// (inputs from a previous full forward; used for per-layer timing)
// one net's forward operands
struct FwdNet {
    const float *th, *wt;
    const uint16_t *wtb;
    BoardSrc src;
    QWork *w;
};
// conv1 .. Dense1 of two independent nets over S samples each, both in every launch (grid z/y = net)
void qnet_forward_pair(const QLayout &L, const FwdNet *net, int64_t S, hipStream_t s);
// measurement hook: when armed (a, b non-null), the act forward's conv_h3f_kernel launch is
// bracketed by hipEventRecord(a) / hipEventRecord(b) on its stream (eager launches only)
void h3f_timing_hook(hipEvent_t a, hipEvent_t b);
// the update's two forwards (net[0] = t_net on s', net[1] = q_net on s, which keeps the
// training activations) up to the Dense1 slabs: conv1-conv3 in one launch
// (snk_upd_fwd.hpp, with Dense1 at S <= 64) when the geometry allows, else the layer-by-layer
// path; returns the number of Dense1 partial slabs for the head
// (and, given `head` (HEAD_LOSS arguments), both heads in the same launch: returns 0)
int qnet_forward_update_pair(const QLayout &L, const FwdNet *net, int64_t S, hipStream_t s,
                             const HeadArgs *head = nullptr);
// TD-target head of t_net and loss head of q_net (HeadArgs as for HEAD_LOSS) in one launch,
// over ks Dense1 slabs (qnet_forward_update_pair's count)
void qnet_head_pair(const QLayout &L, const float *theta_t, QWork &wt, const float *theta_q, QWork &wq, int64_t S,
                    const HeadArgs &ha, hipStream_t s, int ks);
// the head (Dense1 bias + relu, Dense2, mode epilogue) after the layers
void qnet_head(const QLayout &L, const float *theta, int64_t S, QWork &w, HeadMode mode, const HeadArgs &ha,
               hipStream_t s);
// only: -1 all layers + head; 0..3 one layer; 4 the head; QNET_ONLY_CONV23 conv2 and conv3
constexpr int QNET_ONLY_CONV23 = 12;
// the act forward up to Dense1's partial slabs (w.slab) without the head; returns the slab
// count (the trainer runs the act head inside env_step_kernel)
int qnet_forward_act_slabs(const QLayout &L, const float *th, const float *wt, const BoardSrc &src, int64_t S,
                           QWork &w, hipStream_t s, const uint16_t *wtb, const SampleRider *rider);
// the number of Dense1 slabs an act forward of S samples writes
int qnet_act_slab_count(const QLayout &L, int64_t S);
// whether an act forward of S samples runs conv2 + conv3 fused (conv_h3f_kernel)
bool qnet_fused23(const QLayout &L, const float *theta, const float *wt, const uint16_t *wtb, int64_t S, QWork &w);
// wtb (optional): bf16 split planes of the image -> conv2/conv3/Dense1 on the x6 kernels.
// rider (optional): a replay sample run by one extra workgroup of the conv1 launch
void qnet_forward(const QLayout &L, const float *theta, const float *wt, const BoardSrc &src, int64_t S, QWork &w,
                  HeadMode mode, const HeadArgs &ha, hipStream_t s, int only = -1, const uint16_t *wtb = nullptr,
                  const SampleRider *rider = nullptr);
// Weight-gradient sections a backward left as K-split partial slabs (z > 1),
// plus Dense2's gradient (a reduction of dq x h1 over the batch): finished
// inside the update kernel instead of by separate reduce launches.
struct GradSlabs {
    const float *slab[4] = {};
    int z[4] = {};
    int64_t off[4] = {}, n[4] = {};
    const float *dq = nullptr, *h1 = nullptr;
    int64_t S = 0;
};
struct BwdOpts {
    GradSlabs *defer = nullptr;  // leave slabs + Dense2 to grad_update_launch
    bool dz1_ready = false;      // the LOSS head already wrote w.dz1
};
// backward of the loss whose dq sits in w.dq (after HEAD_LOSS): grad (packed) overwritten
void qnet_backward(const QLayout &L, const float *theta, const BoardSrc &src, int64_t S, QWork &w,
                   float *grad, float *slab, int64_t slab_cap, hipStream_t s, const BwdOpts &o = BwdOpts{});
// finish (slabs, Dense2 -> grad) and/or apply (RMSProp, forward weight image,
// update_target_net! when *counter % rate == 0) in one pass over theta
struct UpdateTarget {
    float *theta, *acc, *wt;
    float *theta_t, *wt_t;
    uint16_t *wtb = nullptr, *wtb_t = nullptr;   // bf16 split planes of the images
    const int64_t *counter;   // nullptr: no target copy
    int64_t rate;
    float lr, rho, eps;
    // optional: per-block partial max |w| of the new conv3 image (one per conv3 image
    // block of grad_update_kernel, gu_blocks(32, 36) of them) for the next h3 act forward
    float *wmax_out = nullptr;
    // optional: the new conv2 / conv3 / Dense1 images split for the next act forward
    // (w3_split_kernel's layouts, with the exponents of its last launch): that forward skips
    // w3_split_kernel (QWork::split_fresh)
    uint16_t *s_w3h = nullptr, *s_w2h = nullptr, *s_w1h = nullptr;
    const int *s_w3e = nullptr, *s_w1e = nullptr;
};
constexpr int GU_WMAX_BLOCKS = 36 * (32 / 16);   // conv3 image blocks of grad_update_kernel (gu_blocks(32, 36))
// the trainer's bookkeeping after an update (utils.jl:456-481: track_loss!, epsilon decay,
// nb += 1), done by the last workgroup of the update pass to arrive (ticket)
struct PostUpdate {
    const double *loss;    // [B] per-sample Huber losses
    int64_t B;
    double *loss_out, *last_loss, *log;
    int64_t log_cap;
    int64_t *updates, *nb;
    float *epsilon;
    float decay, eps_end;
    uint32_t *ticket;      // [9 * 32] arrival counters (8 shards + top), 0 between launches
    SampleRider next;      // out != nullptr: the last block also draws the NEXT update's batch
                           // (draw = the advanced update count; one launch fewer per update)
};
// tr.losses (utils.jl:404-406, 456-466): the Huber mean over the batch in a fixed order
// (256-thread strided sums, then a tree) -> loss_out, last_loss, log[updates % cap]. Reads
// only what the update's earlier launches wrote and *updates, which nothing but the
// bookkeeping below advances, so any block of the update pass may run it
__device__ inline void post_loss_block(const PostUpdate &p) {   // 256 threads
    __shared__ double sh[256];   // lds: one per kernel (one caller per update kernel)
    int64_t upd = 0;
    if (threadIdx.x == 0 && p.log) upd = *p.updates;
    double v = 0.0;
    for (int64_t i = threadIdx.x; i < p.B; i += 256) v += p.loss[i];
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    const double l = sh[0] / (double)p.B;
    *p.loss_out = l;
    *p.last_loss = l;
    if (p.log) p.log[upd % p.log_cap] = l;
}
// epsilon decay and the update counters (utils.jl:469-481), after every block of the update
// pass has read *nb (the target-sync decision)
// (upd, nb, eps: the three words as read before the pass, by the caller's thread 0: nothing
// else writes them during the pass, and loading them after the last arrival was one more
// round trip on the update's tail)
__device__ inline void post_count_block(const PostUpdate &p, int64_t upd, int64_t nb, float eps) {
    if (threadIdx.x != 0) return;
    *p.epsilon = fmaxf(eps - p.decay, p.eps_end);   // utils.jl:480
    *p.updates = upd + 1;
    *p.nb = nb + 1;
}
__device__ inline void post_count_block(const PostUpdate &p) {
    if (threadIdx.x != 0) return;
    post_count_block(p, *p.updates, *p.nb, *p.epsilon);
}
__device__ inline void post_update_block(const PostUpdate &p) {   // 256 threads
    post_loss_block(p);
    post_count_block(p);
}
void grad_update_launch(const QLayout &L, const GradSlabs *pending, float *grad, const UpdateTarget *apply,
                        hipStream_t s, const PostUpdate *post = nullptr);
int64_t qnet_backward_slab_floats(const QLayout &L, int64_t S);
// raw launchers shared with the deeper net (snk_deep.hip): the head kernels read
// only L.off_d1b / off_d2w / off_d2b; slab = ks partial Dense1 pre-activations [ks][S][64]
void head_launch(const QLayout &L, const float *th, const float *slab, int ks, int64_t S, float *h1, float *q,
                 HeadMode mode, const HeadArgs &ha, hipStream_t s);
void head_pair_launch(const QLayout &L, const float *th_t, const float *slab_t, float *h1_t, float *q_t,
                      const float *th_q, const float *slab_q, float *h1_q, float *q_q, int ks, int64_t S,
                      const HeadArgs &ha, hipStream_t s);
void d2_grad_launch(const float *dq, const float *h1, int64_t S, const QLayout &L, float *grad, hipStream_t s);
void slab_reduce_launch(const float *slab, int ks, int64_t MN, float *out, hipStream_t s);
// per-sample Jacobian rows J[s] = dQ(x_s)[a_s]/dtheta (packed order, row
// stride ldJ), a_s = act[idx[s]] % 3 (written to act_out). The conv sections
// [0, off_d1w) always; the Dense sections only with dense = true. ev_chain
// (optional) is recorded after the forward + data-gradient chain.
void qnet_jacobian(const QLayout &L, const float *theta, const float *wt, const BoardSrc &src, const uint8_t *act,
                   const int64_t *idx, int64_t S, QWork &w, uint8_t *act_out, float *J, int64_t ldJ, bool dense,
                   hipStream_t s, hipEvent_t ev_chain = nullptr);
void rmsprop_launch(int64_t P, float *theta, float *acc, const float *grad, float eta, float rho, float eps,
                    hipStream_t s);
void loss_mean_launch(const double *loss, int64_t B, double *out, hipStream_t s);

}  // namespace snk

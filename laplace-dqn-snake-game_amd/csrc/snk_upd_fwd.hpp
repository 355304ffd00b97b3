// snk_upd_fwd.hpp — the DQN update's conv stack for small batches in ONE launch.
//
// An update (utils.jl:444-466) runs t_net on the B next states and q_net on the
// B states (B = 64). As separate layer launches that is conv1, conv2 + its
// K-split reduce, conv3 + its reduce: five launches of a few microseconds of
// work each, every one paying the launch boundary and a cold start. Here one
// workgroup owns one sample of one net and half of conv3's 64 output channels
// (grid: 2 * B x nets, i.e. 256 workgroups for the two nets at B = 64):
//   phase 0  the sample's C input planes -> LDS as floats in a zero border
//            (and, for the training net, the float copy x0 the conv1 weight
//            gradient reads); conv2's bf16 split weight planes -> LDS;
//   phase 1  conv1 (3x3, C -> 16, VALU, fp32, the order of conv1_fwd_kernel),
//            bias + relu -> a1 (global, training net) and its exact 3-part bf16
//            split (h + m + l, snk_conv_x6.hpp) into a bordered LDS image;
//   phase 2  conv2 (3x3, 16 -> 32) on v_mfma_f32_16x16x32_bf16 with the six
//            part products of the x6 split (fp32-exact products, fp32
//            accumulation), offsets paired into 5 k-steps of 32; bias + relu
//            -> a2 (global, training net) and its split into LDS;
//   phase 3  conv3 (6x6, 32 -> 64, this workgroup's 32 channels): A from the
//            LDS image, B (the weight planes the update keeps current) staged
//            through LDS three offsets at a time (double-buffered, loaded two stages
//            ahead); bias + relu -> a3.
//   phase 4  (d1) Dense1 over this workgroup's half of the features: the sample's a3
//            channels of this half (NO positions x 32) from LDS against the W1 rows
//            (p * 64 + 32 half + c) straight from L2 (fp32 float4 rows, fp64 FMA sums per
//            channel, the 32 channel sums added in channel order, rounded once) -> the
//            half's partial slab; the head adds the two halves (ks = 2). This replaced
//            dense1_upd_kernel (8.8 us) and its launch boundary in round 5: the 64 samples'
//            W1 re-reads (401 KB per workgroup at 12x12) stay in L2.
//   phase 5  (head) the last of the sample's four workgroups (its two halves in both nets,
//            a relaxed agent-scope ticket per sample, slabs handed over by sc1 stores and
//            loads) runs both heads for it (head_pair_one: the
//            t_net TD target, the q_net Huber loss, dq and dz1), which replaced the
//            head_pair_kernel launch.
// conv1 and conv2 run in both halves of a sample (they are ~20 % of the work);
// only half 0 writes a1, a2 and x0.
#pragma once

#include "snk_conv_h3.hpp"
#include "snk_conv_x6.hpp"
#include "snk_qnet.hpp"

namespace snk {

// Profiling builds only (make clocks): per-workgroup phase timestamps, read back by
// snk_upd_debug_clocks (slots: start, phase 0, 1, 2 done, phase 3 done, phase 4 done (slab stored),
// phase 5 done (the last arriver's heads))
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_upd_clk;
#define UPD_CLK(slot)                                                                                  \
    do {                                                                                               \
        if (threadIdx.x == 0 && g_upd_clk)                                                             \
            g_upd_clk[((int64_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define UPD_CLK(slot) do { } while (0)
#endif

// HEAD_TARGET of t_net then HEAD_LOSS of q_net for the same sample s in one wave
// (the loss needs exactly that sample's target): same arithmetic as
// head_kernel<HEAD_TARGET> / <HEAD_LOSS> (snk_qnet.hip), the ks Dense1 slabs added to the
// bias in slab order. Run by head_pair_kernel (one wave per sample) and by the last of a
// sample's four update-forward workgroups (upd_fwd_kernel phase 5).
// phase 5's slab hand-off by sc1 stores / loads and a relaxed ticket (0: an acq_rel ticket,
// measurement builds only)
#ifndef UPD_SC1
#define UPD_SC1 1
#endif
struct HeadNet {
    const float *slab, *theta;
    float *h1, *q;
};
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
// the sample's replay fields (mask, done, reward, action), two dependent loads (the slot, then
// the fields): upd_fwd_kernel issues them at its start, long before its phase 5 needs them
struct HeadPre {
    uint32_t bits;   // mask | done << 8 | action << 16 (two registers held through the kernel)
    float rw;
};
__device__ __forceinline__ HeadPre head_pre(const HeadArgs &ha, int64_t s) {
    const int64_t m = ha.idx ? ha.idx[s] : s;
    return HeadPre{(uint32_t)ha.mask[m] | ((uint32_t)ha.done[m] << 8) | ((uint32_t)(ha.act_idx[m] % 3) << 16), ha.rew[m]};
}
__device__ __forceinline__ void head_pair_one(const HeadNet &tn, const HeadNet &qn, int ks, int64_t S,
                                              const QLayout &L, const HeadArgs &ha, int64_t s, int lane,
                                              const HeadPre &pre) {
    // every independent load of both nets up front (the kernel is load-latency bound: the
    // q_net half used to start its loads only after the t_net half's reductions)
    constexpr int KMAX = 16;
    float zt[KMAX], zq[KMAX];
    // slab loads sc1 (relaxed agent-scope, L1 bypassed): upd_fwd_kernel's phase 5 reads slabs
    // other workgroups stored sc1 moments ago, with no acquire
#pragma unroll
    for (int z = 0; z < KMAX; ++z) {
        if (z < ks) {
            zt[z] = __hip_atomic_load(tn.slab + ((int64_t)z * S + s) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            zq[z] = __hip_atomic_load(qn.slab + ((int64_t)z * S + s) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    float wt2[3], wq2[3], bt2[3], bq2[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        wt2[a] = tn.theta[L.off_d2w + a * 64 + lane];
        wq2[a] = qn.theta[L.off_d2w + a * 64 + lane];
        bt2[a] = tn.theta[L.off_d2b + a];
        bq2[a] = qn.theta[L.off_d2b + a];
    }
    const float bt1 = tn.theta[L.off_d1b + lane], bq1 = qn.theta[L.off_d1b + lane];
    const uint8_t mk = (uint8_t)(pre.bits & 0xff), dn = (uint8_t)((pre.bits >> 8) & 0xff);
    const float rw = pre.rw;
    const int a_taken = (int)(pre.bits >> 16);
    // t_net(s'): TD target (utils.jl:448-451)
    float h = bt1;
    if (ks <= KMAX) {
#pragma unroll
        for (int z = 0; z < KMAX; ++z)
            if (z < ks) h += zt[z];
    } else {
        for (int z = 0; z < ks; ++z)
            h += __hip_atomic_load(tn.slab + ((int64_t)z * S + s) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    h = h > 0.0f ? h : 0.0f;
    tn.h1[s * 64 + lane] = h;
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) q[a] = bt2[a] + wave_sum(wt2[a] * h);
    float mx = -INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float v = ((mk >> a) & 1) ? -100.0f : q[a];
        mx = v > mx ? v : mx;
    }
    const double tgt = (double)rw + ha.gamma * (double)mx * (double)(1 - (int)dn);
    if (lane == 0) {
        tn.q[s * 3 + 0] = q[0];
        tn.q[s * 3 + 1] = q[1];
        tn.q[s * 3 + 2] = q[2];
        ha.target[s] = tgt;
    }
    // q_net(s): Huber loss, dq and dz1 (utils.jl:453-464)
    h = bq1;
    if (ks <= KMAX) {
#pragma unroll
        for (int z = 0; z < KMAX; ++z)
            if (z < ks) h += zq[z];
    } else {
        for (int z = 0; z < ks; ++z)
            h += __hip_atomic_load(qn.slab + ((int64_t)z * S + s) * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    h = h > 0.0f ? h : 0.0f;
    qn.h1[s * 64 + lane] = h;
#pragma unroll
    for (int a = 0; a < 3; ++a) q[a] = bq2[a] + wave_sum(wq2[a] * h);
    const int a = a_taken;
    const double e = (double)q[a] - tgt;
    const double ae = fabs(e);
    const double g = (ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / (double)ha.B;
    if (ha.dz1) ha.dz1[s * 64 + lane] = h > 0.0f ? (float)g * (a == 0 ? wq2[0] : a == 1 ? wq2[1] : wq2[2]) : 0.0f;
    if (lane != 0) return;
    qn.q[s * 3 + 0] = q[0];
    qn.q[s * 3 + 1] = q[1];
    qn.q[s * 3 + 2] = q[2];
    ha.loss[s] = ae < 1.0 ? 0.5 * e * e : ae - 0.5;
#pragma unroll
    for (int k = 0; k < 3; ++k) ha.dq[s * 3 + k] = k == a ? (float)g : 0.0f;
}

struct UpdFwdNet {
    BoardSrc src;
    const float *th;        // packed theta: conv1 weights/bias, conv2/conv3 biases, Dense1 weights
    const uint16_t *wtb;    // x6 split planes of the forward weight image
    float *a1, *a2, *a3;    // a1/a2 may be null (target net: only a3 is consumed)
    float *x0;              // the input planes as floats [S][C][bs^2] (training net) or null
    float *slab;            // d1: Dense1 partial slabs [2 halves][S][64] (the head sums the two)
};
struct UpdFwdArgs {
    UpdFwdNet net[2];
    QLayout L;
    int S;
    int d1;                 // phase 4 (Dense1 of this workgroup's 32 channels) on
    // phase 5 (d1 and head): the heads of both nets (head_pair_one: net[0] = t_net's TD target,
    // net[1] = q_net's loss, dq, dz1) run by the last of each sample's four workgroups
    int head;
    HeadNet hn[2];
    HeadArgs ha;
    uint32_t *ticket;       // [S] arrivals, 0 between launches (the last arriver resets it)
};

// LDS strides (halves): A1 position record 3 planes x 16 ch + 8 pad
constexpr int UPDF_A1S = 56;
// A2 (conv3's input, conv2's output): three plane images [pl][HIN rows][PJ][32 ch] of 64-byte
// rows, chunk c (8 channels) of row R at slot c ^ ((R >> 1) & 3). conv3's row tiles are TW
// output columns x 16 / TW output rows (TW = 8 while WO <= 8), so each fragment read covers
// rows (qi + du) + (qj + dv) * PJ, which with PJ = 16 (TW = 8) land on distinct bank quads
// (lane groups simulated; the round-2 layout, 104-half position records with tiles running
// across output rows, was 2.25-way conflicted)
__host__ __device__ constexpr int updf_tw(int hin) { return hin - 5 <= 8 ? 8 : 16; }
__host__ __device__ constexpr int updf_pj(int hin) { return updf_tw(hin) == 8 ? 16 : 24; }
constexpr int UPDF_NT = 512;   // 8 waves: two per SIMD, so one wave's LDS / MFMA latency hides under the other's

// floats of the input planes + conv1 weights, rounded up to a 16-byte boundary
__host__ __device__ constexpr int updf_f32_words(int hin, int C) {
    return (C * (hin + 2) * (hin + 2) + 9 * C * 16 + 16 + 3) & ~3;
}
__host__ __device__ constexpr int updf_base_bytes(int hin, int C) {
    return updf_f32_words(hin, C) * 4 + (hin + 2) * (hin + 2) * UPDF_A1S * 2 + 9 * 3 * 32 * 16 * 2 +
           3 * hin * updf_pj(hin) * 32 * 2;
}
// conv3's weight ring: slots of one kernel offset (the workgroup's 32 columns, 3 planes, 6 KB)
// in the LDS beyond the images, filled by LDS-DMA NR - 1 offsets ahead; boards whose images
// leave room for fewer than UPDF_RING_MIN slots keep the register-staged path
constexpr int UPDF_SLOT = 3 * 32 * 32 * 2, UPDF_RING_MAX = 12, UPDF_RING_MIN = 6;
// conv3 ring offsets per barrier step (1, 2, 3 or 4: 36, 18, 12 or 9 barriers): 3 took the
// B = 64 update from 0.0720 to 0.0711 ms (profiles/r05bb_upd_ring_ab.txt)
#ifndef UPDF_KS
#define UPDF_KS 3
#endif
// phase 4's W1 rows: 0 = two batches of loads, D > 0 = a software pipeline D rows deep (8: the B = 64
// update 0.0700 -> 0.0693 ms marginal, 16 / 24 / 32 no better; profiles/r06t_upd_d1_pipe.txt)
#ifndef UPDF_D1_PIPE
#define UPDF_D1_PIPE 8
#endif
__host__ __device__ constexpr int updf_ring(int hin, int C) {
    return (160 * 1024 - updf_base_bytes(hin, C)) / UPDF_SLOT >= UPDF_RING_MAX
               ? UPDF_RING_MAX
               : (160 * 1024 - updf_base_bytes(hin, C)) / UPDF_SLOT;
}
__host__ __device__ constexpr int updf_lds_bytes(int hin, int C) {
    return updf_base_bytes(hin, C) + (updf_ring(hin, C) >= UPDF_RING_MIN ? updf_ring(hin, C) * UPDF_SLOT : 0);
}

// the three bf16 parts h, m, l of x (split_part's values, in one pass)
__device__ __forceinline__ void split3_scalar(float x, uint16_t &h, uint16_t &m, uint16_t &l) {
    f32x2 b;
    f32x2 v{x, 0.0f};
    h = (uint16_t)(bf2(v, b) & 0xffffu);
    v = v - b;
    m = (uint16_t)(bf2(v, b) & 0xffffu);
    v = v - b;
    l = (uint16_t)(bf2(v, b) & 0xffffu);
}

// six part products (the x6 set, conv_x6m16_kernel's order) of one A / B fragment triple
__device__ __forceinline__ f32x4v mfma_x6(const u32x4 *a, const u32x4 *b, f32x4v c) {
    const bf16x8 ah = as_bf(a[0]), am = as_bf(a[1]), al = as_bf(a[2]);
    const bf16x8 bh = as_bf(b[0]), bm = as_bf(b[1]), bl = as_bf(b[2]);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
    return c;
}

// s_waitcnt vmcnt(n) for a value n that is constant only after unrolling (the builtin needs a
// literal): n > 12 waits for vmcnt(12), n < 0 for vmcnt(0)
__device__ __forceinline__ void vm_wait_le12(int n) {
#define VMW(k) else if (n == k) __builtin_amdgcn_s_waitcnt(waitcnt_vm(k));
    if (n >= 12) __builtin_amdgcn_s_waitcnt(waitcnt_vm(12));
    VMW(11) VMW(10) VMW(9) VMW(8) VMW(7) VMW(6) VMW(5) VMW(4) VMW(3) VMW(2) VMW(1)
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
#undef VMW
}

template <int HIN, int C>
__global__ __launch_bounds__(UPDF_NT) void upd_fwd_kernel(UpdFwdArgs args) {
    constexpr int BP = HIN + 2, NB = BP * BP, NC = HIN * HIN;
    constexpr int WO = HIN - 5, NO = WO * WO;
    constexpr int TW = updf_tw(HIN), PJ = updf_pj(HIN), RPT = 16 / TW;   // conv3 tile: TW columns x RPT rows
    constexpr int T2 = (NC + 15) / 16, T3 = (WO + RPT - 1) / RPT;
    constexpr int A2P = HIN * PJ * 32;                                   // halves per A2 plane image
    static_assert(TW + 5 <= PJ && HIN <= PJ && WO <= TW, "conv3 tile geometry");
    extern __shared__ __attribute__((aligned(16))) uint8_t updf_lds[];
    float *xin = reinterpret_cast<float *>(updf_lds);                 // [C][NB]
    float *w1 = xin + C * NB;                                        // [9C*16] + bias [16]
    uint16_t *A1 = reinterpret_cast<uint16_t *>(xin + updf_f32_words(HIN, C));   // [NB][UPDF_A1S]
    uint16_t *B2 = A1 + NB * UPDF_A1S;                               // [9 kk][3][32 co][16 ci]
    uint16_t *A2 = B2 + 9 * 3 * 32 * 16;                             // [3][HIN][PJ][32] (swizzled chunks)
    constexpr int NR = updf_ring(HIN, C);
    constexpr bool RING = NR >= UPDF_RING_MIN;
    uint16_t *R3 = A2 + 3 * A2P;                                     // [NR][3 pl][32 cols][32 ci] (swizzled pieces)
    static_assert((NB * UPDF_A1S * 2) % 16 == 0 && updf_base_bytes(HIN, C) % 16 == 0, "16-B regions");

    UPD_CLK(0);
    const UpdFwdNet &n = args.net[blockIdx.y];
    const QLayout &L = args.L;
    const int s = blockIdx.x >> 1, half = blockIdx.x & 1;
    // phase 5's replay fields, loaded now by wave 0 (only a sample's last workgroup uses them)
    HeadPre hpre{};
    if (args.head && threadIdx.x < 64) hpre = head_pre(args.ha, s);
    const bool wr = half == 0;   // half 0 writes the training activations
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;

    // ---- phase 0: input planes, conv1 weights, conv2 weight planes, A1 border --------
    // (every load of a thread is issued before its first LDS store)
    {
        constexpr int NB2 = 9 * 3 * 32 * 16 / 8, KB2 = (NB2 + UPDF_NT - 1) / UPDF_NT;   // conv2 planes, 16-B pieces
        constexpr int KX = (C * NB + UPDF_NT - 1) / UPDF_NT;
        const u32x4 *src2 = reinterpret_cast<const u32x4 *>(n.wtb + 3 * L.off_t2);
        u32x4 bv[KB2];
#pragma unroll
        for (int k = 0; k < KB2; ++k) bv[k] = src2[min(tid + k * UPDF_NT, NB2 - 1)];
        const int8_t *pl[C];
#pragma unroll
        for (int c = 0; c < C; ++c) pl[c] = n.src.plane(s, c);
        float xv[KX];
#pragma unroll
        for (int k = 0; k < KX; ++k) {
            const int e = tid + k * UPDF_NT;
            const int c = e / NB, b = e - c * NB;
            const int bj = b / BP, bi = b - bj * BP;
            xv[k] = 0.0f;
            if (e < C * NB && bi >= 1 && bi <= HIN && bj >= 1 && bj <= HIN) {
                const int cell = (bi - 1) + (bj - 1) * HIN;
                xv[k] = pl[c] ? (float)pl[c][cell] : n.src.fbase[((int64_t)s * C + c) * NC + cell];
            }
        }
        constexpr int NW1 = 9 * C * 16 + 16;   // conv1 weights + bias: at most two per thread
        static_assert(NW1 <= 2 * UPDF_NT, "conv1 weights");
        float w1v[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            const int e = tid + k * UPDF_NT;
            w1v[k] = e < 9 * C * 16 ? n.th[L.off_w1 + e] : e < NW1 ? n.th[L.off_b1 + e - 9 * C * 16] : 0.0f;
        }
#pragma unroll
        for (int k = 0; k < KX; ++k) {
            const int e = tid + k * UPDF_NT;
            if (e < C * NB) {
                xin[e] = xv[k];
                const int c = e / NB, b = e - c * NB;
                const int bj = b / BP, bi = b - bj * BP;
                if (wr && n.x0 && bi >= 1 && bi <= HIN && bj >= 1 && bj <= HIN)
                    n.x0[((int64_t)s * C + c) * NC + (bi - 1) + (bj - 1) * HIN] = xv[k];
            }
        }
#pragma unroll
        for (int k = 0; k < 2; ++k)
            if (tid + k * UPDF_NT < NW1) w1[tid + k * UPDF_NT] = w1v[k];
#pragma unroll
        for (int k = 0; k < KB2; ++k)
            if (tid + k * UPDF_NT < NB2) reinterpret_cast<u32x4 *>(B2)[tid + k * UPDF_NT] = bv[k];
        for (int e = tid; e < NB * (UPDF_A1S / 8); e += UPDF_NT)   // zero the whole A1 image (border stays 0)
            reinterpret_cast<u32x4 *>(A1)[e] = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();
    UPD_CLK(1);
    // conv3's weight ring (RING): offset k's 384 16-byte pieces (3 planes x 32 columns x 4)
    // go to slot k % NR by waves 0..5, one global_load_lds_dwordx4 each: lane-linear LDS
    // slots, the source piece chosen so that slot piece p of row c holds global piece
    // p ^ ((c >> 2) & 3) (the swizzle the fragment reads expect). Offsets 0 .. NR-2 are issued
    // at the start of conv2
    const uint16_t *wsrc3 = n.wtb + 3 * L.off_t3 + (int64_t)half * 32 * 32;   // planes [kk][3][64 co][32 ci]
    auto dma3 = [&](int k) __attribute__((always_inline)) {
        if constexpr (RING) {
            if (wave < 6) {
                const int q = wave * 64 + lane, row = q >> 2, pl = row >> 5, c = row & 31;
                const int piece = (q & 3) ^ ((row >> 2) & 3);
                __builtin_amdgcn_global_load_lds(
                    (const void *)(wsrc3 + ((int64_t)(k * 3 + pl) * 64 + c) * 32 + piece * 8),
                    (__attribute__((address_space(3))) void *)(R3 + (k % NR) * (UPDF_SLOT / 2) + wave * 512), 16, 0, 0);
            }
        }
    };

    // ---- phase 1: conv1 (VALU), a1 and its split ---------------------------------------
    // four output channels 4q .. 4q + 3 of position p per thread: one input read feeds four
    // FMA chains (each in conv1_fwd_kernel's order), a1 leaves as one float4, the split as
    // 8-byte pieces (one channel per thread read every input nine times per channel)
    for (int o = tid; o < NC * 4; o += UPDF_NT) {
        const int p = o >> 2, q = o & 3;
        const int j = p / HIN, i = p - j * HIN;
        float acc[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = w1[9 * C * 16 + 4 * q + e];
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int du = kk % 3, dv = kk / 3;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float x = xin[c * NB + (i + du) + (j + dv) * BP];
#pragma unroll
                for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(x, w1[(kk * C + c) * 16 + 4 * q + e], acc[e]);
            }
        }
        f32x4 v4;
        uint16_t h[4], m[4], l[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            v4[e] = fmaxf(acc[e], 0.f);
            split3_scalar(v4[e], h[e], m[e], l[e]);
        }
        if (wr && n.a1) *reinterpret_cast<f32x4 *>(n.a1 + ((int64_t)s * NC + p) * 16 + 4 * q) = v4;
        u32x2 *d = reinterpret_cast<u32x2 *>(A1 + ((i + 1) + (j + 1) * BP) * UPDF_A1S + 4 * q);   // 8-byte aligned
        d[0] = u32x2{(uint32_t)h[0] | ((uint32_t)h[1] << 16), (uint32_t)h[2] | ((uint32_t)h[3] << 16)};
        d[4] = u32x2{(uint32_t)m[0] | ((uint32_t)m[1] << 16), (uint32_t)m[2] | ((uint32_t)m[3] << 16)};
        d[8] = u32x2{(uint32_t)l[0] | ((uint32_t)l[1] << 16), (uint32_t)l[2] | ((uint32_t)l[3] << 16)};
    }
    __syncthreads();
    UPD_CLK(2);
    // (issued here, not before conv1: every __syncthreads waits vmcnt(0), and conv2 is long
    // enough to cover the weights' trip from L2 / MALL, conv1 is not)
    if constexpr (RING) {
#pragma unroll
        for (int k = 0; k < NR - UPDF_KS; ++k) dma3(k);
    }

    // ---- phase 2: conv2 on x6 MFMA: rows = the HIN^2 positions, 32 columns -------------
    // wave w owns column tile w & 1 and row tiles (w >> 1) + 4u; offset pair p outermost so
    // each B fragment is read from LDS once
    {
        constexpr int NT2 = (T2 + 3) / 4;
        const int ct = wave & 1, rt0 = wave >> 1;
        const int col = ct * 16 + r;
        const float bv = n.th[L.off_b2 + col];
        int qb[NT2];
        f32x4v acc[NT2];
#pragma unroll
        for (int u = 0; u < NT2; ++u) {
            const int q = min((rt0 + 4 * u) * 16 + r, NC - 1);
            const int qj = q / HIN, qi = q - qj * HIN;
            qb[u] = qi + qj * BP;
            acc[u] = f32x4v{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            const int kk = 2 * p + (g >> 1);   // k 0..15: offset 2p, k 16..31: offset 2p + 1
            const bool live = kk < 9;
            const int kc = live ? kk : 8, du = kc % 3, dv = kc / 3;
            u32x4 b[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                b[pl] = live ? *reinterpret_cast<const u32x4 *>(B2 + ((kc * 3 + pl) * 32 + col) * 16 + 8 * (g & 1))
                             : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
            for (int u = 0; u < NT2; ++u) {
                if (rt0 + 4 * u < T2) {   // wave-uniform
                    const uint16_t *pa = A1 + (qb[u] + du + dv * BP) * UPDF_A1S + 8 * (g & 1);
                    u32x4 a[3];
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        a[pl] = live ? *reinterpret_cast<const u32x4 *>(pa + pl * 16) : u32x4{0u, 0u, 0u, 0u};
                    acc[u] = mfma_x6(a, b, acc[u]);
                }
            }
        }
        // C[row 4g + e][col r]: bias + relu -> a2 and its split
#pragma unroll
        for (int u = 0; u < NT2; ++u) {
            const int t = rt0 + 4 * u;
            if (t >= T2) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = t * 16 + 4 * g + e;
                if (row >= NC) continue;
                const float v = fmaxf(acc[u][e] + bv, 0.f);
                if (wr && n.a2) n.a2[((int64_t)s * NC + row) * 32 + col] = v;
                uint16_t h, m, l;
                split3_scalar(v, h, m, l);
                const int rj = row / HIN, R = (row - rj * HIN) + rj * PJ;
                uint16_t *d = A2 + R * 32 + 8 * ((col >> 3) ^ ((R >> 1) & 3)) + (col & 7);
                d[0] = h;
                d[A2P] = m;
                d[2 * A2P] = l;
            }
        }
    }
    __syncthreads();
    UPD_CLK(3);
    // ---- phase 3: conv3 on x6 MFMA: rows = the WO^2 output positions, 32 columns -------
    // wave w owns column tile w & 1 (16 of the workgroup's 32 columns) and row tiles
    // (w >> 1) + 4u. The workgroup's B (its 32 columns, 6 KB per offset) is staged once
    // per 3-offset stage into the LDS the conv1/conv2 images no longer need (double-buffered,
    // one barrier per stage): read straight from L2 by every wave it cost four times the L1
    // traffic. Even and odd offsets accumulate separately (two MFMA chains).
    {
        constexpr int NTW = (T3 + 3) / 4;   // row tiles per wave
        // offsets per stage; halves per LDS B row (16-byte piece p of row c stored at p ^ ((c >> 2) & 3):
        // the fragment reads of 16 rows hit distinct bank quads)
        constexpr int KB = 3, NSTG = 36 / KB, LDB = 32;
        constexpr int SPL = KB * 3 * 32 * LDB;            // halves per stage buffer
        static_assert(2 * SPL * 2 <= NB * UPDF_A1S * 2 + 9 * 3 * 32 * 16 * 2, "B stages fit the dead A1 + B2 images");
        constexpr int NQ = KB * 3 * 32 * 4;               // 16-byte pieces per stage (4 per 32-ci row)
        constexpr int QPT = (NQ + UPDF_NT - 1) / UPDF_NT;
        uint16_t *B3 = A1;   // [2][KB kk][3 pl][32 cols][LDB]
        const int ct = wave & 1, rt0 = wave >> 1;
        const int col = half * 32 + ct * 16 + r;
        const float *b3 = n.th + L.off_b3;
        const uint16_t *wsrc = n.wtb + 3 * L.off_t3 + (int64_t)half * 32 * 32;   // planes [kk][3][64 co][32 ci]
        // stage s is loaded into registers two stages ahead (sa / sb alternate), stored into
        // LDS buffer s & 1 one stage ahead
        u32x4 sa[QPT], sb[QPT];
        auto sload = [&](int stg, u32x4 (&st)[QPT]) {
#pragma unroll
            for (int u = 0; u < QPT; ++u) {
                const int q = min(tid + u * UPDF_NT, NQ - 1);
                const int row = q >> 2, piece = q & 3;   // row = (kl * 3 + pl) * 32 + c
                const int kl = row / 96, pl = (row / 32) % 3, c = row & 31;
                st[u] = *reinterpret_cast<const u32x4 *>(wsrc + ((int64_t)((stg * KB + kl) * 3 + pl) * 64 + c) * 32 +
                                                         piece * 8);
            }
        };
        auto sstore = [&](int buf, const u32x4 (&st)[QPT]) {
#pragma unroll
            for (int u = 0; u < QPT; ++u) {
                const int q = tid + u * UPDF_NT;
                if (q < NQ)
                    *reinterpret_cast<u32x4 *>(B3 + buf * SPL + (q >> 2) * LDB + ((q & 3) ^ ((q >> 4) & 3)) * 8) = st[u];
            }
        };
        int qb[NTW];   // the lane's first A2 row in row tile rt0 + 4u: column r % TW, row clamped to WO - 1
        f32x4v acc[NTW][2];
#pragma unroll
        for (int u = 0; u < NTW; ++u) {
            const int qj = min((rt0 + 4 * u) * RPT + r / TW, WO - 1), qi = r % TW;
            qb[u] = qi + qj * PJ;
            acc[u][0] = acc[u][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
        }
        auto compute = [&](int stg) {
            const uint16_t *bb = B3 + (stg & 1) * SPL + (ct * 16 + r) * LDB + 8 * (g ^ ((r >> 2) & 3));
#pragma unroll
            for (int kl = 0; kl < KB; ++kl) {
                const int kk = stg * KB + kl, du = kk % 6, dv = kk / 6;
                u32x4 b[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) b[pl] = *reinterpret_cast<const u32x4 *>(bb + (kl * 3 + pl) * 32 * LDB);
#pragma unroll
                for (int u = 0; u < NTW; ++u) {
                    if (rt0 + 4 * u < T3) {   // wave-uniform
                        const int R = qb[u] + du + dv * PJ;
                        const uint16_t *pa = A2 + R * 32 + 8 * (g ^ ((R >> 1) & 3));
                        u32x4 a[3];
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const u32x4 *>(pa + pl * A2P);
                        acc[u][kl & 1] = mfma_x6(a, b, acc[u][kl & 1]);
                    }
                }
            }
        };
        static_assert(NSTG % 2 == 0, "stages come in pairs");
        if constexpr (RING) {
            // UPDF_KS offsets per step, one barrier each: wait for this wave's DMAs of the
            // step's offsets (newer ones may stay in flight), publish with the barrier (every wave
            // has also read step st - 1's slots into registers), refill those slots with offsets
            // st KS + NR - KS .. + KS - 1. Chains as the staged path: offset kk into
            // acc[.][(kk % 3) & 1], in kk order. Software-pipelined: step st reads its offsets'
            // fragments (B from slot kk % NR, A from the image) right after the barrier, then
            // issues step st - 1's MFMAs from registers, so the LDS latency hides under them
            static_assert(NTW == 1, "ring path: one row tile per wave");
            constexpr int KS = UPDF_KS, NS = 36 / KS;
            static_assert(36 % KS == 0 && NR >= 2 * KS + 1, "ring steps");
            const bool live = rt0 < T3;   // wave-uniform
            u32x4 fa[2][KS][3], fb[2][KS][3];
            auto frag = [&](int kk, u32x4 (&xa)[3], u32x4 (&xb)[3]) __attribute__((always_inline)) {
                const int du = kk % 6, dv = kk / 6;
                const uint16_t *bb = R3 + (kk % NR) * (UPDF_SLOT / 2) + (ct * 16 + r) * LDB + 8 * (g ^ ((r >> 2) & 3));
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) xb[pl] = *reinterpret_cast<const u32x4 *>(bb + pl * 32 * LDB);
                const int R = qb[0] + du + dv * PJ;
                const uint16_t *pa = A2 + R * 32 + 8 * (g ^ ((R >> 1) & 3));
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) xa[pl] = *reinterpret_cast<const u32x4 *>(pa + pl * A2P);
            };
#pragma unroll
            for (int st = 0; st <= NS; ++st) {
                if (st < NS) {
                    // this wave's DMAs of the step's offsets landed: the ones issued after them
                    // (offsets up to min(35, st KS + NR - KS - 1)) may stay in flight
                    vm_wait_le12(min(35, st * KS + NR - KS - 1) - (st * KS + KS - 1));
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of step st - 1 done
                    __builtin_amdgcn_s_barrier();
#pragma unroll
                    for (int k = 0; k < KS; ++k)
                        if (st * KS + NR - KS + k < 36) dma3(st * KS + NR - KS + k);
                    if (live) {
#pragma unroll
                        for (int k = 0; k < KS; ++k) frag(st * KS + k, fa[st & 1][k], fb[st & 1][k]);
                    }
                }
                if (st > 0 && live) {
#pragma unroll
                    for (int k = 0; k < KS; ++k) {
                        const int k1 = (st - 1) * KS + k;
                        if (((k1 % 3) & 1) == 0)
                            acc[0][0] = mfma_x6(fa[(st - 1) & 1][k], fb[(st - 1) & 1][k], acc[0][0]);
                        else
                            acc[0][1] = mfma_x6(fa[(st - 1) & 1][k], fb[(st - 1) & 1][k], acc[0][1]);
                    }
                }
            }
        } else {
        sload(0, sa);
        sload(1, sb);
        sstore(0, sa);
        sload(2, sa);
        __syncthreads();
        for (int stg = 0; stg < NSTG; stg += 2) {
            compute(stg);                          // buffer 0
            sstore(1, sb);                         // stage stg + 1 (buffer 1 last read at stg - 1)
            __syncthreads();
            if (stg + 3 < NSTG) sload(stg + 3, sb);
            compute(stg + 1);                      // buffer 1
            if (stg + 2 < NSTG) sstore(0, sa);     // stage stg + 2 (buffer 0 last read at stg)
            __syncthreads();
            if (stg + 4 < NSTG) sload(stg + 4, sa);
        }
        }
        UPD_CLK(4);
        const float bv = b3[col];
        float a3v[NTW][4];
#pragma unroll
        for (int u = 0; u < NTW; ++u) {
            const int t = rt0 + 4 * u;
            if (t >= T3) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int qi = (4 * g + e) % TW, qj = t * RPT + (4 * g + e) / TW;
                a3v[u][e] = fmaxf((acc[u][0][e] + acc[u][1][e]) + bv, 0.f);
                if (qi < WO && qj < WO) n.a3[((int64_t)s * NO + qi + qj * WO) * 64 + col] = a3v[u][e];
            }
        }
        if (!args.d1) return;
        // ---- phase 4: Dense1 over this half's 32 channels ------------------------------------
        // every wave's conv3 reads of the images and the ring are done past this barrier
        __syncthreads();
        float *a3s = reinterpret_cast<float *>(updf_lds);                        // [NO][32]
        double *red = reinterpret_cast<double *>(updf_lds + ((NO * 32 * 4 + 15) & ~15));   // [32 c][64 o]
#pragma unroll
        for (int u = 0; u < NTW; ++u) {
            const int t = rt0 + 4 * u;
            if (t >= T3) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int qi = (4 * g + e) % TW, qj = t * RPT + (4 * g + e) / TW;
                if (qi < WO && qj < WO) a3s[(qi + qj * WO) * 32 + ct * 16 + r] = a3v[u][e];
            }
        }
        __syncthreads();
        {
            const int o4 = tid & 15, c = tid >> 4;   // outputs 4 o4 .. +3, channel c of this half
            const f32x4 *w1 = reinterpret_cast<const f32x4 *>(n.th + L.off_d1w + (int64_t)(32 * half + c) * 64 + 4 * o4);
            double z0 = 0.0, z1 = 0.0, z2 = 0.0, z3 = 0.0;
#if UPDF_D1_PIPE
            // software pipeline: row p + D is requested as row p is consumed
            constexpr int D = UPDF_D1_PIPE < NO ? UPDF_D1_PIPE : NO;
            f32x4 wv[NO];
#pragma unroll
            for (int k = 0; k < D; ++k) wv[k] = w1[(int64_t)k * 64 * 16];
#pragma unroll
            for (int k = 0; k < NO; ++k) {
                if (k + D < NO) wv[k + D] = w1[(int64_t)(k + D) * 64 * 16];
                const double av = (double)a3s[k * 32 + c];
                z0 = __builtin_fma(av, (double)wv[k][0], z0);
                z1 = __builtin_fma(av, (double)wv[k][1], z1);
                z2 = __builtin_fma(av, (double)wv[k][2], z2);
                z3 = __builtin_fma(av, (double)wv[k][3], z3);
            }
#else
            constexpr int PB = (NO + 1) / 2;   // W1 rows in flight per thread: two batches (L2 round trips)
            for (int p0 = 0; p0 < NO; p0 += PB) {
                f32x4 wv[PB];
#pragma unroll
                for (int k = 0; k < PB; ++k) wv[k] = p0 + k < NO ? w1[(int64_t)(p0 + k) * 64 * 16] : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int k = 0; k < PB; ++k) {
                    if (p0 + k >= NO) break;
                    const double av = (double)a3s[(p0 + k) * 32 + c];
                    z0 = __builtin_fma(av, (double)wv[k][0], z0);
                    z1 = __builtin_fma(av, (double)wv[k][1], z1);
                    z2 = __builtin_fma(av, (double)wv[k][2], z2);
                    z3 = __builtin_fma(av, (double)wv[k][3], z3);
                }
            }
#endif
            double *rd = red + c * 64 + 4 * o4;
            rd[0] = z0;
            rd[1] = z1;
            rd[2] = z2;
            rd[3] = z3;
        }
        __syncthreads();
        if (tid >= 64) return;   // wave 0 stores the slab and, if last, runs the heads
        double z = 0.0;
#pragma unroll 8
        for (int c = 0; c < 32; ++c) z += red[c * 64 + tid];
#if UPD_SC1
        // sc1 store (relaxed agent-scope): the line leaves the XCD's L2 for memory
        __hip_atomic_store(n.slab + ((int64_t)half * args.S + s) * 64 + tid, (float)z, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
#else
        n.slab[((int64_t)half * args.S + s) * 64 + tid] = (float)z;
#endif
        UPD_CLK(5);
        if (!args.head) return;
        // ---- phase 5: the last of the sample's four workgroups (2 halves x 2 nets) runs the
        // heads. The hand-off without fences (an agent release / acquire pair is a write-back of
        // the XCD's L2 and an L1 invalidate, ~3.5 us per workgroup): this wave stores its
        // slab with sc1 stores and waits for them, then one lane counts with a relaxed agent
        // atomic; the last arriver, told by the value its add returned, reads every slab with
        // sc1 loads (head_pair_one), which bypass the stale L1 and find the data in memory.
        // Why this is ordered without a release / acquire pair (an ISA-level
        // argument, gfx950 only, not one the HIP / C++ memory model gives):
        //  (1) the slab stores are agent-scope relaxed atomic stores: `global_store ... sc1`,
        //      which write through the XCD's L2 to the memory side (MALL / HBM) that every XCD
        //      reads;
        //  (2) stores retire in vmcnt in issue order and a store's count drops only when the
        //      memory side acknowledged it at the requested scope, so after `s_waitcnt
        //      vmcnt(0)` every lane's slab value is visible to agent-scope readers;
        //  (3) the asm's "memory" clobber keeps the compiler from sinking the stores below it
        //      or hoisting the ticket above it, so the ticket add is issued after (2);
        //  (4) the add is an agent-scope RMW on one address: its results are totally ordered,
        //      so the workgroup that reads 3 comes after the other three's adds, hence after
        //      their slabs were visible;
        //  (5) the reader loads the slabs with agent-scope relaxed atomic loads (`global_load
        //      ... sc1`: L1 bypassed, no stale line), issued only after its own add returned
        //      (a control dependence plus the compiler barrier below, so no load is
        //      speculated above the branch).
        // The UPD_SC1 = 0 build (an acq_rel ticket: wbl2 + inv per workgroup, 0.0703 against
        // 0.0734 ms per update, profiles/r05n_ab.txt) is the formally ordered cross-check:
        // libsnakehip_acqrel.so (csrc/Makefile, built with the library) and
        // test_update_sc1_handoff_matches_acq_rel_build (bit-identical loss and gradient).
        uint32_t last = 0;
#if UPD_SC1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (tid == 0)
            last = __hip_atomic_fetch_add(args.ticket + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 3u;
#else   // (A/B builds) the release / acquire pair
        if (tid == 0)
            last = __hip_atomic_fetch_add(args.ticket + s, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == 3u;
#endif
        last = __shfl(last, 0, 64);
        if (!last) return;
        asm volatile("" ::: "memory");   // (5): no slab load above the ticket's result
        if (tid == 0) __hip_atomic_store(args.ticket + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        head_pair_one(args.hn[0], args.hn[1], 2, args.S, L, args.ha, s, tid, hpre);
        UPD_CLK(6);
    }
}

}  // namespace snk

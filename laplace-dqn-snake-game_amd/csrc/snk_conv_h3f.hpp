// snk_conv_h3f.hpp — conv1 + conv2 + conv3 of the large-batch act forward in ONE
// kernel on the h3 split (snk_conv_h3.hpp).
//
// conv1 (3x3, C -> 16, fp32 VALU in conv1_fwd_kernel's order, bit-identical) runs
// first, from the workgroup's four boards staged as floats in LDS (in the conv3 B
// buffers, idle until conv2 is done): a1 never goes to memory either, which saves
// the conv1 launch and a1's write + re-read (9.2 KB per sample at 12x12).
//
// conv_h3s_kernel stages four samples' fp32 conv2 outputs (a2, 18 KB each at
// 12x12) from HBM, takes a per-sample max and splits them into its LDS A image.
// Here the same workgroup computes those four samples' conv2 itself: it stages
// their fp32 conv1 outputs (a1, half the bytes of a2) with a per-sample scale
// into a zero-bordered fp16 h/l image, splits the conv2 weights (9 x 32 x 16,
// per-tensor scale) into paired-offset fragments, runs conv2's 16-row tiles on
// v_mfma_f32_16x16x32_f16 (3 part products), applies bias + relu, reduces the
// per-sample max of the result in the workgroup and writes the split conv2
// output straight into conv3's A image (which overlays the conv2 staging
// area). conv3 then runs conv_h3s_kernel's pipeline unchanged. a2 never goes
// to memory: per sample this saves the a2 write and re-read (2 x 18 KB) and
// the conv2 launch; the arithmetic and the error class of each conv are those
// of conv_h3c2_kernel + conv_h3s_kernel.
#pragma once

#include "snk_conv_h3.hpp"
#include "snk_qnet.hpp"

namespace snk {

struct H3FArgs {
    BoardSrc src;        // the input planes (env frame ring, replay slots or floats)
    const float *w1;     // conv1 weights W[(kk * C + ci) * 16 + co] (packed theta; C = the CF template)
    const float *b1;     // conv1 bias [16]
    const float *w2;     // conv2 forward image [9 kk][32 co][16 ci]
    const float *b2;     // conv2 bias [32]
    const float *w3;     // conv3 forward image [36 kk][64 co][32 ci]
    const float *wmax;   // partial max |w3| (conv1_fwd_kernel / wmax_scan_kernel)
    int nwmax;
    const float *b3;     // conv3 bias [64]
    float *out;          // a3 [S][ho^2][64]
    SampleRider rider;   // rider.out: one extra workgroup runs this replay draw (the trainer's update sample)
    // NBUF = 8: w3 pre-split (w3_split_kernel) into the B buffers' byte order, copied by LDS-DMA;
    // w2h the conv2 weights pre-split into the B2 image's bytes (H3F_B2_CHUNKS 16-byte chunks)
    const uint16_t *w3h;
    const int *w3e;      // w3h's exponent (ew), then w2h's (ew2)
    const uint16_t *w2h;
    float *a3max;        // optional: max of each sample's a3 (>= 0: post-relu), for Dense1's h3 scale
    uint32_t *ticket;    // optional (NBUF 8, boards from the env frame ring or floats): persistent
                         // launch, one workgroup per CU; the group counter, zero between launches
};
// conv2's split weight image in LDS: [5 offset pairs][h | l][32 co][48 halves] (k = 16 (kk & 1)
// + ci in the first 32 halves of a row; kk = 9 is zero), 1,920 16-byte chunks, padded to 2,048
constexpr int H3F_B2_BR = 48, H3F_B2_CHUNKS = 2048;
// conv3 LDS-DMA lookahead (NBUF 8): offset kk + H3F_LA is issued while kk runs
#ifndef H3F_LA
#define H3F_LA 4
#endif
// measurement builds (-DSNK_H3F_VAR=n with SNK_ENV_CLOCKS, phase clocks): the conv3 offset
// loop without its LDS-DMA (1), its barriers (2), its MFMAs (3) or its fragment reads (4)
#ifndef SNK_H3F_VAR
#define SNK_H3F_VAR 0
#endif
#if SNK_H3F_VAR && !defined(SNK_ENV_CLOCKS)
#error "SNK_H3F_VAR: measurement (clocks) builds only"
#endif
// persistent passes after the first read conv1's weights from LDS (0: from L2, A/B builds)
#ifndef H3F_W1LDS
#define H3F_W1LDS 1
#endif
// conv3's output stored from the accumulators instead of through LDS
#ifndef H3F_DIRECT
#define H3F_DIRECT 0
#endif
// persistent conv_h3f_kernel launches (H3FArgs::ticket) for the act forward: +0.3-0.6 % on the
// headline loop in three interleaved A/B rounds (profiles/r05o_h3f_ab.txt); 0 = one workgroup
// per group of four samples (measurement builds)
#ifndef H3F_PERSIST
#define H3F_PERSIST 1
#endif
static_assert(H3F_LA >= 4 && H3F_LA <= 7, "lookahead: 4..7 (buffer 7 holds conv1's boards in the prologue)");

// conv3's weight image [36 kk][64 co][32 ci] (fp32) -> fp16 h / l parts of w * 2^ew, ew from the
// partial maxima, laid out exactly as conv_h3f_kernel's register path stores one offset into a B
// buffer (512 16-byte chunks per offset: h chunk x6s_bswz(c), l chunk x6s_bswz(256 + c) for the
// chunk c = (co, ci / 8); each of its two 8-byte halves one float4 of the image): a lane-linear
// copy of an offset's 8 KB is then a B buffer. One thread per float4 of the image.
// Blocks 72..76: conv2's image [9 kk][32 co][16 ci] (fp32, 1,152 float4) split with its own
// per-tensor exponent ew2 = h3_exp(max |w2|) into the B2 image (out2, zero-initialised: the
// pad offset and the pad columns stay zero), eout[1] = ew2.
// Blocks 77.. (when out1): Dense1's image [nkk positions][64 out][64 in] split row by row
// (one row = 64 inputs of one output at one position = 16 lanes, one float4 each) with the
// row's own exponent e1[kk * 64 + out] = h3_exp(max |row|) into planes
// out1[kk][h | l][64 out][64 in], 16-byte chunk q of a row at q ^ (out & 7) (dense_h3_kernel's
// fragment reads: distinct bank quads). A per-(position, output) scale factors out of the
// position's partial sum, so each is scaled back on its own.
constexpr int W3S_BLOCKS = 36 * 512 / 256, W2S_BLOCKS = (9 * 32 * 16 / 4 + 255) / 256;
// The weight splits' exponents leave H3_W_HEADROOM bits of fp16 range above the maximum (scaled
// maximum in [2^10, 2^11) instead of h3_exp's [2^14, 2^15)): the training loop's grad_update_kernel
// re-splits the updated weights with the exponents of the last w3_split_kernel (a chained act
// forward skips the split launch), which stays exact while no weight has grown 32-fold since;
// the trainer runs w3_split_kernel again at the start of every captured graph. The cost is
// nil: each element keeps its 22-bit h + l form, only values below 2^-14 of the maximum (whose l
// part falls into the fp16 subnormals) carry an absolute error <= 2^-36 of the maximum
// The headroom alone does not bound a tensor (or Dense1 row) whose maximum is tiny: RMSProp moves
// a weight by up to lr / sqrt(1 - rho) per step whatever its size (|g| / sqrt(acc) <= 1 / sqrt(1 -
// rho)), so a row with max 1e-3 can grow past 32x its max within a graph. The trainer
// passes `grow`, a bound on that movement until the next fresh split (steps x lr / sqrt(1 - rho),
// doubled for the fp32 rounding of the update), and the exponent is also capped so that
// (max + grow) 2^e < 2^15: a chained split then stays below 2^15 < 65504 (the fp16 maximum) by
// construction. The cap binds only when grow > ~15x the maximum (a maximum below ~0.007 at
// lr 5e-4 and 64 chained steps), so the usual exponents, and the bits, are unchanged
// (test_split_chain_exponent_cap_keeps_q_finite).
constexpr int H3_W_HEADROOM = 4;
__device__ __forceinline__ int h3_exp_w(float m, float grow = 0.0f) {
    const int e = h3_exp(m) - H3_W_HEADROOM;
    return grow > 0.0f ? min(e, h3_exp(m + grow)) : e;
}
__host__ __device__ constexpr int w1s_blocks(int nkk) { return nkk * 64 * 16 / 256; }
static __global__ __launch_bounds__(256) void w3_split_kernel(const float *__restrict__ img, const float *__restrict__ wmax,
                                                       int nwmax, uint16_t *__restrict__ out, int *__restrict__ eout,
                                                       const float *__restrict__ img2, uint16_t *__restrict__ out2,
                                                       const float *__restrict__ img1 = nullptr,
                                                       uint16_t *__restrict__ out1 = nullptr, int *__restrict__ e1 = nullptr,
                                                       float grow = 0.0f) {
    __shared__ float red4[4];
    if (blockIdx.x >= W3S_BLOCKS + W2S_BLOCKS) {   // Dense1
        const int t = (blockIdx.x - W3S_BLOCKS - W2S_BLOCKS) * 256 + threadIdx.x;
        const int row = t >> 4, q4 = t & 15, kk = row >> 6, o = row & 63;
        const f32x4 v = reinterpret_cast<const f32x4 *>(img1)[t];
        float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        m = dpp_max<0xB1>(m);    // the 16-lane row's max (wave_max's first four steps)
        m = dpp_max<0x4E>(m);
        m = dpp_max<0x141>(m);
        m = dpp_max<0x140>(m);
        const int ex = h3_exp_w(m, grow);
        if (q4 == 0) e1[row] = ex;
        u32x2 hh, ll;
        h3_split4(v, ex, hh, ll);
        const int off = (o * 64 + (((q4 >> 1) ^ (o & 7)) << 3) + ((q4 & 1) << 2)) / 4;   // in u32x2 units
        u32x2 *o1 = reinterpret_cast<u32x2 *>(out1 + (int64_t)kk * 2 * 4096);
        o1[off] = hh;
        o1[1024 + off] = ll;
        return;
    }
    if (blockIdx.x >= W3S_BLOCKS) {   // conv2
        constexpr int NW4 = 9 * 32 * 16 / 4;
        const f32x4 *w4 = reinterpret_cast<const f32x4 *>(img2);
        const int e = (blockIdx.x - W3S_BLOCKS) * 256 + threadIdx.x;
        float m = 0.0f;
        for (int i = threadIdx.x; i < NW4; i += 256) {
            const f32x4 v = w4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
        m = wave_max(m);
        if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
        __syncthreads();
        const int ew2 = h3_exp_w(fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3])), grow);
        if (blockIdx.x == W3S_BLOCKS && threadIdx.x == 0) eout[1] = ew2;
        if (e < NW4) {
            const int kk = e >> 7, co = (e >> 2) & 31, ci0 = 4 * (e & 3);
            const int p = kk >> 1, k0 = 16 * (kk & 1) + ci0;
            u32x2 hh, ll;
            h3_split4(w4[e], ew2, hh, ll);
            u32x2 *o2 = reinterpret_cast<u32x2 *>(out2);
            o2[(((p * 2 + 0) * 32 + co) * H3F_B2_BR + k0) / 4] = hh;
            o2[(((p * 2 + 1) * 32 + co) * H3F_B2_BR + k0) / 4] = ll;
        }
        return;
    }
    const int t = blockIdx.x * 256 + threadIdx.x;   // < 36 * 512
    const int kk = t >> 9, tt = t & 511;
    const f32x4 v = reinterpret_cast<const f32x4 *>(img)[t];   // in flight beside the partial maxima
    float m = 0.0f;
    for (int i = threadIdx.x; i < nwmax; i += 256) m = fmaxf(m, wmax[i]);
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
    const int ew = h3_exp_w(fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3])), grow);
    if (blockIdx.x == 0 && threadIdx.x == 0) *eout = ew;
    const int bch = (tt >> 3) * 4 + ((tt & 7) >> 1), bhalf = tt & 1;
    u32x2 h, l;
    h3_split4(v, ew, h, l);
    u32x2 *o = reinterpret_cast<u32x2 *>(out) + (int64_t)kk * 512 * 2;
    o[x6s_bswz(bch) * 2 + bhalf] = h;
    o[x6s_bswz(256 + bch) * 2 + bhalf] = l;
}

// Profiling builds only (make clocks): per-workgroup phase timestamps, read back by
// snk_h3f_debug_clocks (slots: start, conv1, scales + splits, conv2, conv3 image + B
// stages, conv3 offsets, end)
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_h3f_clk;
#define H3F_CLK(slot)                                                                                 \
    do {                                                                                              \
        if (threadIdx.x == 0 && g_h3f_clk) g_h3f_clk[(int64_t)grp * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define H3F_CLK(slot) do { } while (0)
#endif

template <int HIN, int NBUF = 4>
constexpr int h3f_lds_bytes() {
    constexpr int ho = HIN - 5, XW = ho + 8, PL = (HIN * XW + 3) & ~3, XS = 4 * 2 * PL + 4;
    constexpr int BP = HIN + 2;
    constexpr int c2 = (4 * 2 * BP * BP * 16 + 2048 * 8) * 2;   // conv2 staging: A1 image + the B2 image (2,048 chunks)
    constexpr int c3 = 4 * XS * 16;                                     // conv3 A image
    constexpr int cs = 4 * ho * ho * 80 * 4;                            // output staging
    constexpr int m = c2 > c3 ? (c2 > cs ? c2 : cs) : (c3 > cs ? c3 : cs);
    return NBUF * 512 * 16 + m;
}

// NBUF conv3 B buffers: 2 = one barrier per kernel offset (B(kk+2) staged while kk
// runs); 4 = one barrier per offset PAIR (B(kk+3) staged, read two offsets later)
template <int HIN, int NBUF = 4, int CF = 2>
__global__ __launch_bounds__(512) void conv_h3f_kernel(H3FArgs a_, int S) {
    static_assert(NBUF == 2 || NBUF == 4 || NBUF == 8, "B buffers");
    // NBUF 8: the B buffers are filled by LDS-DMA from the pre-split image a.w3h (no
    // register staging, no split): offset kk + 4 is issued while kk runs
    constexpr bool DMA = NBUF == 8;
    constexpr int KS = 6, CN = 64, CK = 32, NSG = 4, NB = 2 * CN * CK / 8;
    constexpr int NKK = KS * KS;
    constexpr int hin = HIN, ho = HIN - KS + 1, ho2 = ho * ho, hin2 = hin * hin;
    constexpr int XW = ho + 8, PL = (hin * XW + 3) & ~3, GG = 2 * PL, XS = 4 * GG + 4;
    // A1 rows of 16 halves and B2 rows of 48: 2 and 6 16-byte units per row, for which
    // the ds_read_b128 lane groups of the conv2 fragment reads hit 16 distinct bank quads
    constexpr int BP = HIN + 2, NPB = BP * BP, XR = 16, BR = 48, XP = XR / 8;
    constexpr int A1_H = NSG * 2 * NPB * XR;   // the B2 image (5 x 2 x 32 x BR halves) follows
    constexpr int R2 = NSG * hin2, T2 = (R2 + 15) / 16, U2 = (T2 + 7) / 8;
    constexpr int NW4 = 9 * 32 * 16 / 4, LW = (NW4 + 511) / 512, LA = (NSG * hin2 * 4 + 511) / 512;
    static_assert(XR % 8 == 0 && BR % 8 == 0, "16-byte pieces");
    // the rider's workgroup is workgroup 0 (dispatched first: its serial draw overlaps the
    // sample groups instead of trailing them); it touches no LDS and no barrier
    const int rb = a_.rider.out ? 1 : 0;
    if (rb && blockIdx.x == 0) {
        if (threadIdx.x < 64) sample_wave(a_.rider);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) u32x4 h3f_lds[];
    __shared__ float red[8][7];
    __shared__ float a3red[8][4][4];   // [wave][row][sample]: the epilogue's per-sample a3 maxima
    u32x4 *Bs = h3f_lds;               // conv3 B [NBUF][NB]
    u32x4 *As = h3f_lds + NBUF * NB;   // conv3 A image; during conv2: A1 image, B2 image
    u32x2 *Bs2 = reinterpret_cast<u32x2 *>(Bs);
    uint16_t *A1 = reinterpret_cast<uint16_t *>(As), *B2 = A1 + A1_H;
    u32x2 *A1v = reinterpret_cast<u32x2 *>(A1), *B2v = reinterpret_cast<u32x2 *>(B2);
    // persistent mode (a.ticket; H3F_PERSIST builds, env frame ring boards): the grid is at most one workgroup per CU; each runs group
    // blockIdx - rb first, then group nwg + t for each ticket t it draws (one draw per group,
    // at the group's start; the draw that returns ngroups - 1 is the launch's last and resets
    // the counter). The next group's board cells are loaded into registers between the
    // current group's conv3 offsets and its epilogue, so their latency hides behind it.
    const bool persist = H3F_PERSIST && DMA && a_.ticket != nullptr;
    const int ngroups = (S + NSG - 1) / NSG, nwg = (int)gridDim.x - rb;
    int grp = (int)blockIdx.x - rb;
    constexpr int NX = NSG * CF * NPB, LB = (NX + 511) / 512;
    int bv[LB];                // this thread's board cells of the group ([sample][channel][bordered cell])
    bool have_boards = false;  // bv holds the group's cells already (persistent passes after the first)
    const int8_t *cbase0 = nullptr, *cbase1 = nullptr;   // persistent, env frame ring: plane(s, c) = cbase_c + s * pitch
    __shared__ int s_next;     // persistent: the group this workgroup runs next
#if H3F_PERSIST
    for (;;) {
    // the weights' pointers and the thread index through an empty asm per pass: their loads
    // and the address arithmetic on tid stay in the pass (hoisted out of the group loop they
    // held ~100 VGPRs through conv3 and spilled); & 511 restores tid's range
    H3FArgs a = a_;
    asm volatile("" : "+s"(a.w1), "+s"(a.b1), "+s"(a.b2), "+s"(a.b3), "+s"(a.w3e), "+s"(a.w2), "+s"(a.w3), "+s"(a.wmax));
    int z_ = 0;
    asm volatile("" : "+s"(z_));
    const int tid = ((int)threadIdx.x + z_) & 511;
#else
    const H3FArgs &a = a_;
    const int tid = threadIdx.x;
#endif
    const int lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int s0 = grp * NSG;
    const int ns = min(NSG, S - s0);
    H3F_CLK(0);
    uint32_t tk = 0;
    if (persist && tid == 0) tk = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);

    // conv3 B register sets (as conv_h3s_kernel)
    const f32x4 *__restrict__ wsrc = reinterpret_cast<const f32x4 *>(a.w3);
    f32x4 bst[2];
    auto b_load = [&](int kk, int set) {
        if constexpr (!DMA) bst[set] = wsrc[(int64_t)min(kk, NKK - 1) * NB + tid];
    };
    const int bch = (tid >> 3) * 4 + ((tid & 7) >> 1);
    const int bhalf = tid & 1;
    int ew = 0;
    auto b_store = [&](int buf, int set) {
        if constexpr (!DMA) {
            u32x2 h, l;
            h3_split4(bst[set], ew, h, l);
            Bs2[(buf * NB + x6s_bswz(bch)) * 2 + bhalf] = h;
            Bs2[(buf * NB + x6s_bswz(256 + bch)) * 2 + bhalf] = l;
        }
    };
    // DMA: offset kk's pre-split 8 KB into buffer kk & 7, chunk tid by lane tid (past the
    // last offset: harmless reloads of it)
    auto dma = [&](int kk) __attribute__((always_inline)) {
        if constexpr (DMA) {
            const int k = min(kk, NKK - 1);
            __builtin_amdgcn_global_load_lds((const void *)(a.w3h + ((int64_t)k * NB + tid) * 8),
                                             (__attribute__((address_space(3))) void *)(Bs + (kk & (NBUF - 1)) * NB + wave * 64),
                                             16, 0, 0);
        }
    };
    // DMA: conv2's weights and conv3's offsets 0..3 are issued once the boards are staged
    // (below): vmcnt retires in order, so a load issued after them and used during conv1
    // would wait for them (they sat in front of the boards, and every __syncthreads drained
    // them)
    auto dma_prologue = [&]() __attribute__((always_inline)) {
        if constexpr (DMA) {
            static_assert(H3F_B2_CHUNKS == 4 * 512, "four B2 pieces per thread");
#pragma unroll
            for (int q = 0; q < 4; ++q)
                __builtin_amdgcn_global_load_lds((const void *)(a.w2h + ((int64_t)q * 512 + tid) * 8),
                                                 (__attribute__((address_space(3))) void *)(B2 + (q * 512 + wave * 64) * 8),
                                                 16, 0, 0);
#pragma unroll
            for (int k = 0; k < H3F_LA; ++k) dma(k);   // conv1 stages its boards in buffer 7
        }
    };
    // LDS-only barrier (no vmcnt drain) while the prologue DMAs are in flight
    auto lds_barrier = [&]() __attribute__((always_inline)) {
        if constexpr (DMA) {
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
            __builtin_amdgcn_s_barrier();
        } else {
            __syncthreads();
        }
    };
    if constexpr (!DMA) {
        b_load(0, 0);
        b_load(1, 1);
    }
    // conv3 weight-max partials: loaded here, reduced after conv1 (their latency hides
    // behind the board loads instead of following conv1)
    const float wmx = !DMA && tid < a.nwmax ? a.wmax[tid] : 0.0f;
    const int ew_dma = DMA ? a.w3e[0] : 0, ew2_dma = DMA ? a.w3e[1] : 0;

    // conv2 bias of this lane's output channels (16 ct + 4 g + e), early
    float b2v[2][4];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 4; ++e) b2v[ct][e] = a.b2[ct * 16 + 4 * g + e];

    // ---- conv2 staging: zero the A1 image's border positions and B2's pad offset
    // (kk = 9: k 16..31 of pair 4); the rest is overwritten below
    {
        constexpr int NBD = 4 * (BP - 1);   // border positions per plane
        for (int q = tid; q < NSG * 2 * NBD * XP; q += 512) {
            const int pc = q / (NBD * XP), rem = q - pc * NBD * XP, bpos = rem / XP, piece = rem - bpos * XP;
            const int side = bpos / (BP - 1), t = bpos - side * (BP - 1);
            const int pb = side == 0 ? t : side == 1 ? (BP - 1) + t * BP : side == 2 ? (BP * BP - 1) - t
                                                                                     : (BP - 1 - t) * BP;
            reinterpret_cast<u32x4 *>(A1)[((pc * NPB + pb) * XR) / 8 + piece] = u32x4{0u, 0u, 0u, 0u};
        }
        if (!DMA && tid < 2 * 32 * 2) {   // plane, co, two 16-byte pieces (k 16..31)
            const int pl = tid >> 6, co = (tid >> 1) & 31, piece = tid & 1;
            reinterpret_cast<u32x4 *>(B2)[(((4 * 2 + pl) * 32 + co) * BR + 16) / 8 + piece] = u32x4{0u, 0u, 0u, 0u};
        }
    }
    f32x4 wv[LW], av[LA];
    float a1b = 0.0f;   // the group's bound on conv1's output (below)
    const f32x4 *w4 = reinterpret_cast<const f32x4 *>(a.w2);
    const int na4 = ns * hin2 * 4;
#pragma unroll
    for (int u = 0; u < LW; ++u)
        if (!DMA) wv[u] = w4[min(u * 512 + tid, NW4 - 1)];
    {
        // ---- conv1: boards -> bordered float planes in the B buffers; each thread always
        // computes the same four output channels (4 (tid & 3) .. +3), so its 9 CF weight
        // quads live in registers and a tap costs one LDS float
        constexpr int C = CF;
        // [NSG][C][NPB]; DMA: in buffer 7 (buffers 0..3 are filling already)
        float *xin = reinterpret_cast<float *>(Bs + (DMA ? 7 * NB : 0));
        static_assert(NSG * C * NPB <= (DMA ? NB : NBUF * NB) * 4, "conv1 staging fits the B buffers");
        __shared__ const int8_t *pbase[NSG * C];
        if (!have_boards && tid < NSG * C) pbase[tid] = tid / C < ns ? a.src.plane(s0 + tid / C, tid % C) : nullptr;
        const int cq = tid & 3;
        f32x4 w1r[9 * C], b1r;
        // the conv1 weights and bias: from L2 in the first pass, which also parks them in LDS; the
        // persistent passes after it read them there (an L2 round trip in front of conv1 each)
        __shared__ f32x4 w1s[9 * C * 4 + 4];
        if (!have_boards || !H3F_W1LDS) {
#pragma unroll
            for (int q = 0; q < 9 * C; ++q) w1r[q] = reinterpret_cast<const f32x4 *>(a.w1)[q * 4 + cq];
            b1r = reinterpret_cast<const f32x4 *>(a.b1)[cq];
            if (persist && H3F_W1LDS && tid < 9 * C * 4 + 4)
                w1s[tid] = tid < 9 * C * 4 ? reinterpret_cast<const f32x4 *>(a.w1)[tid]
                                           : reinterpret_cast<const f32x4 *>(a.b1)[tid - 9 * C * 4];
        } else {
#pragma unroll
            for (int q = 0; q < 9 * C; ++q) w1r[q] = w1s[q * 4 + cq];
            b1r = w1s[9 * C * 4 + cq];
        }
        const bool fl = a.src.fbase != nullptr;
        if (!have_boards) {
            __syncthreads();
            // every cell load of the thread goes out before the first is used (a loop of
            // load-then-store waited out one round trip per cell), through global (not flat)
            // pointers: the plane pointers come from LDS as generic ones
            typedef const __attribute__((address_space(1))) int8_t gi8;
            int bsc[LB], bcell[LB];
            bool bin[LB];
#pragma unroll
            for (int u = 0; u < LB; ++u) {
                const int q = u * 512 + tid;
                const int sc = min(q / NPB, NSG * C - 1), b = q - sc * NPB;
                const int bj = b / BP, bi = b - bj * BP;
                bsc[u] = sc;
                bcell[u] = (bi - 1) + (bj - 1) * hin;
                bin[u] = q < NX && sc / C < ns && bi >= 1 && bi <= hin && bj >= 1 && bj <= hin;
            }
            if (fl) {
#pragma unroll
                for (int u = 0; u < LB; ++u)
                    bv[u] = bin[u] ? __float_as_int(a.src.fbase[((int64_t)(s0 + bsc[u] / C) * C + bsc[u] % C) * hin2 + bcell[u]]) : 0;
            } else {
                gi8 *pl[LB];
#pragma unroll
                for (int u = 0; u < LB; ++u) pl[u] = (gi8 *)pbase[bsc[u]];
#pragma unroll
                for (int u = 0; u < LB; ++u) bv[u] = bin[u] ? (int)pl[u][bcell[u]] : 0;
            }
            // the ring's slot of each channel is the launch's (one step counter): the first
            // group's sample-0 planes give every later group's
            // (two scalars, not an array: a selected array element went to scratch)
            if (persist) {
                cbase0 = pbase[0] - (int64_t)s0 * a.src.pitch;
                cbase1 = pbase[C - 1] - (int64_t)s0 * a.src.pitch;
            }
        }
        float xm = 0.0f;   // max |x| over the thread's cells (absent cells are 0)
#pragma unroll
        for (int u = 0; u < LB; ++u) {
            const int q = u * 512 + tid;
            const float xv = fl ? __int_as_float(bv[u]) : (float)bv[u];
            if (q < NX) {   // [sample][bordered cell][channel]: a tap's C channels in one LDS read
                const int sc = q / NPB, b = q - sc * NPB;
                xin[((sc / C) * NPB + b) * C + sc % C] = xv;
            }
            xm = fmaxf(xm, fabsf(xv));
        }
        xm = wave_max(xm);
        if (lane == 0) red[wave][6] = xm;
        // after the boards are consumed: the compiler does not count LDS-DMAs in its vmcnt
        // waits, so a wait for a load issued before them comes out as vmcnt(0)
        __builtin_amdgcn_sched_barrier(0);
        dma_prologue();
        __builtin_amdgcn_sched_barrier(0);
        lds_barrier();
#pragma unroll
        for (int u = 0; u < LA; ++u) {   // output (sample, position, channels 4 cq..): a1's layout
            const int e = min(u * 512 + tid, na4 - 1);
            const int sr = e / (hin2 * 4), pos = (e - sr * hin2 * 4) >> 2;
            const int j = pos / hin, i = pos - j * hin;
            // channel pairs on v_pk_fma_f32 (two fp32 FMAs per lane and instruction; each
            // channel's FMA chain and rounding are the scalar form's)
            f32x2 acc01{b1r[0], b1r[1]}, acc23{b1r[2], b1r[3]};
#pragma unroll
            for (int kk = 0; kk < 9; ++kk) {
                const int du = kk % 3, dv = kk / 3;
                const float *xp = xin + (sr * NPB + (i + du) + (j + dv) * BP) * C;
                float xc[C];
                if constexpr (C == 2) {
                    const f32x2 x2 = *reinterpret_cast<const f32x2 *>(xp);
                    xc[0] = x2[0];
                    xc[C - 1] = x2[1];
                } else {
#pragma unroll
                    for (int c = 0; c < C; ++c) xc[c] = xp[c];
                }
#pragma unroll
                for (int c = 0; c < C; ++c) {
                    const float x = xc[c];
                    const f32x2 xx{x, x};
                    const f32x4 w = w1r[kk * C + c];
                    acc01 = __builtin_elementwise_fma(xx, f32x2{w[0], w[1]}, acc01);
                    acc23 = __builtin_elementwise_fma(xx, f32x2{w[2], w[3]}, acc23);
                }
            }
            av[u] = f32x4{fmaxf(acc01[0], 0.f), fmaxf(acc01[1], 0.f), fmaxf(acc23[0], 0.f), fmaxf(acc23[1], 0.f)};
        }
        // conv1's output bound: a1[c] <= |b1[c]| + max|x| * sum over taps |w1[tap][c]| for every
        // sample of the group; the thread's four channels, then the quad's sixteen by DPP
        float xg = red[0][6];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) xg = fmaxf(xg, red[w8][6]);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float sw = 0.0f;
#pragma unroll
            for (int q = 0; q < 9 * C; ++q) sw += fabsf(w1r[q][e]);
            a1b = fmaxf(a1b, fabsf(b1r[e]) + xg * sw);
        }
        a1b = dpp_max<0x4E>(dpp_max<0xB1>(a1b));
    }
    H3F_CLK(1);
    float wm3 = wmx;
    if (!DMA)
        for (int i = tid + 512; i < a.nwmax; i += 512) wm3 = fmaxf(wm3, a.wmax[i]);
    // A1's exponent is the group's bound's, not each sample's max |a1| (a reduction and a
    // barrier fewer): the h3 split is scale-free, so this changes nothing but where an
    // element's l part meets the fp16 subnormals (values below ~2^-27 of the bound)
    int ea1[NSG], ew2 = ew2_dma;
#pragma unroll
    for (int q = 0; q < NSG; ++q) ea1[q] = h3_exp(a1b);
    if constexpr (!DMA) {   // conv2 / conv3 weight exponents from the data
        float mw2 = 0.0f;
#pragma unroll
        for (int u = 0; u < LW; ++u) {
            const f32x4 v = wv[u];
            if (u * 512 + tid < NW4)
                mw2 = fmaxf(mw2, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
        }
        mw2 = wave_max(mw2);
        wm3 = wave_max(wm3);
        if (lane == 0) {
            red[wave][4] = mw2;
            red[wave][5] = wm3;
        }
        lds_barrier();
        float m4 = red[0][4], m5 = red[0][5];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) {
            m4 = fmaxf(m4, red[w8][4]);
            m5 = fmaxf(m5, red[w8][5]);
        }
        ew2 = h3_exp(m4);
        ew = h3_exp(m5);
    } else {
        ew = ew_dma;
    }
#pragma unroll
    for (int u = 0; u < LW; ++u) {   // image [kk][co][ci]: k = 16 * (kk - 2p) + ci in offset pair p
        const int e = u * 512 + tid;
        if (!DMA && e < NW4) {
            const int kk = e >> 7, co = (e >> 2) & 31, ci0 = 4 * (e & 3);
            const int p = kk >> 1, k0 = 16 * (kk & 1) + ci0;
            u32x2 hh, ll;
            h3_split4(wv[u], ew2, hh, ll);
            B2v[(((p * 2 + 0) * 32 + co) * BR + k0) / 4] = hh;
            B2v[(((p * 2 + 1) * 32 + co) * BR + k0) / 4] = ll;
        }
    }
#pragma unroll
    for (int u = 0; u < LA; ++u) {   // a1 [s][pos][16] -> bordered [s][part][pos][24 halves]
        const int e = u * 512 + tid;
        if (e < na4) {
            const int sr = e / (hin2 * 4), loc = e - sr * hin2 * 4;
            const int pos = loc >> 2, c0 = 4 * (loc & 3);
            const int j = pos / hin, i = pos - j * hin;
            const int pb = (i + 1) + (j + 1) * BP;
            const int es = sr == 0 ? ea1[0] : sr == 1 ? ea1[1] : sr == 2 ? ea1[2] : ea1[3];
            u32x2 hh, ll;
            h3_split4(av[u], es, hh, ll);
            A1v[(((sr * 2 + 0) * NPB + pb) * XR + c0) / 4] = hh;
            A1v[(((sr * 2 + 1) * NPB + pb) * XR + c0) / 4] = ll;
        }
    }
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(waitcnt_vm(H3F_LA));   // conv2's weights landed (the offsets may not)
    lds_barrier();
    H3F_CLK(2);

    // ---- conv2, transposed: C^T[co][row] = sum_k W[co][k] * A[row][k] with the weight
    // fragments as the MFMA's A operand and the activation fragments as its B (the
    // same register layouts): a lane then holds 4 consecutive channels of one row,
    // written to conv3's image as one 8-byte piece per part. 16-row tiles
    // t = wave + 8u; offset pair p outermost so each weight fragment is read once
    f32x4v acc2[U2][2];
    // this lane's row (column r of tile u): sample, A1-image position, conv3 image slot
    int rsl[U2], rpos[U2], aslot[U2];
#pragma unroll
    for (int u = 0; u < U2; ++u) {
        acc2[u][0] = acc2[u][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
        const int q = min((wave + 8 * u) * 16 + r, R2 - 1);
        rsl[u] = q / hin2;
        const int pos = q - rsl[u] * hin2, j = pos / hin, i = pos - j * hin;
        rpos[u] = i + j * BP;
        aslot[u] = rsl[u] * XS + (g >> 1) * GG + j * XW + i;
    }
#pragma unroll
    for (int p = 0; p < 5; ++p) {
        f16x8 wh[2], wl[2];
#pragma unroll
        for (int ct = 0; ct < 2; ++ct) {
            const uint16_t *pb = B2 + ((p * 2) * 32 + ct * 16 + r) * BR + 8 * g;
            wh[ct] = as_h(*reinterpret_cast<const u32x4 *>(pb));
            wl[ct] = as_h(*reinterpret_cast<const u32x4 *>(pb + 32 * BR));
        }
        const int kk = min(2 * p + (g >> 1), 8), du = kk % 3, dv = kk / 3;
        // every wave has tiles u < UF: their fragments are all read before any MFMA of
        // the pair (no wave-uniform branch between a read and its use, so the reads go
        // out together and overlap the previous pair's MFMAs); tile UF, which only
        // waves < T2 - 8 UF have, runs under its branch
        constexpr int UF = T2 / 8;
        f16x8 fah[U2], fal[U2];
        auto frag = [&](int u) {
            const uint16_t *pa = A1 + ((rsl[u] * 2) * NPB + rpos[u] + du + dv * BP) * XR + 8 * (g & 1);
            fah[u] = as_h(*reinterpret_cast<const u32x4 *>(pa));
            fal[u] = as_h(*reinterpret_cast<const u32x4 *>(pa + NPB * XR));
        };
        auto tile = [&](int u) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                f32x4v c = acc2[u][ct];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ct], fal[u], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[ct], fah[u], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ct], fah[u], c, 0, 0, 0);
                acc2[u][ct] = c;
            }
        };
#pragma unroll
        for (int u = 0; u < UF; ++u) frag(u);
        if (U2 > UF && wave + 8 * UF < T2) {
            frag(U2 - 1);
            tile(U2 - 1);
        }
#pragma unroll
        for (int u = 0; u < UF; ++u) tile(u);
    }
    // acc2[u][ct][e]: channel co = 16 ct + 4 g + e of row (wave + 8u) * 16 + r.
    // bias + relu in place; per-sample max: the row's eight channels first, then one
    // select per sample (the lane's row is one sample's). Rows past R2 in the last tile
    // repeat row R2 - 1 (rsl is clamped), so they leave the maxima unchanged; rows of
    // absent samples only reach their own maxima and image rows, which no stored output
    // reads; a tile the wave does not have counts nothing
    float m2[NSG] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
    for (int u = 0; u < U2; ++u) {
        const int sr = rsl[u];
        const int es = (sr == 0 ? ea1[0] : sr == 1 ? ea1[1] : sr == 2 ? ea1[2] : ea1[3]) + ew2;
        float lm = 0.0f;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float v = fmaxf(__builtin_ldexpf(acc2[u][ct][e], -es) + b2v[ct][e], 0.0f);
                acc2[u][ct][e] = v;
                lm = fmaxf(lm, v);
            }
        if (wave + 8 * u >= T2) lm = 0.0f;
#pragma unroll
        for (int q = 0; q < NSG; ++q) m2[q] = sr == q ? fmaxf(m2[q], lm) : m2[q];
    }
#pragma unroll
    for (int q = 0; q < NSG; ++q) m2[q] = wave_max(m2[q]);
    if (lane == 0) {
#pragma unroll
        for (int q = 0; q < NSG; ++q) red[wave][q] = m2[q];
    }
    lds_barrier();   // also: every conv2 fragment read is done (the A image overlays them)
    H3F_CLK(3);
    int ea[NSG];
#pragma unroll
    for (int q = 0; q < NSG; ++q) {
        float m = red[0][q];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) m = fmaxf(m, red[w8][q]);
        ea[q] = h3_exp(m);
    }
    // conv2 output -> conv3's A image: slot(sample, channel group co >> 3, j, i); the lane's
    // four channels 4g..4g+3 (+16 ct) are halves 4 (g & 1) .. + 3 of one slot: 8-byte pieces
    u32x2 *Ah2 = reinterpret_cast<u32x2 *>(As);
#pragma unroll
    for (int u = 0; u < U2; ++u) {
        const int row = (wave + 8 * u) * 16 + r;
        if (wave + 8 * u < T2 && row < R2) {
            const int sr = rsl[u];
            const int es = sr == 0 ? ea[0] : sr == 1 ? ea[1] : sr == 2 ? ea[2] : ea[3];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int slot = aslot[u] + ct * 2 * GG;
                u32x2 hh, ll;
                h3_split4(f32x4{acc2[u][ct][0], acc2[u][ct][1], acc2[u][ct][2], acc2[u][ct][3]}, es, hh, ll);
                Ah2[slot * 2 + (g & 1)] = hh;
                Ah2[(slot + PL) * 2 + (g & 1)] = ll;
            }
        }
    }
    b_store(0, 0);
    b_store(1, 1);
    if constexpr (DMA) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // offsets 0..H3F_LA-1 landed (published below)

    constexpr int T = (NSG * ho2 + 15) / 16;
    const int rg = wave >> 1, cg = wave & 1;
    const int nt = __builtin_amdgcn_readfirstlane(T > rg ? (T - rg + 3) / 4 : 0);
    const int bslot = (cg * 32 + r) * 4 + (g ^ ((4 - ((r >> 2) & 3)) & 3));
    if (persist && tid == 0) {   // (the ticket returned long ago: the DMA waits above are in order)
        s_next = nwg + (int)tk;
        if (tk == (uint32_t)(ngroups - 1)) __hip_atomic_store(a.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // persistent: the next group's board cells into bv (after the conv3 offsets: no LDS-DMA in
    // flight, so the compiler's own vmcnt waits stay exact), as the first pass loads them
    auto prefetch = [&]() __attribute__((always_inline)) {
        const int gn = s_next;
        if (!persist || gn >= ngroups) return;
        const int s1 = gn * NSG, ns1 = min(NSG, S - s1);
        typedef const __attribute__((address_space(1))) int8_t gi8;
#pragma unroll
        for (int u = 0; u < LB; ++u) {
            const int q = u * 512 + tid;
            const int sc = min(q / NPB, NSG * CF - 1), b = q - sc * NPB;
            const int bj = b / BP, bi = b - bj * BP;
            const int sr = sc / CF, c = sc - sr * CF;
            const int cell = (bi - 1) + (bj - 1) * hin;
            const bool in = q < NX && sr < ns1 && bi >= 1 && bi <= hin && bj >= 1 && bj <= hin;
            const int8_t *cb = (CF > 1 && c) ? cbase1 : cbase0;
            bv[u] = in ? (int)((gi8 *)(cb + (int64_t)(s1 + sr) * a.src.pitch))[cell] : 0;
        }
    };

    // ---- conv3: conv_h3s_kernel's pipeline
    auto run = [&](auto ntc) {
        constexpr int NT = decltype(ntc)::value;
        int abase[NT];
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            const int q = 16 * (rg + 4 * k) + r;
            const int p = min(q >> 2, ho2 - 1), sr = q & 3;
            const int j = p / ho, i = p - j * ho;
            abase[k] = sr * XS + g * GG + j * XW + i;
        }
        f32x4v acc[NT][2];
#pragma unroll
        for (int k = 0; k < NT; ++k)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) acc[k][ct] = f32x4v{0.f, 0.f, 0.f, 0.f};
        // the epilogue's two bias values, loaded before the offsets (inside the epilogue the
        // compiler re-loaded and waited on them per row tile: three serial round trips)
        const float bv2[2] = {a.b3[cg * 32 + r], a.b3[cg * 32 + 16 + r]};
        struct Frag {
            u32x4 a[NT][2], b[2][2];
        };
        auto frag_read = [&](int kk, Frag &f) {
            kk = min(kk, NKK - 1);
            const int dv = kk / KS, du = kk - dv * KS;
            const int off = dv * XW + du;
            const u32x4 *pb = Bs + (kk & (NBUF - 1)) * NB + bslot;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) f.b[ct][pl] = pb[ct * 64 + pl * 256];
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const u32x4 *pa = As + abase[k] + off;
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) f.a[k][pl] = pa[pl * PL];
            }
        };
        // part 0: only the first MFMA (tile 0, column tile 0, l*h); 1: the rest; 2: all
        auto mfma_block = [&](const Frag &f, int part = 2) {
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const f16x8 ah = as_h(f.a[k][0]), al = as_h(f.a[k][1]);
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const f16x8 bh = as_h(f.b[ct][0]), bl = as_h(f.b[ct][1]);
                    const bool first = k == 0 && ct == 0;
                    f32x4v c = acc[k][ct];
                    if (part == 2 || (part == 0) == first) c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
                    if (part != 0) {
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
                    }
                    acc[k][ct] = c;
                }
            }
        };
        // NBUF 2: B(kk+3) -> registers, B(kk+2) -> LDS buffer kk & 1, barrier every offset.
        // NBUF 4: B(kk+4) -> register set kk & 1, B(kk+3) (loaded one offset earlier) ->
        // buffer (kk+3) & 3, barrier after odd offsets: a buffer written at offset kk is
        // read at kk+2 and last read at kk-2, so a barrier always separates the two
        auto step = [&](int kk, const Frag &cur, Frag &nxt, int set) {
            if constexpr (DMA) {
                // offset kk + LA into buffer (kk + LA) & 7, last read at step kk + LA - 9 (an odd
                // step, so a barrier, lies between for LA <= 7); after odd offsets: everything
                // but the newest LA - 3 DMAs landed (offsets <= kk + 3, read at steps <= kk + 2),
                // the barrier publishes them
#if SNK_H3F_VAR == 0
                // (round 6 measured pinning this order with scheduling barriers, the first MFMA,
                // then the next offset's 12 fragment reads, then the other MFMAs, as the Gram
                // kernel does: 3.4 % slower on the headline than the compiler's own interleave,
                // gpurun_out r06g; not kept)
                dma(kk + H3F_LA);
                frag_read(kk + 1, nxt);
                mfma_block(cur);
                if (kk & 1) {
                    __builtin_amdgcn_s_waitcnt(waitcnt_vm(H3F_LA - 3));
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                    __builtin_amdgcn_s_barrier();
                }
#else   // measurement builds only (wrong results by design): one part of the step left out
                if (SNK_H3F_VAR != 1) dma(kk + H3F_LA);
                if (SNK_H3F_VAR != 4) {
                    frag_read(kk + 1, nxt);
                } else {
#pragma unroll
                    for (int k = 0; k < NT; ++k) asm volatile("" : "+v"(nxt.a[k][0]), "+v"(nxt.a[k][1]));
                    asm volatile("" : "+v"(nxt.b[0][0]), "+v"(nxt.b[0][1]), "+v"(nxt.b[1][0]), "+v"(nxt.b[1][1]));
                }
                if (SNK_H3F_VAR != 3) {
                    mfma_block(cur);
                } else {
#pragma unroll
                    for (int k = 0; k < NT; ++k) asm volatile("" :: "v"(cur.a[k][0]), "v"(cur.a[k][1]));
                    asm volatile("" :: "v"(cur.b[0][0]), "v"(cur.b[0][1]), "v"(cur.b[1][0]), "v"(cur.b[1][1]));
                }
                if (kk & 1) {
                    __builtin_amdgcn_s_waitcnt(waitcnt_vm(H3F_LA - 3));
                    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                    if (SNK_H3F_VAR != 2) __builtin_amdgcn_s_barrier();
                }
#endif
            } else if (NBUF == 2) {
                b_load(kk + 3, set ^ 1);
                frag_read(kk + 1, nxt);
                mfma_block(cur);
                b_store(kk & 1, set);
                __syncthreads();
            } else {
                b_load(kk + 4, set);
                frag_read(kk + 1, nxt);
                mfma_block(cur);
                b_store((kk + 3) & 3, set ^ 1);
                if (kk & 1) __syncthreads();
            }
        };
        Frag f0, f1;
        frag_read(0, f0);
        b_load(2, 0);
        if (NBUF == 4) {
            b_load(3, 1);
            b_store(2, 0);
        }
        __syncthreads();
        H3F_CLK(4);
        static_assert(NKK % 2 == 0, "offsets come in pairs");
        for (int kk = 0; kk < NKK; kk += 2) {
            step(kk, f0, f1, 0);
            step(kk + 1, f1, f0, 1);
        }
        H3F_CLK(5);
        if constexpr (DMA) __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // the tail reloads landed
        prefetch();
        // output through LDS as conv_h3s_kernel (H3F_DIRECT builds: straight from the
        // accumulators, each store 4 positions x 64 contiguous bytes)
        constexpr int CS = 80;
        static_assert(NSG * ho2 * CS * 4 <= h3f_lds_bytes<HIN, NBUF>() - NBUF * NB * 16, "output staging fits");
        [[maybe_unused]] float *Cs = reinterpret_cast<float *>(As);
        float vm[4] = {0.0f, 0.0f, 0.0f, 0.0f};   // this lane's max per sample (post-relu: >= 0)
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            const int p = 4 * (rg + 4 * k) + g;
            if (p >= ho2) continue;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = cg * 32 + ct * 16 + r;
                const float bv = bv2[ct];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const float v = __builtin_ldexpf(acc[k][ct][e], -(ea[e] + ew)) + bv;
                    const float rv = v > 0.0f ? v : 0.0f;
#if H3F_DIRECT
                    if (e < ns) a.out[((int64_t)(s0 + e) * ho2 + p) * CN + col] = rv;
#else
                    Cs[(e * ho2 + p) * CS + col] = rv;
#endif
                    vm[e] = fmaxf(vm[e], rv);
                }
            }
        }
        // per-sample maxima for Dense1's h3 scale: DPP within each 16-lane row (no readlane
        // chain), the 4 row maxima of each wave to LDS (a3red: kernel scope, as waves of
        // different tile counts run different instantiations of this lambda), 32 values per
        // sample after the barrier
        if (a.a3max) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float v = vm[e];
                v = dpp_max<0xB1>(v);
                v = dpp_max<0x4E>(v);
                v = dpp_max<0x141>(v);
                v = dpp_max<0x140>(v);
                if (r == 0) a3red[wave][g][e] = v;
            }
        }
        __syncthreads();
        if (a.a3max && tid < ns) {
            float m = 0.0f;
#pragma unroll
            for (int w = 0; w < 8; ++w)
#pragma unroll
                for (int q = 0; q < 4; ++q) m = fmaxf(m, a3red[w][q][tid]);
            a.a3max[s0 + tid] = m;
        }
#if !H3F_DIRECT
        const int n4o = ns * ho2 * 16;
        f32x4 *o4 = reinterpret_cast<f32x4 *>(a.out + (int64_t)s0 * ho2 * CN);
        const f32x4 *c4 = reinterpret_cast<const f32x4 *>(Cs);
        for (int q = tid; q < n4o; q += 512) o4[q] = c4[(q >> 4) * (CS / 4) + (q & 15)];
#endif
        H3F_CLK(6);
    };
    if (nt == 4) run(std::integral_constant<int, 4>{});
    else if (nt == 3) run(std::integral_constant<int, 3>{});
    else if (nt == 2) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 1>{});
#if H3F_PERSIST
    if (!persist) return;
    __syncthreads();   // the epilogue's reads of the A region are done before the next group stages there
    grp = s_next;
    if (grp >= ngroups) return;
    have_boards = true;
    }
#endif
}

}  // namespace snk

// snk_bwd3.hpp — conv3's backward for the small-batch DQN update (B = 64).
//
// The generic path ran conv3's weight gradient as a split-K GEMM whose lanes
// gathered im2col elements one float at a time (two divisions per element:
// VALU-bound, 19 us) and its data gradient as an implicit GEMM over the
// HOUT^2 = bs^2 input positions, 4/5 of whose 36 kernel offsets fall outside
// the Wo x Wo gradient (1.36 GFLOP of MFMA work for 0.34 useful, plus a
// partial-slab reduce). Both are reorganised around LDS-staged samples, in
// one launch (blocks [0, S * 8) data gradient, the rest weight gradient):
//
//  * dW (grid: Z chunks of 2 samples x C3_DWG = 8 groups, exact-fp32
//    v_mfma_f32_32x32x2_f32):
//    the chunk's a2 [2][bs^2][32] and dz3 [2][Wo^2][64] go to LDS once;
//    the 72 tiles (kk, co half) of 32 (ci) x 32 (co) are 9 per group, two per wave
//    and a third for wave 0 (8 groups, not 9 groups of four offsets: at B = 64 the
//    grid is then 768 = 3 x 256 workgroups, one dispatch round on 256 CUs; with 800
//    the last 32 started when the first finished and ran 3 us past the rest). MFMA k-step
//    t = output position (io, jo), its two k lanes = the two samples:
//    A[ci][s] = a2[s][(io + du, jo + dv)][ci], B[s][co] = dz3[s][(io, jo)][co],
//    lane-consecutive LDS reads at wave-uniform offsets. The chunk's partial
//    goes to slab z (the bias row: column sums of dz3, group 0) and
//    grad_update_kernel sums the Z slabs.
//  * dX (grid: S samples x 32/CG channel groups): T[pout][(kk, ci)] =
//    sum_co dz3[s][pout][co] * W[kk][ci][co] (a dense GEMM, K = 64) into LDS,
//    on the fp16 h3 split (v_mfma_f32_16x16x32_f16, block-local power-of-two
//    scales; see c3_dx_block), then col2im: dz2[s][pin][ci] = sum over the offsets with
//    pout = pin - (du, dv) inside the Wo x Wo grid of T[pout][(kk, ci)],
//    kk ascending, relu-masked by a2. No wasted products, no slab, no reduce.
#pragma once
#include "snk_conv.hpp"
#include "snk_conv_h3.hpp"
#include "snk_qnet.hpp"

namespace snk {

// Profiling builds only (make clocks): per-workgroup phase stamps of conv3_bwd_kernel,
// read back by snk_c3b_debug_clocks (slots: start, operands staged, MFMA done,
// epilogue done, end; slot 6 = 1 + XCC_ID, slot 7 = 1 + the HW_ID word)
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_c3b_clk;
#define C3B_CLK(slot)                                                                                 \
    do {                                                                                              \
        if (threadIdx.x == 0 && g_c3b_clk) g_c3b_clk[(int64_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
__device__ uint64_t *g_c2b_clk;
#define C2B_CLK(slot)                                                                                 \
    do {                                                                                              \
        if (threadIdx.x == 0 && g_c2b_clk) g_c2b_clk[(int64_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define C3B_CLK(slot) do { } while (0)
#define C2B_CLK(slot) do { } while (0)
#endif

struct Conv3BwdArgs {
    const float *a2;    // [S][bs*bs][32]  conv2 output (relu'd)
    const float *dz3;   // [S][wo*wo][64]  gradient at conv3's pre-activation
    const float *w;     // conv3 weights, parameter layout [36 kk][32 ci][64 co]
    float *slab;        // dW partials [Z][1153][64] (row 1152: bias)
    float *dz2;         // [S][bs*bs][32]
    int S, bs, wo, nsc, Z, nW;
};
constexpr int C3_CG = 4;          // dX input channels per workgroup
constexpr int C3_DWG = 8;         // dW workgroups per chunk (72 tiles of 32 ci x 32 co, 9 per workgroup)
constexpr int C3_TLD = 148;       // LDS row stride of T in dX (tools/lds_banks.py: stores 1x, col2im reads 1.3x)

__host__ __device__ inline int c3_dw_lds_floats(int bs, int wo, int nsc) {   // the chunk's a2 (dz3 in registers)
    (void)wo;
    return nsc * bs * bs * 32;
}
__host__ __device__ inline int c3_dx_lds_floats(int wo) {   // T (+ a zero row) overlays the h / l planes
    const int op = 36 * C3_CG * 64 + wo * wo * 64, t = (wo * wo + 1) * C3_TLD;
    return op > t ? op : t;
}

// global -> LDS copies with U loads in flight per thread (a plain strided loop
// waits for each load before the next: ~20 serialised round trips per block)
template <int U>
__device__ __forceinline__ void c3_copy(f32x4 *__restrict__ dst, const f32x4 *__restrict__ src, int n) {
    for (int b = 0; b < n; b += U * 256) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * 256 + (int)threadIdx.x;
            v[u] = src[e < n ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * 256 + (int)threadIdx.x;
            if (e < n) dst[e] = v[u];
        }
    }
}
template <int WO>
__device__ __forceinline__ void c3_dw_block(const Conv3BwdArgs &a, int z, int grp, float *sm) {
    // lane half h takes sample s0 + h of the chunk (NSC = 2), the k-step t its position t:
    // every lane's im2col address follows from the wave-uniform (io, jo) of t
    constexpr int BS = WO + 5, BS2 = BS * BS, WO2 = WO * WO;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s0 = z * 2, ns = min(2, a.S - s0);
    const int r = lane & 31, h = lane >> 5;
    const bool hv = h < ns;
    // the lane's B operands, dz3[s0 + h][t][r] and [r + 32] for every position t, straight
    // into registers (issued first, consumed in order by the MFMA chain; every wave of the
    // block reads the same rows, from L2): only a2 goes through LDS
    const float *gd = a.dz3 + (int64_t)(s0 + (hv ? h : 0)) * WO2 * 64 + r;
    float y0[WO2], y1[WO2];
#pragma unroll
    for (int t = 0; t < WO2; ++t) {
        y0[t] = gd[t * 64];
        y1[t] = gd[t * 64 + 32];
    }
    float *A = sm;
    c3_copy<12>(reinterpret_cast<f32x4 *>(A), reinterpret_cast<const f32x4 *>(a.a2 + (int64_t)s0 * BS2 * 32),
                ns * BS2 * 8);
    __syncthreads();
    C3B_CLK(1);
    // tiles ht = 9 grp + wave + 4 c: offset kk = ht >> 1, output columns [32 (ht & 1), +32);
    // wave 0 also takes 9 grp + 8. A wave's tiles share one column half (ht, ht + 4, ht + 8
    // have one parity), so each k-step selects one dz3 column and feeds every chain
    const int ht0 = 9 * grp + wave;
    const bool odd = ht0 & 1;
    float *out = a.slab + (int64_t)z * 1153 * 64;
    auto chains = [&](auto nch) {
        constexpr int NCH = decltype(nch)::value;
        const float *pa[NCH];
        f32x16 acc[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int kk = (ht0 + 4 * c) >> 1, dv = kk / 6, du = kk - dv * 6;
            pa[c] = A + ((hv ? h : 0) * BS2 + du + dv * BS) * 32 + r;
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[c][g] = 0.0f;
        }
#pragma unroll
        for (int jo = 0; jo < WO; ++jo)
#pragma unroll
            for (int io = 0; io < WO; ++io) {
                const float y = odd ? y1[jo * WO + io] : y0[jo * WO + io];
#pragma unroll
                for (int c = 0; c < NCH; ++c) {
                    const float x = pa[c][(io + jo * BS) * 32];
                    acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv ? x : 0.0f, y, acc[c], 0, 0, 0);
                }
            }
        C3B_CLK(2);
#pragma unroll
        for (int c = 0; c < NCH; ++c) {
            const int kk = (ht0 + 4 * c) >> 1;
#pragma unroll
            for (int g = 0; g < 16; ++g) out[(kk * 32 + acc_row(g, lane)) * 64 + (odd ? 32 : 0) + r] = acc[c][g];
        }
    };
    if (wave == 0)
        chains(std::integral_constant<int, 3>{});
    else
        chains(std::integral_constant<int, 2>{});
    if (grp == 0 && wave == 3) {   // bias row: column sums of the chunk's dz3, positions ascending per sample
        float b0 = 0.0f, b1 = 0.0f;
#pragma unroll
        for (int t = 0; t < WO2; ++t) {
            b0 += y0[t];
            b1 += y1[t];
        }
        b0 = hv ? b0 : 0.0f;
        b1 = hv ? b1 : 0.0f;
        const float o0 = __shfl_xor(b0, 32), o1 = __shfl_xor(b1, 32);
        if (h == 0) {
            out[1152 * 64 + r] = b0 + o0;
            out[1152 * 64 + 32 + r] = b1 + o1;
        }
    }
}

typedef float f32x4m __attribute__((ext_vector_type(4)));

// dX block (sample s, input channels [4 cg, 4 cg + 4)) on the fp16 h3 split
// (snk_conv_h3.hpp): the block's 144 weight rows W[kk][ci][.] and dz3[s] are
// scaled by one power of two each (the block's own max |w|, the sample's max
// |dz3|: both factor out of T and come back by one ldexp), split into fp16
// h / l planes in LDS ([row][64 co] halves, 16-byte chunk c of row n at c ^ (n & 7):
// conflict-free b128 fragment reads and b64 stores), then
// T = Dz3 x W' as v_mfma_f32_16x16x32_f16 tiles, hl + lh + hh per 32-wide co step
// (3 x 2 = 6 MFMAs per 16 x 16 tile against 16 v_mfma_f32_16x16x4_f32 before).
template <int WO>
__device__ __forceinline__ void c3_dx_block(const Conv3BwdArgs &a, int s, int cg, float *sm) {
    constexpr int BS = WO + 5, BS2 = BS * BS, WO2 = WO * WO;
    constexpr int NN = 36 * C3_CG;                 // T columns / weight rows (kk, ci)
    constexpr int NW4 = NN * 16 / 256;             // float4 of W per thread (9)
    constexpr int ND4 = (WO2 * 16 + 255) / 256;    // float4 of dz3 per thread
    constexpr int NMK = (BS2 * C3_CG + 255) / 256; // (pin, ci) outputs per thread
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint16_t *Wh = reinterpret_cast<uint16_t *>(sm), *Wl = Wh + NN * 64;
    uint16_t *Dh = Wl + NN * 64, *Dl = Dh + WO2 * 64;
    float *Tl = sm;
    __shared__ float red[4][2];   // lds: one per kernel (conv3_bwd / conv2_bwd call this block helper once)
    // relu-mask values of this block's outputs, loaded now (used by the col2im)
    float mk[NMK];
#pragma unroll
    for (int u = 0; u < NMK; ++u) {
        const int e = u * 256 + tid, ee = e < BS2 * C3_CG ? e : 0;
        mk[u] = a.a2[((int64_t)s * BS2 + (ee >> 2)) * 32 + cg * C3_CG + (ee & 3)];
    }
    // W rows n = kk*4 + ci <- parameter row kk*32 + 4 cg + ci; dz3[s] rows = positions
    f32x4 wv[NW4], dv[ND4];
    float mw = 0.0f, md = 0.0f;
#pragma unroll
    for (int u = 0; u < NW4; ++u) {
        const int e = u * 256 + tid, n = e >> 4;
        wv[u] = *reinterpret_cast<const f32x4 *>(a.w + ((n >> 2) * 32 + cg * C3_CG + (n & 3)) * 64 + (e & 15) * 4);
    }
#pragma unroll
    for (int u = 0; u < ND4; ++u) {
        const int e = u * 256 + tid;
        dv[u] = e < WO2 * 16 ? *reinterpret_cast<const f32x4 *>(a.dz3 + (int64_t)s * WO2 * 64 + e * 4)
                             : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < NW4; ++u)
        mw = fmaxf(mw, fmaxf(fmaxf(fabsf(wv[u][0]), fabsf(wv[u][1])), fmaxf(fabsf(wv[u][2]), fabsf(wv[u][3]))));
#pragma unroll
    for (int u = 0; u < ND4; ++u)
        md = fmaxf(md, fmaxf(fmaxf(fabsf(dv[u][0]), fabsf(dv[u][1])), fmaxf(fabsf(dv[u][2]), fabsf(dv[u][3]))));
    mw = wave_max(mw);
    md = wave_max(md);
    if (lane == 0) {
        red[wave][0] = mw;
        red[wave][1] = md;
    }
    __syncthreads();
    const int ew = h3_exp(fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0])));
    const int ed = h3_exp(fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1])));
#pragma unroll
    for (int u = 0; u < NW4; ++u) {
        const int e = u * 256 + tid, n = e >> 4, q = e & 15;
        const int o = n * 64 + (((q >> 1) ^ (n & 7)) << 3) + ((q & 1) << 2);
        u32x2 h, l;
        h3_split4(wv[u], ew, h, l);
        *reinterpret_cast<u32x2 *>(Wh + o) = h;
        *reinterpret_cast<u32x2 *>(Wl + o) = l;
    }
#pragma unroll
    for (int u = 0; u < ND4; ++u) {
        const int e = u * 256 + tid, n = e >> 4, q = e & 15;
        if (e < WO2 * 16) {
            const int o = n * 64 + (((q >> 1) ^ (n & 7)) << 3) + ((q & 1) << 2);
            u32x2 h, l;
            h3_split4(dv[u], ed, h, l);
            *reinterpret_cast<u32x2 *>(Dh + o) = h;
            *reinterpret_cast<u32x2 *>(Dl + o) = l;
        }
    }
    __syncthreads();
    C3B_CLK(1);
    // T in 16x16 tiles round robin over the waves (C rows 4*(l>>4) + e, column l&15),
    // all kept in registers, then written over the operands after a barrier
    const int r = lane & 15, g = lane >> 4;
    constexpr int RT = (WO2 + 15) / 16, CT = NN / 16, NT = RT * CT, MT = (NT + 3) / 4;
    f32x4m acc[MT];
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int t = wave + 4 * u;
        acc[u] = f32x4m{0.0f, 0.0f, 0.0f, 0.0f};
        if (t < NT) {
            const int tr = t / CT, tc = t - tr * CT;
            const int ar = min(tr * 16 + r, WO2 - 1), br = tc * 16 + r;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int c = ks * 4 + g;
                const int ao = ar * 64 + ((c ^ (ar & 7)) << 3), bo = br * 64 + ((c ^ (br & 7)) << 3);
                const f16x8 ah = as_h(*reinterpret_cast<const u32x4 *>(Dh + ao));
                const f16x8 al = as_h(*reinterpret_cast<const u32x4 *>(Dl + ao));
                const f16x8 bh = as_h(*reinterpret_cast<const u32x4 *>(Wh + bo));
                const f16x8 bl = as_h(*reinterpret_cast<const u32x4 *>(Wl + bo));
                acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc[u], 0, 0, 0);
                acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc[u], 0, 0, 0);
                acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc[u], 0, 0, 0);
            }
        }
    }
    __syncthreads();
    C3B_CLK(2);
    const int esc = -(ew + ed);
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int t = wave + 4 * u;
        if (t < NT) {
            const int tr = t / CT, tc = t - tr * CT;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int rr = tr * 16 + 4 * g + e;
                if (rr < WO2) Tl[rr * C3_TLD + tc * 16 + r] = __builtin_ldexpf(acc[u][e], esc);
            }
        }
    }
    if (tid < NN) Tl[WO2 * C3_TLD + tid] = 0.0f;   // the zero row out-of-grid terms read
    __syncthreads();
    C3B_CLK(3);
    // col2im + relu mask, (pin, ci) per thread: dz2[pin][ci] = sum over kk ascending of
    // T[pin - (du, dv)][(kk, ci)] inside the Wo x Wo grid (the zero row outside)
#pragma unroll
    for (int u = 0; u < NMK; ++u) {
        const int e = u * 256 + tid;
        if (e >= BS2 * C3_CG) break;
        const int pin = e >> 2, ci = e & 3;
        const int j = pin / BS, i = pin - j * BS;
        const float *tb = Tl + ci;
        float t[36];
#pragma unroll
        for (int kk = 0; kk < 36; ++kk) {
            const int dv = kk / 6, du = kk - dv * 6;
            const bool v = (unsigned)(i - du) < (unsigned)WO && (unsigned)(j - dv) < (unsigned)WO;
            t[kk] = tb[(v ? (i - du) + (j - dv) * WO : WO2) * C3_TLD + kk * C3_CG];
        }
        float v = 0.0f;
#pragma unroll
        for (int kk = 0; kk < 36; ++kk) v += t[kk];
        const int64_t o = ((int64_t)s * BS2 + pin) * 32 + cg * C3_CG + ci;
        a.dz2[o] = mk[u] > 0.0f ? v : 0.0f;
    }
}

// one instantiation per Wo: the register footprint (dz3 columns of the weight-gradient
// blocks) and with it the occupancy are the board's own; three workgroups per CU
// (LDS: 49.4 KB each at Wo = 7) need <= 168 VGPRs (Wo = 8 keeps two: its 64 dz3 column
// pairs would spill)
template <int WO>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WO >= 8 ? 2 : 3))) void conv3_bwd_kernel(
    Conv3BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float c3sm[];
    const int b = blockIdx.x;
    C3B_CLK(0);
#ifdef SNK_ENV_CLOCKS
    if (threadIdx.x == 0 && g_c3b_clk) {
        g_c3b_clk[(int64_t)b * 8 + 7] = 1 + (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_c3b_clk[(int64_t)b * 8 + 6] = 1 + (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    }
#endif
    const int nX = a.S * (32 / C3_CG);   // data-gradient blocks first: they wait on more staging
    if (b < nX)
        c3_dx_block<WO>(a, b / (32 / C3_CG), b % (32 / C3_CG), c3sm);
    else
        c3_dw_block<WO>(a, (b - nX) / C3_DWG, (b - nX) % C3_DWG, c3sm);
    C3B_CLK(4);
}

// ---------------------------------------------------------------- conv2 (3x3, pad 1, 16 -> 32)
// One launch: blocks [0, S) the weight gradient of sample b, then C2_NXB
// data-gradient blocks per sample, on v_mfma_f32_16x16x4_f32 from LDS.
//  * dW block: a1[s] inside a zero border ([(bs+2)^2][16]) and dz2[s]
//    ([bs^2][48-float rows]); wave w takes a quarter of the output positions
//    (4 per MFMA step) for all nine 16 (ci) x 32 (co) offset tiles:
//    A[ci][t] = a1b[(io + du, jo + dv)][ci], B[t][co] = dz2[t][co]; the four
//    partials are summed in LDS. Slab z = s (grad_update_kernel sums them);
//    wave 3 also writes the bias row.
//  * dX block: dz2[s] inside a zero border and the weights [kk][ci][co], both as
//    fp16 h / l planes of power-of-two-scaled values (the sample's max |dz2|, the
//    block's max |w|: snk_conv_h3.hpp's h3 split, the scales factored out and
//    returned by one multiply); 4x4-position tiles round robin over the waves,
//    K = 9 offsets x 32 channels on v_mfma_f32_16x16x32_f16 (hl + lh + hh):
//    dzc1[pin][ci] = sum dz2b[pin + (1,1) - (du,dv)][co] * W[kk][ci][co],
//    relu-masked by a1.
struct Conv2BwdArgs {
    const float *a1;    // [S][bs*bs][16]
    const float *dz2;   // [S][bs*bs][32]
    const float *w;     // conv2 weights [9 kk][16 ci][32 co]
    float *slab;        // dW partials [S][145][32] (row 144: bias)
    float *dzc1;        // [S][bs*bs][16]
    int S, bs;
    // conv1's weight gradient, fused into the data-gradient blocks (c1slab != nullptr):
    // block (s, xb) writes the partial over its position tiles to c1slab[s*C2_NXB + xb][9C+1][16]
    BoardSrc x;         // conv1's input planes (the forward's float copy or the replay frames)
    float *c1slab;
    int C;
};
// dX image of dz2 as fp16 h / l planes: position (pi, pj) of the zero-bordered grid at
// (pi + pj * C2X_PJ) * C2X_PS halves (32 co + 16 pad), no swizzle: every b128 fragment read
// of a 4x4 position tile at every kernel offset on 16 distinct bank quads (tools/lds_banks.py
// model; the epilogue-side writes are 2-way and few)
constexpr int C2X_PJ = 20, C2X_PS = 48;
constexpr int C2_DS = 48;   // LDS row stride of dz2 in the weight gradient (floats), conflict-free reads

__host__ __device__ inline int c2_bwd_lds_floats(int bs) {
    const int bp2 = (bs + 2) * (bs + 2);
    // dX: the h / l planes of the bordered dz2 image (halves) and of W2, + conv1's planes (C <= 2)
    int dw = bp2 * 16 + bs * bs * C2_DS, dx = (bs + 2) * C2X_PJ * C2X_PS + 144 * 32 + 2 * bp2;
    if (dw < 4 * 4608) dw = 4 * 4608;   // the weight-gradient block's cross-wave sum
    return dw > dx ? dw : dx;
}

__device__ __forceinline__ void c2_dw_block(const Conv2BwdArgs &a, int s, float *sm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs = a.bs, bp = bs + 2, bs2 = bs * bs, bp2 = bp * bp;
    float *A1 = sm, *D2 = sm + bp2 * 16;
    // a1[s] (4 float4 per position) and dz2[s] (8 per position) into registers first (boards up
    // to 13 x 13; larger ones load the rest after), then the zero border ring of A1 and the
    // scatter: border and interior are disjoint, so one barrier orders everything
    constexpr int NA = 3, ND = 6;
    const f32x4 *src = reinterpret_cast<const f32x4 *>(a.a1 + (int64_t)s * bs2 * 16);
    const f32x4 *srd = reinterpret_cast<const f32x4 *>(a.dz2 + (int64_t)s * bs2 * 32);
    f32x4 av[NA], dv[ND];
#pragma unroll
    for (int u = 0; u < NA; ++u) {
        const int e = u * 256 + tid;
        av[u] = src[e < bs2 * 4 ? e : 0];
    }
#pragma unroll
    for (int u = 0; u < ND; ++u) {
        const int e = u * 256 + tid;
        dv[u] = srd[e < bs2 * 8 ? e : 0];
    }
    for (int e = tid; e < 4 * (bs + 1) * 4; e += 256) {
        const int c = e & 3, q = e >> 2, side = q / (bs + 1), k = q - side * (bs + 1);
        const int pi = side == 0 ? k : side == 1 ? bs + 1 : side == 2 ? k + 1 : 0;
        const int pj = side == 0 ? 0 : side == 1 ? k : side == 2 ? bs + 1 : k + 1;
        reinterpret_cast<f32x4 *>(A1 + (pi + pj * bp) * 16)[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto put_a = [&](int e, const f32x4 &v) {
        const int p = e >> 2, j = p / bs, i = p - j * bs;
        reinterpret_cast<f32x4 *>(A1 + ((i + 1) + (j + 1) * bp) * 16)[e & 3] = v;
    };
#pragma unroll
    for (int u = 0; u < NA; ++u) {
        const int e = u * 256 + tid;
        if (e < bs2 * 4) put_a(e, av[u]);
    }
    for (int e = NA * 256 + tid; e < bs2 * 4; e += 256) put_a(e, src[e]);
#pragma unroll
    for (int u = 0; u < ND; ++u) {
        const int e = u * 256 + tid;
        if (e < bs2 * 8) reinterpret_cast<f32x4 *>(D2 + (e >> 3) * C2_DS)[e & 7] = dv[u];
    }
    for (int e = ND * 256 + tid; e < bs2 * 8; e += 256) reinterpret_cast<f32x4 *>(D2 + (e >> 3) * C2_DS)[e & 7] = srd[e];
    __syncthreads();
    C2B_CLK(1);
    // wave w: output positions [w*q, w*q + q) (q = bs^2/4 rounded up to 4) for all
    // nine offsets (18 independent accumulator chains), then a fixed-order LDS sum
    const int r = lane & 15, g = lane >> 4;
    const int q = ((bs2 + 15) / 16) * 4, t0 = wave * q, t1 = min(bs2, t0 + q);
    f32x4m acc[9][2];
#pragma unroll
    for (int kk = 0; kk < 9; ++kk) acc[kk][0] = acc[kk][1] = f32x4m{0.f, 0.f, 0.f, 0.f};
    for (int tb = t0; tb < t1; tb += 4) {
        const int t = tb + g;
        const bool v = t < t1;
        const int tt = v ? t : t0;
        const int jo = tt / bs, io = tt - jo * bs;
        const float *pa = A1 + (io + jo * bp) * 16 + r;
        const float y0 = D2[tt * C2_DS + r], y1 = D2[tt * C2_DS + 16 + r];
        const float b0 = v ? y0 : 0.0f, b1 = v ? y1 : 0.0f;
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const float x = pa[((kk % 3) + (kk / 3) * bp) * 16];
            acc[kk][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, b0, acc[kk][0], 0, 0, 0);
            acc[kk][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(x, b1, acc[kk][1], 0, 0, 0);
        }
    }
    float bsum = 0.0f;
    if (wave == 3 && lane < 32) {   // bias row: dz2 column sums, position order
        int t = 0;
        for (; t + 8 <= bs2; t += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = D2[(t + u) * C2_DS + lane];
#pragma unroll
            for (int u = 0; u < 8; ++u) bsum += v[u];
        }
        for (; t < bs2; ++t) bsum += D2[t * C2_DS + lane];
    }
    float *out = a.slab + (int64_t)s * 145 * 32;
    C2B_CLK(2);
    __syncthreads();   // staging buffers are free: partial tiles [wave][kk][ct][e][lane]
    float *red = sm;
#pragma unroll
    for (int kk = 0; kk < 9; ++kk)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int e = 0; e < 4; ++e) red[(((wave * 9 + kk) * 2 + ct) * 4 + e) * 64 + lane] = acc[kk][ct][e];
    __syncthreads();
    for (int x = tid; x < 9 * 2 * 4 * 64; x += 256) {
        const float v = ((red[x] + red[4608 + x]) + red[2 * 4608 + x]) + red[3 * 4608 + x];
        const int ln = x & 63, e = (x >> 6) & 3, ct = (x >> 8) & 1, kk = x >> 9;
        out[(kk * 16 + 4 * (ln >> 4) + e) * 32 + ct * 16 + (ln & 15)] = v;
    }
    if (wave == 3 && lane < 32) out[144 * 32 + lane] = bsum;
}

constexpr int C2_NXB = 2;   // data-gradient blocks per sample (interleaved 4x4 position tiles)

__device__ __forceinline__ void c2_dx_block(const Conv2BwdArgs &a, int s, int xb, float *sm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs = a.bs, bp = bs + 2, bs2 = bs * bs, bp2 = bp * bp;
    const int npos = bp * C2X_PJ;
    uint16_t *Dh = reinterpret_cast<uint16_t *>(sm), *Dl = Dh + npos * C2X_PS;
    uint16_t *Wh = Dl + npos * C2X_PS, *Wl = Wh + 144 * 32;
    float *Xb = reinterpret_cast<float *>(Wl + 144 * 32);
    __shared__ float red[4][2];   // lds: one per kernel (conv3_bwd / conv2_bwd call this block helper once)
    // dz2[s] (bs^2 x 32) and W2 [kk][ci][co] (144 x 32) into registers: 8 float4 per position,
    // 8 per weight row (boards up to 13 x 13 fit NU; larger ones read the rest twice from L2)
    constexpr int NU = 6;   // 169 * 8 = 1352 <= 6 * 256
    f32x4 dv[NU], wv[5];
    float md = 0.0f, mw = 0.0f;
    const f32x4 *srd = reinterpret_cast<const f32x4 *>(a.dz2 + (int64_t)s * bs2 * 32);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = u * 256 + tid;
        dv[u] = e < bs2 * 8 ? srd[e] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    const f32x4 *sw = reinterpret_cast<const f32x4 *>(a.w);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
        const int e = u * 256 + tid;
        wv[u] = e < 1152 ? sw[e] : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // zero border of both planes (positions with pi or pj in {0, bs + 1}); the interior is
    // written below
    for (int e = tid; e < 4 * (bs + 1) * 6 * 2; e += 256) {
        const int c = e % 6, q = (e / 6) % (4 * (bs + 1)), pl = e / (6 * 4 * (bs + 1));
        const int side = q / (bs + 1), k = q - side * (bs + 1);
        const int pi = side == 0 ? k : side == 1 ? bs + 1 : side == 2 ? k + 1 : 0;
        const int pj = side == 0 ? 0 : side == 1 ? k : side == 2 ? bs + 1 : k + 1;
        *reinterpret_cast<u32x4 *>((pl ? Dl : Dh) + (pi + pj * C2X_PJ) * C2X_PS + c * 8) = u32x4{0u, 0u, 0u, 0u};
    }
    // conv1's input planes inside a zero border (the fused conv1 weight gradient reads them
    // from LDS: a global load per MFMA operand left the MFMA chain waiting on each)
    if (a.c1slab) {
        for (int e = tid; e < a.C * bp2; e += 256) {
            const int c = e / bp2, pb = e - c * bp2, jj = pb / bp - 1, ii = pb - (jj + 1) * bp - 1;
            Xb[e] = (ii >= 0 && ii < bs && jj >= 0 && jj < bs) ? a.x.load(s, c, ii + jj * bs) : 0.0f;
        }
    }
#pragma unroll
    for (int u = 0; u < NU; ++u)
        md = fmaxf(md, fmaxf(fmaxf(fabsf(dv[u][0]), fabsf(dv[u][1])), fmaxf(fabsf(dv[u][2]), fabsf(dv[u][3]))));
    for (int e = NU * 256 + tid; e < bs2 * 8; e += 256) {   // boards over 13 x 13: the rest from L2
        const f32x4 x = srd[e];
        md = fmaxf(md, fmaxf(fmaxf(fabsf(x[0]), fabsf(x[1])), fmaxf(fabsf(x[2]), fabsf(x[3]))));
    }
#pragma unroll
    for (int u = 0; u < 5; ++u)
        mw = fmaxf(mw, fmaxf(fmaxf(fabsf(wv[u][0]), fabsf(wv[u][1])), fmaxf(fabsf(wv[u][2]), fabsf(wv[u][3]))));
    // the relu mask a1 of this wave's first two tiles' outputs (tile t = xb + C2_NXB*wave + 8u:
    // position (4 bi + e, 4 bj + g), channel r), loaded before the barriers
    float mk1[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int nbm = (bs + 3) >> 2, t = xb + C2_NXB * wave + 4 * C2_NXB * u;
        const int bi = t % nbm, bj = t / nbm, oj = min(4 * bj + (lane >> 4), bs - 1);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int oi = min(4 * bi + e, bs - 1);
            mk1[u][e] = t < nbm * nbm ? a.a1[((int64_t)s * bs2 + oi + oj * bs) * 16 + (lane & 15)] : 0.0f;
        }
    }
    md = wave_max(md);
    mw = wave_max(mw);
    if (lane == 0) {
        red[wave][0] = md;
        red[wave][1] = mw;
    }
    __syncthreads();
    const int ed = h3_exp(fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0])));
    const int ew = h3_exp(fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1])));
#pragma unroll
    for (int u = 0; u < NU; ++u) {
        const int e = u * 256 + tid;
        if (e < bs2 * 8) {
            const int p = e >> 3, q = e & 7, j = p / bs, i = p - j * bs;
            const int o = ((i + 1) + (j + 1) * C2X_PJ) * C2X_PS + q * 4;
            u32x2 h, l;
            h3_split4(dv[u], ed, h, l);
            *reinterpret_cast<u32x2 *>(Dh + o) = h;
            *reinterpret_cast<u32x2 *>(Dl + o) = l;
        }
    }
    for (int e = NU * 256 + tid; e < bs2 * 8; e += 256) {
        const int p = e >> 3, q = e & 7, j = p / bs, i = p - j * bs;
        const int o = ((i + 1) + (j + 1) * C2X_PJ) * C2X_PS + q * 4;
        u32x2 h, l;
        h3_split4(srd[e], ed, h, l);
        *reinterpret_cast<u32x2 *>(Dh + o) = h;
        *reinterpret_cast<u32x2 *>(Dl + o) = l;
    }
#pragma unroll
    for (int u = 0; u < 5; ++u) {   // weight row n = kk*16 + ci (64-byte rows), 16-byte piece g at g ^ ((n >> 1) & 3)
        const int e = u * 256 + tid;
        if (e < 1152) {
            const int n = e >> 3, q = e & 7;
            const int o = n * 32 + (((q >> 1) ^ ((n >> 1) & 3)) << 3) + ((q & 1) << 2);
            u32x2 h, l;
            h3_split4(wv[u], ew, h, l);
            *reinterpret_cast<u32x2 *>(Wh + o) = h;
            *reinterpret_cast<u32x2 *>(Wl + o) = l;
        }
    }
    __syncthreads();
    C2B_CLK(1);
    const int r = lane & 15, g = lane >> 4;
    const int nb = (bs + 3) >> 2, nt = nb * nb;
    const float sc = __builtin_ldexpf(1.0f, -(ed + ew));
    // conv1 weight gradient over this wave's tiles: C1[(kk, c) | bias][co] = sum over the
    // tile's positions p of x[p + (du-1, dv-1)][c] * dzc1[p][co], as v_mfma_f32_16x16x4_f32
    // with k = position: step m takes tile row m (positions (4 bi + m, 4 bj + g)), whose dzc1
    // this lane already holds in acc[m] (column co = r); rows 0..15 and 16..31 of (kk, c)
    // (9C of them, then the bias row of ones, then zeros)
    f32x4m c1acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int nrow = 9 * a.C;
    for (int t = xb + C2_NXB * wave, u = 0; t < nt; t += 4 * C2_NXB, ++u) {
        // tile t = 4x4 positions (i, j) = (4 bi + (r & 3), 4 bj + (r >> 2)); A rows = positions
        const int bi = t % nb, bj = t / nb;
        const int i = min(4 * bi + (r & 3), bs - 1), j = min(4 * bj + (r >> 2), bs - 1);
        f32x4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int dv = kk / 3, du = kk - dv * 3;
            // dz2 at (i + 1 - du, j + 1 - dv) in the input grid = bordered (i + 2 - du, j + 2 - dv)
            const uint16_t *pa = Dh + ((i + 2 - du) + (j + 2 - dv) * C2X_PJ) * C2X_PS + g * 8;
            const int n = kk * 16 + r;
            const uint16_t *pb = Wh + n * 32 + ((g ^ ((n >> 1) & 3)) << 3);
            const f16x8 ah = as_h(*reinterpret_cast<const u32x4 *>(pa));
            const f16x8 al = as_h(*reinterpret_cast<const u32x4 *>(pa + npos * C2X_PS));
            const f16x8 bh = as_h(*reinterpret_cast<const u32x4 *>(pb));
            const f16x8 bl = as_h(*reinterpret_cast<const u32x4 *>(pb + 144 * 32));
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, acc, 0, 0, 0);
        }
        // C row 4g + e = position (4 bi + e, 4 bj + g), column ci = r
        f32x4m dzm;
        const int oj = 4 * bj + g;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int oi = 4 * bi + e;
            dzm[e] = 0.0f;
            if (oi < bs && oj < bs) {
                const int64_t o = ((int64_t)s * bs2 + oi + oj * bs) * 16 + r;
                const float m1 = u == 0 ? mk1[0][e] : u == 1 ? mk1[1][e] : a.a1[o];
                dzm[e] = m1 > 0.0f ? acc[e] * sc : 0.0f;
                a.dzc1[o] = dzm[e];
            }
        }
        if (!a.c1slab) continue;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int pi = 4 * bi + m, pj = 4 * bj + g;   // k = g of this step
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int k1 = rt * 16 + r;           // row (kk, c) of this lane's A element
                float xv = 0.0f;
                if (pi < bs && pj < bs) {
                    if (k1 < nrow) {
                        const int kk = k1 / a.C, c = k1 - kk * a.C;
                        // bordered (pi + kk % 3, pj + kk / 3) = input (pi + kk % 3 - 1, pj + kk / 3 - 1)
                        xv = Xb[c * bp2 + (pi + kk % 3) + (pj + kk / 3) * bp];
                    } else if (k1 == nrow) {
                        xv = 1.0f;
                    }
                }
                c1acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, dzm[m], c1acc[rt], 0, 0, 0);
            }
        }
    }
    C2B_CLK(2);
    if (!a.c1slab) return;
    // the block's four wave partials, summed in wave order through LDS (the staging is free)
    __syncthreads();
    float *red4 = sm;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int e = 0; e < 4; ++e) red4[((wave * 2 + rt) * 4 + e) * 64 + lane] = c1acc[rt][e];
    __syncthreads();
    float *out = a.c1slab + ((int64_t)s * C2_NXB + xb) * (nrow + 1) * 16;
    for (int q = tid; q < 2 * 4 * 64; q += 256) {
        const float v = ((red4[q] + red4[512 + q]) + red4[1024 + q]) + red4[1536 + q];
        const int ln = q & 63, e = (q >> 6) & 3, rt = q >> 8;
        const int row = rt * 16 + 4 * (ln >> 4) + e;   // C[row][col = ln & 15]
        if (row <= nrow) out[row * 16 + (ln & 15)] = v;
    }
}

__global__ __launch_bounds__(256) void conv2_bwd_kernel(Conv2BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float c2sm[];
    const int b = blockIdx.x;
    C2B_CLK(0);
    if (b < a.S)
        c2_dw_block(a, b, c2sm);
    else
        c2_dx_block(a, (b - a.S) / C2_NXB, (b - a.S) % C2_NXB, c2sm);
    C2B_CLK(4);
}

}  // namespace snk

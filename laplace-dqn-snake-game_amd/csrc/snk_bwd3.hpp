// snk_bwd3.hpp — conv3's backward for the small-batch DQN update (B = 64).
//
// The generic path ran conv3's weight gradient as a split-K GEMM whose lanes
// gathered im2col elements one float at a time (two divisions per element:
// VALU-bound, 19 us) and its data gradient as an implicit GEMM over the
// HOUT^2 = bs^2 input positions, 4/5 of whose 36 kernel offsets fall outside
// the Wo x Wo gradient (1.36 GFLOP of MFMA work for 0.34 useful, plus a
// partial-slab reduce). Both are reorganised around LDS-staged samples, in
// one launch (blocks [0, nW) weight gradient, the rest data gradient), on the
// exact-fp32 v_mfma_f32_32x32x2_f32:
//
//  * dW (grid: Z chunks of 2 samples x 9 groups of four kernel offsets):
//    the chunk's a2 [2][bs^2][32] and dz3 [2][Wo^2][64] go to LDS once;
//    wave w owns offset kk = 4*group + w, a 32 (ci) x 64 (co) tile. MFMA k-step
//    t = output position (io, jo), its two k lanes = the two samples:
//    A[ci][s] = a2[s][(io + du, jo + dv)][ci], B[s][co] = dz3[s][(io, jo)][co],
//    lane-consecutive LDS reads at wave-uniform offsets. The chunk's partial
//    goes to slab z (the bias row: column sums of dz3, group 0) and
//    grad_update_kernel sums the Z slabs.
//  * dX (grid: S samples x 32/CG channel groups): T[pout][(kk, ci)] =
//    sum_co dz3[s][pout][co] * W[kk][ci][co] (a dense GEMM, K = 64) into LDS,
//    (v_mfma_f32_16x16x4_f32 tiles), then col2im: dz2[s][pin][ci] = sum over the offsets with
//    pout = pin - (du, dv) inside the Wo x Wo grid of T[pout][(kk, ci)],
//    kk ascending, relu-masked by a2. No wasted products, no slab, no reduce.
#pragma once
#include "snk_conv.hpp"
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
#else
#define C3B_CLK(slot) do { } while (0)
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
constexpr int C3_DLD = 68;        // LDS row stride of dz3 / weights in dX (16x16x4 reads conflict-free)
constexpr int C3_TLD = 36 * C3_CG + 1;

__host__ __device__ inline int c3_dw_lds_floats(int bs, int wo, int nsc) {
    return nsc * bs * bs * 32 + nsc * wo * wo * 64;
}
__host__ __device__ inline int c3_dx_lds_floats(int wo) {   // T overlays the staged operands
    const int op = wo * wo * C3_DLD + 36 * C3_CG * C3_DLD, t = wo * wo * C3_TLD;
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
// rows of 64 floats -> LDS rows of C3_DLD floats; row e>>4 of the source at src + srow(e>>4)*64
template <int U, class F>
__device__ __forceinline__ void c3_copy_rows(float *__restrict__ dst, const float *__restrict__ src, int rows, F srow) {
    const int n = rows * 16;
    for (int b = 0; b < n; b += U * 256) {
        f32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * 256 + (int)threadIdx.x;
            const int ee = e < n ? e : 0;
            v[u] = *reinterpret_cast<const f32x4 *>(src + (int64_t)srow(ee >> 4) * 64 + (ee & 15) * 4);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = b + u * 256 + (int)threadIdx.x;
            if (e < n) *reinterpret_cast<f32x4 *>(dst + (e >> 4) * C3_DLD + (e & 15) * 4) = v[u];
        }
    }
}

template <int WO>
__device__ __forceinline__ void c3_dw_block(const Conv3BwdArgs &a, int z, int grp, float *sm) {
    // lane half h takes sample s0 + h of the chunk (NSC = 2), the k-step t its position t:
    // every lane's im2col address follows from the wave-uniform (io, jo) of t
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs2 = a.bs * a.bs, wo2 = WO * WO;
    const int s0 = z * 2, ns = min(2, a.S - s0);
    float *A = sm, *D = sm + 2 * bs2 * 32;
    c3_copy<12>(reinterpret_cast<f32x4 *>(A), reinterpret_cast<const f32x4 *>(a.a2 + (int64_t)s0 * bs2 * 32),
                ns * bs2 * 8);
    c3_copy<8>(reinterpret_cast<f32x4 *>(D), reinterpret_cast<const f32x4 *>(a.dz3 + (int64_t)s0 * wo2 * 64),
               ns * wo2 * 16);
    __syncthreads();
    C3B_CLK(1);
    const int r = lane & 31, h = lane >> 5;
    const int kk = grp * 4 + wave;
    const int dv = kk / 6, du = kk - dv * 6;
    const bool hv = h < ns;
    const float *pa = A + ((hv ? h : 0) * bs2 + du + dv * a.bs) * 32 + r;
    const float *pd = D + (hv ? h : 0) * wo2 * 64 + r;
    f32x16 acc[2];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[nt][g] = 0.0f;
    for (int jo = 0; jo < WO; ++jo) {
        const float *ra = pa + jo * a.bs * 32;
        const float *rd = pd + jo * WO * 64;
#pragma unroll
        for (int io = 0; io < WO; ++io) {
            const float x = ra[io * 32], y0 = rd[io * 64], y1 = rd[io * 64 + 32];
            acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv ? x : 0.0f, y0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(hv ? x : 0.0f, y1, acc[1], 0, 0, 0);
        }
    }
    C3B_CLK(2);
    float *out = a.slab + (int64_t)z * 1153 * 64;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) out[(kk * 32 + acc_row(g, lane)) * 64 + nt * 32 + r] = acc[nt][g];
    if (grp == 0) {   // bias row: column sums of the chunk's dz3 (four partial runs, then in order)
        __shared__ float bpart[4][64];
        const int K = ns * wo2, co = tid & 63, q = tid >> 6, len = (K + 3) / 4;
        const int k0 = q * len, k1 = min(K, k0 + len);
        float b = 0.0f;
        int k = k0;
        for (; k + 8 <= k1; k += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = D[(k + u) * 64 + co];
#pragma unroll
            for (int u = 0; u < 8; ++u) b += v[u];
        }
        for (; k < k1; ++k) b += D[k * 64 + co];
        bpart[q][co] = b;
        __syncthreads();
        if (tid < 64) out[1152 * 64 + tid] = ((bpart[0][tid] + bpart[1][tid]) + bpart[2][tid]) + bpart[3][tid];
    }
}

typedef float f32x4m __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void c3_dx_block(const Conv3BwdArgs &a, int s, int cg, float *sm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs2 = a.bs * a.bs, wo2 = a.wo * a.wo;
    constexpr int NN = 36 * C3_CG;   // T columns (kk, ci)
    float *Dz = sm, *Wl = sm + wo2 * C3_DLD, *Tl = sm;
    // relu-mask values of this block's outputs, loaded now (used by the col2im)
    constexpr int NMK = 3;   // (pin, ci) per thread: bs^2 * CG <= 3 * 256 for bs <= 13
    float mk[NMK];
#pragma unroll
    for (int u = 0; u < NMK; ++u) {
        const int e = u * 256 + tid, ee = e < bs2 * C3_CG ? e : 0;
        mk[u] = a.a2[((int64_t)s * bs2 + ee / C3_CG) * 32 + cg * C3_CG + ee % C3_CG];
    }
    // dz3[s] and W[kk][cg*CG + ci][co] (row n = kk*CG + ci)
    c3_copy_rows<4>(Dz, a.dz3 + (int64_t)s * wo2 * 64, wo2, [](int row) { return row; });
    c3_copy_rows<9>(Wl, a.w, NN, [cg](int n) { return (n / C3_CG) * 32 + cg * C3_CG + n % C3_CG; });
    __syncthreads();
    C3B_CLK(1);
    // T in 16x16 tiles (v_mfma_f32_16x16x4_f32: lane l holds A[l&15][k + (l>>4)],
    // B[k + (l>>4)][l&15]; C rows 4*(l>>4) + e, column l&15), round robin over the waves
    // (all tiles kept in registers, then written over the operands after a barrier)
    const int r = lane & 15, g = lane >> 4;
    const int rt = (wo2 + 15) / 16, ct = NN / 16;
    constexpr int MT = 9;   // tiles per wave: rt <= 4 (Wo <= 8), ct = 9
    f32x4m acc[MT];
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int t = wave + 4 * u;
        acc[u] = f32x4m{0.0f, 0.0f, 0.0f, 0.0f};
        if (t < rt * ct) {
            const int tr = t / ct, tc = t - tr * ct;
            const float *pa = Dz + min(tr * 16 + r, wo2 - 1) * C3_DLD + g;
            const float *pb = Wl + (tc * 16 + r) * C3_DLD + g;
#pragma unroll
            for (int k = 0; k < 64; k += 4) acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[k], pb[k], acc[u], 0, 0, 0);
        }
    }
    __syncthreads();
    C3B_CLK(2);
#pragma unroll
    for (int u = 0; u < MT; ++u) {
        const int t = wave + 4 * u;
        if (t < rt * ct) {
            const int tr = t / ct, tc = t - tr * ct;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int rr = tr * 16 + 4 * g + e;
                if (rr < wo2) Tl[rr * C3_TLD + tc * 16 + r] = acc[u][e];
            }
        }
    }
    __syncthreads();
    C3B_CLK(3);
    // col2im + relu mask, (pin, ci) per thread: the 36 terms load together (out-of-grid
    // terms read a valid slot and add 0), summed kk ascending
#pragma unroll
    for (int u = 0; u < NMK; ++u) {
        const int e = u * 256 + tid;
        if (e >= bs2 * C3_CG) break;
        const int pin = e / C3_CG, ci = e - pin * C3_CG;
        const int j = pin / a.bs, i = pin - j * a.bs;
        float t[36];
#pragma unroll
        for (int kk = 0; kk < 36; ++kk) {
            const int dv = kk / 6, du = kk - dv * 6;
            const int io = i - du, jo = j - dv;
            const bool v = io >= 0 && io < a.wo && jo >= 0 && jo < a.wo;
            const float x = Tl[(v ? io + jo * a.wo : 0) * C3_TLD + kk * C3_CG + ci];
            t[kk] = v ? x : 0.0f;
        }
        float v = 0.0f;
#pragma unroll
        for (int kk = 0; kk < 36; ++kk) v += t[kk];
        const int64_t o = ((int64_t)s * bs2 + pin) * 32 + cg * C3_CG + ci;
        a.dz2[o] = mk[u] > 0.0f ? v : 0.0f;
    }
}

__global__ __launch_bounds__(256) void conv3_bwd_kernel(Conv3BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float c3sm[];
    const int b = blockIdx.x;
    C3B_CLK(0);
#ifdef SNK_ENV_CLOCKS
    if (threadIdx.x == 0 && g_c3b_clk) {
        g_c3b_clk[(int64_t)b * 8 + 7] = 1 + (uint64_t)__builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
        g_c3b_clk[(int64_t)b * 8 + 6] = 1 + (uint64_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11));
    }
#endif
    if (b < a.nW) {
        switch (a.wo) {
            case 3: c3_dw_block<3>(a, b / 9, b % 9, c3sm); break;
            case 4: c3_dw_block<4>(a, b / 9, b % 9, c3sm); break;
            case 5: c3_dw_block<5>(a, b / 9, b % 9, c3sm); break;
            case 6: c3_dw_block<6>(a, b / 9, b % 9, c3sm); break;
            case 7: c3_dw_block<7>(a, b / 9, b % 9, c3sm); break;
            default: c3_dw_block<8>(a, b / 9, b % 9, c3sm); break;
        }
    } else
        c3_dx_block(a, (b - a.nW) / (32 / C3_CG), (b - a.nW) % (32 / C3_CG), c3sm);
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
//  * dX block: dz2[s] inside a zero border ([(bs+2)^2][36]) and the weights
//    [kk][ci][co] ([144][36]); 16-row position tiles round robin over the waves,
//    K = 9 offsets x 32 channels: dzc1[pin][ci] = sum dz2b[pin + (1,1) - (du,dv)][co]
//    * W[kk][ci][co], relu-masked by a1.
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
constexpr int C2_DS = 48, C2_BS = 36, C2_WS = 36;   // LDS row strides (floats), conflict-free reads

__host__ __device__ inline int c2_bwd_lds_floats(int bs) {
    const int bp2 = (bs + 2) * (bs + 2);
    int dw = bp2 * 16 + bs * bs * C2_DS, dx = bp2 * C2_BS + 144 * C2_WS + 2 * bp2;   // + conv1's planes (C <= 2)
    if (dw < 4 * 4608) dw = 4 * 4608;   // the weight-gradient block's cross-wave sum
    return dw > dx ? dw : dx;
}

__device__ __forceinline__ void c2_dw_block(const Conv2BwdArgs &a, int s, float *sm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs = a.bs, bp = bs + 2, bs2 = bs * bs, bp2 = bp * bp;
    float *A1 = sm, *D2 = sm + bp2 * 16;
    for (int e = tid; e < bp2 * 4; e += 256) reinterpret_cast<f32x4 *>(A1)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    {
        constexpr int U = 8;   // loads in flight per thread
        const f32x4 *src = reinterpret_cast<const f32x4 *>(a.a1 + (int64_t)s * bs2 * 16);
        for (int b = 0; b < bs2 * 4; b += U * 256) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                v[u] = src[e < bs2 * 4 ? e : 0];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                if (e < bs2 * 4) {
                    const int p = e >> 2, j = p / bs, i = p - j * bs;
                    reinterpret_cast<f32x4 *>(A1 + ((i + 1) + (j + 1) * bp) * 16)[e & 3] = v[u];
                }
            }
        }
        const f32x4 *srd = reinterpret_cast<const f32x4 *>(a.dz2 + (int64_t)s * bs2 * 32);
        for (int b = 0; b < bs2 * 8; b += U * 256) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                v[u] = srd[e < bs2 * 8 ? e : 0];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                if (e < bs2 * 8) reinterpret_cast<f32x4 *>(D2 + (e >> 3) * C2_DS)[e & 7] = v[u];
            }
        }
    }
    __syncthreads();
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

constexpr int C2_NXB = 2;   // data-gradient blocks per sample (interleaved 16-row tiles)

__device__ __forceinline__ void c2_dx_block(const Conv2BwdArgs &a, int s, int xb, float *sm) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int bs = a.bs, bp = bs + 2, bs2 = bs * bs, bp2 = bp * bp;
    float *Db = sm, *Wl = sm + bp2 * C2_BS;
    for (int e = tid; e < bp2 * (C2_BS / 4); e += 256) reinterpret_cast<f32x4 *>(Db)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    {
        constexpr int U = 8;
        const f32x4 *srd = reinterpret_cast<const f32x4 *>(a.dz2 + (int64_t)s * bs2 * 32);
        for (int b = 0; b < bs2 * 8; b += U * 256) {
            f32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                v[u] = srd[e < bs2 * 8 ? e : 0];
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 256 + tid;
                if (e < bs2 * 8) {
                    const int p = e >> 3, j = p / bs, i = p - j * bs;
                    reinterpret_cast<f32x4 *>(Db + ((i + 1) + (j + 1) * bp) * C2_BS)[e & 7] = v[u];
                }
            }
        }
        // conv1's input planes inside a zero border (the fused conv1 weight gradient reads them
        // from LDS: a global load per MFMA operand left the MFMA chain waiting on each)
        if (a.c1slab) {
            float *Xb = Wl + 144 * C2_WS;
            for (int e = tid; e < a.C * bp2; e += 256) {
                const int c = e / bp2, pb = e - c * bp2, jj = pb / bp - 1, ii = pb - (jj + 1) * bp - 1;
                Xb[e] = (ii >= 0 && ii < bs && jj >= 0 && jj < bs) ? a.x.load(s, c, ii + jj * bs) : 0.0f;
            }
        }
        const f32x4 *sw = reinterpret_cast<const f32x4 *>(a.w);
        f32x4 v[5];   // 144 rows x 8 float4 = 1152 = 4.5 per thread
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int e = u * 256 + tid;
            v[u] = sw[e < 1152 ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < 5; ++u) {
            const int e = u * 256 + tid;
            if (e < 1152) reinterpret_cast<f32x4 *>(Wl + (e >> 3) * C2_WS)[e & 7] = v[u];
        }
    }
    __syncthreads();
    const int r = lane & 15, g = lane >> 4;
    const int nt = (bs2 + 15) / 16;
    // conv1 weight gradient over this wave's tiles: C1[(kk, c) | bias][co] = sum over the
    // tile's positions p of x[p + (du-1, dv-1)][c] * dzc1[p][co], as v_mfma_f32_16x16x4_f32
    // with k = position: step m takes positions 4g + m, whose dzc1 this lane already holds
    // in acc[m] (column co = r); rows 0..15 and 16..31 of (kk, c) (9C of them, then the bias
    // row of ones, then zeros)
    f32x4m c1acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
    const int nrow = 9 * a.C;
    for (int t = xb + C2_NXB * wave; t < nt; t += 4 * C2_NXB) {
        const int p = min(t * 16 + r, bs2 - 1);
        const int j = p / bs, i = p - j * bs;
        f32x4m acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int dv = kk / 3, du = kk - dv * 3;
            // dz2 at (i + 1 - du, j + 1 - dv) in the input grid = bordered (i + 2 - du, j + 2 - dv)
            const float *pa = Db + ((i + 2 - du) + (j + 2 - dv) * bp) * C2_BS + g;
            const float *pb = Wl + (kk * 16 + r) * C2_WS + g;
#pragma unroll
            for (int c = 0; c < 32; c += 4) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[c], pb[c], acc, 0, 0, 0);
        }
        f32x4m dzm;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int row = t * 16 + 4 * g + e;
            dzm[e] = 0.0f;
            if (row < bs2) {
                const int64_t o = ((int64_t)s * bs2 + row) * 16 + r;
                dzm[e] = a.a1[o] > 0.0f ? acc[e] : 0.0f;
                a.dzc1[o] = dzm[e];
            }
        }
        if (!a.c1slab) continue;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int pos = t * 16 + 4 * g + m;   // k = g of this step
            const int pj = pos / bs, pi = pos - pj * bs;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt) {
                const int k1 = rt * 16 + r;           // row (kk, c) of this lane's A element
                float xv = 0.0f;
                if (pos < bs2) {
                    if (k1 < nrow) {
                        const int kk = k1 / a.C, c = k1 - kk * a.C;
                        // bordered (pi + kk % 3, pj + kk / 3) = input (pi + kk % 3 - 1, pj + kk / 3 - 1)
                        xv = Wl[144 * C2_WS + c * bp2 + (pi + kk % 3) + (pj + kk / 3) * bp];
                    } else if (k1 == nrow) {
                        xv = 1.0f;
                    }
                }
                c1acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, dzm[m], c1acc[rt], 0, 0, 0);
            }
        }
    }
    if (!a.c1slab) return;
    // the block's four wave partials, summed in wave order through LDS (the staging is free)
    __syncthreads();
    float *red = sm;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int e = 0; e < 4; ++e) red[((wave * 2 + rt) * 4 + e) * 64 + lane] = c1acc[rt][e];
    __syncthreads();
    float *out = a.c1slab + ((int64_t)s * C2_NXB + xb) * (nrow + 1) * 16;
    for (int q = tid; q < 2 * 4 * 64; q += 256) {
        const float v = ((red[q] + red[512 + q]) + red[1024 + q]) + red[1536 + q];
        const int ln = q & 63, e = (q >> 6) & 3, rt = q >> 8;
        const int row = rt * 16 + 4 * (ln >> 4) + e;   // C[row][col = ln & 15]
        if (row <= nrow) out[row * 16 + (ln & 15)] = v;
    }
}

__global__ __launch_bounds__(256) void conv2_bwd_kernel(Conv2BwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) float c2sm[];
    const int b = blockIdx.x;
    if (b < a.S)
        c2_dw_block(a, b, c2sm);
    else
        c2_dx_block(a, (b - a.S) / C2_NXB, (b - a.S) % C2_NXB, c2sm);
}

}  // namespace snk

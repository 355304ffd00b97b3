// snk_deep_bwd.hpp — L3's backward (6x6, 64 -> 64, valid) of the configs[2]
// deep net at the update's batch (B = 64), on v_mfma_f32_16x16x32_bf16.
//
// The generic engine (gemm_bf16_kernel + snk_loaders.hpp) gathered every
// im2col element with two integer divisions and a scalar load: the data
// gradient took 335 us and the weight gradient 156 us + a reduce for 2 x 4.2
// GFLOP. Both are reorganised around LDS images of the sample(s) a workgroup
// owns, with the arithmetic of the contract unchanged (snk_deep.hpp header,
// oracle/snake_oracle.c conv_bwd_bf16): the masked gradient dz3 is rounded to
// bf16 (RNE) as the operand, the weights are the bf16 image, a2 is bf16, every
// product is exact and the sums are fp32.
//
//  * deep_conv3_dx_kernel (grid: NB tile rows x S samples, 8 waves):
//    dz2[s][pin][ci] = (a2 > 0) * sum_{du,dv,co} dz3[s][pin - (du,dv)][co] * W[kk][ci][co].
//    The workgroup's 4 output rows need dz3 rows 4tj-5 .. 4tj+3: a bordered bf16
//    image of 9 rows x PJ = 28 columns, 160 bytes per position (64 channels + 16
//    bytes of pad), zeros outside the Wo x Wo grid. Row tiles are 4x4 blocks of
//    output positions (as deep_front_kernel); with the 160-byte stride and
//    PJ = 28 every ds_read_b128 lane group of a B fragment hits 16 distinct bank
//    quads (simulated), and a read's address is one lane constant minus a
//    wave-uniform (kernel offset, tile) term. A = the weights in packed order
//    [kk][ci][co] (the image's W3T section), straight from L2 into a four-offset
//    register ring: rows = ci, k = co. Wave = (ci tile, contraction half); the
//    halves meet in LDS. (One wave per (ci tile, 2-3 row tiles) with both halves
//    and a two-offset ring waited on L2 every offset: 38 us at B = 64, 20x20.)
//  * deep_conv3_dw_kernel (grid: 6 kernel rows dv x ceil(S/2) sample pairs):
//    slab[z][(kk*64 + ci)*64 + co] = sum_{s in pair z, pout} dz3[s][pout][co] *
//    a2[s][pout + (du,dv)][ci]; the dv == 0 blocks also write the bias row
//    (column sums of the rounded dz3). The sum runs over positions, so both
//    operands are read k-major with ds_read_b64_tr_b16 (gfx950's transposing
//    LDS read) from natural [position][channel] images: each lane supplies its
//    own position's row address, which makes the shifted window (pout + (du,
//    dv)) and the 225 -> 256 k padding (a zero dz3 row) free. 152-byte rows
//    keep both kinds of read at most 2-way (simulated). slab_reduce_kernel sums
//    the pairs in pair order.
#pragma once
#include "snk_deep.hpp"

namespace snk {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ---------------------------------------------------------------- data gradient
template <int H>
struct DeepL3DxShape {
    static constexpr int WO = H - 5, NB = (H + 3) / 4, PJ = 28, ROWS = 9, PST = 80;   // PST: halves per position
    static constexpr int IMG = ROWS * PJ * PST * 2;                                   // bytes
    static constexpr int RED = 4 * NB * 4 * 64 * 4;                                   // the k-half partials
    static constexpr int LDS = IMG > RED ? IMG : RED;
    static_assert(4 * NB + 5 <= PJ, "image columns");
};

// 8 waves: wave w takes ci tile w & 3 and channel half c = w >> 2 of the contraction
// (co 32c .. 32c + 31) for all NB row tiles of the workgroup's tile row; the two halves'
// partials meet in LDS at the end (half 1 adds into half 0's sums, in that order).
// Per kernel offset a wave loads ONE weight fragment and runs NB MFMAs; the weights
// go through a 4-offset register ring (L2 latency covered by 4 x NB MFMAs).
template <int H>
__global__ __launch_bounds__(512) void deep_conv3_dx_kernel(const float *__restrict__ dz3,
                                                            const uint16_t *__restrict__ wt,
                                                            const uint16_t *__restrict__ a2, float *__restrict__ dz2,
                                                            int64_t S) {
    using Sh = DeepL3DxShape<H>;
    constexpr int WO = Sh::WO, NB = Sh::NB, PJ = Sh::PJ, PST = Sh::PST, ROWS = Sh::ROWS;
    constexpr int RING = 4;
    static_assert(36 % RING == 0, "ring");
    extern __shared__ __attribute__((aligned(16))) uint16_t dxsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4, ct = wave & 3, c = wave >> 2;
    const int tj = blockIdx.x;
    const int64_t s = blockIdx.y;
    if (s >= S) return;
    // the weight fragment of kernel offset kk: rows ci = 16 ct + r, k = co 32 c + 8 g .. +7
    const uint16_t *wl = wt + (ct * 16 + r) * 64 + 32 * c + 8 * g;
    u32x4 wf[RING];
#pragma unroll
    for (int o = 0; o < RING; ++o) wf[o] = *reinterpret_cast<const u32x4 *>(wl + o * 4096);
    // stage dz3 rows 4tj-5 .. 4tj+3 (image row y), columns -5 .. PJ-6 (image column c) as bf16
    {
        constexpr int NP = ROWS * PJ * 16, PT = (NP + 511) / 512;
        const float *src = dz3 + s * (WO * WO * 64);
        const int jlo = 4 * tj - 5;
        f32x4 v[PT];
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q >> 4, pc = q & 15;
            const int y = pos / PJ, cc = pos - y * PJ, jj = jlo + y, ii = cc - 5;
            const bool ok = q < NP && jj >= 0 && jj < WO && ii >= 0 && ii < WO;
            v[u] = ok ? *reinterpret_cast<const f32x4 *>(src + (jj * WO + ii) * 64 + pc * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q >> 4, pc = q & 15;
            if (q < NP)
                *reinterpret_cast<u32x2 *>(dxsm + pos * PST + pc * 4) =
                    u32x2{pk_bf16(v[u][0], v[u][1]), pk_bf16(v[u][2], v[u][3])};
        }
    }
    __syncthreads();
    // lane position (4 ti + (r & 3), 4 tj + (r >> 2)): its dz3 cell at offset (du, dv) is
    // image row 5 + (r >> 2) - dv, column 4 ti + (r & 3) + 5 - du
    const int lbase = ((5 + (r >> 2)) * PJ + 5 + (r & 3)) * PST + 32 * c + 8 * g;
    f32x4 acc[NB];
#pragma unroll
    for (int i = 0; i < NB; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k4 = 0; k4 < 36; k4 += RING) {
#pragma unroll
        for (int o = 0; o < RING; ++o) {
            const int kk = k4 + o, du = kk % 6, dv = kk / 6;
            const uint16_t *Bk = dxsm + lbase - (dv * PJ + du) * PST;
            bf16x8 xv[NB];
#pragma unroll
            for (int i = 0; i < NB; ++i) xv[i] = as_bf(*reinterpret_cast<const u32x4 *>(Bk + 4 * i * PST));
#pragma unroll
            for (int i = 0; i < NB; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(wf[o]), xv[i], acc[i], 0, 0, 0);
            if (kk + RING < 36) wf[o] = *reinterpret_cast<const u32x4 *>(wl + (kk + RING) * 4096);
        }
    }
    // the two contraction halves: half 1 parks its sums, half 0 adds them (after the image is dead)
    __syncthreads();
    f32x4 *red = reinterpret_cast<f32x4 *>(dxsm);
    if (c == 1) {
#pragma unroll
        for (int i = 0; i < NB; ++i) red[(ct * NB + i) * 64 + lane] = acc[i];
    }
    __syncthreads();
    if (c == 1) return;
    // epilogue: lane holds ci = 16 ct + 4 g + e of its position; relu mask of a2, fp32 out
#pragma unroll
    for (int i = 0; i < NB; ++i) {
        const f32x4 p = red[(ct * NB + i) * 64 + lane];
        const int ii = 4 * i + (r & 3), jj = 4 * tj + (r >> 2);
        if (ii >= H || jj >= H) continue;
        const int64_t o = (s * (H * H) + ii + jj * H) * 64 + ct * 16 + 4 * g;
        const u32x2 m = *reinterpret_cast<const u32x2 *>(a2 + o);
        f32x4 y;
        y[0] = bf2f((uint16_t)(m[0] & 0xffffu)) > 0.0f ? acc[i][0] + p[0] : 0.0f;
        y[1] = bf2f((uint16_t)(m[0] >> 16)) > 0.0f ? acc[i][1] + p[1] : 0.0f;
        y[2] = bf2f((uint16_t)(m[1] & 0xffffu)) > 0.0f ? acc[i][2] + p[2] : 0.0f;
        y[3] = bf2f((uint16_t)(m[1] >> 16)) > 0.0f ? acc[i][3] + p[3] : 0.0f;
        *reinterpret_cast<f32x4 *>(dz2 + o) = y;
    }
}

// ---------------------------------------------------------------- weight gradient
template <int H>
struct DeepL3DwShape {
    static constexpr int WO = H - 5, NO = WO * WO, KST = (NO + 31) / 32;
    static constexpr int RST = 76;                      // halves per row (152 bytes)
    static constexpr int DZR = NO + 1, AR = WO * H;     // dz3 rows (+ the zero row NO), a2 window rows
    static constexpr int SMP = (DZR + AR) * RST;        // halves per sample
    static constexpr int LDS = 2 * SMP * 2;
    static constexpr int MN = (36 * 64 + 1) * 64;       // one slab (the bias row last)
    static_assert(LDS <= 160 * 1024, "two samples per workgroup");
    static_assert((SMP * 2) % 8 == 0 && (DZR * RST * 2) % 8 == 0, "8-byte aligned transposed reads");
};

__device__ __forceinline__ u32x2 tr_read(const uint16_t *p) {
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
    return __builtin_bit_cast(u32x2, v);
}

template <int H>
__global__ __launch_bounds__(512) void deep_conv3_dw_kernel(const float *__restrict__ dz3,
                                                            const uint16_t *__restrict__ a2, float *__restrict__ slab,
                                                            int64_t S) {
    using Sh = DeepL3DwShape<H>;
    constexpr int WO = Sh::WO, NO = Sh::NO, KST = Sh::KST, RST = Sh::RST, DZR = Sh::DZR, AR = Sh::AR, SMP = Sh::SMP;
    extern __shared__ __attribute__((aligned(16))) uint16_t dwsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int dv = blockIdx.x;
    const int64_t z = blockIdx.y;
    // ---- staging: per sample q, dz3 rows 0 .. NO-1 as bf16 + the zero row NO; a2 rows dv*H .. dv*H + AR - 1
    {
        constexpr int NDZ = 2 * DZR * 16, NA = 2 * AR * 8, NTOT = NDZ + NA, U = 12;
        for (int b = 0; b < NTOT; b += U * 512) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 512 + tid;
                v[u] = u32x4{0u, 0u, 0u, 0u};
                if (e < NDZ) {
                    const int q = e / (DZR * 16), rem = e - q * (DZR * 16), row = rem >> 4, pc = rem & 15;
                    const int64_t sg = 2 * z + q;
                    if (row < NO && sg < S) {
                        const f32x4 f = *reinterpret_cast<const f32x4 *>(dz3 + (sg * NO + row) * 64 + pc * 4);
                        v[u] = u32x4{pk_bf16(f[0], f[1]), pk_bf16(f[2], f[3]), 0u, 0u};
                    }
                } else if (e < NTOT) {
                    const int ea = e - NDZ, q = ea / (AR * 8), rem = ea - q * (AR * 8), row = rem >> 3, pc = rem & 7;
                    const int64_t sg = min(2 * z + q, S - 1);   // finite values (a missing sample's dz3 is zero)
                    v[u] = *reinterpret_cast<const u32x4 *>(a2 + (sg * (H * H) + dv * H + row) * 64 + pc * 8);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 512 + tid;
                if (e < NDZ) {
                    const int q = e / (DZR * 16), rem = e - q * (DZR * 16), row = rem >> 4, pc = rem & 15;
                    *reinterpret_cast<u32x2 *>(dwsm + q * SMP + row * RST + pc * 4) = u32x2{v[u][0], v[u][1]};
                } else if (e < NTOT) {
                    const int ea = e - NDZ, q = ea / (AR * 8), rem = ea - q * (AR * 8), row = rem >> 3, pc = rem & 7;
                    uint16_t *d = dwsm + q * SMP + (DZR + row) * RST + pc * 8;
                    *reinterpret_cast<u32x2 *>(d) = u32x2{v[u][0], v[u][1]};
                    *reinterpret_cast<u32x2 *>(d + 4) = u32x2{v[u][2], v[u][3]};
                }
            }
        }
    }
    __syncthreads();
    float *sl = slab + z * Sh::MN;
    if (dv == 0 && tid < 64) {   // bias row: column sums of the rounded dz3, sample then position order
        float b = 0.0f;
        for (int q = 0; q < 2; ++q)
            for (int row = 0; row < NO; ++row) b += bf2f(dwsm[q * SMP + row * RST + tid]);
        sl[36 * 64 * 64 + tid] = b;
    }
    // ---- wave tile: co tiles 2cp, 2cp+1; ci tiles 2ip, 2ip+1; kernel columns du = 3dh .. 3dh+2
    const int cp = wave & 1, ip = (wave >> 1) & 1, dh = wave >> 2;
    const int G = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    f32x4 acc[3][2][2];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b][0] = acc[a][b][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int q = 0; q < 2; ++q) {
        const uint16_t *dzb = dwsm + q * SMP + (32 * cp + 4 * pp);             // + row * RST (+ 16 for tile 2cp+1)
        const uint16_t *a2b = dwsm + q * SMP + DZR * RST + (32 * ip + 4 * pp);  // + (apos + du) * RST
#pragma unroll 1
        for (int ks = 0; ks < KST; ++ks) {
            int drow[2], arow[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int k = 32 * ks + 8 * G + qq + 4 * hh;
                drow[hh] = (k < NO ? k : NO) * RST;
                const int kc = k < NO ? k : NO - 1, kj = kc / WO;
                arow[hh] = (kc - kj * WO + kj * H + 3 * dh) * RST;
            }
            bf16x8 A[2];
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const u32x2 lo = tr_read(dzb + drow[0] + 16 * t), hi = tr_read(dzb + drow[1] + 16 * t);
                A[t] = as_bf(u32x4{lo[0], lo[1], hi[0], hi[1]});
            }
#pragma unroll
            for (int d = 0; d < 3; ++d) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const u32x2 lo = tr_read(a2b + arow[0] + d * RST + 16 * t);
                    const u32x2 hi = tr_read(a2b + arow[1] + d * RST + 16 * t);
                    const bf16x8 Bv = as_bf(u32x4{lo[0], lo[1], hi[0], hi[1]});
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        acc[d][c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[c], Bv, acc[d][c][t], 0, 0, 0);
                }
            }
        }
    }
    // lane holds co = 16 (2cp + c) + 4 G + e, ci = 16 (2ip + t) + (lane & 15) of offset kk = 3dh + d + 6dv
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        const int kk = 3 * dh + d + 6 * dv;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int co = 16 * (2 * cp + c) + 4 * G, ci = 16 * (2 * ip + t) + (lane & 15);
                *reinterpret_cast<f32x4 *>(sl + (kk * 64 + ci) * 64 + co) = acc[d][c][t];
            }
    }
}

}  // namespace snk

// snk_conv_x6.hpp — fp32-accurate implicit-GEMM convolution on bf16 MFMA.
//
// gfx950 runs v_mfma_f32_32x32x16_bf16 at 16x the FLOP rate of the exact-f32
// v_mfma_f32_32x32x2_f32. Every fp32 value splits into three bf16 parts by
// round-to-nearest: h = bf16(x), m = bf16(x - h), l = bf16(x - h - m), each
// difference exact, |m| <= 2^-8 |x|, |l| <= 2^-16 |x|, and x - (h+m+l) within
// 2^-25 |x|. A product then needs the 6 part products of magnitude >= 2^-16:
//   x*y ~= hh + hm + mh + hl + mm + lh       (dropped: ml + lm + ll <= 2^-23)
// each exact in fp32 (8-bit x 8-bit mantissas) and accumulated in fp32 by the
// MFMA: the error class of an fp32 dot product, at 6 x 32 = 192 MFMA cycles
// per 32x32x16 block instead of 8 x 64 = 512 (2.7x).
//
// Same structure as conv_mfma_kernel (snk_conv.hpp): 4 waves x 32 rows, per
// kernel offset kk the three bf16 planes of the CK x CN weight block are
// staged into LDS ([plane][n][c], rows padded by 8 bf16: conflict-free
// ds_read_b128), double buffered with one barrier per offset; A is read as
// fp32 float4s from global/L2 one offset ahead and split in registers after
// the MFMA block. Weight planes come from an image [kk][plane][n][c] built
// with the fp32 image (transpose_fwd / grad_update).
//
// MFMA 32x32x16 bf16 operand map: lane l (r = l&31, h = l>>5) holds
// A[row r][k = 8h + j] and B[k = 8h + j][col r], j = 0..7; C/D as the f32 form.
#pragma once
#include <type_traits>

#include "snk_conv.hpp"

namespace snk {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

struct Split3 {
    u32x4 h, m, l;   // 8 bf16 each, element j in half (j & 1) of dword j >> 1
};

// bf16 pair (round to nearest even: v_cvt_pk_bf16_f32) and its value as floats
__device__ __forceinline__ uint32_t bf2(const f32x2 &x, f32x2 &back) {
    const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(x, bf16x2));
    back = f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
    return u;
}

// split of 8 floats into bf16 planes h, m, l
__device__ __forceinline__ Split3 split3(const f32x4 &x0, const f32x4 &x1) {
    Split3 s;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 x = i < 2 ? f32x2{x0[2 * i], x0[2 * i + 1]} : f32x2{x1[2 * i - 4], x1[2 * i - 3]};
        f32x2 b;
        s.h[i] = bf2(x, b);
        const f32x2 r1 = x - b;
        s.m[i] = bf2(r1, b);
        const f32x2 r2 = r1 - b;
        s.l[i] = bf2(r2, b);
    }
    return s;
}

__device__ __forceinline__ bf16x8 as_bf(const u32x4 &v) { return __builtin_bit_cast(bf16x8, v); }

// bf16 plane p (0 = h, 1 = m, 2 = l) of x, as split3 computes it
__device__ __forceinline__ uint16_t split_part(float x, int p) {
    f32x2 b;
    f32x2 v{x, 0.0f};
    uint32_t u = bf2(v, b);
    for (int q = 0; q < p; ++q) {
        v = v - b;
        u = bf2(v, b);
    }
    return (uint16_t)(u & 0xffffu);
}

// PRE: A comes pre-split (a.xb, written by the producing layer's epilogue),
// so the main loop does no conversion work at all.
// BSPLIT: the weights come as the fp32 image a.w ([kk][n][c]) and are split
// while staged (one 8-channel piece per thread and offset at CN x CK = 2048:
// the B = 64 conv3 data gradient, whose weights change every update).
// MODE_DX: A = dz[s][p - (du,dv) + PAD][c] with the bounds check (HIN < HOUT).
template <int CK, int CN, int KS, int PAD, int MODE, int EPI, bool PRE, bool BSPLIT = false>
__device__ __forceinline__ void conv_x6_body(const ConvPair &pr, dim3 bid) {
    const ConvArgs &a = pr.g[bid.z];
    const uint16_t *__restrict__ wb = pr.wb[bid.z];
    constexpr int NT = CN / 32;
    constexpr int KC = CK / 16;                  // 16-channel MFMA chunks per offset
    constexpr int LDB = CK + 8;                  // bf16 per LDS row
    constexpr int PLANE = CN * LDB;              // bf16 per LDS plane
    constexpr int NE = BSPLIT ? CN * CK / 8 : 3 * CN * CK / 8;   // staged units per block: 8-channel
    constexpr int NV = (NE + 255) / 256;                          //   pieces (BSPLIT) or 16-byte plane pieces
    __shared__ __attribute__((aligned(16))) uint16_t Bs[2][3 * PLANE + 8];   // + pad piece for idle stagers; lds: one per kernel (a paired launch's two bodies never share it)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int m = bid.x * 128 + wave * 32 + r;
    const bool ok = m < a.M;
    const int mm = ok ? m : 0;
    int s, i = 0, j = 0;
    if (MODE == MODE_DENSE) {
        s = mm;
    } else {
        s = (int)fdiv((uint32_t)mm, a.d2m, a.d2s);
        const int p = mm - s * a.HOUT * a.HOUT;
        j = (int)fdiv((uint32_t)p, a.d1m, a.d1s);
        i = p - j * a.HOUT;
    }
    const float *xs = a.x + (int64_t)s * a.HIN * a.HIN * CK + 8 * h;
    const uint16_t *xsb = PRE ? a.xb + (int64_t)s * a.HIN * a.HIN * 3 * CK + 8 * h : nullptr;
    const int kk0 = bid.y * a.kk_per_split;
    const int kk1 = min(a.nkk, kk0 + a.kk_per_split);

    f32x16 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[nt][g] = 0.0f;

    const u32x4 *wsrc = reinterpret_cast<const u32x4 *>(wb);
    int s_src[NV], s_dst[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int e = tid + q * 256;
        const bool in = (NE % 256 == 0) || e < NE;
        const int ee = in ? e : 0;
        const int pl = BSPLIT ? 0 : ee / (CN * CK / 8), rem = ee - pl * (CN * CK / 8);
        const int n = rem / (CK / 8), c8 = rem - n * (CK / 8);
        s_src[q] = ee;
        s_dst[q] = in ? pl * PLANE + n * LDB + c8 * 8 : 3 * PLANE;
    }

    // input position of row m at kernel offset kk (-1: outside the board / past M)
    auto a_pos = [&](int kk) -> int {
        if (MODE == MODE_DENSE) return ok ? kk : -1;
        const int dv = kk / KS, du = kk - dv * KS;
        const int xi = MODE == MODE_DX ? i - du + PAD : i + du - PAD;
        const int xj = MODE == MODE_DX ? j - dv + PAD : j + dv - PAD;
        if (PAD == 0 && MODE == MODE_FWD) return xi + xj * a.HIN;   // always inside; rows past M are never stored
        const bool v = ok && xi >= 0 && xi < a.HIN && xj >= 0 && xj < a.HIN;
        return v ? xi + xj * a.HIN : -1;
    };
    // A of one offset: raw floats (split later) or the pre-split planes
    f32x4 araw[PRE ? 1 : 2 * KC];
    u32x4 abf[PRE ? KC : 1][3];
    auto a_load = [&](int kk) -> bool {
        const int pos = a_pos(kk);
        const int pp = pos < 0 ? 0 : pos;
        if (PRE) {
            const uint16_t *pb = xsb + (int64_t)pp * 3 * CK;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) abf[kc][pl] = *reinterpret_cast<const u32x4 *>(pb + pl * CK + kc * 16);
        } else {
            const float *p = xs + (int64_t)pp * CK;
#pragma unroll
            for (int c = 0; c < 2 * KC; ++c) araw[c] = *reinterpret_cast<const f32x4 *>(p + (c >> 1) * 16 + (c & 1) * 4);
        }
        return pos >= 0;
    };
    auto a_finish = [&](bool v, Split3 (&cur)[KC]) {
        if (PRE) {
            const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
            for (int kc = 0; kc < KC; ++kc) {
                cur[kc].h = v ? abf[kc][0] : z;
                cur[kc].m = v ? abf[kc][1] : z;
                cur[kc].l = v ? abf[kc][2] : z;
            }
        } else {
            const float msk = v ? 1.0f : 0.0f;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
                cur[kc] = (PAD == 0 && MODE == MODE_FWD) ? split3(araw[2 * kc], araw[2 * kc + 1])
                                                           : split3(araw[2 * kc] * msk, araw[2 * kc + 1] * msk);
        }
    };

    u32x4 bst[NV][BSPLIT ? 2 : 1];
    const u32x4 *wsrc32 = reinterpret_cast<const u32x4 *>(a.w);
    auto b_load = [&](int kk) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            if (BSPLIT) {
                bst[q][0] = wsrc32[((int64_t)kk * NE + s_src[q]) * 2];
                bst[q][1] = wsrc32[((int64_t)kk * NE + s_src[q]) * 2 + 1];
            } else {
                bst[q][0] = wsrc[(int64_t)kk * NE + s_src[q]];
            }
        }
    };
    auto b_store = [&](uint16_t *B) {
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            if (BSPLIT) {
                const Split3 sp = split3(__builtin_bit_cast(f32x4, bst[q][0]), __builtin_bit_cast(f32x4, bst[q][1]));
                if (s_dst[q] < 3 * PLANE) {
                    *reinterpret_cast<u32x4 *>(&B[s_dst[q]]) = sp.h;
                    *reinterpret_cast<u32x4 *>(&B[s_dst[q] + PLANE]) = sp.m;
                    *reinterpret_cast<u32x4 *>(&B[s_dst[q] + 2 * PLANE]) = sp.l;
                }
            } else {
                *reinterpret_cast<u32x4 *>(&B[s_dst[q]]) = bst[q][0];
            }
        }
    };
    Split3 acur[KC];
    {
        b_load(kk0);
        const bool v0 = a_load(kk0);
        b_store(Bs[0]);
        a_finish(v0, acur);
    }
    __syncthreads();
    for (int kk = kk0; kk < kk1; ++kk) {
        const int buf = (kk - kk0) & 1;
        const bool more = kk + 1 < kk1;
        const int kn = more ? kk + 1 : kk;
        b_load(kn);
        const bool v_n = a_load(kn);
        __builtin_amdgcn_sched_barrier(0);
        const uint16_t *bb = &Bs[buf][r * LDB + 8 * h];
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
            bf16x8 bh[NT], bm[NT], bl[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const uint16_t *pb = bb + nt * 32 * LDB + kc * 16;
                bh[nt] = as_bf(*reinterpret_cast<const u32x4 *>(pb));
                bm[nt] = as_bf(*reinterpret_cast<const u32x4 *>(pb + PLANE));
                bl[nt] = as_bf(*reinterpret_cast<const u32x4 *>(pb + 2 * PLANE));
            }
            const bf16x8 ah = as_bf(acur[kc].h), am = as_bf(acur[kc].m), al = as_bf(acur[kc].l);
            // small terms first; the NT accumulator chains interleave
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh[nt], acc[nt], 0, 0, 0);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm[nt], acc[nt], 0, 0, 0);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl[nt], acc[nt], 0, 0, 0);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh[nt], acc[nt], 0, 0, 0);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm[nt], acc[nt], 0, 0, 0);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh[nt], acc[nt], 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
        b_store(Bs[buf ^ 1]);
        __syncthreads();
        a_finish(v_n, acur);
    }

    const int mrow0 = bid.x * 128 + wave * 32;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = nt * 32 + r;
        const float b = EPI == EPI_BIAS_RELU ? a.bias[col] : 0.0f;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int row = mrow0 + acc_row(g, lane);
            if (row >= a.M) continue;
            const int64_t o = (int64_t)row * CN + col;
            if (EPI == EPI_BIAS_RELU) {
                float v = acc[nt][g] + b;
                v = v > 0.0f ? v : 0.0f;
                if (a.out) a.out[o] = v;
                if (a.outb) {
                    uint16_t *pb = a.outb + (int64_t)row * 3 * CN + col;
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) pb[pl * CN] = split_part(v, pl);
                }
            } else if (EPI == EPI_SLAB) {
                a.out[(int64_t)bid.y * a.M * CN + o] = acc[nt][g];
            } else {
                a.out[o] = a.act[o] > 0.0f ? acc[nt][g] : 0.0f;
            }
        }
    }
}

template <int CK, int CN, int KS, int PAD, int MODE, int EPI, bool PRE>
__global__ __launch_bounds__(256) void conv_x6_kernel(ConvPair pr) {
    conv_x6_body<CK, CN, KS, PAD, MODE, EPI, PRE>(pr, blockIdx);
}
template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
__global__ __launch_bounds__(256) void conv_x6_split_kernel(ConvPair pr) {
    conv_x6_body<CK, CN, KS, PAD, MODE, EPI, false, true>(pr, blockIdx);
}

}  // namespace snk

namespace snk {

typedef float f32x4v __attribute__((ext_vector_type(4)));

// conv_x6 with the 16x16x32 bf16 MFMA for pre-split inputs with CK a multiple
// of 32 (conv3). Lane l (r = l&15, g = l>>4) holds A[row r][k = 8g + j] and
// B[k = 8g + j][col r]: one 16-byte A load covers a full 32-channel plane
// segment of 16 rows (64 contiguous bytes per row), so a load instruction
// touches 16 cache lines instead of the 32 of the 32x32x16 layout (the L1 tag
// lookups, not bytes, bounded that kernel). A wave owns 32 rows x CN columns
// (2 x CN/16 tiles of 16x16); C/D: col = l&15, row = 4*(l>>4) + reg.
// B rows in LDS are padded to CK + 16 bf16 (96 B at CK = 32): conflict-free
// for the four ds_read_b128 lane groups.
// WPW waves per workgroup (4: 128 rows)
template <int CK, int CN, int KS, int PAD, int EPI, int WPW>
__global__ __launch_bounds__(64 * WPW) void conv_x6m16_kernel(ConvPair pr) {
    const ConvArgs &a = pr.g[blockIdx.z];
    const uint16_t *__restrict__ wb = pr.wb[blockIdx.z];
    static_assert(CK % 32 == 0 && CN % 16 == 0, "shape");
    constexpr int NCT = CN / 16;                 // 16-column tiles
    constexpr int KC = CK / 32;                  // 32-channel MFMA chunks per offset
    constexpr int LDB = CK + 16;                 // bf16 per LDS row
    constexpr int PLANE = CN * LDB;
    constexpr int NE = 3 * CN * CK / 8;
    constexpr int NT_ = 64 * WPW;
    constexpr int NV = (NE + NT_ - 1) / NT_;
    __shared__ __attribute__((aligned(16))) uint16_t Bs[2][3 * PLANE + 8];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    // the two 16-row tiles of this wave: rows m0 + 16*rt + r
    int srow[2], ii[2], jj[2];
    bool okr[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int m = blockIdx.x * (32 * WPW) + wave * 32 + rt * 16 + r;
        okr[rt] = m < a.M;
        const int mm = okr[rt] ? m : 0;
        const int s = (int)fdiv((uint32_t)mm, a.d2m, a.d2s);
        const int p = mm - s * a.HOUT * a.HOUT;
        jj[rt] = (int)fdiv((uint32_t)p, a.d1m, a.d1s);
        ii[rt] = p - jj[rt] * a.HOUT;
        srow[rt] = s * a.HIN * a.HIN;
    }
    const int kk0 = blockIdx.y * a.kk_per_split;
    const int kk1 = min(a.nkk, kk0 + a.kk_per_split);

    f32x4v acc[2][NCT];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) acc[rt][ct] = f32x4v{0.f, 0.f, 0.f, 0.f};

    const u32x4 *wsrc = reinterpret_cast<const u32x4 *>(wb);
    int s_src[NV], s_dst[NV];
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int e = tid + q * NT_;
        const bool in = (NE % NT_ == 0) || e < NE;
        const int ee = in ? e : 0;
        const int pl = ee / (CN * CK / 8), rem = ee - pl * (CN * CK / 8);
        const int n = rem / (CK / 8), c8 = rem - n * (CK / 8);
        s_src[q] = ee;
        s_dst[q] = in ? pl * PLANE + n * LDB + c8 * 8 : 3 * PLANE;
    }

    u32x4 anx[2][KC][3];
    bool vnx[2];
    auto a_load = [&](int kk) {
        const int dv = kk / KS, du = kk - dv * KS;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
            const int xi = ii[rt] + du - PAD, xj = jj[rt] + dv - PAD;
            const bool v = PAD == 0 ? true : (okr[rt] && xi >= 0 && xi < a.HIN && xj >= 0 && xj < a.HIN);
            const int pos = v ? srow[rt] + xi + xj * a.HIN : 0;
            const uint16_t *pb = a.xb + (int64_t)pos * 3 * CK + 8 * g;
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) anx[rt][kc][pl] = *reinterpret_cast<const u32x4 *>(pb + pl * CK + kc * 32);
            vnx[rt] = v;
        }
    };
    u32x4 acur[2][KC][3];
    auto a_take = [&]() {
        const u32x4 z = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int kc = 0; kc < KC; ++kc)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) acur[rt][kc][pl] = (PAD == 0 || vnx[rt]) ? anx[rt][kc][pl] : z;
    };

    u32x4 bst[NV];
    {
#pragma unroll
        for (int q = 0; q < NV; ++q) bst[q] = wsrc[(int64_t)kk0 * NE + s_src[q]];
        a_load(kk0);
#pragma unroll
        for (int q = 0; q < NV; ++q) *reinterpret_cast<u32x4 *>(&Bs[0][s_dst[q]]) = bst[q];
        a_take();
    }
    __syncthreads();
    for (int kk = kk0; kk < kk1; ++kk) {
        const int buf = (kk - kk0) & 1;
        const bool more = kk + 1 < kk1;
        const int kn = more ? kk + 1 : kk;
#pragma unroll
        for (int q = 0; q < NV; ++q) bst[q] = wsrc[(int64_t)kn * NE + s_src[q]];
        a_load(kn);
        __builtin_amdgcn_sched_barrier(0);
        const uint16_t *bb = &Bs[buf][r * LDB + 8 * g];
#pragma unroll
        for (int kc = 0; kc < KC; ++kc) {
#pragma unroll
            for (int ct = 0; ct < NCT; ++ct) {
                const uint16_t *pb = bb + ct * 16 * LDB + kc * 32;
                const bf16x8 bh = as_bf(*reinterpret_cast<const u32x4 *>(pb));
                const bf16x8 bm = as_bf(*reinterpret_cast<const u32x4 *>(pb + PLANE));
                const bf16x8 bl = as_bf(*reinterpret_cast<const u32x4 *>(pb + 2 * PLANE));
#pragma unroll
                for (int rt = 0; rt < 2; ++rt) {
                    const bf16x8 ah = as_bf(acur[rt][kc][0]), am = as_bf(acur[rt][kc][1]),
                                 al = as_bf(acur[rt][kc][2]);
                    f32x4v c = acc[rt][ct];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
                    acc[rt][ct] = c;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NV; ++q) *reinterpret_cast<u32x4 *>(&Bs[buf ^ 1][s_dst[q]]) = bst[q];
        __syncthreads();
        a_take();
    }

    // epilogue: acc[rt][ct][e] is C[row 4g + e][col r] of tile (rt, ct)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
        const int rbase = blockIdx.x * (32 * WPW) + wave * 32 + rt * 16 + 4 * g;
#pragma unroll
        for (int ct = 0; ct < NCT; ++ct) {
            const int col = ct * 16 + r;
            const float b = EPI == EPI_BIAS_RELU ? a.bias[col] : 0.0f;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = rbase + e;
                if (row >= a.M) continue;
                const int64_t o = (int64_t)row * CN + col;
                if (EPI == EPI_BIAS_RELU) {
                    float v = acc[rt][ct][e] + b;
                    v = v > 0.0f ? v : 0.0f;
                    if (a.out) a.out[o] = v;
                    if (a.outb) {
                        uint16_t *pb = a.outb + (int64_t)row * 3 * CN + col;
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) pb[pl * CN] = split_part(v, pl);
                    }
                } else {   // EPI_SLAB
                    a.out[(int64_t)blockIdx.y * a.M * CN + o] = acc[rt][ct][e];
                }
            }
        }
    }
}

}  // namespace snk

namespace snk {

// conv3 (CK = 32 -> CN = 64, pad 0) of a large batch with the input of FOUR
// samples resident in LDS: the 36 kernel offsets read A from LDS, so L2 moves
// each sample's planes once plus one weight stream per four samples
// (~0.6 GB per 4096-sample launch against the ~2.1 GB x6m16 re-reads).
// Tile rows interleave the samples: row q of a workgroup is output position
// p = q >> 2 of sample q & 3, so the 16 rows of an MFMA tile are 4 positions
// x 4 samples. LDS image of A, in 16-byte slots (8 channels of one plane):
//   slot(s, g, pl, j, i) = s*XS + g*GG + pl*PL + j*XW + i
//   XW = HOUT + 8 (== HOUT mod 4: a row wrap advances the slot by 1 mod 4,
//   like a step inside the row), PL = HIN*XW rounded to 4, GG = 3*PL,
//   XS = 4*GG + 4 (samples 4 slots apart)
// so the 16 lanes of every ds_read_b128 lane group land on 16 distinct slots
// of a 256-byte bank row (bank simulation: 4.3 LDS cycles per read, 4 ideal).
// B (the offset's three weight planes, [pl][n][c]) is double buffered with
// an XOR swizzle of the 16-byte chunk by (n >> 2) & 3 instead of padding.
// 8 waves: wave w owns columns 32*(w & 1) .. +31 and row tiles
// (w >> 1) + 4k. The 6 part products accumulate in x6m16's order: the result
// equals x6m16's bit for bit.
__device__ __forceinline__ int x6s_bswz(int e) { return e ^ ((4 - ((e >> 4) & 3)) & 3); }

template <int KS, int EPI>
__global__ __launch_bounds__(512) void conv_x6s_kernel(ConvPair pr, int S) {
    constexpr int CN = 64, NSG = 4, NB = 3 * CN * 32 / 8;   // 768 B chunks per offset
    const ConvArgs &a = pr.g[blockIdx.z];
    const u32x4 *__restrict__ wsrc = reinterpret_cast<const u32x4 *>(pr.wb[blockIdx.z]);
    extern __shared__ __attribute__((aligned(16))) u32x4 x6s_lds[];
    u32x4 *Bs = x6s_lds;            // [2][NB]
    u32x4 *As = x6s_lds + 2 * NB;   // A image
    const int hin = a.HIN, ho = a.HOUT, ho2 = ho * ho, hin2 = hin * hin;
    const int XW = ho + 8, PL = (hin * XW + 3) & ~3, GG = 3 * PL, XS = 4 * GG + 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int s0 = blockIdx.x * NSG;
    const int ns = min(NSG, S - s0);

    // B register sets: set kk & 1 carries B(kk) from global to LDS
    u32x4 bst[2][2];
    constexpr int NKK = KS * KS;
    auto b_load = [&](int kk, int set) {
        const int kc = min(kk, NKK - 1);
        bst[set][0] = wsrc[(int64_t)kc * NB + tid];
        bst[set][1] = wsrc[(int64_t)kc * NB + 512 + (tid & 255)];
    };
    auto b_store = [&](int buf, int set) {
        Bs[buf * NB + x6s_bswz(tid)] = bst[set][0];
        if (tid < NB - 512) Bs[buf * NB + x6s_bswz(512 + tid)] = bst[set][1];
    };
    b_load(0, 0);
    b_load(1, 1);
    {   // stage the group's planes: global [s][pos][pl][g] -> As
        const u32x4 *src = reinterpret_cast<const u32x4 *>(a.xb) + (int64_t)s0 * hin2 * 12;
        const int n16 = ns * hin2 * 12;
        for (int e0 = 0; e0 < n16; e0 += 14 * 512) {
            u32x4 v[14];   // branch-free (clamped) loads: one round trip for a 12 x 12 group
#pragma unroll
            for (int u = 0; u < 14; ++u) v[u] = src[min(e0 + u * 512 + tid, n16 - 1)];
#pragma unroll
            for (int u = 0; u < 14; ++u) {
                const int e = e0 + u * 512 + tid;
                if (e < n16) {
                    const int pos = e / 12, c = e - pos * 12;
                    const int sr = pos / hin2, qq = pos - sr * hin2;
                    const int j = qq / hin, i = qq - j * hin;
                    As[sr * XS + (c & 3) * GG + (c >> 2) * PL + j * XW + i] = v[u];
                }
            }
        }
    }
    b_store(0, 0);
    b_store(1, 1);

    const int T = (NSG * ho2 + 15) / 16;
    const int rg = wave >> 1, cg = wave & 1;
    // tiles rg, rg+4, ... of this wave (wave-uniform)
    const int nt = __builtin_amdgcn_readfirstlane(T > rg ? (T - rg + 3) / 4 : 0);
    const int bslot = (cg * 32 + r) * 4 + (g ^ ((4 - ((r >> 2) & 3)) & 3));
    __syncthreads();

    // Pipeline: offset kk's MFMAs run on fragments read during offset kk-1.
    // B(kk+1) sits in Bs[(kk+1)&1] (stored at kk-1, before its barrier);
    // B(kk+2), loaded from global one offset earlier, goes into Bs[kk&1]
    // (whose B(kk) every wave read before the last barrier) while B(kk+3)
    // is in flight. Indices past the last offset clamp to it (redundant,
    // harmless loads, reads and stores), so the loop body has no branches
    // and the waitcnt counts stay exact. The tile count per wave is a
    // template constant for the same reason.
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
        struct Frag {
            u32x4 a[NT][3], b[2][3];
        };
        auto frag_read = [&](int kk, Frag &f) {
            kk = min(kk, NKK - 1);
            const int dv = kk / KS, du = kk - dv * KS;
            const int off = dv * XW + du;
            const u32x4 *pb = Bs + (kk & 1) * NB + bslot;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) f.b[ct][pl] = pb[ct * 64 + pl * 256];
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const u32x4 *pa = As + abase[k] + off;
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) f.a[k][pl] = pa[pl * PL];
            }
        };
        auto mfma_block = [&](const Frag &f) {
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const bf16x8 ah = as_bf(f.a[k][0]), am = as_bf(f.a[k][1]), al = as_bf(f.a[k][2]);
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const bf16x8 bh = as_bf(f.b[ct][0]), bm = as_bf(f.b[ct][1]), bl = as_bf(f.b[ct][2]);
                    f32x4v c = acc[k][ct];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
                    acc[k][ct] = c;
                }
            }
        };
        // kk even: B(kk+2) is in set 0, B(kk+3) loads into set 1; kk odd: the reverse
        auto step = [&](int kk, const Frag &cur, Frag &nxt, int set) {
            b_load(kk + 3, set ^ 1);
            frag_read(kk + 1, nxt);
            mfma_block(cur);
            b_store(kk & 1, set);
            __syncthreads();
        };
        Frag f0, f1;
        frag_read(0, f0);
        b_load(2, 0);
        __syncthreads();   // every wave has B(0) in registers before step 0 overwrites Bs[0]
        static_assert(NKK % 2 == 0, "offsets come in pairs");
        for (int kk = 0; kk < NKK; kk += 2) {
            step(kk, f0, f1, 0);
            step(kk + 1, f1, f0, 1);
        }

        // acc[k][ct][e]: tile row 4g + e = position 4t + g of sample e; column 16ct + r
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            const int p = 4 * (rg + 4 * k) + g;
            if (p >= ho2) continue;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = cg * 32 + ct * 16 + r;
                const float bv = EPI == EPI_BIAS_RELU ? a.bias[col] : 0.0f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (e >= ns) continue;
                    const int64_t row = (int64_t)(s0 + e) * ho2 + p;
                    float v = acc[k][ct][e] + bv;
                    v = v > 0.0f ? v : 0.0f;
                    if (a.out) a.out[row * CN + col] = v;
                    if (a.outb) {
                        uint16_t *pb = a.outb + row * 3 * CN + col;
#pragma unroll
                        for (int pl = 0; pl < 3; ++pl) pb[pl * CN] = split_part(v, pl);
                    }
                }
            }
        }
    };
    // every wave passes the same number of barriers whatever its tile count
    if (nt == 4) run(std::integral_constant<int, 4>{});
    else if (nt == 3) run(std::integral_constant<int, 3>{});
    else if (nt == 2) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 1>{});
}

// dynamic LDS bytes of conv_x6s_kernel for an HIN x HIN input (0: does not fit)
static inline size_t conv_x6s_lds(int hin) {
    const int ho = hin - 5, XW = ho + 8, PL = (hin * XW + 3) & ~3, XS = 12 * PL + 4;
    const size_t b = (size_t)(2 * 768 + 4 * XS) * 16;
    return (ho >= 1 && (4 * ho * ho + 15) / 16 <= 16 && b <= 160 * 1024) ? b : 0;
}

}  // namespace snk

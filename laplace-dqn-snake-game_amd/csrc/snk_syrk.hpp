// snk_syrk.hpp — symmetric Gram G = X X^T on the matrix cores.
//
// X is row-major [N][ld] (a row = one snapshot column of the reference's D, or
// one per-sample Jacobian row), reduction over k < K. Only lower-triangle
// 128 x 128 tiles (bj <= bi) are launched; a mirror pass fills the upper
// triangle bit-identically. Three kernels:
//   - syrk_h3q_kernel: the Jacobian Gram (conv sections, and with DENSE the
//     Dense-section terms) on rows pre-split into power-of-two-scaled fp16
//     hi/lo planes, v_mfma_f32_16x16x32_f16, LDS-DMA staging;
//   - syrk_h3_kernel: its round-2 predecessor on v_mfma_f32_32x32x16_f16
//     (measurement build, SNK_SYRK=h3);
//   - syrk_kernel<SYRK_SLAB64>: the snapshot Gram D'D on fp32 rows split in the
//     kernel into three bf16 planes (6 products of v_mfma_f32_32x32x16_bf16),
//     one fp64 slab per split of the reduction.
// The fp32 accumulators are flushed into fp64 every SY_FLUSH stages (1024 k),
// so the error is that of 1024-long fp32 dot products summed in fp64,
// independent of K (K is ~79k for the Jacobian Gram).
#pragma once
#include "snk_conv_h3.hpp"

namespace snk {

constexpr int SY_T = 128, SY_KS = 32, SY_FLUSH = 32;

// lower-triangle tile t -> (bi, bj), bj <= bi
__device__ __forceinline__ void syrk_tile(int64_t t, int &bi, int &bj) {
    int i = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((int64_t)i * (i + 1) / 2 > t) --i;
    while ((int64_t)(i + 1) * (i + 2) / 2 <= t) ++i;
    bi = i;
    bj = (int)(t - (int64_t)i * (i + 1) / 2);
}

// consecutive workgroups land on different XCDs (round robin over 8): give
// each XCD a contiguous run of tiles so the row blocks it streams are shared
// in its own L2
__device__ __forceinline__ int64_t syrk_xcd_remap(int64_t w, int64_t ntiles) {
    const int64_t per = ntiles / 8;
    if (w >= per * 8) return w;
    return (w % 8) * per + w / 8;
}

// A 128 x 128 tile on the bf16 x6 split (snk_conv_x6.hpp): each 32-k stage of
// both 128-row blocks is loaded as fp32 (two float4 per row chunk of 8 k),
// split once into h/m/l bf16 planes while parked in LDS ([op][plane][row][40]:
// 80-byte rows, conflict-free ds_read_b128 for both lane halves), and each
// wave runs 2 k-steps x 2 x 2 tiles x 6 part products of
// v_mfma_f32_32x32x16_bf16: 1536 MFMA cycles per stage against 4096 for the
// 32x32x2 f32 form, with the error class of an fp32 dot product. Double
// buffered (120 KB: the fp64 flush accumulators hold the kernel to one
// workgroup per CU anyway): the next stage is split and parked right after
// this stage's MFMAs, one barrier per stage. Each wave owns a 64 x 64 quarter
// of the tile (2 x 2 MFMA tiles of 32 x 32).
constexpr int SX_LD = 40;
struct SyrkX6Lds {
    uint16_t p[2][2][3][SY_T * SX_LD];   // [buffer][operand][plane]
};

template <bool FLUSH>
__device__ __forceinline__ void syrk_loop_x6(const float *__restrict__ x, int64_t ld, int N, int64_t k0, int64_t k1,
                                             int bi, int bj, SyrkX6Lds &s, f32x16 (&acc)[2][2],
                                             double (&accd)[2][2][16]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
    // staging: rows (tid >> 2) + 64q of each block, k chunk 8*(tid & 3) .. +7
    const int c8 = 8 * (tid & 3);
    const float *pa[2], *pb[2];
    float ma[2], mb[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int ra = bi * SY_T + (tid >> 2) + 64 * q, rb = bj * SY_T + (tid >> 2) + 64 * q;
        pa[q] = x + (int64_t)(ra < N ? ra : N - 1) * ld;
        pb[q] = x + (int64_t)(rb < N ? rb : N - 1) * ld;
        ma[q] = ra < N ? 1.0f : 0.0f;
        mb[q] = rb < N ? 1.0f : 0.0f;
    }
    const int nst = (int)((k1 - k0 + SY_KS - 1) / SY_KS);
    // two register sets: stage st+1 waits parked in one while stage st computes,
    // the loads of stage st+2 go into the other (three sets, with stage st+3 also
    // in flight, spilled the fp64 accumulators to scratch)
    struct Stage {
        f32x4 va[2][2], vb[2][2];
        float km[2];
    };
    Stage rs[2];
    auto issue = [&](int st, Stage &g) __attribute__((always_inline)) {
#pragma unroll
        for (int hf = 0; hf < 2; ++hf) {
            const int64_t k = k0 + (int64_t)st * SY_KS + c8 + 4 * hf;
            const bool v = k < k1;
            const int64_t kk = v ? k : k0;
            g.km[hf] = v ? 1.0f : 0.0f;
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                g.va[q][hf] = *reinterpret_cast<const f32x4 *>(pa[q] + kk);
                g.vb[q][hf] = *reinterpret_cast<const f32x4 *>(pb[q] + kk);
            }
        }
    };
    auto park = [&](int buf, const Stage &g) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int off = ((tid >> 2) + 64 * q) * SX_LD + c8;
            const Split3 sa = split3(g.va[q][0] * (ma[q] * g.km[0]), g.va[q][1] * (ma[q] * g.km[1]));
            const Split3 sb = split3(g.vb[q][0] * (mb[q] * g.km[0]), g.vb[q][1] * (mb[q] * g.km[1]));
            *reinterpret_cast<u32x4 *>(&s.p[buf][0][0][off]) = sa.h;
            *reinterpret_cast<u32x4 *>(&s.p[buf][0][1][off]) = sa.m;
            *reinterpret_cast<u32x4 *>(&s.p[buf][0][2][off]) = sa.l;
            *reinterpret_cast<u32x4 *>(&s.p[buf][1][0][off]) = sb.h;
            *reinterpret_cast<u32x4 *>(&s.p[buf][1][1][off]) = sb.m;
            *reinterpret_cast<u32x4 *>(&s.p[buf][1][2][off]) = sb.l;
        }
    };
    // one quarter of park(): operand op (0: A rows, 1: B rows), row group q
    auto park_piece = [&](int buf, const Stage &g, int op, int q) __attribute__((always_inline)) {
        const int off = ((tid >> 2) + 64 * q) * SX_LD + c8;
        const float m = op == 0 ? ma[q] : mb[q];
        const f32x4 *v = op == 0 ? g.va[q] : g.vb[q];
        const Split3 sp = split3(v[0] * (m * g.km[0]), v[1] * (m * g.km[1]));
        *reinterpret_cast<u32x4 *>(&s.p[buf][op][0][off]) = sp.h;
        *reinterpret_cast<u32x4 *>(&s.p[buf][op][1][off]) = sp.m;
        *reinterpret_cast<u32x4 *>(&s.p[buf][op][2][off]) = sp.l;
    };
    // the MFMAs of one stage with the park of the next woven in (source order)
    auto compute_park = [&](int buf, bool pk, const Stage &nx) __attribute__((always_inline)) {
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 fa[2][3], fb[2][3];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    fa[i][pl] = as_bf(*reinterpret_cast<const u32x4 *>(
                        &s.p[buf][0][pl][(wr + 32 * i + r) * SX_LD + 16 * ks + 8 * h]));
                    fb[i][pl] = as_bf(*reinterpret_cast<const u32x4 *>(
                        &s.p[buf][1][pl][(wc + 32 * i + r) * SX_LD + 16 * ks + 8 * h]));
                }
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni) {
                    f32x16 c = acc[mi][ni];
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][2], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][1], fb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][0], fb[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][1], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][0], fb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[mi][0], fb[ni][0], c, 0, 0, 0);
                    acc[mi][ni] = c;
                    if (ks == 1 && pk) park_piece(buf ^ 1, nx, mi, ni);
                }
        }
    };
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    accd[mi][ni][g] += (double)acc[mi][ni][g];
                    acc[mi][ni][g] = 0.0f;
                }
    };
    // stage st: the loads of st+2 go out into set st % 2 (whose stage st was
    // parked at st-1), stage st+1 (set (st+1) % 2) is parked after the MFMAs.
    // Stage indices past the end clamp (the loads are masked by km and unused).
    // BUF = st & 1 is a template constant (the loop is unrolled by 2), so the
    // compiler sees that the park's LDS stores and this stage's fragment
    // reads touch different buffers; the split VALU work and the stores are
    // woven between the MFMAs in source order to fill their issue slots
    // (one wave per SIMD: nothing else would hide them).
    auto step = [&](int st, auto bufc, Stage &ld2, Stage &nx) __attribute__((always_inline)) {
        constexpr int BUF = decltype(bufc)::value;
        const bool more = st + 1 < nst;
        issue(st + 2 < nst ? st + 2 : nst - 1, ld2);
        __builtin_amdgcn_sched_barrier(0);
        // park of stage st+1 into the other buffer (last read in stage st-1,
        // before the barrier), woven between the second k-step's MFMAs
        compute_park(BUF, more, nx);
        if (FLUSH && (st % SY_FLUSH == SY_FLUSH - 1 || !more)) flush();
        __syncthreads();
    };
    using B0 = std::integral_constant<int, 0>;
    using B1 = std::integral_constant<int, 1>;
    issue(0, rs[0]);
    if (nst > 1) issue(1, rs[1]);
    park(0, rs[0]);
    __syncthreads();
    int st = 0;
    for (; st + 2 <= nst; st += 2) {
        step(st, B0{}, rs[0], rs[1]);
        step(st + 1, B1{}, rs[1], rs[0]);
    }
    if (st < nst) step(st, B0{}, rs[0], rs[1]);
}

__device__ __forceinline__ void syrk_zero(f32x16 (&acc)[2][2]) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[mi][ni][g] = 0.0f;
}

enum SyrkOut { SYRK_F32 = 0, SYRK_SLAB64 = 1 };

struct SyrkArgs {
    const float *x;
    int64_t ld, K, kchunk;   // reduction range of split z: [z*kchunk, min(K, (z+1)*kchunk))
    int N;
    int64_t ntiles;          // tiles of this launch: [t0, t0 + ntiles) of the order
    int64_t t0;
    const int2 *tiles;       // optional tile order (bi, bj), indexed by the XCD remap; null: row-major
    int direct;              // tiles[t0 + blockIdx.x] as is (the table already interleaves the XCDs)
    uint64_t *stamps;        // measurement builds (SNK_SYRK_MEASURE): per workgroup s_memtime /
                             // s_memrealtime at start and end, 4 words
    float *g32;              // SYRK_F32 (h3q): G [N][ldg]
    double *g64;             // SYRK_SLAB64: slab [z][N][N]
    int64_t ldg;
    const uint8_t *act;      // DENSE h3q: replay actions of the N samples
    // syrk_h3_kernel: x pre-split by h3_rows_kernel into xh [N][ldh/32][2][32] fp16
    // (per row and 32-k stage: the h part, then the l part: one 128-byte line;
    // ldh a multiple of SY_KS, zero tail), row i scaled by 2^xe[i]
    const uint16_t *xh, *xl;
    const int32_t *xe;
    int64_t ldh;
    // syrk_h3q_kernel<.., DENSE = true>: xh holds three h3 segments per row,
    // a3 (stages [0, s1)), dz1 ([s1, s2)), h1 ([s2, ldh/32)), each with its own
    // row exponent xe[seg * xes + row] (h3_seg_rows_kernel)
    int s1, s2;
    int64_t xes;
    int dstore;              // DENSE: store the terms into G (syrk_ksum_kernel adds the conv Gram) instead of adding
};

// h3 operands for the Gram (snk_conv_h3.hpp's split, one scale per ROW):
// row i of x [N][ld] -> fp16 parts h, l of x * 2^e_i with e_i = h3_exp(max_k |x_ik|),
// zero-padded to ldh, stored per 32-k stage as [h 32][l 32] (one 128-byte line,
// so a stage fetch uses whole lines). One workgroup per row: the max pass,
// then the split pass (the row is L2-resident by then).
// G_ij = 2^-(e_i + e_j) (Xs Xs')_ij exactly.
static __global__ __launch_bounds__(256) void h3_rows_kernel(const float *__restrict__ x, int64_t ld, int64_t K,
                                                      uint16_t *__restrict__ xhl, int32_t *__restrict__ xe,
                                                      int64_t ldh) {
    __shared__ float red4[4];
    const int64_t row = blockIdx.x;
    const f32x4 *src = reinterpret_cast<const f32x4 *>(x + row * ld);
    const int64_t n4 = K / 4, nh4 = ldh / 4;
    float m = 0.0f;
    for (int64_t i = threadIdx.x; i < n4; i += 256) {
        const f32x4 v = src[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
    const int e = h3_exp(fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3])));
    if (threadIdx.x == 0) xe[row] = e;
    u32x2 *o = reinterpret_cast<u32x2 *>(xhl + row * 2 * ldh);   // 4 halves per u32x2
    for (int64_t i = threadIdx.x; i < nh4; i += 256) {
        const f32x4 v = i < n4 ? src[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        u32x2 h, l;
        h3_split4(v, e, h, l);
        const int64_t q = (i >> 3) * 16 + (i & 7);   // stage i / 8, 4-half piece i % 8
        o[q] = h;
        o[q + 8] = l;
    }
}

// The Dense-section operands of the Jacobian Gram, pre-split like h3_rows_kernel
// but one wave per (row, segment): segment g of row i is x_g[i][0, K_g) (K_g a
// multiple of 4), zero-padded to nst_g stages, stored at stage offset st_g of the row's plane line
// (row stride 2 * ldh halves), scaled by 2^xe[g * xes + i]. Rows n <= i < npad
// are zero.
struct H3Segs {
    const float *x[3];
    int64_t ld[3], K[3], st[3], nst[3];
};
static __global__ __launch_bounds__(256) void h3_seg_rows_kernel(H3Segs sg, int64_t n, int64_t npad, uint16_t *__restrict__ xhl,
                                                          int32_t *__restrict__ xe, int64_t xes, int64_t ldh) {
    const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int seg = blockIdx.y, lane = threadIdx.x & 63;
    if (row >= npad) return;
    const int64_t n4 = sg.K[seg] / 4, np4 = sg.nst[seg] * (SY_KS / 4);
    const bool live = row < n;
    const f32x4 *src = reinterpret_cast<const f32x4 *>(sg.x[seg] + (live ? row : 0) * sg.ld[seg]);
    float m = 0.0f;
    for (int64_t i = lane; i < n4 && live; i += 64) {
        const f32x4 v = src[i];
        m = fmaxf(m, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
    const int e = h3_exp(wave_max(m));
    if (lane == 0 && live) xe[seg * xes + row] = e;
    u32x2 *o = reinterpret_cast<u32x2 *>(xhl + row * 2 * ldh + sg.st[seg] * 2 * SY_KS);
    for (int64_t i = lane; i < np4; i += 64) {
        const f32x4 v = live && i < n4 ? src[i] : f32x4{0.f, 0.f, 0.f, 0.f};
        u32x2 h, l;
        h3_split4(v, e, h, l);
        const int64_t q = (i >> 3) * 16 + (i & 7);
        o[q] = h;
        o[q + 8] = l;
    }
}

// The production h3 Gram kernel: 8 waves (two per SIMD) on a 128 x 128
// lower-triangle tile, each wave a 64 x 32 quarter-half (2 x 1 tiles of
// 32 x 32; fp64 flush accumulators 32 doubles, so two waves fit a SIMD), the
// stages moved global -> LDS by LDS-DMA (global_load_lds_dwordx4: no VGPR
// staging, no ds_write), four stage buffers [op][plane][128][32 halves]
// (128 KB) with the 16-byte chunk of row r stored at slot chunk ^ ((r>>2)&3)
// (the swizzle is applied on the global source address: the DMA destination
// is lane-linear; the fragment ds_read_b128 lane groups then hit 16 distinct
// bank quads). Per step: DMA of stage st+3, k-step-1 fragments of st, the
// k-step-0 MFMAs, a counted vmcnt (stage st+1 landed; st+2, st+3 stay in
// flight) and a raw s_barrier, k-step-0 fragments of st+1, the k-step-1
// MFMAs. Rows past N read row N-1 (never stored); the zero tail of ldh
// covers the k range.
constexpr int SH_BUF = 4, SH_ROW = 32;   // halves per LDS row (one 32-k stage)

// NW waves: 8 (two per SIMD, 64 x 32 per wave) or 4 (one per SIMD, 64 x 64 per wave:
// half the fragment reads per MFMA)
// VAR (measurement builds selected by SNK_SYRK_VAR): 0 the kernel, 1 no MFMA (the
// fragments feed one VALU op each: data movement + LDS reads + barriers alone),
// 2 no stage DMA after the prologue (MFMAs + fragment reads + barriers alone),
// 3 (syrk_h3q_kernel) the B operand's stages not reloaded: half the DMA stream, as a tile
// twice as wide would have per FLOP
template <int NW, int VAR = 0>
__global__ __launch_bounds__(64 * NW) void syrk_h3_kernel(SyrkArgs a) {
    constexpr int NC = NW == 4 ? 2 : 1, NJ = 32 / NW;   // column tiles per wave, DMA jobs per wave and stage
    __shared__ __attribute__((aligned(16))) uint16_t lds[SH_BUF * 2 * 2 * SY_T * SH_ROW];   // 128 KB
    int bi, bj;
    {
        const int64_t t = a.t0 + (a.direct ? (int64_t)blockIdx.x : syrk_xcd_remap(blockIdx.x, a.ntiles));
        if (a.tiles) {
            const int2 tb = a.tiles[t];
            bi = tb.x;
            bj = tb.y;
        } else {
            syrk_tile(t, bi, bj);
        }
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wr = (wave / (NW / 2)) * 64, wc = (wave % (NW / 2)) * 32 * NC;
    const int N = a.N;
    const int nst = (int)(a.ldh / SY_KS);

    // this wave's NJ DMA jobs per stage: j = NJ * wave + q -> op = j >> 4, plane = (j >> 3) & 1, row block j & 7
    const uint16_t *dsrc[NJ];
    int ddst[NJ];   // LDS offset (halves) inside a stage buffer
#pragma unroll
    for (int q = 0; q < NJ; ++q) {
        const int j = NJ * wave + q, op = j >> 4, pl = (j >> 3) & 1, rb = j & 7;
        const int row = rb * 16 + (lane >> 2);
        const int chunk = (lane & 3) ^ ((row >> 2) & 3);
        const int grow = (op ? bj : bi) * SY_T + row;
        dsrc[q] = a.xh + (int64_t)(grow < N ? grow : N - 1) * 2 * a.ldh + pl * SY_KS + chunk * 8;
        ddst[q] = ((op * 2 + pl) * SY_T + rb * 16) * SH_ROW;
    }
    auto dma = [&](int st, int buf) {
        if (VAR == 2 && st > 2) return;
        const int64_t k = (int64_t)min(st, nst - 1) * 2 * SY_KS;   // past the end: harmless reloads
#pragma unroll
        for (int q = 0; q < NJ; ++q)
            __builtin_amdgcn_global_load_lds((const void *)(dsrc[q] + k),
                                             (__attribute__((address_space(3))) void *)(lds + buf * (4 * SY_T * SH_ROW) + ddst[q]),
                                             16, 0, 0);
    };
    struct Frag {
        f16x8 a[2][2], b[NC][2];   // [tile][plane]
    };
    auto frag = [&](int buf, int ks, Frag &f) {
        const uint16_t *base = lds + buf * (4 * SY_T * SH_ROW);
        const int c = 2 * ks + h;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn) {
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = wr + 32 * i + r;
                f.a[i][pn] = as_h(*reinterpret_cast<const u32x4 *>(
                    base + ((0 * 2 + pn) * SY_T + row) * SH_ROW + 8 * (c ^ ((row >> 2) & 3))));
            }
#pragma unroll
            for (int j = 0; j < NC; ++j) {
                const int row = wc + 32 * j + r;
                f.b[j][pn] = as_h(*reinterpret_cast<const u32x4 *>(
                    base + ((1 * 2 + pn) * SY_T + row) * SH_ROW + 8 * (c ^ ((row >> 2) & 3))));
            }
        }
    };
    f32x16 acc[2][NC];
    double accd[2][NC][16];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                acc[i][j][g] = 0.0f;
                accd[i][j][g] = 0.0;
            }
    // the six MFMAs of one k-step, split after the first: the next fragments'
    // ds_reads go out between the two parts (see step)
    auto mfma_first = [&](const Frag &f) {
        if (VAR == 1) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NC; ++j)
                    acc[i][j][0] += (float)(f.a[i][0][0] * f.b[j][0][0]) + (float)(f.a[i][1][1] * f.b[j][1][1]);
            return;
        }
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[0][1], f.b[0][0], acc[0][0], 0, 0, 0);
    };
    auto mfma_rest = [&](const Frag &f) {
        if (VAR == 1) return;
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                if (mi == 0 && j == 0) continue;
                acc[mi][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[mi][1], f.b[j][0], acc[mi][j], 0, 0, 0);
            }
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                acc[mi][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[mi][0], f.b[j][1], acc[mi][j], 0, 0, 0);
#pragma unroll
        for (int j = 0; j < NC; ++j)
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
                acc[mi][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.a[mi][0], f.b[j][0], acc[mi][j], 0, 0, 0);
    };
    auto flush = [&]() {
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int j = 0; j < NC; ++j)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    accd[mi][j][g] += (double)acc[mi][j][g];
                    acc[mi][j][g] = 0.0f;
                }
    };
    // prologue: stages 0, 1, 2 in flight; stage 0 landed everywhere
    dma(0, 0);
    dma(1, 1);
    dma(2, 2);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NJ));
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) (vmcnt 63, expcnt 7)
    __builtin_amdgcn_s_barrier();
    Frag f0, f1;
    frag(0, 0, f0);
    // ROCm 7.2's waitcnt pass drains lgkmcnt to 0 before the first MFMA of a
    // k-step whatever is in flight, so the next fragments are read AFTER that
    // first MFMA (they then overlap the remaining five and the other wave's)
    auto step = [&](int st, auto bc) {
        constexpr int B = decltype(bc)::value;   // st % 4
        mfma_first(f0);
        __builtin_amdgcn_sched_barrier(0);
        frag(B, 1, f1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rest(f0);
        __builtin_amdgcn_sched_barrier(0);
        dma(st + 3, (B + 3) & 3);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * NJ));   // my part of stage st+1 landed
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        mfma_first(f1);
        __builtin_amdgcn_sched_barrier(0);
        frag((B + 1) & 3, 0, f0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_rest(f1);
        __builtin_amdgcn_sched_barrier(0);
        if (st % SY_FLUSH == SY_FLUSH - 1) flush();
    };
    int st = 0;
    for (; st + 4 <= nst; st += 4) {
        step(st, std::integral_constant<int, 0>{});
        step(st + 1, std::integral_constant<int, 1>{});
        step(st + 2, std::integral_constant<int, 2>{});
        step(st + 3, std::integral_constant<int, 3>{});
    }
    if (st < nst) step(st, std::integral_constant<int, 0>{});
    if (st + 1 < nst) step(st + 1, std::integral_constant<int, 1>{});
    if (st + 2 < nst) step(st + 2, std::integral_constant<int, 2>{});
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // drain the clamped tail DMAs before the workgroup ends
    flush();
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
            const int col = bj * SY_T + wc + 32 * j + r;
            if (col >= N) continue;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int row = bi * SY_T + wr + mi * 32 + acc_row(g, lane);
                if (row >= N) continue;
                a.g32[(int64_t)row * a.ldg + col] = (float)__builtin_ldexp(accd[mi][j][g], -(a.xe[row] + a.xe[col]));
            }
        }
}

// syrk_h3q_kernel: syrk_h3_kernel's tile, waves, stages and LDS-DMA ring on
// v_mfma_f32_16x16x32_f16 (one MFMA per 32-k stage and 16 x 16 tile; at equal
// cycles per FLOP the 16 x 16 shape holds a higher clock under load,
// MI355X_MICROARCH.md 'DVFS give-back' (7)). Wave w owns rows 64 (w / 4) ..
// +63 and columns 32 (w % 4) .. +31: 4 x 2 tiles of 16 x 16, the same LDS bytes
// per wave as the 32 x 32 form. A fragment is a 16-row x 32-k slice: lane l
// reads row (l & 15), 16-byte chunk (l >> 4) of the stage. The chunk of row r is
// stored at slot chunk ^ swz(r), swz(r) = (-(r >> 2)) & 3, which puts every
// ds_read_b128 lane group of that pattern on 16 distinct bank quads.
// Per step: see `step` below (row tiles 2-3 of a stage are read during the
// MFMAs of tiles 0-1, the next stage's tiles 0-1 and B during those of 2-3).
__device__ __forceinline__ int syrk_swz16(int row) { return (-(row >> 2)) & 3; }

// NB stage buffers (32 KB each): NB - 1 stages in flight
// DENSE: the Dense-section terms of the Jacobian Gram over the three segments
// of h3_seg_rows_kernel, added into G (lower-triangle tiles):
//   G_ij += (a3_i.a3_j + 1)(dz1_i.dz1_j) + [act_i == act_j](h1_i.h1_j + 1)
// (the Dense1 weight+bias and Dense2 weight+bias Jacobian blocks; the fp32
// accumulators are folded at the segment ends, hook_a / hook_z below; the
// a3 segment (K1 = 576 at 12x12) accumulates in fp32 like one flush interval of
// the conv Gram)
// SB: stages per barrier. 1: one barrier per 32-k stage, stage st + NB - 1 issued at step st;
// 2 (NB = 4): the stages go in pairs, one barrier per pair, the next pair's two stages issued
// right after the barrier that freed their buffers (the same 2-stage lead).
template <int VAR = 0, int NB = 4, bool DENSE = false, int SB = 1>
__global__ __launch_bounds__(512) void syrk_h3q_kernel(SyrkArgs a) {
    static_assert(SB == 1 || (SB == 2 && NB == 4), "stage pairs need four buffers");
    constexpr int NJ = 4;   // DMA jobs per wave and stage (32 KB / 8 waves / 1 KB)
    __shared__ __attribute__((aligned(16))) uint16_t lds[NB * 2 * 2 * SY_T * SH_ROW];
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    int bi, bj;
    {
        const int64_t t = a.t0 + (a.direct ? (int64_t)blockIdx.x : syrk_xcd_remap(blockIdx.x, a.ntiles));
        if (a.tiles) {
            const int2 tb = a.tiles[t];
            bi = tb.x;
            bj = tb.y;
        } else {
            syrk_tile(t, bi, bj);
        }
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int wr = (wave >> 2) * 64, wc = (wave & 3) * 32;
    const int N = a.N;
    const int nst = (int)(a.ldh / SY_KS);
    // this wave's NJ DMA jobs per stage: j = NJ * wave + q -> operand j >> 4, plane
    // (j >> 3) & 1, 16-row block j & 7; operand and plane are the wave's, the row
    // blocks consecutive, and the swizzle of row 16 rb + (lane >> 2) does not depend
    // on rb: one source pointer per lane. Rows past N exist (the planes are zero-padded
    // to whole SW_ROWS_B blocks) and are never stored.
    const uint16_t *dsrc;
    int ddst;
    {
        const int j = NJ * wave, op = j >> 4, pl = (j >> 3) & 1, rb = j & 7;
        const int row = rb * 16 + (lane >> 2);
        const int chunk = (lane & 3) ^ syrk_swz16(row);
        dsrc = a.xh + (int64_t)((op ? bj : bi) * SY_T + row) * 2 * a.ldh + pl * SY_KS + chunk * 8;
        ddst = ((op * 2 + pl) * SY_T + rb * 16) * SH_ROW;
    }
    const int64_t qstride = 16 * 2 * a.ldh;
    auto dma_job = [&](int st, int buf, int q) __attribute__((always_inline)) {
        if (VAR == 2 && st > NB - 2) return;
        if (VAR == 3 && st > NB - 2 && wave >= 4) return;   // B (waves 4-7) loaded once: half the stream
        const int64_t k = (int64_t)min(st, nst - 1) * 2 * SY_KS;
        __builtin_amdgcn_global_load_lds((const void *)(dsrc + k + q * qstride),
                                         (__attribute__((address_space(3))) void *)(lds + buf * (4 * SY_T * SH_ROW) + ddst +
                                                                                   q * 16 * SH_ROW),
                                         16, 0, 0);
    };
    auto dma = [&](int st, int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int q = 0; q < NJ; ++q) dma_job(st, buf, q);
    };
    // fragments: A row tiles 0-1 (lo) and 2-3 (hi), B column tiles 0-1 twice (this
    // stage's and the next's): [tile][plane]
    typedef f16x8 FA[2][2];
    typedef f16x8 FB[2][2];
    auto frag_a = [&](int buf, int t0, FA &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * (4 * SY_T * SH_ROW);
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = wr + 16 * (t0 + i) + r;
                f[i][pn] = as_h(*reinterpret_cast<const u32x4 *>(
                    base + ((0 * 2 + pn) * SY_T + row) * SH_ROW + 8 * (g ^ syrk_swz16(row))));
            }
    };
    auto frag_b = [&](int buf, FB &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * (4 * SY_T * SH_ROW);
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = wc + 16 * j + r;
                f[j][pn] = as_h(*reinterpret_cast<const u32x4 *>(
                    base + ((1 * 2 + pn) * SY_T + row) * SH_ROW + 8 * (g ^ syrk_swz16(row))));
            }
    };
    f32x4 acc[4][2];
    double accd[4][2][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc[i][j][e] = 0.0f;
                accd[i][j][e] = 0.0;
            }
    // half of a stage's 24 MFMAs: row tiles t0, t0+1 x both column tiles; per
    // tile pair l*h, h*l, then h*h (small products first)
    // part 0: only the first MFMA (tile t0 x column 0, l*h); part 1: the other 11;
    // part 2: all 12
    auto mfma_half = [&](const FA &fa, const FB &fb, int t0, int part) __attribute__((always_inline)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int i = t0 + ii;
                const bool first = ii == 0 && j == 0;
                if (VAR == 1) {
                    if (part != 0 && (part == 2 || !first))
                        acc[i][j][0] += (float)(fa[ii][0][0] * fb[j][0][0]) + (float)(fa[ii][1][1] * fb[j][1][1]);
                    continue;
                }
                if (part == 2 || (part == 0) == first)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][1], fb[j][0], acc[i][j], 0, 0, 0);
                if (part != 0) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[j][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[j][0], acc[i][j], 0, 0, 0);
                }
            }
    };
    auto flush = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    accd[i][j][e] += (double)acc[i][j][e];
                    acc[i][j][e] = 0.0f;
                }
    };
    // DENSE segment ends: the exponents of the tile's rows and columns per segment,
    // staged in LDS before the prologue barrier ([seg][128 rows | 128 columns],
    // clamped to N - 1: rows past N are never stored). Read at the hooks, so no
    // addresses stay live across the stage loop.
    __shared__ __attribute__((aligned(16))) int ex_s[DENSE ? 3 * 2 * SY_T : 4];
    if constexpr (DENSE) {
        for (int t = tid; t < 3 * 2 * SY_T; t += 512) {
            const int seg = t / (2 * SY_T), k = t % (2 * SY_T);
            const int idx = k < SY_T ? bi * SY_T + k : bj * SY_T + k - SY_T;
            ex_s[t] = a.xe[seg * a.xes + min(idx, N - 1)];
        }
    }
    auto rowe = [&](int seg, int i, int e) __attribute__((always_inline)) {
        return ex_s[seg * 2 * SY_T + wr + 16 * i + 4 * g + e];
    };
    auto cole = [&](int seg, int j) __attribute__((always_inline)) {
        return ex_s[seg * 2 * SY_T + SY_T + wc + 16 * j + r];
    };
    // DENSE keeps fp32 partial terms instead of the fp64 flush accumulators (each
    // segment is at most a few hundred k long; G is fp32): after the a3 segment
    // pd = a3_i.a3_j + 1, after the dz1 segment pd *= dz1_i.dz1_j
    float pd[4][2][4];
    auto hook_a = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ec = cole(0, j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    pd[i][j][e] = __builtin_ldexpf(acc[i][j][e], -(rowe(0, i, e) + ec)) + 1.0f;
                    acc[i][j][e] = 0.0f;
                }
        }
    };
    auto hook_z = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int ec = cole(1, j);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    pd[i][j][e] *= __builtin_ldexpf(acc[i][j][e], -(rowe(1, i, e) + ec));
                    acc[i][j][e] = 0.0f;
                }
        }
    };
#pragma unroll
    for (int q = 0; q < (SB == 1 ? NB - 1 : 2); ++q) dma(q, q);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(SB == 1 ? (NB - 2) * NJ : 0));
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    FA lo, hi;
    FB b0, b1;
    frag_a(0, 0, lo);
    frag_b(0, b0);
    // step st (buffer B = st % NB; lo / bc hold stage st's row tiles 0-1 and B):
    // read stage st's row tiles 2-3, MFMAs of tiles 0-1, DMA of stage st+NB-1 (into
    // the buffer of stage st-1, whose last readers passed step st-1's barrier),
    // wait for stage st+1 and the barrier, read stage st+1's tiles 0-1 and B
    // (lo is free now), MFMAs of tiles 2-3
    auto step = [&](int st, auto bc_, FB &bc, FB &bn) __attribute__((always_inline)) {
        constexpr int B = decltype(bc_)::value;
        // the compiler's waitcnt pass drains lgkmcnt to 0 before the first MFMA of
        // the step: issue the row-tile 2-3 reads after it
        mfma_half(lo, bc, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        frag_a(B, 2, hi);
        __builtin_amdgcn_sched_barrier(0);
        mfma_half(lo, bc, 0, 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (SB == 1) {
            dma(st + NB - 1, (B + NB - 1) % NB);
            __builtin_amdgcn_s_waitcnt(waitcnt_vm((NB - 2) * NJ));   // my part of stage st+1 landed
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
        } else if constexpr (B % 2 == 0) {   // pair start: the next pair into the previous pair's buffers
            dma(st + 2, (B + 2) % NB);
            dma(st + 3, (B + 3) % NB);
        } else {                              // pair end: the next pair landed, this pair's reads done
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
            __builtin_amdgcn_s_waitcnt(0xC07F);
            __builtin_amdgcn_s_barrier();
        }
        __builtin_amdgcn_sched_barrier(0);
        frag_a((B + 1) % NB, 0, lo);
        frag_b((B + 1) % NB, bn);
        __builtin_amdgcn_sched_barrier(0);
        mfma_half(hi, bc, 2, 2);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (DENSE) {
            if (st == a.s1 - 1) hook_a();
            else if (st == a.s2 - 1) hook_z();
        } else if (st % SY_FLUSH == SY_FLUSH - 1) {
            flush();
        }
    };
    // U = lcm(NB, 2) steps per loop trip: buffer and B-fragment roles are constants
    constexpr int U = NB % 2 ? 2 * NB : NB;
    auto one = [&](int st0, bool tail, auto ic) __attribute__((always_inline)) {
        constexpr int I = decltype(ic)::value;
        if (!tail || st0 + I < nst)
            step(st0 + I, std::integral_constant<int, I % NB>{}, I % 2 ? b1 : b0, I % 2 ? b0 : b1);
    };
    auto trip = [&](int st0, bool tail) __attribute__((always_inline)) {
        static_assert(U <= 10, "unrolled trip");
        one(st0, tail, std::integral_constant<int, 0>{});
        one(st0, tail, std::integral_constant<int, 1>{});
        if constexpr (U > 2) {
            one(st0, tail, std::integral_constant<int, 2>{});
            one(st0, tail, std::integral_constant<int, 3>{});
        }
        if constexpr (U > 4) {
            one(st0, tail, std::integral_constant<int, 4>{});
            one(st0, tail, std::integral_constant<int, 5>{});
        }
        if constexpr (U > 6) {
            one(st0, tail, std::integral_constant<int, 6>{});
            one(st0, tail, std::integral_constant<int, 7>{});
        }
        if constexpr (U > 8) {
            one(st0, tail, std::integral_constant<int, 8>{});
            one(st0, tail, std::integral_constant<int, 9>{});
        }
    };
    int st = 0;
    for (; st + U <= nst; st += U) trip(st, false);
    if (st < nst) trip(st, true);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    if constexpr (DENSE) {   // the h1 segment: + [act_i == act_j](h1_i.h1_j + 1)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = bj * SY_T + wc + 16 * j + r;
            if (col >= N) continue;
            const int ec = cole(2, j);
            const uint8_t ac = a.act[col];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = bi * SY_T + wr + 16 * i + 4 * g + e;
                    if (row >= N) continue;
                    double v = (double)pd[i][j][e];
                    if (a.act[row] == ac) v += (double)__builtin_ldexpf(acc[i][j][e], -(rowe(2, i, e) + ec)) + 1.0;
                    float *o = a.g32 + (int64_t)row * a.ldg + col;
                    *o = a.dstore ? (float)v : (float)((double)*o + v);
                }
        }
        return;
    }
    flush();
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = bj * SY_T + wc + 16 * j + r;
            if (col >= N) continue;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = bi * SY_T + wr + 16 * i + 4 * g + e;
                if (row >= N) continue;
                a.g32[(int64_t)row * a.ldg + col] = (float)__builtin_ldexp(accd[i][j][e], -(a.xe[row] + a.xe[col]));
            }
        }
}

// ---------------------------------------------------------------------------
// syrk_h3k_kernel (round 6, the production conv-column Gram): 256 x 256
// lower-triangle tiles with the reduction split into chunks of cs stages.
//
// Why: the 128 x 128 kernel above is bound by its stage stream (32 KB of
// L2 -> LDS bytes per 192 MFMAs; without its MFMAs it runs as long as with
// them), and its fp64 flush accumulators (64 registers) are what
// kept a bigger tile from fitting two waves per SIMD. A 256 x 256 tile moves
// 64 KB per 768 MFMAs (half the bytes per MFMA) and each wave's 128 x 64 block
// reads a quarter KB of fragments per MFMA (half again). Accumulating in fp32
// only, a chunk of cs stages is a cs-long fp32 dot product; the chunks' fp32
// partial tiles go to `part` and syrk_ksum_kernel sums them in fp64, so the
// error is that of cs-stage fp32 sums added in fp64 (chunks of 320 stages:
// ~1/8 of a one-chunk fp32 sum's error).
//
// Workgroup = (tile, chunk) from the host-built item table (I, J, z, local tile);
// 8 waves, wave w owns rows 128 (w >> 2) .. +127 and columns 64 (w & 3) .. +63
// of the tile: 8 x 4 MFMA tiles of 16 x 16 (128 fp32 accumulators). Two stage
// buffers [operand][plane][256 rows][32 halves] (64 KB each, the 16-byte chunk of
// row r at slot chunk ^ syrk_swz16(r), lane-linear LDS-DMA destinations as in
// syrk_h3q_kernel: 8 pieces of 16 rows x 64 B per wave and stage). Per step the
// four row-tile pairs' MFMAs run in groups of 24 with the next pair's fragments
// read under them; before the last group every wave has its fragments in
// registers, so the barrier that certifies stage st+1 also frees stage st's
// buffer for the DMA of st+2 (one barrier per stage, one stage in flight).
// The partial tile is stored in the accumulators' own order (one 1 KB
// dwordx4 store per MFMA tile): part[((z * ntl + tile) * 8 + wave) * 8192 +
// (4 i + j) * 256 + 4 lane + e].
constexpr int SK_T = 256;                           // tile side
constexpr int SK_STG = 2 * 2 * SK_T * SH_ROW;       // halves per stage buffer (64 KB)
constexpr int SK_SUB = 128 * 64;                    // floats of one wave's block
constexpr int SK_CHUNK = 160;                       // stages per chunk (5,120 k)

struct SyrkKArgs {
    const uint16_t *xh;     // h3 row planes [npad][ldh / 32][2][32] (h3_rows_kernel), npad % 256 == 0
    int64_t ldh;
    int nst;                // stages of the whole reduction (ldh / 32)
    int cs;                 // stages per chunk: chunk z = stages [z cs, min(nst, (z + 1) cs))
    const int4 *items;      // per workgroup: (I, J, z, local tile)
    float *part;            // partial tiles (layout above)
    int64_t ntl;            // tiles of this launch
    uint64_t *stamps;       // measurement builds (SNK_SYRK_MEASURE): 4 words per workgroup
};

__global__ __launch_bounds__(512) void syrk_h3k_kernel(SyrkKArgs a) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[2 * SK_STG];   // 128 KB
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    const int4 it = a.items[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int wr = (wave >> 2) * 128, wc = (wave & 3) * 64;
    const int s0 = it.z * a.cs, nst = min(a.nst - s0, a.cs);
    // DMA: wave w moves operand w >> 2, plane (w >> 1) & 1, rows 128 (w & 1) .. +127 as 8
    // pieces of 16 rows, through one buffer descriptor on its operand's 256-row panel: the
    // lane's part of the source (row 128 (w & 1) + (lane >> 2) of the piece and its swizzled
    // chunk; the swizzle does not depend on the piece) is one 32-bit offset, the piece and
    // stage part a scalar offset, so no 64-bit address per piece stays live across the loop
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const int op = wv >> 2, pl = (wv >> 1) & 1;
    const uint32_t rowb = (uint32_t)(2 * a.ldh * 2);   // bytes per plane row
    const int drow = 128 * (wv & 1) + (lane >> 2);
    const uint32_t voff = (uint32_t)drow * rowb + (uint32_t)(pl * SY_KS * 2) +
                          (uint32_t)(((lane & 3) ^ syrk_swz16(drow)) * 16) + (uint32_t)s0 * (2 * SY_KS * 2);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.xh + (int64_t)(op ? it.y : it.x) * SK_T * 2 * a.ldh), 0, (int)(SK_T * rowb), 0x00020000);
    const int ddst = ((op * 2 + pl) * SK_T + 128 * (wv & 1)) * SH_ROW;
    auto dma = [&](int st, int buf) __attribute__((always_inline)) {
        const uint32_t kb = (uint32_t)st * (2 * SY_KS * 2);
#pragma unroll
        for (int q = 0; q < 8; ++q)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rs, (__attribute__((address_space(3))) void *)(lds + buf * SK_STG + ddst + q * 16 * SH_ROW), 16, voff,
                (uint32_t)(q * 16) * rowb + kb, 0, 0);
    };
    typedef f16x8 F2[2][2];   // [tile][plane]
    auto frag_a = [&](int buf, int t0, F2 &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * SK_STG;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = wr + 16 * (t0 + i) + r;
                f[i][pn] = as_h(*reinterpret_cast<const u32x4 *>(base + (pn * SK_T + row) * SH_ROW +
                                                                 8 * (g ^ syrk_swz16(row))));
            }
    };
    auto frag_b = [&](int buf, int j0, F2 &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * SK_STG;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = wc + 16 * (j0 + j) + r;
                f[j][pn] = as_h(*reinterpret_cast<const u32x4 *>(base + ((2 + pn) * SK_T + row) * SH_ROW +
                                                                 8 * (g ^ syrk_swz16(row))));
            }
    };
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // row tiles t0, t0+1 x column tiles j0, j0+1: the l*h products, then h*l, then h*h (the
    // same order for every element: a tile's values do not depend on its position); part
    // 0: the first MFMA only, 1: the other 11, 2: all 12
    auto mfma4 = [&](const F2 &fa, const F2 &fb, int t0, int j0, int part) __attribute__((always_inline)) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int ii = 0; ii < 2; ++ii)
#pragma unroll
                for (int jj = 0; jj < 2; ++jj) {
                    const bool first = p == 0 && ii == 0 && jj == 0;
                    if (part == 0 && !first) continue;
                    if (part == 1 && first) continue;
                    acc[t0 + ii][j0 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(
                        p == 0 ? fa[ii][1] : fa[ii][0], p == 1 ? fb[jj][1] : fb[jj][0], acc[t0 + ii][j0 + jj], 0, 0, 0);
                }
    };
    F2 fa0, fa1, fb0, fb1;   // A row-tile pairs (alternating), B column tiles 0-1 and 2-3
    // prologue: stage 0 landed everywhere, stage 1 in flight, stage 0's first fragments read
    dma(0, 0);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    __builtin_amdgcn_s_barrier();
    if (nst > 1) dma(1, 1);
    frag_a(0, 0, fa0);
    frag_b(0, 0, fb0);
    frag_b(0, 2, fb1);
    // one row-tile pair's 24 MFMAs with the next pair's fragments read after the first
    // (ROCm's waitcnt pass drains lgkmcnt before the first MFMA of a block of them)
    auto group = [&](const F2 &fa, int t0, auto rd) __attribute__((always_inline)) {
        mfma4(fa, fb0, t0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        rd();
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa, fb0, t0, 0, 1);
        mfma4(fa, fb1, t0, 2, 2);
        __builtin_amdgcn_sched_barrier(0);
    };
    auto step = [&](int st, auto bc) __attribute__((always_inline)) {
        constexpr int B = decltype(bc)::value;
        const bool more = st + 1 < nst;
        group(fa0, 0, [&]() __attribute__((always_inline)) { frag_a(B, 2, fa1); });
        group(fa1, 2, [&]() __attribute__((always_inline)) { frag_a(B, 4, fa0); });
        group(fa0, 4, [&]() __attribute__((always_inline)) { frag_a(B, 6, fa1); });
        // every wave's reads of this buffer are in registers and stage st+1 landed
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (st + 2 < nst) dma(st + 2, B);
        __builtin_amdgcn_sched_barrier(0);
        // the last pair: its column tiles 0-1, then 2-3, each B half refilled from stage
        // st+1 right after its last MFMA of this stage
        mfma4(fa1, fb0, 6, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (more) frag_a(B ^ 1, 0, fa0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb0, 6, 0, 1);
        __builtin_amdgcn_sched_barrier(0);
        if (more) frag_b(B ^ 1, 0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        mfma4(fa1, fb1, 6, 2, 2);
        __builtin_amdgcn_sched_barrier(0);
        if (more) frag_b(B ^ 1, 2, fb1);
        __builtin_amdgcn_sched_barrier(0);
    };
    int st = 0;
    for (; st + 2 <= nst; st += 2) {
        step(st, std::integral_constant<int, 0>{});
        step(st + 1, std::integral_constant<int, 1>{});
    }
    if (st < nst) step(st, std::integral_constant<int, 0>{});
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    float *o = a.part + (((int64_t)it.z * a.ntl + it.w) * 8 + wave) * SK_SUB + 4 * lane;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4 *>(o + (4 * i + j) * 256) = acc[i][j];
}

// G from syrk_h3k_kernel's partial tiles. One workgroup per 4 MFMA tiles (16 x 16) of a wave
// block, one thread per accumulator lane: its float4 of each chunk (S coalesced 1 KB loads
// per wave, many workgroups in flight, no LDS) summed in fp64 in chunk order and scaled by
// 2^-(e_row + e_col) (xes == 0: one exponent per row for every chunk, applied to the sum;
// xes > 0: chunk z's rows carry exponents xe[z * xes + row], applied per chunk), plus
// (dense) the Dense-section terms syrk_h3q_kernel<0, 4, true> stored in G's lower
// triangle, rounded once to OutT and written to G[row][col] and G[col][row] (the mirror: G
// is exactly symmetric; the lane's 4 rows are 4 consecutive columns of the mirror row). Only
// row >= col is taken from a diagonal tile (its upper half computed the same sums in the
// other operand order).
template <typename OutT>
struct SyrkSumArgs {
    const float *part;
    int S;
    int64_t ntl;
    const int2 *tiles;      // the launch's tiles (I, J) by local index
    const int32_t *xe;
    int64_t xes;
    int N;
    OutT *G;
    int64_t ldg;
    int dense;
};

template <typename OutT>
__global__ __launch_bounds__(256) void syrk_ksum_kernel(SyrkSumArgs<OutT> a) {
    const int64_t b = blockIdx.x;
    const int t = (int)(b >> 6), w = (int)((b >> 3) & 7), m = (int)(b & 7);
    const int2 tb = a.tiles[t];
    const int q = 256 * m + threadIdx.x, ij = q >> 6, ln = q & 63;   // float4 q of the wave block
    const int row0 = tb.x * SK_T + (w >> 2) * 128 + 16 * (ij >> 2) + 4 * (ln >> 4);   // + e
    const int col = tb.y * SK_T + (w & 3) * 64 + 16 * (ij & 3) + (ln & 15);
    const int N = a.N;
    if (row0 + 3 < col || row0 >= N || col >= N) return;   // no lower-triangle element
    const int rc[4] = {min(row0, N - 1), min(row0 + 1, N - 1), min(row0 + 2, N - 1), min(row0 + 3, N - 1)};
    double s[4] = {0.0, 0.0, 0.0, 0.0};
    const f32x4 *p = reinterpret_cast<const f32x4 *>(a.part + ((int64_t)t * 8 + w) * SK_SUB) + q;
    const int64_t zst = a.ntl * 8 * (SK_SUB / 4);   // float4 stride between chunks
    for (int z = 0; z < a.S; ++z) {
        const f32x4 v = p[z * zst];
        if (a.xes) {
            const int32_t *xz = a.xe + z * a.xes;
            const int ec = xz[col];
#pragma unroll
            for (int e = 0; e < 4; ++e) s[e] += __builtin_ldexp((double)v[e], -(xz[rc[e]] + ec));
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) s[e] += (double)v[e];
        }
    }
    OutT f[4];
    const int ec = a.xes ? 0 : a.xe[col];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int row = row0 + e;
        double v = a.xes ? s[e] : __builtin_ldexp(s[e], -(a.xe[rc[e]] + ec));
        f[e] = (OutT)0;
        if (row >= N || col > row) continue;
        OutT *g = a.G + (int64_t)row * a.ldg + col;
        if (a.dense) v += (double)*g;
        f[e] = (OutT)v;
        *g = f[e];
    }
    // the mirror: G[col][row0 .. row0 + 3], the entries with row > col
    OutT *u = a.G + (int64_t)col * a.ldg + row0;
    if (row0 > col && row0 + 3 < N && ((uintptr_t)u % (4 * sizeof(OutT))) == 0) {
        if constexpr (sizeof(OutT) == 4) {
            *reinterpret_cast<f32x4 *>(u) = f32x4{(float)f[0], (float)f[1], (float)f[2], (float)f[3]};
        } else {
            typedef double f64x2 __attribute__((ext_vector_type(2)));
            reinterpret_cast<f64x2 *>(u)[0] = f64x2{(double)f[0], (double)f[1]};
            reinterpret_cast<f64x2 *>(u)[1] = f64x2{(double)f[2], (double)f[3]};
        }
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (row0 + e < N && row0 + e > col) u[e] = f[e];
    }
}

#ifdef SNK_SYRK_MEASURE
// MEASURED, NOT KEPT (tools/syrk_lab.hip only; gpurun_out r05f / r05h): with the two-level
// fp32 sum it spills (713-752 ms at n = 50,000); with one fp32 sum over all K (VAR 4: 2^-24 x
// 2461 steps, 3.5e-6 of sqrt(G_ii G_jj) against syrk_h3q_kernel) 457-461 ms against 472-482
// for syrk_h3q_kernel in the chip-wide order on the same box (its clock 2.1 GHz, but 59 % of
// MFMA-busy cycles against 69 %): not worth the accuracy.
// syrk_h3r_kernel: the conv-column Gram on RECTANGULAR 256 x 128 tiles (round 5). The
// 128 x 128 kernel is bound by its stage stream, not by the matrix cores: at n = 50,000 its
// build without MFMAs (tools/syrk_lab.hip, VAR 1) takes as long as the real one at a higher
// clock, and without the stage DMAs (VAR 2) it runs in 0.63 of the time. A 256-row A block
// against a 128-row B block moves 48 KB per 32-k stage for twice the MFMAs of the 32 KB
// stage of a 128 x 128 tile: 3/4 of the L2 -> LDS bytes per FLOP, and 2/3 of the fragment
// bytes per MFMA (each wave a 64 x 64 block: 4 x 4 tiles of 16 x 16, 48 MFMAs per stage
// on 16 fragment reads instead of 24 on 12).
// Tile (bi, bj): rows 256 bi .. +255, columns 128 bj .. +127, bj <= 2 bi + 1; only entries
// with column <= row are stored (the mirror pass fills the rest). 8 waves: wave w owns rows
// 64 (w >> 1) .. +63 and columns 64 (w & 1) .. +63. Stage buffer [A h][A l][B h][B l] x rows
// x 32 halves (48 KB), NB = 3 buffers (two stages in flight), the same swizzle and LDS-DMA
// scheme as syrk_h3q_kernel (6 jobs of 16 rows x 64 B per wave and stage).
// Accumulation: fp32 MFMA accumulators, added every SY_FLUSH stages (1024 k) into a second
// fp32 sum (the 64 + 64 registers of a 64 x 64 block leave no room for fp64): the error is
// that of a 77-term fp32 sum of 1024-long fp32 dot products, <= 2^-24 (77 + 32) sum|x_i x_j|,
// i.e. below 6.5e-6 sqrt(G_ii G_jj) in the worst case and ~1e-7 in practice.
constexpr int SR_A = 256, SR_B = 128;
// NW waves: 8 (two per SIMD, 64 x 64 each) or 4 (one per SIMD, 512 registers, 128 x 64 each:
// a quarter fewer fragment reads per MFMA again)
// GL: the stage pieces by global_load_lds with one 64-bit source per job (as syrk_h3q_kernel)
// instead of the buffer descriptors
// LEAN (NW = 8): the B fragments single-buffered in two column-tile halves (each refilled
// with the next stage's right after its last MFMA of this stage), 64 fragment registers
// instead of 96, which leaves room for the second-level sum
template <int VAR = 0, int NB = 3, int NW = 8, int GL = 0, int LEAN = 0>
__global__ __launch_bounds__(64 * NW) void syrk_h3r_kernel(SyrkArgs a) {
    static_assert(!LEAN || NW == 8, "lean B fragments: 8 waves");
    constexpr int NJ = 48 / NW;                         // DMA jobs per wave and stage (48 KB / NW waves / 1 KB)
    constexpr int NTA = 2 * SR_A / NW / 16;             // A row tiles per wave (4 or 8)
    constexpr int NG = NTA / 2;                         // groups of two row tiles
    constexpr int STG = 2 * (SR_A + SR_B) * SH_ROW;    // halves per stage buffer
    __shared__ __attribute__((aligned(16))) uint16_t lds[NB * STG];
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
#endif
    int bi, bj;
    {
        const int2 tb = a.tiles[a.t0 + blockIdx.x];
        bi = tb.x;
        bj = tb.y;
    }
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int wr = (wave >> 1) * (2 * SR_A / NW), wc = (wave & 1) * 64;
    const int N = a.N;
    const int nst = (int)(a.ldh / SY_KS);
    // DMA job j = NJ * wave + q: j < 32: A plane j >> 4, 16-row block j & 15; else B plane
    // (j - 32) >> 3, block (j - 32) & 7. Rows past N exist (planes padded to SW_ROWS_B rows).
    // LDS-DMA through two buffer descriptors (the A and the B row block; T8 / T20 of the
    // programming guide): the lane's part of every job's source is one 32-bit offset (row
    // lane >> 2 of the 16-row block and its swizzled chunk: the swizzle of row 16 rb +
    // (lane >> 2) does not depend on rb), the job / stage part a scalar offset, so no 64-bit
    // address per job stays live across the loop
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    const uint32_t rowb = (uint32_t)(2 * a.ldh * 2);   // bytes per plane row
    const uint32_t lane_off = (uint32_t)(lane >> 2) * rowb + (uint32_t)(((lane & 3) ^ syrk_swz16(lane >> 2)) * 16);
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.xh + (int64_t)bi * SR_A * 2 * a.ldh), 0, (int)(SR_A * rowb), 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
        (void *)(a.xh + (int64_t)bj * SR_B * 2 * a.ldh), 0, (int)(SR_B * rowb), 0x00020000);
    const uint16_t *gsrc[GL ? NJ : 1];
    if constexpr (GL) {
#pragma unroll
        for (int q = 0; q < NJ; ++q) {
            const int j = NJ * wv + q, op = j >= 32 ? 1 : 0, jj = op ? j - 32 : j;
            const int pl = op ? jj >> 3 : jj >> 4, rb = op ? jj & 7 : jj & 15;
            const int64_t grow = (op ? (int64_t)bj * SR_B : (int64_t)bi * SR_A) + rb * 16 + (lane >> 2);
            gsrc[q] = a.xh + grow * 2 * a.ldh + pl * SY_KS + ((lane & 3) ^ syrk_swz16(lane >> 2)) * 8;
        }
    }
    auto dma = [&](int st, int buf) __attribute__((always_inline)) {
        if (VAR == 2 && st > NB - 2) return;
        if constexpr (GL) {
            const int64_t k = (int64_t)min(st, nst - 1) * 2 * SY_KS;
#pragma unroll
            for (int q = 0; q < NJ; ++q) {
                const int j = NJ * wv + q, op = j >= 32 ? 1 : 0, jj = op ? j - 32 : j;
                const int pl = op ? jj >> 3 : jj >> 4, rb = op ? jj & 7 : jj & 15;
                const int dst = ((op ? 2 * SR_A + pl * SR_B : pl * SR_A) + rb * 16) * SH_ROW;
                __builtin_amdgcn_global_load_lds((const void *)(gsrc[q] + k),
                                                 (__attribute__((address_space(3))) void *)(lds + buf * STG + dst), 16, 0, 0);
            }
            return;
        }
        const uint32_t kb = (uint32_t)min(st, nst - 1) * (2 * SY_KS * 2);
#pragma unroll
        for (int q = 0; q < NJ; ++q) {
            const int j = NJ * wv + q, op = j >= 32 ? 1 : 0, jj = op ? j - 32 : j;
            const int pl = op ? jj >> 3 : jj >> 4, rb = op ? jj & 7 : jj & 15;
            const uint32_t soff = (uint32_t)(rb * 16) * rowb + (uint32_t)(pl * SY_KS * 2) + kb;
            const int dst = ((op ? 2 * SR_A + pl * SR_B : pl * SR_A) + rb * 16) * SH_ROW;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(op ? rsb : rsa,
                                                     (__attribute__((address_space(3))) void *)(lds + buf * STG + dst),
                                                     16, lane_off, soff, 0, 0);
        }
    };
    typedef f16x8 FA[2][2];   // [tile][plane]
    typedef f16x8 FB[4][2];
    auto frag_a = [&](int buf, int t0, FA &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * STG;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int row = wr + 16 * (t0 + i) + r;
                f[i][pn] = as_h(*reinterpret_cast<const u32x4 *>(base + (pn * SR_A + row) * SH_ROW +
                                                                 8 * (g ^ syrk_swz16(row))));
            }
    };
    auto frag_b = [&](int buf, FB &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * STG;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int row = wc + 16 * j + r;
                f[j][pn] = as_h(*reinterpret_cast<const u32x4 *>(base + (2 * SR_A + pn * SR_B + row) * SH_ROW +
                                                                 8 * (g ^ syrk_swz16(row))));
            }
    };
    // VAR 4 (measurement): no second-level sum (one fp32 accumulation over all K)
    f32x4 acc[NTA][4];
    float mid[VAR == 4 ? 1 : NTA][4][4];
#pragma unroll
    for (int i = 0; i < NTA; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                acc[i][j][e] = 0.0f;
                if (VAR != 4) mid[i][j][e] = 0.0f;
            }
    // half of a stage's 48 MFMAs: row tiles t0, t0+1 x the four column tiles (l*h, h*l, h*h);
    // part 0: only the first MFMA, part 1: the other 23, part 2: all 24
    auto mfma_half = [&](const FA &fa, const FB &fb, int t0, int part) __attribute__((always_inline)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = t0 + ii;
                const bool first = ii == 0 && j == 0;
                if (VAR == 1) {
                    if (part != 0 && (part == 2 || !first))
                        acc[i][j][0] += (float)(fa[ii][0][0] * fb[j][0][0]) + (float)(fa[ii][1][1] * fb[j][1][1]);
                    continue;
                }
                if (part == 2 || (part == 0) == first)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][1], fb[j][0], acc[i][j], 0, 0, 0);
                if (part != 0) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[j][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[j][0], acc[i][j], 0, 0, 0);
                }
            }
    };
    auto flush = [&]() __attribute__((always_inline)) {
        if (VAR == 4) return;
#pragma unroll
        for (int i = 0; i < NTA; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    mid[i][j][e] += acc[i][j][e];
                    acc[i][j][e] = 0.0f;
                }
    };
#pragma unroll
    for (int q = 0; q < NB - 1; ++q) dma(q, q);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm((NB - 2) * NJ));
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    FA f0, f1;   // row-tile groups alternate: group gi in f(gi & 1)
    FB b0, b1;
    frag_a(0, 0, f0);
    if constexpr (!LEAN) frag_b(0, b0);
    // step st (buffer B = st % NB; f0 / bc hold stage st's row-tile group 0 and B): the first
    // MFMA, group 1's fragments, the rest of group 0; each further group's MFMAs with the next
    // group's fragments read under them; the DMA of stage st+NB-1 (into the buffer of stage
    // st-1), the wait for stage st+1 and the barrier; stage st+1's group 0 and B read; the
    // last group's MFMAs (as syrk_h3q_kernel's step)
    auto step = [&](int st, auto bc_, FB &bc, FB &bn) __attribute__((always_inline)) {
        constexpr int B = decltype(bc_)::value;
        mfma_half(f0, bc, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        frag_a(B, 2, f1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_half(f0, bc, 0, 1);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (NG == 4) {
            frag_a(B, 4, f0);
            __builtin_amdgcn_sched_barrier(0);
            mfma_half(f1, bc, 2, 2);
            __builtin_amdgcn_sched_barrier(0);
            frag_a(B, 6, f1);
            __builtin_amdgcn_sched_barrier(0);
            mfma_half(f0, bc, 4, 2);
            __builtin_amdgcn_sched_barrier(0);
        }
        dma(st + NB - 1, (B + NB - 1) % NB);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm((NB - 2) * NJ));   // my part of stage st+1 landed
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        frag_a((B + 1) % NB, 0, f0);
        frag_b((B + 1) % NB, bn);
        __builtin_amdgcn_sched_barrier(0);
        mfma_half(f1, bc, NTA - 2, 2);
        __builtin_amdgcn_sched_barrier(0);
        if (st % SY_FLUSH == SY_FLUSH - 1) flush();
    };
    typedef f16x8 FB2[2][2];   // two column tiles x plane
    auto frag_b2 = [&](int buf, int j0, FB2 &f) __attribute__((always_inline)) {
        const uint16_t *base = lds + buf * STG;
#pragma unroll
        for (int pn = 0; pn < 2; ++pn)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int row = wc + 16 * (j0 + j) + r;
                f[j][pn] = as_h(*reinterpret_cast<const u32x4 *>(base + (2 * SR_A + pn * SR_B + row) * SH_ROW +
                                                                 8 * (g ^ syrk_swz16(row))));
            }
    };
    // 2 row tiles x 2 column tiles (12 MFMAs); part as mfma_half
    auto mfma_q = [&](const FA &fa, const FB2 &fb, int t0, int j0, int part) __attribute__((always_inline)) {
#pragma unroll
        for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int jj = 0; jj < 2; ++jj) {
                const int i = t0 + ii, j = j0 + jj;
                const bool first = ii == 0 && jj == 0;
                if (VAR == 1) {
                    if (part != 0 && (part == 2 || !first))
                        acc[i][j][0] += (float)(fa[ii][0][0] * fb[jj][0][0]) + (float)(fa[ii][1][1] * fb[jj][1][1]);
                    continue;
                }
                if (part == 2 || (part == 0) == first)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][1], fb[jj][0], acc[i][j], 0, 0, 0);
                if (part != 0) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[jj][1], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[ii][0], fb[jj][0], acc[i][j], 0, 0, 0);
                }
            }
    };
    FB2 q01, q23;
    if constexpr (LEAN) {
        frag_b2(0, 0, q01);
        frag_b2(0, 2, q23);
    }
    auto step_lean = [&](int st, auto bc_) __attribute__((always_inline)) {
        constexpr int B = decltype(bc_)::value;
        mfma_q(f0, q01, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        frag_a(B, 2, f1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_q(f0, q01, 0, 0, 1);
        __builtin_amdgcn_sched_barrier(0);
        mfma_q(f0, q23, 0, 2, 2);
        __builtin_amdgcn_sched_barrier(0);
        dma(st + NB - 1, (B + NB - 1) % NB);
        __builtin_amdgcn_s_waitcnt(waitcnt_vm((NB - 2) * NJ));   // my part of stage st+1 landed
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        frag_a((B + 1) % NB, 0, f0);
        __builtin_amdgcn_sched_barrier(0);
        mfma_q(f1, q01, 2, 0, 2);
        __builtin_amdgcn_sched_barrier(0);
        frag_b2((B + 1) % NB, 0, q01);
        __builtin_amdgcn_sched_barrier(0);
        mfma_q(f1, q23, 2, 2, 2);
        __builtin_amdgcn_sched_barrier(0);
        frag_b2((B + 1) % NB, 2, q23);
        __builtin_amdgcn_sched_barrier(0);
        if (st % SY_FLUSH == SY_FLUSH - 1) flush();
    };
    constexpr int U = LEAN ? NB : NB % 2 ? 2 * NB : NB;
    auto one = [&](int st0, bool tail, auto ic) __attribute__((always_inline)) {
        constexpr int I = decltype(ic)::value;
        if (!tail || st0 + I < nst) {
            if constexpr (LEAN)
                step_lean(st0 + I, std::integral_constant<int, I % NB>{});
            else
                step(st0 + I, std::integral_constant<int, I % NB>{}, I % 2 ? b1 : b0, I % 2 ? b0 : b1);
        }
    };
    auto trip = [&](int st0, bool tail) __attribute__((always_inline)) {
        static_assert(U <= 6, "unrolled trip");
        one(st0, tail, std::integral_constant<int, 0>{});
        one(st0, tail, std::integral_constant<int, 1>{});
        if constexpr (U > 2) {
            one(st0, tail, std::integral_constant<int, 2>{});
            one(st0, tail, std::integral_constant<int, 3>{});
        }
        if constexpr (U > 4) {
            one(st0, tail, std::integral_constant<int, 4>{});
            one(st0, tail, std::integral_constant<int, 5>{});
        }
    };
    int st = 0;
    for (; st + U <= nst; st += U) trip(st, false);
    if (st < nst) trip(st, true);
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    flush();
#ifdef SNK_SYRK_MEASURE
    if (a.stamps && threadIdx.x == 0) {
        a.stamps[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memtime();
        a.stamps[4 * blockIdx.x + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
#pragma unroll
    for (int i = 0; i < NTA; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int col = bj * SR_B + wc + 16 * j + r;
            if (col >= N) continue;
            const int ec = a.xe[col];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = bi * SR_A + wr + 16 * i + 4 * g + e;
                if (row >= N || col > row) continue;
                a.g32[(int64_t)row * a.ldg + col] = __builtin_ldexpf(VAR == 4 ? acc[i][j][e] : mid[i][j][e], -(a.xe[row] + ec));
            }
        }
}

#endif  // SNK_SYRK_MEASURE

constexpr int SW_ROWS_B = 256;   // Jacobian-plane rows are padded to a multiple of this

// D'D: slab[z] = X[:, z-th k chunk] X[:, z-th k chunk]^T (lower-triangle
// tiles), fp32 rows split into bf16 x6 in the kernel
__global__ __launch_bounds__(256) void syrk_slab_kernel(SyrkArgs a) {
    __shared__ __attribute__((aligned(16))) SyrkX6Lds sm;
    int bi, bj;
    {
        const int64_t t = a.t0 + (a.direct ? (int64_t)blockIdx.x : syrk_xcd_remap(blockIdx.x, a.ntiles));
        if (a.tiles) {
            const int2 tb = a.tiles[t];
            bi = tb.x;
            bj = tb.y;
        } else {
            syrk_tile(t, bi, bj);
        }
    }
    f32x16 acc[2][2];
    double accd[2][2][16];
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                acc[mi][ni][g] = 0.0f;
                accd[mi][ni][g] = 0.0;
            }
    const int64_t k0 = (int64_t)blockIdx.y * a.kchunk;
    const int64_t k1 = k0 + a.kchunk < a.K ? k0 + a.kchunk : a.K;
    if (k0 < k1) syrk_loop_x6<true>(a.x, a.ld, a.N, k0, k1, bi, bj, sm, acc, accd);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = bj * SY_T + wc + ni * 32 + (lane & 31);
            if (col >= a.N) continue;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int row = bi * SY_T + wr + mi * 32 + acc_row(g, lane);
                if (row >= a.N) continue;
                a.g64[(int64_t)blockIdx.y * a.N * a.N + (int64_t)row * a.N + col] = accd[mi][ni][g];
            }
        }
}

}  // namespace snk

// snk_deep_bwd.hpp — the conv backward of the configs[2] deep net at the
// update's batch (B = 64), on v_mfma_f32_16x16x32_bf16: L3 (6x6, 64 -> 64,
// valid), L2 (3x3 pad 1, 32 -> 64) and L1 (3x3 pad 1, 32 -> 32).
//
// The generic engine (gemm_bf16_kernel + snk_loaders.hpp) gathered every
// im2col element with two integer divisions and a scalar load: L3's data
// gradient took 335 us and its weight gradient 156 us + a reduce for 2 x 4.2
// GFLOP; L2 and L1 together 183 us + two reduces. Both directions are
// reorganised around LDS images of the sample(s) a workgroup owns, with the
// arithmetic of the contract unchanged (snk_deep.hpp header, oracle/
// snake_oracle.c conv_bwd_bf16): the masked gradient dz is rounded to bf16
// (RNE) as the operand, the weights are the bf16 image, the layer input is
// bf16, every product is exact and the sums are fp32.
//
//  * deep_conv_dx_kernel<CI, CO, KS, PAD, H> (grid: NB tile rows x S samples,
//    8 waves): dx[s][pin][ci] = (x > 0) * sum_{du,dv,co} dz[s][pin - (du,dv) +
//    PAD][co] * W[kk][ci][co]. The workgroup's 4 output rows need dz rows
//    4tj - (KS-1) + PAD .. 4tj + 3 + PAD: a bordered bf16 image of KS + 3 rows x
//    PJ = 28 columns, CO + 16 halves per position (160 or 96 bytes), zeros
//    outside the dz grid. Row tiles are 4x4 blocks of output positions (as
//    deep_front_kernel); with those strides and PJ = 28 every ds_read_b128 lane
//    group of a B fragment hits 16 distinct bank quads (simulated), and a read's
//    address is one lane constant minus a wave-uniform (kernel offset, tile)
//    term. A = the weights in packed order [kk][ci][co] (the image's WT
//    sections), straight from L2 into a register ring (4 offsets at 6x6, 3 at
//    3x3): rows = ci, k = co. Wave = (ci tile, contraction half of 32 co, group
//    of row tiles); the halves meet in LDS. (At L3, one wave per (ci tile, 2-3
//    row tiles) with both halves and a two-offset ring waited on L2 every
//    offset: 38 us against 22 at B = 64, 20x20.)
//  * deep_conv_dw_kernel<CI, CO, KS, PAD, H, NS> (grid: KS kernel rows dv x
//    ceil(S/NS) sample chunks): slab[z][(kk*CI + ci)*CO + co] = sum_{s in chunk
//    z, pout} dz[s][pout][co] * x[s][pout + (du,dv) - PAD][ci]; the dv == 0
//    blocks also write the bias row (column sums of the rounded dz). The sum
//    runs over positions, so both operands are read k-major with
//    ds_read_b64_tr_b16 (gfx950's transposing LDS read) from natural
//    [position][channel] images: each lane supplies its own position's row
//    address, which makes the shifted window (pout + (du, dv)) and the k padding
//    to a multiple of 32 (a zero dz row) free. The x window carries the padding
//    as zero border columns. 152-byte rows for 64 channels and plain 64-byte rows
//    for 32 keep both kinds of read at most 2-way (simulated). slab_reduce_kernel
//    sums the chunks in chunk order.
#pragma once
#include "snk_deep.hpp"

namespace snk {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

// ---------------------------------------------------------------- data gradient
template <int CI, int CO, int KS, int PAD, int H>
struct DeepDxShape {
    static constexpr int HO = H + 2 * PAD - KS + 1;                       // dz grid side
    static constexpr int NB = (H + 3) / 4, PJ = 28, ROWS = KS + 3, PST = CO + 16;
    static constexpr int CT = CI / 16, KH = CO / 32, PG = 8 / (CT * KH), NTW = (NB + PG - 1) / PG;
    static constexpr int RING = (KS * KS) % 4 == 0 ? 4 : 3;
    static constexpr int IMG = ROWS * PJ * PST * 2;                       // bytes
    static constexpr int RED = KH == 2 ? CT * NB * 64 * 16 : 0;           // the k-half partials
    static constexpr int LDS = IMG > RED ? IMG : RED;
    static_assert(4 * NB + KS - 1 <= PJ, "image columns");
    static_assert(CT * KH * PG == 8 && (KS * KS) % RING == 0, "wave split / ring");
};

template <int CI, int CO, int KS, int PAD, int H>
__global__ __launch_bounds__(512) void deep_conv_dx_kernel(const float *__restrict__ dz,
                                                           const uint16_t *__restrict__ wt,
                                                           const uint16_t *__restrict__ xin, float *__restrict__ dx,
                                                           int64_t S) {
    using Sh = DeepDxShape<CI, CO, KS, PAD, H>;
    constexpr int HO = Sh::HO, NB = Sh::NB, PJ = Sh::PJ, PST = Sh::PST, ROWS = Sh::ROWS;
    constexpr int CT = Sh::CT, KH = Sh::KH, PG = Sh::PG, NTW = Sh::NTW, RING = Sh::RING, NKK = KS * KS;
    extern __shared__ __attribute__((aligned(16))) uint16_t dxsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int ct = wave % CT, kh = (wave / CT) % KH, pg = wave / (CT * KH);
    const int tj = blockIdx.x;
    const int64_t s = blockIdx.y;
    if (s >= S) return;
    // the weight fragment of kernel offset kk: rows ci = 16 ct + r, k = co 32 kh + 8 g .. +7
    const uint16_t *wl = wt + (ct * 16 + r) * CO + 32 * kh + 8 * g;
    u32x4 wf[RING];
#pragma unroll
    for (int o = 0; o < RING; ++o) wf[o] = *reinterpret_cast<const u32x4 *>(wl + o * (CI * CO));
    // stage dz rows jlo .. jlo + ROWS - 1 (image row y), columns clo .. clo + PJ - 1 (image column c) as bf16
    {
        constexpr int PPP = CO / 4;   // 4-channel pieces per position
        constexpr int NP = ROWS * PJ * PPP, PT = (NP + 511) / 512;
        const float *src = dz + s * (HO * HO * CO);
        const int jlo = 4 * tj - (KS - 1) + PAD, clo = PAD - (KS - 1);
        f32x4 v[PT];
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q / PPP, pc = q - pos * PPP;
            const int y = pos / PJ, cc = pos - y * PJ, jj = jlo + y, ii = clo + cc;
            const bool ok = q < NP && jj >= 0 && jj < HO && ii >= 0 && ii < HO;
            v[u] = ok ? *reinterpret_cast<const f32x4 *>(src + (jj * HO + ii) * CO + pc * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q / PPP, pc = q - pos * PPP;
            if (q < NP)
                *reinterpret_cast<u32x2 *>(dxsm + pos * PST + pc * 4) =
                    u32x2{pk_bf16(v[u][0], v[u][1]), pk_bf16(v[u][2], v[u][3])};
        }
    }
    __syncthreads();
    // lane position (4 ti + (r & 3), 4 tj + (r >> 2)): its dz cell at offset (du, dv) is
    // image row (KS-1) + (r >> 2) - dv, column 4 ti + (r & 3) + (KS-1) - du
    const int lbase = ((KS - 1 + (r >> 2)) * PJ + KS - 1 + (r & 3)) * PST + 32 * kh + 8 * g;
    f32x4 acc[NTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k4 = 0; k4 < NKK; k4 += RING) {
#pragma unroll
        for (int o = 0; o < RING; ++o) {
            const int kk = k4 + o, du = kk % KS, dv = kk / KS;
            const uint16_t *Bk = dxsm + lbase - (dv * PJ + du) * PST;
            // branch-free: a wave's tiles past NB repeat tile NB-1 and are dropped in the epilogue (a
            // branch per tile split the loads from the MFMAs: 22 -> 59 us at L3)
            bf16x8 xv[NTW];
#pragma unroll
            for (int i = 0; i < NTW; ++i)
                xv[i] = as_bf(*reinterpret_cast<const u32x4 *>(Bk + 4 * min(pg + PG * i, NB - 1) * PST));
#pragma unroll
            for (int i = 0; i < NTW; ++i)
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(wf[o]), xv[i], acc[i], 0, 0, 0);
            if (kk + RING < NKK) wf[o] = *reinterpret_cast<const u32x4 *>(wl + (kk + RING) * (CI * CO));
        }
    }
    f32x4 *red = reinterpret_cast<f32x4 *>(dxsm);
    if (KH == 2) {   // the two contraction halves: half 1 parks its sums, half 0 adds them (the image is dead)
        __syncthreads();
        if (kh == 1) {
#pragma unroll
            for (int i = 0; i < NTW; ++i)
                if (pg + PG * i < NB) red[(ct * NB + pg + PG * i) * 64 + lane] = acc[i];
        }
        __syncthreads();
        if (kh == 1) return;
    }
    // epilogue: lane holds ci = 16 ct + 4 g + e of its position; relu mask of the layer input, fp32 out
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
        const int ti = pg + PG * i;
        if (ti >= NB) continue;
        const f32x4 p = KH == 2 ? red[(ct * NB + ti) * 64 + lane] : f32x4{0.f, 0.f, 0.f, 0.f};
        const int ii = 4 * ti + (r & 3), jj = 4 * tj + (r >> 2);
        if (ii >= H || jj >= H) continue;
        const int64_t o = (s * (H * H) + ii + jj * H) * CI + ct * 16 + 4 * g;
        const u32x2 m = *reinterpret_cast<const u32x2 *>(xin + o);
        f32x4 y;
        y[0] = bf2f((uint16_t)(m[0] & 0xffffu)) > 0.0f ? acc[i][0] + p[0] : 0.0f;
        y[1] = bf2f((uint16_t)(m[0] >> 16)) > 0.0f ? acc[i][1] + p[1] : 0.0f;
        y[2] = bf2f((uint16_t)(m[1] & 0xffffu)) > 0.0f ? acc[i][2] + p[2] : 0.0f;
        y[3] = bf2f((uint16_t)(m[1] >> 16)) > 0.0f ? acc[i][3] + p[3] : 0.0f;
        *reinterpret_cast<f32x4 *>(dx + o) = y;
    }
}

// ---------------------------------------------------------------- L3 forward, small batches
// deep_conv3_small_kernel: L3's forward (6x6, 64 -> 64, valid) at the update's batch, on the
// data-gradient kernel's tiling (4x4 output tiles, a bordered LDS image of the tile row's input
// rows, the weight fragments through a 4-offset register ring), so grid = NB tile rows x S
// samples (256
// workgroups at B = 64) instead of the persistent pair kernel's
// B / 2 = 32 (41 us per net). Input a2 is bf16 (staged as is), the epilogue is bias + relu ->
// bf16 a3, and the weights are the forward image [kk][co][ci] (rows co, k = ci).
template <int H>
__global__ __launch_bounds__(512) void deep_conv3_small_kernel(const uint16_t *__restrict__ x,
                                                               const uint16_t *__restrict__ wimg,
                                                               const float *__restrict__ bias,
                                                               uint16_t *__restrict__ y, int64_t S) {
    constexpr int WO = H - 5;
    using Sh = DeepDxShape<64, 64, 6, 5, WO>;   // output grid WO x WO, input grid H x H
    constexpr int NB = Sh::NB, PJ = Sh::PJ, PST = Sh::PST, ROWS = Sh::ROWS, RING = 4, NT = (NB + 1) / 2;
    static_assert(Sh::HO == H, "input grid");
    extern __shared__ __attribute__((aligned(16))) uint16_t c3ssm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4, ct = wave & 3, th = wave >> 2;
    const int tj = blockIdx.x;
    const int64_t s = blockIdx.y;
    if (s >= S) return;
    // weight fragments of offset kk: rows co = 16 ct + r, k = ci 32 c + 8 g .. +7 (c = 0, 1)
    const uint16_t *wl = wimg + (ct * 16 + r) * 64 + 8 * g;
    u32x4 wf[RING][2];
#pragma unroll
    for (int o = 0; o < RING; ++o)
#pragma unroll
        for (int c = 0; c < 2; ++c) wf[o][c] = *reinterpret_cast<const u32x4 *>(wl + o * 4096 + 32 * c);
    // stage input rows 4tj .. 4tj + ROWS - 1 (image row y), columns 0 .. PJ - 1 (image column c)
    {
        constexpr int NP = ROWS * PJ * 8, PT = (NP + 511) / 512;   // 16-byte pieces (8 channels)
        const uint16_t *src = x + s * (H * H * 64);
        u32x4 v[PT];
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q >> 3, pc = q & 7;
            const int yy = pos / PJ, cc = pos - yy * PJ, jj = 4 * tj + yy;
            const bool ok = q < NP && jj < H && cc < H;
            v[u] = ok ? *reinterpret_cast<const u32x4 *>(src + (jj * H + cc) * 64 + pc * 8) : u32x4{0u, 0u, 0u, 0u};
        }
#pragma unroll
        for (int u = 0; u < PT; ++u) {
            const int q = tid + u * 512, pos = q >> 3, pc = q & 7;
            if (q < NP) *reinterpret_cast<u32x4 *>(c3ssm + pos * PST + pc * 8) = v[u];
        }
    }
    __syncthreads();
    // lane position (4 ti + (r & 3), 4 tj + (r >> 2)) reads input (i + du, j + dv): image row
    // (r >> 2) + dv, column 4 ti + (r & 3) + du. Wave th takes row tiles th*NT .. th*NT + NT - 1
    // (a tile past NB repeats NB - 1 and is dropped); per accumulator the MFMAs run offset by
    // offset, channel half 0 then 1: deep_conv3_kernel's order, so a3 is bit-identical.
    const int lbase = ((r >> 2) * PJ + (r & 3)) * PST + 8 * g;
    f32x4 acc[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int k4 = 0; k4 < 36; k4 += RING) {
#pragma unroll
        for (int o = 0; o < RING; ++o) {
            const int kk = k4 + o, du = kk % 6, dv = kk / 6;
            const uint16_t *Bk = c3ssm + lbase + (dv * PJ + du) * PST;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                bf16x8 xv[NT];
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    xv[i] = as_bf(*reinterpret_cast<const u32x4 *>(Bk + 4 * min(th * NT + i, NB - 1) * PST + 32 * c));
#pragma unroll
                for (int i = 0; i < NT; ++i)
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(wf[o][c]), xv[i], acc[i], 0, 0, 0);
            }
            if (kk + RING < 36) {
#pragma unroll
                for (int c = 0; c < 2; ++c) wf[o][c] = *reinterpret_cast<const u32x4 *>(wl + (kk + RING) * 4096 + 32 * c);
            }
        }
    }
    const f32x4 bb = *reinterpret_cast<const f32x4 *>(bias + ct * 16 + 4 * g);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
        const int ti = th * NT + i;
        const int ii = 4 * ti + (r & 3), jj = 4 * tj + (r >> 2);
        if (ti >= NB || ii >= WO || jj >= WO) continue;
        *reinterpret_cast<u32x2 *>(y + (s * (WO * WO) + ii + jj * WO) * 64 + ct * 16 + 4 * g) = relu_bf16x4(acc[i], bb);
    }
}

// ---------------------------------------------------------------- weight gradient
// wave tile: COW co tiles x CIW ci tiles x DUW kernel columns; the first NWB of the 8
// waves cover the KS columns x CO/16 x CI/16 tiles of one kernel row
template <int CI, int CO, int KS, int PAD, int H, int NS>
struct DeepDwShape {
    static constexpr int HO = H + 2 * PAD - KS + 1, NO = HO * HO, KST = (NO + 31) / 32;
    static constexpr int RSTD = CO == 64 ? 76 : 32, RSTX = CI == 64 ? 76 : 32;   // halves per row
    static constexpr int XW = HO + KS - 1;                                       // x window columns
    static constexpr int DZR = NO + 1, AR = HO * XW;                             // dz rows (+ the zero row NO), x rows
    static constexpr int SMP = DZR * RSTD + AR * RSTX;                           // halves per sample
    static constexpr int LDS = NS * SMP * 2;
    static constexpr int MN = (KS * KS * CI + 1) * CO;                           // one slab (the bias row last)
    static constexpr int COW = 2, CIW = CI / 16 >= 2 ? 2 : 1, DUW = KS % 3 == 0 && KS > 3 ? 3 : 1;
    static constexpr int GCO = CO / 16 / COW, GCI = CI / 16 / CIW, GDU = KS / DUW, NWB = GCO * GCI * GDU;
    static_assert(LDS <= 160 * 1024, "samples per workgroup");
    static_assert(NWB <= 8 && GCO * COW * 16 == CO && GCI * CIW * 16 == CI && GDU * DUW == KS, "wave tiles");
    static_assert((SMP * 2) % 8 == 0 && (DZR * RSTD * 2) % 8 == 0, "8-byte aligned transposed reads");
};

__device__ __forceinline__ u32x2 tr_read(const uint16_t *p) {
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4 *)(p));
    return __builtin_bit_cast(u32x2, v);
}

template <int CI, int CO, int KS, int PAD, int H, int NS>
__global__ __launch_bounds__(512) void deep_conv_dw_kernel(const float *__restrict__ dz,
                                                           const uint16_t *__restrict__ xin, float *__restrict__ slab,
                                                           int64_t S) {
    using Sh = DeepDwShape<CI, CO, KS, PAD, H, NS>;
    constexpr int HO = Sh::HO, NO = Sh::NO, KST = Sh::KST, RSTD = Sh::RSTD, RSTX = Sh::RSTX, XW = Sh::XW;
    constexpr int DZR = Sh::DZR, AR = Sh::AR, SMP = Sh::SMP;
    constexpr int COW = Sh::COW, CIW = Sh::CIW, DUW = Sh::DUW, GCO = Sh::GCO, GCI = Sh::GCI;
    extern __shared__ __attribute__((aligned(16))) uint16_t dwsm[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int dv = blockIdx.x;
    const int64_t z = blockIdx.y;
    // ---- staging: per sample q, dz rows 0 .. NO-1 as bf16 + the zero row NO; the x window
    // rows dv - PAD .. dv - PAD + HO - 1, columns -PAD .. XW - 1 - PAD (zero outside the board)
    {
        constexpr int PZ = CO / 4, PX = CI / 8;   // 4-channel dz pieces, 8-channel x pieces per row
        constexpr int NDZ = NS * DZR * PZ, NA = NS * AR * PX, NTOT = NDZ + NA, U = 12;
        for (int b = 0; b < NTOT; b += U * 512) {
            u32x4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 512 + tid;
                v[u] = u32x4{0u, 0u, 0u, 0u};
                if (e < NDZ) {
                    const int q = e / (DZR * PZ), rem = e - q * (DZR * PZ), row = rem / PZ, pc = rem - row * PZ;
                    const int64_t sg = NS * z + q;
                    if (row < NO && sg < S) {
                        const f32x4 f = *reinterpret_cast<const f32x4 *>(dz + (sg * NO + row) * CO + pc * 4);
                        v[u] = u32x4{pk_bf16(f[0], f[1]), pk_bf16(f[2], f[3]), 0u, 0u};
                    }
                } else if (e < NTOT) {
                    const int ea = e - NDZ, q = ea / (AR * PX), rem = ea - q * (AR * PX), row = rem / PX;
                    const int pc = rem - row * PX, wj = row / XW, wi = row - wj * XW;
                    const int xr = wj + dv - PAD, xc = wi - PAD;
                    const int64_t sg = min(NS * z + q, S - 1);   // finite values (a missing sample's dz is zero)
                    if (xr >= 0 && xr < H && xc >= 0 && xc < H)
                        v[u] = *reinterpret_cast<const u32x4 *>(xin + (sg * (H * H) + xr * H + xc) * CI + pc * 8);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int e = b + u * 512 + tid;
                if (e < NDZ) {
                    const int q = e / (DZR * PZ), rem = e - q * (DZR * PZ), row = rem / PZ, pc = rem - row * PZ;
                    *reinterpret_cast<u32x2 *>(dwsm + q * SMP + row * RSTD + pc * 4) = u32x2{v[u][0], v[u][1]};
                } else if (e < NTOT) {
                    const int ea = e - NDZ, q = ea / (AR * PX), rem = ea - q * (AR * PX), row = rem / PX;
                    const int pc = rem - row * PX;
                    uint16_t *d = dwsm + q * SMP + DZR * RSTD + row * RSTX + pc * 8;
                    *reinterpret_cast<u32x2 *>(d) = u32x2{v[u][0], v[u][1]};
                    *reinterpret_cast<u32x2 *>(d + 4) = u32x2{v[u][2], v[u][3]};
                }
            }
        }
    }
    __syncthreads();
    float *sl = slab + z * Sh::MN;
    if (dv == 0 && tid < CO) {   // bias row: column sums of the rounded dz, sample then position order
        float b = 0.0f;
        for (int q = 0; q < NS; ++q)
            for (int row = 0; row < NO; ++row) b += bf2f(dwsm[q * SMP + row * RSTD + tid]);
        sl[KS * KS * CI * CO + tid] = b;
    }
    if (wave >= Sh::NWB) return;
    // ---- wave tile: co tiles COW*cg + c, ci tiles CIW*ig + t, kernel columns du = DUW*dg + d
    const int cg = wave % GCO, ig = (wave / GCO) % GCI, dg = wave / (GCO * GCI);
    const int G = lane >> 4, qq = (lane & 15) >> 2, pp = lane & 3;
    f32x4 acc[DUW][COW][CIW];
#pragma unroll
    for (int a = 0; a < DUW; ++a)
#pragma unroll
        for (int b = 0; b < COW; ++b)
#pragma unroll
            for (int c = 0; c < CIW; ++c) acc[a][b][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int q = 0; q < NS; ++q) {
        const uint16_t *dzb = dwsm + q * SMP + (16 * COW * cg + 4 * pp);               // + row * RSTD + 16 c
        const uint16_t *xb = dwsm + q * SMP + DZR * RSTD + (16 * CIW * ig + 4 * pp);    // + (wpos + du) * RSTX + 16 t
#pragma unroll 1
        for (int ks = 0; ks < KST; ++ks) {
            int drow[2], arow[2];
#pragma unroll
            for (int hh = 0; hh < 2; ++hh) {
                const int k = 32 * ks + 8 * G + qq + 4 * hh;
                drow[hh] = (k < NO ? k : NO) * RSTD;
                const int kc = k < NO ? k : NO - 1, kj = kc / HO;
                arow[hh] = (kc - kj * HO + kj * XW + DUW * dg) * RSTX;
            }
            bf16x8 A[COW];
#pragma unroll
            for (int c = 0; c < COW; ++c) {
                const u32x2 lo = tr_read(dzb + drow[0] + 16 * c), hi = tr_read(dzb + drow[1] + 16 * c);
                A[c] = as_bf(u32x4{lo[0], lo[1], hi[0], hi[1]});
            }
#pragma unroll
            for (int d = 0; d < DUW; ++d) {
#pragma unroll
                for (int t = 0; t < CIW; ++t) {
                    const u32x2 lo = tr_read(xb + arow[0] + d * RSTX + 16 * t);
                    const u32x2 hi = tr_read(xb + arow[1] + d * RSTX + 16 * t);
                    const bf16x8 Bv = as_bf(u32x4{lo[0], lo[1], hi[0], hi[1]});
#pragma unroll
                    for (int c = 0; c < COW; ++c)
                        acc[d][c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[c], Bv, acc[d][c][t], 0, 0, 0);
                }
            }
        }
    }
    // lane holds co = 16 (COW cg + c) + 4 G + e, ci = 16 (CIW ig + t) + (lane & 15) of offset kk = du + KS dv
#pragma unroll
    for (int d = 0; d < DUW; ++d) {
        const int kk = DUW * dg + d + KS * dv;
#pragma unroll
        for (int c = 0; c < COW; ++c)
#pragma unroll
            for (int t = 0; t < CIW; ++t) {
                const int co = 16 * (COW * cg + c) + 4 * G, ci = 16 * (CIW * ig + t) + (lane & 15);
                *reinterpret_cast<f32x4 *>(sl + (kk * CI + ci) * CO + co) = acc[d][c][t];
            }
    }
}

}  // namespace snk

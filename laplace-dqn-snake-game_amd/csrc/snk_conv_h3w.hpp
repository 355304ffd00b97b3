// snk_conv_h3w.hpp — the large-batch act forward's conv1 + conv2 + conv3 as ONE
// persistent, weight-stationary kernel on the h3 split (snk_conv_h3.hpp).
//
// conv_h3f_kernel (snk_conv_h3f.hpp) runs one workgroup of four samples per CU
// and streams all 73,728 conv3 weights through LDS for every group: each group
// loads them from L2, splits them into fp16 h / l parts on the VALU, writes them
// to LDS and waits on a barrier every two kernel offsets (its offset loop ran at
// about half the MFMA rate). Here the weights stay in registers:
//
//   - one workgroup per CU (4 waves, one per SIMD), looping over groups of four
//     samples (grid-stride); the conv3 weights are loaded and split ONCE, wave w
//     holding output channels 32 (w & 1) .. +31 for kernel offsets 18 (w >> 1) .. +17
//     as 72 f16x8 MFMA B fragments (288 registers, VGPRs and AGPRs: MFMA reads
//     its B operand from either);
//   - conv3 per group is 18 offsets x 13 row tiles x 2 column tiles x 3 products
//     of v_mfma_f32_16x16x32_f16 per wave, with only the A fragments (the split
//     conv2 output, conv_h3f_kernel's LDS image) read from LDS: no weight staging,
//     no barrier inside the loop;
//   - the two offset halves of a channel block meet once per group in LDS (the
//     output staging area): waves 2-3 store their partial sums, waves 0-1 add
//     theirs, scale, add the bias, relu;
//   - conv2's split weights stay resident in LDS for the workgroup's life;
//   - the next group's board cells are loaded into registers while conv3 runs.
//
// conv1 (fp32 VALU, conv1_fwd_kernel's FMA order: a1 bit-identical), conv2 (three
// f16 products, per-sample a1 scale, per-tensor w2 scale), the per-sample a2
// scale and conv3's products are those of conv_h3f_kernel; only conv3's
// summation order differs (two offset halves, then their sum), so the result has
// the same error class (test_h3s_error_class_vs_fp32, the 1e-5 oracle tests).
#pragma once

#include "snk_conv_h3f.hpp"

namespace snk {

template <int HIN>
struct H3W {
    static constexpr int KS = 6, CN = 64, CK = 32, NSG = 4, NTHR = 256, NKK = KS * KS, KH = NKK / 2;
    static constexpr int hin = HIN, ho = HIN - KS + 1, ho2 = ho * ho, hin2 = hin * hin;
    // conv3 A image (conv_h3f_kernel's): [sample][channel group of 8][part][j][i], 16-byte units
    static constexpr int XW = ho + 8, PL = (hin * XW + 3) & ~3, GG = 2 * PL, XS = 4 * GG + 4;
    // conv2: bordered A1 image rows of XR halves, weight rows of BR halves (conflict-free reads)
    static constexpr int BP = HIN + 2, NPB = BP * BP, XR = 16, BR = 48, XP = XR / 8;
    static constexpr int A1_H = NSG * 2 * NPB * XR;
    static constexpr int B2_H = 5 * 2 * 32 * BR;
    static constexpr int R2 = NSG * hin2, T2 = (R2 + 15) / 16, U2 = (T2 + 3) / 4;
    static constexpr int T3 = (NSG * ho2 + 15) / 16;    // conv3 row tiles (sample-interleaved rows)
    static constexpr int CS = 80;                        // output staging row stride (floats)
    static constexpr int NW4 = 9 * 32 * 16 / 4, LW = (NW4 + NTHR - 1) / NTHR;
    static constexpr int LA = (NSG * hin2 * 4 + NTHR - 1) / NTHR;
    // LDS: conv2 weights | board floats [NSG][C][NPB] | A1 image / conv3 A image / output staging
    static constexpr int OFF_X = B2_H * 2;
    static constexpr int xbytes(int C) { return NSG * C * NPB * 4; }
    static constexpr int abytes() {
        const int a1 = A1_H * 2, a3 = NSG * XS * 16, cs = NSG * ho2 * CS * 4;
        return a1 > a3 ? (a1 > cs ? a1 : cs) : (a3 > cs ? a3 : cs);
    }
    static constexpr int off_a(int C) { return (OFF_X + xbytes(C) + 15) & ~15; }
    static constexpr int lds_bytes(int C) { return off_a(C) + abytes(); }
};

template <int HIN, int CF>
__global__ __launch_bounds__(256) void conv_h3w_kernel(H3FArgs a, int S) {
    using G = H3W<HIN>;
    constexpr int C = CF, NSG = G::NSG, NTHR = G::NTHR, KS = G::KS, KH = G::KH;
    constexpr int hin = G::hin, ho = G::ho, ho2 = G::ho2, hin2 = G::hin2;
    constexpr int XW = G::XW, PL = G::PL, GG = G::GG, XS = G::XS;
    constexpr int BP = G::BP, NPB = G::NPB, XR = G::XR, BR = G::BR, XP = G::XP;
    constexpr int R2 = G::R2, T2 = G::T2, U2 = G::U2, T3 = G::T3, CS = G::CS;
    constexpr int NW4 = G::NW4, LW = G::LW, LA = G::LA;
    constexpr int NX = NSG * C * NPB, LB = (NX + NTHR - 1) / NTHR;
    static_assert(G::lds_bytes(C) <= 160 * 1024, "conv_h3w LDS");
    const int rb = a.rider.out ? 1 : 0;
    if (rb && blockIdx.x == 0) {   // the trainer's replay draw rides workgroup 0 (no LDS, no barrier)
        if (threadIdx.x < 64) sample_wave(a.rider);
        return;
    }
    extern __shared__ __attribute__((aligned(16))) u32x4 h3w_lds[];
    __shared__ float red[4][8];
    __shared__ const int8_t *pbase[NSG * C];
    uint8_t *lb = reinterpret_cast<uint8_t *>(h3w_lds);
    uint16_t *B2 = reinterpret_cast<uint16_t *>(lb);
    float *xin = reinterpret_cast<float *>(lb + G::OFF_X);
    u32x4 *As = reinterpret_cast<u32x4 *>(lb + G::off_a(C));
    uint16_t *A1 = reinterpret_cast<uint16_t *>(As);
    u32x2 *A1v = reinterpret_cast<u32x2 *>(A1), *B2v = reinterpret_cast<u32x2 *>(B2);
    float *Cs = reinterpret_cast<float *>(As);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4;
    const int cp = wave & 1, oh = wave >> 1;
    const int nwg = (int)gridDim.x - rb, wg = (int)blockIdx.x - rb;
    const int ngroups = (S + NSG - 1) / NSG;

    // ---- once per workgroup: the weight scales (conv3 from the partial maxima, conv2 from
    // its 4,608 weights), conv2's split weights into LDS, conv3's into registers
    float wm3 = 0.0f;
    for (int i = tid; i < a.nwmax; i += NTHR) wm3 = fmaxf(wm3, a.wmax[i]);
    f32x4 wv[LW];
    const f32x4 *w4 = reinterpret_cast<const f32x4 *>(a.w2);
    float mw2 = 0.0f;
#pragma unroll
    for (int u = 0; u < LW; ++u) {
        wv[u] = w4[min(u * NTHR + tid, NW4 - 1)];
        if (u * NTHR + tid < NW4)
            mw2 = fmaxf(mw2, fmaxf(fmaxf(fabsf(wv[u][0]), fabsf(wv[u][1])), fmaxf(fabsf(wv[u][2]), fabsf(wv[u][3]))));
    }
    wm3 = wave_max(wm3);
    mw2 = wave_max(mw2);
    if (lane == 0) {
        red[wave][0] = wm3;
        red[wave][1] = mw2;
    }
    __syncthreads();
    const int ew = h3_exp(fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0])));
    const int ew2 = h3_exp(fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1])));
#pragma unroll
    for (int u = 0; u < LW; ++u) {   // conv2 image [kk][co][ci] -> offset pair p, k = 16 (kk - 2p) + ci
        const int e = u * NTHR + tid;
        if (e < NW4) {
            const int kk = e >> 7, co = (e >> 2) & 31, ci0 = 4 * (e & 3);
            const int p = kk >> 1, k0 = 16 * (kk & 1) + ci0;
            u32x2 hh, ll;
            h3_split4(wv[u], ew2, hh, ll);
            B2v[(((p * 2 + 0) * 32 + co) * BR + k0) / 4] = hh;
            B2v[(((p * 2 + 1) * 32 + co) * BR + k0) / 4] = ll;
        }
    }
    if (tid < 2 * 32 * 2) {   // pair 4's pad offset (kk = 9: k 16..31) is zero
        const int pl = tid >> 6, co = (tid >> 1) & 31, piece = tid & 1;
        reinterpret_cast<u32x4 *>(B2)[(((4 * 2 + pl) * 32 + co) * BR + 16) / 8 + piece] = u32x4{0u, 0u, 0u, 0u};
    }
    // conv3 B fragments: B[k = ci 8g .. 8g+7][n = co] of offset kk = KH oh + q, column tile ct
    f16x8 wf[KH][2][2];
    {
        const f32x4 *w3 = reinterpret_cast<const f32x4 *>(a.w3);
#pragma unroll
        for (int q = 0; q < KH; ++q)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int kk = KH * oh + q, co = 32 * cp + 16 * ct + r;
                const f32x4 *p = w3 + ((int64_t)(kk * 64 + co) * 32 + 8 * g) / 4;
                const f32x4 v0 = p[0], v1 = p[1];
                u32x2 h0, l0, h1, l1;
                h3_split4(v0, ew, h0, l0);
                h3_split4(v1, ew, h1, l1);
                wf[q][ct][0] = as_h(u32x4{h0[0], h0[1], h1[0], h1[1]});
                wf[q][ct][1] = as_h(u32x4{l0[0], l0[1], l1[0], l1[1]});
            }
    }
    float b2v[2][4];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
#pragma unroll
        for (int e = 0; e < 4; ++e) b2v[ct][e] = a.b2[ct * 16 + 4 * g + e];

    // board cells of group grp into registers (bv), through the plane pointers in pbase
    typedef const __attribute__((address_space(1))) int8_t gi8;
    const bool fl = a.src.fbase != nullptr;
    int bv[LB];
    auto set_planes = [&](int grp) __attribute__((always_inline)) {   // threads < NSG * C, before a barrier
        if (tid < NSG * C) {
            const int s = grp * NSG + tid / C;
            pbase[tid] = (!fl && s < S) ? a.src.plane(s, tid % C) : nullptr;
        }
    };
    auto load_boards = [&](int grp) __attribute__((always_inline)) {
        const int s0 = grp * NSG, ns = min(NSG, S - s0);
#pragma unroll
        for (int u = 0; u < LB; ++u) {
            const int q = u * NTHR + tid;
            const int sc = min(q / NPB, NSG * C - 1), b = q - sc * NPB;
            const int bj = b / BP, bi = b - bj * BP;
            const bool in = q < NX && sc / C < ns && bi >= 1 && bi <= hin && bj >= 1 && bj <= hin;
            const int cell = (bi - 1) + (bj - 1) * hin;
            if (fl) {
                bv[u] = in ? __float_as_int(a.src.fbase[((int64_t)(s0 + sc / C) * C + sc % C) * hin2 + cell]) : 0;
            } else {
                gi8 *pl = (gi8 *)pbase[sc];
                bv[u] = in ? (int)pl[cell] : 0;
            }
        }
    };
    int grp = wg;
    if (grp < ngroups) set_planes(grp);
    __syncthreads();   // B2, pbase
    if (grp < ngroups) load_boards(grp);

    for (; grp < ngroups; grp += nwg) {
        const int s0 = grp * NSG, ns = min(NSG, S - s0);
        // ---- (a) board floats into LDS
#pragma unroll
        for (int u = 0; u < LB; ++u) {
            const int q = u * NTHR + tid;
            if (q < NX) xin[q] = fl ? __int_as_float(bv[u]) : (float)bv[u];
        }
        __syncthreads();   // 1: xin ready; the previous group's output stores have read the A region
        // ---- (b) conv1: thread e = (sample, position, channels 4 (tid & 3) ..), weights in registers
        f32x4 av[LA];
        {
            const int cq = tid & 3;
            f32x4 w1r[9 * C];
#pragma unroll
            for (int q = 0; q < 9 * C; ++q) w1r[q] = reinterpret_cast<const f32x4 *>(a.w1)[q * 4 + cq];
            const f32x4 b1r = reinterpret_cast<const f32x4 *>(a.b1)[cq];
            const int na4 = ns * hin2 * 4;
#pragma unroll
            for (int u = 0; u < LA; ++u) {
                const int e = min(u * NTHR + tid, na4 - 1);
                const int sr = e / (hin2 * 4), pos = (e - sr * hin2 * 4) >> 2;
                const int j = pos / hin, i = pos - j * hin;
                f32x2 acc01{b1r[0], b1r[1]}, acc23{b1r[2], b1r[3]};
#pragma unroll
                for (int kk = 0; kk < 9; ++kk) {
                    const int du = kk % 3, dv = kk / 3;
#pragma unroll
                    for (int c = 0; c < C; ++c) {
                        const float x = xin[(sr * C + c) * NPB + (i + du) + (j + dv) * BP];
                        const f32x2 xx{x, x};
                        const f32x4 w = w1r[kk * C + c];
                        acc01 = __builtin_elementwise_fma(xx, f32x2{w[0], w[1]}, acc01);
                        acc23 = __builtin_elementwise_fma(xx, f32x2{w[2], w[3]}, acc23);
                    }
                }
                av[u] = f32x4{fmaxf(acc01[0], 0.f), fmaxf(acc01[1], 0.f), fmaxf(acc23[0], 0.f), fmaxf(acc23[1], 0.f)};
            }
            float ms[NSG] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int u = 0; u < LA; ++u) {
                const int e = u * NTHR + tid;
                const int sr = e < na4 ? e / (hin2 * 4) : NSG;
                const float m = fmaxf(fmaxf(fabsf(av[u][0]), fabsf(av[u][1])), fmaxf(fabsf(av[u][2]), fabsf(av[u][3])));
#pragma unroll
                for (int q = 0; q < NSG; ++q) ms[q] = sr == q ? fmaxf(ms[q], m) : ms[q];
            }
#pragma unroll
            for (int q = 0; q < NSG; ++q) ms[q] = wave_max(ms[q]);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < NSG; ++q) red[wave][q] = ms[q];
            }
        }
        __syncthreads();   // 2: conv1 maxima
        // ---- (c) the A1 image: zero border, split a1 with the per-sample scale
        int ea1[NSG];
#pragma unroll
        for (int q = 0; q < NSG; ++q)
            ea1[q] = h3_exp(fmaxf(fmaxf(red[0][q], red[1][q]), fmaxf(red[2][q], red[3][q])));
        {
            constexpr int NBD = 4 * (BP - 1);
            for (int q = tid; q < NSG * 2 * NBD * XP; q += NTHR) {
                const int pc = q / (NBD * XP), rem = q - pc * NBD * XP, bpos = rem / XP, piece = rem - bpos * XP;
                const int side = bpos / (BP - 1), t = bpos - side * (BP - 1);
                const int pb = side == 0 ? t : side == 1 ? (BP - 1) + t * BP : side == 2 ? (BP * BP - 1) - t
                                                                                         : (BP - 1 - t) * BP;
                reinterpret_cast<u32x4 *>(A1)[((pc * NPB + pb) * XR) / 8 + piece] = u32x4{0u, 0u, 0u, 0u};
            }
            const int na4 = ns * hin2 * 4;
#pragma unroll
            for (int u = 0; u < LA; ++u) {
                const int e = u * NTHR + tid;
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
        }
        __syncthreads();   // 3: A1 image ready
        // ---- (d) conv2, transposed (weights as the MFMA A operand): tiles t = wave + 4u
        f32x4v acc2[U2][2];
        int rsl[U2], aslot[U2];
        {
            int rpos[U2];
#pragma unroll
            for (int u = 0; u < U2; ++u) {
                acc2[u][0] = acc2[u][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
                const int q = min((wave + 4 * u) * 16 + r, R2 - 1);
                rsl[u] = q / hin2;
                const int pos = q - rsl[u] * hin2, j = pos / hin, i = pos - j * hin;
                rpos[u] = i + j * BP;
                aslot[u] = rsl[u] * XS + (g >> 1) * GG + j * XW + i;
            }
            constexpr int UF = T2 / 4;   // tiles every wave has; tile UF only waves < T2 - 4 UF
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
                auto tile = [&](int u) __attribute__((always_inline)) {
                    const uint16_t *pa = A1 + ((rsl[u] * 2) * NPB + rpos[u] + du + dv * BP) * XR + 8 * (g & 1);
                    const f16x8 fah = as_h(*reinterpret_cast<const u32x4 *>(pa));
                    const f16x8 fal = as_h(*reinterpret_cast<const u32x4 *>(pa + NPB * XR));
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) {
                        f32x4v c = acc2[u][ct];
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ct], fal, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[ct], fah, c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ct], fah, c, 0, 0, 0);
                        acc2[u][ct] = c;
                    }
                };
#pragma unroll
                for (int u = 0; u < UF; ++u) tile(u);
                if (U2 > UF && wave + 4 * UF < T2) tile(U2 - 1);
            }
        }
        // bias + relu in place, per-sample max (rows past R2 repeat row R2 - 1)
        {
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
                if (wave + 4 * u >= T2) lm = 0.0f;
#pragma unroll
                for (int q = 0; q < NSG; ++q) m2[q] = sr == q ? fmaxf(m2[q], lm) : m2[q];
            }
#pragma unroll
            for (int q = 0; q < NSG; ++q) m2[q] = wave_max(m2[q]);
            if (lane == 0) {
#pragma unroll
                for (int q = 0; q < NSG; ++q) red[wave][4 + q] = m2[q];
            }
        }
        const int nxt = grp + nwg;
        if (nxt < ngroups) set_planes(nxt);
        __syncthreads();   // 4: conv2 maxima; every A1 read done (the conv3 image overlays it)
        // ---- (e) conv2 output -> conv3's A image
        int ea[NSG];
#pragma unroll
        for (int q = 0; q < NSG; ++q)
            ea[q] = h3_exp(fmaxf(fmaxf(red[0][4 + q], red[1][4 + q]), fmaxf(red[2][4 + q], red[3][4 + q])));
        {
            u32x2 *Ah2 = reinterpret_cast<u32x2 *>(As);
#pragma unroll
            for (int u = 0; u < U2; ++u) {
                const int row = (wave + 4 * u) * 16 + r;
                if (wave + 4 * u < T2 && row < R2) {
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
        }
        __syncthreads();   // 5: conv3 A image ready; next group's plane pointers set
        // ---- (f) the next group's boards (their latency hides behind conv3), then conv3
        if (nxt < ngroups) load_boards(nxt);
        f32x4v acc[T3][2];
        {
            int abase[T3];
#pragma unroll
            for (int k = 0; k < T3; ++k) {
                acc[k][0] = acc[k][1] = f32x4v{0.f, 0.f, 0.f, 0.f};
                const int q = 16 * k + r;
                const int p = min(q >> 2, ho2 - 1), sr = q & 3;
                const int j = p / ho, i = p - j * ho;
                abase[k] = sr * XS + g * GG + j * XW + i;
            }
#pragma unroll
            for (int q = 0; q < KH; ++q) {
                const int kk = KH * oh + q, dv = kk / KS, du = kk - dv * KS;
                const u32x4 *pa = As + dv * XW + du;
#pragma unroll
                for (int k = 0; k < T3; ++k) {
                    const f16x8 ah = as_h(pa[abase[k]]), al = as_h(pa[abase[k] + PL]);
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) {
                        f32x4v c = acc[k][ct];
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wf[q][ct][0], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wf[q][ct][1], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wf[q][ct][0], c, 0, 0, 0);
                        acc[k][ct] = c;
                    }
                }
            }
        }
        __syncthreads();   // 6: every A-image read done (the output staging overlays it)
        // ---- (g) offset halves meet in the output staging: waves 2-3 store partial sums,
        // waves 0-1 add theirs, undo the scales, bias, relu
        if (oh == 1) {
#pragma unroll
            for (int k = 0; k < T3; ++k) {
                const int p = 4 * k + g;
                if (p >= ho2) continue;
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const int col = 32 * cp + 16 * ct + r;
#pragma unroll
                    for (int e = 0; e < 4; ++e) Cs[(e * ho2 + p) * CS + col] = acc[k][ct][e];
                }
            }
        }
        __syncthreads();   // 7
        if (oh == 0) {
#pragma unroll
            for (int k = 0; k < T3; ++k) {
                const int p = 4 * k + g;
                if (p >= ho2) continue;
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const int col = 32 * cp + 16 * ct + r;
                    const float bv3 = a.b3[col];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float *o = Cs + (e * ho2 + p) * CS + col;
                        const float v = __builtin_ldexpf(acc[k][ct][e] + *o, -(ea[e] + ew)) + bv3;
                        *o = v > 0.0f ? v : 0.0f;
                    }
                }
            }
        }
        __syncthreads();   // 8
        const int n4o = ns * ho2 * 16;
        f32x4 *o4 = reinterpret_cast<f32x4 *>(a.out + (int64_t)s0 * ho2 * G::CN);
        const f32x4 *c4 = reinterpret_cast<const f32x4 *>(Cs);
        for (int q = tid; q < n4o; q += NTHR) o4[q] = c4[(q >> 4) * (CS / 4) + (q & 15)];
    }
}

}  // namespace snk

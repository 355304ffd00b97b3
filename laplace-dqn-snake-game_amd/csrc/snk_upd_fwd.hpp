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
//            LDS image, B (the weight planes the update keeps current) streamed
//            from L2 into registers one offset ahead; bias + relu -> a3.
// conv1 and conv2 run in both halves of a sample (they are ~20 % of the work);
// only half 0 writes a1, a2 and x0. Dense1 and the heads follow as before.
#pragma once

#include "snk_conv_x6.hpp"
#include "snk_qnet.hpp"

namespace snk {

struct UpdFwdNet {
    BoardSrc src;
    const float *th;        // packed theta: conv1 weights/bias, conv2/conv3 biases
    const uint16_t *wtb;    // x6 split planes of the forward weight image
    float *a1, *a2, *a3;    // a1/a2 may be null (target net: only a3 is consumed)
    float *x0;              // the input planes as floats [S][C][bs^2] (training net) or null
};
struct UpdFwdArgs {
    UpdFwdNet net[2];
    QLayout L;
    int S;
};

// LDS strides (halves): A1 position record 3 planes x 16 ch + 8 pad, A2 3 x 32 + 8
constexpr int UPDF_A1S = 56, UPDF_A2S = 104;

// floats of the input planes + conv1 weights, rounded up to a 16-byte boundary
__host__ __device__ constexpr int updf_f32_words(int hin, int C) {
    return (C * (hin + 2) * (hin + 2) + 9 * C * 16 + 16 + 3) & ~3;
}
__host__ __device__ constexpr int updf_lds_bytes(int hin, int C) {
    return updf_f32_words(hin, C) * 4 + (hin + 2) * (hin + 2) * UPDF_A1S * 2 + 9 * 3 * 32 * 16 * 2 +
           hin * hin * UPDF_A2S * 2;
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

template <int HIN, int C>
__global__ __launch_bounds__(256) void upd_fwd_kernel(UpdFwdArgs args) {
    constexpr int BP = HIN + 2, NB = BP * BP, NC = HIN * HIN;
    constexpr int WO = HIN - 5, NO = WO * WO;
    constexpr int T2 = (NC + 15) / 16, T3 = (NO + 15) / 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t updf_lds[];
    float *xin = reinterpret_cast<float *>(updf_lds);                 // [C][NB]
    float *w1 = xin + C * NB;                                        // [9C*16] + bias [16]
    uint16_t *A1 = reinterpret_cast<uint16_t *>(xin + updf_f32_words(HIN, C));   // [NB][UPDF_A1S]
    uint16_t *B2 = A1 + NB * UPDF_A1S;                               // [9 kk][3][32 co][16 ci]
    uint16_t *A2 = B2 + 9 * 3 * 32 * 16;                             // [NC][UPDF_A2S]
    static_assert((NB * UPDF_A1S * 2) % 16 == 0, "16-B regions");

    const UpdFwdNet &n = args.net[blockIdx.y];
    const QLayout &L = args.L;
    const int s = blockIdx.x >> 1, half = blockIdx.x & 1;
    const bool wr = half == 0;   // half 0 writes the training activations
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;

    // ---- phase 0: input planes, conv1 weights, conv2 weight planes, A1 border --------
    for (int e = tid; e < C * NB; e += 256) {
        const int c = e / NB, b = e - c * NB;
        const int bj = b / BP, bi = b - bj * BP;
        float v = 0.0f;
        if (bi >= 1 && bi <= HIN && bj >= 1 && bj <= HIN) {
            const int cell = (bi - 1) + (bj - 1) * HIN;
            v = n.src.load(s, c, cell);
            if (wr && n.x0) n.x0[((int64_t)s * C + c) * NC + cell] = v;
        }
        xin[e] = v;
    }
    for (int e = tid; e < 9 * C * 16; e += 256) w1[e] = n.th[L.off_w1 + e];
    if (tid < 16) w1[9 * C * 16 + tid] = n.th[L.off_b1 + tid];
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(n.wtb + 3 * L.off_t2);
        u32x4 *dst = reinterpret_cast<u32x4 *>(B2);
        for (int e = tid; e < 9 * 3 * 32 * 16 / 8; e += 256) dst[e] = src[e];
    }
    for (int e = tid; e < NB * (UPDF_A1S / 8); e += 256) {   // zero the whole A1 image (border stays 0)
        reinterpret_cast<u32x4 *>(A1)[e] = u32x4{0u, 0u, 0u, 0u};
    }
    __syncthreads();

    // ---- phase 1: conv1 (VALU), a1 and its split ---------------------------------------
    for (int o = tid; o < NC * 16; o += 256) {
        const int p = o >> 4, co = o & 15;
        const int j = p / HIN, i = p - j * HIN;
        float acc = w1[9 * C * 16 + co];
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int du = kk % 3, dv = kk / 3;
#pragma unroll
            for (int c = 0; c < C; ++c)
                acc = __builtin_fmaf(xin[c * NB + (i + du) + (j + dv) * BP], w1[(kk * C + c) * 16 + co], acc);
        }
        const float v = fmaxf(acc, 0.f);
        if (wr && n.a1) n.a1[((int64_t)s * NC + p) * 16 + co] = v;
        uint16_t h, m, l;
        split3_scalar(v, h, m, l);
        uint16_t *d = A1 + ((i + 1) + (j + 1) * BP) * UPDF_A1S + co;
        d[0] = h;
        d[16] = m;
        d[32] = l;
    }
    __syncthreads();

    // ---- phase 2: conv2 on x6 MFMA: rows = the HIN^2 positions, 32 columns -------------
    {
        const float *b2 = n.th + L.off_b2;
        for (int t = wave; t < T2; t += 4) {
            const int q = min(t * 16 + r, NC - 1);
            const int qj = q / HIN, qi = q - qj * HIN;
            f32x4v acc[2] = {f32x4v{0.f, 0.f, 0.f, 0.f}, f32x4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                const int kk = 2 * p + (g >> 1);   // k 0..15: offset 2p, k 16..31: offset 2p + 1
                const bool live = kk < 9;
                const int kc = live ? kk : 8, du = kc % 3, dv = kc / 3;
                u32x4 a[3], b[2][3];
                const uint16_t *pa = A1 + ((qi + du) + (qj + dv) * BP) * UPDF_A1S + 8 * (g & 1);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) {
                    a[pl] = live ? *reinterpret_cast<const u32x4 *>(pa + pl * 16) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct)
                        b[ct][pl] = live ? *reinterpret_cast<const u32x4 *>(
                                               B2 + ((kc * 3 + pl) * 32 + ct * 16 + r) * 16 + 8 * (g & 1))
                                         : u32x4{0u, 0u, 0u, 0u};
                }
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) acc[ct] = mfma_x6(a, b[ct], acc[ct]);
            }
            // C[row 4g + e][col r]: bias + relu -> a2 and its split
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = ct * 16 + r;
                const float bv = b2[col];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = t * 16 + 4 * g + e;
                    if (row >= NC) continue;
                    const float v = fmaxf(acc[ct][e] + bv, 0.f);
                    if (wr && n.a2) n.a2[((int64_t)s * NC + row) * 32 + col] = v;
                    uint16_t h, m, l;
                    split3_scalar(v, h, m, l);
                    uint16_t *d = A2 + row * UPDF_A2S + col;
                    d[0] = h;
                    d[32] = m;
                    d[64] = l;
                }
            }
        }
    }
    __syncthreads();

    // ---- phase 3: conv3 on x6 MFMA: rows = the WO^2 output positions, 32 columns -------
    {
        const int n0 = half * 32;
        const float *b3 = n.th + L.off_b3;
        // B fragment of column n0 + 16 ct + r, k = 8g..8g+7 of offset kk, plane pl:
        // planes [kk][3][64 co][32 ci] -> 16 contiguous bytes
        const uint16_t *wb3 = n.wtb + 3 * L.off_t3 + (n0 + r) * 32 + 8 * g;
        auto bload = [&](int kk, u32x4 (&b)[2][3]) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    b[ct][pl] = *reinterpret_cast<const u32x4 *>(wb3 + ((int64_t)(kk * 3 + pl) * 64 + ct * 16) * 32);
        };
        for (int t = wave; t < T3; t += 4) {
            const int q = min(t * 16 + r, NO - 1);
            const int qj = q / WO, qi = q - qj * WO;
            f32x4v acc[2] = {f32x4v{0.f, 0.f, 0.f, 0.f}, f32x4v{0.f, 0.f, 0.f, 0.f}};
            u32x4 bc[2][3], bn[2][3];
            bload(0, bc);
            for (int kk = 0; kk < 36; ++kk) {
                if (kk + 1 < 36) bload(kk + 1, bn);
                const int du = kk % 6, dv = kk / 6;
                const uint16_t *pa = A2 + ((qi + du) + (qj + dv) * HIN) * UPDF_A2S + 8 * g;
                u32x4 a[3];
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) a[pl] = *reinterpret_cast<const u32x4 *>(pa + pl * 32);
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) acc[ct] = mfma_x6(a, bc[ct], acc[ct]);
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) bc[ct][pl] = bn[ct][pl];
            }
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = n0 + ct * 16 + r;
                const float bv = b3[col];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int row = t * 16 + 4 * g + e;
                    if (row < NO) n.a3[((int64_t)s * NO + row) * 64 + col] = fmaxf(acc[ct][e] + bv, 0.f);
                }
            }
        }
    }
}

}  // namespace snk

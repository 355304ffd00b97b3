// snk_conv.hpp — LDS-staged implicit-GEMM convolution on v_mfma_f32_32x32x2_f32.
//
// out[m][n] = sum_{kk, c} A[m][(kk, c)] * Wk[kk][c][n]
//   m  = (sample, output position)           -> MFMA rows (32 per wave)
//   kk = kernel offset (du, dv), c = channel -> reduction, CK channels per kk
//   n  = output channel                      -> MFMA columns (CN = 32 or 64)
// MODE_FWD    A = x[s][p + (du,dv) - PAD][c]      (true conv, packed weights)
// MODE_DX     A = dz[s][p - (du,dv) + PAD][c]     (data gradient: c = conv COUT,
//             n = conv CIN, weights used untransposed)
// MODE_DENSE  A = x[s][kk][c] (Dense1: kk enumerates the Wo^2 positions)
//
// Workgroup = 4 waves = 128 rows x CN columns. Per kernel offset kk the
// workgroup stages that offset's CK x CN weight block into LDS as [n][c]
// (c contiguous, row padded by 4 floats: conflict-free ds_read_b128; filled by
// 16-byte copies from a weight image already laid out [kk][n][c]), double
// buffered with one barrier per offset; each lane reads its A operand as
// float4 along c straight from global/L2 (every im2col row is a contiguous
// channel run) one offset ahead. A lane's float4 covers 4 consecutive MFMA
// k-steps: lane half h holds k = 8*kb + 4h + j at step j of channel block kb,
// and the B fragment is read with the same (kb, h, j) mapping.
// grid = (ceil(M/128), kk splits); with splits the epilogue writes partial
// slabs that a reduce kernel finishes.
#pragma once
#include "snk_gemm.hpp"

namespace snk {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum ConvMode { MODE_FWD = 0, MODE_DX = 1, MODE_DENSE = 2 };
enum ConvEpi { EPI_BIAS_RELU = 0, EPI_SLAB = 1, EPI_RELU_MASK = 2 };

struct ConvArgs {
    const float *x;      // A source [S][HIN*HIN][CK]
    const float *w;      // weight image [nkk][CN][CK]
    const float *bias;   // EPI_BIAS_RELU
    const float *act;    // EPI_RELU_MASK: mask source, same shape as out
    float *out;          // [M][CN] or slab [split][M][CN]
    const uint16_t *xb;  // x6 kernels: A pre-split into bf16 planes [S][HIN*HIN][3][CK] (else split x)
    uint16_t *outb;      // x6 EPI_BIAS_RELU: also write the output's bf16 planes [M][3][CN]
    const float *wmax;   // h3 kernels: per-block partial max |w| of the weight image (conv1 writes them)
    int nwmax;           //   their count
    int M, HIN, HOUT, nkk, kk_per_split;
    uint32_t d2m, d2s, d1m, d1s;   // FastDiv(HOUT*HOUT), FastDiv(HOUT) magic/shift
};

// one launch can run the same convolution for two independent nets
// (grid.z = group): the target and online forwards of a DQN update
struct ConvPair {
    ConvArgs g[2];
    const uint16_t *wb[2];   // x6 kernels: weight planes per group
};

__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t m, uint32_t s) { return (__umulhi(n, m) + n) >> s; }

template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
__device__ __forceinline__ void conv_mfma_body(const ConvPair &pr, dim3 bid) {
    const ConvArgs &a = pr.g[bid.z];
    constexpr int NT = CN / 32;
    constexpr int KB = CK / 8;
    constexpr int LDB = CK + 4;
    constexpr int NV = (CK * CN / 4 + 255) / 256;  // float4 staging loads per thread
    __shared__ __attribute__((aligned(16))) float Bs[2][CN * LDB + 4];   // + pad slot for idle stagers; lds: one per kernel (a paired launch's two bodies never share it)

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
    const float *xs = a.x + (int64_t)s * a.HIN * a.HIN * CK + 4 * h;
    const int kk0 = bid.y * a.kk_per_split;
    const int kk1 = min(a.nkk, kk0 + a.kk_per_split);

    f32x16 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[nt][g] = 0.0f;

    // Every global load below is unconditional: out-of-range lanes read a safe
    // in-bounds address and their value is zeroed arithmetically. A branch
    // around a load makes hipcc wait vmcnt(0) for the in-flight prefetch.
    constexpr int NE4 = CK * CN / 4;   // float4s per weight block
    const f32x4 *wsrc = reinterpret_cast<const f32x4 *>(a.w);
    int s_src[NV], s_dst[NV];          // staging: source float4 and LDS float offset
#pragma unroll
    for (int q = 0; q < NV; ++q) {
        const int e4 = tid + q * 256;
        const bool in = (NE4 % 256 == 0) || e4 < NE4;
        const int e = (in ? e4 : 0) * 4;
        const int n = e / CK, c = e - n * CK;
        s_src[q] = in ? e4 : 0;
        s_dst[q] = in ? n * LDB + c : CN * LDB;   // idle lanes write the pad slot
    }

    f32x4 bst[NV], a_cur[KB], a_nxt[KB];
    // ---- prologue: weights of kk0 -> LDS, A of kk0 -> registers
    {
#pragma unroll
        for (int q = 0; q < NV; ++q) bst[q] = wsrc[(int64_t)kk0 * NE4 + s_src[q]];
        const float *p = xs;
        float msk = ok ? 1.0f : 0.0f;
        if (MODE == MODE_DENSE) {
            p = xs + kk0 * CK;
        } else {
            const int dv = kk0 / KS, du = kk0 - dv * KS;
            const int xi = MODE == MODE_FWD ? i + du - PAD : i - du + PAD;
            const int xj = MODE == MODE_FWD ? j + dv - PAD : j - dv + PAD;
            const bool v = ok && xi >= 0 && xi < a.HIN && xj >= 0 && xj < a.HIN;
            p = v ? xs + (xi + xj * a.HIN) * CK : xs;
            msk = v ? 1.0f : 0.0f;
        }
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
            a_cur[kb] = *reinterpret_cast<const f32x4 *>(p + kb * 8) * msk;
        }
#pragma unroll
        for (int q = 0; q < NV; ++q) *reinterpret_cast<f32x4 *>(&Bs[0][s_dst[q]]) = bst[q];
    }
    __syncthreads();
    for (int kk = kk0; kk < kk1; ++kk) {
        const int buf = (kk - kk0) & 1;
        const bool more = kk + 1 < kk1;   // wave-uniform
        const int kn = more ? kk + 1 : kk;
        // ---- prefetch kk+1 (weights to registers, A to registers)
#pragma unroll
        for (int q = 0; q < NV; ++q) bst[q] = wsrc[(int64_t)kn * NE4 + s_src[q]];
        float msk_n = ok ? 1.0f : 0.0f;
        {
            const float *p = xs;
            if (MODE == MODE_DENSE) {
                p = xs + kn * CK;
            } else {
                const int dv = kn / KS, du = kn - dv * KS;
                const int xi = MODE == MODE_FWD ? i + du - PAD : i - du + PAD;
                const int xj = MODE == MODE_FWD ? j + dv - PAD : j - dv + PAD;
                const bool v = ok && xi >= 0 && xi < a.HIN && xj >= 0 && xj < a.HIN;
                p = v ? xs + (xi + xj * a.HIN) * CK : xs;
                msk_n = v ? 1.0f : 0.0f;
            }
#pragma unroll
            for (int kb = 0; kb < KB; ++kb) a_nxt[kb] = *reinterpret_cast<const f32x4 *>(p + kb * 8);
        }
        // keep the prefetch issued here, ahead of the MFMAs that hide its latency
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA on kk
        const float *bb = &Bs[buf][r * LDB + 4 * h];
#pragma unroll
        for (int kb = 0; kb < KB; ++kb) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const f32x4 b4 = *reinterpret_cast<const f32x4 *>(bb + nt * 32 * LDB + kb * 8);
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[kb][0], b4[0], acc[nt], 0, 0, 0);
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[kb][1], b4[1], acc[nt], 0, 0, 0);
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[kb][2], b4[2], acc[nt], 0, 0, 0);
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[kb][3], b4[3], acc[nt], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- weights of kk+1 -> the other LDS buffer (last read one barrier ago)
#pragma unroll
        for (int q = 0; q < NV; ++q) *reinterpret_cast<f32x4 *>(&Bs[buf ^ 1][s_dst[q]]) = bst[q];
        __syncthreads();
#pragma unroll
        for (int kb = 0; kb < KB; ++kb)
            a_cur[kb] = a_nxt[kb] * msk_n;
    }

    // epilogue: acc register g of lane l is C[(g&3) + 8*(g>>2) + 4*(l>>5)][l&31]
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
                const float v = acc[nt][g] + b;
                a.out[o] = v > 0.0f ? v : 0.0f;
            } else if (EPI == EPI_SLAB) {
                a.out[(int64_t)bid.y * a.M * CN + o] = acc[nt][g];
            } else {
                a.out[o] = a.act[o] > 0.0f ? acc[nt][g] : 0.0f;
            }
        }
    }
}

template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
__global__ __launch_bounds__(256) void conv_mfma_kernel(ConvPair pr) {
    conv_mfma_body<CK, CN, KS, PAD, MODE, EPI>(pr, blockIdx);
}

}  // namespace snk

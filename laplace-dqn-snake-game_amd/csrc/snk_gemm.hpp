// snk_gemm.hpp — generic fp32 MFMA implicit-GEMM engine for the Q-net.
//
// C[M][N] = sum_k A[M][K] * B[K][N] on v_mfma_f32_32x32x2_f32 (exact f32,
// gfx950 has no xf32). A wave owns a 32-row tile and NT 32-column tiles; a
// 256-thread workgroup stacks 4 waves along M. grid = (M tiles / 4, N groups,
// K splits). Operands come from LOADER functors so one engine serves the
// forward convolutions (implicit im2col), the data-gradient "transposed"
// convolutions and the weight-gradient reductions of the backward pass.
//
// MFMA 32x32x2 f32 operand map: lane l holds A[row l&31][k l>>5] and
// B[k l>>5][col l&31]; accumulator register g of lane l is
// C[(g&3) + 8*(g>>2) + 4*(l>>5)][l&31].
#pragma once
#include "snk_common.hpp"

namespace snk {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int acc_row(int g, int lane) { return (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5); }

template <int NT, class AL, class BL, class EP>
__global__ __launch_bounds__(256) void gemm_kernel(AL al, BL bl, EP ep, int M, int K, int kchunk) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = (blockIdx.x * 4 + wave) * 32;
    if (m0 >= M) return;
    const int r = lane & 31, h = lane >> 5;
    const int n0 = blockIdx.y * (NT * 32);
    const int kb = blockIdx.z * kchunk;
    const int ke = min(K, kb + kchunk);
    f32x16 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[nt][g] = 0.0f;
    const auto ctx = al.row(m0 + r, M);
#pragma unroll 4
    for (int k = kb; k < ke; k += 2) {
        const float a = al.load(ctx, k + h, ke);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const float b = bl.load(k + h, n0 + nt * 32 + r, ke);
            acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[nt], 0, 0, 0);
        }
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ep.store(acc[nt], m0, n0 + nt * 32, lane, (int)blockIdx.z);
}

// ---------------------------------------------------------------- epilogues
struct EpBiasRelu {  // y[row][col] = relu?(acc + bias[col])
    float *y;
    const float *bias;
    int M, N, relu;
    __device__ void store(const f32x16 &acc, int m0, int c0, int lane, int) const {
        const int col = c0 + (lane & 31);
        if (col >= N) return;
        const float b = bias ? bias[col] : 0.0f;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int row = m0 + acc_row(g, lane);
            if (row < M) {
                float v = acc[g] + b;
                if (relu) v = v > 0.0f ? v : 0.0f;
                y[(int64_t)row * N + col] = v;
            }
        }
    }
};
struct EpSlab {  // partial sums of K-split z: slab[z][row][col]
    float *slab;
    int M, N;
    __device__ void store(const f32x16 &acc, int m0, int c0, int lane, int z) const {
        const int col = c0 + (lane & 31);
        if (col >= N) return;
        float *s = slab + (int64_t)z * M * N;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int row = m0 + acc_row(g, lane);
            if (row < M) s[(int64_t)row * N + col] = acc[g];
        }
    }
};
struct EpReluMask {  // y = (act > 0) ? acc : 0   (backward through relu)
    float *y;
    const float *act;
    int M, N;
    __device__ void store(const f32x16 &acc, int m0, int c0, int lane, int) const {
        const int col = c0 + (lane & 31);
        if (col >= N) return;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int row = m0 + acc_row(g, lane);
            if (row < M) {
                const int64_t o = (int64_t)row * N + col;
                y[o] = act[o] > 0.0f ? acc[g] : 0.0f;
            }
        }
    }
};

// ---------------------------------------------------------------- B loaders
struct BRowMajor {  // B[k][n] = W[k*N + n]
    const float *w;
    int K, N;
    __device__ float load(int k, int n, int) const { return (k < K && n < N) ? w[(int64_t)k * N + n] : 0.0f; }
};
// B for the data gradient of a conv: k = (kk, co), n = ci, B = W[(kk*CIN + ci)*COUT + co]
template <int CIN, int COUT>
struct BConvT {
    const float *w;
    int K;  // KS*KS*COUT
    __device__ float load(int k, int n, int) const {
        if (k >= K || n >= CIN) return 0.0f;
        const int kk = k / COUT, co = k - kk * COUT;
        return w[(kk * CIN + n) * COUT + co];
    }
};
// B[k][n] = W[n*KW + k]  (dense data gradient: W stored [k_w][o] -> B[o][k_w])
struct BTrans {
    const float *w;
    int K, N, ld;
    __device__ float load(int k, int n, int) const { return (k < K && n < N) ? w[(int64_t)n * ld + k] : 0.0f; }
};
// B[r][n] = dz[r*N + n] for the weight-gradient reduction over rows r < R
struct BRows {
    const float *dz;
    int64_t R;
    int N;
    __device__ float load(int k, int n, int) const { return (k < R && n < N) ? dz[(int64_t)k * N + n] : 0.0f; }
};

}  // namespace snk

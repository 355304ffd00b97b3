// snk_gemm.hpp — generic fp32 MFMA implicit-GEMM engine for the Q-net.
//
// C[M][N] = sum_k A[M][K] * B[K][N] on v_mfma_f32_32x32x2_f32 (exact f32,
// gfx950 has no xf32). A workgroup owns a 32-row x NT*32-column tile.
// grid = (M tiles, N groups, K splits). Operands come from LOADER functors so one engine serves the
// forward convolutions (implicit im2col), the data-gradient "transposed"
// convolutions and the weight-gradient reductions of the backward pass.
//
// MFMA 32x32x2 f32 operand map: lane l holds A[row l&31][k l>>5] and
// B[k l>>5][col l&31]; accumulator register g of lane l is
// C[(g&3) + 8*(g>>2) + 4*(l>>5)][l&31].
#pragma once
#include <type_traits>
#include "snk_common.hpp"

namespace snk {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int acc_row(int g, int lane) { return (g & 3) + 8 * (g >> 2) + 4 * (lane >> 5); }

// KW waves per workgroup share ONE 32 x (NT*32) output tile and split its
// K range among themselves; their accumulators are summed through LDS by the
// whole workgroup (no global partials). grid.z adds K splits across workgroups that
// write partial slabs (EpSlab) when even that is too little parallelism.
// The k loop moves 8 k (4 MFMA steps) per iteration with the next
// iteration's operands loaded ahead (software pipeline).
// body with an explicit block index (also run as one half of a paired launch)
template <int NT, int KW, class AL, class BL, class EP>
__device__ __forceinline__ void gemm_body(const AL &al, const BL &bl, const EP &ep, int M, int K, int kchunk,
                                          dim3 bid) {
    __shared__ float red[KW > 1 ? KW * NT * 16 * 64 : 1];   // lds: one per kernel (a paired launch's two bodies never share it)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = bid.x * 32;
    const int r = lane & 31, h = lane >> 5;
    const int n0 = bid.y * (NT * 32);
    const int kb = bid.z * kchunk;
    const int ke = min(K, kb + kchunk);
    const int sub = (((ke - kb) + KW - 1) / KW + 7) & ~7;
    const int wb = kb + wave * sub;
    const int we = min(ke, wb + sub);
    f32x16 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int g = 0; g < 16; ++g) acc[nt][g] = 0.0f;
    const auto ctx = al.row(m0 + r, M);
    // 8-k steps in a 3-slot register ring, loads two steps ahead (these GEMMs are short and
    // latency-bound: one step ahead left most of each load's latency exposed)
    float a_r[3][4], b_r[3][4][NT];
    auto load = [&](int k, float (&av)[4], float (&bv)[4][NT]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int kk = k + 2 * i + h;
            const bool v = kk < we;
            av[i] = v ? al.load(ctx, kk, we) : 0.0f;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) bv[i][nt] = v ? bl.load(kk, n0 + nt * 32 + r, we) : 0.0f;
        }
    };
    auto step = [&](int k, auto slot_c) __attribute__((always_inline)) {
        constexpr int SL = decltype(slot_c)::value;
        if (k + 16 < we) load(k + 16, a_r[(SL + 2) % 3], b_r[(SL + 2) % 3]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
                acc[nt] = __builtin_amdgcn_mfma_f32_32x32x2f32(a_r[SL][i], b_r[SL][i][nt], acc[nt], 0, 0, 0);
    };
    if (wb < we) load(wb, a_r[0], b_r[0]);
    if (wb + 8 < we) load(wb + 8, a_r[1], b_r[1]);
    for (int k = wb; k < we; k += 24) {
        step(k, std::integral_constant<int, 0>{});
        if (k + 8 < we) step(k + 8, std::integral_constant<int, 1>{});
        if (k + 16 < we) step(k + 16, std::integral_constant<int, 2>{});
    }
    if (KW > 1) {
        // every wave parks its tile in LDS; the workgroup then sums the KW
        // copies element by element (fixed wave order: deterministic)
        float *dst = red + wave * NT * 16 * 64;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int g = 0; g < 16; ++g) dst[(nt * 16 + g) * 64 + lane] = acc[nt][g];
        __syncthreads();
        if (m0 >= M) return;
        for (int e = threadIdx.x; e < NT * 16 * 64; e += 64 * KW) {
            float v = red[e];
#pragma unroll
            for (int w = 1; w < KW; ++w) v += red[w * NT * 16 * 64 + e];
            const int nt = e >> 10, g = (e >> 6) & 15, ln = e & 63;
            ep.store1(v, m0 + acc_row(g, ln), n0 + nt * 32 + (ln & 31), (int)bid.z);
        }
        return;
    }
    if (m0 >= M) return;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ep.store(acc[nt], m0, n0 + nt * 32, lane, (int)bid.z);
}

template <int NT, int KW, class AL, class BL, class EP>
__global__ __launch_bounds__(64 * KW) void gemm_kernel(AL al, BL bl, EP ep, int M, int K, int kchunk) {
    gemm_body<NT, KW>(al, bl, ep, M, K, kchunk, blockIdx);
}

// ---------------------------------------------------------------- epilogues
struct EpBiasRelu {  // y[row][col] = relu?(acc + bias[col])
    float *y;
    const float *bias;
    int M, N, relu;
    __device__ void store1(float v, int row, int col, int) const {
        if (row >= M || col >= N) return;
        v += bias ? bias[col] : 0.0f;
        if (relu) v = v > 0.0f ? v : 0.0f;
        y[(int64_t)row * N + col] = v;
    }
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
    __device__ void store1(float v, int row, int col, int z) const {
        if (row < M && col < N) slab[(int64_t)z * M * N + (int64_t)row * N + col] = v;
    }
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
    __device__ void store1(float v, int row, int col, int) const {
        if (row >= M || col >= N) return;
        const int64_t o = (int64_t)row * N + col;
        y[o] = act[o] > 0.0f ? v : 0.0f;
    }
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

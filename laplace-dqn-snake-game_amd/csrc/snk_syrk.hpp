// snk_syrk.hpp — symmetric Gram G = X X^T on v_mfma_f32_32x32x2_f32.
//
// X is row-major [N][ld] fp32 (a row = one snapshot column of the reference's
// D, or one per-sample Jacobian row), reduction over k < K (K, ld and every
// k-range boundary multiples of 4 so a float4 never straddles the end).
// Only lower-triangle 128 x 128 tiles (bj <= bi) are launched; a mirror pass
// fills the upper triangle bit-identically.
//
// Workgroup = 4 waves, each owning a 64 x 64 quarter of the tile (2 x 2 MFMA
// tiles, 64 accumulator registers). Per 32-k stage the workgroup stages the
// 128 x 32 row blocks of both operands into LDS ([row][k], rows padded to 36
// floats: conflict-free ds_read_b128), double buffered with one barrier per
// stage; the next stage's global float4 loads are issued before the current
// stage's 64 MFMAs per wave (sched_barrier keeps them there) and land in LDS
// after them. A lane's float4 covers 4 MFMA k-steps (lane half h holds
// k = 8*kb + 4h + j at step j) identically for both operands, so the k
// permutation cancels.
//
// Accuracy: the fp32 accumulators are flushed into fp64 every 32 stages
// (1024 k), so the error is that of 1024-long fp32 dot products summed in
// fp64, independent of K (K is ~79k for the Jacobian Gram).
#pragma once
#include "snk_conv.hpp"

namespace snk {

constexpr int SY_T = 128, SY_KS = 32, SY_LD = 36, SY_FLUSH = 32;

struct SyrkLds {
    float a[2][SY_T * SY_LD];
    float b[2][SY_T * SY_LD];
};

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

struct SyrkRows {  // the 4 staging rows of this thread for one operand
    const float *p[4];
    float m[4];
};

__device__ __forceinline__ SyrkRows syrk_rows(const float *x, int64_t ld, int N, int blk, int tid) {
    SyrkRows r;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = blk * SY_T + (tid >> 3) + 32 * q;
        const bool ok = row < N;
        r.p[q] = x + (int64_t)(ok ? row : N - 1) * ld;
        r.m[q] = ok ? 1.0f : 0.0f;
    }
    return r;
}

// acc (+)= X[bi block][k0:k1] X[bj block][k0:k1]^T; with FLUSH the fp32
// accumulators are folded into accd every SY_FLUSH stages and at the end
template <bool FLUSH>
__device__ __forceinline__ void syrk_loop(const float *__restrict__ x, int64_t ld, int N, int64_t k0, int64_t k1,
                                          int bi, int bj, SyrkLds &s, f32x16 (&acc)[2][2],
                                          double (&accd)[2][2][16]) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
    const SyrkRows ra = syrk_rows(x, ld, N, bi, tid), rb = syrk_rows(x, ld, N, bj, tid);
    const int c4 = 4 * (tid & 7);
    const int sdst = (tid >> 3) * SY_LD + c4;
    const int nst = (int)((k1 - k0 + SY_KS - 1) / SY_KS);
    f32x4 va[4], vb[4];
    float km = 1.0f;
    auto issue = [&](int st) {
        const int64_t k = k0 + (int64_t)st * SY_KS + c4;
        const bool v = k < k1;
        const int64_t kk = v ? k : k0;   // k1 - k0 >= 4: the fallback float4 is in range
        km = v ? 1.0f : 0.0f;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            va[q] = *reinterpret_cast<const f32x4 *>(ra.p[q] + kk);
            vb[q] = *reinterpret_cast<const f32x4 *>(rb.p[q] + kk);
        }
    };
    auto park = [&](int buf, float kmask) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            *reinterpret_cast<f32x4 *>(&s.a[buf][sdst + 32 * q * SY_LD]) = va[q] * (ra.m[q] * kmask);
            *reinterpret_cast<f32x4 *>(&s.b[buf][sdst + 32 * q * SY_LD]) = vb[q] * (rb.m[q] * kmask);
        }
    };
    issue(0);
    park(0, km);
    __syncthreads();
    for (int st = 0; st < nst; ++st) {
        const int buf = st & 1;
        const bool more = st + 1 < nst;
        issue(more ? st + 1 : st);
        const float km_n = km;
        __builtin_amdgcn_sched_barrier(0);
        const float *pa = &s.a[buf][(wr + r) * SY_LD + 4 * h];
        const float *pb = &s.b[buf][(wc + r) * SY_LD + 4 * h];
#pragma unroll
        for (int kb = 0; kb < SY_KS / 8; ++kb) {
            const f32x4 a0 = *reinterpret_cast<const f32x4 *>(pa + kb * 8);
            const f32x4 a1 = *reinterpret_cast<const f32x4 *>(pa + 32 * SY_LD + kb * 8);
            const f32x4 b0 = *reinterpret_cast<const f32x4 *>(pb + kb * 8);
            const f32x4 b1 = *reinterpret_cast<const f32x4 *>(pb + 32 * SY_LD + kb * 8);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[j], b0[j], acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[j], b1[j], acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[j], b0[j], acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[j], b1[j], acc[1][1], 0, 0, 0);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        if (FLUSH && (st % SY_FLUSH == SY_FLUSH - 1 || !more)) {
#pragma unroll
            for (int mi = 0; mi < 2; ++mi)
#pragma unroll
                for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                    for (int g = 0; g < 16; ++g) {
                        accd[mi][ni][g] += (double)acc[mi][ni][g];
                        acc[mi][ni][g] = 0.0f;
                    }
        }
        if (more) park(buf ^ 1, km_n);
        __syncthreads();
    }
}

__device__ __forceinline__ void syrk_zero(f32x16 (&acc)[2][2]) {
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[mi][ni][g] = 0.0f;
}

enum SyrkOut { SYRK_F32 = 0, SYRK_SLAB64 = 1, SYRK_DENSE_ADD = 2 };

struct SyrkArgs {
    const float *x;
    int64_t ld, K, kchunk;   // reduction range of split z: [z*kchunk, min(K, (z+1)*kchunk))
    int N;
    int64_t ntiles;
    float *g32;              // SYRK_F32 / SYRK_DENSE_ADD: G [N][ldg]
    double *g64;             // SYRK_SLAB64: slab [z][N][N]
    int64_t ldg;
    // SYRK_DENSE_ADD: G += (x_i.x_j + 1)(z_i.z_j) + [a_i == a_j](h_i.h_j + 1)
    const float *z, *hh;
    const uint8_t *act;
    int64_t ldz;
};

template <int OUT>
__global__ __launch_bounds__(256) void syrk_kernel(SyrkArgs a) {
    __shared__ __attribute__((aligned(16))) SyrkLds s;
    int bi, bj;
    syrk_tile(syrk_xcd_remap(blockIdx.x, a.ntiles), bi, bj);
    f32x16 acc[2][2];
    double accd[2][2][16];
    syrk_zero(acc);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int g = 0; g < 16; ++g) accd[mi][ni][g] = 0.0;
    const int64_t k0 = (int64_t)blockIdx.y * a.kchunk;
    const int64_t k1 = k0 + a.kchunk < a.K ? k0 + a.kchunk : a.K;
    if (k0 < k1) syrk_loop<true>(a.x, a.ld, a.N, k0, k1, bi, bj, s, acc, accd);
    if (OUT == SYRK_DENSE_ADD) {
        // (A3 Gram + 1) * (dz1 Gram)
        syrk_zero(acc);
        syrk_loop<false>(a.z, a.ldz, a.N, 0, 64, bi, bj, s, acc, accd);
#pragma unroll
        for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int ni = 0; ni < 2; ++ni)
#pragma unroll
                for (int g = 0; g < 16; ++g) accd[mi][ni][g] = (accd[mi][ni][g] + 1.0) * (double)acc[mi][ni][g];
        syrk_zero(acc);
        syrk_loop<false>(a.hh, a.ldz, a.N, 0, 64, bi, bj, s, acc, accd);
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int wr = (wave >> 1) * 64, wc = (wave & 1) * 64;
#pragma unroll
    for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
            const int col = bj * SY_T + wc + ni * 32 + (lane & 31);
            if (col >= a.N) continue;
            const uint8_t ac = OUT == SYRK_DENSE_ADD ? a.act[col] : 0;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int row = bi * SY_T + wr + mi * 32 + acc_row(g, lane);
                if (row >= a.N) continue;
                if (OUT == SYRK_F32) {
                    a.g32[(int64_t)row * a.ldg + col] = (float)accd[mi][ni][g];
                } else if (OUT == SYRK_SLAB64) {
                    a.g64[(int64_t)blockIdx.y * a.N * a.N + (int64_t)row * a.N + col] = accd[mi][ni][g];
                } else {
                    double v = accd[mi][ni][g];
                    if (a.act[row] == ac) v += (double)acc[mi][ni][g] + 1.0;
                    float *o = a.g32 + (int64_t)row * a.ldg + col;
                    *o = (float)((double)*o + v);
                }
            }
        }
}

}  // namespace snk

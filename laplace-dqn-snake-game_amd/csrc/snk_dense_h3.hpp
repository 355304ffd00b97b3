// snk_dense_h3.hpp — Dense1 of the act forward (3136 -> 64 at 12x12) on the fp16 h3 split.
//
// The x6 form (conv_x6_kernel MODE_DENSE) split every fp32 a3 element into three bf16
// parts in registers and ran six part products per fp32 product; here A and B move as
// fp16 h / l planes and a product takes three MFMAs (snk_conv_h3.hpp):
//  * A = a3 rows (samples), fp32 from global, scaled by 2^ea[row] with
//    ea = h3_exp(max of the sample's a3), which conv_h3f_kernel's epilogue writes
//    (H3FArgs::a3max), split in registers;
//  * B = the Dense1 image pre-split by w3_split_kernel with one exponent per (position,
//    output) (its own row max), planes [kk][h | l][64 out][64 in], chunk-swizzled;
//  * each position's six MFMAs (two 32-channel k-steps x hl + lh + hh) start from zero and
//    are added into the tile's accumulator scaled by 2^-ew[kk][out] (exact: a power of two),
//    the row scale 2^-ea comes back once at the end.
// Grid: (S / 128 row blocks) x (slabs of KPZ positions), 8 waves of 16 rows (one 16-row tile,
// four 16-column tiles each); slab[z][s][o] as the x6 kernel's EPI_SLAB, summed by the head.
// B of each position (16 KB) goes through an LDS ring of 4 slots filled by LDS-DMA three
// positions ahead; A is loaded two positions ahead (the kernel is bound by the a3 stream:
// 4 waves with one position in flight moved ~3 TB/s). KPZ is a
// template constant and the position loop unrolled: straight-line code keeps the compiler's
// vmcnt waits on the A registers exact (a loop back edge merged them to waits on the newest
// loads, which also count the DMAs).
#pragma once
#include <utility>
#include "snk_conv_h3.hpp"

namespace snk {

struct DenseH3Args {
    const float *a3;       // [S][nkk * 64]
    const float *a3max;    // [S] max of each row (>= 0)
    const uint16_t *w1h;   // [nkk][2][64][64] (w3_split_kernel)
    const int *w1e;        // [nkk][64]
    float *slab;           // [nkk / KPZ][S][64]
    int S, nkk;
};
constexpr int DH3_RING = 4, DH3_SLOT = 2 * 64 * 64 * 2;   // bytes per slot: both planes of one position
// waves per workgroup (16 rows each): 8 = 128-row blocks (224 workgroups at 4096 x 7 slabs)
#ifndef DH3_WAVES
#define DH3_WAVES 8
#endif
constexpr int DH3_NT = DH3_WAVES * 64, DH3_ROWS = DH3_WAVES * 16;
// A (a3) loaded DH3_AD positions ahead (D + 1 register sets)
#ifndef DH3_AD
#define DH3_AD 2
#endif

// vector-memory ops a lane has issued after the later of A(j) (4 loads) and B(j) (1024 /
// DH3_NT LDS-DMA pieces) when position j's wait comes: prologue B0 B1 B2 (the row maxima and
// exponents) A0 .. A(D-1), then after the barrier of each step s: B(s + 3), A(s + D)
__host__ __device__ constexpr int dh3_newer(int j, int D, int KPZ) {
    constexpr int NBP = 1024 / DH3_NT;
    int t = 0, pa[64] = {}, pb[64] = {};
    for (int p = 0; p < 3 && p < KPZ; ++p) { t += NBP; pb[p] = t; }
    for (int p = 0; p < D && p < KPZ; ++p) { t += 4; pa[p] = t; }
    for (int q = 0; q < j; ++q) {
        if (q + 3 < KPZ) { t += NBP; pb[q + 3] = t; }
        if (q + D < KPZ) { t += 4; pa[q + D] = t; }
    }
    return t - (pa[j] > pb[j] ? pa[j] : pb[j]);
}

template <typename F, int... J>
__device__ __forceinline__ void dh3_for(F &&f, std::integer_sequence<int, J...>) {
    (f(std::integral_constant<int, J>{}), ...);
}

template <int KPZ>   // positions per slab; the launch guarantees nkk % KPZ == 0
__global__ __launch_bounds__(DH3_NT) void dense_h3_kernel(DenseH3Args a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t dh3_lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int z = blockIdx.y, kk0 = z * KPZ;
    const int K1 = a.nkk * 64;
    const int row0 = blockIdx.x * DH3_ROWS + wave * 16;
    // B ring: position j of the slab in slot j % DH3_RING; 1024 16-byte pieces, 2 per lane
    auto dma = [&](int j) __attribute__((always_inline)) {
        const uint16_t *src = a.w1h + (int64_t)(kk0 + j) * 2 * 4096;
        static_assert(1024 % DH3_NT == 0, "whole pieces per lane");
#pragma unroll
        for (int u = 0; u < 1024 / DH3_NT; ++u)
            __builtin_amdgcn_global_load_lds((const void *)(src + (u * DH3_NT + tid) * 8),
                                             (__attribute__((address_space(3))) void *)(dh3_lds + (j % DH3_RING) * (DH3_SLOT / 2) +
                                                                                         (u * DH3_NT + wave * 64) * 8),
                                             16, 0, 0);
    };
    // A: row row0 + r (clamped), channels 32ks + 8g .. +7 of position kk0 + j
    const int ar = min(row0 + r, a.S - 1);
    auto aload = [&](int j, f32x4 (&x)[2][2]) __attribute__((always_inline)) {
        const float *p = a.a3 + (int64_t)ar * K1 + (kk0 + j) * 64 + 8 * g;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            x[ks][0] = *reinterpret_cast<const f32x4 *>(p + 32 * ks);
            x[ks][1] = *reinterpret_cast<const f32x4 *>(p + 32 * ks + 4);
        }
    };
    // B(0..2) first: the compiler does not count LDS-DMAs in its own vmcnt waits, so a register
    // load issued before them is waited for with vmcnt(0) (which drained the A prefetches too)
#pragma unroll
    for (int p = 0; p < 3; ++p)
        if (p < KPZ) dma(p);
    const int ea = h3_exp(a.a3max[ar]);
    // the maxima of the C rows this lane writes (sample row0 + 4g + e), and the slab's B
    // exponents of its four columns, up front (a load inside the loop would be the newest
    // VMEM op at its use, and its wait would drain the A / B prefetches)
    float cm[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) cm[e] = a.a3max[min(row0 + 4 * g + e, a.S - 1)];
    int ewc[KPZ][4];
#pragma unroll
    for (int j = 0; j < KPZ; ++j)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) ewc[j][ct] = a.w1e[(kk0 + j) * 64 + ct * 16 + r];
    f32x4v acc[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) acc[ct] = f32x4v{0.f, 0.f, 0.f, 0.f};
    // issue order (vmcnt retires loads and DMAs together, in order): B(0) B(1) B(2) (above)
    // A(0) .. A(D-1), then per position j: B(j+3) A(j+D). At j, A(j) and B(j) must have landed;
    // what was issued after the later of them may stay in flight (dh3_newer, a constant per j:
    // the position loop is a fold over an index sequence)
    constexpr int D = DH3_AD < KPZ - 1 ? DH3_AD : KPZ - 1, NSET = D + 1;
    f32x4 xa[NSET][2][2];   // [set][k-step][half]
#pragma unroll
    for (int p = 0; p < D; ++p) aload(p, xa[p % NSET]);
    auto position = [&](auto jc) __attribute__((always_inline)) {
        constexpr int j = decltype(jc)::value;
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(dh3_newer(j, D, KPZ)));
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of slot (j - 1) % 4 done
        __builtin_amdgcn_s_barrier();         // every wave's pieces of B(j) landed; slot (j + 3) % 4 free
        // pinned here: left to itself the scheduler sank the prefetches behind this
        // position's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (j + 3 < KPZ) dma(j + 3);
        if constexpr (j + D < KPZ) aload(j + D, xa[(j + D) % NSET]);
        __builtin_amdgcn_sched_barrier(0);
        // A fragments: the position's 16 values per lane, scaled and split
        f16x8 ah[2], al[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            u32x2 h0, l0, h1, l1;
            h3_split4(xa[j % NSET][ks][0], ea, h0, l0);
            h3_split4(xa[j % NSET][ks][1], ea, h1, l1);
            ah[ks] = as_h(u32x4{h0[0], h0[1], h1[0], h1[1]});
            al[ks] = as_h(u32x4{l0[0], l0[1], l1[0], l1[1]});
        }
        const uint16_t *slot = dh3_lds + (j % DH3_RING) * (DH3_SLOT / 2);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            const int o = ct * 16 + r;
            const float sc = __builtin_ldexpf(1.0f, -ewc[j][ct]);
            f16x8 bh[2], bl[2];
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int off = o * 64 + (((4 * ks + g) ^ (o & 7)) << 3);
                bh[ks] = as_h(*reinterpret_cast<const u32x4 *>(slot + off));
                bl[ks] = as_h(*reinterpret_cast<const u32x4 *>(slot + 4096 + off));
            }
            f32x4v c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[ks], bl[ks], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[ks], bh[ks], c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[ks], bh[ks], c, 0, 0, 0);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e) acc[ct][e] = __builtin_fmaf(c[e], sc, acc[ct][e]);
        }
    };
    dh3_for(position, std::make_integer_sequence<int, KPZ>{});
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    // C row 4g + e = sample row0 + 4g + e, column ct*16 + r; the row scale back
    float *out = a.slab + (int64_t)z * a.S * 64;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int row = row0 + 4 * g + e;
        if (row >= a.S) continue;
        const int ex = h3_exp(cm[e]);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) out[(int64_t)row * 64 + ct * 16 + r] = __builtin_ldexpf(acc[ct][e], -ex);
    }
}

}  // namespace snk

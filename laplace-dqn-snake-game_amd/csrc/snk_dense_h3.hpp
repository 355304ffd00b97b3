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
//
// HEAD (the act forward): the act head (head_kernel<HEAD_ACT>) runs in the kernel's tail. The
// slabs go out as sc1 stores; after every wave's stores completed, one lane per workgroup counts
// on a relaxed agent-scope ticket per 128-row block, and the last of the block's gridDim.y
// workgroups (told by the value its add returned) reads the block's slabs with sc1 loads and
// runs the heads of its 128 samples, four threads per sample (no fences: see
// upd_fwd_kernel's phase 5). The head's arithmetic is head_kernel's to the bit: h = bias +
// slabs in slab order, relu, and Dense2's sums in wave_sum's butterfly order (below).
#pragma once
#include "snk_conv_h3.hpp"
#include "snk_qnet.hpp"

namespace snk {

struct DenseH3Args {
    const float *a3;       // [S][nkk * 64]
    const float *a3max;    // [S] max of each row (>= 0)
    const uint16_t *w1h;   // [nkk][2][64][64] (w3_split_kernel)
    const int *w1e;        // [nkk][64]
    float *slab;           // [nkk / KPZ][S][64]
    int S, nkk;
    // HEAD: the fused act head (head_kernel<HEAD_ACT>'s operands), ticket[S / 128] zero between launches
    uint32_t *ticket = nullptr;
    const float *theta = nullptr;
    QLayout L{};
    float *h1 = nullptr, *q = nullptr;
    HeadArgs ha{};
};

// The act head of sample s from its Dense1 slabs, thread t = 0..3 of the sample's quad (adjacent
// lanes): the thread owns outputs o = 4t + i + 16m (i, m = 0..3; f32x4 loads of each slab row).
// Dense2's sum sum_o w2[a][o] h[o] in wave_sum's order (xor butterfly 32, 16, 8, 4, 2, 1 over
// o): the 32 and 16 steps pair outputs the thread owns, 8 and 4 pair thread t with t ^ 2 and
// t ^ 1 (DPP quad permutes; both partners compute the same commutative sums), 2 and 1 are
// local again. Slab loads sc1 (the fused tail's hand-off).
__device__ __forceinline__ float quad_xchg(float v, int ctrl_xor) {
    const int o = ctrl_xor == 1 ? __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false)
                                : __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false);
    return __builtin_bit_cast(float, o);
}
__device__ __forceinline__ void act_head_quad(const float *slab, int ks, int64_t S, const float *theta, const QLayout &L,
                                              float *h1o, float *qo, const HeadArgs &ha, int64_t s, int t, bool valid) {
    constexpr int KMAX = 8;
    const int64_t sl = valid ? s : 0;
    f32x4 z[KMAX][4];
#pragma unroll
    for (int k = 0; k < KMAX; ++k)
        if (k < ks)
#pragma unroll
            for (int m = 0; m < 4; ++m) {   // two 8-byte sc1 loads (16-byte atomics are not lock-free)
                const uint64_t *p = reinterpret_cast<const uint64_t *>(slab + ((int64_t)k * S + sl) * 64 + 16 * m + 4 * t);
                const uint64_t lo = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const uint64_t hi = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                z[k][m] = f32x4{__builtin_bit_cast(float, (uint32_t)lo), __builtin_bit_cast(float, (uint32_t)(lo >> 32)),
                                __builtin_bit_cast(float, (uint32_t)hi), __builtin_bit_cast(float, (uint32_t)(hi >> 32))};
            }
    f32x4 h[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        h[m] = *reinterpret_cast<const f32x4 *>(theta + L.off_d1b + 16 * m + 4 * t);
#pragma unroll
        for (int k = 0; k < KMAX; ++k)
            if (k < ks) h[m] += z[k][m];
#pragma unroll
        for (int i = 0; i < 4; ++i) h[m][i] = h[m][i] > 0.0f ? h[m][i] : 0.0f;
    }
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float v[4];   // a2[4t + i] = (p[o] + p[o + 32]) + (p[o + 16] + p[o + 48]), o = 4t + i
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float p[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) p[m] = theta[L.off_d2w + a * 64 + 16 * m + 4 * t + i] * h[m][i];
            v[i] = (p[0] + p[2]) + (p[1] + p[3]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + quad_xchg(v[i], 2);   // o ^ 8: thread t ^ 2
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = v[i] + quad_xchg(v[i], 1);   // o ^ 4: thread t ^ 1
        const float r = (v[0] + v[2]) + (v[1] + v[3]);                      // o ^ 2, o ^ 1
        q[a] = theta[L.off_d2b + a] + r;
    }
    if (!valid) return;
#pragma unroll
    for (int m = 0; m < 4; ++m) *reinterpret_cast<f32x4 *>(h1o + s * 64 + 16 * m + 4 * t) = h[m];
    if (t != 0) return;
    qo[s * 3 + 0] = q[0];
    qo[s * 3 + 1] = q[1];
    qo[s * 3 + 2] = q[2];
    // head_kernel<HEAD_ACT> (utils.jl:161-169)
    const uint64_t tt = *ha.tptr;
    const float eps = ha.eps_dev ? *ha.eps_dev : ha.epsilon;
    const float u = rng_uniform(rng_hash(ha.seed, (uint64_t)s, tt));
    int act;
    if (u < eps) {
        act = (int)((rng_hash(ha.seed ^ 0xA5A5A5A5A5A5A5A5ULL, (uint64_t)s, tt) >> 32) % 3);
    } else {
        act = 0;   // argmax: first maximum
        if (q[1] > q[act]) act = 1;
        if (q[2] > q[act]) act = 2;
    }
    ha.act[s] = (uint8_t)act;
}
constexpr int DH3_RING = 4, DH3_SLOT = 2 * 64 * 64 * 2;   // bytes per slot: both planes of one position
constexpr int DH3_NT = 512;                                  // 8 waves x 16 rows

template <int KPZ, bool HEAD = false>   // positions per slab; the launch guarantees nkk % KPZ == 0
__global__ __launch_bounds__(DH3_NT) void dense_h3_kernel(DenseH3Args a) {
    extern __shared__ __attribute__((aligned(16))) uint16_t dh3_lds[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int z = blockIdx.y, kk0 = z * KPZ;
    const int K1 = a.nkk * 64;
    const int row0 = blockIdx.x * 128 + wave * 16;
    // B ring: position j of the slab in slot j % DH3_RING; 1024 16-byte pieces, 2 per lane
    auto dma = [&](int j) __attribute__((always_inline)) {
        const uint16_t *src = a.w1h + (int64_t)(kk0 + j) * 2 * 4096;
#pragma unroll
        for (int u = 0; u < 2; ++u)
            __builtin_amdgcn_global_load_lds((const void *)(src + (u * 512 + tid) * 8),
                                             (__attribute__((address_space(3))) void *)(dh3_lds + (j % DH3_RING) * (DH3_SLOT / 2) +
                                                                                         (u * 512 + wave * 64) * 8),
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
    // issue order (vmcnt retires loads and DMAs together, in order): B(0) A(0) B(1) A(1) B(2),
    // then per position j: A(j+2) B(j+3). At j, A(j) and everything older (B(<= j)) must have
    // landed; B(j+1), A(j+1) and B(j+2), issued after A(j), may stay in flight
    f32x4 xa[3][2][2];   // [set][k-step][half]
    dma(0);
    aload(0, xa[0]);
    if (KPZ > 1) {
        dma(1);
        aload(1, xa[1]);
    }
    if (KPZ > 2) dma(2);
#pragma unroll
    for (int j = 0; j < KPZ; ++j) {
        const int newer = (j + 1 < KPZ ? 6 : 0) + (j + 2 < KPZ ? 2 : 0);
        if (newer == 8) __builtin_amdgcn_s_waitcnt(waitcnt_vm(8));
        else if (newer == 6) __builtin_amdgcn_s_waitcnt(waitcnt_vm(6));
        else __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's reads of slot (j - 1) % 4 done
        __builtin_amdgcn_s_barrier();         // every wave's pieces of B(j) landed; slot (j + 3) % 4 free
        // pinned here: left to itself the scheduler sank the prefetches behind this
        // position's MFMAs
        __builtin_amdgcn_sched_barrier(0);
        if (j + 2 < KPZ) aload(j + 2, xa[(j + 2) % 3]);
        if (j + 3 < KPZ) dma(j + 3);
        __builtin_amdgcn_sched_barrier(0);
        // A fragments: the position's 16 values per lane, scaled and split
        f16x8 ah[2], al[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            u32x2 h0, l0, h1, l1;
            h3_split4(xa[j % 3][ks][0], ea, h0, l0);
            h3_split4(xa[j % 3][ks][1], ea, h1, l1);
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
    }
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
    // C row 4g + e = sample row0 + 4g + e, column ct*16 + r; the row scale back
    float *out = a.slab + (int64_t)z * a.S * 64;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int row = row0 + 4 * g + e;
        if (row >= a.S) continue;
        const int ex = h3_exp(cm[e]);
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
            float *o = out + (int64_t)row * 64 + ct * 16 + r;
            const float v = __builtin_ldexpf(acc[ct][e], -ex);
            if constexpr (HEAD) __hip_atomic_store(o, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // sc1
            else *o = v;
        }
    }
    if constexpr (HEAD) {
        __shared__ int s_last;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's slab stores completed
        __syncthreads();                                    // ... and every other wave's
        if (tid == 0) {
            const uint32_t old = __hip_atomic_fetch_add(a.ticket + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = old == gridDim.y - 1;
            if (s_last) __hip_atomic_store(a.ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
        if (!s_last) return;
        const int64_t sm = (int64_t)blockIdx.x * 128 + (tid >> 2);
        act_head_quad(a.slab, (int)gridDim.y, a.S, a.theta, a.L, a.h1, a.q, a.ha, sm, tid & 3, sm < a.S);
    }
}

}  // namespace snk

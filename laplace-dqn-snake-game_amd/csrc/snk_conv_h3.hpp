// snk_conv_h3.hpp — fp32-accurate conv3 of large batches on fp16 MFMA ("h3").
//
// The x6 kernels (snk_conv_x6.hpp) split each fp32 operand into three bf16
// parts and need six part products. fp16 carries 11 significant bits against
// bf16's 8, so TWO parts reach the same place: h = f16(x), l = f16(x - h)
// (x - h is exact in fp32: Sterbenz), |x - h| <= 2^-11 |x|, |x - h - l| <=
// 2^-22 |x|, and a product needs THREE MFMAs:
//   x*y ~= hl + lh + hh          (dropped: ll <= 2^-22 |xy|)
// each part product exact in the fp32 accumulator (11 x 11 bits). That is
// half the MFMA issue of x6 (v_mfma_f32_16x16x32_f16 runs at the bf16 rate),
// and A/B move as two 16-bit planes instead of three.
//
// fp16's exponent range is what bf16 did not need: the parts are taken of a
// power-of-two-scaled value, one scale per SAMPLE for the activations (its
// max |a| lands in [2^14, 2^15): no overflow, l normal down to 2^-18 of the
// max, below that an absolute error <= 2^-40 of the max) and one per TENSOR
// for the weights (the same rule on max |w| over the weight image). Both
// scales factor out of the dot product and come back exactly in the
// epilogue (one v_ldexp_f32). max |w| arrives as per-block partials that
// conv1_fwd_kernel (or wmax_scan_kernel) wrote from the same image; each
// workgroup folds them in its prologue. Activations come in as fp32 (the
// producing conv2 writes floats, 2/3 of the bytes of the x6 planes), and
// the per-sample max is a workgroup reduction over the staged samples.
//
// Error: per product <= 3 * 2^-22 relative, random in sign across the 1152
// terms of a conv3 dot product; the fp32 accumulation (shared with the x6 and
// fp32 MFMA paths) dominates. Pinned against the fp64 oracle (1e-5) and
// against the fp32-MFMA forward's own error in tests/test_qnet_gpu.py.
//
// Geometry and pipeline are conv_x6s_kernel's (four samples' inputs resident
// in LDS, sample-interleaved 16-row tiles, B double buffered per kernel
// offset with the XOR chunk swizzle); B is split in registers while it is
// staged (one float4 of the fp32 image per thread per offset).
#pragma once

#include "snk_conv_x6.hpp"
#include "snk_internal.hpp"

namespace snk {

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f16x8 as_h(const u32x4 &v) { return __builtin_bit_cast(f16x8, v); }

// s_waitcnt immediate: vmcnt(n) (LDS-DMA, loads and stores count together, in issue order),
// lgkmcnt and expcnt left at their maxima
__device__ __forceinline__ constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4) | (15 << 8); }

// e such that max * 2^e < 2^15 (>= 2^14 for a normal max); 0 for a zero or non-finite max
__device__ __forceinline__ int h3_exp(float m) {
    const uint32_t b = __float_as_uint(m) & 0x7fffffffu;
    if (b == 0 || b >= 0x7f800000u) return 0;
    return 15 - (max((int)(b >> 23), 1) - 126);
}

// four floats scaled by 2^e, split into fp16 h / l (two halves per dword, RNE)
__device__ __forceinline__ void h3_split4(const f32x4 &x, int e, u32x2 &h, u32x2 &l) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const f32x2 v{__builtin_ldexpf(x[2 * i], e), __builtin_ldexpf(x[2 * i + 1], e)};
        const f16x2 hv = __builtin_convertvector(v, f16x2);
        const f32x2 r = v - __builtin_convertvector(hv, f32x2);
        h[i] = __builtin_bit_cast(uint32_t, hv);
        l[i] = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, f16x2));
    }
}

// max over the wave, returned to every lane: DPP within each row of 16 lanes (xor 1,
// xor 2, half mirror, mirror), then the four row maxima by v_readlane. max is exact and
// order-free, so the result equals any other reduction order's (no LDS round trips,
// which the ds_bpermute form of __shfl_xor costs six of, each dependent on the last)
template <int CTRL>
__device__ __forceinline__ float dpp_max(float v) {
    const int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false);
    return fmaxf(v, __builtin_bit_cast(float, o));
}
__device__ __forceinline__ float wave_max(float v) {
    v = dpp_max<0xB1>(v);    // quad_perm [1,0,3,2]
    v = dpp_max<0x4E>(v);    // quad_perm [2,3,0,1]
    v = dpp_max<0x141>(v);   // row_half_mirror
    v = dpp_max<0x140>(v);   // row_mirror: every lane holds its row's max
    const float a = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 0));
    const float b = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 16));
    const float c = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 32));
    const float d = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 48));
    return fmaxf(fmaxf(a, b), fmaxf(c, d));
}

// partial max |w| of w[0, n): block b (256 threads) covers a grid-stride share; part[b]
// scanning block bid of nblk (a launch may hold other workgroups too)
__device__ __forceinline__ void wmax_block(const float *__restrict__ w, int64_t n, float *__restrict__ part,
                                           float *red4, int nblk, int bid) {
    float m = 0.0f;
    for (int64_t i = (int64_t)bid * 256 + threadIdx.x; i < n; i += (int64_t)nblk * 256)
        m = fmaxf(m, fabsf(w[i]));
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) part[bid] = fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
}

// rd.out: workgroup 0 runs the replay sample instead (the trainer's rider, see SampleRider)
static __global__ __launch_bounds__(256) void wmax_scan_kernel(const float *__restrict__ w, int64_t n,
                                                        float *__restrict__ part, SampleRider rd) {
    const int rb = rd.out ? 1 : 0;
    if (rb && blockIdx.x == 0) {
        if (threadIdx.x < 64) sample_wave(rd);
        return;
    }
    __shared__ float red4[4];
    wmax_block(w, n, part, red4, (int)gridDim.x - rb, (int)blockIdx.x - rb);
}

// conv3 (CK = 32 -> CN = 64, pad 0, EPI_BIAS_RELU) on the h3 split; ConvArgs:
// x = fp32 input [S][HIN^2][32], w = fp32 weight image [kk][64][32],
// wmax/nwmax = partial max |w| of that image; out (fp32) and/or outb (x6 planes)
// HIN (= board side) is a template constant: the index arithmetic of the
// staging and of the epilogue then has no integer division.
template <int KS, int EPI, int HIN>
__global__ __launch_bounds__(512) void conv_h3s_kernel(ConvPair pr, int S) {
    constexpr int CN = 64, CK = 32, NSG = 4, NB = 2 * CN * CK / 8;   // 512 16-byte chunks per offset
    constexpr int NKK = KS * KS, NLA = 11;   // A float4 loads per thread: 4 samples of <= 13 x 13 x 32
    static_assert(NB == 512 && CN * CK / 4 == 512, "one float4 of the image per thread per offset");
    const ConvArgs &a = pr.g[blockIdx.z];
    const f32x4 *__restrict__ wsrc = reinterpret_cast<const f32x4 *>(a.w);
    extern __shared__ __attribute__((aligned(16))) u32x4 h3s_lds[];
    __shared__ float red[8][5];
    u32x4 *Bs = h3s_lds;            // [2][NB]
    u32x4 *As = h3s_lds + 2 * NB;   // A image, conv_x6s_kernel's slot map with two planes per group
    u32x2 *Bs2 = reinterpret_cast<u32x2 *>(Bs);
    u32x2 *As2 = reinterpret_cast<u32x2 *>(As);
    constexpr int hin = HIN, ho = HIN - KS + 1, ho2 = ho * ho, hin2 = hin * hin;
    constexpr int XW = ho + 8, PL = (hin * XW + 3) & ~3, GG = 2 * PL, XS = 4 * GG + 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int s0 = blockIdx.x * NSG;
    const int ns = min(NSG, S - s0);

    // B register sets: set kk & 1 carries B(kk) (fp32, unsplit) from global to LDS
    f32x4 bst[2];
    auto b_load = [&](int kk, int set) { bst[set] = wsrc[(int64_t)min(kk, NKK - 1) * NB + tid]; };
    const int bch = (tid >> 3) * 4 + ((tid & 7) >> 1);   // 16-byte chunk of column tid >> 3, channels 8*(..)
    const int bhalf = tid & 1;
    int ew = 0;
    auto b_store = [&](int buf, int set) {
        u32x2 h, l;
        h3_split4(bst[set], ew, h, l);
        Bs2[(buf * NB + x6s_bswz(bch)) * 2 + bhalf] = h;
        Bs2[(buf * NB + x6s_bswz(256 + bch)) * 2 + bhalf] = l;
    };
    b_load(0, 0);
    b_load(1, 1);

    // A: the group's fp32 inputs, then one max per sample and the weight max
    constexpr int per = hin2 * 8;
    const int n4 = ns * per;
    const f32x4 *src = reinterpret_cast<const f32x4 *>(a.x) + (int64_t)s0 * per;
    f32x4 av[NLA];
#pragma unroll
    for (int u = 0; u < NLA; ++u) av[u] = src[min(u * 512 + tid, n4 - 1)];
    float wm = 0.0f;
    for (int i = tid; i < a.nwmax; i += 512) wm = fmaxf(wm, a.wmax[i]);
    float sm0 = 0.0f, sm1 = 0.0f, sm2 = 0.0f, sm3 = 0.0f;
#pragma unroll
    for (int u = 0; u < NLA; ++u) {
        const int e = u * 512 + tid;
        const int sr = e < n4 ? e / per : NSG;
        const f32x4 v = av[u];
        const float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        sm0 = sr == 0 ? fmaxf(sm0, m) : sm0;
        sm1 = sr == 1 ? fmaxf(sm1, m) : sm1;
        sm2 = sr == 2 ? fmaxf(sm2, m) : sm2;
        sm3 = sr == 3 ? fmaxf(sm3, m) : sm3;
    }
    sm0 = wave_max(sm0);
    sm1 = wave_max(sm1);
    sm2 = wave_max(sm2);
    sm3 = wave_max(sm3);
    wm = wave_max(wm);
    if (lane == 0) {
        red[wave][0] = sm0; red[wave][1] = sm1; red[wave][2] = sm2; red[wave][3] = sm3; red[wave][4] = wm;
    }
    __syncthreads();
    int ea[NSG];
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        float m = red[0][q];
#pragma unroll
        for (int w8 = 1; w8 < 8; ++w8) m = fmaxf(m, red[w8][q]);
        if (q < NSG) ea[q] = h3_exp(m);
        else ew = h3_exp(m);
    }
#pragma unroll
    for (int u = 0; u < NLA; ++u) {
        const int e = u * 512 + tid;
        if (e < n4) {
            const int sr = e / per, loc = e - sr * per;
            const int pos = loc >> 3, c4 = loc & 7;
            const int j = pos / hin, i = pos - j * hin;
            const int slot = sr * XS + (c4 >> 1) * GG + j * XW + i;
            const int es = sr == 0 ? ea[0] : sr == 1 ? ea[1] : sr == 2 ? ea[2] : ea[3];
            u32x2 h, l;
            h3_split4(av[u], es, h, l);
            As2[slot * 2 + (c4 & 1)] = h;
            As2[(slot + PL) * 2 + (c4 & 1)] = l;
        }
    }
    b_store(0, 0);
    b_store(1, 1);

    constexpr int T = (NSG * ho2 + 15) / 16;
    const int rg = wave >> 1, cg = wave & 1;
    const int nt = __builtin_amdgcn_readfirstlane(T > rg ? (T - rg + 3) / 4 : 0);
    const int bslot = (cg * 32 + r) * 4 + (g ^ ((4 - ((r >> 2) & 3)) & 3));
    __syncthreads();

    // conv_x6s_kernel's pipeline (see there): offset kk's MFMAs on fragments
    // read during kk-1, B(kk+2) split into LDS while B(kk+3) is in flight
    auto run = [&](auto ntc) {
        constexpr int NT = decltype(ntc)::value;
        int abase[NT];
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            const int q = 16 * (rg + 4 * k) + r;
            const int p = min(q >> 2, ho2 - 1), sr = q & 3;
            const int j = p / ho, i = p - j * ho;
            abase[k] = sr * XS + g * GG + j * XW + i;
        }
        f32x4v acc[NT][2];
#pragma unroll
        for (int k = 0; k < NT; ++k)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) acc[k][ct] = f32x4v{0.f, 0.f, 0.f, 0.f};
        struct Frag {
            u32x4 a[NT][2], b[2][2];
        };
        auto frag_read = [&](int kk, Frag &f) {
            kk = min(kk, NKK - 1);
            const int dv = kk / KS, du = kk - dv * KS;
            const int off = dv * XW + du;
            const u32x4 *pb = Bs + (kk & 1) * NB + bslot;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) f.b[ct][pl] = pb[ct * 64 + pl * 256];
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const u32x4 *pa = As + abase[k] + off;
#pragma unroll
                for (int pl = 0; pl < 2; ++pl) f.a[k][pl] = pa[pl * PL];
            }
        };
        auto mfma_block = [&](const Frag &f) {
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const f16x8 ah = as_h(f.a[k][0]), al = as_h(f.a[k][1]);
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const f16x8 bh = as_h(f.b[ct][0]), bl = as_h(f.b[ct][1]);
                    f32x4v c = acc[k][ct];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
                    acc[k][ct] = c;
                }
            }
        };
        auto step = [&](int kk, const Frag &cur, Frag &nxt, int set) {
            b_load(kk + 3, set ^ 1);
            frag_read(kk + 1, nxt);
            mfma_block(cur);
            b_store(kk & 1, set);
            __syncthreads();
        };
        Frag f0, f1;
        frag_read(0, f0);
        b_load(2, 0);
        __syncthreads();   // every wave has B(0) in registers before step 0 overwrites Bs[0]
        static_assert(NKK % 2 == 0, "offsets come in pairs");
        for (int kk = 0; kk < NKK; kk += 2) {
            step(kk, f0, f1, 0);
            step(kk + 1, f1, f0, 1);
        }

        // acc[k][ct][e]: tile row 4g + e = position 4t + g of sample e; column 16ct + r
        if (!a.outb) {
            // through LDS (the A image is dead after the last offset's barrier): rows of
            // CS floats (CS = 80: the two 32-lane halves of a ds_write_b32 land 16 banks
            // apart), then the group's contiguous [ns*ho2][64] block as float4 stores
            constexpr int CS = 80;
            static_assert(NSG * ho2 * CS * 4 <= 4 * XS * 16, "output staging fits the A image");
            float *Cs = reinterpret_cast<float *>(As);
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const int p = 4 * (rg + 4 * k) + g;
                if (p >= ho2) continue;
#pragma unroll
                for (int ct = 0; ct < 2; ++ct) {
                    const int col = cg * 32 + ct * 16 + r;
                    const float bv = EPI == EPI_BIAS_RELU ? a.bias[col] : 0.0f;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const float v = __builtin_ldexpf(acc[k][ct][e], -(ea[e] + ew)) + bv;
                        Cs[(e * ho2 + p) * CS + col] = v > 0.0f ? v : 0.0f;
                    }
                }
            }
            __syncthreads();
            if (a.out) {
                const int n4o = ns * ho2 * 16;
                f32x4 *o4 = reinterpret_cast<f32x4 *>(a.out + (int64_t)s0 * ho2 * CN);
                const f32x4 *c4 = reinterpret_cast<const f32x4 *>(Cs);
                for (int q = tid; q < n4o; q += 512) o4[q] = c4[(q >> 4) * (CS / 4) + (q & 15)];
            }
            return;
        }
#pragma unroll
        for (int k = 0; k < NT; ++k) {
            const int p = 4 * (rg + 4 * k) + g;
            if (p >= ho2) continue;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = cg * 32 + ct * 16 + r;
                const float bv = EPI == EPI_BIAS_RELU ? a.bias[col] : 0.0f;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    if (e >= ns) continue;
                    const int64_t row = (int64_t)(s0 + e) * ho2 + p;
                    float v = __builtin_ldexpf(acc[k][ct][e], -(ea[e] + ew)) + bv;
                    v = v > 0.0f ? v : 0.0f;
                    if (a.out) a.out[row * CN + col] = v;
                    uint16_t *pb = a.outb + row * 3 * CN + col;
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) pb[pl * CN] = split_part(v, pl);
                }
            }
        }
    };
    if (nt == 4) run(std::integral_constant<int, 4>{});
    else if (nt == 3) run(std::integral_constant<int, 3>{});
    else if (nt == 2) run(std::integral_constant<int, 2>{});
    else run(std::integral_constant<int, 1>{});
}

// conv2 (3x3, 16 -> 32, pad 1, EPI_BIAS_RELU) of a large batch on the h3 split.
// A workgroup (4 waves) owns two whole samples: their fp32 conv1 outputs are
// staged with a per-sample power-of-two scale as fp16 h/l parts into LDS inside
// a zero border ([sample][part][(BS+2)^2 positions][24 halves]: 48-byte
// position rows, conflict-free for 16 consecutive positions), and the whole
// weight tensor goes to LDS once (scale from its own max, split, paired
// offsets: k = 16 * (kk - 2p) + ci for offset pair p, the 10th offset zero).
// Each wave then runs its 16-row tiles over the 5 offset pairs on
// v_mfma_f32_16x16x32_f16 with every B fragment held in registers: no barrier
// after the staging. Output: fp32 a2 (the h3s conv3 consumes it).
template <int BS>
__global__ __launch_bounds__(256) void conv_h3c2_kernel(const float *__restrict__ x, const float *__restrict__ wimg,
                                                        const float *__restrict__ bias, float *__restrict__ out, int S) {
    constexpr int BP = BS + 2, NPB = BP * BP, NC = BS * BS, NSG = 2, XR = 24, BR = 40;
    constexpr int ROWS = NSG * NC, T = (ROWS + 15) / 16;
    constexpr int A_H = NSG * 2 * NPB * XR;          // halves of the A image
    constexpr int B_H = 5 * 2 * 32 * BR;             // halves of the B image
    extern __shared__ __attribute__((aligned(16))) uint16_t c2l[];
    uint16_t *As = c2l, *Bs = c2l + A_H;
    __shared__ float red[4][3];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int s0 = blockIdx.x * NSG, ns = min(NSG, S - s0);
    // zero the A image (borders) and the pad offset of B
    for (int q = tid; q < A_H / 8; q += 256) reinterpret_cast<u32x4 *>(As)[q] = u32x4{0, 0, 0, 0};
    for (int q = tid; q < B_H / 8; q += 256) reinterpret_cast<u32x4 *>(Bs)[q] = u32x4{0, 0, 0, 0};
    // loads: weights (9 x 32 x 16 fp32 = 1152 float4) and the two samples' a1 (2 x NC x 16 = 8*NC float4)
    constexpr int NW4 = 9 * 32 * 16 / 4, NA4 = NSG * NC * 4, LW = (NW4 + 255) / 256, LA = (NA4 + 255) / 256;
    f32x4 wv[LW], av[LA];
    const f32x4 *w4 = reinterpret_cast<const f32x4 *>(wimg);
    const f32x4 *x4 = reinterpret_cast<const f32x4 *>(x) + (int64_t)s0 * NC * 4;
    const int na4 = ns * NC * 4;
#pragma unroll
    for (int u = 0; u < LW; ++u) wv[u] = w4[min(u * 256 + tid, NW4 - 1)];
#pragma unroll
    for (int u = 0; u < LA; ++u) av[u] = x4[min(u * 256 + tid, na4 - 1)];
    float mw = 0.0f, m0 = 0.0f, m1 = 0.0f;
#pragma unroll
    for (int u = 0; u < LW; ++u) {
        const f32x4 v = wv[u];
        if (u * 256 + tid < NW4)
            mw = fmaxf(mw, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    }
#pragma unroll
    for (int u = 0; u < LA; ++u) {
        const int e = u * 256 + tid;
        const f32x4 v = av[u];
        const float m = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
        if (e < na4) {
            if (e < NC * 4) m0 = fmaxf(m0, m);
            else m1 = fmaxf(m1, m);
        }
    }
    mw = wave_max(mw);
    m0 = wave_max(m0);
    m1 = wave_max(m1);
    if (lane == 0) {
        red[wave][0] = mw; red[wave][1] = m0; red[wave][2] = m1;
    }
    __syncthreads();   // also: the zero fill is done
    const int ew = h3_exp(fmaxf(fmaxf(red[0][0], red[1][0]), fmaxf(red[2][0], red[3][0])));
    const int ea0 = h3_exp(fmaxf(fmaxf(red[0][1], red[1][1]), fmaxf(red[2][1], red[3][1])));
    const int ea1 = h3_exp(fmaxf(fmaxf(red[0][2], red[1][2]), fmaxf(red[2][2], red[3][2])));
    u32x2 *As2 = reinterpret_cast<u32x2 *>(As), *Bs2 = reinterpret_cast<u32x2 *>(Bs);
#pragma unroll
    for (int u = 0; u < LW; ++u) {   // image [kk][co][ci]: float4 e -> kk, co, ci0 = 4 * (e & 3)
        const int e = u * 256 + tid;
        if (e < NW4) {
            const int kk = e >> 7, co = (e >> 2) & 31, ci0 = 4 * (e & 3);
            const int p = kk >> 1, k0 = 16 * (kk & 1) + ci0;
            u32x2 hh, ll;
            h3_split4(wv[u], ew, hh, ll);
            Bs2[(((p * 2 + 0) * 32 + co) * BR + k0) / 4] = hh;
            Bs2[(((p * 2 + 1) * 32 + co) * BR + k0) / 4] = ll;
        }
    }
#pragma unroll
    for (int u = 0; u < LA; ++u) {   // a1 [s][pos][16]: float4 e -> sample, position, channels 4*(e & 3)
        const int e = u * 256 + tid;
        if (e < na4) {
            const int sr = e / (NC * 4), loc = e - sr * NC * 4;
            const int pos = loc >> 2, c0 = 4 * (loc & 3);
            const int j = pos / BS, i = pos - j * BS;
            const int pb = (i + 1) + (j + 1) * BP;
            u32x2 hh, ll;
            h3_split4(av[u], sr ? ea1 : ea0, hh, ll);
            As2[(((sr * 2 + 0) * NPB + pb) * XR + c0) / 4] = hh;
            As2[(((sr * 2 + 1) * NPB + pb) * XR + c0) / 4] = ll;
        }
    }
    __syncthreads();
    const int r = lane & 15, g = lane >> 4;
    // every B fragment of the layer in registers: [pair][col tile][part]
    u32x4 bf[5][2][2];
#pragma unroll
    for (int p = 0; p < 5; ++p)
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int pl = 0; pl < 2; ++pl)
                bf[p][ct][pl] = *reinterpret_cast<const u32x4 *>(Bs + ((p * 2 + pl) * 32 + ct * 16 + r) * BR + 8 * g);
    for (int t = wave; t < T; t += 4) {
        const int q = min(t * 16 + r, ROWS - 1);
        const int sr = q >= NC ? 1 : 0, pos = q - sr * NC;
        const int j = pos / BS, i = pos - j * BS;
        f32x4v acc[2] = {f32x4v{0.f, 0.f, 0.f, 0.f}, f32x4v{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            const int kk = min(2 * p + (g >> 1), 8), du = kk % 3, dv = kk / 3;
            const int pb = (i + du) + (j + dv) * BP;
            const uint16_t *pa = As + ((sr * 2) * NPB + pb) * XR + 8 * (g & 1);
            const f16x8 ah = as_h(*reinterpret_cast<const u32x4 *>(pa));
            const f16x8 al = as_h(*reinterpret_cast<const u32x4 *>(pa + NPB * XR));
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                f32x4v c = acc[ct];
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, as_h(bf[p][ct][0]), c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, as_h(bf[p][ct][1]), c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, as_h(bf[p][ct][0]), c, 0, 0, 0);
                acc[ct] = c;
            }
        }
        // acc[ct][e]: row 4g + e of the tile, column 16 ct + r
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int row = t * 16 + 4 * g + e;
            if (row >= ns * NC) continue;
            const int es = (row >= NC ? ea1 : ea0) + ew;
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                const int col = ct * 16 + r;
                const float v = __builtin_ldexpf(acc[ct][e], -es) + bias[col];
                out[((int64_t)s0 * NC + row) * 32 + col] = v > 0.0f ? v : 0.0f;
            }
        }
    }
}
template <int BS>
static inline size_t conv_h3c2_lds() {
    return (size_t)(2 * 2 * (BS + 2) * (BS + 2) * 24 + 5 * 2 * 32 * 40) * sizeof(uint16_t);
}

// dynamic LDS bytes of conv_h3s_kernel for an HIN x HIN input (0: does not fit)
static inline size_t conv_h3s_lds(int hin) {
    const int ho = hin - 5, XW = ho + 8, PL = (hin * XW + 3) & ~3, XS = 8 * PL + 4;
    const size_t b = (size_t)(2 * 512 + 4 * XS) * 16;
    return (ho >= 1 && hin <= 13 && (4 * ho * ho + 15) / 16 <= 16 && b <= 160 * 1024) ? b : 0;
}

}  // namespace snk

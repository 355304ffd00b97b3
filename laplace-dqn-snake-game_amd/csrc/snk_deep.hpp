// snk_deep.hpp — the deeper bf16 Q-net of BASELINE.json configs[2] on gfx950.
//
// configs[2] names "65536 envs, 20x20 grid, deeper conv Q-net, bf16" with no
// reference counterpart (builder-defined). The net extends
// structs.jl:127-139 by one more 3x3 convolution and wider channels, with the
// same Flux conventions (true convolution, column-major flatten):
//   L0 Conv(3,3,C=>32,relu;pad=1)  L1 Conv(3,3,32=>32,relu;pad=1)
//   L2 Conv(3,3,32=>64,relu;pad=1) L3 Conv(6,6,64=>64,relu)
//   flatten -> Dense((bs-5)^2*64 => 64, relu) -> Dense(64 => 3)
// bf16 semantics (oracle/snake_oracle.c restates them exactly): conv and
// Dense1 weight matrices are used rounded to bf16, every conv output (after
// bias + relu) is stored as bf16, sums accumulate in fp32 on the matrix cores;
// biases, Dense2, the TD target / Huber head and RMSProp stay fp32 (fp64 for
// the target, as the reference). Backward: native bf16 MFMA products with the
// relu-masked gradient rounded to bf16 as the operand, fp32 accumulation.
//
// Forward kernels (activations [sample][position p = i + j*H][channel] bf16):
//   deep_conv0_kernel  L0 on VALU (K = 9C): boards -> bf16
//   deep_conv_kernel   L1..L3: one sample per workgroup, its whole input
//                      staged in LDS inside a zero border, the layer's weights
//                      streamed per kernel offset through a double-buffered
//                      LDS tile, v_mfma_f32_16x16x32_bf16
//   deep_dense1_kernel Dense1 on v_mfma_f32_16x16x32_bf16, K-split slabs the
//                      shared head kernel sums (snk_qnet.hip head_launch)
// Backward: gemm_bf16_kernel, the snk_gemm.hpp engine on
//   v_mfma_f32_32x32x16_bf16 with the snk_loaders.hpp implicit-im2col loaders.
#pragma once
#include "snk_conv_x6.hpp"
#include "snk_loaders.hpp"

namespace snk {

// ---------------------------------------------------------------- bf16
__host__ __device__ inline uint16_t f2bf(float f) {   // round to nearest even
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)(u >> 16);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (uint16_t)(u >> 16);
}
__host__ __device__ inline float bf2f(uint16_t b) {
    const uint32_t u = (uint32_t)b << 16;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// ---------------------------------------------------------------- layout
struct DeepLayout {
    int bs, C, Wo, K1;                         // K1 = Wo^2 * 64 (Dense1 fan-in)
    int cin[4], cout[4], ks[4], pad[4];
    int64_t off_w[4], off_b[4], off_d1w, off_d1b, off_d2w, off_d2b, P;
    // bf16 weight image: conv L1..L3 [kk][co][ci], Dense1 [o][f]; L0 as
    // bf16-rounded fp32 [9C][32] (VALU)
    int64_t img_w[4], img_d1, img_n;
    int64_t img0_n;                            // floats of the L0 image
};
DeepLayout deep_layout(int bs, int C);
// a QLayout whose head offsets (off_d1b, off_d2w, off_d2b) and P are the deep
// net's: what the shared head / Dense2-gradient kernels read
QLayout deep_head_layout(const DeepLayout &D);
void deep_packed_to_flux(const DeepLayout &D, int32_t *perm);

// ---------------------------------------------------------------- weight image
__global__ void deep_image_kernel(const float *__restrict__ th, uint16_t *__restrict__ img,
                                  float *__restrict__ img0, DeepLayout D) {
    const int64_t n = D.img_n + D.img0_n;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        if (t >= D.img_n) {   // L0: [9C][32] weights then 32 biases, weights bf16-rounded
            const int64_t u = t - D.img_n;
            const int64_t nw = 9LL * D.C * 32;
            img0[u] = u < nw ? bf2f(f2bf(th[D.off_w[0] + u])) : th[D.off_b[0] + (u - nw)];
            continue;
        }
        if (t >= D.img_d1) {   // Dense1 [o][f] <- packed W[f][o]
            const int64_t u = t - D.img_d1;
            const int64_t o = u / D.K1, f = u - o * D.K1;
            img[t] = f2bf(th[D.off_d1w + f * 64 + o]);
            continue;
        }
        int l = 1;
        while (l < 3 && t >= D.img_w[l + 1]) ++l;
        const int64_t u = t - D.img_w[l];
        const int CI = D.cin[l], CO = D.cout[l];
        const int64_t kk = u / (CI * CO);
        const int r = (int)(u - kk * CI * CO);
        const int co = r / CI, ci = r - co * CI;
        img[t] = f2bf(th[D.off_w[l] + (kk * CI + ci) * CO + co]);   // packed W[(kk*CI + ci)*CO + co]
    }
}

// ---------------------------------------------------------------- L0 (VALU)
// 3x3, C -> 32, pad 1: NS samples per workgroup staged as floats inside a zero
// border; one thread per output position, 32 accumulators, bf16 out (4 x 16 B).
template <int C>
__global__ __launch_bounds__(256) void deep_conv0_kernel(BoardSrc src, const float *__restrict__ img0,
                                                         uint16_t *__restrict__ y, int64_t S, int bs, int NS) {
    extern __shared__ __attribute__((aligned(16))) float d0sm[];
    float *sw = d0sm;                       // [9C][32] + [32]
    float *sx = d0sm + 9 * C * 32 + 32;     // [NS][C][(bs+2)^2]
    const int bp = bs + 2, plane = bp * bp, nc = bs * bs;
    for (int i = threadIdx.x; i < 9 * C * 32 + 32; i += blockDim.x) sw[i] = img0[i];
    const int64_t s0 = (int64_t)blockIdx.x * NS;
    const int ns = (int)min((int64_t)NS, S - s0);
    for (int i = threadIdx.x; i < NS * C * plane; i += blockDim.x) sx[i] = 0.0f;
    __syncthreads();
    for (int e = threadIdx.x; e < ns * C * nc; e += blockDim.x) {
        const int sc = e / nc, cell = e - sc * nc;
        const int sl = sc / C, c = sc - sl * C;
        const int jj = cell / bs, ii = cell - jj * bs;
        sx[sc * plane + (ii + 1) + (jj + 1) * bp] = src.load(s0 + sl, c, cell);
    }
    __syncthreads();
    const float4 *sw4 = reinterpret_cast<const float4 *>(sw);
    for (int q = threadIdx.x; q < ns * nc; q += blockDim.x) {
        const int sl = q / nc, p = q - sl * nc;
        const int j = p / bs, i = p - j * bs;
        float acc[32];
#pragma unroll
        for (int v4 = 0; v4 < 8; ++v4) {
            const float4 b4 = sw4[9 * C * 8 + v4];
            acc[4 * v4] = b4.x; acc[4 * v4 + 1] = b4.y; acc[4 * v4 + 2] = b4.z; acc[4 * v4 + 3] = b4.w;
        }
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int du = kk % 3, dv = kk / 3;
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float v = sx[(sl * C + c) * plane + (i + du) + (j + dv) * bp];
#pragma unroll
                for (int v4 = 0; v4 < 8; ++v4) {
                    const float4 w4 = sw4[(kk * C + c) * 8 + v4];
                    acc[4 * v4] = __builtin_fmaf(v, w4.x, acc[4 * v4]);
                    acc[4 * v4 + 1] = __builtin_fmaf(v, w4.y, acc[4 * v4 + 1]);
                    acc[4 * v4 + 2] = __builtin_fmaf(v, w4.z, acc[4 * v4 + 2]);
                    acc[4 * v4 + 3] = __builtin_fmaf(v, w4.w, acc[4 * v4 + 3]);
                }
            }
        }
        u32x4 o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            uint32_t w[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const float a = fmaxf(acc[8 * k + 2 * e], 0.f), b = fmaxf(acc[8 * k + 2 * e + 1], 0.f);
                w[e] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
            }
            o[k] = u32x4{w[0], w[1], w[2], w[3]};
        }
        u32x4 *dst = reinterpret_cast<u32x4 *>(y + ((s0 + sl) * nc + p) * 32);
#pragma unroll
        for (int k = 0; k < 4; ++k) dst[k] = o[k];
    }
}

// ---------------------------------------------------------------- L1..L3 (MFMA)
// One workgroup = one sample, NW waves. LDS: the sample's input [HB][HB][CIN]
// bf16 at a CST = CIN + 8 position stride (16-byte A reads of 16 consecutive
// positions land on distinct banks), the zero border written explicitly; the
// weights of one kernel offset [COUT][CIN + 8] double buffered, the next
// offset's tile loaded into registers during this offset's MFMAs (one barrier
// per offset). Wave w owns row tiles w, w + NW, ... of the HO^2 output
// positions, all COUT / 16 column tiles: per offset and 32-channel chunk one
// B fragment per column tile, then per row tile one A fragment and COUT / 16
// MFMAs. Epilogue: bias + relu + bf16, straight to [S][HO^2][COUT].
template <int CIN, int COUT, int KS, int PAD, int H>
struct DeepConvShape {
    static constexpr int HB = H + 2 * PAD, HO = H + 2 * PAD - KS + 1, CST = CIN + 8, BST = CIN + 8;
    static constexpr int M = HO * HO, TILES = (M + 15) / 16, NT = COUT / 16, KC = CIN / 32;
    static constexpr int A_ELEMS = HB * HB * CST, B_ELEMS = COUT * BST;
    static constexpr int LDS = (A_ELEMS + 2 * B_ELEMS) * 2;
    static constexpr int BCH = COUT * CIN / 8;   // 16-byte chunks of one offset's weights
};

template <int CIN, int COUT, int KS, int PAD, int H, int NW>
__global__ __launch_bounds__(64 * NW) void deep_conv_kernel(const uint16_t *__restrict__ x,
                                                            const uint16_t *__restrict__ wimg,
                                                            const float *__restrict__ bias,
                                                            uint16_t *__restrict__ y) {
    using Sh = DeepConvShape<CIN, COUT, KS, PAD, H>;
    constexpr int HB = Sh::HB, HO = Sh::HO, CST = Sh::CST, BST = Sh::BST, M = Sh::M, NT = Sh::NT, KC = Sh::KC;
    constexpr int TPW = (Sh::TILES + NW - 1) / NW;
    constexpr int NTH = 64 * NW, BPT = (Sh::BCH + NTH - 1) / NTH;
    extern __shared__ __attribute__((aligned(16))) uint16_t dsm[];
    uint16_t *As = dsm;
    uint16_t *Bs = dsm + Sh::A_ELEMS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int64_t s = blockIdx.x;
    // ---- stage the input (interior) and zero the border positions
    {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(x + s * (int64_t)H * H * CIN);
        constexpr int NCH = H * H * CIN / 8, CPP = CIN / 8;
        for (int q = tid; q < NCH; q += NTH) {
            const int p = q / CPP, part = q - p * CPP;
            const int jj = p / H, ii = p - jj * H;
            *reinterpret_cast<u32x4 *>(As + ((ii + PAD) + (jj + PAD) * HB) * CST + part * 8) = src[q];
        }
        if constexpr (PAD > 0) {
            constexpr int NB = HB * HB - H * H;   // border positions
            const u32x4 z = {0u, 0u, 0u, 0u};
            for (int q = tid; q < NB * CPP; q += NTH) {
                const int b = q / CPP, part = q - b * CPP;
                int bi, bj;   // b enumerates the top row, the bottom row, then the left/right columns
                if (b < HB) { bi = b; bj = 0; }
                else if (b < 2 * HB) { bi = b - HB; bj = HB - 1; }
                else { const int t = b - 2 * HB; bj = 1 + (t >> 1); bi = (t & 1) ? HB - 1 : 0; }
                *reinterpret_cast<u32x4 *>(As + (bi + bj * HB) * CST + part * 8) = z;
            }
        }
    }
    // ---- stage offset 0's weights
    u32x4 breg[BPT];
    auto bload = [&](int kk) {
        const u32x4 *src = reinterpret_cast<const u32x4 *>(wimg + (int64_t)kk * COUT * CIN);
#pragma unroll
        for (int u = 0; u < BPT; ++u) {
            const int q = tid + u * NTH;
            if (q < Sh::BCH) breg[u] = src[q];
        }
    };
    auto bstore = [&](int buf) {
        uint16_t *dst = Bs + buf * Sh::B_ELEMS;
#pragma unroll
        for (int u = 0; u < BPT; ++u) {
            const int q = tid + u * NTH;
            if (q < Sh::BCH) {
                const int co = q / (CIN / 8), part = q - co * (CIN / 8);
                *reinterpret_cast<u32x4 *>(dst + co * BST + part * 8) = breg[u];
            }
        }
    };
    bload(0);
    bstore(0);
    // ---- per row tile: bordered base position of this lane's A row
    int abase[TPW];
#pragma unroll
    for (int t = 0; t < TPW; ++t) {
        int row = (wave + t * NW) * 16 + r;
        row = row < M ? row : M - 1;
        const int j = row / HO, i = row - j * HO;
        abase[t] = (i + j * HB) * CST + g * 8;
    }
    f32x4 acc[TPW][NT];
#pragma unroll
    for (int t = 0; t < TPW; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    for (int kk = 0; kk < KS * KS; ++kk) {
        if (kk + 1 < KS * KS) bload(kk + 1);
        const int du = kk % KS, dv = kk / KS;
        const int koff = (du + dv * HB) * CST;
        const uint16_t *Bc = Bs + (kk & 1) * Sh::B_ELEMS + r * BST + g * 8;
#pragma unroll
        for (int c = 0; c < KC; ++c) {
            bf16x8 bf[NT];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) bf[nt] = as_bf(*reinterpret_cast<const u32x4 *>(Bc + nt * 16 * BST + c * 32));
#pragma unroll
            for (int t = 0; t < TPW; ++t) {
                if ((wave + t * NW) < Sh::TILES) {
                    const bf16x8 a = as_bf(*reinterpret_cast<const u32x4 *>(As + abase[t] + koff + c * 32));
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bf[nt], acc[t][nt], 0, 0, 0);
                }
            }
        }
        if (kk + 1 < KS * KS) bstore((kk + 1) & 1);
        __syncthreads();
    }
    // ---- epilogue: C[row 4g + e][col nt*16 + r]
    uint16_t *ys = y + s * (int64_t)M * COUT;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int col = nt * 16 + r;
        const float b = bias[col];
#pragma unroll
        for (int t = 0; t < TPW; ++t) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int row = (wave + t * NW) * 16 + 4 * g + e;
                if (row < M) ys[row * COUT + col] = f2bf(fmaxf(acc[t][nt][e] + b, 0.f));
            }
        }
    }
}

// ---------------------------------------------------------------- L0..L2 fused (MFMA)
// deep_front_kernel: L0 -> L1 -> L2 of one sample at a time inside one
// workgroup, the activations never leaving LDS. Persistent: one workgroup per
// CU (151 KB of LDS at 20x20) walks samples blockIdx.x, + gridDim.x, ...; the
// L0, L1 and L2 weight images are staged into LDS once per workgroup.
// LDS (halves): W1 [9][32 co][ST], W2 [9][64 co][ST], W0 [32 co][ST] (k < 9C,
// zero above), X0 / X1 the bordered L0 / L1 outputs [(H+2)^2][ST], BD the
// bordered boards [C][(H+2)^2] bf16; ST = 40 halves per row (32 + 8 pad: the
// 16-byte fragment reads of 16 consecutive rows land on distinct bank quads).
// Every MFMA is v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand
// (rows = output channels) and the activations as B (columns = positions), so a
// lane's accumulator holds 4 consecutive channels of one position: the
// epilogues store 8 bytes per lane. Work split: row tile t (16 positions) goes
// to SIMD t % 4 (waves w and w + 4 share a SIMD): L0 wave half h = w >> 2 takes
// column tile h of the SIMD's tiles; L1 the two halves split the SIMD's tiles,
// both column tiles each; L2 both halves run all the SIMD's tiles, column tiles
// 2h, 2h + 1 each. At 20x20: 25 tiles = 7/6/6/6 per SIMD.
// L0 on the matrix cores: the boards (-1 .. 2) and the bf16-rounded weights are
// exact bf16, so every product is exact; only the fp32 summation order differs
// from the VALU form (bias added last).
// KEEP: also store the L0 / L1 outputs (the training forward's backward reads
// them); L2's output always goes to a2 [S][H^2][64].
template <int H>
struct DeepFrontShape {
    static constexpr int HB = H + 2, M = H * H, TILES = (M + 15) / 16, TPS = (TILES + 3) / 4, HALF = (TPS + 1) / 2;
    static constexpr int ST = 40;
    static constexpr int W1 = 9 * 32 * ST, W2 = 9 * 64 * ST, W0 = 32 * ST, X = HB * HB * ST, BD = 2 * HB * HB;
    static constexpr int LDS = (W1 + W2 + W0 + 2 * X + BD) * 2;
};

template <int C, int H, bool KEEP>
__global__ __launch_bounds__(512) void deep_front_kernel(BoardSrc src, const float *__restrict__ img0,
                                                         const uint16_t *__restrict__ wimg1,
                                                         const float *__restrict__ bias1,
                                                         const uint16_t *__restrict__ wimg2,
                                                         const float *__restrict__ bias2, uint16_t *__restrict__ a0,
                                                         uint16_t *__restrict__ a1, uint16_t *__restrict__ a2,
                                                         int64_t S) {
    using Sh = DeepFrontShape<H>;
    constexpr int HB = Sh::HB, M = Sh::M, TILES = Sh::TILES, TPS = Sh::TPS, HALF = Sh::HALF, ST = Sh::ST;
    constexpr int PL = HB * HB, NBV = (C * M + 511) / 512;
    static_assert(9 * C <= 32, "L0 fan-in beyond one k step");
    extern __shared__ __attribute__((aligned(16))) uint16_t fsm[];
    uint16_t *W1s = fsm, *W2s = W1s + Sh::W1, *W0s = W2s + Sh::W2, *X0 = W0s + Sh::W0, *X1 = X0 + Sh::X,
             *BD = X1 + Sh::X;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4, simd = wave & 3, half = wave >> 2;
    // ---- weights, zero borders
    for (int q = tid; q < 9 * 32 * 4; q += 512)
        *reinterpret_cast<u32x4 *>(W1s + (q >> 2) * ST + (q & 3) * 8) = reinterpret_cast<const u32x4 *>(wimg1)[q];
    for (int q = tid; q < 9 * 64 * 4; q += 512)
        *reinterpret_cast<u32x4 *>(W2s + (q >> 2) * ST + (q & 3) * 8) = reinterpret_cast<const u32x4 *>(wimg2)[q];
    for (int q = tid; q < 32 * 32; q += 512) {
        const int co = q >> 5, k = q & 31;
        W0s[co * ST + k] = k < 9 * C ? f2bf(img0[k * 32 + co]) : (uint16_t)0;
    }
    for (int q = tid; q < (2 * Sh::X + Sh::BD) / 8; q += 512)   // X0, X1, BD are contiguous
        *reinterpret_cast<u32x4 *>(X0 + q * 8) = u32x4{0u, 0u, 0u, 0u};
    // per-lane biases of the channels this lane's accumulators hold (4g + e of a column tile)
    float b0[4], b1[2][4], b2[2][4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        b0[e] = img0[9 * C * 32 + half * 16 + 4 * g + e];
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) {
            b1[c2][e] = bias1[c2 * 16 + 4 * g + e];
            b2[c2][e] = bias2[(2 * half + c2) * 16 + 4 * g + e];
        }
    }
    // bordered base of this lane's position in row tile t (clamped past M)
    auto xbase = [&](int t) __attribute__((always_inline)) {
        const int p = min(t * 16 + r, M - 1);
        return ((p % H) + (p / H) * HB) * ST + 8 * g;
    };
    auto pack4 = [](const f32x4 &v, const float (&b)[4]) __attribute__((always_inline)) {
        u32x2 o;
        o[0] = (uint32_t)f2bf(fmaxf(v[0] + b[0], 0.f)) | ((uint32_t)f2bf(fmaxf(v[1] + b[1], 0.f)) << 16);
        o[1] = (uint32_t)f2bf(fmaxf(v[2] + b[2], 0.f)) | ((uint32_t)f2bf(fmaxf(v[3] + b[3], 0.f)) << 16);
        return o;
    };
    float bv[NBV];
    auto bload = [&](int64_t s) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < NBV; ++u) {
            const int e = tid + u * 512;
            if (e < C * M) bv[u] = src.load(s, e / M, e % M);
        }
    };
    int64_t s = blockIdx.x;
    if (s < S) bload(s);
    __syncthreads();
    for (; s < S; s += gridDim.x) {
#pragma unroll
        for (int u = 0; u < NBV; ++u) {
            const int e = tid + u * 512;
            if (e < C * M) {
                const int c = e / M, cell = e % M;
                BD[c * PL + (cell % H + 1) + (cell / H + 1) * HB] = f2bf(bv[u]);
            }
        }
        __syncthreads();   // boards in; X0 free (last read by the previous sample's L1)
        // ---- L0: column tile `half` of the SIMD's row tiles
        {
            const bf16x8 wa = as_bf(*reinterpret_cast<const u32x4 *>(W0s + (half * 16 + r) * ST + 8 * g));
#pragma unroll
            for (int i = 0; i < TPS; ++i) {
                const int t = simd + 4 * i;
                if (t >= TILES) continue;
                const int pr = t * 16 + r, p = min(pr, M - 1), pi = p % H, pj = p / H;
                uint32_t w[4];
#pragma unroll
                for (int e2 = 0; e2 < 4; ++e2) {
                    uint32_t v2 = 0;
#pragma unroll
                    for (int o = 0; o < 2; ++o) {
                        const int k = 8 * g + 2 * e2 + o;
                        const int kk = k / C, c = k - kk * C;
                        const uint32_t v = k < 9 * C ? BD[c * PL + (pi + kk % 3) + (pj + kk / 3) * HB] : 0u;
                        v2 |= v << (16 * o);
                    }
                    w[e2] = v2;
                }
                const f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, as_bf(u32x4{w[0], w[1], w[2], w[3]}),
                                                                          f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
                if (pr < M) {
                    const u32x2 o = pack4(acc, b0);
                    *reinterpret_cast<u32x2 *>(X0 + ((pi + 1) + (pj + 1) * HB) * ST + half * 16 + 4 * g) = o;
                    if (KEEP) *reinterpret_cast<u32x2 *>(a0 + (s * M + pr) * 32 + half * 16 + 4 * g) = o;
                }
            }
        }
        __syncthreads();
        // ---- L1: this half's share of the SIMD's row tiles, both column tiles
        {
            f32x4 acc[HALF][2];
            int xb[HALF];
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii) {
                xb[ii] = xbase(simd + 4 * (half * HALF + ii));
                acc[ii][0] = acc[ii][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll 1
            for (int kk = 0; kk < 9; ++kk) {
                const int koff = ((kk % 3) + (kk / 3) * HB) * ST;
                bf16x8 wa[2];
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    wa[c2] = as_bf(*reinterpret_cast<const u32x4 *>(W1s + (kk * 32 + c2 * 16 + r) * ST + 8 * g));
#pragma unroll
                for (int ii = 0; ii < HALF; ++ii) {
                    const int i = half * HALF + ii, t = simd + 4 * i;
                    if (i >= TPS || t >= TILES) continue;
                    const bf16x8 xv = as_bf(*reinterpret_cast<const u32x4 *>(X0 + xb[ii] + koff));
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                        acc[ii][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[c2], xv, acc[ii][c2], 0, 0, 0);
                }
            }
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii) {
                const int i = half * HALF + ii, t = simd + 4 * i, pr = t * 16 + r;
                if (i >= TPS || t >= TILES || pr >= M) continue;
                const int pi = pr % H, pj = pr / H;
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2) {
                    const u32x2 o = pack4(acc[ii][c2], b1[c2]);
                    *reinterpret_cast<u32x2 *>(X1 + ((pi + 1) + (pj + 1) * HB) * ST + c2 * 16 + 4 * g) = o;
                    if (KEEP) *reinterpret_cast<u32x2 *>(a1 + (s * M + pr) * 32 + c2 * 16 + 4 * g) = o;
                }
            }
        }
        __syncthreads();
        if (s + gridDim.x < S) bload(s + gridDim.x);   // the next sample's boards, in flight through L2
        // ---- L2: all the SIMD's row tiles, column tiles 2*half, 2*half + 1
        {
            f32x4 acc[TPS][2];
            int xb[TPS];
#pragma unroll
            for (int i = 0; i < TPS; ++i) {
                xb[i] = xbase(simd + 4 * i);
                acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
#pragma unroll 1
            for (int kk = 0; kk < 9; ++kk) {
                const int koff = ((kk % 3) + (kk / 3) * HB) * ST;
                bf16x8 wa[2];
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    wa[c2] = as_bf(*reinterpret_cast<const u32x4 *>(W2s + (kk * 64 + (2 * half + c2) * 16 + r) * ST + 8 * g));
#pragma unroll
                for (int i = 0; i < TPS; ++i) {
                    if (simd + 4 * i >= TILES) continue;
                    const bf16x8 xv = as_bf(*reinterpret_cast<const u32x4 *>(X1 + xb[i] + koff));
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                        acc[i][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[c2], xv, acc[i][c2], 0, 0, 0);
                }
            }
#pragma unroll
            for (int i = 0; i < TPS; ++i) {
                const int pr = (simd + 4 * i) * 16 + r;
                if (simd + 4 * i >= TILES || pr >= M) continue;
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    *reinterpret_cast<u32x2 *>(a2 + (s * M + pr) * 64 + (2 * half + c2) * 16 + 4 * g) =
                        pack4(acc[i][c2], b2[c2]);
            }
        }
    }
}

// ---------------------------------------------------------------- L3 (MFMA, two samples)
// deep_conv3_kernel: L3 (6x6, 64 -> 64, valid) for TWO samples per step of a
// persistent workgroup (one per CU, 8 waves), so each kernel offset's 8 KB of
// weights, staged through LDS, serves both: the weight stream from L2 is half
// of deep_conv_kernel's one-sample form (295 KB per sample there). LDS: the
// pair's inputs [2][H*H][72] (115 KB at 20x20) and the weights of two offsets
// [co][72] double buffered. The 2*WO^2 output positions of the pair are packed
// into row tiles of 16 across the samples (29 tiles at 20x20 instead of 2 x 15);
// row tile t goes to SIMD t % 4, wave half h takes column tiles 2h, 2h + 1.
// The NEXT pair's inputs are loaded into registers during the first offsets of
// this pair (one 16-byte piece per thread per offset, behind that offset's
// weight load) and parked in LDS after the last offset's barrier.
// MFMA operands as deep_front_kernel: weights A (rows = channels), activations
// B, 8-byte epilogue stores of 4 channels.
template <int H>
struct DeepL3Shape {
    static constexpr int WO = H - 5, MS = WO * WO, M = 2 * MS, TILES = (M + 15) / 16, TPS = (TILES + 3) / 4;
    static constexpr int CST = 72, XS = H * H * CST, B_ELEMS = 64 * CST;
    static constexpr int LDS = (2 * XS + 2 * B_ELEMS) * 2;
    static constexpr int APIECES = 2 * H * H * 8, APT = (APIECES + 511) / 512;
};

template <int H>
__global__ __launch_bounds__(512) void deep_conv3_kernel(const uint16_t *__restrict__ x,
                                                         const uint16_t *__restrict__ wimg,
                                                         const float *__restrict__ bias, uint16_t *__restrict__ y,
                                                         int64_t S) {
    using Sh = DeepL3Shape<H>;
    constexpr int WO = Sh::WO, MS = Sh::MS, M = Sh::M, TILES = Sh::TILES, TPS = Sh::TPS, CST = Sh::CST;
    constexpr int XS = Sh::XS, APT = Sh::APT, APIECES = Sh::APIECES;
    static_assert(APT <= 36, "input prefetch spans more offsets than the layer has");
    extern __shared__ __attribute__((aligned(16))) uint16_t l3sm[];
    uint16_t *As = l3sm, *Bs = l3sm + 2 * XS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, g = lane >> 4, simd = wave & 3, half = wave >> 2;
    const int64_t npairs = (S + 1) / 2;
    // input piece q of pair p: sample 2p + q / (H*H*8) (clamped to S - 1), position, 16-byte chunk
    auto apiece = [&](int64_t p, int u) __attribute__((always_inline)) {
        const int q = tid + u * 512;
        const int smp = q / (H * H * 8), rem = q - smp * (H * H * 8);
        const int64_t sg = min(2 * p + smp, S - 1);
        return *reinterpret_cast<const u32x4 *>(x + (sg * H * H + (rem >> 3)) * 64 + (rem & 7) * 8);
    };
    auto apark = [&](int u, const u32x4 &v) __attribute__((always_inline)) {
        const int q = tid + u * 512;
        const int smp = q / (H * H * 8), rem = q - smp * (H * H * 8);
        *reinterpret_cast<u32x4 *>(As + smp * XS + (rem >> 3) * CST + (rem & 7) * 8) = v;
    };
    // one offset's weights: 512 pieces of 16 bytes, one per thread
    auto bload = [&](int kk) __attribute__((always_inline)) {
        return reinterpret_cast<const u32x4 *>(wimg + (int64_t)kk * 64 * 64)[tid];
    };
    auto bstore = [&](int buf, const u32x4 &v) __attribute__((always_inline)) {
        *reinterpret_cast<u32x4 *>(Bs + buf * Sh::B_ELEMS + (tid >> 3) * CST + (tid & 7) * 8) = v;
    };
    float bb[2][4];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2)
#pragma unroll
        for (int e = 0; e < 4; ++e) bb[c2][e] = bias[(2 * half + c2) * 16 + 4 * g + e];
    // this lane's A row base per row tile (position packed across the pair, clamped past M)
    int abase[TPS];
#pragma unroll
    for (int i = 0; i < TPS; ++i) {
        const int q = min((simd + 4 * i) * 16 + r, M - 1);
        const int smp = q / MS, o = q - smp * MS;
        abase[i] = smp * XS + ((o % WO) + (o / WO) * H) * CST + 8 * g;
    }
    int64_t p = blockIdx.x;
    if (p < npairs) {
#pragma unroll
        for (int u = 0; u < APT; ++u)
            if (tid + u * 512 < APIECES) apark(u, apiece(p, u));
        bstore(0, bload(0));
    }
    __syncthreads();
    for (; p < npairs; p += gridDim.x) {
        const bool more = p + gridDim.x < npairs;
        u32x4 apf[APT];
        f32x4 acc[TPS][2];
#pragma unroll
        for (int i = 0; i < TPS; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
        for (int kk = 0; kk < 36; ++kk) {
            const u32x4 bn = bload(kk + 1 < 36 ? kk + 1 : 0);   // the next offset (offset 0 of the next pair)
#pragma unroll
            for (int u = 0; u < APT; ++u)
                if (u == kk && more && tid + u * 512 < APIECES) apf[u] = apiece(p + gridDim.x, u);
            const int koff = ((kk % 6) + (kk / 6) * H) * CST;
            const uint16_t *Bc = Bs + (kk & 1) * Sh::B_ELEMS;
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                bf16x8 wa[2];
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    wa[c2] = as_bf(*reinterpret_cast<const u32x4 *>(Bc + ((2 * half + c2) * 16 + r) * CST + c * 32 + 8 * g));
#pragma unroll
                for (int i = 0; i < TPS; ++i) {
                    if (simd + 4 * i >= TILES) continue;
                    const bf16x8 xv = as_bf(*reinterpret_cast<const u32x4 *>(As + abase[i] + koff + c * 32));
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                        acc[i][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[c2], xv, acc[i][c2], 0, 0, 0);
                }
            }
            bstore((kk + 1) & 1, bn);
            __syncthreads();
        }
        // epilogue: bias + relu + bf16, 4 channels per lane
#pragma unroll
        for (int i = 0; i < TPS; ++i) {
            const int q = (simd + 4 * i) * 16 + r;
            if (simd + 4 * i >= TILES || q >= M) continue;
            const int smp = q / MS, o = q - smp * MS;
            const int64_t sg = 2 * p + smp;
            if (sg >= S) continue;
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2) {
                const f32x4 v = acc[i][c2];
                u32x2 w;
                w[0] = (uint32_t)f2bf(fmaxf(v[0] + bb[c2][0], 0.f)) | ((uint32_t)f2bf(fmaxf(v[1] + bb[c2][1], 0.f)) << 16);
                w[1] = (uint32_t)f2bf(fmaxf(v[2] + bb[c2][2], 0.f)) | ((uint32_t)f2bf(fmaxf(v[3] + bb[c2][3], 0.f)) << 16);
                *reinterpret_cast<u32x2 *>(y + (sg * MS + o) * 64 + (2 * half + c2) * 16 + 4 * g) = w;
            }
        }
        // the next pair's inputs (every wave passed the last offset's barrier: A is free)
        if (more) {
#pragma unroll
            for (int u = 0; u < APT; ++u)
                if (tid + u * 512 < APIECES) apark(u, apf[u]);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- Dense1
// slab[z][s][o] = sum_{f in split z} a4[s][f] * W1[f][o]; 4 waves x 16*NR
// samples per workgroup, all 64 outputs (4 column tiles); A and B fragments
// straight from global (the 1.8 MB bf16 image stays L2-resident), two k-steps
// in flight. NR row tiles per wave reuse each B fragment NR times: the B
// stream from L2 is 1.8 MB per wave, so at 65,536 samples NR = 4 cuts it from
// 7.4 GB (NR = 1) to 1.8 GB; small batches keep NR = 1 and split K instead.
template <int NR>
__global__ __launch_bounds__(256) void deep_dense1_kernel(const uint16_t *__restrict__ a4,
                                                          const uint16_t *__restrict__ w1img, int64_t S, int K1,
                                                          int kchunk, float *__restrict__ slab) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * 64 * NR + wave * 16 * NR;
    const int k0 = blockIdx.y * kchunk, k1 = min(K1, k0 + kchunk);
    const uint16_t *pa[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t) pa[t] = a4 + min(row0 + 16 * t + r, S - 1) * K1 + g * 8;
    const uint16_t *pb = w1img + (int64_t)r * K1 + g * 8;
    f32x4 acc[NR][4];
#pragma unroll
    for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    int k = k0;
    for (; k + 64 <= k1; k += 64) {
        u32x4 a[NR][2], b[2][4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int t = 0; t < NR; ++t) a[t][u] = *reinterpret_cast<const u32x4 *>(pa[t] + k + 32 * u);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) b[u][nt] = *reinterpret_cast<const u32x4 *>(pb + nt * 16 * (int64_t)K1 + k + 32 * u);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int t = 0; t < NR; ++t)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
                    acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(a[t][u]), as_bf(b[u][nt]), acc[t][nt], 0, 0, 0);
    }
    for (; k < k1; k += 32) {
        u32x4 b[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) b[nt] = *reinterpret_cast<const u32x4 *>(pb + nt * 16 * (int64_t)K1 + k);
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(pa[t] + k);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
                acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(a), as_bf(b[nt]), acc[t][nt], 0, 0, 0);
        }
    }
    float *o = slab + (int64_t)blockIdx.y * S * 64;
#pragma unroll
    for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t row = row0 + 16 * t + 4 * g + e;
                if (row < S) o[row * 64 + nt * 16 + r] = acc[t][nt][e];
            }
}

// ---------------------------------------------------------------- backward engine (bf16)
// gemm_body (snk_gemm.hpp) on v_mfma_f32_32x32x16_bf16: lane (r = l & 31,
// h = l >> 5) holds A[row r][k + 8h + j] and B[k + 8h + j][col r], j < 8;
// every loaded operand is rounded to bf16 (RNE), sums accumulate in fp32.
// KW waves split K and sum through LDS; grid.z K-splits write slabs (EpSlab).
template <int NT, int KW, class AL, class BL, class EP>
__global__ __launch_bounds__(64 * KW) void gemm_bf16_kernel(AL al, BL bl, EP ep, int M, int K, int kchunk) {
    __shared__ float red[KW > 1 ? KW * NT * 16 * 64 : 1];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m0 = blockIdx.x * 32;
    const int r = lane & 31, h = lane >> 5;
    const int n0 = blockIdx.y * (NT * 32);
    const int kb = blockIdx.z * kchunk;
    const int ke = min(K, kb + kchunk);
    const int sub = (((ke - kb) + KW - 1) / KW + 15) & ~15;
    const int wb = kb + wave * sub;
    const int we = min(ke, wb + sub);
    f32x16 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[nt][e] = 0.0f;
    const auto ctx = al.row(m0 + r, M);
    for (int k = wb; k < we; k += 16) {
        uint32_t aw[4], bw[NT][4];
#pragma unroll
        for (int j = 0; j < 8; j += 2) {
            const int k0 = k + 8 * h + j, k1 = k0 + 1;
            const float a0 = k0 < we ? al.load(ctx, k0, we) : 0.0f, a1 = k1 < we ? al.load(ctx, k1, we) : 0.0f;
            aw[j / 2] = (uint32_t)f2bf(a0) | ((uint32_t)f2bf(a1) << 16);
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int n = n0 + nt * 32 + r;
                const float b0 = k0 < we ? bl.load(k0, n, we) : 0.0f, b1 = k1 < we ? bl.load(k1, n, we) : 0.0f;
                bw[nt][j / 2] = (uint32_t)f2bf(b0) | ((uint32_t)f2bf(b1) << 16);
            }
        }
        const bf16x8 av = as_bf(u32x4{aw[0], aw[1], aw[2], aw[3]});
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
            acc[nt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, as_bf(u32x4{bw[nt][0], bw[nt][1], bw[nt][2], bw[nt][3]}),
                                                             acc[nt], 0, 0, 0);
    }
    if (KW > 1) {
        float *dst = red + wave * NT * 16 * 64;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int e = 0; e < 16; ++e) dst[(nt * 16 + e) * 64 + lane] = acc[nt][e];
        __syncthreads();
        if (m0 >= M) return;
        for (int e = threadIdx.x; e < NT * 16 * 64; e += 64 * KW) {
            float v = red[e];
#pragma unroll
            for (int w = 1; w < KW; ++w) v += red[w * NT * 16 * 64 + e];
            const int nt = e >> 10, gg = (e >> 6) & 15, ln = e & 63;
            ep.store1(v, m0 + acc_row(gg, ln), n0 + nt * 32 + (ln & 31), (int)blockIdx.z);
        }
        return;
    }
    if (m0 >= M) return;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) ep.store(acc[nt], m0, n0 + nt * 32, lane, (int)blockIdx.z);
}

struct EpReluMaskB {  // y = (bf16 act > 0) ? acc : 0
    float *y;
    const uint16_t *act;
    int64_t M;
    int N;
    __device__ void store1(float v, int row, int col, int) const {
        if (row >= M || col >= N) return;
        const int64_t o = (int64_t)row * N + col;
        y[o] = bf2f(act[o]) > 0.0f ? v : 0.0f;
    }
    __device__ void store(const f32x16 &acc, int m0, int c0, int lane, int) const {
        const int col = c0 + (lane & 31);
        if (col >= N) return;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int row = m0 + acc_row(e, lane);
            if (row < M) {
                const int64_t o = (int64_t)row * N + col;
                y[o] = bf2f(act[o]) > 0.0f ? acc[e] : 0.0f;
            }
        }
    }
};

}  // namespace snk

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
#include "snk_conv_h3.hpp"
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
    int64_t img_w[4], img_d1, img_wt[4], img_n;   // img_wt[l]: L1..L3 weights in packed order [kk][ci][co] (data gradients)
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
        if (t >= D.img_wt[1]) {   // L1..L3 [kk][ci][co]: the packed order, the data gradients' A operand
            int l = 1;
            while (l < 3 && t >= D.img_wt[l + 1]) ++l;
            img[t] = f2bf(th[D.off_w[l] + (t - D.img_wt[l])]);
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
// two floats -> two bf16 (round to nearest even: v_cvt_pk_bf16_f32, gfx950)
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2v{a, b}, bf16x2v));
}
// relu(v + b) of four channels as four bf16
__device__ __forceinline__ u32x2 relu_bf16x4(const f32x4 &v, const f32x4 &b) {
    return u32x2{pk_bf16(fmaxf(v[0] + b[0], 0.f), fmaxf(v[1] + b[1], 0.f)),
                 pk_bf16(fmaxf(v[2] + b[2], 0.f), fmaxf(v[3] + b[3], 0.f))};
}

// deep_front_kernel: L0 -> L1 -> L2 of one sample at a time inside one
// workgroup, the activations never leaving LDS. Persistent: one workgroup per
// CU walks samples blockIdx.x, + gridDim.x, ...; the L0, L1 and L2 weight
// images are staged into LDS once per workgroup.
// LDS (halves): W1 [9][32 co][32], W2 [9][64 co][32], W0 [32 co][32] (k < 9C,
// zero above): 64-byte rows, chunk c of row `row` at slot c ^ ((row >> 1) & 3),
// which depends only on the lane for the fragment reads (row = 16*tile + lane);
// X, the bordered L0 output and then (after a barrier, in place) the bordered
// L1 output: [(4*NB + 2) rows][PJ][48] (a 96-byte position stride, no
// swizzle); BD the bordered boards [C][(H+2)^2] bf16.
// Row tiles are 4 x 4 blocks of output positions (NB = ceil(H/4) blocks a side;
// positions past H are computed on zeros and never stored). With the 96-byte
// stride and PJ = 28 every fragment read of a tile, at every kernel offset,
// puts each ds_read_b128 lane group on 16 distinct bank quads (the lane groups
// simulated), and the address of a read is one lane-constant register plus a
// wave-uniform offset (tile, kernel offset): no per-read address arithmetic.
// Every MFMA is v_mfma_f32_16x16x32_bf16 with the WEIGHTS as the A operand
// (rows = output channels) and the activations as B (columns = positions), so a
// lane's accumulator holds 4 consecutive channels of one position: the
// epilogues store 8 bytes per lane. Work split: row tile t goes to SIMD t % 4
// (waves w and w + 4 share a SIMD): L0 wave half h = w >> 2 takes column tile
// h of the SIMD's tiles; L1 the two halves split the SIMD's tiles, both column
// tiles each; L2 both halves run all the SIMD's tiles, column tiles 2h, 2h + 1.
// At 20x20: 25 tiles = 7/6/6/6 per SIMD.
// L0 on the matrix cores: the boards (-1 .. 2) and the bf16-rounded weights are
// exact bf16, so every product is exact; only the fp32 summation order differs
// from the VALU form (bias added last).
// KEEP: also store the L0 / L1 outputs (the training forward's backward reads
// them); L2's output always goes to a2 [S][H^2][64].
template <int H>
struct DeepFrontShape {
    static constexpr int HB = H + 2, M = H * H, NB = (H + 3) / 4, TILES = NB * NB, TPS = (TILES + 3) / 4;
    static constexpr int HALF = (TPS + 1) / 2;
    static constexpr int XR = 4 * NB + 2, PJ = XR + (12 - XR % 8) % 8;   // the smallest pitch >= XR, = 4 (mod 8)
    static constexpr int XST = 48;                                        // halves per X position
    static constexpr int W1 = 9 * 32 * 32, W2 = 9 * 64 * 32, W0 = 32 * 32, X = XR * PJ * XST, BD = 2 * HB * HB;
    static constexpr int LDS = (W1 + W2 + W0 + X + BD) * 2;
};
// 16-byte chunk c of a 64-byte weight row
__device__ __forceinline__ int dfr_slot(int row, int c) { return row * 32 + 8 * (c ^ ((row >> 1) & 3)); }
// The L0 / L1 epilogue stores into X: an MFMA accumulator lane (r, g) holds channel quad g of
// tile position (r & 3, r >> 2), so a 16-lane store group (one g) would write four tile rows
// whose X addresses differ by multiples of 128 bytes: 4-way bank conflicts on ds_write_b64
// (bank = dword mod 32; 25 % of the kernel's LDS cycles in profiles/r03_pmc_deep_fwd.json).
// The fragment READS (9x as many) are conflict-free on this layout and no X layout or chunk
// swizzle serves both (tools/), so the store transposes instead: lane
// 16a + 4b + c takes lane 16b + 4a + c's data (ds_bpermute), i.e. channel quad r >> 2 of
// position (r & 3, row g): one tile row per group, 16 distinct bank pairs.
__device__ __forceinline__ u32x2 dfr_tr44(const u32x2 &v, int lane) {
    const int src = (((lane >> 2) & 3) * 16 + ((lane >> 4) & 3) * 4 + (lane & 3)) * 4;
    return u32x2{(uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)v[0]),
                 (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)v[1])};
}

// A workgroup barrier for LDS hand-offs only: this wave's LDS operations complete, then
// s_barrier. __syncthreads' fence also waits for every outstanding global load and store
// (s_waitcnt vmcnt(0)): in deep_front_kernel that put the previous sample's a2 stores and the
// next sample's board loads on the critical path at every one of its four barriers per sample.
__device__ __forceinline__ void dfr_lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0) (vmcnt, expcnt left at their maxima)
    __builtin_amdgcn_s_barrier();
}

// The K loop of one deep_front layer, software-pipelined: for each of the KK kernel offsets
// (fully unrolled) two weight fragments (A, column tiles c2 = 0, 1) and NT activation
// fragments (B, row tiles) feed 2 NT MFMAs. Each row tile's fragment for offset kk+1 is read
// right after that tile's two MFMAs of offset kk (its registers are free then: one buffer of NT
// fragments, as the 256-register budget of two waves per SIMD needs), the next offset's weights
// after the first tile; scheduling barriers pin the order (left to itself the scheduler sank
// every read next to its MFMAs, which then waited a full LDS round trip each). acc[t][c2]
// accumulates over kk in order: the results are those of the plain loop.
// PLAIN (the training forward, KEEP: its extra stores' addresses leave no registers for the
// pipeline at 20x20): each offset's fragments read, then its MFMAs, no pinning.
template <int KK, int NT, bool PLAIN, typename WF, typename XF>
__device__ __forceinline__ void dfr_pipeline(WF wfrag, XF xfrag, f32x4 (&acc)[NT][2]) {
    if constexpr (PLAIN) {
#pragma unroll 3
        for (int kk = 0; kk < KK; ++kk) {
            bf16x8 wa[2];
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2) wa[c2] = wfrag(kk, c2);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const bf16x8 xv = xfrag(kk, t);
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    acc[t][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[c2], xv, acc[t][c2], 0, 0, 0);
            }
        }
        return;
    }
    bf16x8 wa[2][2], xv[NT];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) wa[0][c2] = wfrag(0, c2);
#pragma unroll
    for (int t = 0; t < NT; ++t) xv[t] = xfrag(0, t);
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
        const int b = kk & 1;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2)
                acc[t][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[b][c2], xv[t], acc[t][c2], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (kk + 1 < KK) {
                if (t == 0) {
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2) wa[b ^ 1][c2] = wfrag(kk + 1, c2);
                }
                xv[t] = xfrag(kk + 1, t);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}

// Profiling builds only (make clocks): per-workgroup sums of wave 0's time per phase over its
// samples (0 boards into LDS + barrier, 1 L0 + barrier, 2 L1 offsets, 3 L1 epilogue and its two
// barriers, 4 L2 offsets, 5 L2 epilogue: staging in LDS, two barriers, the a2 stores; 6 the sample
// count), read by snk_dfr_debug_clocks
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_dfr_clk;
#define DFR_CLK(k)                                                                                    \
    do {                                                                                              \
        if (tid == 0 && g_dfr_clk) {                                                                  \
            const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                     \
            dfr_acc[k] += t_ - dfr_t;                                                                 \
            dfr_t = t_;                                                                               \
        }                                                                                             \
    } while (0)
#else
#define DFR_CLK(k) do { } while (0)
#endif
// measurement builds only (-DSNK_DFR_VAR=1 with SNK_ENV_CLOCKS; wrong results by design): the
// a2 copy-out without its global stores
#ifndef SNK_DFR_VAR
#define SNK_DFR_VAR 0
#endif
#if SNK_DFR_VAR && !defined(SNK_ENV_CLOCKS)
#error "SNK_DFR_VAR: measurement (clocks) builds only"
#endif
template <int C, int H, bool KEEP>
__global__ __launch_bounds__(512) void deep_front_kernel(BoardSrc src, const float *__restrict__ img0,
                                                         const uint16_t *__restrict__ wimg1,
                                                         const float *__restrict__ bias1,
                                                         const uint16_t *__restrict__ wimg2,
                                                         const float *__restrict__ bias2, uint16_t *__restrict__ a0,
                                                         uint16_t *__restrict__ a1, uint16_t *__restrict__ a2,
                                                         int64_t S) {
    using Sh = DeepFrontShape<H>;
    constexpr int HB = Sh::HB, M = Sh::M, NB = Sh::NB, TILES = Sh::TILES, TPS = Sh::TPS, HALF = Sh::HALF;
    constexpr int PJ = Sh::PJ, XST = Sh::XST, PL = HB * HB, NBV = (C * M + 511) / 512;
    static_assert(9 * C <= 32, "L0 fan-in beyond one k step");
    static_assert(PJ % 8 == 4 && PJ >= Sh::XR, "image pitch");
    extern __shared__ __attribute__((aligned(16))) uint16_t fsm[];
    uint16_t *W1s = fsm, *W2s = W1s + Sh::W1, *W0s = W2s + Sh::W2, *X = W0s + Sh::W0, *BD = X + Sh::X;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: tile offsets stay scalar
    const int r = lane & 15, g = lane >> 4, simd = wave & 3, half = wave >> 2;
    // ---- weights (rows of 32 ci: four swizzled chunks), zeroed image and boards
    for (int q = tid; q < 9 * 32 * 4; q += 512)
        *reinterpret_cast<u32x4 *>(W1s + dfr_slot(q >> 2, q & 3)) = reinterpret_cast<const u32x4 *>(wimg1)[q];
    for (int q = tid; q < 9 * 64 * 4; q += 512)
        *reinterpret_cast<u32x4 *>(W2s + dfr_slot(q >> 2, q & 3)) = reinterpret_cast<const u32x4 *>(wimg2)[q];
    for (int q = tid; q < 32 * 32; q += 512) {
        const int co = q >> 5, k = q & 31;
        W0s[dfr_slot(co, k >> 3) + (k & 7)] = k < 9 * C ? f2bf(img0[k * 32 + co]) : (uint16_t)0;
    }
    for (int q = tid; q < (Sh::X + Sh::BD) / 8; q += 512)   // X, BD are contiguous
        *reinterpret_cast<u32x4 *>(X + q * 8) = u32x4{0u, 0u, 0u, 0u};
    // per-lane biases of the channels this lane's accumulators hold (4g + e of a column tile)
    const f32x4 b0 = *reinterpret_cast<const f32x4 *>(img0 + 9 * C * 32 + half * 16 + 4 * g);
    f32x4 b1[2], b2[2];
#pragma unroll
    for (int c2 = 0; c2 < 2; ++c2) {
        b1[c2] = *reinterpret_cast<const f32x4 *>(bias1 + c2 * 16 + 4 * g);
        b2[c2] = *reinterpret_cast<const f32x4 *>(bias2 + (2 * half + c2) * 16 + 4 * g);
    }
    // lane-constant parts of the addresses: weight fragment (row 16*tile + r, chunk g);
    // X fragment (position (r & 3, r >> 2) of a tile, chunk g); the L0 board gather
    // (k = 8g + e -> channel k % C, kernel offset k / C; -1 past 9C)
    const int wl = r * 32 + 8 * (g ^ ((r >> 1) & 3));
    const int xl = ((r & 3) + (r >> 2) * PJ) * XST + 8 * g;
    int bofs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const int k = 8 * g + e, kk = k / C, c = k - kk * C;
        // C == 2: k = 2 kk + c, so the pair (2 e2, 2 e2 + 1) is kernel offset 4g + e2, channels
        // 0 and 1: bofs[2 e2] is its word (position) offset in the [position][channel] boards
        bofs[e] = k < 9 * C ? (C == 2 ? kk % 3 + (kk / 3) * HB : c * PL + kk % 3 + (kk / 3) * HB) : -1;
    }
    static_assert(4 * (TPS - 1) < TILES, "tiles 0 .. TPS-2 of every SIMD exist");
    const bool last_ok = simd + 4 * (TPS - 1) < TILES;   // only a SIMD's last tile can be missing
    // wave-uniform top-left position (bordered image) of row tile t
    auto tbase = [&](int t) __attribute__((always_inline)) { return 4 * (t % NB) + 4 * (t / NB) * PJ; };
    auto tpos = [&](int t, int &i, int &j) __attribute__((always_inline)) {
        i = 4 * (t % NB) + (r & 3);
        j = 4 * (t / NB) + (r >> 2);
    };
    int bv[NBV];   // raw: the int8 cell, or the float's bits (converted where stored, so no
                   // wait follows the load)
    // env frame ring (the act forward): the channels' ring slots come from the step counter,
    // which no launch changes: read once, so a cell is one byte load (through src.load each cell
    // was a counter load, a wait, the byte load and a wait)
    const bool ring = !src.fbase && !src.idx;
    const int8_t *cb[C];
#pragma unroll
    for (int c = 0; c < C; ++c) cb[c] = ring ? src.plane(0, c) : nullptr;
    auto bload = [&](int64_t s) __attribute__((always_inline)) {
        int te = tid;   // opaque: the per-cell offsets stay in the loop (hoisted, they were
        asm volatile("" : "+v"(te));   // spilled across it)
#pragma unroll
        for (int u = 0; u < NBV; ++u) {
            const int e = te + u * 512;
            if (e < C * M) {
                const int c = e / M, cell = e - c * M;
                if (ring) {
                    const int8_t *pl = cb[0];
#pragma unroll
                    for (int cc = 1; cc < C; ++cc) pl = c == cc ? cb[cc] : pl;
                    bv[u] = pl[s * (int64_t)src.pitch + cell];
                } else if (src.fbase) {
                    bv[u] = __float_as_int(src.fbase[(s * C + c) * src.ncell + cell]);
                } else {
                    bv[u] = src.plane(s, c)[cell];
                }
            }
        }
    };
    int64_t s = blockIdx.x;
    if (s < S) bload(s);
    __syncthreads();
    // the first boards landed: with this wait on the loop's entry path as on its back edge (the
    // wait ahead of the a2 stores), the compiler puts no wait at the loop head
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
#ifdef SNK_ENV_CLOCKS
    uint64_t dfr_acc[7] = {0, 0, 0, 0, 0, 0, 0}, dfr_t = __builtin_amdgcn_s_memrealtime();
#endif
    for (; s < S; s += gridDim.x) {
#pragma unroll
        for (int u = 0; u < NBV; ++u) {
            const int e = tid + u * 512;
            if (e < C * M) {
                const int c = e / M, cell = e % M;
                const int bp = (cell % H + 1) + (cell / H + 1) * HB;   // C == 2: [position][channel]
                BD[C == 2 ? 2 * bp + c : c * PL + bp] = f2bf(src.fbase ? __int_as_float(bv[u]) : (float)bv[u]);
            }
        }
        // the next sample's boards: in flight through this whole sample (waited for before the
        // a2 stores below, so the wait above never waits for those stores)
        if (s + gridDim.x < S) bload(s + gridDim.x);
        dfr_lds_barrier();   // boards in; X free (last read by the previous sample's L2)
        if constexpr (!KEEP) {
            // the previous sample's a2 staging (below) overwrote X's zero border (the 3x3
            // convolutions' padding, which no epilogue writes): channels 0..31 of its positions
            // zeroed again, beside L0's interior writes and ahead of L0's barrier
            // rows 0 and HB-1 (2 HB positions), then columns 0 and HB-1 of rows 1..HB-2; four
            // 16-byte pieces per position, one per thread
            static_assert(4 * 4 * (HB - 1) <= 512, "one border piece per thread");
            if (tid < 4 * 4 * (HB - 1)) {
                int tz = tid;   // an opaque copy: the address stays in the loop (hoisted, it held
                asm volatile("" : "+v"(tz));   // registers through L2 and the kernel spilled)
                const int bp = tz >> 2, ch = tz & 3, rw = bp < 2 * HB;
                const int x = rw ? bp % HB : (bp - 2 * HB) % 2 * (HB - 1);
                const int y = rw ? bp / HB * (HB - 1) : 1 + (bp - 2 * HB) / 2;
                *reinterpret_cast<u32x4 *>(X + (x + y * PJ) * XST + 8 * ch) = u32x4{0u, 0u, 0u, 0u};
            }
        }
        DFR_CLK(0);
        // ---- L0: column tile `half` of the SIMD's row tiles, in three passes over the tiles
        // (every gather, then every MFMA, then every epilogue: tile by tile, each tile's LDS
        // reads, MFMA, transpose and store waited on one another). C == 2: the boards are
        // [position][channel], so a k pair (channels 0, 1 of one kernel offset) is one u32 read
        {
            const bf16x8 wa = as_bf(*reinterpret_cast<const u32x4 *>(W0s + half * 16 * 32 + wl));
            u32x4 xw[TPS];
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii) {
                // a missing last tile gathers the SIMD's tile 0 again (never stored)
                const int t = simd + 4 * ((ii == TPS - 1 && !last_ok) ? 0 : ii);
                int i, j;
                tpos(t, i, j);
                const int bb = min(i, H - 1) + min(j, H - 1) * HB;
                if constexpr (C == 2) {
                    const uint32_t *BD2 = reinterpret_cast<const uint32_t *>(BD);
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2) {
                        const uint32_t w = BD2[bb + max(bofs[2 * e2], 0)];
                        xw[ii][e2] = bofs[2 * e2] >= 0 ? w : 0u;
                    }
                } else {
                    // branch-free gather: every lane loads (k past 9C reads cell 0 and is masked to zero)
                    uint32_t v[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) v[e] = BD[bb + max(bofs[e], 0)];
#pragma unroll
                    for (int e2 = 0; e2 < 4; ++e2)
                        xw[ii][e2] = (bofs[2 * e2] >= 0 ? v[2 * e2] : 0u) | ((bofs[2 * e2 + 1] >= 0 ? v[2 * e2 + 1] : 0u) << 16);
                }
            }
            f32x4 a0v[TPS];
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii)
                a0v[ii] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, as_bf(xw[ii]), f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
            u32x2 ot[TPS];
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii) ot[ii] = dfr_tr44(relu_bf16x4(a0v[ii], b0), lane);   // quad r >> 2 of (r & 3, row g)
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii) {
                const int t = simd + 4 * ii;
                if (ii == TPS - 1 && !last_ok) continue;
                int i, j;
                tpos(t, i, j);
                if (KEEP && i < H && j < H)
                    *reinterpret_cast<u32x2 *>(a0 + (s * M + i + j * H) * 32 + half * 16 + 4 * g) = relu_bf16x4(a0v[ii], b0);
                const int ti = 4 * (t % NB) + (r & 3), tj = 4 * (t / NB) + g;
                if (ti < H && tj < H)
                    *reinterpret_cast<u32x2 *>(X + ((ti + 1) + (tj + 1) * PJ) * XST + half * 16 + 4 * (r >> 2)) = ot[ii];
            }
        }
        dfr_lds_barrier();
        DFR_CLK(1);
        // ---- L1: this half's share of the SIMD's row tiles, both column tiles; the
        // result replaces L0's in X after a barrier
        {
            f32x4 acc[HALF][2];
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii) acc[ii][0] = acc[ii][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            // branch-free: a missing tile computes the SIMD's tile 0 again (never stored); the
            // nine kernel offsets unrolled with offset kk+1's fragments read under kk's MFMAs
            int xb[HALF];
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii) {
                const int i = half * HALF + ii;
                const bool live = i < TPS && !(i == TPS - 1 && !last_ok);
                xb[ii] = xl + tbase(simd + 4 * (live ? i : 0)) * XST;
            }
            dfr_pipeline<9, HALF, KEEP>(
                [&](int kk, int c2) __attribute__((always_inline)) {
                    return as_bf(*reinterpret_cast<const u32x4 *>(W1s + (kk * 32 + c2 * 16) * 32 + wl));
                },
                [&](int kk, int ii) __attribute__((always_inline)) {
                    return as_bf(*reinterpret_cast<const u32x4 *>(X + xb[ii] + ((kk % 3) + (kk / 3) * PJ) * XST));
                },
                acc);
            DFR_CLK(2);
            dfr_lds_barrier();   // every wave's L1 reads of X are done: X takes the L1 output
            // every tile's transposes first, then the stores (tile by tile, each transpose's LDS
            // round trip was waited out before its store)
            u32x2 ot[HALF][2];
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii)
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2) ot[ii][c2] = dfr_tr44(relu_bf16x4(acc[ii][c2], b1[c2]), lane);
#pragma unroll
            for (int ii = 0; ii < HALF; ++ii) {
                const int i2 = half * HALF + ii, t = simd + 4 * i2;
                if (i2 >= TPS || (i2 == TPS - 1 && !last_ok)) continue;
                int i, j;
                tpos(t, i, j);
                const int ti = 4 * (t % NB) + (r & 3), tj = 4 * (t / NB) + g;   // the transposed store's position
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2) {
                    if (KEEP && i < H && j < H)
                        *reinterpret_cast<u32x2 *>(a1 + (s * M + i + j * H) * 32 + c2 * 16 + 4 * g) =
                            relu_bf16x4(acc[ii][c2], b1[c2]);
                    if (ti < H && tj < H)
                        *reinterpret_cast<u32x2 *>(X + ((ti + 1) + (tj + 1) * PJ) * XST + c2 * 16 + 4 * (r >> 2)) =
                            ot[ii][c2];
                }
            }
        }
        dfr_lds_barrier();
        DFR_CLK(3);
        // ---- L2: all the SIMD's row tiles, column tiles 2*half, 2*half + 1
        {
            f32x4 acc[TPS][2];
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii) acc[ii][0] = acc[ii][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            int xb[TPS];
#pragma unroll
            for (int ii = 0; ii < TPS; ++ii) xb[ii] = xl + tbase(simd + 4 * ((ii == TPS - 1 && !last_ok) ? 0 : ii)) * XST;
            dfr_pipeline<9, TPS, KEEP>(
                [&](int kk, int c2) __attribute__((always_inline)) {
                    return as_bf(*reinterpret_cast<const u32x4 *>(W2s + (kk * 64 + (2 * half + c2) * 16) * 32 + wl));
                },
                [&](int kk, int ii) __attribute__((always_inline)) {
                    return as_bf(*reinterpret_cast<const u32x4 *>(X + xb[ii] + ((kk % 3) + (kk / 3) * PJ) * XST));
                },
                acc);
            DFR_CLK(4);
            // a2 leaves through LDS: the accumulators (8 bytes of one position per lane, four
            // instructions per 128-byte position from two waves) go to a staging image in X,
            // [position][64 channels], 8-byte slot s of position p at s ^ (p & 15) (the sixteen
            // positions of a tile's store land on sixteen distinct bank pairs); then whole
            // positions leave as 16-byte pieces, each 128-byte line written by one instruction
            // (the scattered 8-byte stores took twice as long as the L2 offsets).
            // (KEEP, the training forward at the update's batch: the direct 8-byte stores; the
            // staging below spilled there, next to the a0 / a1 stores' registers)
            if constexpr (KEEP) {
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // the next boards (see below)
#pragma unroll
                for (int ii = 0; ii < TPS; ++ii) {
                    if (ii == TPS - 1 && !last_ok) continue;
                    int i, j;
                    tpos(simd + 4 * ii, i, j);
                    if (i >= H || j >= H) continue;
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                        *reinterpret_cast<u32x2 *>(a2 + (s * M + i + j * H) * 64 + (2 * half + c2) * 16 + 4 * g) =
                            relu_bf16x4(acc[ii][c2], b2[c2]);
                }
            } else {
                dfr_lds_barrier();   // every wave's L2 reads of X are done
#pragma unroll
                for (int ii = 0; ii < TPS; ++ii) {
                    if (ii == TPS - 1 && !last_ok) continue;
                    int i, j;
                    tpos(simd + 4 * ii, i, j);
                    if (i >= H || j >= H) continue;
                    const int p = i + j * H;
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                        *reinterpret_cast<u32x2 *>(X + p * 64 + ((((2 * half + c2) * 4 + g) ^ (p & 15)) << 2)) =
                            relu_bf16x4(acc[ii][c2], b2[c2]);
                }
            }
        }
        if constexpr (!KEEP) {
            dfr_lds_barrier();
            // the next sample's board loads landed long ago: waiting for them here, ahead of the
            // a2 stores, keeps the compiler's wait at the loop head from draining those stores
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
            {
                static_assert(M * 64 <= Sh::X, "a2 staging fits X");
                constexpr int NQ = M * 8, QT = (NQ + 511) / 512;   // 16-byte pieces of the sample's a2
#pragma unroll 2
                for (int u = 0; u < QT; ++u) {
                    const int q = tid + u * 512;
                    if (q < NQ) {
                        const int p = q >> 3, k = q & 7, m = p & 15;
                        const u32x4 v = *reinterpret_cast<const u32x4 *>(X + p * 64 + ((((2 * k) ^ m) & ~1) << 2));
                        // the piece's two 8-byte halves, swapped back when the swizzle swapped them
                        const u32x4 o = (m & 1) ? u32x4{v[2], v[3], v[0], v[1]} : v;
#if SNK_DFR_VAR == 1   // measurement builds: the copy-out without its global stores
                        asm volatile("" :: "v"(o));
#else
                        *reinterpret_cast<u32x4 *>(a2 + (s * M + p) * 64 + 8 * k) = o;
#endif
                    }
                }
            }
        }
        DFR_CLK(5);
#ifdef SNK_ENV_CLOCKS
        if (tid == 0) ++dfr_acc[6];
#endif
    }
#ifdef SNK_ENV_CLOCKS
    if (tid == 0 && g_dfr_clk)
        for (int k = 0; k < 7; ++k) g_dfr_clk[(int64_t)blockIdx.x * 8 + k] = dfr_acc[k];
#endif
}

// ---------------------------------------------------------------- L3 (MFMA, two samples)
// deep_conv3_kernel: L3 (6x6, 64 -> 64, valid) for TWO samples per step of a
// persistent workgroup (one per CU, 8 waves). LDS holds only the pair's
// inputs [2][H rows][PJ = 24][64] (123 KB at 20x20); every row is 128 bytes
// (eight 16-byte chunks) with chunk c of row `row` at slot c ^ (row & 7). The
// weights go straight from global (L2-resident, 295 KB) into registers, two
// kernel offsets ahead, so the 36 offsets run without a single barrier (the
// LDS-staged form paid one per stage: 36 barriers per pair -> 5.7 ms, 18 ->
// 5.1 ms). A row tile is one output row of one sample: 16 consecutive output
// columns (WO = 15 at 20x20: the 16th is computed and dropped), so each
// fragment read covers 16 consecutive LDS rows, which the swizzle puts on 16
// distinct bank quads. PJ and H*PJ are multiples of 8, so row & 7 =
// (lane + du) & 7: one lane-constant address per kernel offset and 32-channel
// step, plus a wave-uniform tile offset.
// Row tile t of the pair (2*WO of them) goes to SIMD t % 4, wave half h takes
// column tiles 2h, 2h + 1: per kernel offset 4 weight fragments (global) and
// 2 x up to 8 activation fragments (LDS) for 32 MFMAs per wave.
// The next pair's inputs are loaded and parked between the pair's two barriers
// (prefetching them into registers during the offsets cost more than it hid:
// 5.05 against 4.95 ms, the slow HBM loads holding up the in-order vmcnt waits
// of the weight loads queued behind them).
// MFMA operands as deep_front_kernel: weights A (rows = channels), activations
// B, 8-byte epilogue stores of 4 channels.
template <int H>
struct DeepL3Shape {
    static constexpr int WO = H - 5, TILES = 2 * WO, TPS = (TILES + 3) / 4, PJ = (H + 1 + 7) / 8 * 8;
    static constexpr int XS = H * PJ * 64;
    static constexpr int WSLOTS = 4, WSLOT = 64 * 64 * 2;   // weight ring: one kernel offset (8 KB) per slot
    static constexpr int LDS = 2 * XS * 2 + WSLOTS * WSLOT;
    static constexpr int APIECES = 2 * H * H * 8, APT = (APIECES + 511) / 512;
};
__device__ __forceinline__ int dl3_slot(int row, int c) { return row * 64 + 8 * (c ^ (row & 7)); }

// measurement builds only (-DSNK_DL3_VAR=n with SNK_ENV_CLOCKS; wrong results by design): the
// pair loop without the next pair's input loads (1), the per-offset barriers (2), the MFMAs (3)
// or the activation fragment reads (4) (`profiles/r06k_dl3_vars.txt`)
#ifndef SNK_DL3_VAR
#define SNK_DL3_VAR 0
#endif
#if SNK_DL3_VAR && !defined(SNK_ENV_CLOCKS)
#error "SNK_DL3_VAR: measurement (clocks) builds only"
#endif
template <int H>
__global__ __launch_bounds__(512) void deep_conv3_kernel(const uint16_t *__restrict__ x,
                                                         const uint16_t *__restrict__ wimg,
                                                         const float *__restrict__ bias, uint16_t *__restrict__ y,
                                                         int64_t S, int blocked) {
    using Sh = DeepL3Shape<H>;
    constexpr int WO = Sh::WO, TILES = Sh::TILES, TPS = Sh::TPS, PJ = Sh::PJ;
    constexpr int APT = Sh::APT, APIECES = Sh::APIECES;
    static_assert(WO <= 16 && PJ % 8 == 0 && PJ > H, "one output row per row tile");
    extern __shared__ __attribute__((aligned(16))) uint16_t l3sm[];
    uint16_t *As = l3sm;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, g = lane >> 4, simd = wave & 3, half = wave >> 2;
    const int64_t npairs = (S + 1) / 2;
    // input piece q of pair p: sample 2p + q / (H*H*8) (clamped to S - 1), position, 16-byte chunk
    auto apiece = [&](int64_t p, int u) __attribute__((always_inline)) {
        int tq = tid;   // opaque: the per-piece offsets stay at the use (hoisted above the offset
        asm volatile("" : "+v"(tq));   // loop, they were spilled across it)
        const int q = tq + u * 512;
        const int smp = q / (H * H * 8), rem = q - smp * (H * H * 8);
        const int64_t sg = min(2 * p + smp, S - 1);
        return *reinterpret_cast<const u32x4 *>(x + (sg * H * H + (rem >> 3)) * 64 + (rem & 7) * 8);
    };
    auto apark = [&](int u, const u32x4 &v) __attribute__((always_inline)) {
        int tq = tid;   // opaque, as in apiece
        asm volatile("" : "+v"(tq));
        const int q = tq + u * 512;
        const int smp = q / (H * H * 8), rem = q - smp * (H * H * 8);
        const int pos = rem >> 3;   // rows are numbered across the pair (the swizzle uses the pair-wide row)
        *reinterpret_cast<u32x4 *>(As + dl3_slot(smp * (H * PJ) + (pos % H) + (pos / H) * PJ, rem & 7)) = v;
    };
    // weight ring (LDS-DMA): kernel offset k of the image [kk][co][ci] goes to slot k % WSLOTS
    // as 64 rows (co) of 128 bytes, 16-byte chunk q of row co at q ^ (co & 7) (every fragment
    // read below on distinct bank quads, tools/lds_banks.py model). Wave w moves rows 8w .. 8w+7:
    // one global_load_lds_dwordx4 per wave and offset, lane-linear in LDS, the source chunk
    // picked to match the swizzle. The loads never land in VGPRs, so no compiler-inserted
    // vmcnt wait can pull them forward (register loads two offsets ahead were waited on right
    // after issue at the loop head: an L2 round trip every other offset)
    uint16_t *Wr = As + 2 * Sh::XS;
    auto wdma = [&](int k) __attribute__((always_inline)) {
        const int kk = k % 36, row = wave * 8 + (lane >> 3), q = (lane & 7) ^ (row & 7);
        __builtin_amdgcn_global_load_lds((const void *)(wimg + (int64_t)kk * 64 * 64 + row * 64 + q * 8),
                                         (__attribute__((address_space(3))) void *)(Wr + (k % Sh::WSLOTS) * (Sh::WSLOT / 2) +
                                                                                     wave * 512),
                                         16, 0, 0);
    };
    // the 4 weight fragments of offset k this wave uses: [c][c2], row (2h + c2)*16 + r, channels
    // 32c + 8g .. +7
    auto wread = [&](int k, u32x4 (&f)[4]) __attribute__((always_inline)) {
        const uint16_t *ws = Wr + (k % Sh::WSLOTS) * (Sh::WSLOT / 2);
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int c2 = 0; c2 < 2; ++c2) {
                const int row = (2 * half + c2) * 16 + r;
                f[2 * c + c2] = *reinterpret_cast<const u32x4 *>(ws + row * 64 + (((4 * c + g) ^ (row & 7)) << 3));
            }
    };
    // wave-uniform first input row of row tile t (sample t / WO, output row t % WO)
    auto trow = [&](int t) __attribute__((always_inline)) { return (t / WO) * (H * PJ) + (t % WO) * PJ; };
    static_assert(4 * (TPS - 1) < TILES, "tiles 0 .. TPS-2 of every SIMD exist");
    const bool last_ok = simd + 4 * (TPS - 1) < TILES;
    int64_t p = blockIdx.x;
    if (p < npairs) {
#pragma unroll
        for (int u = 0; u < APT; ++u)
            if (tid + u * 512 < APIECES) apark(u, apiece(p, u));
    }
    // offsets 0 .. WSLOTS-2 in flight before the first pair (k counts offsets across pairs)
#pragma unroll
    for (int k = 0; k < Sh::WSLOTS - 1; ++k) wdma(k);
    __syncthreads();
    for (; p < npairs; p += gridDim.x) {
        const bool more = p + gridDim.x < npairs;
        const int64_t pn = p + gridDim.x;
        f32x4 acc[TPS][2];
#pragma unroll
        for (int i = 0; i < TPS; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
        // the epilogue's bias quads, loaded before the offsets (the epilogue re-loaded them per
        // row tile; L1 hits, the same time: `profiles/r05j2_l3_bias.txt`)
        f32x4 bb[2];
#pragma unroll
        for (int c2 = 0; c2 < 2; ++c2) bb[c2] = *reinterpret_cast<const f32x4 *>(bias + (2 * half + c2) * 16 + 4 * g);
        // one barrier per offset: wait for this wave's DMAs of offsets kk and kk + 1 (kk + 2 stays
        // in flight), barrier (every wave's pieces landed; every wave is past offset kk - 1, so
        // its slot is free), refill that slot with offset kk + 3. The weight fragments of kk + 1
        // and the activation fragments of the next step are read while kk's MFMAs issue (one
        // activation register per tile, reloaded right after the tile's MFMAs): only the first
        // offset of a pair waits on its reads
        bf16x8 xv[TPS];
        auto xread = [&](int kk, int c, int i) __attribute__((always_inline)) {
            const int du = kk % 6, dv = kk / 6, sw = (r + du) & 7;
            return as_bf(*reinterpret_cast<const u32x4 *>(As + dv * PJ * 64 + trow(simd + 4 * i) * 64 + (r + du) * 64 +
                                                          8 * ((4 * c + g) ^ sw)));
        };
#pragma unroll
        for (int i = 0; i < TPS; ++i)
            if (!(i == TPS - 1 && !last_ok)) xv[i] = xread(0, 0, i);
        u32x4 wcur[4], wnext[4];
#pragma unroll 1
        for (int kk = 0; kk < 36; ++kk) {
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(Sh::WSLOTS - 3));
            __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
            if (SNK_DL3_VAR != 2) __builtin_amdgcn_s_barrier();
            wdma(kk + Sh::WSLOTS - 1);
            if (kk == 0) wread(0, wcur);
            wread(kk + 1, wnext);   // kk = 35: offset 0 of the next pair (slot 36 % 4), harmless
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                const int nk = c == 0 ? kk : (kk + 1 < 36 ? kk + 1 : 0), nc = c ^ 1;   // the next step
#pragma unroll
                for (int i = 0; i < TPS; ++i) {
                    if (i == TPS - 1 && !last_ok) continue;   // only the last tile can be missing
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2) {
                        if (SNK_DL3_VAR != 3)
                            acc[i][c2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(wcur[2 * c + c2]), xv[i], acc[i][c2],
                                                                                 0, 0, 0);
                        else
                            asm volatile("" : "+v"(acc[i][c2]) : "v"(wcur[2 * c + c2]), "v"(xv[i]));
                    }
                    if (SNK_DL3_VAR != 4)
                        xv[i] = xread(nk, nc, i);
                    else
                        asm volatile("" : "+v"(xv[i]));
                }
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) wcur[q] = wnext[q];
        }
        // LDS-only barriers (dfr_lds_barrier): a __syncthreads fence drained the pair's a3 stores
        // (and the ring's refills for the next pair) before the next pair's input loads were even
        // issued; the refills are counted by the offset loop's own vmcnt waits
        if (!blocked) {
            // epilogue: bias + relu + bf16, 4 channels per lane, row-major a3 [sample][position][64]
#pragma unroll
            for (int i = 0; i < TPS; ++i) {
                const int t = simd + 4 * i;
                if ((i == TPS - 1 && !last_ok) || r >= WO) continue;
                const int64_t sg = 2 * p + t / WO;
                if (sg >= S) continue;
                const int o = r + (t % WO) * WO;
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2)
                    *reinterpret_cast<u32x2 *>(y + (sg * WO * WO + o) * 64 + (2 * half + c2) * 16 + 4 * g) =
                        relu_bf16x4(acc[i][c2], bb[c2]);
            }
            dfr_lds_barrier();   // every wave is done reading this pair's inputs
            if (more && SNK_DL3_VAR != 1) {   // the next pair's inputs
#pragma unroll
                for (int u = 0; u < APT; ++u)
                    if (tid + u * 512 < APIECES) apark(u, apiece(pn, u));
            }
        } else {
            // blocked a3 (deep_dense1_kernel<4, true>'s reader): blocks of 16 samples x 32
            // features, 1 KB each, [sample / 16][f / 32][sample % 16][f % 32]. The pair's two
            // samples are two adjacent 64-byte rows of each block: the accumulators are staged in
            // the (now dead) input region as [f / 32][pair sample][32], 8-byte slot k of each
            // 128-byte unit b at k ^ ((b >> 1) & 15) (a store's sixteen positions on sixteen bank
            // pairs), then leave as whole 128-byte lines, 16 bytes per lane. The next pair's input
            // loads go out before those stores, and the wait for them counts the stores out.
            constexpr int NU = WO * WO * 2;   // 128-byte units (blocks) per pair
            static_assert(NU * 128 <= 2 * Sh::XS * 2, "a3 staging fits the input region");
            dfr_lds_barrier();   // every wave is done reading this pair's inputs
            int ln_ = lane, tq_ = tid;   // opaque: the addresses below are computed here (hoisted
            asm volatile("" : "+v"(ln_), "+v"(tq_));   // above the offset loop, they were spilled)
            const int r = ln_ & 15, g = ln_ >> 4;
#pragma unroll
            for (int i = 0; i < TPS; ++i) {
                const int t = simd + 4 * i;
                if ((i == TPS - 1 && !last_ok) || r >= WO) continue;
                const int o = r + (t % WO) * WO, j = t / WO;
#pragma unroll
                for (int c2 = 0; c2 < 2; ++c2) {
                    const int f = o * 64 + (2 * half + c2) * 16 + 4 * g, b = f >> 5;
                    const int slot = (j * 8 + ((f & 31) >> 2)) ^ ((b >> 1) & 15);
                    *reinterpret_cast<u32x2 *>(As + b * 64 + slot * 4) = relu_bf16x4(acc[i][c2], bb[c2]);
                }
            }
            dfr_lds_barrier();
            u32x4 av[APT];
            if (more && SNK_DL3_VAR != 1) {
#pragma unroll
                for (int u = 0; u < APT; ++u)
                    if (tid + u * 512 < APIECES) av[u] = apiece(pn, u);
            }
            asm volatile("" ::: "memory");   // the loads stay ahead of the stores (the counted wait)
            constexpr int NQ = NU * 8, QT = (NQ + 511) / 512;   // 16-byte pieces
            uint16_t *yb = y + ((2 * p) >> 4) * (int64_t)(NU * 512) + ((2 * p) & 15) * 32;
            const bool both = 2 * p + 1 < S;   // an odd S: the last pair's second row stays unwritten
#pragma unroll 2
            for (int u = 0; u < QT; ++u) {
                const int q = tq_ + u * 512;
                if (q < NQ) {
                    const int b = q >> 3, k = q & 7, m = (b >> 1) & 15;
                    const u32x4 v = *reinterpret_cast<const u32x4 *>(As + b * 64 + (((2 * k) ^ m) & ~1) * 4);
                    if (both || k < 4)   // pieces 0..3: the first sample's row
                        *reinterpret_cast<u32x4 *>(yb + b * 512 + k * 8) = (m & 1) ? u32x4{v[2], v[3], v[0], v[1]} : v;
                }
            }
            if (more && SNK_DL3_VAR != 1) {
                // this wave's input loads landed (the stores after them may not): every wave issued
                // at least MINST of them (the last wave the fewest)
                constexpr int MINST = NQ > 448 ? (NQ - 449) / 512 + 1 : 0;
                __builtin_amdgcn_s_waitcnt(waitcnt_vm(MINST));
                dfr_lds_barrier();   // every wave's staging reads are done: the region takes the inputs
#pragma unroll
                for (int u = 0; u < APT; ++u)
                    if (tid + u * 512 < APIECES) apark(u, av[u]);
            }
        }
        dfr_lds_barrier();
    }
    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // the ring's last refills land before the workgroup ends
}

// ---------------------------------------------------------------- Dense1
// slab[z][s][o] = sum_{f in split z} a4[s][f] * W1[f][o]; 4 waves x 16*NR
// samples per workgroup, all 64 outputs (4 column tiles); A and B fragments
// straight from global (the 1.8 MB bf16 image stays L2-resident), two k-steps
// in flight. NR row tiles per wave reuse each B fragment NR times: the B
// stream from L2 is 1.8 MB per wave, so at 65,536 samples NR = 4 cuts it from
// 7.4 GB (NR = 1) to 1.8 GB; small batches keep NR = 1 and split K instead.
// BLOCKED: a4 in deep_conv3_kernel's blocked layout (16 samples x 32 features per 1 KB block):
// each A fragment load reads one whole block, 1 KB contiguous, where the row-major layout gave
// 16 rows x 64 bytes 28.8 KB apart (4.4 TB/s of HBM on the 1.89 GB a3 stream)
template <int NR, bool BLOCKED = false>
__global__ __launch_bounds__(256) void deep_dense1_kernel(const uint16_t *__restrict__ a4,
                                                          const uint16_t *__restrict__ w1img, int64_t S, int K1,
                                                          int kchunk, float *__restrict__ slab) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * 64 * NR + wave * 16 * NR;
    const int k0 = blockIdx.y * kchunk, k1 = min(K1, k0 + kchunk);
    const uint16_t *pa[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t)
        pa[t] = BLOCKED ? a4 + min((row0 + 16 * t) >> 4, (S - 1) >> 4) * (int64_t)(K1 / 32) * 512 + r * 32 + g * 8
                        : a4 + min(row0 + 16 * t + r, S - 1) * K1 + g * 8;
    // the A fragment of k offset kk (a multiple of 32) of row tile t
    auto aptr = [&](int t, int kk) __attribute__((always_inline)) {
        return BLOCKED ? pa[t] + (int64_t)(kk >> 5) * 512 : pa[t] + kk;
    };
    const uint16_t *pb = w1img + (int64_t)r * K1 + g * 8;
    f32x4 acc[NR][4];
#pragma unroll
    for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // 64-k steps through a ring of RING register sets, loaded RING - 1 steps ahead: the A
    // stream comes from HBM (a4 is written by L3 just before and is far larger than the
    // MALL), and two steps in flight per wave (one ahead) left it latency-bound
#ifndef DEEP_D1_RING
#define DEEP_D1_RING 6
#endif
    constexpr int RING = NR == 4 ? DEEP_D1_RING : 4;
    const int nst = (k1 - k0) / 64;
    u32x4 a[RING][NR][2], b[RING][2][4];
    auto load = [&](int st, u32x4 (&ar)[NR][2], u32x4 (&br)[2][4]) __attribute__((always_inline)) {
        const int kk = k0 + 64 * st;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
#pragma unroll
            for (int t = 0; t < NR; ++t) ar[t][u] = *reinterpret_cast<const u32x4 *>(aptr(t, kk + 32 * u));
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) br[u][nt] = *reinterpret_cast<const u32x4 *>(pb + nt * 16 * (int64_t)K1 + kk + 32 * u);
        }
    };
#pragma unroll
    for (int o = 0; o < RING - 1; ++o)
        if (o < nst) load(o, a[o], b[o]);
#pragma unroll 1
    for (int st = 0; st < nst; st += RING) {
#pragma unroll
        for (int o = 0; o < RING; ++o) {
            if (st + o < nst) {   // wave-uniform
                if (st + o + RING - 1 < nst) load(st + o + RING - 1, a[(o + RING - 1) % RING], b[(o + RING - 1) % RING]);
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int t = 0; t < NR; ++t)
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt)
                            acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(a[o][t][u]), as_bf(b[o][u][nt]),
                                                                                 acc[t][nt], 0, 0, 0);
            }
        }
    }
    for (int k = k0 + 64 * nst; k < k1; k += 32) {
        u32x4 b[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) b[nt] = *reinterpret_cast<const u32x4 *>(pb + nt * 16 * (int64_t)K1 + k);
#pragma unroll
        for (int t = 0; t < NR; ++t) {
            const u32x4 a = *reinterpret_cast<const u32x4 *>(aptr(t, k));
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

// deep_dense1_ldsb_kernel: deep_dense1_kernel<NR, true> for an unsplit K (K1 % 64 == 0) with
// the W1 (B) fragments of each 64-k step staged ONCE per workgroup in LDS by LDS-DMA (8 KB:
// 64 output rows x 128 bytes, 16-byte chunk c of row n at c ^ (n & 7), so a fragment read's
// eight-lane groups hit distinct banks), each wave issuing two of the step's eight 1 KB DMAs,
// instead of each of the four waves loading all eight from L2 itself. A wave's vector-memory
// queue (vmcnt <= 63) then holds the A (HBM) loads of D1L_RB - 1 steps ahead, where 16 loads a
// step had left room for ~4; one LDS-only barrier per step publishes the step's B. Same
// products and fp32 accumulation order as deep_dense1_kernel (per accumulator: k ascending).
#ifndef DEEP_D1L_RB
#define DEEP_D1L_RB 8
#endif
constexpr int D1L_RB = DEEP_D1L_RB;   // LDS slots = register ring entries; loads run D1L_RB - 1 steps ahead
template <int NR>
__global__ __launch_bounds__(256) void deep_dense1_ldsb_kernel(const uint16_t *__restrict__ a4,
                                                               const uint16_t *__restrict__ w1img, int64_t S, int K1,
                                                               float *__restrict__ slab) {
    constexpr int RB = D1L_RB, SLOT = 64 * 64;   // halves per slot
    static_assert(RB >= 3 && 10 * (RB - 2) <= 63, "the counted wait: vmcnt holds at most 63");
    __shared__ __attribute__((aligned(16))) uint16_t Bs[RB * SLOT];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r = lane & 15, g = lane >> 4;
    const int64_t row0 = (int64_t)blockIdx.x * 64 * NR + wave * 16 * NR;
    const uint16_t *pa[NR];
#pragma unroll
    for (int t = 0; t < NR; ++t)
        pa[t] = a4 + min((row0 + 16 * t) >> 4, (S - 1) >> 4) * (int64_t)(K1 / 32) * 512 + r * 32 + g * 8;
    // this lane's DMA sources: instruction j of this wave fills rows n = 8 (2 wave + j) + (lane >> 3),
    // lane-linear slot chunk lane & 7 <- global chunk (lane & 7) ^ (n & 7)
    const uint16_t *pbs[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = 8 * (2 * wave + j) + (lane >> 3);
        pbs[j] = w1img + (int64_t)n * K1 + (((lane & 7) ^ (n & 7)) << 3);
    }
    // B[k = 32u + 8g + (0..7)][n = 16 nt + r]: row n, chunk 4u + g of the slot
    int bo[2][4];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int n = 16 * nt + r;
            bo[u][nt] = n * 64 + (((4 * u + g) ^ (n & 7)) << 3);
        }
    f32x4 acc[NR][4];
#pragma unroll
    for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int nst = K1 / 64;
    u32x4 a[RB][NR][2];
    // step st: this wave's two B DMAs into slot st % RB, then its A loads (10 vector-memory
    // instructions, in this order, per step)
    auto issue = [&](int st, int slot, u32x4 (&ar)[NR][2]) __attribute__((always_inline)) {
        const int kk = 64 * st;
#pragma unroll
        for (int j = 0; j < 2; ++j)
            __builtin_amdgcn_global_load_lds((const void *)(pbs[j] + kk),
                                             (__attribute__((address_space(3))) void *)(Bs + slot * SLOT + (2 * wave + j) * 512),
                                             16, 0, 0);
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
            for (int t = 0; t < NR; ++t)
                ar[t][u] = *reinterpret_cast<const u32x4 *>(pa[t] + (int64_t)((kk >> 5) + u) * 512);
    };
#pragma unroll
    for (int o = 0; o < RB - 1; ++o)
        if (o < nst) issue(o, o, a[o]);
#pragma unroll 1
    for (int st = 0; st < nst; st += RB) {
#pragma unroll
        for (int o = 0; o < RB; ++o) {
            const int cs = st + o;
            if (cs < nst) {   // wave-uniform
                // step cs's loads landed (the RB - 2 later steps' may stay in flight), then every
                // wave's: slot o holds step cs's B, and every wave's reads of step cs - 1 are done
                if (cs + RB - 2 < nst)
                    __builtin_amdgcn_s_waitcnt(waitcnt_vm(10 * (RB - 2)));
                else
                    __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
                __builtin_amdgcn_s_barrier();
                // step cs + RB - 1 refills slot (o + RB - 1) % RB, last read at step cs - 1
                if (cs + RB - 1 < nst) issue(cs + RB - 1, (o + RB - 1) % RB, a[(o + RB - 1) % RB]);
                u32x4 b[2][4];
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt) b[u][nt] = *reinterpret_cast<const u32x4 *>(Bs + o * SLOT + bo[u][nt]);
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int t = 0; t < NR; ++t)
#pragma unroll
                        for (int nt = 0; nt < 4; ++nt)
                            acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf(a[o][t][u]), as_bf(b[u][nt]),
                                                                                 acc[t][nt], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int t = 0; t < NR; ++t)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int64_t row = row0 + 16 * t + 4 * g + e;
                if (row < S) slab[row * 64 + nt * 16 + r] = acc[t][nt][e];
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

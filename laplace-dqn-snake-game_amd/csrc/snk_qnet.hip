// snk_qnet.hip — Q-net forward / backward / RMSProp on gfx950.
//
// Forward (structs.jl:127-139 Chain): conv1 on VALU (K = 9*C is tiny), conv2,
// conv3 and Dense1 as implicit GEMMs on v_mfma_f32_32x32x2_f32, then one
// wave per sample for Dense2 with a mode-specific epilogue: epsilon_greedy
// (utils.jl:153-172), the TD target (utils.jl:448-451) or the Huber loss and
// its gradient (utils.jl:453-458). Backward (Zygote's gradient,
// utils.jl:461-464) runs the same GEMM engine with data-gradient and
// weight-gradient loaders; RMSProp (Optimisers.jl, utils.jl:429,466) is
// element-wise over the packed parameter vector.
#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "snk_conv_h3.hpp"
#include "snk_conv_h3f.hpp"
#include "snk_dense_h3.hpp"
#include "snk_bwd3.hpp"
#include "snk_conv_x6.hpp"
#include "snk_loaders.hpp"

#include "snk_qnet.hpp"
#include "snk_upd_fwd.hpp"

namespace snk {

// ---------------------------------------------------------------- layout
QLayout make_layout(int bs, int C) {
    QLayout L{};
    L.bs = bs;
    L.C = C;
    L.ncell = bs * bs;
    L.Wo = bs - 5;
    L.K1 = L.Wo * L.Wo * 64;
    int64_t o = 0;
    L.off_w1 = o; o += 9 * C * 16;
    L.off_b1 = o; o += 16;
    L.off_w2 = o; o += 9 * 16 * 32;
    L.off_b2 = o; o += 32;
    L.off_w3 = o; o += 36 * 32 * 64;
    L.off_b3 = o; o += 64;
    L.off_d1w = o; o += (int64_t)L.K1 * 64;
    L.off_d1b = o; o += 64;
    L.off_d2w = o; o += 3 * 64;
    L.off_d2b = o; o += 3;
    L.P = o;
    L.off_t2 = 0;
    L.off_t3 = 9 * 32 * 16;
    L.off_td = L.off_t3 + 36 * 64 * 32;
    L.T = L.off_td + (int64_t)L.Wo * L.Wo * 64 * 64;
    return L;
}

// block [nkk][CK][CN] of theta -> [nkk][CN][CK] of the image (c contiguous per output),
// and (wtb) its exact bf16 split planes [nkk][plane][CN][CK]
__global__ void transpose_fwd_kernel(const float *__restrict__ th, float *__restrict__ wt, uint16_t *__restrict__ wtb,
                                     QLayout L) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < L.T; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t base, u;
        int CK, CN;
        if (t < L.off_t3) {
            u = t; base = L.off_w2; CK = 16; CN = 32;
        } else if (t < L.off_td) {
            u = t - L.off_t3; base = L.off_w3; CK = 32; CN = 64;
        } else {
            u = t - L.off_td; base = L.off_d1w; CK = 64; CN = 64;
        }
        const int64_t kk = u / (CK * CN);
        const int r = (int)(u - kk * CK * CN);
        const int n = r / CK, c = r - n * CK;
        const float v = th[base + (kk * CK + c) * CN + n];
        wt[t] = v;
        if (wtb) {
            const int64_t x6 = 3 * (t - u) + kk * 3 * CK * CN + r;   // section base * 3 + [kk][plane][n][c]
#pragma unroll
            for (int p = 0; p < 3; ++p) wtb[x6 + p * CK * CN] = split_part(v, p);
        }
    }
}

void transpose_fwd_launch(const QLayout &L, const float *theta, float *wt, uint16_t *wtb, hipStream_t s) {
    transpose_fwd_kernel<<<(unsigned)std::min<int64_t>(ceil_div(L.T, 256), 2048), 256, 0, s>>>(theta, wt, wtb, L);
    launch_check("transpose_fwd_kernel");
}

void packed_to_flux_index(const QLayout &L, int32_t *perm) {
    auto conv = [&](int64_t off, int KS, int Cin, int Cout) {
        // packed W[(kk*Cin + ci)*Cout + co], kk = du + KS*dv  <-  flux w[KS-1-du, KS-1-dv, ci, co]
        for (int dv = 0; dv < KS; ++dv)
            for (int du = 0; du < KS; ++du)
                for (int ci = 0; ci < Cin; ++ci)
                    for (int co = 0; co < Cout; ++co) {
                        const int64_t pk = ((int64_t)(du + KS * dv) * Cin + ci) * Cout + co;
                        const int64_t fx = (KS - 1 - du) + (int64_t)KS * (KS - 1 - dv) + (int64_t)KS * KS * ci +
                                           (int64_t)KS * KS * Cin * co;
                        perm[off + pk] = (int32_t)(off + fx);
                    }
        const int64_t boff = off + (int64_t)KS * KS * Cin * Cout;
        for (int co = 0; co < Cout; ++co) perm[boff + co] = (int32_t)(boff + co);
    };
    conv(L.off_w1, 3, L.C, 16);
    conv(L.off_w2, 3, 16, 32);
    conv(L.off_w3, 6, 32, 64);
    const int np = L.Wo * L.Wo;
    // Dense1: packed W[p*64 + c][o] <- flux W[o, p + c*np] (Flux.flatten is column-major (i,j,c))
    for (int p = 0; p < np; ++p)
        for (int c = 0; c < 64; ++c)
            for (int o = 0; o < 64; ++o)
                perm[L.off_d1w + ((int64_t)p * 64 + c) * 64 + o] = (int32_t)(L.off_d1w + o + ((int64_t)p + (int64_t)c * np) * 64);
    for (int o = 0; o < 64; ++o) perm[L.off_d1b + o] = (int32_t)(L.off_d1b + o);
    // Dense2: packed W[a][o] <- flux W[a, o] (column-major a + 3o)
    for (int a = 0; a < 3; ++a)
        for (int o = 0; o < 64; ++o) perm[L.off_d2w + a * 64 + o] = (int32_t)(L.off_d2w + a + 3 * o);
    for (int a = 0; a < 3; ++a) perm[L.off_d2b + a] = (int32_t)(L.off_d2b + a);
}

// ---------------------------------------------------------------- paired launches
// Two independent jobs in one launch: blocks [0, n1) run job 1, the rest job 2
// (equal block sizes). The backward's weight and data gradients of a layer
// only share inputs, so each such pair costs one launch and runs side by side.
__device__ __forceinline__ dim3 unflatten(unsigned b, dim3 g) {
    dim3 r;
    r.x = b % g.x;
    b /= g.x;
    r.y = b % g.y;
    r.z = b / g.y;
    return r;
}
template <int NT, int KW, class AL, class BL, class EP>
struct GemmJob {
    AL al;
    BL bl;
    EP ep;
    int M, K, kchunk;
    dim3 grid;
    __device__ void operator()(dim3 bid) const { gemm_body<NT, KW>(al, bl, ep, M, K, kchunk, bid); }
};
template <int NT, int KW, class AL, class BL, class EP>
static GemmJob<NT, KW, AL, BL, EP> gemm_job(const AL &al, const BL &bl, const EP &ep, int64_t M, int N, int64_t K,
                                           const GemmPlan &p) {
    SNK_CHECK(p.kw == KW, SNK_ERR_INTERNAL, "paired GEMM plan has %d waves, job %d", p.kw, KW);
    return GemmJob<NT, KW, AL, BL, EP>{al, bl, ep, (int)M, (int)K, p.kchunk,
                                       dim3((unsigned)ceil_div(M, 32), (unsigned)ceil_div(N, NT * 32), (unsigned)p.z)};
}
template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
struct ConvJob {
    ConvPair pr;
    dim3 grid;
    __device__ void operator()(dim3 bid) const { conv_mfma_body<CK, CN, KS, PAD, MODE, EPI>(pr, bid); }
};
// the bf16x6 conv (snk_conv_x6.hpp) as a paired job; BSPLIT: weights split while staged
template <int CK, int CN, int KS, int PAD, int MODE, int EPI, bool PRE, bool BSPLIT>
struct ConvX6Job {
    ConvPair pr;
    dim3 grid;
    __device__ void operator()(dim3 bid) const { conv_x6_body<CK, CN, KS, PAD, MODE, EPI, PRE, BSPLIT>(pr, bid); }
};
template <int NTH, class J1, class J2>
__global__ __launch_bounds__(NTH) void pair_kernel(J1 j1, J2 j2) {
    const unsigned n1 = j1.grid.x * j1.grid.y * j1.grid.z;
    if (blockIdx.x < n1)
        j1(unflatten(blockIdx.x, j1.grid));
    else
        j2(unflatten(blockIdx.x - n1, j2.grid));
}
template <int NTH, class J1, class J2>
static void pair_launch(const J1 &j1, const J2 &j2, hipStream_t s) {
    const unsigned n1 = j1.grid.x * j1.grid.y * j1.grid.z, n2 = j2.grid.x * j2.grid.y * j2.grid.z;
    pair_kernel<NTH><<<n1 + n2, NTH, 0, s>>>(j1, j2);
    launch_check("pair_kernel");
}

template <int NT, class AL, class BL, class EP>
static void gemm(const AL &al, const BL &bl, const EP &ep, int64_t M, int N, int64_t K, const GemmPlan &p,
                 hipStream_t s) {
    dim3 grid((unsigned)ceil_div(M, 32), (unsigned)ceil_div(N, NT * 32), (unsigned)p.z);
    switch (p.kw) {
        case 1: gemm_kernel<NT, 1><<<grid, 64, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        case 2: gemm_kernel<NT, 2><<<grid, 128, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        case 4: gemm_kernel<NT, 4><<<grid, 256, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        default: gemm_kernel<NT, 8><<<grid, 512, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
    }
    launch_check("gemm_kernel");
}

// ---------------------------------------------------------------- LDS-staged conv
static int conv_splits(int64_t M, int nkk) {
    const int64_t wgs = ceil_div(M, 128);
    if (wgs >= 512) return 1;
    return (int)std::min<int64_t>(std::min(nkk, 16), ceil_div(512, wgs));
}

// kk splits of the conv3 data gradient (36 offsets)
static int dx_splits(int64_t M) { return conv_splits(M, 36); }

// wb != nullptr: the bf16x6 split-precision kernel on the weight planes wb
// ng groups (1 or 2) of the same geometry in one launch (grid.z = group);
// wb[g] != nullptr: the bf16x6 split-precision kernels on those weight planes
// kernel arguments of ng (1 or 2) groups, kk split in `splits` (updated to the used count)
static ConvPair make_conv_pair(const ConvArgs *ga, int ng, int &splits, const uint16_t *const *wb) {
    ConvPair pr{};
    const int kper = ceil_div(ga[0].nkk, splits);
    splits = ceil_div(ga[0].nkk, kper);
    const FastDiv d2((uint32_t)std::max(1, ga[0].HOUT * ga[0].HOUT)), d1((uint32_t)std::max(1, ga[0].HOUT));
    for (int g = 0; g < 2; ++g) {
        ConvArgs a = ga[g < ng ? g : 0];
        a.kk_per_split = kper;
        a.d2m = d2.m; a.d2s = d2.s; a.d1m = d1.m; a.d1s = d1.s;
        pr.g[g] = a;
        pr.wb[g] = wb ? wb[g < ng ? g : 0] : nullptr;
    }
    return pr;
}

// conv3 on the h3 kernel (snk_conv_h3.hpp) for an HIN x HIN input
template <int KS, int EPI, int HIN>
static void h3s_launch(const ConvPair &pr, int ng, int splits, hipStream_t s) {
    const ConvArgs &a = pr.g[0];
    const int ho2 = a.HOUT * a.HOUT;
    const int S = a.M / ho2;
    const size_t lds = conv_h3s_lds(a.HIN);
    SNK_CHECK(splits == 1 && lds && S * ho2 == a.M && a.HOUT == HIN - KS + 1 && !a.xb && a.x && a.w &&
                  (ng == 1 || pr.g[1].wmax),
              SNK_ERR_INTERNAL, "h3s conv3 geometry");
    // dynamic bytes only: the kernel's static LDS counts against the 160 KB
    set_lds_limit((const void *)conv_h3s_kernel<KS, EPI, HIN>, lds);
    const dim3 g3((unsigned)ceil_div(S, 4), 1, (unsigned)ng);
    conv_h3s_kernel<KS, EPI, HIN><<<g3, 512, lds, s>>>(pr, S);
    launch_check("conv_h3s_kernel");
}

template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
static void conv_launch(const ConvArgs *ga, int ng, int splits, hipStream_t s, const uint16_t *const *wb = nullptr) {
    const ConvPair pr = make_conv_pair(ga, ng, splits, wb);
    const ConvArgs &a = pr.g[0];
    dim3 grid((unsigned)ceil_div(a.M, 128), (unsigned)splits, (unsigned)ng);
    if constexpr (MODE == MODE_FWD && CN == 64 && CK == 32 && KS == 6 && PAD == 0 && EPI == EPI_BIAS_RELU) {
        if (a.wmax) {   // fp16 h3 split, four samples resident in LDS (forward_layers chose it: h3s_ok)
            switch (a.HIN) {
                case 8: h3s_launch<KS, EPI, 8>(pr, ng, splits, s); return;
                case 9: h3s_launch<KS, EPI, 9>(pr, ng, splits, s); return;
                case 10: h3s_launch<KS, EPI, 10>(pr, ng, splits, s); return;
                case 11: h3s_launch<KS, EPI, 11>(pr, ng, splits, s); return;
                case 12: h3s_launch<KS, EPI, 12>(pr, ng, splits, s); return;
                case 13: h3s_launch<KS, EPI, 13>(pr, ng, splits, s); return;
                default: SNK_CHECK(false, SNK_ERR_INTERNAL, "h3s conv3: board side outside 8..13");
            }
        }
    }
    if constexpr (MODE == MODE_DX) {
        // conv3 data gradients on the bf16x6 split (dz3 and the fp32 weights split in
        // the kernel: 2.7x the exact-fp32 MFMA rate, same error class)
        conv_x6_split_kernel<CK, CN, KS, PAD, MODE, EPI><<<grid, 256, 0, s>>>(pr);
        launch_check("conv_x6_split_kernel");
        return;
    }
    if constexpr (MODE != MODE_DX) {
        if (pr.wb[0]) {
            if constexpr (MODE == MODE_FWD && CK % 32 == 0 && EPI != EPI_RELU_MASK) {
                if (a.xb) {   // pre-split input, 32-channel chunks: the 16x16x32 layouts
                    if constexpr (CN == 64 && PAD == 0 && CK == 32 && KS == 6 && EPI == EPI_BIAS_RELU) {
                        // large batches: four samples' planes resident in LDS per workgroup
                        // SNK_ARITH_X6S = 0 (tests): x6m16 instead, the same sums in the same order
                        const bool x6s = arith(SNK_ARITH_X6S) != 0;
                        constexpr int smin = 1024;
                        const int ho2 = a.HOUT * a.HOUT;
                        const int S = a.M / ho2;
                        const size_t lds = conv_x6s_lds(a.HIN);
                        if (x6s && splits == 1 && lds && S >= smin && S * ho2 == a.M && a.HOUT == a.HIN - 5) {
                            set_lds_limit((const void *)conv_x6s_kernel<KS, EPI>, lds);
                            const dim3 g3((unsigned)ceil_div(S, 4), 1, (unsigned)ng);
                            conv_x6s_kernel<KS, EPI><<<g3, 512, lds, s>>>(pr, S);
                            launch_check("conv_x6s_kernel");
                            return;
                        }
                    }
                    conv_x6m16_kernel<CK, CN, KS, PAD, EPI, 4><<<grid, 256, 0, s>>>(pr);
                    launch_check("conv_x6m16_kernel");
                    return;
                }
            }
            if (a.xb)
                conv_x6_kernel<CK, CN, KS, PAD, MODE, EPI, true><<<grid, 256, 0, s>>>(pr);
            else
                conv_x6_kernel<CK, CN, KS, PAD, MODE, EPI, false><<<grid, 256, 0, s>>>(pr);
            launch_check("conv_x6_kernel");
            return;
        }
    }
    SNK_CHECK(!a.xb && !a.outb, SNK_ERR_INTERNAL, "bf16 planes need the x6 kernels");
    conv_mfma_kernel<CK, CN, KS, PAD, MODE, EPI><<<grid, 256, 0, s>>>(pr);
    launch_check("conv_mfma_kernel");
}
template <int CK, int CN, int KS, int PAD, int MODE, int EPI>
static void conv_launch(ConvArgs a, int splits, hipStream_t s, const uint16_t *wb = nullptr) {
    conv_launch<CK, CN, KS, PAD, MODE, EPI>(&a, 1, splits, s, &wb);
}

// finish a kk-split conv: out = relu(sum_z slab[z] + bias)  or  (act > 0) * sum_z slab[z]
struct ReduceArgs {
    const float *slab, *bias, *act;
    float *out;
    uint16_t *outb;   // bf16 planes [row][3][N]
};
struct ReducePair {
    ReduceArgs g[2];
};
__global__ void conv_reduce_kernel(ReducePair rp, int splits, int64_t MN, int N) {
    const ReduceArgs &r = rp.g[blockIdx.y];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < MN; i += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.0f;
        for (int z = 0; z < splits; ++z) v += r.slab[(int64_t)z * MN + i];
        if (r.bias) {
            v += r.bias[i % N];
            v = v > 0.0f ? v : 0.0f;
            if (r.out) r.out[i] = v;
            if (r.outb) {
                const int64_t row = i / N;
                const int col = (int)(i - row * N);
#pragma unroll
                for (int p = 0; p < 3; ++p) r.outb[(row * 3 + p) * N + col] = split_part(v, p);
            }
        } else {
            r.out[i] = r.act[i] > 0.0f ? v : 0.0f;
        }
    }
}
static void conv_reduce_launch(const ReduceArgs *ra, int ng, int splits, int64_t MN, int N, hipStream_t s) {
    ReducePair rp{};
    rp.g[0] = ra[0];
    rp.g[1] = ra[ng > 1 ? 1 : 0];
    dim3 grid((unsigned)std::min<int64_t>(ceil_div(MN, 256), 4096), (unsigned)ng);
    conv_reduce_kernel<<<grid, 256, 0, s>>>(rp, splits, MN, N);
    launch_check("conv_reduce_kernel");
}

// one forward layer's operands for one net
struct FwdIO {
    const float *x, *w, *bias;
    float *out;
    const uint16_t *wb, *xb;   // x6: weight planes, pre-split input planes
    uint16_t *outb;            // x6: also write the output's planes
    QWork *wk;                 // its workspace (conv slab)
    const float *wmax = nullptr;   // h3 conv3: partial max |w| of the fp32 image w
    int nwmax = 0;
};

// out = conv (bias + relu) for ng nets at once, kk-split through the conv slabs when the grid is small
template <int CK, int CN, int KS, int PAD>
static void conv_fwd(const FwdIO *io, int ng, int64_t M, int HIN, int HOUT, hipStream_t s) {
    ConvArgs ga[2];
    const uint16_t *wb[2];
    const int sp = conv_splits(M * ng, KS * KS);
    for (int g = 0; g < ng; ++g) {
        ConvArgs a{};
        a.x = io[g].x; a.w = io[g].w; a.bias = io[g].bias; a.M = (int)M; a.HIN = HIN; a.HOUT = HOUT;
        a.nkk = KS * KS; a.xb = io[g].xb; a.wmax = io[g].wmax; a.nwmax = io[g].nwmax;
        if (sp == 1) {
            a.out = io[g].out;
            a.outb = io[g].outb;
        } else {
            a.out = io[g].wk->cslab;
            SNK_CHECK((int64_t)sp * M * CN <= io[g].wk->cslab_floats, SNK_ERR_INTERNAL, "conv slab too small");
        }
        ga[g] = a;
        wb[g] = io[g].wb;
    }
    if (sp == 1) {
        conv_launch<CK, CN, KS, PAD, MODE_FWD, EPI_BIAS_RELU>(ga, ng, 1, s, wb);
        return;
    }
    conv_launch<CK, CN, KS, PAD, MODE_FWD, EPI_SLAB>(ga, ng, sp, s, wb);
    const int used = ceil_div(KS * KS, ceil_div(KS * KS, sp));
    ReduceArgs ra[2];
    for (int g = 0; g < ng; ++g) ra[g] = ReduceArgs{io[g].wk->cslab, io[g].bias, nullptr, io[g].out, io[g].outb};
    conv_reduce_launch(ra, ng, used, M * CN, CN, s);
}

// ---------------------------------------------------------------- conv1 (VALU)
// 3x3, C -> 16, pad 1 (K = 9C is too small for MFMA). A workgroup owns NS
// samples: their input planes go to LDS once as floats inside a zero border
// ((bs+2)^2 per plane), so the 9C taps of an output are unconditional LDS
// reads; one thread per output position writes its 16 channels as 4 float4.
// yb (optional): the output also as bf16 split planes [S*bs*bs][3][16] (x6 conv2 input);
// y may then be null. NS samples per workgroup (fewer for small batches: more CUs busy).
// Two nets per launch (grid.y = group) as for the conv_* kernels.
struct Conv1Args {
    BoardSrc src;
    const float *w, *b;
    float *y;
    uint16_t *yb;
    float *x0;   // optional: the input planes as floats [S][C][bs*bs] (training: conv1 weight gradient)
    const float *wscan;   // optional: also write per-block partial max |wscan[0, wscan_n)| to wpart
    int64_t wscan_n;      //   (the h3 conv3's weight scale, see snk_conv_h3.hpp)
    float *wpart;
};
struct Conv1Pair {
    Conv1Args g[2];
    SampleRider rider;   // rider.out: the last workgroup of grid.y = 0 runs the replay sample
};
template <int C>
__global__ __launch_bounds__(256) void conv1_fwd_kernel(Conv1Pair cp, int64_t S, int bs, int NS) {
    // the rider is workgroup 0 (dispatched first, so its serial loop overlaps conv1)
    const int rb = cp.rider.out ? 1 : 0;
    if (rb && blockIdx.x == 0) {
        if (blockIdx.y == 0 && threadIdx.x < 64) sample_wave(cp.rider);
        return;
    }
    const int bx = (int)blockIdx.x - rb;
    const Conv1Args &ca = cp.g[blockIdx.y];
    const BoardSrc &src = ca.src;
    const float *__restrict__ w = ca.w;
    const float *__restrict__ b = ca.b;
    float *__restrict__ y = ca.y;
    uint16_t *__restrict__ yb = ca.yb;
    extern __shared__ __attribute__((aligned(16))) float sm[];
    float *sw = sm;                       // [9*C*16 + 16]
    float *sx = sm + 9 * C * 16 + 16;     // [NS][C][(bs+2)^2]
    const int bp = bs + 2, plane = bp * bp, ncell = bs * bs;
    for (int i = threadIdx.x; i < 9 * C * 16; i += blockDim.x) sw[i] = w[i];
    if (threadIdx.x < 16) sw[9 * C * 16 + threadIdx.x] = b[threadIdx.x];
    const int64_t s0 = (int64_t)bx * NS;
    const int ns = (int)min((int64_t)NS, S - s0);
    // plane base pointers once per (sample, channel): the element loads below
    // are then independent (no per-element ring-counter / slot-index load)
    __shared__ const int8_t *pbase[8 * C];
    if ((int)threadIdx.x < ns * C) pbase[threadIdx.x] = src.plane(s0 + threadIdx.x / C, threadIdx.x % C);
    for (int i = threadIdx.x; i < NS * C * plane; i += blockDim.x) sx[i] = 0.0f;
    if (ca.wscan) {   // block-uniform
        __shared__ float red4[4];
        wmax_block(ca.wscan, ca.wscan_n, ca.wpart, red4, (int)gridDim.x - rb, bx);
    }
    __syncthreads();
    const int nel = ns * C * ncell;
    for (int i0 = 0; i0 < nel; i0 += 8 * 256) {
        float v[8];   // eight loads in flight, then the stores
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + threadIdx.x;
            v[u] = 0.0f;
            if (i < nel) {
                const int sc = i / ncell, cell = i - sc * ncell;
                const int8_t *pl = pbase[sc];
                v[u] = pl ? (float)pl[cell] : src.fbase[(s0 * C + sc) * ncell + cell];
            }
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int i = i0 + u * 256 + threadIdx.x;
            if (i < nel) {
                const int sc = i / ncell, cell = i - sc * ncell;
                const int jj = cell / bs, ii = cell - jj * bs;
                sx[sc * plane + (ii + 1) + (jj + 1) * bp] = v[u];
                if (ca.x0) ca.x0[s0 * C * ncell + i] = v[u];
            }
        }
    }
    __syncthreads();
    // yb rows go out through LDS: 256 rows x 96 B per pass, written back as
    // consecutive 16-byte pieces (the direct stores were 16 B at a 96-B lane stride)
    u32x4 *stg = reinterpret_cast<u32x4 *>(sx + ((NS * C * plane + 3) & ~3));
    const int nq = ns * ncell;
    for (int q0 = 0; q0 < nq; q0 += 256) {
        const int q = q0 + threadIdx.x;
        if (q < nq) {
        // weights are re-read from LDS (16-byte broadcasts) for every position:
        // hoisted into registers they took 288 VGPRs at C = 2 (one wave per SIMD)
        asm volatile("" ::: "memory");
        const int sl = q / ncell, p = q - sl * ncell;
        const int j = p / bs, i = p - j * bs;
        const float4 *sw4 = reinterpret_cast<const float4 *>(sw);
        float acc[16];
#pragma unroll
        for (int v4 = 0; v4 < 4; ++v4) {
            const float4 b4 = sw4[9 * C * 4 + v4];
            acc[4 * v4] = b4.x; acc[4 * v4 + 1] = b4.y; acc[4 * v4 + 2] = b4.z; acc[4 * v4 + 3] = b4.w;
        }
#pragma unroll
        for (int kk = 0; kk < 9; ++kk) {
            const int du = kk % 3, dv = kk / 3;   // input (i+du-1, j+dv-1) = bordered (i+du, j+dv)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const float v = sx[(sl * C + c) * plane + (i + du) + (j + dv) * bp];
#pragma unroll
                for (int v4 = 0; v4 < 4; ++v4) {
                    const float4 w4 = sw4[(kk * C + c) * 4 + v4];
                    acc[4 * v4] = __builtin_fmaf(v, w4.x, acc[4 * v4]);
                    acc[4 * v4 + 1] = __builtin_fmaf(v, w4.y, acc[4 * v4 + 1]);
                    acc[4 * v4 + 2] = __builtin_fmaf(v, w4.z, acc[4 * v4 + 2]);
                    acc[4 * v4 + 3] = __builtin_fmaf(v, w4.w, acc[4 * v4 + 3]);
                }
            }
        }
#pragma unroll
        for (int co = 0; co < 16; ++co) acc[co] = fmaxf(acc[co], 0.f);
        const int64_t row = s0 * ncell + q;
        if (y) {
            float4 *o = reinterpret_cast<float4 *>(y + row * 16);
#pragma unroll
            for (int v = 0; v < 4; ++v) o[v] = make_float4(acc[4 * v], acc[4 * v + 1], acc[4 * v + 2], acc[4 * v + 3]);
        }
        if (yb) {
            u32x4 *o = stg + threadIdx.x * 6;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                const Split3 sp = split3(f32x4{acc[8 * half], acc[8 * half + 1], acc[8 * half + 2], acc[8 * half + 3]},
                                         f32x4{acc[8 * half + 4], acc[8 * half + 5], acc[8 * half + 6],
                                               acc[8 * half + 7]});
                o[0 + half] = sp.h;   // plane p, channels 8*half..8*half+7
                o[2 + half] = sp.m;
                o[4 + half] = sp.l;
            }
        }
        }
        if (yb) {
            __syncthreads();
            const int n16 = min(256, nq - q0) * 6;
            u32x4 *dst = reinterpret_cast<u32x4 *>(yb + (s0 * ncell + q0) * 48);
            for (int e = threadIdx.x; e < n16; e += 256) dst[e] = stg[e];
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------- heads
// (wave_sum: snk_upd_fwd.hpp)

template <int MODE>
__global__ __launch_bounds__(256) void head_kernel(const float *__restrict__ slab, int ks, int64_t S,
                                                   const float *__restrict__ theta, QLayout L,
                                                   float *__restrict__ h1o, float *__restrict__ qo, HeadArgs ha) {
    const int lane = threadIdx.x & 63;
    if (MODE == HEAD_ACT && ha.rider.out && blockIdx.x == gridDim.x - 1) {   // the rider's workgroup
        if (threadIdx.x < 64) sample_wave(ha.rider);
        return;
    }
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    // the K-split slab loads all in flight at once (a runtime-bounded loop waited for each)
    constexpr int KMAX = 16;
    float zv[KMAX];
#pragma unroll
    for (int z = 0; z < KMAX; ++z)
        if (z < ks) zv[z] = slab[((int64_t)z * S + s) * 64 + lane];
    float w2[3], b2[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        w2[a] = theta[L.off_d2w + a * 64 + lane];
        b2[a] = theta[L.off_d2b + a];
    }
    float h = theta[L.off_d1b + lane];
    if (ks <= KMAX) {
#pragma unroll
        for (int z = 0; z < KMAX; ++z)
            if (z < ks) h += zv[z];
    } else {
        for (int z = 0; z < ks; ++z) h += slab[((int64_t)z * S + s) * 64 + lane];
    }
    h = h > 0.0f ? h : 0.0f;
    h1o[s * 64 + lane] = h;
    float q[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) q[a] = b2[a] + wave_sum(w2[a] * h);
    if (MODE == HEAD_LOSS && ha.dz1) {
        // head_bwd fused: dz1 = (h1 > 0) * sum_a dq[a] W2[a][o] with dq one-hot at the taken action
        const int64_t m = ha.idx ? ha.idx[s] : s;
        const int a = ha.act_idx[m] % 3;
        const double e = (double)q[a] - ha.target[s];
        const double ae = fabs(e);
        const float g = (float)((ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / (double)ha.B);
        ha.dz1[s * 64 + lane] = h > 0.0f ? g * (a == 0 ? w2[0] : a == 1 ? w2[1] : w2[2]) : 0.0f;
    }
    if (lane != 0) return;
    qo[s * 3 + 0] = q[0];
    qo[s * 3 + 1] = q[1];
    qo[s * 3 + 2] = q[2];
    if (MODE == HEAD_ACT) {
        // utils.jl:161-169: Float32(rand()) < epsilon ? rand(av) : av[argmax(Q)]
        const uint64_t t = *ha.tptr;
        const float eps = ha.eps_dev ? *ha.eps_dev : ha.epsilon;
        const float u = rng_uniform(rng_hash(ha.seed, (uint64_t)s, t));
        int a;
        if (u < eps) {
            a = (int)((rng_hash(ha.seed ^ 0xA5A5A5A5A5A5A5A5ULL, (uint64_t)s, t) >> 32) % 3);
        } else {
            a = 0;  // argmax: first maximum
            if (q[1] > q[a]) a = 1;
            if (q[2] > q[a]) a = 2;
        }
        ha.act[s] = (uint8_t)a;
    } else if (MODE == HEAD_TARGET) {
        // utils.jl:448-451 (Float64 promotion of the 0.97 literal)
        const int64_t m = ha.idx ? ha.idx[s] : s;
        const uint8_t mk = ha.mask[m];
        float mx = -INFINITY;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float v = ((mk >> a) & 1) ? -100.0f : q[a];
            mx = v > mx ? v : mx;
        }
        ha.target[s] = (double)ha.rew[m] + ha.gamma * (double)mx * (double)(1 - (int)ha.done[m]);
    } else if (MODE == HEAD_LOSS) {
        // utils.jl:453-458 Flux.huber_loss(delta = 1, agg = mean), its gradient
        const int64_t m = ha.idx ? ha.idx[s] : s;
        const int a = ha.act_idx[m] % 3;
        const double e = (double)q[a] - ha.target[s];
        const double ae = fabs(e);
        ha.loss[s] = ae < 1.0 ? 0.5 * e * e : ae - 0.5;
        const double g = (ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / (double)ha.B;
#pragma unroll
        for (int k = 0; k < 3; ++k) ha.dq[s * 3 + k] = k == a ? (float)g : 0.0f;
    }
}

// HEAD_TARGET of t_net then HEAD_LOSS of q_net for the same sample in one wave
// (head_pair_one, snk_upd_fwd.hpp): the two head launches of an update in one
__global__ __launch_bounds__(256) void head_pair_kernel(HeadNet tn, HeadNet qn, int ks, int64_t S, QLayout L,
                                                        HeadArgs ha) {
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    head_pair_one(tn, qn, ks, S, L, ha, s, threadIdx.x & 63, head_pre(ha, s));
}

// backward of Dense2 + relu: dz1[s][o] = (h1 > 0) * sum_a dq[s][a] W2[a][o]
// Dense1's backward at the update's batch (S <= 64) in one launch of small LDS-staged
// GEMMs on the fp64 matrix cores (v_mfma_f64_16x16x4_f64: fp32 operands converted exactly,
// products exact, sums in fp64, rounded once). The generic split-K pair (pair_kernel, f32
// MFMA, operands gathered element by element through the implicit loaders) took 11 us for
// 2 x 26 MFLOP. Blocks, each owning a block of D1B_F features f (K1 is a multiple of 64):
//  * [0, nfb): dz3[s][f] = (a3[s][f] > 0) * sum_o dz1[s][o] W1[f][o]   (M = s, N = f, K = o)
//  * [nfb, 2 nfb): dW1[f][o] = sum_s a3[s][f] dz1[s][o]                 (M = f, N = o, K = s)
//  * 2 nfb: the bias row dW1[K1][o] = sum_s dz1[s][o]
// The sums are more accurate than the fp32-accumulating forms (a VALU version with fp32 fma
// chains drifted the free-running configs[0] trajectory to 2e-5 of the oracle's loss).
// f64 16x16x4 operand map: lane l holds A[l & 15][k = l >> 4], B[k = l >> 4][l & 15]; D row
// (l >> 4) + 4i, column l & 15.
typedef double f64x4 __attribute__((ext_vector_type(4)));
constexpr int D1B_F = 32, D1B_P = 98, D1B_PA = 48;   // features per block, LDS row pitches (floats)
// D1B_P = 98 (34 mod 64): the dX fragment reads (row r, column kq: 34r + kq) and the dW reads
// of dz1 (row kq, column r: 34kq + r) both land on distinct banks per 32-lane half (66 made
// the dW reads 2-way)
__global__ __launch_bounds__(512) void d1_bwd_kernel(const float *__restrict__ a3, const float *__restrict__ dz1,
                                                     const float *__restrict__ w1, float *__restrict__ dz3,
                                                     float *__restrict__ dw, int S, int K1, int nfb) {
    __shared__ float sdz[64 * D1B_P];             // dz1 [s][o]
    __shared__ float sx[64 * D1B_P];              // dX: W1 rows [f][o]; dW: a3 [s][f] (pitch D1B_PA)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int r = lane & 15, kq = lane >> 4;
    const int b = blockIdx.x;
    const bool dx = b < nfb;
    const int f0 = (dx ? b : b - nfb) * D1B_F;
    // dX blocks: the relu mask a3 of this lane's four outputs, loaded with the staging (read after
    // the MFMAs it was one more round trip at the block's end)
    float mk[4] = {0.f, 0.f, 0.f, 0.f};
    if (dx) {
        const int mt = wave >> 1, nt = wave & 1;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = 16 * mt + kq + 4 * i;
            if (s < S) mk[i] = a3[(int64_t)s * K1 + f0 + 16 * nt + r];
        }
    }
    {   // staging: every float4 load first (dz1: 2 per thread, the W1 or a3 block: 1), then the LDS stores
        f32x4 vz[2], vx = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int q = tid + 512 * u, s = q >> 4;
            vz[u] = s < S ? *reinterpret_cast<const f32x4 *>(dz1 + q * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const int fx = tid >> 4, px = tid & 15;             // dX: W1 row f0 + fx, quad px
        const int sa = tid >> 3, pa = tid & 7;              // dW: a3 row sa, quad pa of the block
        if (b < 2 * nfb) {
            if (dx) vx = *reinterpret_cast<const f32x4 *>(w1 + (int64_t)(f0 + fx) * 64 + 4 * px);
            else if (sa < S) vx = *reinterpret_cast<const f32x4 *>(a3 + (int64_t)sa * K1 + f0 + 4 * pa);
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int q = tid + 512 * u, s = q >> 4, o = (q & 15) * 4;
#pragma unroll
            for (int e = 0; e < 4; ++e) sdz[s * D1B_P + o + e] = vz[u][e];
        }
        if (dx) {
#pragma unroll
            for (int e = 0; e < 4; ++e) sx[fx * D1B_P + 4 * px + e] = vx[e];
        } else {
#pragma unroll
            for (int e = 0; e < 4; ++e) sx[sa * D1B_PA + 4 * pa + e] = vx[e];
        }
    }
    __syncthreads();
    if (b == 2 * nfb) {   // bias row
        if (tid < 64) {
            double v = 0.0;
            for (int s = 0; s < S; ++s) v += (double)sdz[s * D1B_P + tid];
            dw[(int64_t)K1 * 64 + tid] = (float)v;
        }
        return;
    }
    // 8 output tiles per block, one per wave
    f64x4 acc = f64x4{0.0, 0.0, 0.0, 0.0};
    if (dx) {   // tile = wave: s tile wave >> 1 (of 4), f tile wave & 1 (of 2)
        const int mt = wave >> 1, nt = wave & 1;
#pragma unroll
        for (int k = 0; k < 64; k += 4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)sdz[(16 * mt + r) * D1B_P + k + kq],
                                                       (double)sx[(16 * nt + r) * D1B_P + k + kq], acc, 0, 0, 0);
        const int f = f0 + 16 * nt + r;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int s = 16 * mt + kq + 4 * i;
            if (s < S) dz3[(int64_t)s * K1 + f] = mk[i] > 0.0f ? (float)acc[i] : 0.0f;
        }
    } else {    // tile = wave: f tile wave >> 2 (of 2), o tile wave & 3 (of 4)
        const int mt = wave >> 2, nt = wave & 3;
#pragma unroll
        for (int k = 0; k < 64; k += 4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)sx[(k + kq) * D1B_PA + 16 * mt + r],
                                                       (double)sdz[(k + kq) * D1B_P + 16 * nt + r], acc, 0, 0, 0);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int f = f0 + 16 * mt + kq + 4 * i;
            dw[(int64_t)f * 64 + 16 * nt + r] = (float)acc[i];
        }
    }
}

__global__ __launch_bounds__(256) void head_bwd_kernel(const float *__restrict__ dq, const float *__restrict__ h1,
                                                       const float *__restrict__ theta, QLayout L, int64_t S,
                                                       float *__restrict__ dz1) {
    const int lane = threadIdx.x & 63;
    const int64_t s = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (s >= S) return;
    const float *w2 = theta + L.off_d2w;
    const float g = dq[s * 3] * w2[lane] + dq[s * 3 + 1] * w2[64 + lane] + dq[s * 3 + 2] * w2[128 + lane];
    dz1[s * 64 + lane] = h1[s * 64 + lane] > 0.0f ? g : 0.0f;
}

// Dense2 weight/bias gradient: 195 outputs reduced over S, the batch staged
// through LDS 64 samples at a time (coalesced loads, no dependent global reads)
__global__ __launch_bounds__(256) void d2_grad_kernel(const float *__restrict__ dq, const float *__restrict__ h1,
                                                      int64_t S, QLayout L, float *__restrict__ grad) {
    __shared__ float sdq[64 * 3], sh[64 * 64];
    const int t = threadIdx.x;
    const int a = t < 192 ? t / 64 : t - 192, o = t < 192 ? t - a * 64 : 0;
    float acc = 0.0f;
    for (int64_t s0 = 0; s0 < S; s0 += 64) {
        const int n = (int)min((int64_t)64, S - s0);
        __syncthreads();
        for (int i = t; i < n * 64; i += 256) sh[i] = h1[s0 * 64 + i];
        if (t < n * 3) sdq[t] = dq[s0 * 3 + t];
        __syncthreads();
        if (t < 192)
            for (int k = 0; k < n; ++k) acc = __builtin_fmaf(sdq[k * 3 + a], sh[k * 64 + o], acc);
        else if (t < 195)
            for (int k = 0; k < n; ++k) acc += sdq[k * 3 + a];
    }
    if (t < 192) grad[L.off_d2w + t] = acc;
    else if (t < 195) grad[L.off_d2b + a] = acc;
}

// out[i] = sum_z slab[z][i], z ascending; the slab loads go out 8 at a time (one load per
// dependent add waited on every load: 14.7 us for the 32 pair slabs of the deep L3 gradient)
__global__ void slab_reduce_kernel(const float *__restrict__ slab, int ks, int64_t MN, float *__restrict__ out) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < MN; i += (int64_t)gridDim.x * blockDim.x) {
        float v = 0.0f;
        int z = 0;
        for (; z + 8 <= ks; z += 8) {
            float t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = slab[(int64_t)(z + u) * MN + i];
#pragma unroll
            for (int u = 0; u < 8; ++u) v += t[u];
        }
        for (; z < ks; ++z) v += slab[(int64_t)z * MN + i];
        out[i] = v;
    }
}

__global__ void rmsprop_kernel(int64_t P, float *__restrict__ theta, float *__restrict__ acc,
                               const float *__restrict__ grad, float eta, float rho, float eps) {
    const float omr = 1.0f - rho;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x) {
        const float g = grad[i];
        const float qd = rho * acc[i] + omr * (g * g);
        acc[i] = qd;
        // correctly rounded sqrt and divide (HIP default; __fsqrt_rn would be
        // the native approximation) so the update matches Optimisers' Float32
        theta[i] = theta[i] - (g * eta) / (__builtin_sqrtf(qd) + eps);
    }
}

__global__ void loss_mean_kernel(const double *__restrict__ loss, int64_t B, double *__restrict__ out) {
    __shared__ double sh[256];
    double v = 0.0;
    for (int64_t i = threadIdx.x; i < B; i += blockDim.x) v += loss[i];
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) *out = sh[0] / (double)B;
}

// ---------------------------------------------------------------- workspace
void qwork_free(QWork &w) {
    for (void *p : {(void *)w.a1, (void *)w.a2, (void *)w.a2b, (void *)w.a1b, (void *)w.a3, (void *)w.slab, (void *)w.cslab,
                    (void *)w.h1, (void *)w.q,
                    (void *)w.dq, (void *)w.dz1, (void *)w.dz3, (void *)w.dz2, (void *)w.dzc1, (void *)w.x0, (void *)w.target,
                    (void *)w.loss, (void *)w.upd_ticket, (void *)w.h3f_ticket, (void *)w.wmax_part, (void *)w.w3h, (void *)w.w3e,
                    (void *)w.w2h, (void *)w.w1h, (void *)w.w1e, (void *)w.a3max})
        dfree(p);
    w = QWork{};
}

// Dense1 split over its Wo^2 positions: returns the number of partial slabs
// Dense1's K (the Wo^2 positions) split into partial slabs. Small batches: conv_splits.
// Batches of 1024+: about one workgroup per CU (4096 samples: 7 slabs of 7 positions on
// 224 workgroups, 1.6 % of the training iteration faster than 13 slabs of 4 on 416)
static int d1_split(const QLayout &L, int64_t S, int &kk_per) {
    const int nkk = L.Wo * L.Wo;
    int sp = conv_splits(S, nkk);
    if (S >= 1024) sp = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(nkk, 16), 256 / ceil_div(S, 128)));
    kk_per = ceil_div(nkk, sp);
    return ceil_div(nkk, kk_per);
}

static int64_t conv_slab_floats(const QLayout &L, int64_t S, bool train) {
    int64_t need = 0;
    auto add = [&](int64_t M, int nkk, int N) {
        const int sp = conv_splits(M, nkk);
        if (sp > 1) need = std::max(need, (int64_t)sp * M * N);
    };
    add(S * L.ncell, 9, 32);
    add(S * L.Wo * L.Wo, 36, 64);
    if (train) {
        const int sp = dx_splits(S * L.ncell);
        if (sp > 1) need = std::max(need, (int64_t)sp * S * L.ncell * 32);
    }
    return need;
}

void qwork_ensure(QWork &w, const QLayout &L, int64_t S, bool train) {
    int kc;
    const int64_t need_slab = (int64_t)d1_split(L, S, kc) * S * 64;
    const int64_t need_cslab = conv_slab_floats(L, S, train || w.has_train);
    if (S <= w.cap && need_slab <= w.slab_floats && need_cslab <= w.cslab_floats && (!train || w.has_train)) return;
    (void)hipStreamSynchronize(stream());
    const int64_t cap = std::max(S, w.cap);
    const int64_t slab = std::max({need_slab, w.slab_floats, (int64_t)d1_split(L, cap, kc) * cap * 64});
    const bool tr = train || w.has_train;
    const int64_t cslab = std::max({need_cslab, w.cslab_floats, conv_slab_floats(L, cap, tr)});
    const int64_t gen = w.gen + 1;
    qwork_free(w);
    w.gen = gen;
    w.cap = cap;
    w.slab_floats = slab;
    w.cslab_floats = cslab;
    w.cslab = dalloc<float>((size_t)std::max<int64_t>(cslab, 1));
    w.a1 = dalloc<float>((size_t)cap * L.ncell * 16);
    w.a2 = dalloc<float>((size_t)cap * L.ncell * 32);
    w.a2b = dalloc<uint16_t>((size_t)cap * L.ncell * 96);
    w.a1b = dalloc<uint16_t>((size_t)cap * L.ncell * 48);
    w.a3 = dalloc<float>((size_t)cap * L.K1);
    w.slab = dalloc<float>((size_t)slab);
    w.h1 = dalloc<float>((size_t)cap * 64);
    w.q = dalloc<float>((size_t)cap * 3);
    w.wmax_part = dalloc<float>((size_t)std::max<int64_t>(cap, 256));
    w.w3h = dalloc<uint16_t>((size_t)36 * 512 * 8);
    w.w3e = dalloc<int>(2);
    w.w2h = dalloc<uint16_t>((size_t)H3F_B2_CHUNKS * 8);
    w.w1h = dalloc<uint16_t>((size_t)L.Wo * L.Wo * 2 * 4096);
    w.w1e = dalloc<int>((size_t)L.Wo * L.Wo * 64);
    w.a3max = dalloc<float>((size_t)cap);
    w.h3f_ticket = dalloc<uint32_t>(1);
    SNK_HIP(hipMemsetAsync(w.h3f_ticket, 0, 4, stream()));
    SNK_HIP(hipMemsetAsync(w.w2h, 0, (size_t)H3F_B2_CHUNKS * 16, stream()));   // pads stay zero
    if (tr) {
        w.has_train = 1;
        w.dq = dalloc<float>((size_t)cap * 3);
        w.dz1 = dalloc<float>((size_t)cap * 64);
        w.dz3 = dalloc<float>((size_t)cap * L.K1);
        w.dz2 = dalloc<float>((size_t)cap * L.ncell * 32);
        w.dzc1 = dalloc<float>((size_t)cap * L.ncell * 16);
        w.x0 = dalloc<float>((size_t)cap * L.ncell * L.C);
        w.target = dalloc<double>(cap);
        w.loss = dalloc<double>(cap);
        w.upd_ticket = dalloc<uint32_t>(cap);
        SNK_HIP(hipMemsetAsync(w.upd_ticket, 0, (size_t)cap * 4, stream()));
    }
}

// ---------------------------------------------------------------- forward
// conv1 .. Dense1 (layers lo..hi) of ng nets over S samples each, one launch per layer
// conv3 of this forward on the fp16 h3 kernel (snk_conv_h3.hpp): split-precision
// (x6) nets, large batches, one unsplit launch. SNK_ARITH_H3S = 0: the bf16 x6 kernels.
static bool h3s_ok(const QLayout &L, const FwdNet *net, int ng, int64_t S) {
    const bool on = arith(SNK_ARITH_H3S) != 0;   // tests: x6 comparisons
    constexpr int smin = 1024;
    for (int g = 0; g < ng; ++g)
        if (!net[g].wtb) return false;
    return on && S >= smin && L.bs >= 8 && L.bs <= 13 && conv_h3s_lds(L.bs) && L.Wo == L.bs - 5 &&
           conv_splits(S * L.Wo * L.Wo * ng, 36) == 1;
}

template <int BS>
static void h3c2_launch_bs(const float *a1, const float *wimg, const float *b2, float *a2, int64_t S, hipStream_t s) {
    const size_t lds = conv_h3c2_lds<BS>();
    set_lds_limit((const void *)conv_h3c2_kernel<BS>, lds);
    conv_h3c2_kernel<BS><<<(unsigned)ceil_div(S, 2), 256, lds, s>>>(a1, wimg, b2, a2, (int)S);
    launch_check("conv_h3c2_kernel");
}

// the measurement hook's events (h3f_timing_hook): when armed, the launch goes through
// hipExtLaunchKernelGGL, which records them in the dispatch itself (kernel start / end, as
// rocprofv3's kernel trace: hipEventRecord packets around the launch also timed the CP's
// packet processing and the previous kernel's tail, +15 us)
static hipEvent_t g_h3f_ev[2] = {nullptr, nullptr};
template <class K>
static void h3f_dispatch(K kern, unsigned grid, size_t lds, hipStream_t s, const H3FArgs &fa, int S) {
    if (g_h3f_ev[0])
        hipExtLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, g_h3f_ev[0], g_h3f_ev[1], 0, fa, S);
    else
        kern<<<grid, 512, lds, s>>>(fa, S);
}
// conv3 B staging: 8 LDS buffers filled by LDS-DMA from the pre-split image (fa.w3h,
// w3_split_kernel) where they fit (board side <= 12); else 4 buffers split in registers.
// One barrier per offset pair either way.
template <int HIN, int CF>
static void h3f_launch_t(const H3FArgs &fa, int64_t S, hipStream_t s) {
    const int64_t ngroups = ceil_div(S, 4);
    const unsigned rb = fa.rider.out ? 1 : 0;
    if constexpr (h3f_lds_bytes<HIN, 8>() <= 160 * 1024) {
        // persistent (fa.ticket): one workgroup per CU (the LDS admits one), the groups by ticket
        const unsigned grid = (unsigned)((fa.ticket ? std::min<int64_t>(ngroups, cu_count()) : ngroups) + rb);
        constexpr size_t lds = (size_t)h3f_lds_bytes<HIN, 8>();
        SNK_CHECK(fa.w3h && fa.w3e, SNK_ERR_INTERNAL, "conv_h3f: no pre-split conv3 weights");
        set_lds_limit((const void *)conv_h3f_kernel<HIN, 8, CF>, lds);
        h3f_dispatch(conv_h3f_kernel<HIN, 8, CF>, grid, lds, s, fa, (int)S);
    } else {
        const unsigned grid = (unsigned)(ngroups + rb);
        SNK_CHECK(!fa.ticket, SNK_ERR_INTERNAL, "conv_h3f: persistent mode needs the LDS-DMA path");
        constexpr size_t lds = (size_t)h3f_lds_bytes<HIN, 4>();
        static_assert(lds <= 160 * 1024, "conv_h3f LDS");
        set_lds_limit((const void *)conv_h3f_kernel<HIN, 4, CF>, lds);
        h3f_dispatch(conv_h3f_kernel<HIN, 4, CF>, grid, lds, s, fa, (int)S);
    }
    launch_check("conv_h3f_kernel");
}
static bool h3f_dma(int bs) { return bs <= 12; }

// dense_h3_kernel instantiations: KPZ positions per slab (d1_split's kk_per), all slabs full
static bool dh3_ok(const QLayout &L, int ks, int kpz) {
    const bool on = arith(SNK_ARITH_DH3) != 0;   // tests: x6 comparisons
    return on && kpz == 7 && ks * kpz == L.Wo * L.Wo;
}
static void dh3_launch(const DenseH3Args &a, int ks, int kpz, hipStream_t s) {
    SNK_CHECK(kpz == 7 && ks * kpz == a.nkk && a.S > 0, SNK_ERR_INTERNAL, "dense_h3: slab split");
    constexpr size_t lds = (size_t)DH3_RING * DH3_SLOT;
    set_lds_limit((const void *)dense_h3_kernel<7>, lds);
    dense_h3_kernel<7><<<dim3((unsigned)ceil_div(a.S, DH3_ROWS), (unsigned)ks), DH3_NT, lds, s>>>(a);
    launch_check("dense_h3_kernel");
}
template <int HIN>
static void h3f_launch_bs(const H3FArgs &fa, int C, int64_t S, hipStream_t s) {
    if (C == 1)
        h3f_launch_t<HIN, 1>(fa, S, s);
    else
        h3f_launch_t<HIN, 2>(fa, S, s);
}

void h3f_timing_hook(hipEvent_t a, hipEvent_t b) {
    g_h3f_ev[0] = a;
    g_h3f_ev[1] = b;
}

static void conv_h3f_launch_(int bs, int C, const H3FArgs &fa, int64_t S, hipStream_t s);
static void conv_h3f_launch(int bs, int C, const H3FArgs &fa, int64_t S, hipStream_t s) {
    conv_h3f_launch_(bs, C, fa, S, s);
}
static void conv_h3f_launch_(int bs, int C, const H3FArgs &fa, int64_t S, hipStream_t s) {
    SNK_CHECK(S <= INT32_MAX, SNK_ERR_INTERNAL, "h3f batch");
    switch (bs) {
        case 8: h3f_launch_bs<8>(fa, C, S, s); return;
        case 9: h3f_launch_bs<9>(fa, C, S, s); return;
        case 10: h3f_launch_bs<10>(fa, C, S, s); return;
        case 11: h3f_launch_bs<11>(fa, C, S, s); return;
        case 12: h3f_launch_bs<12>(fa, C, S, s); return;
        case 13: h3f_launch_bs<13>(fa, C, S, s); return;
        default: SNK_CHECK(false, SNK_ERR_INTERNAL, "h3f: board side outside 8..13");
    }
}

static void conv_h3c2_launch(const QLayout &L, const FwdNet &n, int64_t S, hipStream_t s) {
    const float *a1 = n.w->a1, *wimg = n.wt + L.off_t2, *b2 = n.th + L.off_b2;
    float *a2 = n.w->a2;
    SNK_CHECK(S <= n.w->cap && S <= INT32_MAX, SNK_ERR_INTERNAL, "h3 conv2 batch");
    switch (L.bs) {
        case 8: h3c2_launch_bs<8>(a1, wimg, b2, a2, S, s); return;
        case 9: h3c2_launch_bs<9>(a1, wimg, b2, a2, S, s); return;
        case 10: h3c2_launch_bs<10>(a1, wimg, b2, a2, S, s); return;
        case 11: h3c2_launch_bs<11>(a1, wimg, b2, a2, S, s); return;
        case 12: h3c2_launch_bs<12>(a1, wimg, b2, a2, S, s); return;
        case 13: h3c2_launch_bs<13>(a1, wimg, b2, a2, S, s); return;
        default: SNK_CHECK(false, SNK_ERR_INTERNAL, "h3 conv2: board side outside 8..13");
    }
}

static bool h3c2_on() { return arith(SNK_ARITH_H3C2) != 0; }

// whether an act forward (no training work) of S samples runs conv2 + conv3 as conv_h3f_kernel
bool qnet_fused23(const QLayout &L, const float *th, const float *wt, const uint16_t *wtb, int64_t S, QWork &w) {
    const FwdNet net{th, wt, wtb, BoardSrc{}, &w};
    return h3s_ok(L, &net, 1, S) && h3c2_on() && !w.has_train;
}

static void forward_layers(const QLayout &L, const FwdNet *net, int ng, int64_t S, hipStream_t s, int lo, int hi,
                           const SampleRider *rider = nullptr) {
    const int lo0 = lo;   // lo as called (the fused act forward advances lo past conv3)
    const int bs = L.bs, nc = L.ncell;
    bool fresh_in[2] = {false, false};   // QWork::wmax_fresh holds for this forward only
    bool split_in[2] = {false, false};   // QWork::split_fresh likewise
    for (int g = 0; g < ng; ++g) {
        fresh_in[g] = net[g].w->wmax_fresh != 0;
        net[g].w->wmax_fresh = 0;
        split_in[g] = net[g].w->split_fresh != 0;
        net[g].w->split_fresh = 0;
    }
    const bool h3 = h3s_ok(L, net, ng, S);
    // h3 also for conv2 (conv_h3c2_kernel): conv1 then writes fp32 a1 only. SNK_H3C2=0: x6 conv2.
    const bool h3c2 = h3 && h3c2_on();
    const int64_t n3 = 36LL * 32 * 64;   // conv3 weight image floats
    // act forward (no backward needs a1/a2): conv1 + conv2 + conv3 in conv_h3f_kernel. Its
    // "conv1" slot is the conv3 weight-max scan (the h3 weight scale), which also carries
    // the sample rider.
    bool f123 = h3c2;
    for (int g = 0; g < ng; ++g) f123 = f123 && !net[g].w->has_train;
    // Dense1 on dense_h3_kernel: this call runs conv_h3f (which writes the per-sample a3
    // maxima) with the DMA'd weights (w3_split_kernel also splits Dense1) and then Dense1, at a
    // slab split the kernel is instantiated for
    // (prepared also when this call stops at conv3: a later Dense1-only call can use it)
    bool dh3prep = false;
    if (f123 && lo <= 2 && hi >= 2 && h3f_dma(L.bs)) {
        int kc;
        const int ks = d1_split(L, S, kc);
        dh3prep = dh3_ok(L, ks, kc);
    }
    bool dh3 = dh3prep && hi >= 3;
    if (f123 && hi >= 0 && lo <= 2) {
        for (int g = 0; g < ng; ++g) {
            const FwdNet &n = net[g];
            QWork &w = *n.w;
            const float *img = n.wt + L.off_t3;
            // a full forward rescans the image (it may have changed in place) unless the
            // trainer's previous grad_update wrote its partials (and no sample rides the scan)
            const bool fresh = fresh_in[g] && w.wmax_n && w.wmax_img == img;
            // the sample rider rides the weight-max scan when it runs, else the conv launch
            SampleRider rd = (rider && g == 0) ? *rider : SampleRider{};
            if (((lo <= 0 && hi >= 0) && !fresh) || !w.wmax_n || w.wmax_img != img) {
                wmax_scan_kernel<<<256 + (rd.out ? 1 : 0), 256, 0, s>>>(img, n3, w.wmax_part, rd);
                launch_check("wmax_scan_kernel");
                w.wmax_n = 256;
                w.wmax_img = img;
                rd = SampleRider{};
            }
            SNK_CHECK(!rd.out || (lo <= 2 && hi >= 1), SNK_ERR_INTERNAL, "sample rider without a launch");
            // the conv3 weights pre-split once for every workgroup, unless the grad_update that last
            // changed them wrote the split (the trainer's chained iterations)
            if (lo <= 2 && hi >= 1 && h3f_dma(L.bs) && !(split_in[g] && fresh)) {
                const int nkk = L.Wo * L.Wo;
                w3_split_kernel<<<W3S_BLOCKS + W2S_BLOCKS + (dh3prep ? w1s_blocks(nkk) : 0), 256, 0, s>>>(
                    img, w.wmax_part, w.wmax_n, w.w3h, w.w3e, n.wt + L.off_t2, w.w2h, dh3prep ? n.wt + L.off_td : nullptr,
                    w.w1h, w.w1e, w.split_grow);
                launch_check("w3_split_kernel");
            }
            if (lo <= 2 && hi >= 1) {
                H3FArgs fa{};
                if (h3f_dma(L.bs)) {
                    fa.w3h = w.w3h;
                    fa.w3e = w.w3e;
                    fa.w2h = w.w2h;
                }
                fa.rider = rd;
                fa.src = n.src; fa.w1 = n.th + L.off_w1; fa.b1 = n.th + L.off_b1;
                fa.w2 = n.wt + L.off_t2; fa.b2 = n.th + L.off_b2; fa.w3 = img; fa.wmax = w.wmax_part;
                fa.nwmax = w.wmax_n; fa.b3 = n.th + L.off_b3; fa.out = w.a3;
                fa.a3max = dh3prep ? w.a3max : nullptr;
                // persistent launch: boards from the env frame ring (replay slots would need a
                // per-sample index load for every next group)
                if (H3F_PERSIST && h3f_dma(L.bs) && !n.src.idx && !n.src.fbase) fa.ticket = w.h3f_ticket;
                conv_h3f_launch(L.bs, L.C, fa, S, s);
            }
        }
        lo = std::max(lo, 3);
    }
    if (lo <= 0 && hi >= 0) {
        // samples per workgroup: S*ng/1024 capped at 8 (4 at the 4096-env act forward: measured
        // 20 us against 25 at 8; 1 sample per workgroup costs the per-workgroup weight/board latency)
        constexpr int c1div = 1024;
        const int ns = (int)std::max<int64_t>(1, std::min<int64_t>(8, S * ng / c1div));
        const dim3 grid((unsigned)(ceil_div(S, ns) + (rider ? 1 : 0)), (unsigned)ng);
        const size_t lds = (size_t)(9 * L.C * 16 + 16 + ((ns * L.C * (bs + 2) * (bs + 2) + 3) & ~3) + 256 * 24) * sizeof(float);
        Conv1Pair cp{};
        if (rider) cp.rider = *rider;
        for (int g = 0; g < 2; ++g) {
            const FwdNet &n = net[g < ng ? g : 0];
            // x6: a1 also (acting: only) as bf16 planes for conv2
            cp.g[g] = Conv1Args{n.src, n.th + L.off_w1, n.th + L.off_b1,
                                (n.wtb && !n.w->has_train && !h3c2) ? nullptr : n.w->a1,
                                (n.wtb && !h3c2) ? n.w->a1b : nullptr, n.w->has_train ? n.w->x0 : nullptr,
                                h3 ? n.wt + L.off_t3 : nullptr, n3, h3 ? n.w->wmax_part : nullptr};
        }
        if (L.C == 1)
            conv1_fwd_kernel<1><<<grid, 256, lds, s>>>(cp, S, bs, ns);
        else
            conv1_fwd_kernel<2><<<grid, 256, lds, s>>>(cp, S, bs, ns);
        launch_check("conv1_fwd_kernel");
        for (int g = 0; g < ng; ++g) {
            net[g].w->x0_valid = net[g].w->has_train ? 1 : 0;
            net[g].w->wmax_n = h3 ? (int)ceil_div(S, ns) : 0;
            net[g].w->wmax_img = h3 ? net[g].wt + L.off_t3 : nullptr;
        }
    }
    FwdIO io[2];
    if (lo <= 1 && hi >= 1 && h3c2) {   // conv2 on the h3 kernel: fp32 a1 -> fp32 a2
        for (int g = 0; g < ng; ++g) conv_h3c2_launch(L, net[g], S, s);
    } else if (lo <= 1 && hi >= 1) {   // conv2: M = S*bs^2, K = 9 offsets x 16, N = 32
        // x6: a2 also (acting: only) as bf16 planes for conv3; training keeps fp32 a2 for the backward
        for (int g = 0; g < ng; ++g) {
            const FwdNet &n = net[g];
            // h3: conv3 reads fp32 a2 and splits it itself
            io[g] = FwdIO{n.w->a1, n.wt + L.off_t2, n.th + L.off_b2,
                          (n.wtb && !n.w->has_train && !h3) ? nullptr : n.w->a2,
                          n.wtb ? n.wtb + 3 * L.off_t2 : nullptr, n.wtb ? n.w->a1b : nullptr,
                          (n.wtb && !h3) ? n.w->a2b : nullptr, n.w};
        }
        conv_fwd<16, 32, 3, 1>(io, ng, S * nc, bs, bs, s);
    }
    if (lo <= 2 && hi >= 2) {   // conv3: M = S*Wo^2, K = 36 offsets x 32, N = 64
        for (int g = 0; g < ng; ++g) {
            const FwdNet &n = net[g];
            io[g] = FwdIO{n.w->a2, n.wt + L.off_t3, n.th + L.off_b3, n.w->a3, n.wtb ? n.wtb + 3 * L.off_t3 : nullptr,
                          (n.wtb && !h3) ? n.w->a2b : nullptr, nullptr, n.w};
            if (h3) {
                QWork &w = *n.w;
                if (!w.wmax_n || w.wmax_img != n.wt + L.off_t3) {   // conv1 did not scan this image
                    wmax_scan_kernel<<<256, 256, 0, s>>>(n.wt + L.off_t3, n3, w.wmax_part, SampleRider{});
                    launch_check("wmax_scan_kernel");
                    w.wmax_n = 256;
                    w.wmax_img = n.wt + L.off_t3;
                }
                io[g].wmax = w.wmax_part;
                io[g].nwmax = w.wmax_n;
            }
        }
        conv_fwd<32, 64, 6, 0>(io, ng, S * L.Wo * L.Wo, bs, L.Wo, s);
    }
    // the nets' workspaces: which of them now hold a dense_h3-ready a3 (a forward through conv3
    // without dense_h3 leaves a3 without its maxima)
    if (lo0 <= 2 && hi >= 2)
        for (int g = 0; g < ng; ++g) net[g].w->dh3_ready = dh3prep ? 1 : 0;
    if (lo0 == 3 && hi >= 3) {   // Dense1 alone (per-layer timing): dense_h3 if the last forward prepared it
        int kc;
        const int ks = d1_split(L, S, kc);
        bool ready = dh3_ok(L, ks, kc);
        for (int g = 0; g < ng; ++g) ready = ready && net[g].w->dh3_ready;
        dh3 = ready;
    }
    if (lo <= 3 && hi >= 3 && dh3) {   // Dense1 on the h3 split, the same slab layout
        int kc;
        const int ks = d1_split(L, S, kc);
        for (int g = 0; g < ng; ++g) {
            const FwdNet &n = net[g];
            const DenseH3Args da{n.w->a3, n.w->a3max, n.w->w1h, n.w->w1e, n.w->slab, (int)S, L.Wo * L.Wo};
            dh3_launch(da, ks, kc, s);
        }
        return;
    }
    if (lo <= 3 && hi >= 3) {   // Dense1 (split over the Wo^2 positions into partial slabs; bias + relu in the head)
        int kc;
        const int ks = d1_split(L, S, kc);
        ConvArgs ga[2];
        const uint16_t *wb[2];
        for (int g = 0; g < ng; ++g) {
            const FwdNet &n = net[g];
            ConvArgs a{};
            a.x = n.w->a3; a.w = n.wt + L.off_td; a.out = n.w->slab; a.M = (int)S; a.HIN = L.Wo; a.HOUT = 1;
            a.nkk = L.Wo * L.Wo;
            ga[g] = a;
            wb[g] = n.wtb ? n.wtb + 3 * L.off_td : nullptr;
        }
        conv_launch<64, 64, 0, 0, MODE_DENSE, EPI_SLAB>(ga, ng, ks, s, wb);
    }
}

void qnet_forward(const QLayout &L, const float *th, const float *wt, const BoardSrc &src, int64_t S, QWork &w,
                  HeadMode mode, const HeadArgs &ha, hipStream_t s, int only, const uint16_t *wtb,
                  const SampleRider *rider) {
    const FwdNet net{th, wt, wtb, src, &w};
    SNK_CHECK(!rider || (only < 0 && rider->batch <= 64), SNK_ERR_INTERNAL, "sample rider: full forward, batch <= 64");
    if (only < 0)
        forward_layers(L, &net, 1, S, s, 0, 3, rider);
    else if (only == QNET_ONLY_CONV23)
        forward_layers(L, &net, 1, S, s, 1, 2);
    else if (only < 4)
        forward_layers(L, &net, 1, S, s, only, only);
    if (only >= 0 && only != 4) return;
    qnet_head(L, th, S, w, mode, ha, s);
}

int qnet_forward_act_slabs(const QLayout &L, const float *th, const float *wt, const BoardSrc &src, int64_t S,
                           QWork &w, hipStream_t s, const uint16_t *wtb, const SampleRider *rider) {
    const FwdNet net{th, wt, wtb, src, &w};
    SNK_CHECK(!rider || rider->batch <= 64, SNK_ERR_INTERNAL, "sample rider: batch <= 64");
    forward_layers(L, &net, 1, S, s, 0, 3, rider);
    return qnet_act_slab_count(L, S);
}

int qnet_act_slab_count(const QLayout &L, int64_t S) {
    int kc;
    return d1_split(L, S, kc);
}

void qnet_forward_pair(const QLayout &L, const FwdNet *net, int64_t S, hipStream_t s) {
    forward_layers(L, net, 2, S, s, 0, 3);
}

template <int HIN, int C>
static void upd_fwd_launch_t(const UpdFwdArgs &a, hipStream_t s) {
    constexpr size_t lds = (size_t)updf_lds_bytes(HIN, C);
    static_assert(lds <= 160 * 1024, "upd_fwd LDS");
    set_lds_limit((const void *)upd_fwd_kernel<HIN, C>, lds);
    upd_fwd_kernel<HIN, C><<<dim3((unsigned)(2 * a.S), 2), UPDF_NT, lds, s>>>(a);
    launch_check("upd_fwd_kernel");
}

// board sides with an instantiated fused update forward (the others take the layer path)
static bool upd_fwd_launch(const UpdFwdArgs &a, hipStream_t s) {
#define SNK_UPDF(B)                                                             \
    case B:                                                                     \
        if (a.L.C == 1) upd_fwd_launch_t<B, 1>(a, s); else upd_fwd_launch_t<B, 2>(a, s); \
        return true;
    switch (a.L.bs) {
        SNK_UPDF(8) SNK_UPDF(10) SNK_UPDF(12) SNK_UPDF(13) SNK_UPDF(16)
        default: return false;
    }
#undef SNK_UPDF
}

// Dense1 of the update's two nets (S <= 64 samples each) into the head's K-split slabs, on
// the fp64 matrix cores: block (output half, slab z, net) stages its slab's a3 columns
// (S x F, F = the slab's features <= 256) and W1 rows (F x 32) by float4 loads into LDS, one
// 16x16 output tile per wave over k = F (v_mfma_f64_16x16x4_f64: fp32 operands, fp64 sums,
// rounded once per slab). The x6 conv kernel (MODE_DENSE) ran these 26 slab blocks of 128
// rows (64 of them real) at 10.3 us.
constexpr int D1U_FMAX = 256, D1U_AP = D1U_FMAX + 2, D1U_WP = 48;   // LDS pitches (floats): conflict-free reads
struct D1UpdNet {
    const float *a3, *w1;   // a3 [S][K1], W1 [K1][64] (packed: theta + off_d1w)
    float *slab;            // [ks][S][64]
};
__global__ __launch_bounds__(512) void dense1_upd_kernel(D1UpdNet n0, D1UpdNet n1, int S, int K1, int F) {
    extern __shared__ __attribute__((aligned(16))) float d1sm[];
    float *As = d1sm, *Ws = d1sm + 64 * D1U_AP;
    const D1UpdNet n = blockIdx.z ? n1 : n0;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int half = blockIdx.x, z = blockIdx.y;
    const int f0 = z * F, fn = min(F, K1 - f0);   // features of this slab (a multiple of 64)
    {
        constexpr int PA = 64 * D1U_FMAX / 4 / 512, PW = D1U_FMAX * 32 / 4 / 512;   // float4 per thread
        f32x4 va[PA], vw[PW];
#pragma unroll
        for (int u = 0; u < PA; ++u) {   // a3 row s, quad c of the slab
            const int e = tid + 512 * u, sr = e / (D1U_FMAX / 4), c = e - sr * (D1U_FMAX / 4);
            va[u] = (sr < S && 4 * c < fn) ? *reinterpret_cast<const f32x4 *>(n.a3 + (int64_t)sr * K1 + f0 + 4 * c)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PW; ++u) {   // W1 row f, quad c of this output half
            const int e = tid + 512 * u, f = e >> 3, c = e & 7;
            vw[u] = f < fn ? *reinterpret_cast<const f32x4 *>(n.w1 + (int64_t)(f0 + f) * 64 + 32 * half + 4 * c)
                           : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < PA; ++u) {
            const int e = tid + 512 * u, sr = e / (D1U_FMAX / 4), c = e - sr * (D1U_FMAX / 4);
#pragma unroll
            for (int q = 0; q < 4; ++q) As[sr * D1U_AP + 4 * c + q] = va[u][q];
        }
#pragma unroll
        for (int u = 0; u < PW; ++u) {
            const int e = tid + 512 * u, f = e >> 3, c = e & 7;
            *reinterpret_cast<f32x4 *>(Ws + f * D1U_WP + 4 * c) = vw[u];
        }
    }
    __syncthreads();
    // wave: sample tile mt = wave >> 1, output tile nt = wave & 1 (of this half)
    const int r = lane & 15, kq = lane >> 4, mt = wave >> 1, nt = wave & 1;
    typedef double f64x4u __attribute__((ext_vector_type(4)));
    f64x4u acc = {0.0, 0.0, 0.0, 0.0};
    const float *pa = As + (16 * mt + r) * D1U_AP + kq, *pw = Ws + kq * D1U_WP + 16 * nt + r;
    for (int k = 0; k < fn; k += 4)
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64((double)pa[k], (double)pw[k * D1U_WP], acc, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int sr = 16 * mt + kq + 4 * i;
        if (sr < S) n.slab[((int64_t)z * S + sr) * 64 + 32 * half + 16 * nt + r] = (float)acc[i];
    }
}

// returns the number of Dense1 partial slabs the head sums: 2 when the update forward ran
// Dense1 itself (phase 4 of upd_fwd_kernel, S <= 64), else d1_split's; 0 when it also ran
// both heads (phase 5, `head` given: HEAD_LOSS arguments and the two nets' thetas)
int qnet_forward_update_pair(const QLayout &L, const FwdNet *net, int64_t S, hipStream_t s, const HeadArgs *head) {
    int kc;
    const int ks = d1_split(L, S, kc);
    // the x6 weight planes of both nets are kept current by every theta change
    if (net[0].wtb && net[1].wtb && (L.C == 1 || L.C == 2) && S >= 1 && S <= 4096) {
        UpdFwdArgs a{};
        a.L = L;
        a.S = (int)S;
        a.d1 = S <= 64 && net[0].w->slab_floats >= 2 * S * 64 && net[1].w->slab_floats >= 2 * S * 64;
        for (int g = 0; g < 2; ++g) {
            QWork &w = *net[g].w;
            const bool train = w.has_train != 0;
            a.net[g] = UpdFwdNet{net[g].src, net[g].th, net[g].wtb, train ? w.a1 : nullptr, train ? w.a2 : nullptr,
                                 w.a3, train ? w.x0 : nullptr, w.slab};
            a.hn[g] = HeadNet{w.slab, net[g].th, w.h1, w.q};
        }
        a.head = a.d1 && head && net[1].w->upd_ticket && net[1].w->cap >= S && arith(SNK_ARITH_UPD_HEAD);
        if (a.head) {
            a.ha = *head;
            a.ticket = net[1].w->upd_ticket;
        }
        if (upd_fwd_launch(a, s)) {
            for (int g = 0; g < 2; ++g) {
                net[g].w->x0_valid = net[g].w->has_train ? 1 : 0;
                net[g].w->wmax_n = 0;   // no conv3 weight-max partials from this path
            }
            if (a.d1) return a.head ? 0 : 2;   // Dense1 (and the heads) done in the same launch
            if (S <= 64 && kc * 64 <= D1U_FMAX) {   // Dense1 slabs on dense1_upd_kernel
                const D1UpdNet d0{net[0].w->a3, net[0].th + L.off_d1w, net[0].w->slab};
                const D1UpdNet d1{net[1].w->a3, net[1].th + L.off_d1w, net[1].w->slab};
                const size_t lds = (size_t)(64 * D1U_AP + D1U_FMAX * D1U_WP) * 4;
                set_lds_limit((const void *)dense1_upd_kernel, lds);
                dense1_upd_kernel<<<dim3(2, (unsigned)ks, 2), 512, lds, s>>>(d0, d1, (int)S, L.K1, kc * 64);
                launch_check("dense1_upd_kernel");
            } else {
                forward_layers(L, net, 2, S, s, 3, 3);   // Dense1 slabs
            }
            return ks;
        }
    }
    forward_layers(L, net, 2, S, s, 0, 3);
    return ks;
}

void qnet_head_pair(const QLayout &L, const float *th_t, QWork &wt_, const float *th_q, QWork &wq, int64_t S,
                    const HeadArgs &ha, hipStream_t s, int ks) {
    head_pair_kernel<<<ceil_div(S, 4), 256, 0, s>>>(HeadNet{wt_.slab, th_t, wt_.h1, wt_.q},
                                                    HeadNet{wq.slab, th_q, wq.h1, wq.q}, ks, S, L, ha);
    launch_check("head_pair_kernel");
}

void head_launch(const QLayout &L, const float *th, const float *slab, int ks, int64_t S, float *h1, float *qo,
                 HeadMode mode, const HeadArgs &ha, hipStream_t s) {
    const int grid = ceil_div(S, 4) + (mode == HEAD_ACT && ha.rider.out ? 1 : 0);
    switch (mode) {
        case HEAD_Q: head_kernel<HEAD_Q><<<grid, 256, 0, s>>>(slab, ks, S, th, L, h1, qo, ha); break;
        case HEAD_ACT: head_kernel<HEAD_ACT><<<grid, 256, 0, s>>>(slab, ks, S, th, L, h1, qo, ha); break;
        case HEAD_TARGET: head_kernel<HEAD_TARGET><<<grid, 256, 0, s>>>(slab, ks, S, th, L, h1, qo, ha); break;
        case HEAD_LOSS: head_kernel<HEAD_LOSS><<<grid, 256, 0, s>>>(slab, ks, S, th, L, h1, qo, ha); break;
    }
    launch_check("head_kernel");
}

void head_pair_launch(const QLayout &L, const float *th_t, const float *slab_t, float *h1_t, float *q_t,
                      const float *th_q, const float *slab_q, float *h1_q, float *q_q, int ks, int64_t S,
                      const HeadArgs &ha, hipStream_t s) {
    head_pair_kernel<<<ceil_div(S, 4), 256, 0, s>>>(HeadNet{slab_t, th_t, h1_t, q_t}, HeadNet{slab_q, th_q, h1_q, q_q},
                                                    ks, S, L, ha);
    launch_check("head_pair_kernel");
}

void d2_grad_launch(const float *dq, const float *h1, int64_t S, const QLayout &L, float *grad, hipStream_t s) {
    d2_grad_kernel<<<1, 256, 0, s>>>(dq, h1, S, L, grad);
    launch_check("d2_grad_kernel");
}

void slab_reduce_launch(const float *slab, int ks, int64_t MN, float *out, hipStream_t s) {
    slab_reduce_kernel<<<(unsigned)std::min<int64_t>(ceil_div(MN, 256), 2048), 256, 0, s>>>(slab, ks, MN, out);
    launch_check("slab_reduce_kernel");
}

void qnet_head(const QLayout &L, const float *th, int64_t S, QWork &w, HeadMode mode, const HeadArgs &ha,
               hipStream_t s) {
    int kc;
    const int ks = d1_split(L, S, kc);
    const int grid = ceil_div(S, 4) + (mode == HEAD_ACT && ha.rider.out ? 1 : 0);
    switch (mode) {
        case HEAD_Q: head_kernel<HEAD_Q><<<grid, 256, 0, s>>>(w.slab, ks, S, th, L, w.h1, w.q, ha); break;
        case HEAD_ACT: head_kernel<HEAD_ACT><<<grid, 256, 0, s>>>(w.slab, ks, S, th, L, w.h1, w.q, ha); break;
        case HEAD_TARGET: head_kernel<HEAD_TARGET><<<grid, 256, 0, s>>>(w.slab, ks, S, th, L, w.h1, w.q, ha); break;
        case HEAD_LOSS: head_kernel<HEAD_LOSS><<<grid, 256, 0, s>>>(w.slab, ks, S, th, L, w.h1, w.q, ha); break;
    }
    launch_check("head_kernel");
}

// ---------------------------------------------------------------- backward
// weight-gradient GEMMs: M = weight rows (+1 bias row of ones), N = out channels,
// K = rows (sample, position) of the layer output
struct BwdPlan {
    GemmPlan d1, c3, c2, c1, d1x, c2x;
};
// waves per tile fixed so that the layer pairs (d1 wgrad | d1x: 2, c3 wgrad |
// conv3 data grad: 4 = the conv kernel's 256 threads, c2 wgrad | c2x: 8) launch together
// conv3's backward on conv3_bwd_kernel (snk_bwd3.hpp): both halves' LDS within a CU's
// 160 KB (boards up to 13x13 at two samples per weight-gradient chunk). Larger boards:
// the generic pair (gemm_body weight gradient | implicit-GEMM data gradient + reduce).
constexpr int C3_NSC = 2;
static bool c3bwd_ok(const QLayout &L, int64_t S) {
    const size_t lim = 160 * 1024 / sizeof(float);
    return S <= (1 << 24) && L.Wo >= 3 && L.Wo <= 8 && (size_t)c3_dw_lds_floats(L.bs, L.Wo, C3_NSC) <= lim &&
           (size_t)c3_dx_lds_floats(L.Wo) <= lim;
}

// conv2's backward on conv2_bwd_kernel (snk_bwd3.hpp); larger boards: the generic pair
static bool c2bwd_ok(const QLayout &L, int64_t S) {   // the dX image pitch C2X_PJ holds bs + 2 <= 20
    return S <= (1 << 20) && L.bs + 2 <= C2X_PJ && (size_t)c2_bwd_lds_floats(L.bs) * sizeof(float) <= 160 * 1024;
}

static BwdPlan bwd_plan(const QLayout &L, int64_t S) {
    BwdPlan p;
    p.d1 = plan_gemm_kw(L.K1 + 1, 64, 2, S, true, 2);
    p.c3 = plan_gemm_kw(1153, 64, 2, S * L.Wo * L.Wo, true, 4);
    if (c3bwd_ok(L, S)) {   // slab z = the partial of samples [z*NSC, z*NSC + NSC)
        const int64_t z = ceil_div(S, C3_NSC);
        p.c3 = GemmPlan{4, (int)z, (int)(C3_NSC * L.Wo * L.Wo)};
    }
    p.c2 = plan_gemm_kw(145, 32, 1, S * L.ncell, true, 8);
    if (c2bwd_ok(L, S)) p.c2 = GemmPlan{8, (int)S, (int)L.ncell};   // slab z = sample z
    p.c1 = plan_gemm(9 * L.C + 1, 16, 1, S * L.ncell, true);
    p.d1x = plan_gemm_kw(S, L.K1, 2, 64, false, 2);
    p.c2x = plan_gemm_kw(S * L.ncell, 16, 1, 288, false, 8);
    return p;
}
static int64_t zslab(const GemmPlan &g, int64_t MN) { return g.z > 1 ? (int64_t)g.z * MN : 0; }
// the four weight-gradient GEMMs may run concurrently: each owns a slab region
struct SlabRegions {
    int64_t d1, c3, c2, c1, total;
};
static SlabRegions slab_regions(const QLayout &L, int64_t S) {
    const BwdPlan p = bwd_plan(L, S);
    SlabRegions r;
    r.d1 = 0;
    r.c3 = r.d1 + zslab(p.d1, (int64_t)(L.K1 + 1) * 64);
    r.c2 = r.c3 + zslab(p.c3, 1153 * 64);
    r.c1 = r.c2 + zslab(p.c2, 145 * 32);
    // conv1's weight gradient: K-split slabs of the gemm, or one slab per data-gradient block of
    // conv2_bwd_kernel (fused there)
    const int64_t c1n = (int64_t)(9 * L.C + 1) * 16;
    const int64_t c1 = c2bwd_ok(L, S) ? S * C2_NXB * c1n : zslab(p.c1, c1n);
    r.total = std::max<int64_t>(r.c1 + c1, 1);
    return r;
}
int64_t qnet_backward_slab_floats(const QLayout &L, int64_t S) { return slab_regions(L, S).total; }


// data-gradient chain shared by the loss backward and the per-sample Jacobian:
// dz1 (from dq) -> dz3 -> dz2 -> dzc1, each relu-masked by its activation
static void backward_data_chain(const QLayout &L, const float *th, int64_t S, QWork &w, const BwdPlan &p,
                                hipStream_t s) {
    const int bs = L.bs, nc = L.ncell;
    head_bwd_kernel<<<ceil_div(S, 4), 256, 0, s>>>(w.dq, w.h1, th, L, S, w.dz1);
    launch_check("head_bwd_kernel");
    gemm<2>(ARowMajor{w.dz1, 64, 64}, BTrans{th + L.off_d1w, 64, L.K1, 64}, EpReluMask{w.dz3, w.a3, (int)S, L.K1},
            S, L.K1, 64, p.d1x, s);
    {
        ConvArgs a{};
        a.x = w.dz3; a.w = th + L.off_w3; a.act = w.a2; a.M = (int)(S * nc); a.HIN = L.Wo; a.HOUT = bs; a.nkk = 36;
        const int sp = dx_splits(S * nc);
        if (sp == 1) {
            a.out = w.dz2;
            conv_launch<64, 32, 6, 0, MODE_DX, EPI_RELU_MASK>(a, 1, s);
        } else {
            a.out = w.cslab;
            SNK_CHECK((int64_t)sp * S * nc * 32 <= w.cslab_floats, SNK_ERR_INTERNAL, "conv slab too small");
            conv_launch<64, 32, 6, 0, MODE_DX, EPI_SLAB>(a, sp, s);
            const int used = ceil_div(36, ceil_div(36, sp));
            const ReduceArgs ra{w.cslab, nullptr, w.a2, w.dz2, nullptr};
            conv_reduce_launch(&ra, 1, used, S * nc * 32, 32, s);
        }
    }
    gemm<1>(AConvDx<32, 3, 1>{w.dz2, bs, bs, FastDiv(nc), FastDiv(bs)}, BConvT<16, 32>{th + L.off_w2, 288},
            EpReluMask{w.dzc1, w.a1, (int)(S * nc), 16}, S * nc, 16, 288, p.c2x, s);
}

void qnet_backward(const QLayout &L, const float *th, const BoardSrc &src, int64_t S, QWork &w, float *grad,
                   float *slab, int64_t slab_cap, hipStream_t s, const BwdOpts &o) {
    const BwdPlan p = bwd_plan(L, S);
    const SlabRegions sr = slab_regions(L, S);
    SNK_CHECK(slab_cap >= sr.total, SNK_ERR_INTERNAL, "backward slab too small");
    const int bs = L.bs, nc = L.ncell, no = L.Wo * L.Wo;
    // the slabs and Dense2 are always finished by grad_update_kernel's summation (the caller's
    // deferred pass, or one finish-only pass here): a gradient is bit-identical whichever path
    // produced it
    GradSlabs local;
    const bool deferred = o.defer != nullptr;
    GradSlabs *D = deferred ? o.defer : &local;
    *D = GradSlabs{};
    D->dq = w.dq;
    D->h1 = w.h1;
    D->S = S;
    {
        // each layer's weight gradient and data gradient in ONE launch
        auto dst = [&](int k, const GemmPlan &g, int64_t off, int64_t n, float *sl) -> float * {
            if (g.z == 1) return grad + off;
            if (D) {
                D->slab[k] = sl; D->z[k] = g.z; D->off[k] = off; D->n[k] = n;
            }
            return sl;
        };
        auto fin = [&](const GemmPlan &, int64_t, int64_t, float *) {};   // grad_update_kernel finishes
        if (!o.dz1_ready) {
            head_bwd_kernel<<<ceil_div(S, 4), 256, 0, s>>>(w.dq, w.h1, th, L, S, w.dz1);
            launch_check("head_bwd_kernel");
        }

        // Dense1: dW (+ bias row) | dX with the relu mask of a3
        const int64_t M1 = L.K1 + 1;
        float *d1d = dst(0, p.d1, L.off_d1w, M1 * 64, slab + sr.d1);
        if (S <= 64 && p.d1.z == 1 && L.K1 % D1B_F == 0) {   // d1_bwd_kernel (fp64 MFMA, one launch)
            const int nfb = L.K1 / D1B_F;
            d1_bwd_kernel<<<2 * nfb + 1, 512, 0, s>>>(w.a3, w.dz1, th + L.off_d1w, w.dz3, d1d, (int)S, L.K1, nfb);
            launch_check("d1_bwd_kernel");
        } else
        pair_launch<128>(gemm_job<2, 2>(ADenseDw<>{w.a3, L.K1, S}, BRows{w.dz1, S, 64}, EpSlab{d1d, (int)M1, 64}, M1,
                                        64, S, p.d1),
                         gemm_job<2, 2>(ARowMajor{w.dz1, 64, 64}, BTrans{th + L.off_d1w, 64, L.K1, 64},
                                        EpReluMask{w.dz3, w.a3, (int)S, L.K1}, S, L.K1, 64, p.d1x),
                         s);
        fin(p.d1, L.off_d1w, M1 * 64, slab + sr.d1);
        // conv3: dW over rows (s, pout) | dX onto the bs x bs x 32 input (relu mask on a2)
        if (c3bwd_ok(L, S)) {
            float *c3d = dst(1, p.c3, L.off_w3, 1153 * 64, slab + sr.c3);
            const Conv3BwdArgs ca{w.a2, w.dz3, th + L.off_w3, c3d, w.dz2, (int)S, bs, L.Wo, C3_NSC, p.c3.z, p.c3.z * C3_DWG};
            const size_t lds = (size_t)std::max(c3_dw_lds_floats(bs, L.Wo, C3_NSC), c3_dx_lds_floats(L.Wo)) * 4;
            const unsigned nb = (unsigned)(ca.nW + S * (32 / C3_CG));
            auto go = [&](auto kern) {
                set_lds_limit((const void *)kern, lds);
                kern<<<nb, 256, lds, s>>>(ca);
            };
            switch (L.Wo) {
                case 3: go(conv3_bwd_kernel<3>); break;
                case 4: go(conv3_bwd_kernel<4>); break;
                case 5: go(conv3_bwd_kernel<5>); break;
                case 6: go(conv3_bwd_kernel<6>); break;
                case 7: go(conv3_bwd_kernel<7>); break;
                default: go(conv3_bwd_kernel<8>); break;
            }
            launch_check("conv3_bwd_kernel");
            fin(p.c3, L.off_w3, 1153 * 64, slab + sr.c3);
        } else {
            float *c3d = dst(1, p.c3, L.off_w3, 1153 * 64, slab + sr.c3);
            const auto wj = gemm_job<2, 4>(AConvDw<32, 6, 0>{w.a2, bs, L.Wo, S * no, FastDiv(no), FastDiv(L.Wo)},
                                           BRows{w.dz3, S * no, 64}, EpSlab{c3d, 1153, 64}, 1153, 64, S * no, p.c3);
            ConvArgs a{};
            a.x = w.dz3; a.w = th + L.off_w3; a.act = w.a2; a.M = (int)(S * nc); a.HIN = L.Wo; a.HOUT = bs;
            a.nkk = 36;
            int sp = dx_splits(S * nc);
            const dim3 cg((unsigned)ceil_div(S * nc, 128), 1, 1);
            if (sp == 1) {
                a.out = w.dz2;
                ConvX6Job<64, 32, 6, 0, MODE_DX, EPI_RELU_MASK, false, true> cj{make_conv_pair(&a, 1, sp, nullptr), cg};
                pair_launch<256>(wj, cj, s);
            } else {
                a.out = w.cslab;
                SNK_CHECK((int64_t)sp * S * nc * 32 <= w.cslab_floats, SNK_ERR_INTERNAL, "conv slab too small");
                ConvX6Job<64, 32, 6, 0, MODE_DX, EPI_SLAB, false, true> cj{make_conv_pair(&a, 1, sp, nullptr), cg};
                cj.grid.y = (unsigned)sp;
                pair_launch<256>(wj, cj, s);
                const ReduceArgs ra{w.cslab, nullptr, w.a2, w.dz2, nullptr};
                conv_reduce_launch(&ra, 1, sp, S * nc * 32, 32, s);
            }
            fin(p.c3, L.off_w3, 1153 * 64, slab + sr.c3);
        }
        // conv1's input planes: the forward's float copy when it made one
        BoardSrc xs = src;
        if (w.x0_valid) {
            xs = BoardSrc{};
            xs.fbase = w.x0;
            xs.C = L.C;
            xs.ncell = nc;
        }
        const int64_t Mc1 = 9 * L.C + 1;
        // conv2: dW | dX (relu mask on a1), and with it conv1's weight gradient
        float *c2d = dst(2, p.c2, L.off_w2, 145 * 32, slab + sr.c2);
        const bool c2f = c2bwd_ok(L, S);
        if (c2f) {
            const GemmPlan c1p{1, (int)(S * C2_NXB), 0};   // one slab per data-gradient block
            float *c1d = dst(3, c1p, L.off_w1, Mc1 * 16, slab + sr.c1);
            Conv2BwdArgs ca{w.a1, w.dz2, th + L.off_w2, c2d, w.dzc1, (int)S, bs, xs, c1d, L.C};
            const size_t lds = (size_t)c2_bwd_lds_floats(bs) * sizeof(float);
            set_lds_limit((const void *)conv2_bwd_kernel, lds);
            conv2_bwd_kernel<<<(unsigned)((1 + C2_NXB) * S), 256, lds, s>>>(ca);
            launch_check("conv2_bwd_kernel");
            fin(p.c2, L.off_w2, 145 * 32, slab + sr.c2);
            fin(c1p, L.off_w1, Mc1 * 16, slab + sr.c1);
        } else
        pair_launch<512>(gemm_job<1, 8>(AConvDw<16, 3, 1>{w.a1, bs, bs, S * nc, FastDiv(nc), FastDiv(bs)},
                                        BRows{w.dz2, S * nc, 32}, EpSlab{c2d, 145, 32}, 145, 32, S * nc, p.c2),
                         gemm_job<1, 8>(AConvDx<32, 3, 1>{w.dz2, bs, bs, FastDiv(nc), FastDiv(bs)},
                                        BConvT<16, 32>{th + L.off_w2, 288}, EpReluMask{w.dzc1, w.a1, (int)(S * nc), 16},
                                        S * nc, 16, 288, p.c2x),
                         s);
        if (!c2f) {
            fin(p.c2, L.off_w2, 145 * 32, slab + sr.c2);
            // conv1: weights only
            float *c1d = dst(3, p.c1, L.off_w1, Mc1 * 16, slab + sr.c1);
            gemm<1>(ABoardDw{xs, bs, L.C, S * nc, FastDiv(nc), FastDiv(bs)}, BRows{w.dzc1, S * nc, 16},
                    EpSlab{c1d, (int)Mc1, 16}, Mc1, 16, S * nc, p.c1, s);
            fin(p.c1, L.off_w1, Mc1 * 16, slab + sr.c1);
        }
    }
    if (!deferred) grad_update_launch(L, D, grad, nullptr, s);   // finish only
}

// ---------------------------------------------------------------- fused update
struct UpdArgs {
    QLayout L;
    GradSlabs g;
    float *grad;
    UpdateTarget u;
    PostUpdate post;
    int finish, apply, has_post;
};


// the finished gradient of the four packed parameters i0 .. i0+3 (i0 % 4 == 0, all in one
// section): the sum of their K-split slabs (z ascending, float4 slab loads, sixteen in
// flight per batch) or the value already there
// (part / nparts: only slabs [zc * part / nparts, zc * (part + 1) / nparts), for blocks that
// split a parameter's slab run over several threads). Where no K-split covers the
// parameters (z <= 1: the gradient was written straight into grad, e.g. conv2's one-slab
// plan at B = 1), part 0 returns grad and the other parts zero, so the parts still sum to
// the gradient.
__device__ __forceinline__ f32x4 finish4(const UpdArgs &a, int64_t i0, int part = 0, int nparts = 1) {
    f32x4 g = {0.0f, 0.0f, 0.0f, 0.0f};
    if (part == 0) g = *reinterpret_cast<const f32x4 *>(a.grad + i0);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t j = i0 - a.g.off[k];
        if (a.g.z[k] > 1 && j >= 0 && j < a.g.n[k]) {
            const float *sl = a.g.slab[k] + j;
            const int64_t n = a.g.n[k];
            const int zc = a.g.z[k] * (part + 1) / nparts;
            f32x4 v = {0.0f, 0.0f, 0.0f, 0.0f};
            int z = a.g.z[k] * part / nparts;
            for (; z + 16 <= zc; z += 16) {
                f32x4 x[16];
#pragma unroll
                for (int u = 0; u < 16; ++u) x[u] = *reinterpret_cast<const f32x4 *>(sl + (int64_t)(z + u) * n);
#pragma unroll
                for (int u = 0; u < 16; ++u) v += x[u];
            }
            if (z < zc) {
                f32x4 x[16];
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (z + u < zc) x[u] = *reinterpret_cast<const f32x4 *>(sl + (int64_t)(z + u) * n);
#pragma unroll
                for (int u = 0; u < 16; ++u)
                    if (z + u < zc) v += x[u];
            }
            g = v;
        }
    }
    return g;
}

// RMSProp of one parameter (rmsprop_kernel order); returns the new theta
__device__ __forceinline__ float rms_one(const UpdArgs &a, int64_t i, float g, bool due, float omr, float acc0,
                                        float th0) {   // acc0 / th0: acc[i] and theta[i], loaded by the caller
    const float qd = a.u.rho * acc0 + omr * (g * g);
    a.u.acc[i] = qd;
    const float th = th0 - (g * a.u.lr) / (__builtin_sqrtf(qd) + a.u.eps);
    a.u.theta[i] = th;
    if (due) a.u.theta_t[i] = th;
    return th;
}

// The weight-image sections (conv2, conv3, Dense1) in blocks of GU_ROWS input
// channels c of one kernel offset kk: the block's parameters (kk*CK + c)*CN + n are one
// contiguous run (coalesced gradient / slab / theta / acc traffic); the new theta goes
// through LDS and leaves in image order [kk][n][c] (float4 of four c, and the three bf16
// planes as 8-byte pieces), so no image write is a stride-CK scatter.
constexpr int GU_ROWS = 16;
struct GuSec {
    int64_t off, base;   // packed offset of the section's weights, image offset
    int CK, CN, nkk;
};
__device__ __forceinline__ GuSec gu_sec(const QLayout &L, int s) {
    if (s == 0) return GuSec{L.off_w2, L.off_t2, 16, 32, 9};
    if (s == 1) return GuSec{L.off_w3, L.off_t3, 32, 64, 36};
    return GuSec{L.off_d1w, L.off_td, 64, 64, L.Wo * L.Wo};
}
__host__ __device__ inline int gu_blocks(int CK, int nkk) { return nkk * (CK / GU_ROWS); }
static_assert(GU_WMAX_BLOCKS == 36 * (32 / GU_ROWS), "conv3 image blocks");

// wmax: where this block's max |new theta| goes (the conv3 section, UpdateTarget::wmax_out)
// sec: 0 conv2, 1 conv3, 2 Dense1 (the split images of UpdateTarget::s_*)
__device__ void gu_image_block(const UpdArgs &a, const GuSec &S, int sec, int kk, int cb, bool due, float omr,
                               float *wmax = nullptr) {
    // rows of CN + 4 floats: the image pass below reads column n of rows c4 .. c4 + 3 with
    // lane groups spanning four c4 values, which a CN-float pitch put on one bank (4-way)
    __shared__ __attribute__((aligned(16))) float th_s[GU_ROWS * (64 + 4)];   // lds: one per kernel (grad_update_kernel only)
    __shared__ float red4[4];   // lds: one per kernel (grad_update_kernel only)
    const int CN = S.CN, n_el = GU_ROWS * CN, lcn = CN == 64 ? 6 : 5;   // CN: 32 or 64
    const int64_t p0 = S.off + ((int64_t)kk * S.CK + cb * GU_ROWS) * CN;   // a multiple of 4
    float m = 0.0f;
    // sections of 128 float4 per block (conv2: 16 x 32) with the finish to do: two threads per
    // float4, each over half of the slab run (conv2's 64 per-sample slabs: two batches of 16
    // loads per thread instead of four), the halves added in order through LDS
    const bool split = a.finish && n_el == 512;
    f32x4 g2 = {0.0f, 0.0f, 0.0f, 0.0f};
    if (split) {
        __shared__ f32x4 part[128];   // lds: one per kernel (grad_update_kernel only)
        const int grp = threadIdx.x & 127, hf = threadIdx.x >> 7;
        const f32x4 pv = finish4(a, p0 + 4 * grp, hf, 2);
        if (hf) part[grp] = pv;
        __syncthreads();
        if (!hf) {
            g2 = pv + part[grp];
            *reinterpret_cast<f32x4 *>(a.grad + p0 + 4 * grp) = g2;
        }
    }
    for (int e = 4 * threadIdx.x; e < n_el; e += 4 * 256) {
        const int64_t i = p0 + e;
        // the optimizer state first: issued with (or before) the slab loads instead of after
        // the gradient store, which the compiler must assume aliases them
        f32x4 ac = {0.f, 0.f, 0.f, 0.f}, th = {0.f, 0.f, 0.f, 0.f};
        if (a.apply) {
            ac = *reinterpret_cast<const f32x4 *>(a.u.acc + i);
            th = *reinterpret_cast<const f32x4 *>(a.u.theta + i);
        }
        f32x4 g;
        if (split) {
            g = g2;
        } else if (a.finish) {
            g = finish4(a, i);
            *reinterpret_cast<f32x4 *>(a.grad + i) = g;
        } else {
            g = *reinterpret_cast<const f32x4 *>(a.grad + i);
        }
        if (!a.apply) continue;
        f32x4 qd, tn;
#pragma unroll
        for (int c = 0; c < 4; ++c) {   // rms_one's arithmetic, component by component
            qd[c] = a.u.rho * ac[c] + omr * (g[c] * g[c]);
            tn[c] = th[c] - (g[c] * a.u.lr) / (__builtin_sqrtf(qd[c]) + a.u.eps);
        }
        *reinterpret_cast<f32x4 *>(a.u.acc + i) = qd;
        *reinterpret_cast<f32x4 *>(a.u.theta + i) = tn;
        if (due) *reinterpret_cast<f32x4 *>(a.u.theta_t + i) = tn;
        *reinterpret_cast<f32x4 *>(&th_s[(e >> lcn) * (CN + 4) + (e & (CN - 1))]) = tn;
        m = fmaxf(m, fmaxf(fmaxf(fabsf(tn[0]), fabsf(tn[1])), fmaxf(fabsf(tn[2]), fabsf(tn[3]))));
    }
    if (!a.apply) return;
    if (wmax) {
        m = wave_max(m);
        if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    }
    __syncthreads();
    if (wmax && threadIdx.x == 0) *wmax = fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
    // image element (kk, n, c) at base + kk*CK*CN + n*CK + c; x6 planes at
    // 3*base + kk*3*CK*CN + p*CK*CN + n*CK + c
    for (int it = threadIdx.x; it < CN * (GU_ROWS / 4); it += 256) {
        const int n = it / (GU_ROWS / 4), c4 = (it % (GU_ROWS / 4)) * 4;
        const float v0 = th_s[(c4 + 0) * (CN + 4) + n], v1 = th_s[(c4 + 1) * (CN + 4) + n];
        const float v2 = th_s[(c4 + 2) * (CN + 4) + n], v3 = th_s[(c4 + 3) * (CN + 4) + n];
        const int64_t t = S.base + (int64_t)kk * S.CK * CN + (int64_t)n * S.CK + cb * GU_ROWS + c4;
        const f32x4 w4 = {v0, v1, v2, v3};
        *reinterpret_cast<f32x4 *>(a.u.wt + t) = w4;
        if (due) *reinterpret_cast<f32x4 *>(a.u.wt_t + t) = w4;
        // the next act forward's split images (w3_split_kernel's layouts and exponents)
        const int ci0 = cb * GU_ROWS + c4;
        if (sec == 1 && a.u.s_w3h) {   // conv3: [kk][512 chunks], chunk (co, ci / 8), 8-byte half (ci / 4) & 1
            const int bch = n * 4 + (ci0 >> 3), bhalf = (ci0 >> 2) & 1;
            u32x2 h, l;
            h3_split4(w4, a.u.s_w3e[0], h, l);
            u32x2 *o = reinterpret_cast<u32x2 *>(a.u.s_w3h) + (int64_t)kk * 512 * 2;
            o[x6s_bswz(bch) * 2 + bhalf] = h;
            o[x6s_bswz(256 + bch) * 2 + bhalf] = l;
        } else if (sec == 0 && a.u.s_w2h) {   // conv2: the B2 image, offset pair kk / 2
            const int p = kk >> 1, k0 = 16 * (kk & 1) + ci0;
            u32x2 h, l;
            h3_split4(w4, a.u.s_w3e[1], h, l);
            u32x2 *o2 = reinterpret_cast<u32x2 *>(a.u.s_w2h);
            o2[(((p * 2 + 0) * 32 + n) * H3F_B2_BR + k0) / 4] = h;
            o2[(((p * 2 + 1) * 32 + n) * H3F_B2_BR + k0) / 4] = l;
        } else if (sec == 2 && a.u.s_w1h) {   // Dense1: row (kk, out n), its own exponent
            const int q4 = ci0 >> 2;
            u32x2 h, l;
            h3_split4(w4, a.u.s_w1e[kk * 64 + n], h, l);
            const int off = (n * 64 + (((q4 >> 1) ^ (n & 7)) << 3) + ((q4 & 1) << 2)) / 4;
            u32x2 *o1 = reinterpret_cast<u32x2 *>(a.u.s_w1h + (int64_t)kk * 2 * 4096);
            o1[off] = h;
            o1[1024 + off] = l;
        }
        if (a.u.wtb) {
            const int64_t x6 = 3 * S.base + (int64_t)kk * 3 * S.CK * CN + (int64_t)n * S.CK + cb * GU_ROWS + c4;
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                const uint32_t lo = (uint32_t)split_part(v0, pl) | ((uint32_t)split_part(v1, pl) << 16);
                const uint32_t hi = (uint32_t)split_part(v2, pl) | ((uint32_t)split_part(v3, pl) << 16);
                const u32x2 pc = {lo, hi};
                *reinterpret_cast<u32x2 *>(a.u.wtb + x6 + (int64_t)pl * S.CK * CN) = pc;
                if (due && a.u.wtb_t) *reinterpret_cast<u32x2 *>(a.u.wtb_t + x6 + (int64_t)pl * S.CK * CN) = pc;
            }
        }
    }
}

// blocks: [0, nimg) image sections (gu_image_block); then GU_OTHER blocks striding
// over the parameters without an image (conv1, the conv2 / conv3 / Dense1 bias rows);
// the LAST block owns Dense2 (195 params): it stages dq and h1 through LDS and reduces
// over the batch (d2_grad_kernel's order)
constexpr int GU_OTHER = 16;
// Profiling builds only (make clocks): grad_update_kernel stamps per block (0 start, 1 work
// done; the last block: 2 all arrived, 3 post-update done, 1 rewritten after the next draw),
// read back by snk_gu_debug_clocks
#ifdef SNK_ENV_CLOCKS
__device__ uint64_t *g_gu_clk;
#define GU_CLK(slot)                                                                                  \
    do {                                                                                              \
        if (threadIdx.x == 0 && g_gu_clk) g_gu_clk[(int64_t)blockIdx.x * 4 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define GU_CLK(slot) do { } while (0)
#endif
__global__ __launch_bounds__(256) void grad_update_kernel(UpdArgs a) {
    GU_CLK(0);
    // the post-update words, read now by every block's thread 0 (only the last block to
    // arrive uses them; no block of this pass writes them before that)
    int64_t pre_upd = 0, pre_nb = 0;
    float pre_eps = 0.0f;
    if (a.has_post && threadIdx.x == 0) {
        pre_upd = *a.post.updates;
        pre_nb = *a.post.nb;
        pre_eps = *a.post.epsilon;
    }
    const QLayout &L = a.L;
    const bool due = a.apply && a.u.counter && (*a.u.counter % a.u.rate) == 0;   // utils.jl:469-472
    const float omr = 1.0f - a.u.rho;
    const int nb2 = gu_blocks(16, 9), nb3 = gu_blocks(32, 36), nbd = gu_blocks(64, L.Wo * L.Wo);
    const int nimg = nb2 + nb3 + nbd;
    const int b = (int)blockIdx.x;
    if (b == (int)gridDim.x - 1) {
        const int t = threadIdx.x;
        float g = 0.0f;
        const int64_t i = L.off_d2w + t;
        if (a.finish) {
            __shared__ float sdq[64 * 3], sh[64 * 64];
            const int ac = t < 192 ? t >> 6 : t - 192, o = t & 63;
            for (int64_t s0 = 0; s0 < a.g.S; s0 += 64) {
                const int n = (int)min((int64_t)64, a.g.S - s0);
                __syncthreads();
                for (int e = t; e < n * 64; e += 256) sh[e] = a.g.h1[s0 * 64 + e];
                if (t < n * 3) sdq[t] = a.g.dq[s0 * 3 + t];
                __syncthreads();
                if (t < 192)
                    for (int k = 0; k < n; ++k) g = __builtin_fmaf(sdq[k * 3 + ac], sh[k * 64 + o], g);
                else if (t < 195)
                    for (int k = 0; k < n; ++k) g += sdq[k * 3 + ac];
            }
            if (t < 195) a.grad[i] = g;
        } else if (t < 195) {
            g = a.grad[i];
        }
        if (a.apply && t < 195) rms_one(a, i, g, due, omr, a.u.acc[i], a.u.theta[i]);
        if (a.has_post) post_loss_block(a.post);   // off the tail: the loss mean needs no other block
    } else if (b < nimg) {
        const int sec = b < nb2 ? 0 : b < nb2 + nb3 ? 1 : 2;
        const int bl = b - (sec == 0 ? 0 : sec == 1 ? nb2 : nb2 + nb3);
        const GuSec S = gu_sec(L, sec);
        const int per = S.CK / GU_ROWS;
        gu_image_block(a, S, sec, bl / per, bl % per, due, omr, sec == 1 && a.u.wmax_out ? a.u.wmax_out + bl : nullptr);
    } else {
        // conv1 [off_w1, off_w2), conv2 bias [off_b2, off_w3), conv3 bias [off_b3, off_d1w),
        // Dense1 bias [off_d1b, off_d2w): one index space over the four runs. These finish from
        // long slab runs (conv1: one slab per conv2 data-gradient block, 128 at B = 64; the conv2
        // bias: one per sample), so 8 lanes share a parameter: lane `sub` sums slabs z = sub,
        // sub + 8, ... (16 loads in flight), then a fixed xor tree over the 8 lanes
        const int64_t r0 = L.off_w2 - L.off_w1, r1 = L.off_w3 - L.off_b2, r2 = L.off_d1w - L.off_b3,
                      r3 = L.off_d2w - L.off_d1b;
        const int64_t tot = r0 + r1 + r2 + r3;
        const int sub = threadIdx.x & 7;
        for (int64_t e = (int64_t)(b - nimg) * 32 + (threadIdx.x >> 3); e < tot; e += (int64_t)GU_OTHER * 32) {
            const int64_t i = e < r0 ? L.off_w1 + e
                            : e < r0 + r1 ? L.off_b2 + (e - r0)
                            : e < r0 + r1 + r2 ? L.off_b3 + (e - r0 - r1)
                                               : L.off_d1b + (e - r0 - r1 - r2);
            float g = a.grad[i];
            const float acc0 = a.apply && sub == 0 ? a.u.acc[i] : 0.0f, th0 = a.apply && sub == 0 ? a.u.theta[i] : 0.0f;
            if (a.finish) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int64_t j = i - a.g.off[k];
                    if (a.g.z[k] > 1 && j >= 0 && j < a.g.n[k]) {
                        const float *sl = a.g.slab[k] + j;
                        const int64_t n = a.g.n[k];
                        const int zc = a.g.z[k];
                        float v = 0.0f;
                        for (int z0 = sub; z0 < zc; z0 += 8 * 16) {
                            float x[16];
#pragma unroll
                            for (int u = 0; u < 16; ++u) x[u] = z0 + 8 * u < zc ? sl[(int64_t)(z0 + 8 * u) * n] : 0.0f;
#pragma unroll
                            for (int u = 0; u < 16; ++u) v += x[u];
                        }
                        v += __shfl_xor(v, 1, 64);
                        v += __shfl_xor(v, 2, 64);
                        v += __shfl_xor(v, 4, 64);
                        g = v;
                    }
                }
                if (sub == 0) a.grad[i] = g;
            }
            if (a.apply && sub == 0) rms_one(a, i, g, due, omr, acc0, th0);
        }
    }
    GU_CLK(1);
    // every block read *counter (nb) above; the last to arrive advances it. The bookkeeping
    // reads nothing another block of this launch wrote, so the ticket needs no fence.
    // Arrivals are counted in 8 shards (blockIdx % 8); the last of a shard adds to the top
    // counter (one word would serialise every block's atomic).
    if (!a.has_post) return;
    __shared__ int s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        const int nwg = (int)gridDim.x, k = (int)(blockIdx.x & 7);
        uint32_t *tk = a.post.ticket;
        int last = 0;
        if (__hip_atomic_fetch_add(tk + k * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            (uint32_t)(((nwg - k + 7) >> 3) - 1)) {
            __hip_atomic_store(tk + k * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last = __hip_atomic_fetch_add(tk + 8 * 32, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                   (uint32_t)(min(nwg, 8) - 1);
        }
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    GU_CLK(2);
    post_count_block(a.post, pre_upd, pre_nb, pre_eps);
    if (threadIdx.x == 0) __hip_atomic_store(a.post.ticket + 8 * 32, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    GU_CLK(3);
    if (!a.post.next.out) return;
    __shared__ int64_t s_draw;
    if (threadIdx.x == 0) s_draw = *a.post.updates;   // this thread's own store above
    __syncthreads();
    if (threadIdx.x < 64) {
        SampleRider r = a.post.next;
        r.draw_dev = nullptr;
        r.draw = (uint64_t)s_draw;
        sample_wave(r);
    }
#ifdef SNK_ENV_CLOCKS
    if (threadIdx.x == 0 && g_gu_clk) g_gu_clk[(int64_t)blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime();
#endif
}

void grad_update_launch(const QLayout &L, const GradSlabs *pending, float *grad, const UpdateTarget *apply,
                        hipStream_t s, const PostUpdate *post) {
    UpdArgs a{};
    a.L = L;
    if (post) {
        a.post = *post;
        a.has_post = 1;
    }
    if (pending) a.g = *pending;
    a.grad = grad;
    if (apply) a.u = *apply;
    a.finish = pending != nullptr;
    a.apply = apply != nullptr;
    if (!a.finish && !a.apply) return;
    if (a.apply && !a.u.counter) a.u.rate = 1;
    const int nimg = gu_blocks(16, 9) + gu_blocks(32, 36) + gu_blocks(64, L.Wo * L.Wo);
    grad_update_kernel<<<(unsigned)(nimg + GU_OTHER + 1), 256, 0, s>>>(a);
    launch_check("grad_update_kernel");
}

// ---------------------------------------------------------------- per-sample Jacobian
// dq = one-hot of the stored action (the direction of dQ(s)[a]/dtheta); act_out[s] = that action
__global__ void jac_onehot_kernel(const uint8_t *__restrict__ act, const int64_t *__restrict__ idx, int64_t S,
                                  float *__restrict__ dq, uint8_t *__restrict__ act_out) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= S) return;
    const int a = act[idx ? idx[s] : s] % 3;   // as the loss head (utils.jl:453-455)
    dq[s * 3 + 0] = a == 0 ? 1.0f : 0.0f;
    dq[s * 3 + 1] = a == 1 ? 1.0f : 0.0f;
    dq[s * 3 + 2] = a == 2 ? 1.0f : 0.0f;
    if (act_out) act_out[s] = (uint8_t)a;
}

// Dense1 / Dense2 sections of a Jacobian row: rank-1 outer products
__global__ void jac_dense_kernel(const float *__restrict__ a3, const float *__restrict__ dz1,
                                 const float *__restrict__ h1, const uint8_t *__restrict__ act, int64_t S, QLayout L,
                                 float *__restrict__ J, int64_t ldJ) {
    const int64_t nd = L.P - L.off_d1w;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < S * nd; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t / nd, e = t - s * nd;
        const int64_t pk = L.off_d1w + e;
        float v;
        if (pk < L.off_d1b) {
            const int64_t f = e >> 6;
            v = a3[s * L.K1 + f] * dz1[s * 64 + (e & 63)];
        } else if (pk < L.off_d2w) {
            v = dz1[s * 64 + (pk - L.off_d1b)];
        } else if (pk < L.off_d2b) {
            const int k = (int)(pk - L.off_d2w);
            v = (k >> 6) == act[s] ? h1[s * 64 + (k & 63)] : 0.0f;
        } else {
            v = (int)(pk - L.off_d2b) == act[s] ? 1.0f : 0.0f;
        }
        J[s * ldJ + pk] = v;
    }
}

struct EpJac {  // per-sample weight gradient z -> J[z][off + row*N + col]
    float *J;
    int64_t ld;
    int M, N;
    __device__ void store1(float v, int row, int col, int z) const {
        if (row < M && col < N) J[(int64_t)z * ld + (int64_t)row * N + col] = v;
    }
    __device__ void store(const f32x16 &acc, int m0, int c0, int lane, int z) const {
        const int col = c0 + (lane & 31);
        if (col >= N) return;
        float *o = J + (int64_t)z * ld;
#pragma unroll
        for (int g = 0; g < 16; ++g) {
            const int row = m0 + acc_row(g, lane);
            if (row < M) o[(int64_t)row * N + col] = acc[g];
        }
    }
};

void qnet_jacobian(const QLayout &L, const float *th, const float *wt, const BoardSrc &src, const uint8_t *act,
                   const int64_t *idx, int64_t S, QWork &w, uint8_t *act_out, float *J, int64_t ldJ, bool dense,
                   hipStream_t s, hipEvent_t ev_chain) {
    const int bs = L.bs, nc = L.ncell, no = L.Wo * L.Wo;
    qnet_forward(L, th, wt, src, S, w, HEAD_Q, HeadArgs{}, s);
    jac_onehot_kernel<<<(unsigned)ceil_div(S, 256), 256, 0, s>>>(act, idx, S, w.dq, act_out);
    launch_check("jac_onehot_kernel");
    backward_data_chain(L, th, S, w, bwd_plan(L, S), s);
    if (ev_chain) SNK_HIP(hipEventRecord(ev_chain, s));
    // per-sample conv weight/bias gradients: one GEMM "split" per sample
    // (grid.z = sample, k = that sample's output positions)
    const int64_t CH = 32768;
    for (int64_t s0 = 0; s0 < S; s0 += CH) {
        const int64_t cs = std::min(CH, S - s0);
        float *Jr = J + s0 * ldJ;
        gemm<2>(AConvDw<32, 6, 0>{w.a2 + s0 * nc * 32, bs, L.Wo, cs * no, FastDiv(no), FastDiv(L.Wo)},
                BRows{w.dz3 + s0 * no * 64, cs * no, 64}, EpJac{Jr + L.off_w3, ldJ, 1153, 64}, 1153, 64, cs * no,
                GemmPlan{1, (int)cs, no}, s);
        gemm<1>(AConvDw<16, 3, 1>{w.a1 + s0 * nc * 16, bs, bs, cs * nc, FastDiv(nc), FastDiv(bs)},
                BRows{w.dz2 + s0 * nc * 32, cs * nc, 32}, EpJac{Jr + L.off_w2, ldJ, 145, 32}, 145, 32, cs * nc,
                GemmPlan{1, (int)cs, nc}, s);
        BoardSrc sh = src;
        if (sh.idx) sh.idx += s0;
        if (sh.fbase) sh.fbase += s0 * L.C * nc;
        gemm<1>(ABoardDw{sh, bs, L.C, cs * nc, FastDiv(nc), FastDiv(bs)}, BRows{w.dzc1 + s0 * nc * 16, cs * nc, 16},
                EpJac{Jr + L.off_w1, ldJ, 9 * L.C + 1, 16}, 9 * L.C + 1, 16, cs * nc, GemmPlan{1, (int)cs, nc}, s);
    }
    if (dense) {
        SNK_CHECK(act_out != nullptr, SNK_ERR_INTERNAL, "dense Jacobian needs the action array");
        jac_dense_kernel<<<4096, 256, 0, s>>>(w.a3, w.dz1, w.h1, act_out, S, L, J, ldJ);
        launch_check("jac_dense_kernel");
    }
}

void rmsprop_launch(int64_t P, float *theta, float *acc, const float *grad, float eta, float rho, float eps,
                    hipStream_t s) {
    rmsprop_kernel<<<(unsigned)std::min<int64_t>(ceil_div(P, 256), 2048), 256, 0, s>>>(P, theta, acc, grad, eta,
                                                                                        rho, eps);
    launch_check("rmsprop_kernel");
}

void loss_mean_launch(const double *loss, int64_t B, double *out, hipStream_t s) {
    loss_mean_kernel<<<1, 256, 0, s>>>(loss, B, out);
    launch_check("loss_mean_kernel");
}

}  // namespace snk

#ifdef SNK_ENV_CLOCKS
using namespace snk;
// profiling builds: out[wg][8] = upd_fwd_kernel phase stamps of the LAST launch (call after it)
extern "C" int snk_upd_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 8);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 8 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_upd_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
// out[wg][4] = grad_update_kernel stamps of the LAST launch
extern "C" int snk_gu_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 4);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 4 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_gu_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
// out[wg][8] = conv3_bwd_kernel phase stamps of the LAST launch
extern "C" int snk_c3b_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 8);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 8 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_c3b_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
// out[wg][8] = conv2_bwd_kernel phase stamps of the LAST launch
extern "C" int snk_c2b_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 8);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 8 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_c2b_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
// out[wg][8] = conv_h3f_kernel phase stamps of the LAST launch
extern "C" int snk_h3f_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
    return guard([&] {
        static uint64_t *buf = nullptr;
        static int64_t cap = 0;
        if (arm) {
            if (n_wg > cap) {
                dfree(buf);
                buf = dalloc<uint64_t>(n_wg * 8);
                cap = n_wg;
            }
            SNK_HIP(hipMemset(buf, 0, n_wg * 8 * sizeof(uint64_t)));
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_h3f_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
#endif

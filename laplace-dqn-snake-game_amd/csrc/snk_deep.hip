// snk_deep.hip — the deeper bf16 Q-net of BASELINE.json configs[2] (the
// kernels and their semantics: snk_deep.hpp) behind the DQNModel handle:
// a snk_dqn created by snk_dqn_create_deep answers the same C ABI (params in
// Flux.destructure order, forward / epsilon_greedy / loss + gradient /
// RMSProp / target sync, the batched trainer) with this network.
#include <algorithm>
#include <cmath>
#include <vector>

#include "snk_deep.hpp"
#include "snk_deep_bwd.hpp"
#include "snk_dqn.hpp"

namespace snk {

DeepLayout deep_layout(int bs, int C) {
    DeepLayout D{};
    D.bs = bs;
    D.C = C;
    D.Wo = bs - 5;
    D.K1 = D.Wo * D.Wo * 64;
    const int ci[4] = {C, 32, 32, 64}, co[4] = {32, 32, 64, 64}, ks[4] = {3, 3, 3, 6}, pd[4] = {1, 1, 1, 0};
    int64_t o = 0;
    for (int l = 0; l < 4; ++l) {
        D.cin[l] = ci[l]; D.cout[l] = co[l]; D.ks[l] = ks[l]; D.pad[l] = pd[l];
        D.off_w[l] = o; o += (int64_t)ks[l] * ks[l] * ci[l] * co[l];
        D.off_b[l] = o; o += co[l];
    }
    D.off_d1w = o; o += (int64_t)D.K1 * 64;
    D.off_d1b = o; o += 64;
    D.off_d2w = o; o += 3 * 64;
    D.off_d2b = o; o += 3;
    D.P = o;
    int64_t t = 0;
    D.img_w[0] = -1;
    for (int l = 1; l < 4; ++l) {
        D.img_w[l] = t;
        t += (int64_t)ks[l] * ks[l] * ci[l] * co[l];
    }
    D.img_d1 = t;
    t += (int64_t)D.K1 * 64;
    D.img_wt[0] = -1;
    for (int l = 1; l < 4; ++l) {
        D.img_wt[l] = t;
        t += (int64_t)ks[l] * ks[l] * ci[l] * co[l];
    }
    D.img_n = t;
    D.img0_n = 9LL * C * 32 + 32;
    return D;
}

QLayout deep_head_layout(const DeepLayout &D) {
    QLayout L{};
    L.bs = D.bs;
    L.C = D.C;
    L.ncell = D.bs * D.bs;
    L.Wo = D.Wo;
    L.K1 = D.K1;
    L.off_d1w = D.off_d1w;
    L.off_d1b = D.off_d1b;
    L.off_d2w = D.off_d2w;
    L.off_d2b = D.off_d2b;
    L.P = D.P;
    return L;
}

void deep_packed_to_flux(const DeepLayout &D, int32_t *perm) {
    for (int l = 0; l < 4; ++l) {   // packed W[(kk*Cin + ci)*Cout + co], kk = du + KS*dv  <-  flux w[KS-1-du, KS-1-dv, ci, co]
        const int KS = D.ks[l], Cin = D.cin[l], Cout = D.cout[l];
        const int64_t off = D.off_w[l];
        for (int dv = 0; dv < KS; ++dv)
            for (int du = 0; du < KS; ++du)
                for (int ci = 0; ci < Cin; ++ci)
                    for (int co = 0; co < Cout; ++co) {
                        const int64_t pk = ((int64_t)(du + KS * dv) * Cin + ci) * Cout + co;
                        const int64_t fx = (KS - 1 - du) + (int64_t)KS * (KS - 1 - dv) + (int64_t)KS * KS * ci +
                                           (int64_t)KS * KS * Cin * co;
                        perm[off + pk] = (int32_t)(off + fx);
                    }
        for (int co = 0; co < Cout; ++co) perm[D.off_b[l] + co] = (int32_t)(D.off_b[l] + co);
    }
    const int np = D.Wo * D.Wo;
    for (int p = 0; p < np; ++p)   // Dense1: packed W[p*64 + c][o] <- flux W[o, p + c*np]
        for (int c = 0; c < 64; ++c)
            for (int o = 0; o < 64; ++o)
                perm[D.off_d1w + ((int64_t)p * 64 + c) * 64 + o] = (int32_t)(D.off_d1w + o + ((int64_t)p + (int64_t)c * np) * 64);
    for (int o = 0; o < 64; ++o) perm[D.off_d1b + o] = (int32_t)(D.off_d1b + o);
    for (int a = 0; a < 3; ++a)
        for (int o = 0; o < 64; ++o) perm[D.off_d2w + a * 64 + o] = (int32_t)(D.off_d2w + a + 3 * o);
    for (int a = 0; a < 3; ++a) perm[D.off_d2b + a] = (int32_t)(D.off_d2b + a);
}

// workspace of one batch geometry
struct DeepWork {
    int64_t cap = 0;
    uint16_t *a[4] = {};          // conv outputs, bf16 [S][pos][c]
    float *slab = nullptr;        // Dense1 partial pre-activations [Z][S][64]
    int64_t slab_floats = 0;
    float *h1 = nullptr, *q = nullptr;
    int has_train = 0;
    float *dq = nullptr, *dz1 = nullptr, *dz[4] = {};   // relu-masked gradients at each layer's output (fp32)
    double *target = nullptr, *loss = nullptr;
};

struct DeepNet {
    DeepLayout D{};
    uint16_t *img_q = nullptr, *img_t = nullptr;   // bf16 weight images of q_net / t_net
    float *img0_q = nullptr, *img0_t = nullptr;    // L0 image (bf16-rounded fp32)
    DeepWork act, tgt, trn;
    float *bslab = nullptr;                        // K-split weight-gradient partials
    int64_t bslab_floats = 0;
    int64_t gen = 0;                               // bumped on every workspace reallocation
};

// Dense1 row tiles per wave (deep_dense1_kernel<NR>)
static int d1_rows(int64_t S) { return S >= 16384 ? 4 : 1; }

// Dense1 K splits: about 256 workgroups in all, each split a multiple of 32 features
static int d1_splits(const DeepLayout &D, int64_t S, int &kchunk) {
    const int64_t bx = (S + 64 * d1_rows(S) - 1) / (64 * d1_rows(S));
    int z = (int)std::max<int64_t>(1, std::min<int64_t>(64, 256 / bx));
    kchunk = ((D.K1 + z - 1) / z + 31) & ~31;
    return (D.K1 + kchunk - 1) / kchunk;
}

static void work_free(DeepWork &w) {
    for (void *p : {(void *)w.a[0], (void *)w.a[1], (void *)w.a[2], (void *)w.a[3], (void *)w.slab, (void *)w.h1,
                    (void *)w.q, (void *)w.dq, (void *)w.dz1, (void *)w.dz[0], (void *)w.dz[1], (void *)w.dz[2],
                    (void *)w.dz[3], (void *)w.target, (void *)w.loss})
        dfree(p);
    w = DeepWork{};
}

static void work_ensure(DeepNet &N, DeepWork &w, int64_t S, bool train) {
    const DeepLayout &D = N.D;
    int kc;
    const int64_t need_slab = (int64_t)d1_splits(D, S, kc) * S * 64;
    if (S <= w.cap && need_slab <= w.slab_floats && (!train || w.has_train)) return;
    (void)hipStreamSynchronize(stream());
    const int64_t cap = std::max(S, w.cap);
    const bool tr = train || w.has_train;
    const int64_t slab = std::max({need_slab, w.slab_floats, (int64_t)d1_splits(D, cap, kc) * cap * 64});
    work_free(w);
    ++N.gen;
    const int64_t nc = (int64_t)D.bs * D.bs, no = (int64_t)D.Wo * D.Wo;
    w.cap = cap;
    w.slab_floats = slab;
    w.a[0] = dalloc<uint16_t>(cap * nc * 32);
    w.a[1] = dalloc<uint16_t>(cap * nc * 32);
    w.a[2] = dalloc<uint16_t>(cap * nc * 64);
    w.a[3] = dalloc<uint16_t>((cap + 15) / 16 * 16 * no * 64);   // whole 16-sample blocks (blocked layout)
    w.slab = dalloc<float>(slab);
    w.h1 = dalloc<float>(cap * 64);
    w.q = dalloc<float>(cap * 3);
    if (tr) {
        w.has_train = 1;
        w.dq = dalloc<float>(cap * 3);
        w.dz1 = dalloc<float>(cap * 64);
        w.dz[0] = dalloc<float>(cap * nc * 32);
        w.dz[1] = dalloc<float>(cap * nc * 32);
        w.dz[2] = dalloc<float>(cap * nc * 64);
        w.dz[3] = dalloc<float>(cap * no * 64);
        w.target = dalloc<double>(cap);
        w.loss = dalloc<double>(cap);
    }
}

// ---------------------------------------------------------------- forward
template <int CIN, int COUT, int KS, int PAD, int H>
static void conv_layer(const uint16_t *x, const uint16_t *img, const float *bias, uint16_t *y, int64_t S,
                       hipStream_t s) {
    using Sh = DeepConvShape<CIN, COUT, KS, PAD, H>;
    static_assert(Sh::LDS <= 160 * 1024, "deep conv LDS");
    set_lds_limit((const void *)deep_conv_kernel<CIN, COUT, KS, PAD, H, 4>, Sh::LDS);
    deep_conv_kernel<CIN, COUT, KS, PAD, H, 4><<<(unsigned)S, 256, Sh::LDS, s>>>(x, img, bias, y);
    launch_check("deep_conv_kernel");
}

template <int BS>
static void conv_layers_bs(const DeepNet &N, const float *th, const uint16_t *img, DeepWork &w, int64_t S,
                           hipStream_t s, int lo, int hi) {
    const DeepLayout &D = N.D;
    if (lo <= 1 && hi >= 1) conv_layer<32, 32, 3, 1, BS>(w.a[0], img + D.img_w[1], th + D.off_b[1], w.a[1], S, s);
    if (lo <= 2 && hi >= 2) conv_layer<32, 64, 3, 1, BS>(w.a[1], img + D.img_w[2], th + D.off_b[2], w.a[2], S, s);
    if (lo <= 3 && hi >= 3 && S <= 512) {   // small batches: tile rows x samples (deep_conv3_small_kernel)
        using Sx = DeepDxShape<64, 64, 6, 5, BS - 5>;
        set_lds_limit((const void *)deep_conv3_small_kernel<BS>, Sx::LDS);
        deep_conv3_small_kernel<BS><<<dim3(Sx::NB, (unsigned)S), 512, Sx::LDS, s>>>(w.a[2], img + D.img_w[3],
                                                                                   th + D.off_b[3], w.a[3], S);
        launch_check("deep_conv3_small_kernel");
    } else if (lo <= 3 && hi >= 3) {   // two samples per step of a persistent workgroup (deep_conv3_kernel)
        using Sh = DeepL3Shape<BS>;
        static_assert(Sh::LDS <= 160 * 1024, "deep L3 LDS");
        set_lds_limit((const void *)deep_conv3_kernel<BS>, Sh::LDS);
        const unsigned grid = (unsigned)std::min<int64_t>((S + 1) / 2, cu_count());
        // a3 in the blocked layout deep_dense1_ldsb_kernel / deep_dense1_kernel<4, true> read (the act
        // forward's large batches)
        deep_conv3_kernel<BS><<<grid, 512, Sh::LDS, s>>>(w.a[2], img + D.img_w[3], th + D.off_b[3], w.a[3], S,
                                                         d1_rows(S) == 4 ? 1 : 0);
        launch_check("deep_conv3_kernel");
    }
}

// L0 + L1 + L2 in one persistent launch (deep_front_kernel): one workgroup per CU
template <int C, int H>
static void front_launch(const DeepNet &N, const float *th, const uint16_t *img, const float *img0, const BoardSrc &src,
                         int64_t S, DeepWork &w, bool keep, hipStream_t s) {
    using Sh = DeepFrontShape<H>;
    static_assert(Sh::LDS <= 160 * 1024, "deep front LDS");
    const DeepLayout &D = N.D;
    const unsigned grid = (unsigned)std::min<int64_t>(S, cu_count());
    if (keep) {
        set_lds_limit((const void *)deep_front_kernel<C, H, true>, Sh::LDS);
        deep_front_kernel<C, H, true><<<grid, 512, Sh::LDS, s>>>(src, img0, img + D.img_w[1], th + D.off_b[1],
                                                                  img + D.img_w[2], th + D.off_b[2], w.a[0], w.a[1],
                                                                  w.a[2], S);
    } else {
        set_lds_limit((const void *)deep_front_kernel<C, H, false>, Sh::LDS);
        deep_front_kernel<C, H, false><<<grid, 512, Sh::LDS, s>>>(src, img0, img + D.img_w[1], th + D.off_b[1],
                                                                   img + D.img_w[2], th + D.off_b[2], nullptr, nullptr,
                                                                   w.a[2], S);
    }
    launch_check("deep_front_kernel");
}

// layers lo..hi of the forward (0..3 convs, 4 Dense1) into w; returns the Dense1 split count.
// L0..L2 run fused (deep_front_kernel) whenever the range covers all three; keep: also
// store the L0 / L1 outputs (the training forward)
static int deep_layers(const DeepNet &N, const float *th, const uint16_t *img, const float *img0,
                       const BoardSrc &src, int64_t S, DeepWork &w, hipStream_t s, int lo = 0, int hi = 4,
                       bool keep = false) {
    const DeepLayout &D = N.D;
    SNK_CHECK(S <= w.cap && S <= INT32_MAX, SNK_ERR_INTERNAL, "deep forward batch");
    if (lo <= 0 && hi >= 2) {
        auto go = [&](auto cc, auto hh) {
            front_launch<decltype(cc)::value, decltype(hh)::value>(N, th, img, img0, src, S, w, keep, s);
        };
        using I1 = std::integral_constant<int, 1>;
        using I2 = std::integral_constant<int, 2>;
        switch (D.bs * 4 + D.C) {
            case 10 * 4 + 1: go(I1{}, std::integral_constant<int, 10>{}); break;
            case 10 * 4 + 2: go(I2{}, std::integral_constant<int, 10>{}); break;
            case 12 * 4 + 1: go(I1{}, std::integral_constant<int, 12>{}); break;
            case 12 * 4 + 2: go(I2{}, std::integral_constant<int, 12>{}); break;
            case 20 * 4 + 1: go(I1{}, std::integral_constant<int, 20>{}); break;
            case 20 * 4 + 2: go(I2{}, std::integral_constant<int, 20>{}); break;
            default: SNK_CHECK(false, SNK_ERR_INVALID, "deep net: board side %d not built (10, 12, 20)", D.bs);
        }
        lo = 3;
    }
    if (lo <= 0 && hi >= 0) {
        const int ns = (int)std::max<int64_t>(1, std::min<int64_t>(8, S / 1024));
        const size_t lds = (size_t)(9 * D.C * 32 + 32 + ns * D.C * (D.bs + 2) * (D.bs + 2)) * sizeof(float);
        const unsigned grid = (unsigned)((S + ns - 1) / ns);
        if (D.C == 1)
            deep_conv0_kernel<1><<<grid, 256, lds, s>>>(src, img0, w.a[0], S, D.bs, ns);
        else
            deep_conv0_kernel<2><<<grid, 256, lds, s>>>(src, img0, w.a[0], S, D.bs, ns);
        launch_check("deep_conv0_kernel");
    }
    if (lo <= 3 && hi >= 1) {
        switch (D.bs) {
            case 10: conv_layers_bs<10>(N, th, img, w, S, s, lo, hi); break;
            case 12: conv_layers_bs<12>(N, th, img, w, S, s, lo, hi); break;
            case 20: conv_layers_bs<20>(N, th, img, w, S, s, lo, hi); break;
            default: SNK_CHECK(false, SNK_ERR_INVALID, "deep net: board side %d not built (10, 12, 20)", D.bs);
        }
    }
    int kc;
    const int z = d1_splits(D, S, kc);
    if (lo <= 4 && hi >= 4) {
#ifndef DEEP_D1_LDSB
#define DEEP_D1_LDSB 1
#endif
        if (DEEP_D1_LDSB && d1_rows(S) == 4 && z == 1 && D.K1 % 64 == 0)
            deep_dense1_ldsb_kernel<4><<<(unsigned)((S + 255) / 256), 256, 0, s>>>(w.a[3], img + D.img_d1, S, D.K1, w.slab);
        else if (d1_rows(S) == 4)
            deep_dense1_kernel<4, true><<<dim3((unsigned)((S + 255) / 256), (unsigned)z), 256, 0, s>>>(w.a[3], img + D.img_d1,
                                                                                                S, D.K1, kc, w.slab);
        else
            deep_dense1_kernel<1><<<dim3((unsigned)((S + 63) / 64), (unsigned)z), 256, 0, s>>>(w.a[3], img + D.img_d1,
                                                                                               S, D.K1, kc, w.slab);
        launch_check("deep_dense1 kernels");
    }
    return z;
}

static void deep_images(const DeepNet &N, const float *th, uint16_t *img, float *img0, hipStream_t s) {
    const int64_t n = N.D.img_n + N.D.img0_n;
    deep_image_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 4096), 256, 0, s>>>(th, img, img0, N.D);
    launch_check("deep_image_kernel");
}

// ---------------------------------------------------------------- backward
template <int NT, class AL, class BL, class EP>
static void gemm_bf16(const AL &al, const BL &bl, const EP &ep, int64_t M, int N, int64_t K, const GemmPlan &p,
                      hipStream_t s) {
    dim3 grid((unsigned)ceil_div(M, 32), (unsigned)ceil_div(N, NT * 32), (unsigned)p.z);
    switch (p.kw) {
        case 1: gemm_bf16_kernel<NT, 1><<<grid, 64, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        case 2: gemm_bf16_kernel<NT, 2><<<grid, 128, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        case 4: gemm_bf16_kernel<NT, 4><<<grid, 256, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
        default: gemm_bf16_kernel<NT, 8><<<grid, 512, 0, s>>>(al, bl, ep, (int)M, (int)K, p.kchunk); break;
    }
    launch_check("gemm_bf16_kernel");
}

static GemmPlan wgrad_plan(int64_t M, int N, int NT, int64_t K) {
    GemmPlan p = plan_gemm(M, N, NT, K, true);
    p.kchunk = (p.kchunk + 15) & ~15;   // whole 16-k MFMA steps per split
    p.z = (int)((K + p.kchunk - 1) / p.kchunk);
    return p;
}

// a weight gradient into grad[off, off + M*N): straight, or through K-split slabs
template <int NT, class AL>
static void wgrad(DeepNet &Nn, const AL &al, const float *dz, int64_t R, int M, int N, float *grad, int64_t off,
                  hipStream_t s) {
    const GemmPlan p = wgrad_plan(M, N, NT, R);
    const int64_t need = p.z > 1 ? (int64_t)p.z * M * N : 0;
    SNK_CHECK(need <= Nn.bslab_floats, SNK_ERR_INTERNAL, "deep backward slab too small");
    float *dst = p.z > 1 ? Nn.bslab : grad + off;
    gemm_bf16<NT>(al, BRows{dz, R, N}, EpSlab{dst, M, N}, M, N, R, p, s);
    if (p.z > 1) slab_reduce_launch(Nn.bslab, p.z, (int64_t)M * N, grad + off, s);
}

// a conv layer's weight gradient (deep_conv_dw_kernel, NS samples per chunk) into grad_w (weights, then bias)
template <int CI, int CO, int KS, int PAD, int H, int NS>
static void conv_dw(DeepNet &Nn, const float *dz, const uint16_t *x, int64_t B, float *grad_w, hipStream_t s) {
    using Sw = DeepDwShape<CI, CO, KS, PAD, H, NS>;
    const int64_t Z = (B + NS - 1) / NS;
    SNK_CHECK(Z * Sw::MN <= Nn.bslab_floats, SNK_ERR_INTERNAL, "deep backward slab too small");
    set_lds_limit((const void *)deep_conv_dw_kernel<CI, CO, KS, PAD, H, NS>, Sw::LDS);
    deep_conv_dw_kernel<CI, CO, KS, PAD, H, NS><<<dim3(KS, (unsigned)Z), 512, Sw::LDS, s>>>(dz, x, Nn.bslab, B);
    launch_check("deep_conv_dw_kernel");
    slab_reduce_launch(Nn.bslab, (int)Z, Sw::MN, grad_w, s);
}
// its data gradient (deep_conv_dx_kernel), relu-masked by the layer input x
template <int CI, int CO, int KS, int PAD, int H>
static void conv_dx(const float *dz, const uint16_t *wt, const uint16_t *x, float *dx, int64_t B, hipStream_t s) {
    using Sx = DeepDxShape<CI, CO, KS, PAD, H>;
    set_lds_limit((const void *)deep_conv_dx_kernel<CI, CO, KS, PAD, H>, Sx::LDS);
    deep_conv_dx_kernel<CI, CO, KS, PAD, H><<<dim3(Sx::NB, (unsigned)B), 512, Sx::LDS, s>>>(dz, wt, x, dx, B);
    launch_check("deep_conv_dx_kernel");
}

template <int BS>
static void deep_backward_bs(DeepNet &Nn, const float *th, const uint16_t *wimg, const BoardSrc &src, int64_t B,
                             DeepWork &w, float *grad, hipStream_t s) {
    const DeepLayout &D = Nn.D;
    constexpr int NC = BS * BS, WO = BS - 5, NO = WO * WO, K1 = NO * 64;
    const QLayout H = deep_head_layout(D);
    d2_grad_launch(w.dq, w.h1, B, H, grad, s);
    // Dense1: dW (+ bias row) | dX with the relu mask of a3
    wgrad<2>(Nn, ADenseDw<uint16_t>{w.a[3], K1, B}, w.dz1, B, K1 + 1, 64, grad, D.off_d1w, s);
    gemm_bf16<2>(ARowMajor{w.dz1, 64, 64}, BTrans{th + D.off_d1w, 64, K1, 64}, EpReluMaskB{w.dz[3], w.a[3], B, K1},
                 B, K1, 64, plan_gemm(B, K1, 2, 64, false), s);
    // L3 (6x6, 64 -> 64, valid), L2 and L1 (3x3 pad 1) on snk_deep_bwd.hpp: weight gradients into
    // chunk slabs (summed in chunk order), data gradients per tile row
    conv_dw<64, 64, 6, 0, BS, 2>(Nn, w.dz[3], w.a[2], B, grad + D.off_w[3], s);
    conv_dx<64, 64, 6, 0, BS>(w.dz[3], wimg + D.img_wt[3], w.a[2], w.dz[2], B, s);
    conv_dw<32, 64, 3, 1, BS, 1>(Nn, w.dz[2], w.a[1], B, grad + D.off_w[2], s);
    conv_dx<32, 64, 3, 1, BS>(w.dz[2], wimg + D.img_wt[2], w.a[1], w.dz[1], B, s);
    conv_dw<32, 32, 3, 1, BS, 1>(Nn, w.dz[1], w.a[0], B, grad + D.off_w[1], s);
    conv_dx<32, 32, 3, 1, BS>(w.dz[1], wimg + D.img_wt[1], w.a[0], w.dz[0], B, s);
    // L0: weights only, from the boards
    wgrad<1>(Nn, ABoardDw{src, BS, D.C, B * NC, FastDiv(NC), FastDiv(BS)}, w.dz[0], B * NC, 9 * D.C + 1, 32, grad,
             D.off_w[0], s);
}

// largest training batch of the deep backward (chunk slabs: 2.4 GB at L3)
constexpr int DEEP_BWD_MAX_B = 8192;

static int64_t backward_slab_floats(const DeepLayout &D, int64_t B) {
    const int64_t nc = (int64_t)D.bs * D.bs;
    int64_t need = 0;
    auto add = [&](int64_t M, int N, int NT, int64_t R) {
        const GemmPlan p = wgrad_plan(M, N, NT, R);
        if (p.z > 1) need = std::max(need, (int64_t)p.z * M * N);
    };
    add(D.K1 + 1, 64, 2, B);
    need = std::max(need, (B + 1) / 2 * ((36 * 64 + 1) * 64));   // deep_conv_dw_kernel's chunk slabs: L3 (pairs),
    need = std::max(need, B * ((9 * 32 + 1) * 64));                 // L2 and L1 (one sample per chunk)
    add(9 * D.C + 1, 32, 1, B * nc);
    return std::max<int64_t>(need, 1);
}

// ---------------------------------------------------------------- handle hooks (snk_dqn.hpp)
void deep_create(snk_dqn_s *h, int bs, int C, uint64_t seed) {
    auto *N = new DeepNet();
    h->deep = N;
    N->D = deep_layout(bs, C);
    const DeepLayout &D = N->D;
    h->L = deep_head_layout(D);
    const int64_t P = D.P;
    h->theta_q = dalloc<float>(P);
    h->theta_t = dalloc<float>(P);
    h->acc = dalloc<float>(P);
    h->grad = dalloc<float>(P);
    h->tmp = dalloc<float>(P);
    h->perm = dalloc<int32_t>(P);
    h->loss_dev = dalloc<double>(1);
    N->img_q = dalloc<uint16_t>(D.img_n);
    N->img_t = dalloc<uint16_t>(D.img_n);
    N->img0_q = dalloc<float>(D.img0_n);
    N->img0_t = dalloc<float>(D.img0_n);
    std::vector<int32_t> perm(P);
    deep_packed_to_flux(D, perm.data());
    // Flux default init (glorot_uniform weights, zero biases) from the counter RNG, in Flux order
    std::vector<float> flux(P, 0.0f);
    uint64_t ctr = 0;
    auto fill = [&](int64_t off, int64_t n, double fan_in, double fan_out) {
        const double lim = std::sqrt(6.0 / (fan_in + fan_out));
        for (int64_t i = 0; i < n; ++i) {
            const double u = (double)(splitmix64(seed ^ splitmix64(++ctr)) >> 11) * (1.0 / 9007199254740992.0);
            flux[off + i] = (float)((2.0 * u - 1.0) * lim);
        }
    };
    for (int l = 0; l < 4; ++l) {
        const double kk = (double)D.ks[l] * D.ks[l];
        fill(D.off_w[l], (int64_t)kk * D.cin[l] * D.cout[l], kk * D.cin[l], kk * D.cout[l]);
    }
    fill(D.off_d1w, (int64_t)D.K1 * 64, D.K1, 64);
    fill(D.off_d2w, 3 * 64, 64, 3);
    hipStream_t s = stream();
    SNK_HIP(hipMemcpyAsync(h->perm, perm.data(), P * 4, hipMemcpyHostToDevice, s));
    SNK_HIP(hipMemcpyAsync(h->tmp, flux.data(), P * 4, hipMemcpyHostToDevice, s));
    dqn_permute(h, h->tmp, h->theta_q, true, s);
    deep_q_changed(h, s);
    deep_sync_target(h, nullptr, 1, s);
    SNK_HIP(hipMemsetAsync(h->acc, 0, P * 4, s));
    SNK_HIP(hipMemsetAsync(h->grad, 0, P * 4, s));
    SNK_HIP(hipMemsetAsync(h->loss_dev, 0, 8, s));
    SNK_HIP(hipStreamSynchronize(s));
}

void deep_free(snk_dqn_s *h) {
    DeepNet *N = h->deep;
    if (!N) return;
    work_free(N->act);
    work_free(N->tgt);
    work_free(N->trn);
    for (void *p : {(void *)N->img_q, (void *)N->img_t, (void *)N->img0_q, (void *)N->img0_t, (void *)N->bslab})
        dfree(p);
    delete N;
    h->deep = nullptr;
}

int64_t deep_ws_gen(const snk_dqn_s *h) { return h->deep ? h->deep->gen : 0; }

void deep_q_changed(snk_dqn_s *h, hipStream_t s) { deep_images(*h->deep, h->theta_q, h->deep->img_q, h->deep->img0_q, s); }
void deep_t_changed(snk_dqn_s *h, hipStream_t s) { deep_images(*h->deep, h->theta_t, h->deep->img_t, h->deep->img0_t, s); }

__global__ void deep_copy_if_due_kernel(const float *__restrict__ src, float *__restrict__ dst, int64_t n,
                                        const int64_t *__restrict__ counter, int64_t rate) {
    if (counter && (*counter % rate) != 0) return;   // update_target_net! when nb % rate == 0 (utils.jl:469)
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

void deep_sync_target(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s) {
    DeepNet &N = *h->deep;
    auto cp = [&](const float *a, float *b, int64_t n) {
        deep_copy_if_due_kernel<<<(unsigned)std::min<int64_t>(ceil_div(n, 256), 2048), 256, 0, s>>>(a, b, n, counter, rate);
        launch_check("deep_copy_if_due_kernel");
    };
    cp(h->theta_q, h->theta_t, N.D.P);
    cp(reinterpret_cast<const float *>(N.img_q), reinterpret_cast<float *>(N.img_t), N.D.img_n / 2);
    cp(N.img0_q, N.img0_t, N.D.img0_n);
}

void deep_prepare(snk_dqn_s *h, int64_t S_act, int64_t B) {
    DeepNet &N = *h->deep;
    if (S_act > 0) work_ensure(N, N.act, S_act, false);
    if (B > 0) {
        // the backward kernels are sized for the reference's B = 64: their chunk slabs grow
        // linearly with B ((B+1)/2 x 147,520 floats at L3) and conv_dx puts B on grid.y, so
        // a batch past this bound is refused here instead of over-allocating or failing a launch
        SNK_CHECK(B <= DEEP_BWD_MAX_B, SNK_ERR_INVALID,
                  "deep net: training batch %lld > %d (the bf16 backward is built for B = 64 batches)",
                  (long long)B, DEEP_BWD_MAX_B);
        work_ensure(N, N.tgt, B, false);
        work_ensure(N, N.trn, B, true);
        const int64_t need = backward_slab_floats(N.D, B);
        if (need > N.bslab_floats) {
            (void)hipStreamSynchronize(stream());
            dfree(N.bslab);
            N.bslab = dalloc<float>(need);
            N.bslab_floats = need;
            ++N.gen;
        }
    }
}

const float *deep_forward(snk_dqn_s *h, int32_t which, const BoardSrc &src, int64_t S, HeadMode mode,
                          const HeadArgs &ha, hipStream_t s) {
    DeepNet &N = *h->deep;
    deep_prepare(h, S, 0);
    const bool t = which == SNK_NET_TARGET;
    const float *th = t ? h->theta_t : h->theta_q;
    const int z = deep_layers(N, th, t ? N.img_t : N.img_q, t ? N.img0_t : N.img0_q, src, S, N.act, s);
    head_launch(h->L, th, N.act.slab, z, S, N.act.h1, N.act.q, mode, ha, s);
    return N.act.q;
}

void deep_time_layers(snk_dqn_s *h, const BoardSrc &src, int64_t S, const HeadArgs &ha, int reps, double *ms,
                      hipStream_t s) {
    DeepNet &N = *h->deep;
    deep_forward(h, SNK_NET_Q, src, S, HEAD_ACT, ha, s);
    hipEvent_t a, b;
    SNK_HIP(hipEventCreate(&a));
    SNK_HIP(hipEventCreate(&b));
    for (int layer = 0; layer < 6; ++layer) {
        if (layer == 1 || layer == 2) {   // inside layer 0's fused launch
            ms[layer] = 0.0;
            continue;
        }
        SNK_HIP(hipEventRecord(a, s));
        for (int r = 0; r < reps; ++r) {
            if (layer < 5) {
                deep_layers(N, h->theta_q, N.img_q, N.img0_q, src, S, N.act, s, layer, layer == 0 ? 2 : layer);
            } else {
                int kc;
                head_launch(h->L, h->theta_q, N.act.slab, d1_splits(N.D, S, kc), S, N.act.h1, N.act.q, HEAD_ACT, ha, s);
            }
        }
        SNK_HIP(hipEventRecord(b, s));
        SNK_HIP(hipEventSynchronize(b));
        float ms1 = 0.0f;
        SNK_HIP(hipEventElapsedTime(&ms1, a, b));
        ms[layer] = (double)ms1 / reps;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
}

void deep_loss_grad(snk_dqn_s *h, const BoardSrc &s_src, const BoardSrc &sn_src, const HeadArgs &meta, int64_t B,
                    double gamma, hipStream_t s, bool loss_mean) {
    DeepNet &N = *h->deep;
    deep_prepare(h, 0, B);
    const int zt = deep_layers(N, h->theta_t, N.img_t, N.img0_t, sn_src, B, N.tgt, s);
    const int zq = deep_layers(N, h->theta_q, N.img_q, N.img0_q, s_src, B, N.trn, s, 0, 4, true);
    SNK_CHECK(zt == zq, SNK_ERR_INTERNAL, "deep head splits");
    HeadArgs la = meta;
    la.gamma = gamma;
    la.target = N.trn.target;
    la.B = B;
    la.loss = N.trn.loss;
    la.dq = N.trn.dq;
    la.dz1 = N.trn.dz1;
    head_pair_launch(h->L, h->theta_t, N.tgt.slab, N.tgt.h1, N.tgt.q, h->theta_q, N.trn.slab, N.trn.h1, N.trn.q, zq, B,
                     la, s);
    if (loss_mean) loss_mean_launch(N.trn.loss, B, h->loss_dev, s);
    switch (N.D.bs) {
        case 10: deep_backward_bs<10>(N, h->theta_q, N.img_q, s_src, B, N.trn, h->grad, s); break;
        case 12: deep_backward_bs<12>(N, h->theta_q, N.img_q, s_src, B, N.trn, h->grad, s); break;
        default: deep_backward_bs<20>(N, h->theta_q, N.img_q, s_src, B, N.trn, h->grad, s); break;
    }
}

const double *deep_batch_losses(snk_dqn_s *h) { return h->deep->trn.loss; }

void deep_apply(snk_dqn_s *h, const int64_t *counter, int64_t rate, hipStream_t s) {
    rmsprop_launch(h->deep->D.P, h->theta_q, h->acc, h->grad, h->lr, h->rho, h->eps, s);
    deep_q_changed(h, s);
    if (counter) deep_sync_target(h, counter, rate, s);
}

}  // namespace snk

using namespace snk;

extern "C" int snk_dqn_create_deep(snk_dqn *out, int32_t bs, int32_t C, float lr, float rho, float eps,
                                   uint64_t seed) {
    return guard([&] {
        SNK_CHECK(out, SNK_ERR_INVALID, "out is NULL");
        SNK_CHECK((bs == 10 || bs == 12 || bs == 20) && (C == 1 || C == 2), SNK_ERR_INVALID,
                  "deep DQNModel: board side 10, 12 or 20 and 1 or 2 frames");
        auto *h = new snk_dqn_s();
        h->lr = lr;
        h->rho = rho;
        h->eps = eps;
        try {
            deep_create(h, bs, C, seed);
        } catch (...) {
            snk_dqn_destroy(h);
            throw;
        }
        *out = h;
    });
}

extern "C" int snk_dqn_time_deep_layers(snk_dqn h, snk_env env, int32_t reps, double *ms_out) {
    return guard([&] {
        SNK_CHECK(h && h->deep && env && ms_out && reps > 0, SNK_ERR_INVALID, "bad time_deep_layers arguments");
        const EnvDev &E = env_dev(env);
        SNK_CHECK(E.bs == h->L.bs && E.C == h->L.C, SNK_ERR_INVALID, "env/model geometry mismatch");
        if (h->meta_cap < E.n) {
            SNK_HIP(hipStreamSynchronize(stream()));
            dfree(h->meta);
            h->meta = dalloc<uint8_t>(2 * E.n);
            h->meta_cap = E.n;
        }
        HeadArgs ha;
        ha.act = h->meta;
        ha.epsilon = 0.05f;
        ha.tptr = &E.ctl->t;
        deep_time_layers(h, src_env(E), E.n, ha, reps, ms_out, stream());
    });
}

#ifdef SNK_ENV_CLOCKS
// profiling builds: out[wg][8] = deep_front_kernel's per-phase time sums of the LAST launch
// (s_memrealtime ticks, 100 MHz; slot 6 = the workgroup's sample count)
extern "C" int snk_dfr_debug_clocks(int64_t n_wg, uint64_t *out_host, int32_t arm) {
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
            SNK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dfr_clk), &buf, sizeof(buf)));
            return;
        }
        SNK_HIP(hipDeviceSynchronize());
        SNK_HIP(hipMemcpy(out_host, buf, n_wg * 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    });
}
#endif

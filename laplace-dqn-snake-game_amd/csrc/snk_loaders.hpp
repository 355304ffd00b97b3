// snk_loaders.hpp — operand loaders of the generic implicit-GEMM engines
// (snk_gemm.hpp fp32, snk_deep.hpp bf16): implicit im2col for the forward,
// data-gradient and weight-gradient convolutions of a Q-net, and the K-split
// planner for the latency-bound B = 64 backward.
#pragma once
#include <algorithm>

#include "snk_qnet.hpp"

namespace snk {

// element loads of fp32 or bf16 (stored as uint16_t) sources
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(uint16_t b) { return __uint_as_float((uint32_t)b << 16); }

// ---------------------------------------------------------------- fast division
struct FastDiv {  // n / d == (umulhi(n, m) + n) >> s for 0 <= n < 2^31
    uint32_t d = 1, m = 1, s = 0;
    FastDiv() = default;
    explicit FastDiv(uint32_t dd) : d(dd) {
        s = 0;
        while ((1u << s) < d) ++s;
        m = (uint32_t)(((((uint64_t)1) << 32) * ((((uint64_t)1) << s) - d)) / d + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, m) + n) >> s; }
};

// ---------------------------------------------------------------- A loaders
template <int CIN, int KS, int PAD>
struct AConvFwd {  // row m=(s,pout), k=(kk,ci): x[s][pin][ci]
    const float *x;
    int H, HO;
    FastDiv dHO2, dHO;
    struct Ctx { const float *xs; int i, j; bool ok; };
    __device__ Ctx row(int m, int M) const {
        Ctx c;
        c.ok = m < M;
        const int mm = c.ok ? m : 0;
        const int s = (int)dHO2.div(mm);
        const int p = mm - s * HO * HO;
        c.j = (int)dHO.div(p);
        c.i = p - c.j * HO;
        c.xs = x + (int64_t)s * H * H * CIN;
        return c;
    }
    __device__ __forceinline__ float load(const Ctx &c, int k, int) const {
        const int kk = k / CIN, ci = k - kk * CIN;
        const int dv = kk / KS, du = kk - dv * KS;
        const int xi = c.i + du - PAD, xj = c.j + dv - PAD;
        return (c.ok && xi >= 0 && xi < H && xj >= 0 && xj < H) ? c.xs[(xi + xj * H) * CIN + ci] : 0.0f;
    }
};

template <int COUT, int KS, int PAD>
struct AConvDx {  // row m=(s,pin), k=(kk,co): dz[s][pout = pin - (du,dv) + PAD][co]
    const float *dz;
    int H, HO;
    FastDiv dH2, dH;
    struct Ctx { const float *zs; int i, j; bool ok; };
    __device__ Ctx row(int m, int M) const {
        Ctx c;
        c.ok = m < M;
        const int mm = c.ok ? m : 0;
        const int s = (int)dH2.div(mm);
        const int p = mm - s * H * H;
        c.j = (int)dH.div(p);
        c.i = p - c.j * H;
        c.zs = dz + (int64_t)s * HO * HO * COUT;
        return c;
    }
    __device__ __forceinline__ float load(const Ctx &c, int k, int) const {
        const int kk = k / COUT, co = k - kk * COUT;
        const int dv = kk / KS, du = kk - dv * KS;
        const int oi = c.i - du + PAD, oj = c.j - dv + PAD;
        return (c.ok && oi >= 0 && oi < HO && oj >= 0 && oj < HO) ? c.zs[(oi + oj * HO) * COUT + co] : 0.0f;
    }
};

template <int CIN, int KS, int PAD, class T = float>
struct AConvDw {  // row m=(kk,ci) (m == KS*KS*CIN: bias row of ones), k = r = (s,pout)
    const T *x;
    int H, HO;
    int64_t R;
    FastDiv dHO2, dHO;
    struct Ctx { int du, dv, ci; bool ok, bias; };
    __device__ Ctx row(int m, int M) const {
        Ctx c;
        c.ok = m < M;
        c.bias = m == KS * KS * CIN;
        const int kk = m / CIN;
        c.ci = m - kk * CIN;
        c.dv = kk / KS;
        c.du = kk - c.dv * KS;
        return c;
    }
    __device__ __forceinline__ float load(const Ctx &c, int k, int) const {
        if (!c.ok || k >= R) return 0.0f;
        if (c.bias) return 1.0f;
        const int s = (int)dHO2.div(k);
        const int p = k - s * HO * HO;
        const int j = (int)dHO.div(p), i = p - j * HO;
        const int xi = i + c.du - PAD, xj = j + c.dv - PAD;
        return (xi >= 0 && xi < H && xj >= 0 && xj < H) ? to_f32(x[((int64_t)s * H * H + xi + xj * H) * CIN + c.ci])
                                                          : 0.0f;
    }
};

struct ABoardDw {  // conv1 weight gradient: row m=(kk,c) (+bias row), k = r = (s,p)
    BoardSrc src;
    int bs, C;
    int64_t R;
    FastDiv dN, dB;
    struct Ctx { int du, dv, c; bool ok, bias; };
    __device__ Ctx row(int m, int M) const {
        Ctx x;
        x.ok = m < M;
        x.bias = m == 9 * C;
        const int kk = m / C;
        x.c = m - kk * C;
        x.dv = kk / 3;
        x.du = kk - x.dv * 3;
        return x;
    }
    __device__ __forceinline__ float load(const Ctx &x, int k, int) const {
        if (!x.ok || k >= R) return 0.0f;
        if (x.bias) return 1.0f;
        const int s = (int)dN.div(k);
        const int p = k - s * bs * bs;
        const int j = (int)dB.div(p), i = p - j * bs;
        const int xi = i + x.du - 1, xj = j + x.dv - 1;
        return (xi >= 0 && xi < bs && xj >= 0 && xj < bs) ? src.load(s, x.c, xi + xj * bs) : 0.0f;
    }
};

struct ARowMajor {  // A[m][k] = a[m*ld + k]
    const float *a;
    int K, ld;
    struct Ctx { const float *p; bool ok; };
    __device__ Ctx row(int m, int M) const { return Ctx{a + (int64_t)(m < M ? m : 0) * ld, m < M}; }
    __device__ __forceinline__ float load(const Ctx &c, int k, int) const { return (c.ok && k < K) ? c.p[k] : 0.0f; }
};

template <class T = float>
struct ADenseDw {  // row m = input feature (m == KW: bias ones), k = sample r: a[r*KW + m]
    const T *a;
    int KW;
    int64_t R;
    struct Ctx { int m; bool ok, bias; };
    __device__ Ctx row(int m, int M) const { return Ctx{m, m < M, m == KW}; }
    __device__ __forceinline__ float load(const Ctx &c, int k, int) const {
        if (!c.ok || k >= R) return 0.0f;
        return c.bias ? 1.0f : to_f32(a[(int64_t)k * KW + c.m]);
    }
};

// ---------------------------------------------------------------- launch helpers

// kw waves per output tile (intra-workgroup split-K, LDS reduce) and z
// workgroup splits (partial slabs) chosen to put ~1 wave on every SIMD while
// keeping >= 64 k per wave.
struct GemmPlan {
    int kw, z, kchunk;
};
inline GemmPlan plan_gemm(int64_t M, int N, int NT, int64_t K, bool allow_z) {
    const int64_t tiles = ceil_div(M, 32) * ceil_div(N, NT * 32);
    // these GEMMs (the B = 64 backward) are latency-bound: many short waves
    // (~4096 waves of >= 32 k each; measured flat from 4096/32 to 16384/8 on the B = 64 update)
    constexpr int64_t target = 4096, mink = 32;
    int kw = 1;
    while (kw < 8 && tiles * kw * 2 <= target && K / (kw * 2) >= mink) kw *= 2;
    int z = 1;
    if (allow_z)
        while (z < 64 && tiles * kw * z * 2 <= target && K / ((int64_t)kw * z * 2) >= mink) z *= 2;
    int64_t chunk = ceil_div(K, z);
    chunk = (chunk + 7) & ~int64_t(7);
    return GemmPlan{kw, (int)ceil_div(K, chunk), (int)chunk};
}

// the same with the waves per tile fixed (paired launches need equal block sizes)
inline GemmPlan plan_gemm_kw(int64_t M, int N, int NT, int64_t K, bool allow_z, int kw) {
    const int64_t tiles = ceil_div(M, 32) * ceil_div(N, NT * 32);
    constexpr int64_t target = 4096, mink = 32;
    int z = 1;
    if (allow_z)
        while (z < 64 && tiles * kw * z * 2 <= target && K / ((int64_t)kw * z * 2) >= mink) z *= 2;
    int64_t chunk = ceil_div(K, z);
    chunk = (chunk + 7) & ~int64_t(7);
    return GemmPlan{kw, (int)ceil_div(K, chunk), (int)chunk};
}

}  // namespace snk

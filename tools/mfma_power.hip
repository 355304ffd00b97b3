// microbenchmark: throughput and held clock of MFMA loops on random operands,
// every CU busy (two waves per SIMD), f16 vs int8 vs bf16 shapes.
// Question it answers (round 5, the Jacobian Gram): does the int8 MFMA hold a
// higher clock than the f16 one on random data? An exact fp32 product needs 3
// f16 MFMAs (h3: hl + lh + hh, 16x16x32) or 3 int8 MFMAs (three 8-bit digits,
// the 6 digit products of weight >= 2^-16 at 16x16x64 = 2x the K), the same
// cycles, so the int8 form wins exactly by its clock and by its 3 bytes per
// element against 4.
// Modes: R = operands in registers; L = A and B fragments re-read from LDS by
// ds_read_b128 every 2 MFMAs (the Gram kernel's 0.5 KB of fragment per MFMA).
// Clock = d(s_memtime) / d(s_memrealtime) x 100 MHz, median over workgroups.
// hipcc --offload-arch=gfx950 -O3 tools/mfma_power.hip -o tools/mfma_power.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T, typename S> __device__ __forceinline__ T bc(S s) { return __builtin_bit_cast(T, s); }

constexpr int NACC = 8;   // independent accumulators per wave

// KIND 0 f16 16x16x32, 1 i8 16x16x64, 2 bf16 16x16x32, 3 i8 32x32x32, 4 f16 32x32x16
template <int KIND, bool LDSR>
__global__ __launch_bounds__(256) void loop(const u32x4 *__restrict__ src, int iters, float *__restrict__ out,
                                            uint64_t *__restrict__ stamps) {
    __shared__ u32x4 lds[1024];   // 16 KB of random fragments
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) lds[i] = src[(blockIdx.x * 1024 + i) & 65535];
    __syncthreads();
    u32x4 a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a[q] = lds[(lane + 64 * q) & 1023];
        b[q] = lds[(lane + 64 * q + 512) & 1023];
    }
    constexpr bool BIG = KIND >= 3;
    f32x4 cf[NACC];
    i32x4 ci[NACC];
    f32x16 cF[BIG ? NACC / 2 : 1];
    i32x16 cI[BIG ? NACC / 2 : 1];
#pragma unroll
    for (int k = 0; k < NACC; ++k) { cf[k] = f32x4{0, 0, 0, 0}; ci[k] = i32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int k = 0; k < (BIG ? NACC / 2 : 1); ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) { cF[k][e] = 0; cI[k][e] = 0; }
    __syncthreads();
    uint64_t t0 = 0, r0 = 0;
    if (tid == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    const int wv = tid >> 6;
    for (int it = 0; it < iters; ++it) {
        if (LDSR) {
            // two fragments (A, B) per pair of MFMAs, addresses rotating over the 16 KB
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] = lds[(lane + 64 * ((it + q + wv) & 7)) & 1023];
                b[q] = lds[(lane + 64 * ((it + q + wv + 3) & 7) + 512) & 1023];
            }
        }
#pragma unroll
        for (int k = 0; k < NACC; ++k) {
            const u32x4 x = a[k & 3], y = b[(k >> 1) & 3];
            if constexpr (KIND == 0)
                cf[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bc<f16x8>(x), bc<f16x8>(y), cf[k], 0, 0, 0);
            else if constexpr (KIND == 1)
                ci[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bc<i32x4>(x), bc<i32x4>(y), ci[k], 0, 0, 0);
            else if constexpr (KIND == 2)
                cf[k] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bc<bf16x8>(x), bc<bf16x8>(y), cf[k], 0, 0, 0);
            else if constexpr (KIND == 3) {
                if (k < NACC / 2) cI[k] = __builtin_amdgcn_mfma_i32_32x32x32_i8(bc<i32x4>(x), bc<i32x4>(y), cI[k], 0, 0, 0);
            } else {
                if (k < NACC / 2) cF[k] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bc<f16x8>(x), bc<f16x8>(y), cF[k], 0, 0, 0);
            }
        }
    }
    __syncthreads();
    if (tid == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < NACC; ++k) s += cf[k][0] + (float)ci[k][1];
#pragma unroll
    for (int k = 0; k < (BIG ? NACC / 2 : 1); ++k) s += cF[k][3] + (float)cI[k][5];
    out[blockIdx.x * 256 + tid] = s;
}

int main(int argc, char **argv) {
    const int NWG = 256 * 2;   // two 4-wave workgroups per CU: two waves per SIMD
    std::vector<uint32_t> h(65536 * 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    // operand fill: f16 kinds get uniform [-1, 1) halves (random mantissas and signs),
    // int8 kinds random bytes, bf16 uniform [-1, 1)
    std::vector<uint32_t> hf(h.size()), hi(h.size()), hb(h.size());
    for (size_t i = 0; i < h.size(); ++i) {
        uint32_t w = 0, v = 0;
        for (int p = 0; p < 2; ++p) {
            const float f = (float)((double)(rnd() >> 11) / 9007199254740992.0 * 2.0 - 1.0);
            _Float16 hh = (_Float16)f;
            uint16_t u; __builtin_memcpy(&u, &hh, 2);
            w |= (uint32_t)u << (16 * p);
            uint32_t fb; __builtin_memcpy(&fb, &f, 4);
            v |= (fb >> 16) << (16 * p);
        }
        hf[i] = w; hb[i] = v; hi[i] = (uint32_t)rnd();
    }
    u32x4 *df, *di, *db; float *dout; uint64_t *dst;
    CK(hipMalloc(&df, h.size() * 4)); CK(hipMalloc(&di, h.size() * 4)); CK(hipMalloc(&db, h.size() * 4));
    CK(hipMemcpy(df, hf.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(di, hi.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), h.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dout, NWG * 256 * 4)); CK(hipMalloc(&dst, NWG * 16));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 20000;
    struct K { const char *name; int kind; bool lds; double macs_per_mfma; int mfma_per_iter; };
    const K ks[] = {
        {"f16_16x16x32 R", 0, false, 16 * 16 * 32, NACC}, {"i8_16x16x64 R", 1, false, 16 * 16 * 64, NACC},
        {"bf16_16x16x32 R", 2, false, 16 * 16 * 32, NACC}, {"i8_32x32x32 R", 3, false, 32 * 32 * 32, NACC / 2},
        {"f16_32x32x16 R", 4, false, 32 * 32 * 16, NACC / 2},
        {"f16_16x16x32 L", 0, true, 16 * 16 * 32, NACC}, {"i8_16x16x64 L", 1, true, 16 * 16 * 64, NACC},
        {"i8_32x32x32 L", 3, true, 32 * 32 * 32, NACC / 2}, {"f16_32x32x16 L", 4, true, 32 * 32 * 16, NACC / 2},
    };
    for (int rep = 0; rep < 2; ++rep)
        for (const K &k : ks) {
            const u32x4 *s = k.kind == 1 || k.kind == 3 ? di : (k.kind == 2 ? db : df);
            auto launch = [&]() {
#define L(KD, LD) loop<KD, LD><<<NWG, 256>>>(s, iters, dout, dst)
                if (k.lds) { if (k.kind == 0) L(0, true); else if (k.kind == 1) L(1, true); else if (k.kind == 3) L(3, true); else L(4, true); }
                else { if (k.kind == 0) L(0, false); else if (k.kind == 1) L(1, false); else if (k.kind == 2) L(2, false); else if (k.kind == 3) L(3, false); else L(4, false); }
#undef L
            };
            // ~2 s of back-to-back launches, then 20 timed ones
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms1; CK(hipEventElapsedTime(&ms1, e0, e1));
            const int warm = std::max(1, (int)(2000.0f / std::max(ms1, 0.01f)));
            for (int i = 0; i < warm; ++i) launch();
            const int reps = std::max(1, (int)(1000.0f / std::max(ms1, 0.01f)));
            CK(hipEventRecord(e0));
            for (int i = 0; i < reps; ++i) launch();
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint64_t> st(NWG * 2);
            CK(hipMemcpy(st.data(), dst, NWG * 16, hipMemcpyDeviceToHost));
            std::vector<double> clk;
            for (int w = 0; w < NWG; ++w)
                if (st[2 * w + 1]) clk.push_back((double)st[2 * w] / (double)st[2 * w + 1] * 100.0);
            std::sort(clk.begin(), clk.end());
            const double per = ms / reps * 1e-3;
            const double mfma = (double)NWG * 4 * iters * k.mfma_per_iter;
            const double cyc_per_mfma = clk[clk.size() / 2] * 1e6 * per / (mfma / 1024.0);   // per SIMD (1024 SIMDs)
            printf("{\"rep\": %d, \"kernel\": \"%s\", \"ms\": %.3f, \"mfma_per_s\": %.4g, \"tops\": %.1f, \"clock_mhz\": %.0f, "
                   "\"cyc_per_mfma_simd\": %.2f}\n",
                   rep, k.name, per * 1e3, mfma / per, mfma * k.macs_per_mfma * 2 / per * 1e-12, clk[clk.size() / 2], cyc_per_mfma);
            fflush(stdout);
        }
    return 0;
}

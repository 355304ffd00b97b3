// microbenchmark: throughput and held clock of MFMA loops on dense random operands,
// every CU busy (two waves per SIMD), one kernel per MFMA kind.
// Question (round 5, the Jacobian Gram on dense rows holds ~1.5 GHz): does an int8 MFMA
// cost less power than the f16 one? An exact fp32 product needs 3 f16 MFMAs (h3: hl + lh +
// hh at 16x16x32) or, as three 8-bit fixed-point digits, 8 int8 digit products at 16x16x64
// (2x the K): 4 f16-equivalents. So int8 pays only if its MFMAs/s on random data exceed
// f16's by more than 4/3.
// Modes: R = operands in registers (rotated each iteration so nothing is loop-invariant);
// L = one A and one B fragment re-read from LDS by ds_read_b128 every 2 MFMAs (the Gram
// kernel's 0.5 KB of fragment per MFMA).
// Clock = d(s_memtime) / d(s_memrealtime) x 100 MHz, median over workgroups.
// hipcc --offload-arch=gfx950 -O3 tools/mfma_power.hip -o tools/mfma_power.bin
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T, typename S> __device__ __forceinline__ T bc(S s) { return __builtin_bit_cast(T, s); }

constexpr int NACC = 8;

template <bool I8> struct Acc { typedef f32x4 T; };
template <> struct Acc<true> { typedef i32x4 T; };

template <bool I8, bool LDSR>
__global__ __launch_bounds__(256) void loop(const u32x4 *__restrict__ src, int iters, u32x4 *__restrict__ out,
                                            uint64_t *__restrict__ stamps) {
    __shared__ u32x4 lds[1024];
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 1024; i += 256) lds[i] = src[(blockIdx.x * 1024 + i) & 65535];
    __syncthreads();
    u32x4 a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        a[q] = lds[(lane + 64 * q) & 1023];
        b[q] = lds[(lane + 64 * q + 512) & 1023];
    }
    typename Acc<I8>::T c[NACC];
#pragma unroll
    for (int k = 0; k < NACC; ++k) c[k] = typename Acc<I8>::T{0, 0, 0, 0};
    uint64_t t0 = 0, r0 = 0;
    if (tid == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    const int wv = tid >> 6;
    for (int it = 0; it < iters; ++it) {
        if (LDSR) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                a[q] = lds[(lane + 64 * ((it + q + wv) & 7)) & 1023];
                b[q] = lds[(lane + 64 * ((it + q + wv + 3) & 7) + 512) & 1023];
            }
        }
#pragma unroll
        for (int k = 0; k < NACC; ++k) {
            const u32x4 x = a[k & 3], y = b[(k >> 1) & 3];
            if constexpr (I8)
                c[k] = __builtin_amdgcn_mfma_i32_16x16x64_i8(bc<i32x4>(x), bc<i32x4>(y), c[k], 0, 0, 0);
            else
                c[k] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bc<f16x8>(x), bc<f16x8>(y), c[k], 0, 0, 0);
        }
        if (!LDSR) {   // rotate the operand registers (a cheap permutation: no loop-invariant MFMAs)
            const u32x4 t = a[0];
            a[0] = a[1]; a[1] = a[2]; a[2] = a[3]; a[3] = b[0];
            b[0] = b[1]; b[1] = b[2]; b[2] = b[3]; b[3] = t;
        }
    }
    if (tid == 0) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    u32x4 s = u32x4{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < NACC; ++k) s += bc<u32x4>(c[k]);
    out[blockIdx.x * 256 + tid] = s;
}

int main() {
    const int NWG = 256 * 2;   // two 4-wave workgroups per CU: two waves per SIMD
    std::vector<uint32_t> hf(65536 * 4), hi(65536 * 4);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (size_t i = 0; i < hf.size(); ++i) {
        uint32_t w = 0;
        for (int p = 0; p < 2; ++p) {   // f16 uniform in [-1, 1): random mantissas, signs, exponents near 0
            const float f = (float)((double)(rnd() >> 11) / 9007199254740992.0 * 2.0 - 1.0);
            _Float16 hh = (_Float16)f;
            uint16_t u; __builtin_memcpy(&u, &hh, 2);
            w |= (uint32_t)u << (16 * p);
        }
        hf[i] = w;
        hi[i] = (uint32_t)rnd();     // int8: uniform random bytes
    }
    u32x4 *df, *di, *dout; uint64_t *dst;
    CK(hipMalloc(&df, hf.size() * 4)); CK(hipMalloc(&di, hi.size() * 4));
    CK(hipMemcpy(df, hf.data(), hf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(di, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&dout, NWG * 256 * 16)); CK(hipMalloc(&dst, NWG * 16));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 20000;
    struct K { const char *name; bool i8, lds; double macs; };
    const K ks[] = {{"f16_16x16x32 R", false, false, 16 * 16 * 32}, {"i8_16x16x64 R", true, false, 16 * 16 * 64},
                    {"f16_16x16x32 L", false, true, 16 * 16 * 32}, {"i8_16x16x64 L", true, true, 16 * 16 * 64}};
    for (int rep = 0; rep < 2; ++rep)
        for (const K &k : ks) {
            auto launch = [&]() {
                if (k.i8) { if (k.lds) loop<true, true><<<NWG, 256>>>(di, iters, dout, dst); else loop<true, false><<<NWG, 256>>>(di, iters, dout, dst); }
                else { if (k.lds) loop<false, true><<<NWG, 256>>>(df, iters, dout, dst); else loop<false, false><<<NWG, 256>>>(df, iters, dout, dst); }
            };
            CK(hipEventRecord(e0)); launch(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
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
            const double mfma = (double)NWG * 4 * iters * NACC;
            printf("{\"rep\": %d, \"kernel\": \"%s\", \"ms\": %.3f, \"mfma_per_s\": %.4g, \"tops\": %.1f, \"clock_mhz\": %.0f, "
                   "\"cyc_per_mfma_simd\": %.2f}\n",
                   rep, k.name, per * 1e3, mfma / per, mfma * k.macs * 2 / per * 1e-12, clk[clk.size() / 2],
                   clk[clk.size() / 2] * 1e6 * per / (mfma / 1024.0));
            fflush(stdout);
        }
    return 0;
}

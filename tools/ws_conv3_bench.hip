// Microbenchmark (tools/, not the library): the conv3 phase of a weight-stationary
// act forward. 4 waves per workgroup (one per SIMD), wave w holds the fp16 h/l
// conv3 weight fragments of 32 output channels (w & 1) x 18 kernel offsets (w >> 1)
// in registers (288 VGPR/AGPR) and runs 18 offsets x 13 row tiles x 2 column tiles
// x 3 products of v_mfma_f32_16x16x32_f16 per group of four samples, A fragments
// from conv_h3f_kernel's LDS image layout (12x12 boards). Persistent grid of 256
// workgroups x G groups. hipcc --offload-arch=gfx950 -O3 tools/ws_conv3_bench.hip -o /tmp/wsb
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int HIN = 12, ho = 7, XW = ho + 8, PL = (HIN * XW + 3) & ~3, GG = 2 * PL, XS = 4 * GG + 4;
constexpr int NT = 13;

template <int SPLIT>
__global__ __launch_bounds__(256) void ws(const u32x4 *w, const u32x4 *img, float *out, int groups) {
    extern __shared__ u32x4 As[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, r = lane & 15, g = lane >> 4;
    const int cp = wave & 1, oh = wave >> 1;
    f16x8 wf[18][2][2];
#pragma unroll
    for (int a = 0; a < 18; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) wf[a][b][c] = __builtin_bit_cast(f16x8, w[(((oh * 18 + a) * 4 + cp * 2 + b) * 2 + c) * 64 + lane]);
    for (int i = tid; i < 4 * XS; i += 256) As[i] = img[i];
    __syncthreads();
    int abase[NT];
#pragma unroll
    for (int k = 0; k < NT; ++k) {
        const int q = 16 * k + r, p = min(q >> 2, ho * ho - 1), sr = q & 3, j = p / ho, i = p - j * ho;
        abase[k] = sr * XS + g * GG + j * XW + i;
    }
    for (int grp = blockIdx.x; grp < groups; grp += gridDim.x) {
        // two passes over the offsets, row tiles [0, 7) then [7, 13): 56 accumulator registers
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            constexpr int TP = 7;
            const int t0 = pass * TP, tn = pass ? NT - TP : TP;
            f32x4 acc[TP][2];
#pragma unroll
            for (int k = 0; k < TP; ++k) acc[k][0] = acc[k][1] = f32x4{0, 0, 0, 0};
            // A fragments two tiles ahead (named rotation: stage n holds tile n of the flattened (kq, k) walk)
            constexpr int NST = 3;
            f16x8 fh[NST], fl[NST];
            auto rd = [&](int n, int slot) __attribute__((always_inline)) {
                const int kq = n / TP, k = n % TP;
                if (kq >= 18 || k >= tn) return;
                const int kk = oh * 18 + kq, dv = kk / 6, du = kk - dv * 6, off = dv * XW + du;
                fh[slot] = __builtin_bit_cast(f16x8, As[abase[t0 + k] + off]);
                fl[slot] = __builtin_bit_cast(f16x8, As[abase[t0 + k] + off + PL]);
            };
            rd(0, 0);
            rd(1, 1);
#pragma unroll
            for (int n = 0; n < 18 * TP; ++n) {
                const int kq = n / TP, k = n % TP;
                rd(n + 2, (n + 2) % NST);
                if (k < tn) {
                    const f16x8 ah = fh[n % NST], al = fl[n % NST];
#pragma unroll
                    for (int ct = 0; ct < 2; ++ct) {
                        f32x4 c = acc[k][ct];
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, wf[kq][ct][0], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wf[kq][ct][1], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, wf[kq][ct][0], c, 0, 0, 0);
                        acc[k][ct] = c;
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < TP; ++k)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        if (k < tn) out[(((int64_t)grp * NT * 2 + (t0 + k) * 2 + ct) * 4 + e) * 256 + tid] = acc[k][ct][e];
        }
    }
}

int main() {
    const int groups = 1024;
    std::vector<unsigned> hw(18 * 2 * 4 * 2 * 64 * 4), hi(4 * XS * 4);
    unsigned s = 1;
    for (auto &x : hw) { s = s * 1664525u + 1013904223u; x = (s & 0x3bff3bffu); }
    for (auto &x : hi) { s = s * 1664525u + 1013904223u; x = (s & 0x3bff3bffu); }
    u32x4 *dw, *di; float *dout;
    hipMalloc(&dw, hw.size() * 4); hipMalloc(&di, hi.size() * 4);
    hipMalloc(&dout, (size_t)groups * NT * 2 * 4 * 256 * 4);
    hipMemcpy(dw, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    hipMemcpy(di, hi.data(), hi.size() * 4, hipMemcpyHostToDevice);
    const size_t lds = 4 * XS * 16;
    hipFuncSetAttribute((const void *)ws<0>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; ++rep) {
        for (int i = 0; i < 200; ++i) ws<0><<<256, 256, lds>>>(dw, di, dout, groups);
        hipEventRecord(a);
        for (int i = 0; i < 200; ++i) ws<0><<<256, 256, lds>>>(dw, di, dout, groups);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        const double us = 1e3 * ms / 200, fl = 2.0 * 4096 * 49 * 64 * 1152 * 3;
        printf("{\"groups\": %d, \"us\": %.2f, \"fp16_tflops\": %.1f, \"frac_fp16_peak\": %.3f}\n", groups, us, fl / us / 1e6, fl / us / 1e6 / 2516);
    }
    return 0;
}

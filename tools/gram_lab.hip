// gram_lab: the D(50k) conv-column Gram, round 6. Times the round-5 kernel
// (syrk_h3q_kernel, 128 x 128 tiles, fp64 flush every 1024 k) and the K-split
// 256 x 256 kernel (syrk_h3k_kernel + syrk_ksum_kernel) on the same random
// Jacobian-sized rows in ONE process, with the in-kernel clock of every
// workgroup (measurement build: -DSNK_SYRK_MEASURE, stamps to their own buffer),
// and measures each K-split chunk length's error against the fp64-flush Gram
// on sampled rows: max |G - G_ref| / sqrt(G_ii G_jj).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSNK_SYRK_MEASURE -I include \
//   -I laplace-dqn-snake-game_amd/csrc tools/gram_lab.hip -o tools/gram_lab.bin
// ./tools/gram_lab.bin [n=50000] [reps=2] [chunk stages, comma list=320] [zero %=0]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "snk_syrk.hpp"

namespace snk {
void set_error(const char *, ...) {}
hipStream_t stream() { return nullptr; }
int arith(int) { return 0; }
}  // namespace snk
using namespace snk;

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            printf("{\"error\": \"%s line %d\"}\n", hipGetErrorString(e), __LINE__);       \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// as tools/syrk_lab.hip: normal values, a per-row binade spread, zero_pct % exact zeros
__global__ void fill_rows(float *x, int64_t n, int64_t K, uint64_t seed, int zero256) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * K; t += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)t * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        const float u1 = ((z >> 40) + 0.5f) * (1.0f / 16777216.0f), u2 = ((z & 0xFFFFFF) + 0.5f) * (1.0f / 16777216.0f);
        const float g = sqrtf(-2.0f * logf(u1)) * cosf(6.2831853f * u2);
        const int64_t row = t / K;
        const bool dead = (int)((z >> 24) & 0xFF) < zero256;
        x[t] = dead ? 0.0f : ldexpf(g, (int)(row % 9) - 4);
    }
}

static std::vector<int2> order128(int N) {   // round 5's supertile order (8 x 4)
    const int T = (N + SY_T - 1) / SY_T;
    std::vector<int2> t;
    for (int i0 = 0; i0 < T; i0 += 8)
        for (int j0 = 0; j0 <= std::min(T - 1, i0 + 7); j0 += 4)
            for (int i = i0; i < std::min(T, i0 + 8); ++i)
                for (int j = j0; j < std::min(j0 + 4, i + 1); ++j) t.push_back(int2{i, j});
    return t;
}

// 256-tiles in supertiles of SI x SJ; items (I, J, z, tile) supertile-major, then chunk,
// dealt to 8 XCD queues in contiguous runs and interleaved (workgroup w -> XCD w % 8)
static void order256(int N, int nst, int cs, int SI, int SJ, std::vector<int2> &tiles, std::vector<int4> &items) {
    const int T = (N + SK_T - 1) / SK_T, S = (nst + cs - 1) / cs;
    tiles.clear();
    std::vector<int4> list;
    for (int i0 = 0; i0 < T; i0 += SI)
        for (int j0 = 0; j0 <= std::min(T - 1, i0 + SI - 1); j0 += SJ) {
            const int first = (int)tiles.size();
            for (int i = i0; i < std::min(T, i0 + SI); ++i)
                for (int j = j0; j < std::min(j0 + SJ, i + 1); ++j) tiles.push_back(int2{i, j});
            for (int z = 0; z < S; ++z)
                for (int t = first; t < (int)tiles.size(); ++t) list.push_back(int4{tiles[t].x, tiles[t].y, z, t});
        }
    const size_t L = list.size();
    std::vector<std::vector<int4>> q(8);
    size_t p = 0;
    for (int x = 0; x < 8; ++x) {
        const size_t len = L / 8 + ((size_t)x < L % 8 ? 1 : 0);
        for (size_t e = 0; e < len; ++e) q[x].push_back(list[p++]);
    }
    items.clear();
    for (size_t j = 0; j < q[0].size(); ++j)
        for (int x = 0; x < 8; ++x)
            if (j < q[x].size()) items.push_back(q[x][j]);
}

static void clock_stats(const uint64_t *st, int64_t nwg, double &med, double &p10, double &p90) {
    std::vector<uint64_t> h(nwg * 4);
    CK(hipMemcpy(h.data(), st, nwg * 32, hipMemcpyDeviceToHost));
    std::vector<double> clk;
    for (int64_t w = 0; w < nwg; w += 7) {
        const double dt = (double)(h[4 * w + 2] - h[4 * w]), dr = (double)(h[4 * w + 3] - h[4 * w + 1]);
        if (dr > 0) clk.push_back(dt / dr * 100.0);
    }
    std::sort(clk.begin(), clk.end());
    med = clk[clk.size() / 2];
    p10 = clk[clk.size() / 10];
    p90 = clk[clk.size() * 9 / 10];
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 50000;
    const int reps = argc > 2 ? atoi(argv[2]) : 2;
    std::vector<int> chunks;
    {
        const char *s = argc > 3 ? argv[3] : "320";
        while (*s) {
            chunks.push_back(atoi(s));
            while (*s && *s != ',') ++s;
            if (*s == ',') ++s;
        }
    }
    const int zero_pct = argc > 4 ? atoi(argv[4]) : 0;
    const int SI = argc > 5 ? atoi(argv[5]) : 8, SJ = argc > 6 ? atoi(argv[6]) : 4;
    const int64_t K = 9 * 2 * 16 + 16 + 4640 + 73792;   // conv columns of a 12x12, 2-frame Jacobian row
    const int64_t ldh = (K + SY_KS - 1) / SY_KS * SY_KS;
    const int nst = (int)(ldh / SY_KS);
    const int64_t npad = (n + SW_ROWS_B - 1) / SW_ROWS_B * SW_ROWS_B;
    float *x;
    uint16_t *xhl;
    int32_t *xe;
    float *G;
    CK(hipMalloc(&x, (size_t)n * K * 4));
    CK(hipMalloc(&xhl, (size_t)npad * 2 * ldh * 2));
    CK(hipMalloc(&xe, (size_t)npad * 4));
    CK(hipMemset(xhl, 0, (size_t)npad * 2 * ldh * 2));
    CK(hipMemset(xe, 0, (size_t)npad * 4));
    fill_rows<<<4096, 256>>>(x, n, K, 12345, zero_pct * 256 / 100);
    h3_rows_kernel<<<n, 256>>>(x, K, K, xhl, xe, ldh);
    CK(hipDeviceSynchronize());
    CK(hipFree(x));
    CK(hipMalloc(&G, (size_t)n * n * 4));
    // the round-5 kernel's tiles and stamps
    const std::vector<int2> o128 = order128(n);
    const int64_t nt128 = (int64_t)o128.size();
    int2 *d128;
    CK(hipMalloc(&d128, nt128 * 8));
    CK(hipMemcpy(d128, o128.data(), nt128 * 8, hipMemcpyHostToDevice));
    // the K-split kernel's tables for every chunk length, and the largest partial buffer
    const int T256 = (n + SK_T - 1) / SK_T;
    const int64_t nt256 = (int64_t)T256 * (T256 + 1) / 2;
    int maxS = 0;
    for (int c : chunks) maxS = std::max(maxS, (nst + c - 1) / c);
    float *part;
    CK(hipMalloc(&part, (size_t)maxS * nt256 * SK_T * SK_T * 4));
    const int64_t maxwg = std::max<int64_t>(nt128, maxS * nt256);
    uint64_t *st;
    CK(hipMalloc(&st, maxwg * 32));
    hipEvent_t e0, e1, e2;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&e2));
    const double flop = (double)n * (n + 1) * K;   // the lower triangle's FLOP
    const int nrow = 8;
    std::vector<int> rows(nrow);
    for (int k = 0; k < nrow; ++k) rows[k] = (int)((int64_t)(k * 2 + 1) * n / (2 * nrow));
    std::vector<float> ref((size_t)nrow * n), diag(n), got((size_t)nrow * n);
    for (int rep = 0; rep < reps; ++rep) {
        {   // round 5: syrk_h3q_kernel (lower tiles), no mirror
            SyrkArgs a{};
            a.N = n; a.ntiles = nt128; a.t0 = 0; a.tiles = d128; a.direct = 0; a.g32 = G; a.ldg = n;
            a.xh = xhl; a.xe = xe; a.ldh = ldh; a.K = K; a.ld = K; a.kchunk = K; a.stamps = st;
            CK(hipEventRecord(e0));
            syrk_h3q_kernel<0, 4, false, 1><<<(unsigned)nt128, 512>>>(a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            double med, p10, p90;
            clock_stats(st, nt128, med, p10, p90);
            if (rep == 0) {
                for (int k = 0; k < nrow; ++k)
                    CK(hipMemcpy(&ref[(size_t)k * n], G + (int64_t)rows[k] * n, (size_t)n * 4, hipMemcpyDeviceToHost));
                CK(hipMemcpy2D(diag.data(), 4, G, (size_t)(n + 1) * 4, 4, n, hipMemcpyDeviceToHost));
            }
            printf("{\"rep\": %d, \"variant\": \"syrk_h3q 128x128 fp64 flush (round 5)\", \"n\": %d, \"ms\": %.2f, "
                   "\"tflops_fp32eq\": %.1f, \"frac_h3_peak\": %.4f, \"clock_mhz_median\": %.0f, \"clock_mhz_p10\": %.0f, "
                   "\"clock_mhz_p90\": %.0f}\n",
                   rep, n, ms, flop / (ms * 1e-3) * 1e-12, flop / (ms * 1e-3) * 1e-12 / (2516.0 / 3), med, p10, p90);
            fflush(stdout);
        }
        for (int cs : chunks) {
            std::vector<int2> tiles;
            std::vector<int4> items;
            order256(n, nst, cs, SI, SJ, tiles, items);
            const int S = (nst + cs - 1) / cs;
            int2 *dt;
            int4 *di;
            CK(hipMalloc(&dt, tiles.size() * 8));
            CK(hipMalloc(&di, items.size() * 16));
            CK(hipMemcpy(dt, tiles.data(), tiles.size() * 8, hipMemcpyHostToDevice));
            CK(hipMemcpy(di, items.data(), items.size() * 16, hipMemcpyHostToDevice));
            SyrkKArgs k{};
            k.xh = xhl; k.ldh = ldh; k.nst = nst; k.cs = cs; k.items = di; k.part = part; k.ntl = nt256; k.stamps = st;
            SyrkSumArgs<float> s{};
            s.part = part; s.S = S; s.ntl = nt256; s.tiles = dt; s.xe = xe; s.xes = 0; s.N = n; s.G = G; s.ldg = n; s.dense = 0;
            CK(hipMemset(G, 0, (size_t)n * n * 4));
            CK(hipEventRecord(e0));
            syrk_h3k_kernel<<<(unsigned)items.size(), 512>>>(k);
            CK(hipEventRecord(e1));
            syrk_ksum_kernel<float><<<(unsigned)(nt256 * 64), 256>>>(s);
            CK(hipEventRecord(e2));
            CK(hipEventSynchronize(e2));
            CK(hipGetLastError());
            float ms, ms2;
            CK(hipEventElapsedTime(&ms, e0, e1));
            CK(hipEventElapsedTime(&ms2, e1, e2));
            double med, p10, p90;
            clock_stats(st, (int64_t)items.size(), med, p10, p90);
            for (int k2 = 0; k2 < nrow; ++k2)
                CK(hipMemcpy(&got[(size_t)k2 * n], G + (int64_t)rows[k2] * n, (size_t)n * 4, hipMemcpyDeviceToHost));
            double rel = 0.0;
            int64_t asym = 0;
            for (int k2 = 0; k2 < nrow; ++k2)
                for (int j = 0; j <= rows[k2]; ++j)
                    rel = std::max(rel, fabs((double)got[(size_t)k2 * n + j] - ref[(size_t)k2 * n + j]) /
                                            sqrt((double)diag[rows[k2]] * diag[j]));
            {   // symmetry: row rows[0] against column rows[0]
                std::vector<float> col(n);
                CK(hipMemcpy2D(col.data(), 4, G + rows[0], (size_t)n * 4, 4, n, hipMemcpyDeviceToHost));
                for (int j = 0; j < n; ++j) asym += col[j] != got[j];
            }
            printf("{\"rep\": %d, \"variant\": \"syrk_h3k 256x256 k-split\", \"chunk_stages\": %d, \"chunks\": %d, "
                   "\"super\": \"%dx%d\", \"n\": %d, \"ms\": %.2f, \"ksum_ms\": %.2f, \"tflops_fp32eq\": %.1f, "
                   "\"frac_h3_peak\": %.4f, \"frac_with_ksum\": %.4f, \"clock_mhz_median\": %.0f, \"clock_mhz_p10\": %.0f, "
                   "\"clock_mhz_p90\": %.0f, \"max_abs_diff_over_sqrt_gii_gjj_vs_fp64_flush\": %.3g, \"asym\": %lld}\n",
                   rep, cs, S, SI, SJ, n, ms, ms2, flop / (ms * 1e-3) * 1e-12, flop / (ms * 1e-3) * 1e-12 / (2516.0 / 3),
                   flop / ((ms + ms2) * 1e-3) * 1e-12 / (2516.0 / 3), med, p10, p90, rel, (long long)asym);
            fflush(stdout);
            CK(hipFree(dt));
            CK(hipFree(di));
        }
    }
    return 0;
}

// syrk_lab: the D(50k) conv-column Gram kernel (syrk_h3q_kernel, snk_syrk.hpp) on
// random Jacobian-sized rows, in variants, timed back to back in ONE process with the
// in-kernel clock of every workgroup (s_memtime / s_memrealtime stamps: this is a
// measurement build, -DSNK_SYRK_MEASURE; the stamps go to their own buffer).
//   order 0: the library's supertile order (8 x 4 per XCD) through syrk_xcd_remap
//   order 1: the chip-wide order (syrk_order_chip below): the 256 workgroups of a
//            dispatch round work one 16 x 16 block of tiles, each XCD an 8 x 4 sub-block,
//            so the 8 XCDs share the block's 32 row panels in the Infinity Cache
//   sb 1 / 2: stages per barrier
// Every variant's G is compared bit for bit with the first one's on sampled rows (the
// variants only reorder tiles and barriers: identical per-tile arithmetic).
// hipcc --offload-arch=gfx950 -O3 -std=c++17 -DSNK_SYRK_MEASURE -I include \
//   -I laplace-dqn-snake-game_amd/csrc tools/syrk_lab.hip -o tools/syrk_lab.bin
// ./tools/syrk_lab.bin [n=50000] [reps=2] [variant mask=0x3F] [zero %=0]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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

// rows of roughly Jacobian-like statistics: normal values, a per-row binade spread and
// zero_pct % exact zeros (dead relu channels), from a counter hash
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

static std::vector<int2> order_super(int N) {   // = snk_laplace.hip syrk_tile_order_host
    const int T = (N + SY_T - 1) / SY_T;
    std::vector<int2> t;
    constexpr int SI = 8, SJ = 4;
    for (int i0 = 0; i0 < T; i0 += SI)
        for (int j0 = 0; j0 <= std::min(T - 1, i0 + SI - 1); j0 += SJ)
            for (int i = i0; i < std::min(T, i0 + SI); ++i)
                for (int j = j0; j < std::min(j0 + SJ, i + 1); ++j) t.push_back(int2{i, j});
    return t;
}

// the chip-wide order: macro blocks of 16 x 16 tiles (lower triangle, row-major over the
// blocks); a block's tiles in sub-block-major order (sub-blocks of 8 rows x 4 columns) are
// dealt to the 8 XCD queues in contiguous chunks (a full block: one sub-block each), extra
// tiles round-robin so the queue lengths differ by at most one; entry j * 8 + x of the table
// is XCD x's j-th tile (workgroup w runs on XCD w % 8)
static std::vector<int2> order_chip(int N) {
    const int T = (N + SY_T - 1) / SY_T;
    constexpr int MB = 16, SI = 8, SJ = 4;
    std::vector<std::vector<int2>> q(8);
    int rr = 0;
    for (int I0 = 0; I0 < T; I0 += MB)
        for (int J0 = 0; J0 <= I0; J0 += MB) {
            std::vector<int2> blk;
            for (int si = I0; si < std::min(T, I0 + MB); si += SI)
                for (int sj = J0; sj < std::min(T, J0 + MB); sj += SJ)
                    for (int i = si; i < std::min(T, si + SI); ++i)
                        for (int j = sj; j < std::min(sj + SJ, i + 1); ++j) blk.push_back(int2{i, j});
            const int cnt = (int)blk.size(), base = cnt / 8, extra = cnt % 8;
            int p = 0;
            for (int k = 0; k < 8; ++k) {
                const int x = k;
                const int len = base + (((k - rr + 8) % 8) < extra ? 1 : 0);
                for (int e = 0; e < len; ++e) q[x].push_back(blk[p++]);
            }
            rr = (rr + extra) % 8;
        }
    size_t tot = 0, mx = 0;
    for (auto &v : q) tot += v.size(), mx = std::max(mx, v.size());
    std::vector<int2> out(tot);
    size_t w = 0;
    for (size_t j = 0; j < mx; ++j)
        for (int x = 0; x < 8; ++x)
            if (j < q[x].size()) out[w++] = q[x][j];
    if (w != tot) printf("{\"error\": \"order_chip not dense\"}\n");
    return out;
}

// the h3r tiles (bi: 256-row blocks, bj: 128-row blocks, bj <= 2 bi + 1) in the chip-wide order:
// macro blocks of 16 bi x 32 bj (4096 x 4096), sub-blocks of 4 bi x 8 bj (1024 x 1024, 32 tiles)
static std::vector<int2> order_rect(int N) {
    const int T = (N + 127) / 128, T2 = (N + 255) / 256;
    constexpr int MBI = 16, MBJ = 32, SI = 4, SJ = 8;
    std::vector<std::vector<int2>> q(8);
    int rr = 0;
    for (int I0 = 0; I0 < T2; I0 += MBI)
        for (int J0 = 0; J0 <= std::min(T - 1, 2 * (I0 + MBI - 1) + 1); J0 += MBJ) {
            std::vector<int2> blk;
            for (int si = I0; si < std::min(T2, I0 + MBI); si += SI)
                for (int sj = J0; sj < std::min(T, J0 + MBJ); sj += SJ)
                    for (int i = si; i < std::min(T2, si + SI); ++i)
                        for (int j = sj; j < std::min(std::min(T, sj + SJ), 2 * i + 2); ++j) blk.push_back(int2{i, j});
            const int cnt = (int)blk.size(), base = cnt / 8, extra = cnt % 8;
            int p = 0;
            for (int x = 0; x < 8; ++x) {
                const int len = base + ((x - rr + 8) % 8 < extra ? 1 : 0);
                for (int e = 0; e < len; ++e) q[x].push_back(blk[p++]);
            }
            rr = (rr + extra) % 8;
        }
    size_t tot = 0, mx = 0;
    for (auto &v : q) tot += v.size(), mx = std::max(mx, v.size());
    std::vector<int2> out;
    for (size_t j = 0; j < mx; ++j)
        for (int x = 0; x < 8; ++x)
            if (j < q[x].size()) out.push_back(q[x][j]);
    return out;
}

int main(int argc, char **argv) {
    const int n = argc > 1 ? atoi(argv[1]) : 50000;
    const int reps = argc > 2 ? atoi(argv[2]) : 2;
    const int64_t K = 9 * 2 * 16 + 16 + 4640 + 73792;   // conv columns of a 12x12, 2-frame Jacobian row
    const int64_t ldh = (K + SY_KS - 1) / SY_KS * SY_KS;
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
    const int zero_pct = argc > 4 ? atoi(argv[4]) : 0;   // 0: dense rows (the library's D(50k) rows are)
    fill_rows<<<4096, 256>>>(x, n, K, 12345, zero_pct * 256 / 100);
    h3_rows_kernel<<<n, 256>>>(x, K, K, xhl, xe, ldh);
    CK(hipDeviceSynchronize());
    CK(hipFree(x));
    CK(hipMalloc(&G, (size_t)n * n * 4));
    const int T = (n + SY_T - 1) / SY_T;
    const int64_t ntiles = (int64_t)T * (T + 1) / 2;
    std::vector<int2> o0 = order_super(n), o1 = order_chip(n), o2 = order_rect(n);
    const int64_t ntiles_r = (int64_t)o2.size();
    int2 *d0, *d1, *d2;
    CK(hipMalloc(&d0, ntiles * 8));
    CK(hipMalloc(&d1, ntiles * 8));
    CK(hipMalloc(&d2, ntiles_r * 8));
    CK(hipMemcpy(d0, o0.data(), ntiles * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d1, o1.data(), ntiles * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(d2, o2.data(), ntiles_r * 8, hipMemcpyHostToDevice));
    uint64_t *st;
    CK(hipMalloc(&st, ntiles * 32));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    struct V { const char *name; int order, sb, var, nb; };
    // var 1 / 2: the measurement variants (no MFMA / no stage DMA after the prologue: wrong
    // results by design, timed for the split of the step's cost)
    const V all[] = {{"super8x4 sb1 nb4 (library)", 0, 1, 0, 4}, {"chip16x16 sb1 nb4", 1, 1, 0, 4},
                     {"super8x4 sb2 nb4", 0, 2, 0, 4},          {"chip16x16 sb2 nb4", 1, 2, 0, 4},
                     {"super8x4 nb4 no-MFMA", 0, 1, 1, 4},      {"super8x4 nb4 no-DMA", 0, 1, 2, 4},
                     {"super8x4 sb1 nb3", 0, 1, 0, 3},          {"chip16x16 sb1 nb3", 1, 1, 0, 3},
                     {"super8x4 sb1 nb5", 0, 1, 0, 5},          {"chip16x16 sb1 nb5", 1, 1, 0, 5},
                     {"chip16x16 nb4 no-MFMA", 1, 1, 1, 4},     {"chip16x16 nb4 no-DMA", 1, 1, 2, 4},
                     {"chip16x16 nb4 half-DMA (B once)", 1, 1, 3, 4},
                     {"h3r 256x128 nb3 rect-chip", 2, 1, 0, 3}, {"h3r 256x128 nb3 no-MFMA", 2, 1, 1, 3},
                     {"h3r 256x128 nb3 no-DMA", 2, 1, 2, 3},
                     {"h3r 256x128 nb3 4 waves", 2, 4, 0, 3}, {"h3r 256x128 nb3 4 waves no-MFMA", 2, 4, 1, 3},
                     {"h3r 256x128 nb3 4 waves no-DMA", 2, 4, 2, 3},
                     {"h3r 256x128 nb3 8w fp32-only", 2, 1, 4, 3}, {"h3r 256x128 nb3 4w fp32-only", 2, 4, 4, 3},

                     {"h3r 8w fp32-only global_load_lds", 2, 1, 14, 3},
                     {"h3r 8w lean two-level", 2, 1, 20, 3}};
    const int nall = sizeof(all) / sizeof(all[0]);
    const int sel = argc > 3 ? (int)strtol(argv[3], nullptr, 0) : 0x3F;   // bit v: run variant v
    std::vector<V> vv;
    for (int v = 0; v < nall; ++v)
        if (sel >> v & 1) vv.push_back(all[v]);
    const V *vs = vv.data();
    const int nv = (int)vv.size();
    const double flop = (double)n * (n + 1) * K;   // the lower triangle's FLOP (h3r's diagonal waste not counted)
    std::vector<float> ref, diag;
    const int nrow = 8;
    std::vector<int> rows(nrow);
    for (int k = 0; k < nrow; ++k) rows[k] = (int)((int64_t)(k * 2 + 1) * n / (2 * nrow));
    for (int rep = 0; rep < reps; ++rep)
        for (int v = 0; v < nv; ++v) {
            SyrkArgs a{};
            a.N = n;
            const bool rect = vs[v].order == 2;
            a.ntiles = rect ? ntiles_r : ntiles;
            a.t0 = 0;
            a.tiles = rect ? d2 : vs[v].order ? d1 : d0;
            a.direct = vs[v].order;
            a.g32 = G;
            a.ldg = n;
            a.xh = xhl;
            a.xe = xe;
            a.ldh = ldh;
            a.K = K;
            a.ld = K;
            a.kchunk = K;
            a.stamps = st;
            CK(hipMemset(G, 0, (size_t)n * n * 4));
            CK(hipEventRecord(e0));
            if (rect && vs[v].sb == 4 && vs[v].var == 0)   // sb field = waves for h3r
                syrk_h3r_kernel<0, 3, 4><<<(unsigned)ntiles_r, 256>>>(a);
            else if (rect && vs[v].sb == 4 && vs[v].var == 1)
                syrk_h3r_kernel<1, 3, 4><<<(unsigned)ntiles_r, 256>>>(a);
            else if (rect && vs[v].sb == 4 && vs[v].var == 2)
                syrk_h3r_kernel<2, 3, 4><<<(unsigned)ntiles_r, 256>>>(a);
            else if (rect && vs[v].sb == 4 && vs[v].var == 4)
                syrk_h3r_kernel<4, 3, 4><<<(unsigned)ntiles_r, 256>>>(a);
            else if (rect && vs[v].var == 4)
                syrk_h3r_kernel<4, 3><<<(unsigned)ntiles_r, 512>>>(a);
            else if (rect && vs[v].var == 20)
                syrk_h3r_kernel<0, 3, 8, 0, 1><<<(unsigned)ntiles_r, 512>>>(a);
            else if (rect && vs[v].var == 14)
                syrk_h3r_kernel<4, 3, 8, 1><<<(unsigned)ntiles_r, 512>>>(a);
            else if (rect && vs[v].var == 0)
                syrk_h3r_kernel<0, 3><<<(unsigned)ntiles_r, 512>>>(a);
            else if (rect && vs[v].var == 1)
                syrk_h3r_kernel<1, 3><<<(unsigned)ntiles_r, 512>>>(a);
            else if (rect && vs[v].var == 2)
                syrk_h3r_kernel<2, 3><<<(unsigned)ntiles_r, 512>>>(a);
            else if (vs[v].var == 1)
                syrk_h3q_kernel<1, 4, false, 1><<<(unsigned)ntiles, 512>>>(a);
            else if (vs[v].var == 2)
                syrk_h3q_kernel<2, 4, false, 1><<<(unsigned)ntiles, 512>>>(a);
            else if (vs[v].var == 3)
                syrk_h3q_kernel<3, 4, false, 1><<<(unsigned)ntiles, 512>>>(a);
            else if (vs[v].sb == 2)
                syrk_h3q_kernel<0, 4, false, 2><<<(unsigned)ntiles, 512>>>(a);
            else if (vs[v].nb == 3)
                syrk_h3q_kernel<0, 3, false, 1><<<(unsigned)ntiles, 512>>>(a);
            else if (vs[v].nb == 5)
                syrk_h3q_kernel<0, 5, false, 1><<<(unsigned)ntiles, 512>>>(a);
            else
                syrk_h3q_kernel<0, 4, false, 1><<<(unsigned)ntiles, 512>>>(a);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            CK(hipGetLastError());
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            std::vector<uint64_t> h(a.ntiles * 4);
            CK(hipMemcpy(h.data(), st, a.ntiles * 32, hipMemcpyDeviceToHost));
            std::vector<double> clk;
            double cyc = 0;
            for (int64_t w = 0; w < a.ntiles; w += 7) {
                const double dt = (double)(h[4 * w + 2] - h[4 * w]), dr = (double)(h[4 * w + 3] - h[4 * w + 1]);
                if (dr > 0) clk.push_back(dt / dr * 100.0), cyc += dt;
            }
            std::sort(clk.begin(), clk.end());
            // bit-exact check of sampled rows against the first variant (lower triangle j <= i)
            std::vector<float> got((size_t)nrow * n);
            for (int k = 0; k < nrow; ++k) CK(hipMemcpy(&got[(size_t)k * n], G + (int64_t)rows[k] * n, (size_t)n * 4, hipMemcpyDeviceToHost));
            int64_t bad = -1;
            double rel = -1.0;
            if (rep == 0 && v == 0) {
                ref = got;
                diag.resize(n);
                CK(hipMemcpy2D(diag.data(), 4, G, (size_t)(n + 1) * 4, 4, n, hipMemcpyDeviceToHost));
            } else if (vs[v].var == 0 || vs[v].var == 4 || vs[v].var == 14 || vs[v].var == 20) {
                bad = 0;
                rel = 0.0;
                for (int k = 0; k < nrow; ++k)
                    for (int j = 0; j <= rows[k]; ++j) {
                        const float x = got[(size_t)k * n + j], y = ref[(size_t)k * n + j];
                        bad += x != y;
                        rel = std::max(rel, fabs((double)x - y) / sqrt((double)diag[rows[k]] * diag[j]));
                    }
            }
            printf("{\"rep\": %d, \"variant\": \"%s\", \"n\": %d, \"ms\": %.2f, \"tflops_fp32eq\": %.1f, \"frac_h3_peak\": %.4f, "
                   "\"clock_mhz_median\": %.0f, \"clock_mhz_p10\": %.0f, \"clock_mhz_p90\": %.0f, \"mismatch_vs_first\": %lld, "
                   "\"max_abs_diff_over_sqrt_gii_gjj\": %.3g}\n",
                   rep, vs[v].name, n, ms, flop / (ms * 1e-3) * 1e-12, flop / (ms * 1e-3) * 1e-12 / (2516.0 / 3),
                   clk[clk.size() / 2], clk[clk.size() / 10], clk[clk.size() * 9 / 10], (long long)bad, rel);
            fflush(stdout);
        }
    return 0;
}

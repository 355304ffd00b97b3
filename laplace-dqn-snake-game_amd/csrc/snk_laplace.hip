// snk_laplace.hip — the Laplace D build on gfx950.
//
// (1) compute_D.jl:33-142 as the reference does it: K Float64 snapshots of
//     theta (compute_D.jl:67-71), Welford mean/var over the columns
//     (compute_D.jl:9-31 fit!), centring (compute_D.jl:80-81), and the Gram
//     G = D'D whose spectrum plot_traj.jl:10-16 takes from svd(D)
//     (lambda = S^2/(K-1) = eig(G)/(K-1)). D lives as [K][P] doubles, which is
//     exactly Julia's P x K column-major matrix. Welford/centring stay in
//     fp64 with the reference's operation order (bit-exact vs the oracle);
//     the Gram runs on fp32 MFMA (snk_syrk.hpp) over an fp32 copy of the
//     centred D with fp64 accumulation.
// (2) the north_star's per-sample-Jacobian Gram G = J J' over the replay
//     buffer. The Dense sections of a Jacobian row are outer products
//     (a3 (x) dz1, h1 (x) onehot), so their Gram contribution is
//     (A3 A3' + 1) o (Z Z') + [a_i = a_j] o (H H' + 1) — computed from the
//     per-sample activations without materialising those 200k columns; only
//     the 79k conv columns of J go through the big MFMA Gram.
#include <cstring>
#include <algorithm>
#include <deque>
#include <mutex>
#include <vector>

#include "snk_dqn.hpp"
#include "snk_syrk.hpp"

struct snk_laplace_s {
    int64_t P = 0, ld32 = 0;
    int32_t K = 0;
    double *D = nullptr, *mean = nullptr, *var = nullptr, *G = nullptr, *slab = nullptr;
    float *D32 = nullptr;
    int64_t slab_cap = 0;
    // the K-split h3 snapshot Gram (SNK_ARITH_SYRK_KSPLIT): the centred rows split by
    // lap_center_split_kernel (valid after a fit_center that made them), their per-chunk
    // exponents, and syrk_h3k_kernel's partial tiles
    uint16_t *planes = nullptr;
    int32_t *pexp = nullptr;
    int64_t ldh = 0;
    int planes_valid = 0;
    float *gpart = nullptr;
    int64_t gpart_floats = 0;
};

namespace snk {

// compute_D.jl:70  deviation_matrix[:, pos] = Float64.(theta)  (theta packed -> Flux order)
__global__ void lap_snapshot_kernel(const float *__restrict__ theta, const int32_t *__restrict__ perm, int64_t P,
                                    double *__restrict__ col) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < P; i += (int64_t)gridDim.x * blockDim.x)
        col[perm[i]] = (double)theta[i];
}

// compute_D.jl:21-27 fit! over the K columns in order, per parameter:
//   n += 1; d = x - mean; mean += d/n; m2 += d*(x - mean);  var = m2/max(n-1, 1)
__global__ __launch_bounds__(256) void lap_welford_kernel(const double *__restrict__ D, int64_t P, int K,
                                                          double *__restrict__ mean, double *__restrict__ var) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= P) return;
    double m = 0.0, m2 = 0.0;
    int k = 0;
    for (; k + 8 <= K; k += 8) {   // 8 independent loads in flight per thread
        double x[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) x[u] = D[(int64_t)(k + u) * P + p];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const double d = x[u] - m;
            m += d / (double)(k + u + 1);
            m2 += d * (x[u] - m);
        }
    }
    for (; k < K; ++k) {
        const double x = D[(int64_t)k * P + p];
        const double d = x - m;
        m += d / (double)(k + 1);
        m2 += d * (x - m);
    }
    mean[p] = m;
    var[p] = m2 / (double)(K - 1 > 1 ? K - 1 : 1);
}

// compute_D.jl:80-81 D .-= mean, plus the fp32 MFMA operand (rows padded to ld32 with zeros)
__global__ void lap_center_kernel(double *__restrict__ D, int64_t P, int K, const double *__restrict__ mean,
                                  float *__restrict__ D32, int64_t ld32) {
    const int64_t total = (int64_t)K * ld32;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t k = t / ld32, p = t - k * ld32;
        float v = 0.0f;
        if (p < P) {
            const double c = D[k * P + p] - mean[p];
            D[k * P + p] = c;
            v = (float)c;
        }
        D32[t] = v;
    }
}

// compute_D.jl:80-81 D .-= mean with lap_center_kernel's arithmetic (bit for bit), fused
// with the fp32 copy and its h3 split for the K-split snapshot Gram (syrk_h3k_kernel): one
// workgroup per (snapshot row, chunk of LAP_CS stages = 1024 columns); the chunk's own
// power-of-two exponent xe[chunk * xes + row] from its max |c| (scales factor out of each
// chunk's partial Gram, syrk_ksum_kernel applies them per chunk). Rows are split as the
// fp32 values D32 holds. 4 more bytes per entry than the plain centring (the planes).
constexpr int LAP_CS = 32;
__global__ __launch_bounds__(256) void lap_center_split_kernel(double *__restrict__ D, int64_t P, int K,
                                                               const double *__restrict__ mean, float *__restrict__ D32,
                                                               int64_t ld32, uint16_t *__restrict__ planes, int64_t ldh,
                                                               int32_t *__restrict__ xe, int64_t xes) {
    constexpr int CW = LAP_CS * SY_KS;   // 1024 columns
    __shared__ __attribute__((aligned(16))) float cs[CW];
    __shared__ float red4[4];
    const int k = blockIdx.y, tid = threadIdx.x;
    const int64_t z = blockIdx.x, p0 = z * CW;
    float m = 0.0f;
    double dv[CW / 256], mv[CW / 256];
    double *drow = D + (int64_t)k * P;
#pragma unroll
    for (int i = 0; i < CW / 256; ++i) {   // coalesced: consecutive lanes, consecutive columns; all loads first
        const int64_t p = p0 + tid + 256 * i;
        dv[i] = p < P ? drow[p] : 0.0;
        mv[i] = p < P ? mean[p] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < CW / 256; ++i) {
        const int64_t p = p0 + tid + 256 * i;
        float v = 0.0f;
        if (p < P) {
            const double cc = dv[i] - mv[i];
            drow[p] = cc;
            v = (float)cc;
        }
        if (p < ld32) D32[(int64_t)k * ld32 + p] = v;
        cs[tid + 256 * i] = v;
        m = fmaxf(m, fabsf(v));
    }
    m = wave_max(m);
    if ((tid & 63) == 0) red4[tid >> 6] = m;
    __syncthreads();
    const int e = h3_exp(fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3])));
    if (tid == 0) xe[z * xes + k] = e;
    const f32x4 c = *reinterpret_cast<const f32x4 *>(&cs[4 * tid]);   // columns 4 tid .. +3
    u32x2 h, l;
    h3_split4(c, e, h, l);
    u32x2 *o = reinterpret_cast<u32x2 *>(planes + (int64_t)k * 2 * ldh + z * 2 * CW);
    const int q = (tid >> 3) * 16 + (tid & 7);   // stage tid / 8, 4-half piece tid % 8
    o[q] = h;
    o[q + 8] = l;
}

// sum the K-split partial Grams (lower triangle) in split order; write both triangles
__global__ void lap_gram_reduce_kernel(const double *__restrict__ slab, int z, int N, double *__restrict__ G) {
    const int64_t NN = (int64_t)N * N;
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < NN; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = t / N, j = t - i * N;
        if (j > i) continue;
        double v = 0.0;
        for (int q = 0; q < z; ++q) v += slab[q * NN + t];
        G[i * N + j] = v;
        G[j * N + i] = v;
    }
}

// copy the lower triangle onto the upper one, 64 x 64 tiles through LDS
__global__ __launch_bounds__(256) void mirror_kernel(float *__restrict__ G, int N, int64_t ld) {
    __shared__ float t[64][65];
    const int bi = blockIdx.y, bj = blockIdx.x;   // source tile (row block bi >= column block bj)
    if (bj > bi) return;
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int i = bi * 64 + r, j = bj * 64 + tx;
        t[r][tx] = (i < N && j < N) ? G[(int64_t)i * ld + j] : 0.0f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int j = bj * 64 + r, i = bi * 64 + tx;   // destination (j, i), i >= j
        if (i < N && j < N && i > j) G[(int64_t)j * ld + i] = t[tx][r];
    }
}

// the same for the 128 x 128 lower tiles [t0, t0 + gridDim.x) of a tile order:
// (bi, bj) -> (bj, bi), strictly-lower elements only
__global__ __launch_bounds__(256) void mirror_tiles_kernel(float *__restrict__ G, int N, int64_t ld,
                                                           const int2 *__restrict__ tiles, int64_t t0) {
    __shared__ float t[64][65];
    const int2 tb = tiles[t0 + blockIdx.x];
    const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int q = 0; q < 4; ++q) {   // four 64 x 64 quarters of the tile
        const int si = tb.x * 128 + (q >> 1) * 64, sj = tb.y * 128 + (q & 1) * 64;
        if (sj > si) continue;      // upper quarter of a diagonal tile
        __syncthreads();
        for (int r = ty; r < 64; r += 4) {
            const int i = si + r, j = sj + tx;
            t[r][tx] = (i < N && j < N) ? G[(int64_t)i * ld + j] : 0.0f;
        }
        __syncthreads();
        for (int r = ty; r < 64; r += 4) {
            const int j = sj + r, i = si + tx;
            if (i < N && j < N && i > j) G[(int64_t)j * ld + i] = t[tx][r];
        }
    }
}

// shard tiles [t0, t0 + gridDim.x) of G <-> a packed [tile][128][128] buffer
// (unpack also writes the mirrored upper half)
__global__ __launch_bounds__(256) void gram_pack_kernel(const float *__restrict__ G, int N, int64_t ld,
                                                        const int2 *__restrict__ tiles, int64_t t0,
                                                        float *__restrict__ buf) {
    const int2 tb = tiles[t0 + blockIdx.x];
    float *o = buf + (int64_t)blockIdx.x * 128 * 128;
    for (int e = threadIdx.x; e < 128 * 128; e += 256) {
        const int i = tb.x * 128 + (e >> 7), j = tb.y * 128 + (e & 127);
        o[e] = (i < N && j < N) ? G[(int64_t)i * ld + j] : 0.0f;
    }
}
__global__ __launch_bounds__(256) void gram_unpack_kernel(float *__restrict__ G, int N, int64_t ld,
                                                          const int2 *__restrict__ tiles, int64_t t0,
                                                          const float *__restrict__ buf) {
    const int2 tb = tiles[t0 + blockIdx.x];
    const float *p = buf + (int64_t)blockIdx.x * 128 * 128;
    for (int e = threadIdx.x; e < 128 * 128; e += 256) {
        const int i = tb.x * 128 + (e >> 7), j = tb.y * 128 + (e & 127);
        if (i < N && j < N && j <= i) {
            const float v = p[e];
            G[(int64_t)i * ld + j] = v;
            G[(int64_t)j * ld + i] = v;
        }
    }
}

__global__ void iota_kernel(int64_t *__restrict__ v, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = i;
}

// Jacobian rows packed -> Flux order
__global__ void jac_permute_kernel(const float *__restrict__ Jp, int64_t ldp, const int32_t *__restrict__ perm,
                                   int64_t P, int64_t n, float *__restrict__ J) {
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * P; t += (int64_t)gridDim.x * blockDim.x) {
        const int64_t s = t / P, i = t - s * P;
        J[s * P + perm[i]] = Jp[s * ldp + i];
    }
}

// The Gram's tile orders. The K-split Jacobian Gram (syrk_h3k_kernel) works on
// 256 x 256 lower-triangle tiles in supertile order: groups of 8 block rows x 4
// block columns, so the 32 workgroups an XCD runs at once share 8 + 4 row panels
// in its L2 instead of 1 + 32 in plain row-major order. Shards are contiguous runs
// of that order. Everything that works on 128 x 128 tiles (the Dense-term pass,
// the round-5 kernel, gather / pack, the D'D slab Gram) uses the same order with
// each 256-tile expanded into its 128-subtiles (three on the diagonal), so a
// shard's 128-tiles are exactly its 256-tiles' area. One device table per N, kept.
// Round 5 measured a chip-wide order (the 8 XCDs of a dispatch round on one 16 x 16 block,
// sharing its panels in the Infinity Cache; tools/syrk_lab.hip order 1): 7 % faster on rows
// with 40 % zeros (505 -> 473 ms, the clock 1.73 -> 1.80 GHz), but 3 % slower on dense rows
// like the D(50k) Jacobian's (525 -> 541 ms at 1.5 GHz, gpurun_out r05j): with dense operands
// the matrix cores' own power holds the clock down, not the HBM stream. Not kept.
static std::vector<int2> gram256_order_host(int64_t N) {
    const int T = (int)ceil_div(N, SK_T);
    std::vector<int2> t;
    t.reserve((size_t)T * (T + 1) / 2);
    constexpr int SI = 8, SJ = 4;
    for (int i0 = 0; i0 < T; i0 += SI)
        for (int j0 = 0; j0 <= std::min(T - 1, i0 + SI - 1); j0 += SJ)
            for (int i = i0; i < std::min(T, i0 + SI); ++i)
                for (int j = j0; j < std::min(j0 + SJ, i + 1); ++j) t.push_back(int2{i, j});
    SNK_CHECK((int64_t)t.size() == (int64_t)T * (T + 1) / 2, SNK_ERR_INTERNAL, "gram tile order");
    return t;
}
// the 128-subtiles (i, j <= i) of 256-tile u, in a fixed order
static int expand256(int2 u, int T128, int2 *out) {
    int c = 0;
    for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) {
            const int i = 2 * u.x + a, j = 2 * u.y + b;
            if (i < T128 && j <= i) out[c++] = int2{i, j};
        }
    return c;
}
static std::vector<int2> syrk_tile_order_host(int N) {
    const int T = (int)ceil_div(N, SY_T);
    std::vector<int2> t;
    t.reserve((size_t)T * (T + 1) / 2);
    for (const int2 u : gram256_order_host(N)) {
        int2 s[4];
        const int c = expand256(u, T, s);
        t.insert(t.end(), s, s + c);
    }
    SNK_CHECK((int64_t)t.size() == (int64_t)T * (T + 1) / 2, SNK_ERR_INTERNAL, "syrk tile order");
    return t;
}
static const int2 *syrk_tile_order(int N) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<int, int>, int2 *>> cache;   // (N, device) -> table
    int dev = 0;
    SNK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    for (auto &c : cache)
        if (c.first.first == N && c.first.second == dev) return c.second;
    const std::vector<int2> t = syrk_tile_order_host(N);
    int2 *d = nullptr;
    SNK_HIP(hipMalloc(&d, t.size() * sizeof(int2)));
    SNK_HIP(hipMemcpy(d, t.data(), t.size() * sizeof(int2), hipMemcpyHostToDevice));
    cache.emplace_back(std::make_pair(N, dev), d);
    return d;
}

// shard `rank` of `nranks`: the run [u0, u1) of the 256-tile order, proportional cuts
// rounded to the nearest tile (contiguous runs: each shard keeps its L2 locality)
static void gram256_range(int64_t N, int rank, int nranks, int64_t &u0, int64_t &u1) {
    const int64_t T = ceil_div(N, SK_T), tot = T * (T + 1) / 2;
    auto cut = [&](int r) { return (tot * r + nranks / 2) / nranks; };
    u0 = cut(rank);
    u1 = cut(rank + 1);
}
// the same shard as 128-tiles [t0, t1) of syrk_tile_order(N)
static void gram_tile_range(int64_t N, int rank, int nranks, int64_t &t0, int64_t &t1) {
    int64_t u0, u1;
    gram256_range(N, rank, nranks, u0, u1);
    const int T128 = (int)ceil_div(N, SY_T);
    const std::vector<int2> o = gram256_order_host(N);
    int64_t c = 0;
    t0 = t1 = 0;
    for (int64_t u = 0; u <= (int64_t)o.size(); ++u) {
        if (u == u0) t0 = c;
        if (u == u1) {
            t1 = c;
            break;
        }
        int2 s[4];
        c += expand256(o[u], T128, s);
    }
}

// The K-split Gram's per-launch tables (one set per N, device, shard and chunk length,
// kept): the shard's 256-tiles by local index, and one item (I, J, z, local tile) per
// workgroup. Items run over consecutive groups of 32 tiles (about one supertile) and, inside
// a group, chunk-major, so the workgroups an XCD runs together share the group's panels at
// the same k; the list is dealt to the 8 XCD queues in contiguous runs and interleaved
// (workgroup w runs on XCD w % 8).
struct KSplitTables {
    int64_t N, u0, u1;
    int dev, nst, cs;
    int2 *tiles;
    int4 *items;
    int64_t nitems;
};
static const KSplitTables &ksplit_tables(int64_t N, int64_t u0, int64_t u1, int nst, int cs) {
    static std::mutex mu;
    static std::deque<KSplitTables> cache;   // references stay valid as it grows
    int dev = 0;
    SNK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    for (auto &c : cache)
        if (c.N == N && c.u0 == u0 && c.u1 == u1 && c.dev == dev && c.nst == nst && c.cs == cs) return c;
    const std::vector<int2> o = gram256_order_host(N);
    const std::vector<int2> tiles(o.begin() + u0, o.begin() + u1);
    const int S = (int)ceil_div(nst, cs), ntl = (int)tiles.size();
    std::vector<int4> list;
    list.reserve((size_t)ntl * S);
    for (int g0 = 0; g0 < ntl; g0 += 32)
        for (int z = 0; z < S; ++z)
            for (int t = g0; t < std::min(ntl, g0 + 32); ++t) list.push_back(int4{tiles[t].x, tiles[t].y, z, t});
    const size_t L = list.size();
    std::vector<int4> items;
    items.reserve(L);
    size_t qb[9];
    for (int x = 0; x <= 8; ++x) qb[x] = L * x / 8;
    for (size_t j = 0; j < qb[1] - qb[0] + 1; ++j)
        for (int x = 0; x < 8; ++x)
            if (qb[x] + j < qb[x + 1]) items.push_back(list[qb[x] + j]);
    SNK_CHECK(items.size() == L, SNK_ERR_INTERNAL, "k-split item table");
    KSplitTables k{N, u0, u1, dev, nst, cs, nullptr, nullptr, (int64_t)L};
    SNK_HIP(hipMalloc(&k.tiles, std::max<size_t>(tiles.size(), 1) * sizeof(int2)));
    SNK_HIP(hipMalloc(&k.items, std::max<size_t>(L, 1) * sizeof(int4)));
    if (!tiles.empty()) SNK_HIP(hipMemcpy(k.tiles, tiles.data(), tiles.size() * sizeof(int2), hipMemcpyHostToDevice));
    if (L) SNK_HIP(hipMemcpy(k.items, items.data(), L * sizeof(int4), hipMemcpyHostToDevice));
    cache.push_back(k);
    return cache.back();
}

static void syrk_launch(int out, const SyrkArgs &a0, int z, hipStream_t s, int rank = 0, int nranks = 1) {
    SyrkArgs a = a0;
    int64_t t1 = 0;
    gram_tile_range(a.N, rank, nranks, a.t0, t1);
    a.ntiles = t1 - a.t0;
    a.tiles = syrk_tile_order(a.N);   // XCD-aware supertile order (through syrk_xcd_remap)
    if (a.ntiles == 0) return;
    SNK_CHECK(a.K % 4 == 0 && a.ld % 4 == 0 && a.kchunk % 4 == 0, SNK_ERR_INTERNAL, "syrk: K/ld not multiples of 4");
    SNK_CHECK(a.ntiles < (int64_t)1 << 31 && z <= 65535, SNK_ERR_INVALID, "syrk: problem too large");
    dim3 grid((unsigned)a.ntiles, (unsigned)z);
    if (a.xh) {   // pre-split rows (h3): fp16 parts, 3 products per fp32 product
        SNK_CHECK(out == SYRK_F32 && z == 1 && a.ldh % SY_KS == 0 && a.xe, SNK_ERR_INTERNAL, "syrk h3 arguments");
        // production: syrk_h3q_kernel (v_mfma_f32_16x16x32_f16); SNK_ARITH_SYRK_H3_32 selects
        // the round-2 32x32x16 kernel (same results class, parity-tested)
        const bool h3_32 = arith(SNK_ARITH_SYRK_H3_32) != 0;
#ifdef SNK_SYRK_MEASURE
        // measurement build only (make measure: libsnakehip_measure.so, never shipped):
        // SNK_SYRK_VAR = 1 / 2 run the kernel without MFMAs / without stage DMAs, i.e.
        // WRONG results by design (snk_syrk.hpp)
        static const int var = getenv("SNK_SYRK_VAR") ? atoi(getenv("SNK_SYRK_VAR")) : 0;
#else
        constexpr int var = 0;
#endif
        if (!h3_32) {
#ifdef SNK_SYRK_MEASURE
            if (var == 1) syrk_h3q_kernel<1><<<grid, 512, 0, s>>>(a);
            else if (var == 2) syrk_h3q_kernel<2><<<grid, 512, 0, s>>>(a);
            else
#endif
                syrk_h3q_kernel<0><<<grid, 512, 0, s>>>(a);
        } else {
#ifdef SNK_SYRK_MEASURE
            if (var == 1) syrk_h3_kernel<8, 1><<<grid, 512, 0, s>>>(a);
            else if (var == 2) syrk_h3_kernel<8, 2><<<grid, 512, 0, s>>>(a);
            else
#endif
                syrk_h3_kernel<8><<<grid, 512, 0, s>>>(a);
        }
        (void)var;
    } else {      // D'D: fp32 rows, bf16 x6 split in the kernel, one fp64 slab per z
        SNK_CHECK(out == SYRK_SLAB64 && a.g64, SNK_ERR_INTERNAL, "syrk: fp32 rows only for the slab Gram");
        syrk_slab_kernel<<<grid, 256, 0, s>>>(a);
    }
    launch_check("syrk_kernel");
}

// G += the Dense-section Gram terms (syrk_h3q_kernel<0, 4, true>) over the
// lower-triangle tiles of shard rank / nranks
static void syrk_dense_launch(const SyrkArgs &a0, hipStream_t s, int rank, int nranks) {
    SyrkArgs a = a0;
    int64_t t1 = 0;
    gram_tile_range(a.N, rank, nranks, a.t0, t1);
    a.ntiles = t1 - a.t0;
    a.tiles = syrk_tile_order(a.N);
    if (a.ntiles == 0) return;
    SNK_CHECK(a.xh && a.xe && a.act && a.g32 && a.ldh % SY_KS == 0 && 0 < a.s1 && a.s1 < a.s2 &&
                  a.s2 < a.ldh / SY_KS && a.xes >= a.N,
              SNK_ERR_INTERNAL, "syrk dense arguments");
    SNK_CHECK(a.ntiles < (int64_t)1 << 31, SNK_ERR_INVALID, "syrk: problem too large");
    syrk_h3q_kernel<0, 4, true><<<dim3((unsigned)a.ntiles), 512, 0, s>>>(a);
    launch_check("syrk_h3q_kernel<dense>");
}

// make sure the dqn's Jacobian workspace holds n samples (and a Jacobian
// buffer of floats elements)
static void jac_ensure(snk_dqn_s *h, int64_t n, int64_t floats) {
    qwork_ensure(h->jw, h->L, n, true);
    if (n > h->jn_cap) {
        (void)hipStreamSynchronize(stream());
        dfree(h->jidx);
        dfree(h->jact);
        h->jidx = dalloc<int64_t>(n);
        h->jact = dalloc<uint8_t>(n);
        h->jn_cap = n;
        iota_kernel<<<ceil_div(n, 256), 256, 0, stream()>>>(h->jidx, n);
        launch_check("iota_kernel");
    }
    if (floats > h->jbuf_floats) {
        (void)hipStreamSynchronize(stream());
        dfree(h->jbuf);
        h->jbuf = dalloc<float>(floats);
        h->jbuf_floats = floats;
        // pad columns of the conv Jacobian stay zero
        SNK_HIP(hipMemsetAsync(h->jbuf, 0, (size_t)floats * 4, stream()));
    }
}

}  // namespace snk

using namespace snk;

// the K-split snapshot Gram's operand planes and exponents (allocated once; rows K..kpad zero)
static void lap_planes_ensure(snk_laplace h, hipStream_t s) {
    const int64_t ldh = ceil_div(h->ld32, LAP_CS * SY_KS) * (LAP_CS * SY_KS), kpad = ceil_div(h->K, SK_T) * SK_T;
    const int64_t nch = ldh / (LAP_CS * SY_KS);
    SNK_CHECK(nch <= 65535 && h->K <= 65535, SNK_ERR_INVALID, "snapshot Gram too large");
    if (h->planes && h->ldh == ldh) return;
    SNK_HIP(hipStreamSynchronize(s));
    dfree(h->planes);
    dfree(h->pexp);
    h->planes = dalloc<uint16_t>(kpad * 2 * ldh);
    h->pexp = dalloc<int32_t>(nch * h->K);
    h->ldh = ldh;
    SNK_HIP(hipMemsetAsync(h->planes, 0, (size_t)kpad * 2 * ldh * 2, s));
}

extern "C" int snk_laplace_create(snk_laplace *out, int64_t P, int32_t K) {
    return guard([&] {
        SNK_CHECK(out && P > 0 && K > 0, SNK_ERR_INVALID, "bad Laplace geometry P=%lld K=%d", (long long)P, K);
        auto *h = new snk_laplace_s;
        h->P = P;
        h->K = K;
        h->ld32 = (P + 3) & ~int64_t(3);
        h->D = dalloc<double>((size_t)K * P);
        h->mean = dalloc<double>(P);
        h->var = dalloc<double>(P);
        h->G = dalloc<double>((size_t)K * K);
        h->D32 = dalloc<float>((size_t)K * h->ld32);
        SNK_HIP(hipMemsetAsync(h->D, 0, (size_t)K * P * 8, stream()));   // zeros(Float64, (P, K))
        if (arith(SNK_ARITH_SYRK_KSPLIT)) lap_planes_ensure(h, stream());  // the K-split Gram's operand planes
        SNK_HIP(hipStreamSynchronize(stream()));
        *out = h;
    });
}

extern "C" int snk_laplace_destroy(snk_laplace h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        for (void *p : {(void *)h->D, (void *)h->mean, (void *)h->var, (void *)h->G, (void *)h->slab, (void *)h->D32,
                        (void *)h->planes, (void *)h->pexp, (void *)h->gpart})
            dfree(p);
        delete h;
    });
}

extern "C" int snk_laplace_snapshot(snk_laplace h, snk_dqn m, int32_t pos) {
    return guard([&] {
        SNK_CHECK(h && m, SNK_ERR_INVALID, "NULL argument");
        SNK_CHECK(m->L.P == h->P, SNK_ERR_INVALID, "model has %lld params, D has %lld", (long long)m->L.P,
                  (long long)h->P);
        SNK_CHECK(pos >= 0 && pos < h->K, SNK_ERR_INVALID, "snapshot position %d outside 0..%d", pos, h->K - 1);
        lap_snapshot_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->P, 256), 2048), 256, 0, stream()>>>(
            m->theta_q, m->perm, h->P, h->D + (int64_t)pos * h->P);
        launch_check("lap_snapshot_kernel");
    });
}

extern "C" int snk_laplace_set_column(snk_laplace h, int32_t pos, const double *col_host) {
    return guard([&] {
        SNK_CHECK(h && col_host, SNK_ERR_INVALID, "NULL argument");
        SNK_CHECK(pos >= 0 && pos < h->K, SNK_ERR_INVALID, "column %d outside 0..%d", pos, h->K - 1);
        SNK_HIP(hipMemcpyAsync(h->D + (int64_t)pos * h->P, col_host, h->P * 8, hipMemcpyHostToDevice, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

static void lap_buf(snk_laplace h, int32_t which, void **p, int64_t *bytes, int64_t *ld) {
    switch (which) {
        case SNK_LAP_D: *p = h->D; *bytes = (int64_t)h->K * h->P * 8; *ld = h->P; return;
        case SNK_LAP_MEAN: *p = h->mean; *bytes = h->P * 8; *ld = h->P; return;
        case SNK_LAP_VAR: *p = h->var; *bytes = h->P * 8; *ld = h->P; return;
        case SNK_LAP_GRAM: *p = h->G; *bytes = (int64_t)h->K * h->K * 8; *ld = h->K; return;
        case SNK_LAP_D32: *p = h->D32; *bytes = (int64_t)h->K * h->ld32 * 4; *ld = h->ld32; return;
    }
    SNK_CHECK(false, SNK_ERR_INVALID, "bad Laplace buffer selector %d", which);
}

extern "C" int snk_laplace_get(snk_laplace h, int32_t which, void *host, int64_t bytes) {
    return guard([&] {
        SNK_CHECK(h && host, SNK_ERR_INVALID, "NULL argument");
        void *p;
        int64_t nb, ld;
        lap_buf(h, which, &p, &nb, &ld);
        SNK_CHECK(bytes <= nb, SNK_ERR_INVALID, "requested %lld bytes of a %lld-byte buffer", (long long)bytes,
                  (long long)nb);
        SNK_HIP(hipMemcpyAsync(host, p, bytes, hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_laplace_buffer_ptr(snk_laplace h, int32_t which, void **dev_out, int64_t *ld_out) {
    return guard([&] {
        SNK_CHECK(h && dev_out, SNK_ERR_INVALID, "NULL argument");
        int64_t nb, ld;
        lap_buf(h, which, dev_out, &nb, &ld);
        if (ld_out) *ld_out = ld;
    });
}

extern "C" int snk_laplace_fit_center(snk_laplace h) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        hipStream_t s = stream();
        lap_welford_kernel<<<ceil_div(h->P, 256), 256, 0, s>>>(h->D, h->P, h->K, h->mean, h->var);
        launch_check("lap_welford_kernel");
        h->planes_valid = 0;
        if (arith(SNK_ARITH_SYRK_KSPLIT)) {   // centring + fp32 copy + the h3 planes of the snapshot Gram
            lap_planes_ensure(h, s);
            const int64_t ldh = h->ldh, nch = ldh / (LAP_CS * SY_KS);
            lap_center_split_kernel<<<dim3((unsigned)nch, (unsigned)h->K), 256, 0, s>>>(
                h->D, h->P, h->K, h->mean, h->D32, h->ld32, h->planes, ldh, h->pexp, h->K);
            launch_check("lap_center_split_kernel");
            h->planes_valid = 1;
        } else {
            lap_center_kernel<<<(unsigned)std::min<int64_t>(ceil_div((int64_t)h->K * h->ld32, 256), 16384), 256, 0, s>>>(
                h->D, h->P, h->K, h->mean, h->D32, h->ld32);
            launch_check("lap_center_kernel");
        }
    });
}

extern "C" int snk_laplace_gram(snk_laplace h, float *ms_out) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        hipStream_t s = stream();
        if (arith(SNK_ARITH_SYRK_KSPLIT) && h->planes_valid) {
            // the h3 K-split Gram over the planes fit_center split (chunks of LAP_CS stages, one
            // exponent per row and chunk), the chunk partials summed in fp64 into G (both triangles)
            const int nst = (int)(h->ldh / SY_KS), S = nst / LAP_CS;
            const int64_t T = ceil_div(h->K, SK_T), ntl = T * (T + 1) / 2;
            const KSplitTables &kt = ksplit_tables(h->K, 0, ntl, nst, LAP_CS);
            const int64_t need = (int64_t)S * ntl * SK_T * SK_T;
            if (need > h->gpart_floats) {
                SNK_HIP(hipStreamSynchronize(s));
                dfree(h->gpart);
                h->gpart = dalloc<float>(need);
                h->gpart_floats = need;
            }
            SNK_CHECK(kt.nitems < (int64_t)1 << 31 && (int64_t)SK_T * 2 * h->ldh * 2 < (int64_t)1 << 31,
                      SNK_ERR_INVALID, "snapshot Gram too large");
            hipEvent_t e0 = nullptr, e1 = nullptr;
            if (ms_out) {
                SNK_HIP(hipEventCreate(&e0));
                SNK_HIP(hipEventCreate(&e1));
                SNK_HIP(hipEventRecord(e0, s));
            }
            SyrkKArgs k{};
            k.xh = h->planes; k.ldh = h->ldh; k.nst = nst; k.cs = LAP_CS; k.items = kt.items; k.part = h->gpart;
            k.ntl = ntl;
            syrk_h3k_kernel<<<(unsigned)kt.nitems, 512, 0, s>>>(k);
            launch_check("syrk_h3k_kernel");
            if (ms_out) SNK_HIP(hipEventRecord(e1, s));
            SyrkSumArgs<double> q{};
            q.part = h->gpart; q.S = S; q.ntl = ntl; q.tiles = kt.tiles; q.xe = h->pexp; q.xes = h->K; q.N = h->K;
            q.G = h->G; q.ldg = h->K; q.dense = 0;
            syrk_ksum_kernel<double><<<(unsigned)(ntl * 64), 256, 0, s>>>(q);
            launch_check("syrk_ksum_kernel");
            if (ms_out) {
                SNK_HIP(hipEventSynchronize(e1));
                SNK_HIP(hipEventElapsedTime(ms_out, e0, e1));
                (void)hipEventDestroy(e0);
                (void)hipEventDestroy(e1);
            }
            return;
        }
        const int64_t T = ceil_div(h->K, SY_T), tiles = T * (T + 1) / 2;
        // split the P reduction so the launch holds ~2 workgroups per CU
        int z = (int)std::max<int64_t>(1, std::min<int64_t>(ceil_div(512, tiles), ceil_div(h->ld32, 4096)));
        int64_t kchunk = (ceil_div(h->ld32, z) + 31) & ~int64_t(31);
        z = ceil_div(h->ld32, kchunk);
        const int64_t need = (int64_t)z * h->K * h->K;
        if (need > h->slab_cap) {
            (void)hipStreamSynchronize(s);
            dfree(h->slab);
            h->slab = dalloc<double>(need);
            h->slab_cap = need;
        }
        SyrkArgs a{};
        a.x = h->D32; a.ld = h->ld32; a.K = h->ld32; a.kchunk = kchunk; a.N = h->K; a.g64 = h->slab;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (ms_out) {
            SNK_HIP(hipEventCreate(&e0));
            SNK_HIP(hipEventCreate(&e1));
            SNK_HIP(hipEventRecord(e0, s));
        }
        syrk_launch(SYRK_SLAB64, a, z, s);
        if (ms_out) SNK_HIP(hipEventRecord(e1, s));
        lap_gram_reduce_kernel<<<(unsigned)std::min<int64_t>(ceil_div((int64_t)h->K * h->K, 256), 8192), 256, 0, s>>>(
            h->slab, z, h->K, h->G);
        launch_check("lap_gram_reduce_kernel");
        if (ms_out) {
            SNK_HIP(hipEventSynchronize(e1));
            SNK_HIP(hipEventElapsedTime(ms_out, e0, e1));
            (void)hipEventDestroy(e0);
            (void)hipEventDestroy(e1);
        }
    });
}

extern "C" int snk_jacobian(snk_dqn m, snk_replay rb, const int64_t *slots_dev, int64_t n, float *J_dev) {
    return guard([&] {
        SNK_CHECK(m && rb && J_dev && n > 0, SNK_ERR_INVALID, "bad argument");
        SNK_CHECK(!m->deep, SNK_ERR_INVALID, "deep net: per-sample Jacobians are not supported");
        const ReplayDev &R = replay_dev(rb);
        SNK_CHECK(R.bs == m->L.bs && R.C == m->L.C, SNK_ERR_INVALID, "replay geometry differs from the model");
        int64_t len = 0;
        if (snk_replay_length(rb, &len) != SNK_OK) throw Error{SNK_ERR_HIP};
        SNK_CHECK(slots_dev || n <= len, SNK_ERR_STATE, "n=%lld exceeds the %lld stored transitions", (long long)n,
                  (long long)len);
        const QLayout &L = m->L;
        const int64_t ldp = (L.P + 3) & ~int64_t(3);
        jac_ensure(m, n, n * ldp);
        hipStream_t s = stream();
        const int64_t *idx = slots_dev ? slots_dev : m->jidx;
        qnet_jacobian(L, m->theta_q, m->wt_q, src_replay(R, idx, 0), R.act, idx, n, m->jw, m->jact, m->jbuf, ldp,
                      true, s);
        jac_permute_kernel<<<4096, 256, 0, s>>>(m->jbuf, ldp, m->perm, L.P, n, J_dev);
        launch_check("jac_permute_kernel");
        SNK_HIP(hipStreamSynchronize(s));
    });
}

// G = J J' tiles of shard rank / nranks (all: 0 / 1), mirrored; the Jacobian
// rows of all n samples are computed by every shard (29 ms at 50k)
static void jacobian_gram_tiles(snk_dqn m, snk_replay rb, int64_t n, float *G_dev, float *ms_out, int rank,
                                int nranks) {
    {
        SNK_CHECK(m && rb && G_dev && n > 0 && nranks >= 1 && rank >= 0 && rank < nranks, SNK_ERR_INVALID,
                  "bad argument");
        SNK_CHECK(!m->deep, SNK_ERR_INVALID, "deep net: the Jacobian Gram is not supported");
        const ReplayDev &R = replay_dev(rb);
        SNK_CHECK(R.bs == m->L.bs && R.C == m->L.C, SNK_ERR_INVALID, "replay geometry differs from the model");
        int64_t len = 0;
        if (snk_replay_length(rb, &len) != SNK_OK) throw Error{SNK_ERR_HIP};
        SNK_CHECK(n <= len, SNK_ERR_STATE, "n=%lld exceeds the %lld stored transitions", (long long)n, (long long)len);
        const QLayout &L = m->L;
        const int64_t Kc = (L.off_d1w + 3) & ~int64_t(3);   // conv sections of a Jacobian row
        jac_ensure(m, n, n * Kc);
        hipStream_t s = stream();
        hipEvent_t ev[5] = {};
        if (ms_out)
            for (auto &e : ev) SNK_HIP(hipEventCreate(&e));
        if (ms_out) SNK_HIP(hipEventRecord(ev[0], s));
        qnet_jacobian(L, m->theta_q, m->wt_q, src_replay(R, m->jidx, 0), R.act, m->jidx, n, m->jw, m->jact, m->jbuf,
                      Kc, false, s, ms_out ? ev[1] : nullptr);
        if (ms_out) SNK_HIP(hipEventRecord(ev[2], s));
        // round 6 (SNK_ARITH_SYRK_KSPLIT, default): the conv-column Gram on syrk_h3k_kernel
        // (256 x 256 tiles, fp32 partial Grams per chunk of SK_CHUNK stages), then the
        // Dense-section pass STORES its terms into G's lower triangle and syrk_ksum_kernel
        // adds the chunk sums (fp64) to them and writes both triangles (no mirror pass);
        // 0: the round-5 syrk_h3q_kernel, the Dense terms added into G, then the mirror
        const bool ksplit = arith(SNK_ARITH_SYRK_KSPLIT) != 0;
        SyrkArgs a{};
        a.x = m->jbuf; a.ld = Kc; a.K = Kc; a.kchunk = Kc; a.N = (int)n; a.g32 = G_dev; a.ldg = n;
        int64_t ldh = 0;
        {   // h3 Gram: rows pre-split once into scaled fp16 planes (snk_syrk.hpp h3_rows_kernel)
            ldh = (Kc + SY_KS - 1) / SY_KS * SY_KS;
            const int64_t npad = (n + SW_ROWS_B - 1) / SW_ROWS_B * SW_ROWS_B;   // zero rows past n (whole row blocks)
            if (2 * npad * ldh > m->jplanes_halves) {
                (void)hipStreamSynchronize(s);
                dfree(m->jplanes);
                m->jplanes = dalloc<uint16_t>(2 * npad * ldh);
                m->jplanes_halves = 2 * npad * ldh;
            }
            if (npad > n)
                SNK_HIP(hipMemsetAsync(m->jplanes + 2 * n * ldh, 0, (size_t)(npad - n) * 2 * ldh * sizeof(uint16_t), s));
            if (n > m->jexp_cap) {
                (void)hipStreamSynchronize(s);
                dfree(m->jexp);
                m->jexp = dalloc<int32_t>(n);
                m->jexp_cap = n;
            }
            h3_rows_kernel<<<(unsigned)n, 256, 0, s>>>(m->jbuf, Kc, Kc, m->jplanes, m->jexp, ldh);
            launch_check("h3_rows_kernel");
            a.xh = m->jplanes; a.xe = m->jexp; a.ldh = ldh;
        }
        int64_t u0 = 0, u1 = 0;
        const KSplitTables *kt = nullptr;
        if (ksplit) {
            gram256_range(n, rank, nranks, u0, u1);
            const int nst = (int)(ldh / SY_KS);
            kt = &ksplit_tables(n, u0, u1, nst, SK_CHUNK);
            const int64_t ntl = u1 - u0, S = ceil_div(nst, SK_CHUNK), need = S * ntl * SK_T * SK_T;
            if (need > m->gpart_floats) {
                (void)hipStreamSynchronize(s);
                dfree(m->gpart);
                m->gpart = dalloc<float>(need);
                m->gpart_floats = need;
            }
            if (kt->nitems) {
                SNK_CHECK(kt->nitems < (int64_t)1 << 31, SNK_ERR_INVALID, "syrk: problem too large");
                SNK_CHECK((int64_t)SK_T * 2 * ldh * 2 < (int64_t)1 << 31, SNK_ERR_INVALID, "syrk: rows too long");
                SyrkKArgs k{};
                k.xh = m->jplanes; k.ldh = ldh; k.nst = nst; k.cs = SK_CHUNK; k.items = kt->items; k.part = m->gpart;
                k.ntl = ntl;
                syrk_h3k_kernel<<<(unsigned)kt->nitems, 512, 0, s>>>(k);
                launch_check("syrk_h3k_kernel");
            }
        } else {
            syrk_launch(SYRK_F32, a, 1, s, rank, nranks);
        }
        if (ms_out) SNK_HIP(hipEventRecord(ev[3], s));
        {   // Dense-section terms: a3 | dz1 | h1 pre-split into h3 segments, one DENSE h3q pass
            const int64_t st1 = ceil_div(L.K1, SY_KS), st2 = st1 + 64 / SY_KS, ldd = (st2 + 64 / SY_KS) * SY_KS;
            const int64_t npad = (n + SW_ROWS_B - 1) / SW_ROWS_B * SW_ROWS_B;
            SNK_CHECK(L.K1 % 4 == 0, SNK_ERR_INTERNAL, "Dense1 fan-in not a multiple of 4");
            if (2 * npad * ldd > m->dplanes_halves) {
                (void)hipStreamSynchronize(s);
                dfree(m->dplanes);
                m->dplanes = dalloc<uint16_t>(2 * npad * ldd);
                m->dplanes_halves = 2 * npad * ldd;
            }
            if (n > m->dexp_cap) {
                (void)hipStreamSynchronize(s);
                dfree(m->dexp);
                m->dexp = dalloc<int32_t>(3 * n);
                m->dexp_cap = n;
            }
            H3Segs sg{};
            sg.x[0] = m->jw.a3; sg.x[1] = m->jw.dz1; sg.x[2] = m->jw.h1;
            sg.ld[0] = sg.K[0] = L.K1; sg.ld[1] = sg.K[1] = sg.ld[2] = sg.K[2] = 64;
            sg.st[0] = 0; sg.st[1] = st1; sg.st[2] = st2;
            sg.nst[0] = st1; sg.nst[1] = sg.nst[2] = 64 / SY_KS;
            h3_seg_rows_kernel<<<dim3((unsigned)ceil_div(npad, 4), 3), 256, 0, s>>>(sg, n, npad, m->dplanes, m->dexp,
                                                                                   m->dexp_cap, ldd);
            launch_check("h3_seg_rows_kernel");
            SyrkArgs d{};
            d.xh = m->dplanes; d.xe = m->dexp; d.xes = m->dexp_cap; d.ldh = ldd; d.s1 = (int)st1; d.s2 = (int)st2;
            d.N = (int)n; d.g32 = G_dev; d.ldg = n; d.act = m->jact; d.dstore = ksplit ? 1 : 0;
            syrk_dense_launch(d, s, rank, nranks);
        }
        if (ksplit) {
            if (u1 > u0) {
                SyrkSumArgs<float> q{};
                q.part = m->gpart; q.S = (int)ceil_div(ldh / SY_KS, SK_CHUNK); q.ntl = u1 - u0; q.tiles = kt->tiles;
                q.xe = m->jexp; q.xes = 0; q.N = (int)n; q.G = G_dev; q.ldg = n; q.dense = 1;
                syrk_ksum_kernel<float><<<(unsigned)((u1 - u0) * 64), 256, 0, s>>>(q);
                launch_check("syrk_ksum_kernel");
            }
        } else if (nranks == 1) {
            const unsigned nb = (unsigned)ceil_div(n, 64);
            mirror_kernel<<<dim3(nb, nb), 256, 0, s>>>(G_dev, (int)n, n);
            launch_check("mirror_kernel");
        } else {
            int64_t t0, t1;
            gram_tile_range(n, rank, nranks, t0, t1);
            if (t1 > t0) {
                mirror_tiles_kernel<<<(unsigned)(t1 - t0), 256, 0, s>>>(G_dev, (int)n, n, syrk_tile_order((int)n), t0);
                launch_check("mirror_tiles_kernel");
            }
        }
        if (ms_out) {
            SNK_HIP(hipEventRecord(ev[4], s));
            SNK_HIP(hipEventSynchronize(ev[4]));
            for (int i = 0; i < 4; ++i) SNK_HIP(hipEventElapsedTime(&ms_out[i], ev[i], ev[i + 1]));
            for (auto &e : ev) (void)hipEventDestroy(e);
        } else {
            SNK_HIP(hipStreamSynchronize(s));
        }
    }
}

extern "C" int snk_jacobian_gram(snk_dqn m, snk_replay rb, int64_t n, float *G_dev, float *ms_out) {
    return guard([&] { jacobian_gram_tiles(m, rb, n, G_dev, ms_out, 0, 1); });
}

extern "C" int snk_jacobian_gram_shard(snk_dqn m, snk_replay rb, int64_t n, int32_t rank, int32_t nranks,
                                       float *G_dev, float *ms_out) {
    return guard([&] { jacobian_gram_tiles(m, rb, n, G_dev, ms_out, rank, nranks); });
}

extern "C" int snk_gram_tiles(int64_t n, int32_t rank, int32_t nranks, int32_t *tiles_host, int64_t *count_out) {
    return guard([&] {
        SNK_CHECK(n > 0 && nranks >= 1 && rank >= 0 && rank < nranks && count_out, SNK_ERR_INVALID, "bad argument");
        int64_t t0, t1;
        gram_tile_range(n, rank, nranks, t0, t1);
        *count_out = t1 - t0;
        if (!tiles_host) return;
        const std::vector<int2> order = syrk_tile_order_host((int)n);
        for (int64_t t = t0; t < t1; ++t) {
            tiles_host[2 * (t - t0)] = order[t].x * SY_T;
            tiles_host[2 * (t - t0) + 1] = order[t].y * SY_T;
        }
    });
}

namespace snk {
void comm_gather_to_root(snk_comm h, const float *send, int64_t n_send, float *const *recv, const int64_t *n_recv,
                         int root, hipStream_t s);
int comm_rank(snk_comm h);
int comm_size(snk_comm h);
}

extern "C" int snk_jacobian_gram_gather(snk_comm c, int64_t n, float *G_dev, int32_t root) {
    return guard([&] {
        SNK_CHECK(c && G_dev && n > 0, SNK_ERR_INVALID, "bad argument");
        const int R = comm_size(c), me = comm_rank(c);
        SNK_CHECK(root >= 0 && root < R, SNK_ERR_INVALID, "bad root");
        if (R == 1) return;
        hipStream_t s = stream();
        const int2 *tiles = syrk_tile_order((int)n);
        constexpr int64_t TF = 128 * 128;
        int64_t t0, t1;
        if (me != root) {
            gram_tile_range(n, me, R, t0, t1);
            DevBuf<float> buf((size_t)std::max<int64_t>(t1 - t0, 1) * TF);
            if (t1 > t0) {
                gram_pack_kernel<<<(unsigned)(t1 - t0), 256, 0, s>>>(G_dev, (int)n, n, tiles, t0, buf);
                launch_check("gram_pack_kernel");
            }
            comm_gather_to_root(c, buf, (t1 - t0) * TF, nullptr, nullptr, root, s);
            SNK_HIP(hipStreamSynchronize(s));
            return;
        }
        std::vector<DevBuf<float>> bufs(R);
        std::vector<float *> rp(R, nullptr);
        std::vector<int64_t> rn(R, 0);
        for (int r = 0; r < R; ++r) {
            if (r == root) continue;
            gram_tile_range(n, r, R, t0, t1);
            bufs[r] = DevBuf<float>((size_t)std::max<int64_t>(t1 - t0, 1) * TF);
            rp[r] = bufs[r];
            rn[r] = (t1 - t0) * TF;
        }
        comm_gather_to_root(c, nullptr, 0, rp.data(), rn.data(), root, s);
        for (int r = 0; r < R; ++r) {
            if (r == root) continue;
            gram_tile_range(n, r, R, t0, t1);
            if (t1 > t0) {
                gram_unpack_kernel<<<(unsigned)(t1 - t0), 256, 0, s>>>(G_dev, (int)n, n, tiles, t0, rp[r]);
                launch_check("gram_unpack_kernel");
            }
        }
        SNK_HIP(hipStreamSynchronize(s));
    });
}

// =========================================================================
// Laplace sampling (la_utils.jl:83-118)
//
// sample_model (:83-95): w = mean + 1/sqrt(2) * sqrt.(Gamma) * z1
//                              + 1/sqrt(2(K-1)) * D * z2,   Gamma = Diagonal(|var|)
// with z1 ~ N(0, I_P), z2 ~ N(0, I_K); restructure(w) -> Float32 model.
// laplace_sampling! (:97-118): the greedy (epsilon 0) episode reward of the
// current model, then n_models x (sample_model, greedy play_episode); the
// transitions of every model that beats it are stored into the buffer, in
// model order.
//
// Here the n_models episodes run in LOCKSTEP, one env per sampled model:
//  * lap_sample_kernel builds the models' weights in the packed layout (the
//    Julia expression above in fp64, term by term; z from a counter-based
//    Box-Muller stream indexed by (seed, model, stream, Flux index), so a
//    model's weights do not depend on the chunking);
//  * lap_act_kernel is one workgroup per env running ITS model's whole
//    forward (conv1, conv2 in LDS, conv3 / Dense1 streaming that model's
//    weights, Dense2 + first-max argmax) — the weights differ per env, so
//    the shared-weight MFMA kernels of the training path do not apply; the
//    launch is HBM-bound on ~1.1 MB of weights per live env and step;
//  * the fused env step stores every transition into a scratch ring (slot
//    t * G + g); lap_track_kernel records each env's first episode end
//    (length, Float32 episode reward);
//  * the better models' transitions are appended to the trainer's buffer in
//    (model, step) order by lap_copy_kernel.
// =========================================================================
namespace snk {

__host__ __device__ inline double lap_u01(uint64_t x) { return ((double)(x >> 11) + 0.5) * 0x1.0p-53; }

// z(seed, model, stream, i) ~ N(0, 1): Box-Muller on two splitmix64 draws
__device__ inline double lap_normal(uint64_t seed, uint64_t model, uint32_t stream, uint64_t i) {
    const uint64_t b = rng_hash(seed ^ ((uint64_t)stream << 56), model, i);
    const double u1 = lap_u01(splitmix64(b)), u2 = lap_u01(splitmix64(b ^ 0x9E3779B97F4A7C15ULL));
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

__global__ void lap_normals_kernel(uint64_t seed, uint64_t model, uint32_t stream, int64_t i0, int64_t n,
                                   double *__restrict__ out) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q < n) out[q] = lap_normal(seed, model, stream, (uint64_t)(i0 + q));
}

// W[g][j] (packed index j, Flux index fi = perm[j]) for models n0 .. n0+G-1:
//   w = (mean[fi] + (c1 * sqrt|var[fi]|) * z1(fi)) + sum_k (c2 * D[k][fi]) * z2(k)   (k ascending)
// LAP_GM models per pass keep their gemv sums in registers; z2 of the G models in LDS
constexpr int LAP_GM = 32;   // models per pass: each pass re-reads D (P x K doubles) once
__global__ __launch_bounds__(256) void lap_sample_kernel(const double *__restrict__ mean, const double *__restrict__ var,
                                                         const double *__restrict__ D, int K, int64_t P,
                                                         const int32_t *__restrict__ perm, uint64_t seed, int64_t n0,
                                                         int G, double c1, double c2, float *__restrict__ W,
                                                         int64_t ldw) {
    extern __shared__ double z2s[];   // [G][K]
    for (int q = threadIdx.x; q < G * K; q += blockDim.x) z2s[q] = lap_normal(seed, (uint64_t)(n0 + q / K), 2, q % K);
    __syncthreads();
    for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < P; j += (int64_t)gridDim.x * blockDim.x) {
        const int64_t fi = perm[j];
        const double a = c1 * sqrt(fabs(var[fi]));
        const double m = mean[fi];
        for (int g0 = 0; g0 < G; g0 += LAP_GM) {
            double d[LAP_GM];
#pragma unroll
            for (int u = 0; u < LAP_GM; ++u) d[u] = 0.0;
            for (int k = 0; k < K; ++k) {
                const double dk = c2 * D[(int64_t)k * P + fi];
#pragma unroll
                for (int u = 0; u < LAP_GM; ++u)
                    if (g0 + u < G) d[u] = d[u] + dk * z2s[(g0 + u) * K + k];
            }
#pragma unroll
            for (int u = 0; u < LAP_GM; ++u)
                if (g0 + u < G) {
                    const double w = (m + a * lap_normal(seed, (uint64_t)(n0 + g0 + u), 1, (uint64_t)fi)) + d[u];
                    W[(int64_t)(g0 + u) * ldw + j] = (float)w;
                }
        }
    }
}

// lap_act_kernel's LDS (floats): a front region holding [xin | a1 | w2s] until conv2 is
// done, then the conv3 weight ring, then [a3 | Dense1 partials | h1]; and a2. About 50 KB
// at 12x12: three workgroups (models) per CU.
constexpr int LAP_RING = 4;          // conv3 weight chunks (one kernel offset, 32 x 64 floats) in flight
constexpr int LAP_CH = 32 * 64;
static inline int64_t lap_act_front_floats(const QLayout &L) {
    const int bp = L.bs + 2, r4 = (L.C * bp * bp + 3) & ~3, a4 = (16 * bp * bp + 3) & ~3;
    const int64_t tail = ((int64_t)L.K1 + 16 * 64 + 64 + 8 + 3) & ~int64_t(3);
    return std::max<int64_t>(std::max<int64_t>((int64_t)r4 + a4 + 9 * 16 * 32, (int64_t)LAP_RING * LAP_CH), tail);
}
static inline int64_t lap_act_lds_floats(const QLayout &L) {
    return lap_act_front_floats(L) + (int64_t)L.ncell * 32;
}

// one workgroup (256 threads) per env g: the greedy action of model g on the env's state.
// Latency matters as much as bandwidth here (the episode tail runs a few live models per
// launch): conv3's weights arrive by LDS-DMA through a ring of LAP_RING kernel offsets
// (each weight fetched once, read from LDS by the 16 position groups that share it), and
// Dense1's stream into a register ring three k-steps deep. The FMAs run on v_pk_fma_f32
// (two accumulators per instruction) in the scalar form's per-accumulator order, so every
// output is bit-identical to an fmaf chain over (kk, ci) / k ascending.
__global__ __launch_bounds__(256) void lap_act_kernel(QLayout L, const float *__restrict__ W, int64_t ldw, BoardSrc src,
                                                      const uint8_t *__restrict__ fin, uint8_t *__restrict__ act,
                                                      float *__restrict__ qout, int front) {
    const int64_t g = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (fin && fin[g]) {
        if (tid == 0) act[g] = 0;
        return;
    }
    extern __shared__ __attribute__((aligned(16))) float lsm[];
    const int bs = L.bs, bp = bs + 2, C = L.C, nc = L.ncell, Wo = L.Wo;
    float *xin = lsm;                       // [C][bp*bp] bordered input planes
    float *a1 = xin + ((C * bp * bp + 3) & ~3);   // [16][bp*bp] bordered conv1 output (16-B aligned sections)
    float *w2s = a1 + ((16 * bp * bp + 3) & ~3);  // conv2 weights [(kk*16+ci)*32+co]
    float *ring = lsm;                      // conv3 weight chunks [LAP_RING][32 ci][64 co] (after conv2)
    float *a2 = lsm + front;                // [ncell][32]
    float *a3 = lsm;                        // [Wo*Wo][64] (after conv3: over the ring)
    float *red = a3 + L.K1;                 // [16][64] Dense1 partial sums
    float *h1 = red + 16 * 64;              // [64]
    const float *th = W + g * ldw;
    for (int q = tid; q < (int)(w2s - xin); q += 256) xin[q] = 0.0f;
    for (int q = tid; q < 9 * 16 * 32; q += 256) w2s[q] = th[L.off_w2 + q];
    __syncthreads();
    for (int q = tid; q < C * nc; q += 256) {
        const int c = q / nc, cell = q - c * nc;
        const int jj = cell / bs, ii = cell - jj * bs;
        xin[c * bp * bp + (ii + 1) + (jj + 1) * bp] = src.load(g, c, cell);
    }
    __syncthreads();
    // conv1 (3x3, pad 1): thread -> co = tid & 15, positions (tid >> 4) + 16 r
    {
        const int co = tid & 15;
        const float *w1 = th + L.off_w1;
        const float b = th[L.off_b1 + co];
        for (int p = tid >> 4; p < nc; p += 16) {
            const int j = p / bs, i = p - j * bs;
            float acc = b;
            for (int kk = 0; kk < 9; ++kk) {
                const int du = kk % 3, dv = kk / 3;
                for (int c = 0; c < C; ++c)
                    acc = __builtin_fmaf(xin[c * bp * bp + (i + du) + (j + dv) * bp], w1[(kk * C + c) * 16 + co], acc);
            }
            a1[co * bp * bp + (i + 1) + (j + 1) * bp] = fmaxf(acc, 0.0f);
        }
    }
    __syncthreads();
    // conv2 (3x3, 16 -> 32, pad 1): thread -> output channels 4 (tid & 7) .. +3 at positions
    // (tid >> 3) + 32 r, r < ceil(ncell / 32): per (kk, ci) one ds_read_b128 of four weights and
    // one a1 read per position feed 4 FMAs per position (packed in pairs); every output's
    // FMA chain runs kk, then ci, ascending, as the scalar form
    {
        constexpr int RP = 6;   // positions per thread: ncell <= 32 * RP (board side <= 13)
        const int cq = tid & 7, pg = tid >> 3;
        const f32x4 b4 = *reinterpret_cast<const f32x4 *>(th + L.off_b2 + 4 * cq);
        f32x2 acc[RP][2];
        int pb[RP];
#pragma unroll
        for (int r = 0; r < RP; ++r) {
            const int p = min(pg + 32 * r, nc - 1);
            const int j = p / bs, i = p - j * bs;
            pb[r] = i + j * bp;
            acc[r][0] = f32x2{b4[0], b4[1]};
            acc[r][1] = f32x2{b4[2], b4[3]};
        }
        for (int kk = 0; kk < 9; ++kk) {
            const int koff = kk % 3 + (kk / 3) * bp;
#pragma unroll 2
            for (int ci = 0; ci < 16; ++ci) {
                const f32x4 w = *reinterpret_cast<const f32x4 *>(w2s + (kk * 16 + ci) * 32 + 4 * cq);
                const float *ap = a1 + ci * bp * bp + koff;
#pragma unroll
                for (int r = 0; r < RP; ++r) {
                    const float x = ap[pb[r]];
                    acc[r][0] = __builtin_elementwise_fma(f32x2{x, x}, f32x2{w[0], w[1]}, acc[r][0]);
                    acc[r][1] = __builtin_elementwise_fma(f32x2{x, x}, f32x2{w[2], w[3]}, acc[r][1]);
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RP; ++r) {
            const int p = pg + 32 * r;
            if (p < nc)
                *reinterpret_cast<f32x4 *>(a2 + p * 32 + 4 * cq) =
                    f32x4{fmaxf(acc[r][0][0], 0.f), fmaxf(acc[r][0][1], 0.f), fmaxf(acc[r][1][0], 0.f),
                          fmaxf(acc[r][1][1], 0.f)};
        }
    }
    __syncthreads();   // conv1/conv2 staging free: the conv3 weight ring overlays it
    // conv3 (6x6, 32 -> 64, pad 0): thread -> 4 output channels 4*(tid & 15) .. +3 at
    // positions (tid >> 4) + 16 r, r < 4 (Wo^2 <= 64); chunk kk of the weights (rows
    // (kk, ci), 64 co) lands in ring slot kk % LAP_RING by LDS-DMA (wave w moves rows
    // 8w .. 8w+7: two 1 KB pieces of 16 B per lane)
    {
        const float *w3g = th + L.off_w3;
        auto dma = [&](int kk) __attribute__((always_inline)) {
            const int k = kk < 36 ? kk : 35;   // past the end: harmless reloads (never read)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
                const int piece = wave * 2 + q;   // 256 floats each
                __builtin_amdgcn_global_load_lds((const void *)(w3g + (int64_t)k * LAP_CH + piece * 256 + lane * 4),
                                                 (__attribute__((address_space(3))) void *)(ring + (kk % LAP_RING) * LAP_CH +
                                                                                           piece * 256),
                                                 16, 0, 0);
            }
        };
#pragma unroll
        for (int q = 0; q < LAP_RING - 1; ++q) dma(q);
        const int cq = tid & 15, pg = tid >> 4;
        const int np = Wo * Wo;
        f32x2 acc[4][2];
        int base[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = pg + 16 * r;
            const int pj = p < np ? p / Wo : 0, pi = p < np ? p - pj * Wo : 0;
            base[r] = (pi + pj * bs) * 32;
            acc[r][0] = f32x2{th[L.off_b3 + 4 * cq], th[L.off_b3 + 4 * cq + 1]};
            acc[r][1] = f32x2{th[L.off_b3 + 4 * cq + 2], th[L.off_b3 + 4 * cq + 3]};
        }
        for (int kk = 0; kk < 36; ++kk) {
            // chunk kk landed (this wave's pieces: the LAP_RING - 2 younger chunks stay in
            // flight), every wave's pieces visible after the barrier; the slot of chunk
            // kk - 1, refilled below, was last read before it
            __builtin_amdgcn_s_waitcnt(waitcnt_vm(2 * (LAP_RING - 2)));
            __syncthreads();
            dma(kk + LAP_RING - 1);
            const int du = kk % 6, dv = kk / 6;
            const int off = (du + dv * bs) * 32;
            const float *wk = ring + (kk % LAP_RING) * LAP_CH + 4 * cq;
#pragma unroll 2
            for (int ci = 0; ci < 32; ci += 4) {
                f32x4 w[4], av[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) w[c] = *reinterpret_cast<const f32x4 *>(wk + (ci + c) * 64);
#pragma unroll
                for (int r = 0; r < 4; ++r) av[r] = *reinterpret_cast<const f32x4 *>(a2 + base[r] + off + ci);
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const f32x2 x{av[r][c], av[r][c]};
                        acc[r][0] = __builtin_elementwise_fma(x, f32x2{w[c][0], w[c][1]}, acc[r][0]);
                        acc[r][1] = __builtin_elementwise_fma(x, f32x2{w[c][2], w[c][3]}, acc[r][1]);
                    }
            }
        }
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));   // the clamped tail reloads
        __syncthreads();                              // every wave's ring reads done: a3 overlays the ring
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = pg + 16 * r;
            if (p < np)
                *reinterpret_cast<f32x4 *>(a3 + p * 64 + 4 * cq) =
                    f32x4{fmaxf(acc[r][0][0], 0.f), fmaxf(acc[r][0][1], 0.f), fmaxf(acc[r][1][0], 0.f),
                          fmaxf(acc[r][1][1], 0.f)};
        }
    }
    __syncthreads();
    // Dense1: thread -> 4 outputs 4*(tid & 15) .. +3 over the 16th (tid >> 4) of the
    // K1 inputs (4 at a time: one ds_read_b128, 4 float4 weight loads, 16 FMAs), the
    // weight loads three k-steps ahead in a register ring; then a 16-way reduction in LDS
    {
        const int oq = tid & 15, part = tid >> 4;
        const int kq = (L.K1 / 4 + 15) / 16 * 4, k0 = part * kq, k1 = min(L.K1, k0 + kq);
        const f32x4 *wd = reinterpret_cast<const f32x4 *>(th + L.off_d1w) + oq;   // [k*16 + oq]
        const int n = k1 > k0 ? (k1 - k0) / 4 : 0;
        constexpr int RD = 4;
        f32x4 wr[RD][4];
        auto ld = [&](int i, int slot) __attribute__((always_inline)) {
            const int k = n > 0 ? k0 + 4 * (i < n ? i : n - 1) : 0;   // past the end: reloads (unused)
#pragma unroll
            for (int c = 0; c < 4; ++c) wr[slot][c] = wd[(int64_t)(k + c) * 16];
        };
#pragma unroll
        for (int q = 0; q < RD - 1; ++q) ld(q, q);
        f32x2 acc[2] = {f32x2{0.f, 0.f}, f32x2{0.f, 0.f}};
        for (int i0 = 0; i0 < n; i0 += RD) {
#pragma unroll
            for (int q = 0; q < RD; ++q) {
                const int i = i0 + q;
                ld(i + RD - 1, (q + RD - 1) % RD);
                if (i < n) {
                    const f32x4 a = *reinterpret_cast<const f32x4 *>(a3 + k0 + 4 * i);
#pragma unroll
                    for (int c = 0; c < 4; ++c) {
                        const f32x2 x{a[c], a[c]};
                        acc[0] = __builtin_elementwise_fma(x, f32x2{wr[q][c][0], wr[q][c][1]}, acc[0]);
                        acc[1] = __builtin_elementwise_fma(x, f32x2{wr[q][c][2], wr[q][c][3]}, acc[1]);
                    }
                }
            }
        }
        *reinterpret_cast<f32x4 *>(red + part * 64 + 4 * oq) = f32x4{acc[0][0], acc[0][1], acc[1][0], acc[1][1]};
    }
    __syncthreads();
    if (tid < 64) {
        float h = 0.0f;
#pragma unroll
        for (int q = 0; q < 16; ++q) h += red[q * 64 + tid];
        h1[tid] = fmaxf(th[L.off_d1b + tid] + h, 0.0f);
    }
    __syncthreads();
    if (tid < 64) {   // Dense2 + first-max argmax (utils.jl:165-169)
        float q[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            float v = h1[tid] * th[L.off_d2w + a * 64 + tid];
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
            q[a] = v + th[L.off_d2b + a];
        }
        if (tid == 0) {
            int best = 0;
            if (q[1] > q[best]) best = 1;
            if (q[2] > q[best]) best = 2;
            act[g] = (uint8_t)best;
            if (qout) {
                qout[g * 3] = q[0]; qout[g * 3 + 1] = q[1]; qout[g * 3 + 2] = q[2];
            }
        }
    }
}

// after the step of iteration t: the first episode end of each env
__global__ void lap_track_kernel(const uint8_t *__restrict__ done, const float *__restrict__ ep, int64_t G, int t,
                                 uint8_t *__restrict__ fin, int32_t *__restrict__ len, float *__restrict__ rew,
                                 int32_t *__restrict__ nfin) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= G || fin[g] || !done[g]) return;
    fin[g] = 1;
    len[g] = t + 1;
    rew[g] = ep[g];
    atomicAdd(nfin, 1);
}

// append the listed scratch slots to the destination ring, in list order (store!)
__global__ void lap_copy_kernel(ReplayDev src, ReplayDev dst, const int64_t *__restrict__ slots, int64_t n,
                                int64_t dcount) {
    const int64_t i = blockIdx.x;
    if (i >= n) return;
    const int64_t s = slots[i], d = (dcount + i) % dst.cap;
    const int nb = (src.C + 1) * src.pitch;
    for (int q = threadIdx.x; q < nb; q += blockDim.x) dst.frames[d * nb + q] = src.frames[s * nb + q];
    if (threadIdx.x == 0) {
        dst.reward[d] = src.reward[s];
        dst.act[d] = src.act[s];
        dst.done[d] = src.done[s];
        dst.mask[d] = src.mask[s];
        dst.dirs[d] = src.dirs[s];
    }
}

__global__ void lap_count_add_kernel(int64_t *count, int64_t n) { *count += n; }

}  // namespace snk

// env / scratch replay handles owned by a host scope (freed on the throw path too)
struct EnvHold {
    snk_env e = nullptr;
    ~EnvHold() {
        if (e) snk_env_destroy(e);
    }
};
struct ReplayHold {
    snk_replay r = nullptr;
    ~ReplayHold() {
        if (r) snk_replay_destroy(r);
    }
};

// greedy lockstep episodes of G models whose packed weights are W [G][ldw];
// per-model length / Float32 reward; scratch ring (slot t*G + g) left in sc
static void lap_rollout(snk_dqn m, const float *W, int64_t ldw, int64_t G, float *rew_dev, int32_t *len_dev,
                        EnvHold &env, ReplayHold &sc) {
    const QLayout &L = m->L;
    hipStream_t s = stream();
    const int T = 501;   // the first episode is over by step 500 (utils.jl:88 truncation)
    if (snk_env_create(&env.e, G, L.bs, L.C, 42, 500, 1) != SNK_OK) throw Error{SNK_ERR_HIP};
    if (snk_replay_create(&sc.r, G * T, L.bs, L.C, 1) != SNK_OK) throw Error{SNK_ERR_HIP};
    const EnvDev &E = env_dev(env.e);
    const ReplayDev &R = replay_dev(sc.r);
    DevBuf<uint8_t> fin(G), act(G);
    DevBuf<int32_t> nfin(1);
    SNK_HIP(hipMemsetAsync(fin, 0, G, s));
    SNK_HIP(hipMemsetAsync(nfin, 0, sizeof(int32_t), s));
    SNK_HIP(hipMemsetAsync(len_dev, 0, G * sizeof(int32_t), s));
    const size_t lds = (size_t)lap_act_lds_floats(L) * sizeof(float);
    SNK_CHECK(lds <= 160 * 1024 && L.Wo * L.Wo <= 64 && L.K1 % 4 == 0 && L.off_w3 % 4 == 0 && L.off_d1w % 4 == 0 &&
                  (G == 1 || ldw % 4 == 0) && lap_act_front_floats(L) % 4 == 0 && L.ncell <= 32 * 6,
              SNK_ERR_INVALID,
              "Laplace sampling: board side %d too large", L.bs);
    set_lds_limit((const void *)lap_act_kernel, lds);
    const BoardSrc src = src_env(E);
    for (int t = 0; t < T; ++t) {
        lap_act_kernel<<<(unsigned)G, 256, lds, s>>>(L, W, ldw, src, fin, act, nullptr, (int)lap_act_front_floats(L));
        launch_check("lap_act_kernel");
        env_launch_step(E, act, SNK_ACT_INDEX, &R, s);
        lap_track_kernel<<<(unsigned)ceil_div(G, 256), 256, 0, s>>>(E.out_done, E.out_ep_reward, G, t, fin, len_dev,
                                                                    rew_dev, nfin);
        launch_check("lap_track_kernel");
        if ((t & 7) == 7) {
            int32_t h = 0;
            SNK_HIP(hipMemcpyAsync(&h, nfin, sizeof(int32_t), hipMemcpyDeviceToHost, s));
            SNK_HIP(hipStreamSynchronize(s));
            if (h == G) break;
        }
    }
    SNK_HIP(hipStreamSynchronize(s));
}

extern "C" int snk_laplace_normals(uint64_t seed, int64_t model, int32_t which, int64_t i0, int64_t n, double *out_host) {
    return guard([&] {
        SNK_CHECK(out_host && n >= 0 && (which == 1 || which == 2), SNK_ERR_INVALID, "bad laplace_normals arguments");
        if (n == 0) return;
        hipStream_t s = stream();
        double *d = dalloc<double>(n);
        lap_normals_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, s>>>(seed, (uint64_t)model, (uint32_t)which, i0, n, d);
        launch_check("lap_normals_kernel");
        SNK_HIP(hipMemcpyAsync(out_host, d, n * sizeof(double), hipMemcpyDeviceToHost, s));
        SNK_HIP(hipStreamSynchronize(s));
        dfree(d);
    });
}

static void lap_build(snk_laplace h, snk_dqn m, uint64_t seed, int64_t n0, int64_t G, float *W, int64_t ldw) {
    SNK_CHECK(h->K >= 2, SNK_ERR_INVALID, "sample_model needs K >= 2 columns of D (la_utils.jl:93)");
    SNK_CHECK(h->P == m->L.P, SNK_ERR_INVALID, "D has %lld parameters, the model %lld", (long long)h->P,
              (long long)m->L.P);
    const double c1 = 1.0 / sqrt(2.0), c2 = 1.0 / sqrt(2.0 * (double)(h->K - 1));
    const int GS = (int)std::max<int64_t>(1, std::min<int64_t>(64, 16384 / h->K));   // z2 of GS models in LDS
    hipStream_t s = stream();
    for (int64_t g0 = 0; g0 < G; g0 += GS) {
        const int gn = (int)std::min<int64_t>(GS, G - g0);
        lap_sample_kernel<<<(unsigned)std::min<int64_t>(ceil_div(h->P, 256), 4096), 256, (size_t)gn * h->K * sizeof(double),
                            s>>>(h->mean, h->var, h->D, h->K, h->P, m->perm, seed, n0 + g0, gn, c1, c2, W + g0 * ldw, ldw);
        launch_check("lap_sample_kernel");
    }
}

extern "C" int snk_laplace_sample_params(snk_laplace h, snk_dqn m, uint64_t seed, int64_t model, float *flux_host) {
    return guard([&] {
        SNK_CHECK(h && m && flux_host && model >= 0, SNK_ERR_INVALID, "bad sample_params arguments");
        const int64_t P = m->L.P;
        float *W = dalloc<float>(P);
        lap_build(h, m, seed, model, 1, W, P);
        std::vector<float> packed(P);
        std::vector<int32_t> perm(P);
        SNK_HIP(hipMemcpyAsync(packed.data(), W, P * sizeof(float), hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipMemcpyAsync(perm.data(), m->perm, P * sizeof(int32_t), hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
        dfree(W);
        for (int64_t j = 0; j < P; ++j) flux_host[perm[j]] = packed[j];
    });
}

extern "C" int snk_laplace_sampling(snk_laplace h, snk_dqn m, snk_replay rb, int64_t n_models, uint64_t seed,
                                    int64_t chunk, float *tr_reward_out, int64_t *n_better_out, float *rewards_host,
                                    int32_t *lengths_host) {
    return guard([&] {
        SNK_CHECK(h && m && rb && n_models >= 0 && tr_reward_out && n_better_out, SNK_ERR_INVALID, "NULL argument");
        SNK_CHECK(!m->deep, SNK_ERR_INVALID, "deep net: laplace_sampling! is not supported (its rollout kernel is the "
                  "reference architecture's)");
        const QLayout &L = m->L;
        const ReplayDev &D = replay_dev(rb);
        SNK_CHECK(D.bs == L.bs && D.C == L.C, SNK_ERR_INVALID, "replay geometry differs from the model");
        hipStream_t s = stream();
        const int64_t P = L.P;
        // every model in ONE lockstep rollout unless a chunk is asked for (16,384 models of
        // 1.1 MB fit easily; each chunk pays a whole rollout's 501 steps); the current q_net's
        // own greedy episode (play_episode(tr.model, 0f0), la_utils.jl:101) rides in the first
        // chunk as one more env: row G of W holds its packed theta
        const int64_t G0 = chunk > 0 ? chunk : std::max<int64_t>(1, std::min<int64_t>(n_models, 16384));
        const int64_t ldw = (P + 3) & ~int64_t(3);   // 16-byte aligned model rows (float4 weight loads)
        DevBuf<float> W((size_t)(std::max<int64_t>(G0, 1) + 1) * ldw);
        DevBuf<float> rew(std::max<int64_t>(G0, 1) + 1);
        DevBuf<int32_t> len(std::max<int64_t>(G0, 1) + 1);
        float tr_reward = 0.0f;
        int64_t n_better = 0;
        std::vector<float> hr;
        std::vector<int32_t> hl;
        for (int64_t n0 = 0; n0 < std::max<int64_t>(n_models, 1); n0 += G0) {
            const int64_t G = std::min(G0, n_models - n0);   // 0 when n_models = 0: the reference episode alone
            const int64_t GR = n0 == 0 ? G + 1 : G;          // + tr.model's env in the first chunk
            if (G > 0) lap_build(h, m, seed, n0, G, W, ldw);
            if (n0 == 0)
                SNK_HIP(hipMemcpyAsync(W + G * ldw, m->theta_q, P * sizeof(float), hipMemcpyDeviceToDevice, s));
            EnvHold e;
            ReplayHold r;
            lap_rollout(m, W, ldw, GR, rew, len, e, r);
            hr.resize(GR);
            hl.resize(GR);
            SNK_HIP(hipMemcpy(hr.data(), rew, GR * sizeof(float), hipMemcpyDeviceToHost));
            SNK_HIP(hipMemcpy(hl.data(), len, GR * sizeof(int32_t), hipMemcpyDeviceToHost));
            if (n0 == 0) {
                SNK_CHECK(hl[G] > 0, SNK_ERR_INTERNAL, "tr.model: episode did not end");
                tr_reward = hr[G];
            }
            std::vector<int64_t> slots;
            for (int64_t g = 0; g < G; ++g) {
                SNK_CHECK(hl[g] > 0, SNK_ERR_INTERNAL, "model %lld: episode did not end", (long long)(n0 + g));
                if (rewards_host) rewards_host[n0 + g] = hr[g];
                if (lengths_host) lengths_host[n0 + g] = hl[g];
                if (hr[g] > tr_reward) {   // la_utils.jl:108
                    ++n_better;
                    for (int t = 0; t < hl[g]; ++t) slots.push_back((int64_t)t * GR + g);
                }
            }
            if (!slots.empty()) {
                // store! in (model, step) order: with more transitions than capacity only
                // the last cap survive, each in the ring slot the sequential stores leave it
                // in; count still advances by all ns (utils.jl:267-277)
                const int64_t ns = (int64_t)slots.size();
                const int64_t skip = ns > D.cap ? ns - D.cap : 0, nc = ns - skip;
                DevBuf<int64_t> sd(nc);
                int64_t dcount = 0;
                SNK_HIP(hipMemcpyAsync(sd, slots.data() + skip, nc * sizeof(int64_t), hipMemcpyHostToDevice, s));
                SNK_HIP(hipMemcpyAsync(&dcount, D.count, sizeof(int64_t), hipMemcpyDeviceToHost, s));
                SNK_HIP(hipStreamSynchronize(s));
                lap_copy_kernel<<<(unsigned)nc, 256, 0, s>>>(replay_dev(r.r), D, sd, nc, dcount + skip);
                launch_check("lap_copy_kernel");
                lap_count_add_kernel<<<1, 1, 0, s>>>(D.count, ns);
                launch_check("lap_count_add_kernel");
                SNK_HIP(hipStreamSynchronize(s));
            }
        }
        *tr_reward_out = tr_reward;
        *n_better_out = n_better;
    });
}

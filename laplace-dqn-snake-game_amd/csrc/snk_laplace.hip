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
#include <vector>

#include "snk_dqn.hpp"
#include "snk_syrk.hpp"

struct snk_laplace_s {
    int64_t P = 0, ld32 = 0;
    int32_t K = 0;
    double *D = nullptr, *mean = nullptr, *var = nullptr, *G = nullptr, *slab = nullptr;
    float *D32 = nullptr;
    int64_t slab_cap = 0;
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

// Lower-triangle tiles in supertile order: groups of 8 block rows x 4 block
// columns, so the ~32 workgroups an XCD runs at once (syrk_xcd_remap hands
// each XCD a contiguous run of this list) share 8 + 4 row blocks in its L2
// instead of 1 + 32 in plain row-major order. One device table per N, kept.
static const int2 *syrk_tile_order(int N) {
    static std::vector<std::pair<int, int2 *>> cache;
    for (auto &c : cache)
        if (c.first == N) return c.second;
    const int T = (int)ceil_div(N, SY_T);
    std::vector<int2> t;
    t.reserve((size_t)T * (T + 1) / 2);
    constexpr int SI = 8, SJ = 4;
    for (int i0 = 0; i0 < T; i0 += SI)
        for (int j0 = 0; j0 <= std::min(T - 1, i0 + SI - 1); j0 += SJ)
            for (int i = i0; i < std::min(T, i0 + SI); ++i)
                for (int j = j0; j < std::min(j0 + SJ, i + 1); ++j) t.push_back(int2{i, j});
    SNK_CHECK((int64_t)t.size() == (int64_t)T * (T + 1) / 2, SNK_ERR_INTERNAL, "syrk tile order");
    int2 *d = nullptr;
    SNK_HIP(hipMalloc(&d, t.size() * sizeof(int2)));
    SNK_HIP(hipMemcpy(d, t.data(), t.size() * sizeof(int2), hipMemcpyHostToDevice));
    cache.emplace_back(N, d);
    return d;
}

static void syrk_launch(int out, const SyrkArgs &a0, int z, hipStream_t s) {
    SyrkArgs a = a0;
    const int64_t T = ceil_div(a.N, SY_T);
    a.ntiles = T * (T + 1) / 2;
    static const bool rowmajor = getenv("SNK_SYRK_ORDER") && strcmp(getenv("SNK_SYRK_ORDER"), "rows") == 0;
    a.tiles = (rowmajor || T < 16) ? nullptr : syrk_tile_order(a.N);
    SNK_CHECK(a.K % 4 == 0 && a.ld % 4 == 0 && a.kchunk % 4 == 0, SNK_ERR_INTERNAL, "syrk: K/ld not multiples of 4");
    SNK_CHECK(a.ntiles < (int64_t)1 << 31 && z <= 65535, SNK_ERR_INVALID, "syrk: problem too large");
    dim3 grid((unsigned)a.ntiles, (unsigned)z);
    // SNK_SYRK=fp32: the exact-f32 32x32x2 MFMA everywhere; =x6: the bf16 x6 split also
    // for pre-split (h3) callers; default: x6, and h3 where the caller pre-split x
    static const char *env = getenv("SNK_SYRK");
    static const bool f32 = env && strcmp(env, "fp32") == 0, nox3 = env && strcmp(env, "x6") == 0;
    if (f32) {
        switch (out) {
            case SYRK_F32: syrk_kernel<SYRK_F32, SY_F32><<<grid, 256, 0, s>>>(a); break;
            case SYRK_SLAB64: syrk_kernel<SYRK_SLAB64, SY_F32><<<grid, 256, 0, s>>>(a); break;
            default: syrk_kernel<SYRK_DENSE_ADD, SY_F32><<<grid, 256, 0, s>>>(a); break;
        }
    } else if (a.xh && !nox3) {
        SNK_CHECK(out == SYRK_F32 && z == 1 && a.ldh % SY_KS == 0 && a.xe, SNK_ERR_INTERNAL, "syrk h3 arguments");
        static const bool w4 = getenv("SNK_SYRK_W4") != nullptr;   // 4 waves of 64 x 64 (one per SIMD)
        if (w4)
            syrk_h3_kernel<4><<<grid, 256, 0, s>>>(a);
        else if (getenv("SNK_SYRK_PRIO"))
            syrk_h3_kernel<8, true><<<grid, 512, 0, s>>>(a);
        else
            syrk_h3_kernel<8><<<grid, 512, 0, s>>>(a);
    } else {
        switch (out) {
            case SYRK_F32: syrk_kernel<SYRK_F32, SY_X6><<<grid, 256, 0, s>>>(a); break;
            case SYRK_SLAB64: syrk_kernel<SYRK_SLAB64, SY_X6><<<grid, 256, 0, s>>>(a); break;
            default: syrk_kernel<SYRK_DENSE_ADD, SY_X6><<<grid, 256, 0, s>>>(a); break;
        }
    }
    launch_check("syrk_kernel");
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
        SNK_HIP(hipStreamSynchronize(stream()));
        *out = h;
    });
}

extern "C" int snk_laplace_destroy(snk_laplace h) {
    return guard([&] {
        if (!h) return;
        (void)hipStreamSynchronize(stream());
        for (void *p : {(void *)h->D, (void *)h->mean, (void *)h->var, (void *)h->G, (void *)h->slab, (void *)h->D32})
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
        lap_center_kernel<<<(unsigned)std::min<int64_t>(ceil_div((int64_t)h->K * h->ld32, 256), 16384), 256, 0, s>>>(
            h->D, h->P, h->K, h->mean, h->D32, h->ld32);
        launch_check("lap_center_kernel");
    });
}

extern "C" int snk_laplace_gram(snk_laplace h, float *ms_out) {
    return guard([&] {
        SNK_CHECK(h, SNK_ERR_INVALID, "NULL argument");
        hipStream_t s = stream();
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

extern "C" int snk_jacobian_gram(snk_dqn m, snk_replay rb, int64_t n, float *G_dev, float *ms_out) {
    return guard([&] {
        SNK_CHECK(m && rb && G_dev && n > 0, SNK_ERR_INVALID, "bad argument");
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
        SyrkArgs a{};
        a.x = m->jbuf; a.ld = Kc; a.K = Kc; a.kchunk = Kc; a.N = (int)n; a.g32 = G_dev; a.ldg = n;
        static const char *senv = getenv("SNK_SYRK");
        if (!senv || strcmp(senv, "h3") == 0) {
            // h3 Gram: rows pre-split once into scaled fp16 planes (snk_syrk.hpp h3_rows_kernel)
            const int64_t ldh = (Kc + SY_KS - 1) / SY_KS * SY_KS;
            if (2 * n * ldh > m->jplanes_halves) {
                (void)hipStreamSynchronize(s);
                dfree(m->jplanes);
                m->jplanes = dalloc<uint16_t>(2 * n * ldh);
                m->jplanes_halves = 2 * n * ldh;
            }
            if (n > m->jexp_cap) {
                (void)hipStreamSynchronize(s);
                dfree(m->jexp);
                m->jexp = dalloc<int32_t>(n);
                m->jexp_cap = n;
            }
            h3_rows_kernel<<<(unsigned)n, 256, 0, s>>>(m->jbuf, Kc, Kc, m->jplanes, m->jexp, ldh);
            launch_check("h3_rows_kernel");
            a.xh = m->jplanes; a.xe = m->jexp; a.ldh = ldh;
            if (getenv("SNK_SYRK_EXP_NOLOAD")) a.kchunk = -4;   // experiment: every stage re-reads k = 0
        }
        syrk_launch(SYRK_F32, a, 1, s);
        if (ms_out) SNK_HIP(hipEventRecord(ev[3], s));
        SyrkArgs d{};
        d.x = m->jw.a3; d.ld = L.K1; d.K = L.K1; d.kchunk = L.K1; d.N = (int)n; d.g32 = G_dev; d.ldg = n;
        d.z = m->jw.dz1; d.hh = m->jw.h1; d.act = m->jact; d.ldz = 64;
        syrk_launch(SYRK_DENSE_ADD, d, 1, s);
        const unsigned nb = (unsigned)ceil_div(n, 64);
        mirror_kernel<<<dim3(nb, nb), 256, 0, s>>>(G_dev, (int)n, n);
        launch_check("mirror_kernel");
        if (ms_out) {
            SNK_HIP(hipEventRecord(ev[4], s));
            SNK_HIP(hipEventSynchronize(ev[4]));
            for (int i = 0; i < 4; ++i) SNK_HIP(hipEventElapsedTime(&ms_out[i], ev[i], ev[i + 1]));
            for (auto &e : ev) (void)hipEventDestroy(e);
        } else {
            SNK_HIP(hipStreamSynchronize(s));
        }
    });
}

// cpu_fast.cpp — the CPU BASELINE of bench.py (test / measurement
// infrastructure, never the product): an optimised multi-threaded C++
// restatement of the same hot path the device runs, so the GPU numbers sit
// next to a fair CPU number, not next to the deliberately
// naive fidelity oracle (snake_oracle.c).
//
//   env     step! + virtual_step + auto-reset (utils.jl:43-132), O(1)
//           collision via the board lookup, snake body in a ring; bit-exact
//           with the oracle (tests/test_cpu_fast.py);
//   Q-net   structs.jl:127-139 in fp32: conv1 direct, conv2 / conv3 as
//           im2col x weights, Dense1 / Dense2 as GEMM rows; the inner loops
//           run over the output channels (contiguous) so they vectorise;
//   update  utils.jl:448-466: TD target on t_net, Huber, backward through
//           the same im2col GEMMs (per-thread gradient accumulators), RMSProp;
//   Gram    G = X X' (the D build), fp32 blocked, lower triangle + mirror.
// OpenMP over envs / samples / rows; `threads` = 1 gives the single-core number.
// Built by oracle/Makefile with -O3 -mavx2 -mfma (x86-64-v3, no -march=native:
// the library travels to the GPU box's host).
#include <omp.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

// ---------------------------------------------------------------- env
const int DI[4] = {-1, 1, 0, 0}, DJ[4] = {0, 0, -1, 1};   // U D L R (utils.jl:8)
inline int avail(int prev, int k) {                          // k-th of available_actions
    static const int T[4][3] = {{0, 2, 3}, {1, 2, 3}, {0, 1, 2}, {0, 1, 3}};
    return T[prev][k];
}

struct Env {
    int bs, C, n, ring_cap, max_hist;
    std::vector<int16_t> food;
    std::vector<int8_t> board, prev_board, init;   // [n][bs*bs]; prev_board = b_{t-1} (C = 2 states)
    std::vector<uint16_t> ring;                    // [n][ring_cap], head at index head[e]
    std::vector<int> head, len, prev, steps, score;
    std::vector<uint64_t> used;
    std::vector<float> ep_reward;
    int64_t t = 0;

    void reset_one(int e) {
        const int nc = bs * bs;
        memcpy(&board[(size_t)e * nc], init.data(), nc);
        memcpy(&prev_board[(size_t)e * nc], init.data(), nc);
        head[e] = 0;
        len[e] = 2;
        ring[(size_t)e * ring_cap] = (uint16_t)((bs - 3) + bs);   // structs.jl:47 (bs-2, 2)
        ring[(size_t)e * ring_cap + 1] = (uint16_t)((bs - 2) + bs);
        prev[e] = 0;
        steps[e] = 0;
        score[e] = 0;
        used[e] = 0;
        ep_reward[e] = 0.0f;
    }
};

int food_search(const int8_t *b, const int16_t *food, int nf, uint64_t used) {
    for (int k = 0; k < nf; ++k)
        if (!((used >> k) & 1ull) && b[food[k]] == 0) return k;
    return -1;
}

// one step of env e; frames (optional) [C+1][nc] = b_{t-C}..b_t
void env_step_one(Env &E, int e, int a, float &reward, uint8_t &done, uint8_t &mask, int8_t *frames) {
    const int bs = E.bs, nc = bs * bs, cap = E.ring_cap;
    int8_t *b = &E.board[(size_t)e * nc];
    uint16_t *ring = &E.ring[(size_t)e * cap];
    if (frames) {
        if (E.C == 2) memcpy(frames, &E.prev_board[(size_t)e * nc], nc);
        memcpy(frames + (E.C == 2 ? nc : 0), b, nc);
        if (E.C == 2) memcpy(&E.prev_board[(size_t)e * nc], b, nc);
    } else if (E.C == 2) {
        memcpy(&E.prev_board[(size_t)e * nc], b, nc);
    }
    const int pv = E.prev[e];
    const int dir = avail(pv, a % 3);
    const int hc = ring[E.head[e]];
    int ti = E.head[e] + E.len[e] - 1;
    if (ti >= cap) ti -= cap;
    const int tc = ring[ti];
    const int nh = hc + DI[dir] + DJ[dir] * bs;
    const int old = b[nh];
    const bool eat = old == 2;
    float r = eat ? 1.0f : -0.01f;
    int fcell = -1;
    if (eat) {
        E.score[e] += 1;
        const int k = food_search(b, E.food.data(), (int)E.food.size(), E.used[e]);
        if (k >= 0) {
            E.used[e] |= 1ull << k;
            fcell = E.food[k];
        }
    }
    const bool body = old == 1 && !(!eat && nh == tc);
    const int st = E.steps[e] + 1;
    const bool lost = old == -1 || body || (E.C + st - 1 > E.max_hist);
    if (lost) r = -1.0f;
    if (!eat) b[tc] = 0;
    b[nh] = 1;
    if (fcell >= 0) b[fcell] = 2;
    const int nhead = E.head[e] == 0 ? cap - 1 : E.head[e] - 1;
    ring[nhead] = (uint16_t)nh;
    const int ntail = eat ? tc : ring[ti == 0 ? cap - 1 : ti - 1];
    uint8_t m = 7;
    if (!lost) {
        m = 0;
        const bool tr2 = E.C + st > E.max_hist;
        for (int k2 = 0; k2 < 3; ++k2) {
            const int d2 = avail(dir, k2);
            const int nh2 = nh + DI[d2] + DJ[d2] * bs;
            const int v = b[nh2];
            const bool vbody = v == 1 && !(v != 2 && nh2 == ntail);
            if (v == -1 || vbody || tr2) m |= (uint8_t)(1 << k2);
        }
    }
    if (frames) memcpy(frames + E.C * nc, b, nc);
    reward = r;
    done = lost;
    mask = m;
    if (lost) {
        E.reset_one(e);   // auto-reset: the next state is SnakeGame()'s (b0, b0)
    } else {
        E.head[e] = nhead;
        E.len[e] += eat ? 1 : 0;
        E.prev[e] = dir;
        E.steps[e] = st;
        E.ep_reward[e] += r;
    }
}

// ---------------------------------------------------------------- Q-net (fp32)
struct Layout {
    int bs, C, Wo, K1, nc;
    int64_t w1, b1, w2, b2, w3, b3, d1w, d1b, d2w, d2b, P;
};
Layout layout(int bs, int C) {
    Layout L{};
    L.bs = bs; L.C = C; L.Wo = bs - 5; L.K1 = L.Wo * L.Wo * 64; L.nc = bs * bs;
    int64_t o = 0;
    L.w1 = o; o += 9 * C * 16; L.b1 = o; o += 16;
    L.w2 = o; o += 9 * 16 * 32; L.b2 = o; o += 32;
    L.w3 = o; o += 36 * 32 * 64; L.b3 = o; o += 64;
    L.d1w = o; o += (int64_t)L.K1 * 64; L.d1b = o; o += 64;
    L.d2w = o; o += 3 * 64; L.d2b = o; o += 3;
    L.P = o;
    return L;
}
// packed index -> Flux.destructure index (the device's packed_to_flux_index)
std::vector<int64_t> perm_of(const Layout &L) {
    std::vector<int64_t> p(L.P);
    auto conv = [&](int64_t off, int KS, int Cin, int Cout) {
        for (int dv = 0; dv < KS; ++dv)
            for (int du = 0; du < KS; ++du)
                for (int ci = 0; ci < Cin; ++ci)
                    for (int co = 0; co < Cout; ++co)
                        p[off + ((int64_t)(du + KS * dv) * Cin + ci) * Cout + co] =
                            off + (KS - 1 - du) + (int64_t)KS * (KS - 1 - dv) + (int64_t)KS * KS * ci +
                            (int64_t)KS * KS * Cin * co;
        const int64_t b = off + (int64_t)KS * KS * Cin * Cout;
        for (int co = 0; co < Cout; ++co) p[b + co] = b + co;
    };
    conv(L.w1, 3, L.C, 16);
    conv(L.w2, 3, 16, 32);
    conv(L.w3, 6, 32, 64);
    const int np = L.Wo * L.Wo;
    for (int q = 0; q < np; ++q)
        for (int c = 0; c < 64; ++c)
            for (int o = 0; o < 64; ++o) p[L.d1w + ((int64_t)q * 64 + c) * 64 + o] = L.d1w + o + ((int64_t)q + (int64_t)c * np) * 64;
    for (int o = 0; o < 64; ++o) p[L.d1b + o] = L.d1b + o;
    for (int a = 0; a < 3; ++a)
        for (int o = 0; o < 64; ++o) p[L.d2w + a * 64 + o] = L.d2w + a + 3 * o;
    for (int a = 0; a < 3; ++a) p[L.d2b + a] = L.d2b + a;
    return p;
}

// C[M][N] (+)= A[M][K] B[K][N]; N small (16..64): the n loop vectorises
template <int N>
inline void gemm_rows(const float *A, int M, int K, const float *B, float *Cm, bool acc) {
    for (int m = 0; m < M; ++m) {
        float c[N];
        if (acc)
            for (int n = 0; n < N; ++n) c[n] = Cm[m * N + n];
        else
            for (int n = 0; n < N; ++n) c[n] = 0.0f;
        const float *a = A + (int64_t)m * K;
        for (int k = 0; k < K; ++k) {
            const float av = a[k];
            const float *b = B + (int64_t)k * N;
            for (int n = 0; n < N; ++n) c[n] += av * b[n];
        }
        for (int n = 0; n < N; ++n) Cm[m * N + n] = c[n];
    }
}
// dB[K][N] += A[M][K]' G[M][N]
template <int N>
inline void gemm_at(const float *A, int M, int K, const float *G, float *dB) {
    for (int m = 0; m < M; ++m) {
        const float *a = A + (int64_t)m * K;
        const float *g = G + (int64_t)m * N;
        for (int k = 0; k < K; ++k) {
            const float av = a[k];
            if (av == 0.0f) continue;
            float *d = dB + (int64_t)k * N;
            for (int n = 0; n < N; ++n) d[n] += av * g[n];
        }
    }
}
// dA[M][K] = G[M][N] B[K][N]'
template <int N>
inline void gemm_bt(const float *G, int M, int K, const float *B, float *dA) {
    for (int m = 0; m < M; ++m) {
        const float *g = G + (int64_t)m * N;
        float *d = dA + (int64_t)m * K;
        for (int k = 0; k < K; ++k) {
            const float *b = B + (int64_t)k * N;
            float s = 0.0f;
            for (int n = 0; n < N; ++n) s += g[n] * b[n];
            d[k] = s;
        }
    }
}

// im2col of x [H*H][Cin] (p = i + j*H) for KS x KS, pad PAD -> col [Ho*Ho][KS*KS*Cin], k = (kk, ci)
void im2col(const float *x, int H, int Cin, int KS, int PAD, float *col) {
    const int Ho = H + 2 * PAD - KS + 1, K = KS * KS * Cin;
    for (int j = 0; j < Ho; ++j)
        for (int i = 0; i < Ho; ++i) {
            float *c = col + (int64_t)(i + j * Ho) * K;
            for (int dv = 0; dv < KS; ++dv)
                for (int du = 0; du < KS; ++du) {
                    const int xi = i + du - PAD, xj = j + dv - PAD;
                    float *d = c + (du + KS * dv) * Cin;
                    if (xi < 0 || xi >= H || xj < 0 || xj >= H)
                        memset(d, 0, sizeof(float) * Cin);
                    else
                        memcpy(d, x + (int64_t)(xi + xj * H) * Cin, sizeof(float) * Cin);
                }
        }
}
void col2im_add(const float *col, int H, int Cin, int KS, int PAD, float *x) {
    const int Ho = H + 2 * PAD - KS + 1, K = KS * KS * Cin;
    for (int j = 0; j < Ho; ++j)
        for (int i = 0; i < Ho; ++i) {
            const float *c = col + (int64_t)(i + j * Ho) * K;
            for (int dv = 0; dv < KS; ++dv)
                for (int du = 0; du < KS; ++du) {
                    const int xi = i + du - PAD, xj = j + dv - PAD;
                    if (xi < 0 || xi >= H || xj < 0 || xj >= H) continue;
                    float *d = x + (int64_t)(xi + xj * H) * Cin;
                    const float *s = c + (du + KS * dv) * Cin;
                    for (int ci = 0; ci < Cin; ++ci) d[ci] += s[ci];
                }
        }
}

struct Acts {   // one sample's forward state
    std::vector<float> x, a1, c2, a2, c3, a3, h1, q;
    void init(const Layout &L) {
        x.resize(L.nc * L.C); a1.resize(L.nc * 16); c2.resize((size_t)L.nc * 144); a2.resize(L.nc * 32);
        c3.resize((size_t)L.Wo * L.Wo * 1152); a3.resize(L.K1); h1.resize(64); q.resize(3);
    }
};

inline void bias_relu(float *y, int M, int N, const float *b) {
    for (int m = 0; m < M; ++m)
        for (int n = 0; n < N; ++n) {
            const float v = y[m * N + n] + b[n];
            y[m * N + n] = v > 0.0f ? v : 0.0f;
        }
}

// forward of one sample; x given as [C][nc] board planes -> A.x [nc][C]
void forward_one(const Layout &L, const float *th, const float *xin, Acts &A) {
    const int bs = L.bs, nc = L.nc, C = L.C, no = L.Wo * L.Wo;
    for (int c = 0; c < C; ++c)
        for (int p = 0; p < nc; ++p) A.x[p * C + c] = xin[c * nc + p];
    // conv1 direct: K = 9C
    for (int j = 0; j < bs; ++j)
        for (int i = 0; i < bs; ++i) {
            float acc[16];
            for (int co = 0; co < 16; ++co) acc[co] = th[L.b1 + co];
            for (int dv = 0; dv < 3; ++dv)
                for (int du = 0; du < 3; ++du) {
                    const int xi = i + du - 1, xj = j + dv - 1;
                    if (xi < 0 || xi >= bs || xj < 0 || xj >= bs) continue;
                    for (int c = 0; c < C; ++c) {
                        const float v = A.x[(xi + xj * bs) * C + c];
                        const float *w = th + L.w1 + ((du + 3 * dv) * C + c) * 16;
                        for (int co = 0; co < 16; ++co) acc[co] += v * w[co];
                    }
                }
            float *o = &A.a1[(i + j * bs) * 16];
            for (int co = 0; co < 16; ++co) o[co] = acc[co] > 0.0f ? acc[co] : 0.0f;
        }
    im2col(A.a1.data(), bs, 16, 3, 1, A.c2.data());
    gemm_rows<32>(A.c2.data(), nc, 144, th + L.w2, A.a2.data(), false);
    bias_relu(A.a2.data(), nc, 32, th + L.b2);
    im2col(A.a2.data(), bs, 32, 6, 0, A.c3.data());
    gemm_rows<64>(A.c3.data(), no, 1152, th + L.w3, A.a3.data(), false);
    bias_relu(A.a3.data(), no, 64, th + L.b3);
    gemm_rows<64>(A.a3.data(), 1, L.K1, th + L.d1w, A.h1.data(), false);
    bias_relu(A.h1.data(), 1, 64, th + L.d1b);
    for (int a = 0; a < 3; ++a) {
        float s = th[L.d2b + a];
        for (int o = 0; o < 64; ++o) s += th[L.d2w + a * 64 + o] * A.h1[o];
        A.q[a] = s;
    }
}

// grad (packed, accumulated) of sum_a dq[a] * Q[a] for one forwarded sample
void backward_one(const Layout &L, const float *th, Acts &A, const float *dq, float *g, std::vector<float> &tmp) {
    const int bs = L.bs, nc = L.nc, no = L.Wo * L.Wo, C = L.C;
    float dh[64];
    for (int a = 0; a < 3; ++a) {
        g[L.d2b + a] += dq[a];
        for (int o = 0; o < 64; ++o) g[L.d2w + a * 64 + o] += dq[a] * A.h1[o];
    }
    for (int o = 0; o < 64; ++o) {
        float s = 0.0f;
        for (int a = 0; a < 3; ++a) s += dq[a] * th[L.d2w + a * 64 + o];
        dh[o] = A.h1[o] > 0.0f ? s : 0.0f;
        g[L.d1b + o] += dh[o];
    }
    gemm_at<64>(A.a3.data(), 1, L.K1, dh, g + L.d1w);
    tmp.resize((size_t)L.K1 + (size_t)no * 1152 + nc * 32 + (size_t)nc * 144 + nc * 16);
    float *dz3 = tmp.data(), *dc3 = dz3 + L.K1, *dz2 = dc3 + (size_t)no * 1152, *dc2 = dz2 + nc * 32,
          *dz1 = dc2 + (size_t)nc * 144;
    gemm_bt<64>(dh, 1, L.K1, th + L.d1w, dz3);
    for (int i = 0; i < L.K1; ++i) if (!(A.a3[i] > 0.0f)) dz3[i] = 0.0f;
    for (int r = 0; r < no; ++r)
        for (int co = 0; co < 64; ++co) g[L.b3 + co] += dz3[r * 64 + co];
    gemm_at<64>(A.c3.data(), no, 1152, dz3, g + L.w3);
    gemm_bt<64>(dz3, no, 1152, th + L.w3, dc3);
    memset(dz2, 0, sizeof(float) * nc * 32);
    col2im_add(dc3, bs, 32, 6, 0, dz2);
    for (int i = 0; i < nc * 32; ++i) if (!(A.a2[i] > 0.0f)) dz2[i] = 0.0f;
    for (int r = 0; r < nc; ++r)
        for (int co = 0; co < 32; ++co) g[L.b2 + co] += dz2[r * 32 + co];
    gemm_at<32>(A.c2.data(), nc, 144, dz2, g + L.w2);
    gemm_bt<32>(dz2, nc, 144, th + L.w2, dc2);
    memset(dz1, 0, sizeof(float) * nc * 16);
    col2im_add(dc2, bs, 16, 3, 1, dz1);
    for (int i = 0; i < nc * 16; ++i) if (!(A.a1[i] > 0.0f)) dz1[i] = 0.0f;
    for (int j = 0; j < bs; ++j)
        for (int i = 0; i < bs; ++i) {
            const float *d = dz1 + (i + j * bs) * 16;
            for (int co = 0; co < 16; ++co) g[L.b1 + co] += d[co];
            for (int dv = 0; dv < 3; ++dv)
                for (int du = 0; du < 3; ++du) {
                    const int xi = i + du - 1, xj = j + dv - 1;
                    if (xi < 0 || xi >= bs || xj < 0 || xj >= bs) continue;
                    for (int c = 0; c < C; ++c) {
                        const float v = A.x[(xi + xj * bs) * C + c];
                        float *gw = g + L.w1 + ((du + 3 * dv) * C + c) * 16;
                        for (int co = 0; co < 16; ++co) gw[co] += v * d[co];
                    }
                }
        }
}

struct Net {
    Layout L;
    std::vector<float> q, t, acc, grad;
    std::vector<int64_t> perm;
};

// utils.jl:448-464 on B samples; returns the mean Huber loss, grad (packed) overwritten
double loss_grad(Net &N, int B, const float *s, const float *sn, const int *a, const float *r, const uint8_t *done,
                 const uint8_t *mask, int threads) {
    const Layout &L = N.L;
    const int in = L.C * L.nc;
    std::vector<double> li(B);
    const int T = threads;
    std::vector<std::vector<float>> gl(T, std::vector<float>(L.P, 0.0f));
#pragma omp parallel num_threads(T)
    {
        Acts A, At;
        A.init(L);
        At.init(L);
        std::vector<float> tmp;
        float *g = gl[omp_get_thread_num()].data();
#pragma omp for schedule(static)
        for (int b = 0; b < B; ++b) {
            forward_one(L, N.t.data(), sn + (size_t)b * in, At);
            float mx = -INFINITY;
            for (int k = 0; k < 3; ++k) {
                const float v = ((mask[b] >> k) & 1) ? -100.0f : At.q[k];
                mx = v > mx ? v : mx;
            }
            const double tgt = (double)r[b] + 0.97 * (double)mx * (double)(1 - (int)done[b]);
            forward_one(L, N.q.data(), s + (size_t)b * in, A);
            const double e = (double)A.q[a[b]] - tgt, ae = std::fabs(e);
            li[b] = ae < 1.0 ? 0.5 * e * e : ae - 0.5;
            float dq[3] = {0, 0, 0};
            dq[a[b]] = (float)((ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / B);
            backward_one(L, N.q.data(), A, dq, g, tmp);
        }
    }
#pragma omp parallel for num_threads(T) schedule(static)
    for (int64_t i = 0; i < L.P; ++i) {
        float v = 0.0f;
        for (int k = 0; k < T; ++k) v += gl[k][i];
        N.grad[i] = v;
    }
    double loss = 0.0;
    for (int b = 0; b < B; ++b) loss += li[b];
    return loss / B;
}

void rmsprop(Net &N, float eta, float rho, float eps, int threads) {
    const float omr = 1.0f - rho;
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int64_t i = 0; i < N.L.P; ++i) {
        const float g = N.grad[i];
        const float qd = rho * N.acc[i] + omr * (g * g);
        N.acc[i] = qd;
        N.q[i] = N.q[i] - (g * eta) / (std::sqrt(qd) + eps);
    }
}

uint64_t smix(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint64_t rhash(uint64_t seed, uint64_t a, uint64_t b) { return smix(smix(seed ^ (a * 0xD1B54A32D192ED03ULL)) ^ b); }

double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

}  // namespace

extern "C" {

// ---- env (tests: bit-exact with orc_batch_*) ----
void *cpuf_env_create(int n, int bs, int C, int max_hist, const int32_t *food, int n_food) {
    auto *E = new Env();
    E->bs = bs; E->C = C; E->n = n; E->max_hist = max_hist; E->ring_cap = bs * bs + 1;
    const int nc = bs * bs;
    E->food.assign(food, food + n_food);
    E->init.assign(nc, 0);
    for (int i = 0; i < bs; ++i)
        for (int j = 0; j < bs; ++j)
            if (i == 0 || j == 0 || i == bs - 1 || j == bs - 1) E->init[i + j * bs] = -1;
    E->init[3 + 4 * bs] = 2;                        // food at (4, 5) (structs.jl:43)
    E->init[(bs - 3) + bs] = 1;                     // snake (bs-2, 2), (bs-1, 2)
    E->init[(bs - 2) + bs] = 1;
    E->board.resize((size_t)n * nc);
    E->prev_board.resize((size_t)n * nc);
    E->ring.resize((size_t)n * E->ring_cap);
    E->head.resize(n); E->len.resize(n); E->prev.resize(n); E->steps.resize(n); E->score.resize(n);
    E->used.resize(n); E->ep_reward.resize(n);
    for (int e = 0; e < n; ++e) E->reset_one(e);
    return E;
}
void cpuf_env_destroy(void *h) { delete static_cast<Env *>(h); }
void cpuf_env_step(void *h, const uint8_t *act, float *reward, uint8_t *done, uint8_t *mask, int threads) {
    Env &E = *static_cast<Env *>(h);
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int e = 0; e < E.n; ++e) env_step_one(E, e, act[e], reward[e], done[e], mask[e], nullptr);
    E.t += 1;
}
void cpuf_env_boards(void *h, int8_t *out) {
    Env &E = *static_cast<Env *>(h);
    memcpy(out, E.board.data(), E.board.size());
}

// ---- Q-net (tests: vs orc_qnet_forward / orc_dqn_loss_grad) ----
void cpuf_qnet_forward(int bs, int C, const float *flux, int B, const float *x, float *q, int threads) {
    Net N;
    N.L = layout(bs, C);
    N.perm = perm_of(N.L);
    N.q.resize(N.L.P);
    for (int64_t i = 0; i < N.L.P; ++i) N.q[i] = flux[N.perm[i]];
#pragma omp parallel num_threads(threads)
    {
        Acts A;
        A.init(N.L);
#pragma omp for schedule(static)
        for (int b = 0; b < B; ++b) {
            forward_one(N.L, N.q.data(), x + (size_t)b * C * N.L.nc, A);
            for (int k = 0; k < 3; ++k) q[b * 3 + k] = A.q[k];
        }
    }
}
double cpuf_loss_grad(int bs, int C, const float *q_flux, const float *t_flux, int B, const float *s, const int32_t *a,
                      const float *r, const float *sn, const uint8_t *done, const uint8_t *mask3, float *grad_flux,
                      int threads) {
    Net N;
    N.L = layout(bs, C);
    N.perm = perm_of(N.L);
    N.q.resize(N.L.P); N.t.resize(N.L.P); N.grad.resize(N.L.P);
    for (int64_t i = 0; i < N.L.P; ++i) { N.q[i] = q_flux[N.perm[i]]; N.t[i] = t_flux[N.perm[i]]; }
    std::vector<uint8_t> mb(B);
    for (int b = 0; b < B; ++b) mb[b] = (uint8_t)(mask3[3 * b] | (mask3[3 * b + 1] << 1) | (mask3[3 * b + 2] << 2));
    const double l = loss_grad(N, B, s, sn, a, r, done, mb.data(), threads);
    for (int64_t i = 0; i < N.L.P; ++i) grad_flux[N.perm[i]] = N.grad[i];
    return l;
}

// ---- the bench iteration: act forward over n envs, env step + store, U updates ----
// times_out[4]: seconds in forward, env step, updates, total; returns env-steps/s
double cpuf_bench(int n, int bs, int C, int threads, int warm, int steps, int U, int capacity, const int32_t *food,
                  int n_food, double *times_out) {
    Env *E = static_cast<Env *>(cpuf_env_create(n, bs, C, 500, food, n_food));
    Net N;
    N.L = layout(bs, C);
    const Layout &L = N.L;
    N.q.resize(L.P); N.t.resize(L.P); N.acc.assign(L.P, 0.0f); N.grad.resize(L.P);
    uint64_t ctr = 0;
    auto fill = [&](int64_t off, int64_t cnt, double fi, double fo) {
        const double lim = std::sqrt(6.0 / (fi + fo));
        for (int64_t i = 0; i < cnt; ++i)
            N.q[off + i] = (float)((2.0 * ((double)(smix(1234 ^ smix(++ctr)) >> 11) / 9007199254740992.0) - 1.0) * lim);
    };
    std::fill(N.q.begin(), N.q.end(), 0.0f);
    fill(L.w1, 9 * C * 16, 9.0 * C, 144); fill(L.w2, 9 * 16 * 32, 144, 288); fill(L.w3, 36 * 32 * 64, 1152, 2304);
    fill(L.d1w, (int64_t)L.K1 * 64, L.K1, 64); fill(L.d2w, 192, 64, 3);
    N.t = N.q;
    const int nc = L.nc, in = C * nc, fs = (C + 1) * nc;
    std::vector<int8_t> rframes((size_t)capacity * fs);
    std::vector<uint8_t> ract(capacity), rdone(capacity), rmask(capacity);
    std::vector<float> rrew(capacity);
    int64_t count = 0;
    std::vector<uint8_t> act(n);
    std::vector<float> qv((size_t)n * 3);
    double tf = 0, ts = 0, tu = 0;
    std::vector<float> bs_(64 * (size_t)in), bsn(64 * (size_t)in), br(64);
    std::vector<int> ba(64);
    std::vector<uint8_t> bd(64), bm(64);
    for (int it = 0; it < warm + steps; ++it) {
        const bool timed = it >= warm;
        double t0 = now();
        // epsilon_greedy over every env (eps 0.05, counter RNG)
#pragma omp parallel num_threads(threads)
        {
            Acts A;
            A.init(L);
            std::vector<float> x(in);
#pragma omp for schedule(static)
            for (int e = 0; e < n; ++e) {
                const int8_t *cur = &E->board[(size_t)e * nc];
                const int8_t *pr = &E->prev_board[(size_t)e * nc];
                for (int p = 0; p < nc; ++p) {
                    if (C == 2) { x[p] = pr[p]; x[nc + p] = cur[p]; } else x[p] = cur[p];
                }
                forward_one(L, N.q.data(), x.data(), A);
                const uint64_t h = rhash(7, (uint64_t)e, (uint64_t)E->t);
                int a;
                if ((float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f) < 0.05f) {
                    a = (int)((rhash(7 ^ 0xA5A5A5A5A5A5A5A5ULL, e, E->t) >> 32) % 3);
                } else {
                    a = 0;
                    if (A.q[1] > A.q[a]) a = 1;
                    if (A.q[2] > A.q[a]) a = 2;
                }
                act[e] = (uint8_t)a;
            }
        }
        double t1 = now();
#pragma omp parallel for num_threads(threads) schedule(static)
        for (int e = 0; e < n; ++e) {
            const int64_t slot = (count + e) % capacity;
            float rw;
            uint8_t dn, mk;
            env_step_one(*E, e, act[e], rw, dn, mk, &rframes[(size_t)slot * fs]);
            rrew[slot] = rw; rdone[slot] = dn; rmask[slot] = mk; ract[slot] = act[e];
        }
        E->t += 1;
        count += n;
        double t2 = now();
        const int64_t len = std::min<int64_t>(count, capacity);
        for (int u = 0; u < U; ++u) {
            for (int b = 0; b < 64; ++b) {   // sample: 64 counter-RNG slots
                const int64_t k = (int64_t)(rhash(11, (uint64_t)(it * U + u), (uint64_t)b) % (uint64_t)len);
                const int8_t *f = &rframes[(size_t)k * fs];
                for (int i = 0; i < in; ++i) { bs_[(size_t)b * in + i] = f[i]; bsn[(size_t)b * in + i] = f[nc + i]; }
                ba[b] = ract[k]; br[b] = rrew[k]; bd[b] = rdone[k]; bm[b] = rmask[k];
            }
            loss_grad(N, 64, bs_.data(), bsn.data(), ba.data(), br.data(), bd.data(), bm.data(), threads);
            rmsprop(N, 5e-4f, 0.9f, 1e-8f, threads);
        }
        double t3 = now();
        if (timed) { tf += t1 - t0; ts += t2 - t1; tu += t3 - t2; }
    }
    cpuf_env_destroy(E);
    const double tot = tf + ts + tu;
    if (times_out) { times_out[0] = tf; times_out[1] = ts; times_out[2] = tu; times_out[3] = tot; }
    return (double)n * steps / tot;
}

// ---- G = X X' (lower triangle + mirror), X [n][K] fp32; returns seconds ----
// 64 x 64 output blocks, k in chunks of 256: the column block's rows are packed
// transposed (Bt[k][j]) so the inner loop runs over 64 contiguous outputs.
double cpuf_gram(int n, int K, const float *X, float *G, int threads) {
    const double t0 = now();
    constexpr int BI = 64, KC = 256;
    const int nb = (n + BI - 1) / BI;
    std::vector<std::pair<int, int>> blocks;
    for (int ib = 0; ib < nb; ++ib)
        for (int jb = 0; jb <= ib; ++jb) blocks.emplace_back(ib, jb);
#pragma omp parallel num_threads(threads)
    {
        std::vector<float> bt((size_t)KC * BI), acc((size_t)BI * BI);
#pragma omp for schedule(dynamic)
        for (size_t q = 0; q < blocks.size(); ++q) {
            const int i0 = blocks[q].first * BI, j0 = blocks[q].second * BI;
            const int ni = std::min(BI, n - i0), nj = std::min(BI, n - j0);
            std::fill(acc.begin(), acc.end(), 0.0f);
            for (int k0 = 0; k0 < K; k0 += KC) {
                const int kc = std::min(KC, K - k0);
                std::fill(bt.begin(), bt.end(), 0.0f);
                for (int j = 0; j < nj; ++j)
                    for (int k = 0; k < kc; ++k) bt[(size_t)k * BI + j] = X[(int64_t)(j0 + j) * K + k0 + k];
                for (int i = 0; i < ni; ++i) {
                    const float *a = X + (int64_t)(i0 + i) * K + k0;
                    float c[BI];
                    for (int j = 0; j < BI; ++j) c[j] = acc[(size_t)i * BI + j];
                    for (int k = 0; k < kc; ++k) {
                        const float av = a[k];
                        const float *b = &bt[(size_t)k * BI];
                        for (int j = 0; j < BI; ++j) c[j] += av * b[j];
                    }
                    for (int j = 0; j < BI; ++j) acc[(size_t)i * BI + j] = c[j];
                }
            }
            for (int i = 0; i < ni; ++i)
                for (int j = 0; j < nj; ++j) {
                    if (j0 + j > i0 + i) continue;
                    const float v = acc[(size_t)i * BI + j];
                    G[(int64_t)(i0 + i) * n + j0 + j] = v;
                    G[(int64_t)(j0 + j) * n + i0 + i] = v;
                }
        }
    }
    return now() - t0;
}

int cpuf_max_threads(void) { return omp_get_num_procs(); }

}  // extern "C"

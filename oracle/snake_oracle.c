/*
 * snake_oracle.c — CPU ORACLE (test infrastructure only; see snake_oracle.h).
 *
 * Literal restatement of the reference Julia algorithm. Each function cites
 * the reference file:line it follows. Written for fidelity, not speed: the
 * env keeps the reference's O(L) list operations and O(bs^2) board passes,
 * and virtual_step deep-copies the game exactly as utils.jl:122 does.
 * Compiled with -ffp-contract=off so Float32/Float64 arithmetic rounds like
 * Julia's (no fused multiply-add).
 */
#include "snake_oracle.h"
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ======================= SHA-256 (for Julia's hash_seed) ================== */
typedef struct { uint32_t h[8]; uint8_t buf[64]; uint64_t len; int fill; } sha256_ctx;
static const uint32_t K256[64] = {
    0x428a2f98,0x71374491,0xb5c0fbcf,0xe9b5dba5,0x3956c25b,0x59f111f1,0x923f82a4,0xab1c5ed5,
    0xd807aa98,0x12835b01,0x243185be,0x550c7dc3,0x72be5d74,0x80deb1fe,0x9bdc06a7,0xc19bf174,
    0xe49b69c1,0xefbe4786,0x0fc19dc6,0x240ca1cc,0x2de92c6f,0x4a7484aa,0x5cb0a9dc,0x76f988da,
    0x983e5152,0xa831c66d,0xb00327c8,0xbf597fc7,0xc6e00bf3,0xd5a79147,0x06ca6351,0x14292967,
    0x27b70a85,0x2e1b2138,0x4d2c6dfc,0x53380d13,0x650a7354,0x766a0abb,0x81c2c92e,0x92722c85,
    0xa2bfe8a1,0xa81a664b,0xc24b8b70,0xc76c51a3,0xd192e819,0xd6990624,0xf40e3585,0x106aa070,
    0x19a4c116,0x1e376c08,0x2748774c,0x34b0bcb5,0x391c0cb3,0x4ed8aa4a,0x5b9cca4f,0x682e6ff3,
    0x748f82ee,0x78a5636f,0x84c87814,0x8cc70208,0x90befffa,0xa4506ceb,0xbef9a3f7,0xc67178f2};
#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))
static void sha_block(sha256_ctx *c, const uint8_t *p) {
    uint32_t w[64], a, b, cc, d, e, f, g, h;
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 | p[4 * i + 3];
    for (int i = 16; i < 64; i++) {
        uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
        uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
        w[i] = w[i - 16] + s0 + w[i - 7] + s1;
    }
    a = c->h[0]; b = c->h[1]; cc = c->h[2]; d = c->h[3]; e = c->h[4]; f = c->h[5]; g = c->h[6]; h = c->h[7];
    for (int i = 0; i < 64; i++) {
        uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
        uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & cc) ^ (b & cc));
        h = g; g = f; f = e; e = d + t1; d = cc; cc = b; b = a; a = t1 + t2;
    }
    c->h[0] += a; c->h[1] += b; c->h[2] += cc; c->h[3] += d; c->h[4] += e; c->h[5] += f; c->h[6] += g; c->h[7] += h;
}
static void sha_init(sha256_ctx *c) {
    static const uint32_t iv[8] = {0x6a09e667,0xbb67ae85,0x3c6ef372,0xa54ff53a,0x510e527f,0x9b05688c,0x1f83d9ab,0x5be0cd19};
    memcpy(c->h, iv, sizeof iv); c->len = 0; c->fill = 0;
}
static void sha_update(sha256_ctx *c, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) {
        c->buf[c->fill++] = p[i]; c->len++;
        if (c->fill == 64) { sha_block(c, c->buf); c->fill = 0; }
    }
}
static void sha_final(sha256_ctx *c, uint8_t out[32]) {
    uint64_t bits = c->len * 8;
    uint8_t pad = 0x80, z = 0;
    sha_update(c, &pad, 1);
    while (c->fill != 56) sha_update(c, &z, 1);
    uint8_t lb[8];
    for (int i = 0; i < 8; i++) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
    sha_update(c, lb, 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(c->h[i] >> 24); out[4 * i + 1] = (uint8_t)(c->h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(c->h[i] >> 8); out[4 * i + 3] = (uint8_t)c->h[i];
    }
}

/* ======================= Julia Random.Xoshiro ============================= */
/* Julia Random hash_seed(seed::Integer): SHA-256 over the seed's UInt32
 * little-endian words (one word for 42); Xoshiro's s0..s3 are the first four
 * little-endian UInt64 of the digest, s4 = s0 + 3s1 + 5s2 + 7s3.
 * Used by structs.jl:33 `food_rng = Xoshiro(42)`. */
void orc_julia_xoshiro_seed(uint32_t seed, uint64_t st[5]) {
    sha256_ctx c; uint8_t dg[32], w[4];
    for (int i = 0; i < 4; i++) w[i] = (uint8_t)(seed >> (8 * i));
    sha_init(&c); sha_update(&c, w, 4); sha_final(&c, dg);
    for (int k = 0; k < 4; k++) {
        uint64_t v = 0;
        for (int i = 7; i >= 0; i--) v = (v << 8) | dg[8 * k + i];
        st[k] = v;
    }
    st[4] = st[0] + 3 * st[1] + 5 * st[2] + 7 * st[3];
}

static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* xoshiro256++ (Julia Random/src/Xoshiro.jl rand(::Xoshiro, UInt64)) */
uint64_t orc_xoshiro_next(uint64_t s[4]) {
    uint64_t res = rotl64(s[0] + s[3], 23) + s[0];
    uint64_t t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
    s[2] ^= t; s[3] = rotl64(s[3], 45);
    return res;
}

/* rand(rng, a:b) for Int64 ranges: Julia SamplerRangeNDL (Lemire). */
int64_t orc_rand_range(uint64_t st[4], int64_t a, int64_t b) {
    uint64_t s = (uint64_t)(b - a) + 1;
    unsigned __int128 m = (unsigned __int128)orc_xoshiro_next(st) * s;
    uint64_t l = (uint64_t)m;
    if (l < s) {
        uint64_t t = (0 - s) % s;
        while (l < t) {
            m = (unsigned __int128)orc_xoshiro_next(st) * s;
            l = (uint64_t)m;
        }
    }
    return a + (int64_t)(uint64_t)(m >> 64);
}

/* structs.jl:70: food_list = [CartesianIndex(rand(rng,2:bs-1), rand(rng,2:bs-1)) for _ in 1:50]
 * (row drawn first). Output cells are column-major 0-based. */
void orc_food_list(int bs, uint32_t seed, int n, int32_t *cells, uint64_t st_after[4]) {
    uint64_t st[5];
    orc_julia_xoshiro_seed(seed, st);
    for (int k = 0; k < n; k++) {
        int64_t r = orc_rand_range(st, 2, bs - 1);
        int64_t c = orc_rand_range(st, 2, bs - 1);
        cells[k] = (int32_t)((r - 1) + (c - 1) * bs);
    }
    if (st_after) memcpy(st_after, st, 4 * sizeof(uint64_t));
}

/* ======================= env ============================================== */
static int dir_delta(int bs, int d) {
    switch (d) { case 0: return -1; case 1: return 1; case 2: return -bs; default: return bs; }
}

int orc_game_sizeof(void) { return (int)sizeof(orc_game); }

/* SnakeGame(board_size, n_frames, ...) structs.jl:33-99 */
void orc_game_init(orc_game *g, int bs, int n_frames, int max_hist, const int32_t *food, int n_food) {
    memset(g, 0, sizeof *g);
    g->bs = bs; g->n_frames = n_frames; g->max_hist = max_hist;
    int8_t *b = g->hist[0];
    for (int j = 0; j < bs; j++)
        for (int i = 0; i < bs; i++)
            b[i + j * bs] = (i == 0 || i == bs - 1 || j == 0 || j == bs - 1) ? -1 : 0;  /* :37-40 walls */
    b[3 + 4 * bs] = 2;                                   /* :43 board[4,5] = 2 */
    g->snake[0] = (int16_t)((bs - 3) + 1 * bs);          /* :47 (bs-2, 2) head */
    g->snake[1] = (int16_t)((bs - 2) + 1 * bs);          /*      (bs-1, 2) tail */
    g->len = 2;
    b[g->snake[0]] = 1; b[g->snake[1]] = 1;              /* :49-51 */
    memcpy(g->hist[1], b, (size_t)bs * bs);
    memcpy(g->hist[2], b, (size_t)bs * bs);
    g->hist_len = n_frames;                              /* :53 n_frames copies */
    g->dir = -1;                                         /* :65 (0,0) */
    g->prev_dir = 0;                                     /* :66 (-1,0) = U */
    g->n_food = n_food;
    memcpy(g->food, food, (size_t)n_food * sizeof(int32_t));
}

/* utils.jl:7-10 */
int orc_available_actions(int prev_dir, int32_t out[3]) {
    int n = 0;
    for (int a = 0; a < 4; a++)
        if (a != (prev_dir ^ 1)) out[n++] = a;
    return n;
}

/* utils.jl:13-40 */
static int sample_food(orc_game *g) {
    int8_t *board = g->hist[0];
    int n = g->bs * g->bs, any = 0;
    for (int c = 0; c < n; c++) if (board[c] == 0) { any = 1; break; }
    if (!any) return 0;                                   /* :18-21 */
    int food_pos = -1;
    for (int k = 0; k < g->n_food; k++) {                 /* :25-34 */
        int f = g->food[k];
        if (board[f] == 0) {
            food_pos = f;
            int idx = -1;                                 /* findfirst(==(f), food_list) */
            for (int q = 0; q < g->n_food; q++) if (g->food[q] == f) { idx = q; break; }
            if (idx >= 0) {
                memmove(&g->food[idx], &g->food[idx + 1], (size_t)(g->n_food - idx - 1) * sizeof(int32_t));
                g->n_food--;
            }
            break;
        }
    }
    if (food_pos < 0) { g->fault = 1; return 2; }         /* :37 board[0] -> BoundsError */
    board[food_pos] = 2;
    return 0;
}

/* utils.jl:43-52 */
static void update_board(orc_game *g) {
    int8_t *board = g->hist[0];
    int n = g->bs * g->bs;
    for (int c = 0; c < n; c++) if (board[c] == 1) board[c] = 0;
    for (int k = 0; k < g->len; k++) board[g->snake[k]] = 1;
}

/* utils.jl:55-58 */
static int check_collision(const orc_game *g) {
    int head = g->snake[0], cnt = 0;
    for (int k = 0; k < g->len; k++) cnt += (g->snake[k] == head);
    return g->hist[0][head] == -1 || cnt > 1 || (g->dir >= 0 && (g->prev_dir ^ 1) == g->dir);
}

/* utils.jl:66-81 */
static int grow_maybe(orc_game *g) {
    int st = 0;
    int nh = g->snake[0] + dir_delta(g->bs, g->dir);
    memmove(&g->snake[1], &g->snake[0], (size_t)g->len * sizeof(int16_t));   /* pushfirst! */
    g->snake[0] = (int16_t)nh; g->len++;
    if (g->hist[0][nh] == 2) {
        g->score += 1;
        g->reward = 1.0f;
        st = sample_food(g);
    } else {
        g->len--;                                         /* remove_tail! = pop! */
        g->reward = -0.01f;
    }
    return st;
}

/* utils.jl:85-96 */
static int move_wrapper(orc_game *g) {
    int st = grow_maybe(g);
    if (check_collision(g) || g->hist_len > g->max_hist) {
        g->lost = 1;
        g->reward = -1.0f;
    }
    update_board(g);
    g->prev_dir = g->dir;
    return st;
}

/* utils.jl:100-109 (board_history keeps its last 3 boards) */
int orc_step(orc_game *g, int dir) {
    int n = g->bs * g->bs;
    memcpy(g->hist[2], g->hist[1], (size_t)n);
    memcpy(g->hist[1], g->hist[0], (size_t)n);
    g->dir = dir;
    int st = move_wrapper(g);
    g->hist_len += 1;                                     /* push!(board_history, deepcopy(board)) */
    g->steps += 1;
    g->episode_reward += g->reward;                       /* utils.jl:207 */
    return st;
}

/* utils.jl:112-132: deepcopy + step! for each available action */
void orc_virtual_mask(const orc_game *g, uint8_t mask[3]) {
    if (g->lost) { mask[0] = mask[1] = mask[2] = 1; return; }
    int32_t av[3];
    orc_available_actions(g->prev_dir, av);
    for (int k = 0; k < 3; k++) {
        orc_game cp = *g;
        orc_step(&cp, av[k]);
        mask[k] = (uint8_t)cp.lost;
    }
}

/* ======================= batched driver =================================== */
struct orc_batch {
    int n, bs, n_frames, max_hist, n_food;
    int32_t food[ORC_MAX_FOOD];
    orc_game *g;
};

orc_batch *orc_batch_create(int n, int bs, int n_frames, int max_hist, const int32_t *food, int n_food) {
    orc_batch *b = (orc_batch *)calloc(1, sizeof *b);
    b->n = n; b->bs = bs; b->n_frames = n_frames; b->max_hist = max_hist; b->n_food = n_food;
    memcpy(b->food, food, (size_t)n_food * sizeof(int32_t));
    b->g = (orc_game *)malloc((size_t)n * sizeof(orc_game));
    for (int e = 0; e < n; e++) orc_game_init(&b->g[e], bs, n_frames, max_hist, food, n_food);
    return b;
}
void orc_batch_destroy(orc_batch *b) { if (b) { free(b->g); free(b); } }

int orc_batch_step(orc_batch *b, const uint8_t *act, float *reward, uint8_t *done, uint8_t *mask3,
                   uint8_t *dir_taken, uint8_t *prev_dir, int8_t *frames) {
    int status = 0, n = b->bs * b->bs, C = b->n_frames;
    for (int e = 0; e < b->n; e++) {
        orc_game *g = &b->g[e];
        int32_t av[3];
        orc_available_actions(g->prev_dir, av);
        int d = av[act[e] % 3];
        if (prev_dir) prev_dir[e] = (uint8_t)g->prev_dir;
        if (dir_taken) dir_taken[e] = (uint8_t)d;
        int st = orc_step(g, d);
        if (st) status = st;
        if (reward) reward[e] = g->reward;
        if (done) done[e] = (uint8_t)g->lost;
        uint8_t m[3];
        orc_virtual_mask(g, m);
        if (!g->lost) {   /* a virtual step that would exhaust the food list also faults */
            int32_t av2[3];
            orc_available_actions(g->prev_dir, av2);
            for (int k = 0; k < 3; k++) {
                orc_game cp = *g;
                if (orc_step(&cp, av2[k]) == 2) { g->fault = 1; status = 2; }
            }
        }
        if (mask3) memcpy(mask3 + 3 * e, m, 3);
        if (frames) {   /* b_{t-C} .. b_t, oldest first */
            int8_t *o = frames + (size_t)e * (C + 1) * n;
            for (int f = 0; f <= C; f++) memcpy(o + (size_t)f * n, g->hist[C - f], (size_t)n);
        }
        if (g->lost) orc_game_init(g, b->bs, b->n_frames, b->max_hist, b->food, b->n_food);   /* auto-reset */
    }
    return status;
}

void orc_batch_boards(const orc_batch *b, int8_t *boards) {
    int n = b->bs * b->bs;
    for (int e = 0; e < b->n; e++) memcpy(boards + (size_t)e * n, b->g[e].hist[0], (size_t)n);
}
void orc_batch_scalars(const orc_batch *b, int32_t *score, int32_t *len, int32_t *steps, int32_t *prev_dir, float *ep) {
    for (int e = 0; e < b->n; e++) {
        const orc_game *g = &b->g[e];
        if (score) score[e] = g->score;
        if (len) len[e] = g->len;
        if (steps) steps[e] = g->steps;
        if (prev_dir) prev_dir[e] = g->prev_dir;
        if (ep) ep[e] = g->episode_reward;
    }
}
/* utils.jl:135-139 assemble_state! (not lost: last n_frames boards, oldest first) */
void orc_batch_states(const orc_batch *b, int8_t *states) {
    int n = b->bs * b->bs, C = b->n_frames;
    for (int e = 0; e < b->n; e++)
        for (int f = 0; f < C; f++)
            memcpy(states + ((size_t)e * C + f) * n, b->g[e].hist[C - 1 - f], (size_t)n);
}

uint64_t orc_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
uint32_t orc_synth_action(uint64_t seed, uint64_t env, uint64_t step) {
    uint64_t h = orc_splitmix64(orc_splitmix64(seed ^ (env * 0xD1B54A32D192ED03ULL)) ^ step);
    return (uint32_t)((h >> 32) % 3);
}

/* ======================= Q-net (structs.jl:127-139) ======================= */
/* Flux Conv = true convolution (kernel flipped), WHCN with dim1 = board row;
 * Flux.flatten is column-major (i, j, c); Dense W is (out, in). */
typedef struct { int off_w1, off_b1, off_w2, off_b2, off_w3, off_b3, off_d1w, off_d1b, off_d2w, off_d2b, P, F1, Wo; } qlayout;
static qlayout qnet_layout(int bs, int C) {
    qlayout L; int o = 0;
    L.Wo = bs - 5; L.F1 = L.Wo * L.Wo * 64;
    L.off_w1 = o; o += 3 * 3 * C * 16; L.off_b1 = o; o += 16;
    L.off_w2 = o; o += 3 * 3 * 16 * 32; L.off_b2 = o; o += 32;
    L.off_w3 = o; o += 6 * 6 * 32 * 64; L.off_b3 = o; o += 64;
    L.off_d1w = o; o += 64 * L.F1; L.off_d1b = o; o += 64;
    L.off_d2w = o; o += 3 * 64; L.off_d2b = o; o += 3;
    L.P = o;
    return L;
}
int64_t orc_qnet_nparams(int bs, int C) { return qnet_layout(bs, C).P; }

/* One relu layer's decision per element: active = s > 0 (the reference's
 * relu), or the decision given in mk (kink-aware parity tests: the device's own
 * decisions, see orc_qnet_backward_ex). mo (if set) receives the decisions, mg
 * the margin s / (|b| + sum |w x|): how close the pre-activation is to the kink
 * relative to the dot product's own scale. */
static void conv_fwd_k(int H, int Cin, int Cout, int K, int pad, const float *w, const float *b,
                       const double *x, double *y, const uint8_t *mk, uint8_t *mo, double *mg) {
    int Ho = H + 2 * pad - K + 1;
    for (int co = 0; co < Cout; co++)
        for (int j = 0; j < Ho; j++)
            for (int i = 0; i < Ho; i++) {
                double s = b[co], sa = fabs((double)b[co]);
                for (int ci = 0; ci < Cin; ci++)
                    for (int v = 0; v < K; v++) {
                        int xj = j + (K - 1 - v) - pad;
                        if (xj < 0 || xj >= H) continue;
                        for (int u = 0; u < K; u++) {
                            int xi = i + (K - 1 - u) - pad;
                            if (xi < 0 || xi >= H) continue;
                            double t = (double)w[u + v * K + ci * K * K + co * K * K * Cin] * x[xi + xj * H + ci * H * H];
                            s += t;
                            sa += fabs(t);
                        }
                    }
                int oi = i + j * Ho + co * Ho * Ho;
                int act = mk ? mk[oi] != 0 : s > 0;
                y[oi] = act ? s : 0;                             /* relu */
                if (mo) mo[oi] = (uint8_t)act;
                if (mg) mg[oi] = sa > 0 ? s / sa : 0.0;
            }
}
static void conv_fwd(int H, int Cin, int Cout, int K, int pad, const float *w, const float *b,
                     const double *x, double *y) {
    conv_fwd_k(H, Cin, Cout, K, pad, w, b, x, y, NULL, NULL, NULL);
}
/* dz = dy .* relu'(z) with relu' = the layer's decisions (act) or y > 0;
 * accumulates dw, db; dx (if non-NULL) overwritten */
static void conv_bwd_k(int H, int Cin, int Cout, int K, int pad, const float *w, const double *x,
                       const uint8_t *act, const double *y, const double *dy, double *dw, double *db, double *dx) {
    int Ho = H + 2 * pad - K + 1;
    if (dx) memset(dx, 0, sizeof(double) * (size_t)H * H * Cin);
    for (int co = 0; co < Cout; co++)
        for (int j = 0; j < Ho; j++)
            for (int i = 0; i < Ho; i++) {
                int oi = i + j * Ho + co * Ho * Ho;
                if (act ? !act[oi] : !(y[oi] > 0)) continue;
                double dz = dy[oi];
                db[co] += dz;
                for (int ci = 0; ci < Cin; ci++)
                    for (int v = 0; v < K; v++) {
                        int xj = j + (K - 1 - v) - pad;
                        if (xj < 0 || xj >= H) continue;
                        for (int u = 0; u < K; u++) {
                            int xi = i + (K - 1 - u) - pad;
                            if (xi < 0 || xi >= H) continue;
                            int wi = u + v * K + ci * K * K + co * K * K * Cin;
                            int xx = xi + xj * H + ci * H * H;
                            dw[wi] += dz * x[xx];
                            if (dx) dx[xx] += dz * (double)w[wi];
                        }
                    }
            }
}
static void conv_bwd(int H, int Cin, int Cout, int K, int pad, const float *w, const double *x,
                     const double *y, const double *dy, double *dw, double *db, double *dx) {
    conv_bwd_k(H, Cin, Cout, K, pad, w, x, NULL, y, dy, dw, db, dx);
}

typedef struct { double *a1, *a2, *a3, *h1; uint8_t *m; } acts;   /* m: decisions [a1 | a2 | a3 | h1] */
static int64_t relu_count(const qlayout *L, int bs) { return (int64_t)bs * bs * 48 + (int64_t)L->Wo * L->Wo * 64 + 64; }
/* mk / mg: this sample's [a1 | a2 | a3 | h1] slices (or NULL) */
static void fwd_one_k(const qlayout *L, int bs, int C, const float *p, const double *x, acts *A, double *q,
                      const uint8_t *mk, double *mg) {
    const int64_t o2 = (int64_t)bs * bs * 16, o3 = o2 + (int64_t)bs * bs * 32, oh = o3 + (int64_t)L->Wo * L->Wo * 64;
    conv_fwd_k(bs, C, 16, 3, 1, p + L->off_w1, p + L->off_b1, x, A->a1, mk, A->m, mg);
    conv_fwd_k(bs, 16, 32, 3, 1, p + L->off_w2, p + L->off_b2, A->a1, A->a2, mk ? mk + o2 : NULL, A->m + o2,
               mg ? mg + o2 : NULL);
    conv_fwd_k(bs, 32, 64, 6, 0, p + L->off_w3, p + L->off_b3, A->a2, A->a3, mk ? mk + o3 : NULL, A->m + o3,
               mg ? mg + o3 : NULL);
    for (int o = 0; o < 64; o++) {                               /* Dense(F1 -> 64, relu) */
        double s = p[L->off_d1b + o], sa = fabs((double)p[L->off_d1b + o]);
        for (int f = 0; f < L->F1; f++) {
            double t = (double)p[L->off_d1w + o + f * 64] * A->a3[f];
            s += t;
            sa += fabs(t);
        }
        int act = mk ? mk[oh + o] != 0 : s > 0;
        A->h1[o] = act ? s : 0;
        A->m[oh + o] = (uint8_t)act;
        if (mg) mg[oh + o] = sa > 0 ? s / sa : 0.0;
    }
    for (int a = 0; a < 3; a++) {                                /* Dense(64 -> 3) */
        double s = p[L->off_d2b + a];
        for (int o = 0; o < 64; o++) s += (double)p[L->off_d2w + a + o * 3] * A->h1[o];
        q[a] = s;
    }
}
static void fwd_one(const qlayout *L, int bs, int C, const float *p, const double *x, acts *A, double *q) {
    fwd_one_k(L, bs, C, p, x, A, q, NULL, NULL);
}
static acts acts_alloc(int bs) {
    acts A; int Wo = bs - 5;
    A.a1 = (double *)malloc(sizeof(double) * bs * bs * 16);
    A.a2 = (double *)malloc(sizeof(double) * bs * bs * 32);
    A.a3 = (double *)malloc(sizeof(double) * Wo * Wo * 64);
    A.h1 = (double *)malloc(sizeof(double) * 64);
    A.m = (uint8_t *)malloc((size_t)bs * bs * 48 + (size_t)Wo * Wo * 64 + 64);
    return A;
}
static void acts_free(acts *A) { free(A->a1); free(A->a2); free(A->a3); free(A->h1); free(A->m); }

void orc_qnet_forward(int bs, int C, const float *params, int B, const double *x, double *q) {
    qlayout L = qnet_layout(bs, C);
    acts A = acts_alloc(bs);
    for (int b = 0; b < B; b++) fwd_one(&L, bs, C, params, x + (size_t)b * C * bs * bs, &A, q + 3 * b);
    acts_free(&A);
}

int64_t orc_qnet_relu_count(int bs, int C) { qlayout L = qnet_layout(bs, C); return relu_count(&L, bs); }

/* orc_qnet_backward with the relu decisions of every sample given (mask_in,
 * [B][relu_count]: a1 (bs*bs*16), a2 (bs*bs*32), a3 (Wo*Wo*64) channel-major
 * like the activations, then h1 (64); NULL = the reference's z > 0), and the
 * decisions taken / margins returned (mask_out, margin_out, same layout, may be
 * NULL). A kink (z within rounding of 0) makes the gradient discontinuous: an
 * fp32 device may decide it the other way than fp64; the parity tests use this
 * to check such differences are kink decisions and nothing else. */
void orc_qnet_backward_ex(int bs, int C, const float *p, int B, const double *x, const double *dq, double *g,
                          const uint8_t *mask_in, uint8_t *mask_out, double *margin_out) {
    qlayout L = qnet_layout(bs, C);
    acts A = acts_alloc(bs);
    const int64_t NR = relu_count(&L, bs);
    const int64_t o2 = (int64_t)bs * bs * 16, o3 = o2 + (int64_t)bs * bs * 32, oh = o3 + (int64_t)L.Wo * L.Wo * 64;
    double *dh1 = (double *)malloc(sizeof(double) * 64);
    double *da3 = (double *)malloc(sizeof(double) * L.F1);
    double *da2 = (double *)malloc(sizeof(double) * bs * bs * 32);
    double *da1 = (double *)malloc(sizeof(double) * bs * bs * 16);
    double q[3];
    for (int b = 0; b < B; b++) {
        const double *xb = x + (size_t)b * C * bs * bs;
        const double *d = dq + 3 * b;
        fwd_one_k(&L, bs, C, p, xb, &A, q, mask_in ? mask_in + b * NR : NULL, margin_out ? margin_out + b * NR : NULL);
        if (mask_out) memcpy(mask_out + b * NR, A.m, (size_t)NR);
        for (int a = 0; a < 3; a++) {
            g[L.off_d2b + a] += d[a];
            for (int o = 0; o < 64; o++) g[L.off_d2w + a + o * 3] += d[a] * A.h1[o];
        }
        for (int o = 0; o < 64; o++) {
            double s = 0;
            for (int a = 0; a < 3; a++) s += d[a] * (double)p[L.off_d2w + a + o * 3];
            dh1[o] = A.m[oh + o] ? s : 0;
        }
        memset(da3, 0, sizeof(double) * L.F1);
        for (int o = 0; o < 64; o++) {
            if (dh1[o] == 0) continue;
            g[L.off_d1b + o] += dh1[o];
            for (int f = 0; f < L.F1; f++) {
                g[L.off_d1w + o + f * 64] += dh1[o] * A.a3[f];
                da3[f] += dh1[o] * (double)p[L.off_d1w + o + f * 64];
            }
        }
        conv_bwd_k(bs, 32, 64, 6, 0, p + L.off_w3, A.a2, A.m + o3, A.a3, da3, g + L.off_w3, g + L.off_b3, da2);
        conv_bwd_k(bs, 16, 32, 3, 1, p + L.off_w2, A.a1, A.m + o2, A.a2, da2, g + L.off_w2, g + L.off_b2, da1);
        conv_bwd_k(bs, C, 16, 3, 1, p + L.off_w1, xb, A.m, A.a1, da1, g + L.off_w1, g + L.off_b1, NULL);
    }
    free(dh1); free(da3); free(da2); free(da1);
    acts_free(&A);
}

void orc_qnet_backward(int bs, int C, const float *p, int B, const double *x, const double *dq, double *g) {
    orc_qnet_backward_ex(bs, C, p, B, x, dq, g, NULL, NULL, NULL);
}

/* utils.jl:448-464: q_next = t_net(s'); q_next[mask] = -100; max; target =
 * r + 0.97*max*(1-done) (Float64); loss = huber(Q(s)[a], target; delta=1, mean). */
double orc_dqn_loss_grad_ex(int bs, int C, const float *qp, const float *tp, int B, const double *s,
                            const int32_t *a_idx, const float *r, const double *s_next, const uint8_t *done,
                            const uint8_t *mask3, double gamma, double *grad, double *target_out,
                            const uint8_t *relu_in, uint8_t *relu_out, double *margin_out) {
    double *qn = (double *)malloc(sizeof(double) * 3 * B);
    double *qs = (double *)malloc(sizeof(double) * 3 * B);
    double *dq = (double *)calloc((size_t)3 * B, sizeof(double));
    orc_qnet_forward(bs, C, tp, B, s_next, qn);
    orc_qnet_forward(bs, C, qp, B, s, qs);
    double loss = 0;
    for (int b = 0; b < B; b++) {
        double mx = -INFINITY;
        for (int a = 0; a < 3; a++) {
            double v = mask3[3 * b + a] ? -100.0 : qn[3 * b + a];
            if (v > mx) mx = v;
        }
        double tgt = (double)r[b] + gamma * mx * (double)(1 - done[b]);
        if (target_out) target_out[b] = tgt;
        double e = qs[3 * b + a_idx[b]] - tgt, ae = fabs(e);
        double li = ae < 1.0 ? 0.5 * e * e : (ae - 0.5);
        loss += li;
        dq[3 * b + a_idx[b]] = (ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / B;
    }
    loss /= B;
    if (grad) orc_qnet_backward_ex(bs, C, qp, B, s, dq, grad, relu_in, relu_out, margin_out);
    free(qn); free(qs); free(dq);
    return loss;
}
double orc_dqn_loss_grad(int bs, int C, const float *qp, const float *tp, int B, const double *s,
                         const int32_t *a_idx, const float *r, const double *s_next, const uint8_t *done,
                         const uint8_t *mask3, double gamma, double *grad, double *target_out) {
    return orc_dqn_loss_grad_ex(bs, C, qp, tp, B, s, a_idx, r, s_next, done, mask3, gamma, grad, target_out,
                                NULL, NULL, NULL);
}

/* ======================= deeper bf16 Q-net (configs[2]) =====================
 * BASELINE.json configs[2] names a "deeper conv Q-net, bf16" with no reference
 * counterpart (builder-defined). It extends structs.jl:127-139
 * by one more 3x3 convolution and wider channels, same Flux conventions:
 *   Conv(3,3,C=>32,relu;pad=1) Conv(3,3,32=>32,relu;pad=1) Conv(3,3,32=>64,relu;pad=1)
 *   Conv(6,6,64=>64,relu) flatten Dense((bs-5)^2*64=>64,relu) Dense(64=>3)
 * bf16 semantics of the device path, restated here exactly:
 *   - conv and Dense1 weight matrices are used rounded to bf16 (RNE); biases
 *     and Dense2 stay fp32;
 *   - every conv output (after bias + relu) is rounded to bf16;
 *   - backward: the relu-masked gradient entering each conv / Dense1 layer is
 *     rounded to bf16 before it is multiplied (both the weight- and the data-
 *     gradient products); Dense2 and the TD/Huber head stay fp32/fp64.
 * Sums are fp64 here (fp32 on the device). */
static float bf16r(double v) {
    float f = (float)v;
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return f;
    u += 0x7fffu + ((u >> 16) & 1u);
    u &= 0xffff0000u;
    memcpy(&f, &u, 4);
    return f;
}
typedef struct { int cin[4], cout[4], ks[4], pad[4]; int off_w[4], off_b[4], off_d1w, off_d1b, off_d2w, off_d2b, P, F1, Wo; } dlayout;
static dlayout deep_layout(int bs, int C) {
    dlayout L; int o = 0;
    const int ci[4] = {C, 32, 32, 64}, co[4] = {32, 32, 64, 64}, ks[4] = {3, 3, 3, 6}, pd[4] = {1, 1, 1, 0};
    for (int l = 0; l < 4; l++) {
        L.cin[l] = ci[l]; L.cout[l] = co[l]; L.ks[l] = ks[l]; L.pad[l] = pd[l];
        L.off_w[l] = o; o += ks[l] * ks[l] * ci[l] * co[l];
        L.off_b[l] = o; o += co[l];
    }
    L.Wo = bs - 5; L.F1 = L.Wo * L.Wo * 64;
    L.off_d1w = o; o += 64 * L.F1; L.off_d1b = o; o += 64;
    L.off_d2w = o; o += 3 * 64; L.off_d2b = o; o += 3;
    L.P = o;
    return L;
}
int64_t orc_deep_nparams(int bs, int C) { return deep_layout(bs, C).P; }

/* params with the conv / Dense1 weight matrices rounded to bf16 */
static float *deep_rounded(const dlayout *L, const float *p) {
    float *r = (float *)malloc(sizeof(float) * L->P);
    memcpy(r, p, sizeof(float) * L->P);
    for (int l = 0; l < 4; l++)
        for (int i = L->off_w[l]; i < L->off_b[l]; i++) r[i] = bf16r(p[i]);
    for (int i = L->off_d1w; i < L->off_d1b; i++) r[i] = bf16r(p[i]);
    return r;
}
typedef struct { double *a[4], *h1; } dacts;
static dacts dacts_alloc(int bs) {
    dacts A; const int Wo = bs - 5;
    A.a[0] = (double *)malloc(sizeof(double) * bs * bs * 32);
    A.a[1] = (double *)malloc(sizeof(double) * bs * bs * 32);
    A.a[2] = (double *)malloc(sizeof(double) * bs * bs * 64);
    A.a[3] = (double *)malloc(sizeof(double) * Wo * Wo * 64);
    A.h1 = (double *)malloc(sizeof(double) * 64);
    return A;
}
static void dacts_free(dacts *A) { for (int l = 0; l < 4; l++) free(A->a[l]); free(A->h1); }
static void deep_fwd_one(const dlayout *L, int bs, const float *pr, const double *x, dacts *A, double *q) {
    const double *in = x;
    int H = bs;
    for (int l = 0; l < 4; l++) {
        conv_fwd(H, L->cin[l], L->cout[l], L->ks[l], L->pad[l], pr + L->off_w[l], pr + L->off_b[l], in, A->a[l]);
        const int Ho = H + 2 * L->pad[l] - L->ks[l] + 1, n = Ho * Ho * L->cout[l];
        for (int i = 0; i < n; i++) A->a[l][i] = bf16r(A->a[l][i]);
        in = A->a[l];
        H = Ho;
    }
    for (int o = 0; o < 64; o++) {
        double s = pr[L->off_d1b + o];
        for (int f = 0; f < L->F1; f++) s += (double)pr[L->off_d1w + o + f * 64] * A->a[3][f];
        A->h1[o] = s > 0 ? s : 0;
    }
    for (int a = 0; a < 3; a++) {
        double s = pr[L->off_d2b + a];
        for (int o = 0; o < 64; o++) s += (double)pr[L->off_d2w + a + o * 3] * A->h1[o];
        q[a] = s;
    }
}
void orc_deep_forward(int bs, int C, const float *params, int B, const double *x, double *q) {
    dlayout L = deep_layout(bs, C);
    float *pr = deep_rounded(&L, params);
    dacts A = dacts_alloc(bs);
    for (int b = 0; b < B; b++) deep_fwd_one(&L, bs, pr, x + (size_t)b * C * bs * bs, &A, q + 3 * b);
    dacts_free(&A);
    free(pr);
}
/* conv_bwd with the masked gradient rounded to bf16 first (the device's MFMA operand) */
static void conv_bwd_bf16(int H, int Cin, int Cout, int K, int pad, const float *w, const double *x,
                          const double *y, const double *dy, double *dw, double *db, double *dx) {
    const int Ho = H + 2 * pad - K + 1, n = Ho * Ho * Cout;
    double *dr = (double *)malloc(sizeof(double) * n);
    for (int i = 0; i < n; i++) dr[i] = y[i] > 0 ? (double)bf16r(dy[i]) : 0.0;
    /* conv_bwd skips y <= 0 itself; feed it the rounded values */
    conv_bwd(H, Cin, Cout, K, pad, w, x, y, dr, dw, db, dx);
    free(dr);
}
void orc_deep_backward(int bs, int C, const float *p, int B, const double *x, const double *dq, double *g) {
    dlayout L = deep_layout(bs, C);
    float *pr = deep_rounded(&L, p);
    dacts A = dacts_alloc(bs);
    const int Wo = L.Wo;
    double *dh1 = (double *)malloc(sizeof(double) * 64);
    double *da[4];
    da[0] = (double *)malloc(sizeof(double) * bs * bs * 32);
    da[1] = (double *)malloc(sizeof(double) * bs * bs * 32);
    da[2] = (double *)malloc(sizeof(double) * bs * bs * 64);
    da[3] = (double *)malloc(sizeof(double) * Wo * Wo * 64);
    double q[3];
    for (int b = 0; b < B; b++) {
        const double *xb = x + (size_t)b * C * bs * bs;
        const double *d = dq + 3 * b;
        deep_fwd_one(&L, bs, pr, xb, &A, q);
        for (int a = 0; a < 3; a++) {
            g[L.off_d2b + a] += d[a];
            for (int o = 0; o < 64; o++) g[L.off_d2w + a + o * 3] += d[a] * A.h1[o];
        }
        for (int o = 0; o < 64; o++) {
            double s = 0;
            for (int a = 0; a < 3; a++) s += d[a] * (double)p[L.off_d2w + a + o * 3];
            dh1[o] = A.h1[o] > 0 ? (double)bf16r(s) : 0;
        }
        memset(da[3], 0, sizeof(double) * L.F1);
        for (int o = 0; o < 64; o++) {
            if (dh1[o] == 0) continue;
            g[L.off_d1b + o] += dh1[o];
            for (int f = 0; f < L.F1; f++) {
                g[L.off_d1w + o + f * 64] += dh1[o] * A.a[3][f];
                da[3][f] += dh1[o] * (double)pr[L.off_d1w + o + f * 64];
            }
        }
        for (int l = 3; l >= 0; l--) {
            const int H = l == 3 ? bs : bs;   /* every conv input is bs x bs */
            const double *xin = l == 0 ? xb : A.a[l - 1];
            conv_bwd_bf16(H, L.cin[l], L.cout[l], L.ks[l], L.pad[l], pr + L.off_w[l], xin, A.a[l], da[l],
                          g + L.off_w[l], g + L.off_b[l], l == 0 ? NULL : da[l - 1]);
        }
    }
    free(dh1);
    for (int l = 0; l < 4; l++) free(da[l]);
    dacts_free(&A);
    free(pr);
}
double orc_deep_loss_grad(int bs, int C, const float *qp, const float *tp, int B, const double *s,
                          const int32_t *a_idx, const float *r, const double *s_next, const uint8_t *done,
                          const uint8_t *mask3, double gamma, double *grad, double *target_out) {
    double *qn = (double *)malloc(sizeof(double) * 3 * B);
    double *qs = (double *)malloc(sizeof(double) * 3 * B);
    double *dq = (double *)calloc((size_t)3 * B, sizeof(double));
    orc_deep_forward(bs, C, tp, B, s_next, qn);
    orc_deep_forward(bs, C, qp, B, s, qs);
    double loss = 0;
    for (int b = 0; b < B; b++) {
        double mx = -INFINITY;
        for (int a = 0; a < 3; a++) {
            /* the device keeps Q in fp32: the masked max is over fp32 values */
            double v = mask3[3 * b + a] ? -100.0 : (double)(float)qn[3 * b + a];
            if (v > mx) mx = v;
        }
        double tgt = (double)r[b] + gamma * mx * (double)(1 - done[b]);
        if (target_out) target_out[b] = tgt;
        double e = qs[3 * b + a_idx[b]] - tgt, ae = fabs(e);
        loss += ae < 1.0 ? 0.5 * e * e : (ae - 0.5);
        dq[3 * b + a_idx[b]] = (ae < 1.0 ? e : (e > 0 ? 1.0 : -1.0)) / B;
    }
    loss /= B;
    if (grad) orc_deep_backward(bs, C, qp, B, s, dq, grad);
    free(qn); free(qs); free(dq);
    return loss;
}

/* Optimisers.jl RMSProp apply! (non-centred), Float32:
 *   quad = rho*quad + (1-rho)*dx^2 ; x -= dx*eta/(sqrt(quad)+eps) */
void orc_rmsprop(int64_t P, float *theta, float *acc, const float *grad, float eta, float rho, float eps) {
    float omr = 1.0f - rho;
    for (int64_t i = 0; i < P; i++) {
        float g = grad[i];
        float q = rho * acc[i] + omr * (g * g);
        acc[i] = q;
        float upd = (g * eta) / (sqrtf(q) + eps);
        theta[i] = theta[i] - upd;
    }
}

/* ======================= Laplace ========================================== */
/* compute_D.jl:21-27 fit! per column, then :80-81 D .-= mean */
void orc_welford_center(int64_t P, int K, double *D, double *mean, double *var) {
    double *m2 = (double *)calloc((size_t)P, sizeof(double));
    for (int64_t p = 0; p < P; p++) mean[p] = 0.0;
    for (int k = 0; k < K; k++) {
        const double *x = D + (size_t)k * P;
        double n = (double)(k + 1);
        for (int64_t p = 0; p < P; p++) {
            double d = x[p] - mean[p];
            mean[p] += d / n;
            m2[p] += d * (x[p] - mean[p]);
        }
    }
    for (int64_t p = 0; p < P; p++) var[p] = m2[p] / (double)(K - 1 > 1 ? K - 1 : 1);
    for (int k = 0; k < K; k++)
        for (int64_t p = 0; p < P; p++) D[(size_t)k * P + p] -= mean[p];
    free(m2);
}

void orc_gram(int64_t P, int K, const double *D, double *G) {
    for (int a = 0; a < K; a++)
        for (int b = 0; b <= a; b++) {
            double s = 0;
            const double *x = D + (size_t)a * P, *y = D + (size_t)b * P;
            for (int64_t p = 0; p < P; p++) s += x[p] * y[p];
            G[a + (size_t)b * K] = s; G[b + (size_t)a * K] = s;
        }
}

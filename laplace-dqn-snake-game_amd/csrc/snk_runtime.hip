// snk_runtime.hip — runtime plumbing of libsnakehip: error reporting, the
// library stream, device memory helpers, and the host-side food list
// (structs.jl:70, Julia Random.Xoshiro seeded through SHA-256).
#include <cstdarg>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include <atomic>

#include "snk_internal.hpp"

namespace snk {

static thread_local std::string g_err;
static thread_local hipStream_t g_user_stream = nullptr;
static thread_local bool g_user_stream_set = false;
// snk_set_arith knobs, production defaults (SNK_ARITH_* in include/snakehip.h)
// (relaxed atomics: a knob set on one thread while another launches is not a data race)
static std::atomic<int> g_arith[SNK_ARITH_COUNT] = {1, 1, 1, 1, 0, 0, 1, 1, 1, 1};
static hipStream_t g_own_stream[64] = {};

void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

void set_lds_limit(const void *kernel, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, size_t> done;
    int dev = 0;
    SNK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    size_t &have = done[{kernel, dev}];
    if (bytes <= have) return;
    SNK_HIP(hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    have = bytes;
}

int cu_count() {
    static std::mutex mu;
    static std::map<int, int> cus;
    int dev = 0;
    SNK_HIP(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(mu);
    int &n = cus[dev];
    if (n == 0) {
        SNK_HIP(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
        n = n > 0 ? n : 1;
    }
    return n;
}

int arith(int knob) { return g_arith[knob].load(std::memory_order_relaxed); }

hipStream_t stream() {
    if (g_user_stream_set) return g_user_stream;
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!g_own_stream[dev]) {
        hipStream_t s;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
        g_own_stream[dev] = s;
    }
    return g_own_stream[dev];
}

// ---------------------------------------------------------------- SHA-256
namespace {
struct Sha256 {
    uint32_t h[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                     0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
    uint8_t buf[64];
    uint64_t len = 0;
    int fill = 0;
    static uint32_t ror(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
    void block(const uint8_t *p) {
        static const uint32_t k[64] = {
            0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
            0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
            0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
            0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
            0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
            0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
            0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
            0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};
        uint32_t w[64];
        for (int i = 0; i < 16; ++i)
            w[i] = (uint32_t)p[4 * i] << 24 | (uint32_t)p[4 * i + 1] << 16 | (uint32_t)p[4 * i + 2] << 8 |
                   p[4 * i + 3];
        for (int i = 16; i < 64; ++i)
            w[i] = w[i - 16] + (ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3)) + w[i - 7] +
                   (ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10));
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int i = 0; i < 64; ++i) {
            uint32_t t1 = hh + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + k[i] + w[i];
            uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
    }
    void update(const uint8_t *p, size_t n) {
        for (size_t i = 0; i < n; ++i) {
            buf[fill++] = p[i];
            ++len;
            if (fill == 64) { block(buf); fill = 0; }
        }
    }
    void digest(uint8_t out[32]) {
        const uint64_t bits = len * 8;
        const uint8_t one = 0x80, zero = 0;
        update(&one, 1);
        while (fill != 56) update(&zero, 1);
        uint8_t lb[8];
        for (int i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
        update(lb, 8);
        for (int i = 0; i < 8; ++i)
            for (int j = 0; j < 4; ++j) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
    }
};

// Julia `Xoshiro(seed)`: state words = first four little-endian UInt64 of
// SHA-256 over the seed's little-endian UInt32 words.
struct JuliaXoshiro {
    uint64_t s[4];
    explicit JuliaXoshiro(uint32_t seed) {
        uint8_t w[4], dg[32];
        for (int i = 0; i < 4; ++i) w[i] = (uint8_t)(seed >> (8 * i));
        Sha256 sha;
        sha.update(w, 4);
        sha.digest(dg);
        for (int k = 0; k < 4; ++k) {
            uint64_t v = 0;
            for (int i = 7; i >= 0; --i) v = (v << 8) | dg[8 * k + i];
            s[k] = v;
        }
    }
    uint64_t next() {  // xoshiro256++
        auto rotl = [](uint64_t x, int k) { return (x << k) | (x >> (64 - k)); };
        const uint64_t res = rotl(s[0] + s[3], 23) + s[0];
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t; s[3] = rotl(s[3], 45);
        return res;
    }
    int64_t range(int64_t a, int64_t b) {  // rand(rng, a:b): Lemire nearly-divisionless
        const uint64_t sz = (uint64_t)(b - a) + 1;
        unsigned __int128 m = (unsigned __int128)next() * sz;
        uint64_t l = (uint64_t)m;
        if (l < sz) {
            const uint64_t thr = (0 - sz) % sz;
            while (l < thr) {
                m = (unsigned __int128)next() * sz;
                l = (uint64_t)m;
            }
        }
        return a + (int64_t)(uint64_t)(m >> 64);
    }
};
}  // namespace

}  // namespace snk

using namespace snk;

extern "C" const char *snk_last_error(void) { return g_err.c_str(); }

extern "C" int snk_version(int32_t *v) {
    return guard([&] {
        SNK_CHECK(v, SNK_ERR_INVALID, "NULL argument");
        *v = 10000;  // 1.0.0
    });
}

extern "C" int snk_device_count(int32_t *n) {
    return guard([&] {
        SNK_CHECK(n, SNK_ERR_INVALID, "NULL argument");
        int c = 0;
        SNK_HIP(hipGetDeviceCount(&c));
        *n = c;
    });
}

extern "C" int snk_set_device(int32_t dev) {
    return guard([&] { SNK_HIP(hipSetDevice(dev)); });
}

extern "C" int snk_set_stream(void *s) {
    return guard([&] {
        g_user_stream = reinterpret_cast<hipStream_t>(s);
        g_user_stream_set = s != nullptr;
    });
}

extern "C" int snk_set_arith(int32_t knob, int32_t value) {
    return guard([&] {
        SNK_CHECK(knob >= 0 && knob < SNK_ARITH_COUNT, SNK_ERR_INVALID, "unknown arithmetic knob %d", knob);
        SNK_CHECK(value == 0 || value == 1, SNK_ERR_INVALID, "arithmetic knob %d: value %d is not 0 or 1", knob,
                  value);
        g_arith[knob].store(value, std::memory_order_relaxed);
    });
}

extern "C" int snk_get_arith(int32_t knob, int32_t *value) {
    return guard([&] {
        SNK_CHECK(value && knob >= 0 && knob < SNK_ARITH_COUNT, SNK_ERR_INVALID, "unknown arithmetic knob %d", knob);
        *value = g_arith[knob].load(std::memory_order_relaxed);
    });
}

extern "C" int snk_synchronize(void) {
    return guard([&] { SNK_HIP(hipStreamSynchronize(stream())); });
}

extern "C" int snk_malloc(void **p, int64_t bytes) {
    return guard([&] {
        SNK_CHECK(p && bytes >= 0, SNK_ERR_INVALID, "bad malloc arguments");
        *p = dalloc<uint8_t>((size_t)bytes);
    });
}

extern "C" int snk_free(void *p) {
    return guard([&] { SNK_HIP(hipFree(p)); });
}

extern "C" int snk_memcpy_h2d(void *d, const void *h, int64_t n) {
    return guard([&] {
        SNK_HIP(hipMemcpyAsync(d, h, (size_t)n, hipMemcpyHostToDevice, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_memcpy_d2h(void *h, const void *d, int64_t n) {
    return guard([&] {
        SNK_HIP(hipMemcpyAsync(h, d, (size_t)n, hipMemcpyDeviceToHost, stream()));
        SNK_HIP(hipStreamSynchronize(stream()));
    });
}

extern "C" int snk_memset(void *d, int32_t v, int64_t n) {
    return guard([&] { SNK_HIP(hipMemsetAsync(d, v, (size_t)n, stream())); });
}

extern "C" int snk_food_list(int32_t bs, uint32_t seed, int32_t n, int32_t *cells) {
    return guard([&] {
        SNK_CHECK(cells && n >= 0 && n <= 64 && bs >= 3, SNK_ERR_INVALID, "bad food_list arguments");
        JuliaXoshiro rng(seed);
        for (int k = 0; k < n; ++k) {
            const int64_t r = rng.range(2, bs - 1);  // row drawn first (structs.jl:70)
            const int64_t c = rng.range(2, bs - 1);
            cells[k] = (int32_t)((r - 1) + (c - 1) * bs);
        }
    });
}

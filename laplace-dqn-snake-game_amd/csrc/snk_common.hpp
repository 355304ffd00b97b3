// snk_common.hpp — shared internals of libsnakehip (gfx950 / CDNA4 only).
//
// Status-code error model (include/snakehip.h): every C-ABI entry point
// returns an int status and records a thread-local message readable through
// snk_last_error(). This replaces the reference's Julia exceptions
// (utils.jl:241 error(), structs.jl:113 throw, utils.jl:37 BoundsError).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "snakehip.h"

namespace snk {

void set_error(const char *fmt, ...);
hipStream_t stream();   // the library's current stream (snk_set_stream)

struct Error {
    int code;
};

#define SNK_HIP(call)                                                                  \
    do {                                                                               \
        hipError_t e_ = (call);                                                        \
        if (e_ != hipSuccess) {                                                        \
            ::snk::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #call,             \
                             hipGetErrorString(e_));                                   \
            throw ::snk::Error{SNK_ERR_HIP};                                           \
        }                                                                              \
    } while (0)

#define SNK_CHECK(cond, code, ...)                                                     \
    do {                                                                               \
        if (!(cond)) {                                                                 \
            ::snk::set_error(__VA_ARGS__);                                             \
            throw ::snk::Error{code};                                                  \
        }                                                                              \
    } while (0)

// Wrap a C-ABI body: converts thrown snk::Error / std exceptions to status.
template <class F>
int guard(F &&f) {
    try {
        f();
        return SNK_OK;
    } catch (const Error &e) {
        return e.code;
    } catch (const std::bad_alloc &) {
        set_error("host allocation failed");
        return SNK_ERR_NOMEM;
    } catch (...) {
        set_error("unexpected C++ exception");
        return SNK_ERR_INTERNAL;
    }
}

// Fork/join of independent launch sequences onto side streams: eagerly, or
// under stream capture, where the side streams join the capture through the
// events and become parallel branches of the graph. With no side streams
// every call is a no-op and everything stays on `main`.
enum ForkBits : unsigned { FK_SAMPLE = 1, FK_STATS = 2, FK_TARGET = 4, FK_WGRAD = 8, FK_LOSS = 16 };
struct Fork {
    static constexpr int NS = 3, NE = 48;
    hipStream_t main = nullptr;
    hipStream_t side[NS] = {};
    hipEvent_t ev[NE] = {};
    int nside = 0, next = 0;
    unsigned enable = ~0u;   // FK_* branches taken (others stay on main)
    bool on_side(unsigned bit) const { return nside && (enable & bit); }
    // returns the stream the branch runs on
    hipStream_t fork(int k, unsigned bit) {
        if (!on_side(bit)) return main;
        hipEvent_t e = ev[next++ % NE];
        SNK_HIP(hipEventRecord(e, main));
        SNK_HIP(hipStreamWaitEvent(side[k % nside], e, 0));
        return side[k % nside];
    }
    void join(int k, unsigned bit) {
        if (!on_side(bit)) return;
        hipEvent_t e = ev[next++ % NE];
        SNK_HIP(hipEventRecord(e, side[k % nside]));
        SNK_HIP(hipStreamWaitEvent(main, e, 0));
    }
    void create() {
        for (auto &q : side) SNK_HIP(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
        for (auto &e : ev) SNK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        nside = NS;
    }
    void destroy() {
        for (auto &q : side)
            if (q) (void)hipStreamDestroy(q);
        for (auto &e : ev)
            if (e) (void)hipEventDestroy(e);
        nside = 0;
    }
};

template <class T>
T *dalloc(size_t n) {
    void *p = nullptr;
    if (n == 0) n = 1;
    hipError_t e = hipMalloc(&p, n * sizeof(T));
    if (e != hipSuccess) {
        set_error("hipMalloc(%zu bytes) failed: %s", n * sizeof(T), hipGetErrorString(e));
        throw Error{SNK_ERR_NOMEM};
    }
    return static_cast<T *>(p);
}
inline void dfree(void *p) {
    if (p) (void)hipFree(p);
}

inline void launch_check(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("kernel launch %s failed: %s", what, hipGetErrorString(e));
        throw Error{SNK_ERR_HIP};
    }
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// ---- counter-based RNG shared with the oracle (orc_splitmix64) ------------
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
__host__ __device__ inline uint64_t rng_hash(uint64_t seed, uint64_t a, uint64_t b) {
    return splitmix64(splitmix64(seed ^ (a * 0xD1B54A32D192ED03ULL)) ^ b);
}
// uniform float in [0,1) with 24 random bits
__host__ __device__ inline float rng_uniform(uint64_t h) {
    return (float)(uint32_t)(h >> 40) * (1.0f / 16777216.0f);
}

// Board geometry: frames are Julia column-major boards (cell = i + j*bs,
// 0-based), each stored with a 16-byte padded pitch so one lane moves a frame
// in 16-byte pieces.
inline int frame_pitch(int bs) { return ((bs * bs) + 15) & ~15; }

}  // namespace snk

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
// process-wide GEMM arithmetic selection (snk_set_arith, include/snakehip.h): the
// production kernels unless a test selects a comparison path; read at launch
// (a captured graph keeps the kernels it was captured with)
int arith(int knob);

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

// hipFuncAttributeMaxDynamicSharedMemorySize of a kernel on the current
// device, raised to at least `bytes` (set once per kernel, device and size)
void set_lds_limit(const void *kernel, size_t bytes);

// compute units of the current device (persistent launches: one workgroup per CU)
int cu_count();

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

// Owning device allocation for host-side scopes that may throw (guard()'s
// catch path then frees it). Moves, never copies.
template <class T>
struct DevBuf {
    T *p = nullptr;
    DevBuf() = default;
    explicit DevBuf(size_t n) : p(dalloc<T>(n)) {}
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p) { o.p = nullptr; }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) {
            dfree(p);
            p = o.p;
            o.p = nullptr;
        }
        return *this;
    }
    ~DevBuf() { dfree(p); }
    T *get() const { return p; }
    operator T *() const { return p; }
};

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

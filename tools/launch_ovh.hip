// microbenchmark: per-kernel cost of back-to-back dependent launches, stream vs graph
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void tiny(float *p) { if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1.0f; }
__global__ void wide(float *p, int n) {   // 256 WGs touching n floats
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] += 1.0f;
}
int main() {
    float *d; CK(hipMalloc(&d, 64 << 20)); CK(hipMemset(d, 0, 64 << 20));
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const int N = 200;
    for (int mode = 0; mode < 4; ++mode) {   // 0 tiny stream, 1 tiny graph, 2 wide(1MB) stream, 3 wide graph
        const bool graph = mode & 1; const bool w = mode >= 2;
        auto body = [&]() { for (int i = 0; i < N; ++i) { if (w) wide<<<256, 256, 0, s>>>(d, 1 << 18); else tiny<<<1, 64, 0, s>>>(d); } };
        hipGraphExec_t ge = nullptr;
        if (graph) {
            hipGraph_t g; CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal)); body(); CK(hipStreamEndCapture(s, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, s));
        } else body();
        CK(hipStreamSynchronize(s));
        float best = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipEventRecord(a, s));
            if (graph) CK(hipGraphLaunch(ge, s)); else body();
            CK(hipEventRecord(b, s)); CK(hipEventSynchronize(b));
            float ms; CK(hipEventElapsedTime(&ms, a, b)); best = ms < best ? ms : best;
        }
        printf("{\"mode\": \"%s %s\", \"us_per_kernel\": %.3f}\n", w ? "wide-1MB" : "tiny", graph ? "graph" : "stream", best * 1000.0 / N);
    }
    return 0;
}

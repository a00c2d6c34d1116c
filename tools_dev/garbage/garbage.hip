// Diagnostic neighbours for the decode (run from another process):
//   garbage fill SECS  - waves that leave NaN in LDS and VGPRs on every CU
//   garbage copy SECS  - small host<->device copies (pinned and pageable) in a loop
//   garbage event SECS - timing events recorded around small kernels, elapsed time read
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
__global__ __launch_bounds__(256) void fill(float *sink, int iters) {
    __shared__ float s[16384];
    const float nan = __int_as_float(0x7fc00000);
    for (int i = threadIdx.x; i < 16384; i += 256) s[i] = nan;
    float r[240];
#pragma unroll
    for (int i = 0; i < 240; ++i) r[i] = nan;
    float ag[192];  // accumulation registers too (MFMA neighbours leave values there)
#pragma unroll
    for (int i = 0; i < 192; ++i) asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(ag[i]) : "v"(nan));
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 240; ++i) asm volatile("" : "+v"(r[i]));
#pragma unroll
        for (int i = 0; i < 192; ++i) asm volatile("" : "+a"(ag[i]));
    }
    __syncthreads();
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < 240; ++i) acc += r[i];
    if (acc == 1.0f) sink[threadIdx.x] = s[threadIdx.x];  // never true: keeps r and s live
}
int main(int argc, char **argv) {
    const bool copy = argc > 1 && !strcmp(argv[1], "copy");
    const bool event = argc > 1 && !strcmp(argv[1], "event");
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    const double secs = argc > 2 ? atof(argv[2]) : 10.0;
    float *sink = nullptr, *dbuf = nullptr, *pinned = nullptr;
    std::vector<float> pageable(1 << 16);
    if (hipMalloc(&sink, 1024) != hipSuccess || hipMalloc(&dbuf, 1 << 18) != hipSuccess ||
        hipHostMalloc(&pinned, 1 << 18, hipHostMallocDefault) != hipSuccess)
        return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    auto t0 = std::chrono::steady_clock::now();
    long n = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
        if (event) {
            if (hipEventRecord(e0, st) != hipSuccess) return 1;
            hipLaunchKernelGGL(fill, dim3(64), dim3(256), 0, st, sink, 1);
            if (hipEventRecord(e1, st) != hipSuccess) return 1;
            if (hipEventSynchronize(e1) != hipSuccess) return 1;
            float ms;
            if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
        } else if (copy) {
            if (hipMemcpyAsync(dbuf, pinned, 4096, hipMemcpyHostToDevice, st) != hipSuccess) return 1;
            if (hipMemcpyAsync(pinned, dbuf, 16384, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
            if (hipMemcpyAsync(dbuf, pageable.data(), 4096, hipMemcpyHostToDevice, st) != hipSuccess) return 1;
            if (hipMemcpyAsync(pageable.data(), dbuf, 16384, hipMemcpyDeviceToHost, st) != hipSuccess) return 1;
            if (hipStreamSynchronize(st) != hipSuccess) return 1;
        } else {
            hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, sink, 64);
            if (++n % 64 == 0 && hipStreamSynchronize(st) != hipSuccess) return 1;
        }
        ++n;
    }
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    printf("%s iterations %ld\n", argv[1], n);
    return 0;
}

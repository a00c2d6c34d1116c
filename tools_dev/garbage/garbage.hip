// Diagnostic neighbours for the decode (run from another process):
//   garbage fill SECS  - waves that leave NaN in LDS and VGPRs on every CU
//   garbage copy SECS  - small host<->device copies (pinned and pageable) in a loop
//   garbage event SECS - timing events recorded around small kernels, elapsed time read
//   garbage mfma SECS  - waves issuing back-to-back v_mfma_f32_16x16x32_f16 (registers only)
//   garbage mfmalds SECS - the same plus LDS reads feeding the MFMA B operand
//   garbage valu SECS  - waves issuing back-to-back v_fma_f32 chains (registers only)
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
typedef _Float16 half8_t __attribute__((ext_vector_type(8)));
typedef float floatx4_t __attribute__((ext_vector_type(4)));
template <bool LDS>
__global__ __launch_bounds__(256) void mfma_loop(float *sink, int iters) {
    __shared__ __attribute__((aligned(16))) _Float16 xs[64 * 80];
    const int lane = threadIdx.x & 63;
    half8_t a, b;
    for (int i = 0; i < 8; ++i) { a[i] = (_Float16)(0.01f * (lane + i)); b[i] = (_Float16)(0.02f * (i - lane)); }
    if (LDS) for (int i = threadIdx.x; i < 64 * 80; i += 256) xs[i] = (_Float16)(0.001f * i);
    __syncthreads();
    floatx4_t acc[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (LDS) b = *(const half8_t *)(xs + ((lane + 8 * j + it) & 63) * 80 + 8 * (lane >> 4));
            acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, acc[j], 0, 0, 0);
        }
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j) s += acc[j][0] + acc[j][1] + acc[j][2] + acc[j][3];
    if (s == 12345.f) sink[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void valu_loop(float *sink, int iters) {
    float r[32];
#pragma unroll
    for (int i = 0; i < 32; ++i) r[i] = 0.001f * (threadIdx.x + i);
    for (int it = 0; it < iters * 16; ++it) {
#pragma unroll
        for (int i = 0; i < 32; ++i) r[i] = fmaf(r[i], 0.999f, 0.0001f);
    }
    float s = 0.f;
    for (int i = 0; i < 32; ++i) s += r[i];
    if (s == 12345.f) sink[threadIdx.x] = s;
}
int main(int argc, char **argv) {
    const bool copy = argc > 1 && !strcmp(argv[1], "copy");
    const bool event = argc > 1 && !strcmp(argv[1], "event");
    const bool mfma = argc > 1 && !strcmp(argv[1], "mfma");
    const bool mfmalds = argc > 1 && !strcmp(argv[1], "mfmalds");
    const bool valu = argc > 1 && !strcmp(argv[1], "valu");
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
        if (valu) {
            hipLaunchKernelGGL(valu_loop, dim3(2048), dim3(256), 0, st, sink, 256);
            if (++n % 16 == 0 && hipStreamSynchronize(st) != hipSuccess) return 1;
        } else if (mfma || mfmalds) {
            if (mfma) hipLaunchKernelGGL(mfma_loop<false>, dim3(2048), dim3(256), 0, st, sink, 256);
            else hipLaunchKernelGGL(mfma_loop<true>, dim3(2048), dim3(256), 0, st, sink, 256);
            if (++n % 16 == 0 && hipStreamSynchronize(st) != hipSuccess) return 1;
        } else if (event) {
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

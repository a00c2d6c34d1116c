// Diagnostic victim: a deterministic VALU/DPP/LDS/transcendental kernel whose
// per-workgroup results are compared, launch after launch, with the first
// launch's; prints the number of launches with any difference. Run it alone,
// then beside `garbage mfma` in another process.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
__device__ __forceinline__ float dpp_sum(float v) {
    v += __shfl_xor(v, 1, 64); v += __shfl_xor(v, 2, 64); v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64); v += __shfl_xor(v, 16, 64); v += __shfl_xor(v, 32, 64);
    return v;
}
__global__ __launch_bounds__(256) void victim(const float *in, float *out, int n) {
    __shared__ float red[4];
    const int tid = threadIdx.x, w = tid >> 6;
    float acc = 0.f;
    for (int i = tid; i < n; i += 256) {
        const float x = in[(size_t)blockIdx.x * n + i];
        acc += expf(x * 0.01f) * sqrtf(fabsf(x) + 1.f) + tanhf(x * 0.1f) / (1.f + x * x);
    }
    acc = dpp_sum(acc);
    if ((tid & 63) == 0) red[w] = acc;
    __syncthreads();
    if (tid == 0) out[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
int main(int argc, char **argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 8.0;
    const int G = 512, N = 4096;
    std::vector<float> h((size_t)G * N);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 20011) / 1000.f - 10.f;
    float *din, *dout;
    if (hipMalloc(&din, h.size() * 4) != hipSuccess || hipMalloc(&dout, G * 4) != hipSuccess) return 1;
    if (hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
    std::vector<float> ref(G), cur(G);
    hipLaunchKernelGGL(victim, dim3(G), dim3(256), 0, 0, din, dout, N);
    if (hipMemcpy(ref.data(), dout, G * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    long runs = 0, bad = 0;
    auto t0 = std::chrono::steady_clock::now();
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
        hipLaunchKernelGGL(victim, dim3(G), dim3(256), 0, 0, din, dout, N);
        if (hipMemcpy(cur.data(), dout, G * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        ++runs;
        if (memcmp(cur.data(), ref.data(), G * 4)) ++bad;
    }
    printf("victim launches %ld, launches with a differing result %ld\n", runs, bad);
    return 0;
}

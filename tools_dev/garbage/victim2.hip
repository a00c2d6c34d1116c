// Diagnostic victim 2: a producer kernel writes a buffer whose contents depend
// on the iteration, the next kernel on the same stream reads it through a
// workgroup -> slice mapping scrambled against the producer's (so producer and
// consumer of a line usually sit on different XCDs) and counts every element
// that is not the current iteration's value. Run alone, then beside `garbage mfma`.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
constexpr int NSL = 1024, SL = 1024;  // slices x floats
__global__ __launch_bounds__(256) void produce(float *x, int iter) {
    const int s = blockIdx.x;
    for (int i = threadIdx.x; i < SL; i += 256) {
        const unsigned e = (unsigned)(s * SL + i);
        x[e] = (float)((e * 31u + (unsigned)iter) & 0xFFFFu);
    }
}
__global__ __launch_bounds__(256) void consume(const float *x, unsigned *bad, int iter) {
    const int s = (int)((blockIdx.x * 613u + 101u) % NSL);
    unsigned nb = 0;
    for (int i = threadIdx.x; i < SL; i += 256) {
        const unsigned e = (unsigned)(s * SL + i);
        nb += x[e] != (float)((e * 31u + (unsigned)iter) & 0xFFFFu);
    }
    if (nb) atomicAdd(bad, nb);
}
int main(int argc, char **argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 8.0;
    float *x;
    unsigned *bad;
    if (hipMalloc(&x, (size_t)NSL * SL * 4) != hipSuccess || hipMalloc(&bad, 4) != hipSuccess) return 1;
    if (hipMemset(bad, 0, 4) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    auto t0 = std::chrono::steady_clock::now();
    int it = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs) {
        for (int k = 0; k < 64; ++k, ++it) {
            hipLaunchKernelGGL(produce, dim3(NSL), dim3(256), 0, st, x, it);
            hipLaunchKernelGGL(consume, dim3(NSL), dim3(256), 0, st, x, bad, it);
        }
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
    }
    unsigned hb = 0;
    if (hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("victim2 iterations %d, stale elements read %u\n", it, hb);
    return 0;
}

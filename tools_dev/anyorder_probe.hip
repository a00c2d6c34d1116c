// Probe: can a dependent kernel's dispatch overlap its predecessor on gfx950?
// (hipExtAnyOrderLaunch = AQL packet without the barrier bit; graph capture of
// such launches; two-stream fork inside a captured graph.) Every spin is bounded
// by s_memrealtime, so nothing here can hang.
//
// K1: one workgroup, lane 0 stamps its start, spins SPIN_US, stamps its end.
// K2: one workgroup, lane 0 stamps its start.
// Reported: K2.start - K1.end in us (negative = K2 ran while K1 was still running).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("ERR %s at %d: %s\n", #x, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

__global__ void spin_kernel(unsigned long long *ts, int slot, int spin_ticks) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned long long t = t0;
        while (t - t0 < (unsigned long long)spin_ticks) { __builtin_amdgcn_s_sleep(2); t = __builtin_amdgcn_s_memrealtime(); }
        ts[2 * slot] = t0;
        ts[2 * slot + 1] = t;
    }
}
__global__ void stamp_kernel(unsigned long long *ts, int slot) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        ts[2 * slot] = t0;
        ts[2 * slot + 1] = t0;
    }
}
// a short chain link: every block's lane 0 stamps nothing; the last link stamps
__global__ void tiny_kernel(float *buf, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) buf[i] = buf[i] * 1.0001f + 1.0f;
}

static void pair(const char *name, hipStream_t s, unsigned long long *d_ts, int flags1, int flags2, bool graph) {
    const int spin = 2000;  // 20 us at 100 MHz
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    auto issue = [&]() {
        hipExtLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, nullptr, nullptr, flags1, d_ts, 0, spin);
        hipExtLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s, nullptr, nullptr, flags2, d_ts, 1);
    };
    if (graph) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        issue();
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    double best = 1e9, worst = -1e9;
    for (int r = 0; r < 20; ++r) {
        if (graph) CK(hipGraphLaunch(ge, s)); else issue();
        CK(hipStreamSynchronize(s));
        unsigned long long h[4];
        CK(hipMemcpy(h, d_ts, sizeof(h), hipMemcpyDeviceToHost));
        const double d = ((double)(long long)(h[2] - h[1])) / 100.0;
        if (r >= 2) { if (d < best) best = d; if (d > worst) worst = d; }
    }
    printf("%-44s K2.start-K1.end: min %7.2f us  max %7.2f us\n", name, best, worst);
    if (ge) hipGraphExecDestroy(ge);
    if (g) hipGraphDestroy(g);
}

static void chain(const char *name, hipStream_t s, float *buf, int n_links, int blocks, int flags, bool graph) {
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    auto issue = [&]() {
        for (int i = 0; i < n_links; ++i)
            hipExtLaunchKernelGGL(tiny_kernel, dim3(blocks), dim3(256), 0, s, nullptr, nullptr, flags, buf, blocks * 256);
    };
    if (graph) {
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        issue();
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int r = 0; r < 10; ++r) {
        CK(hipEventRecord(e0, s));
        if (graph) CK(hipGraphLaunch(ge, s)); else issue();
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2 && ms < best) best = ms;
    }
    printf("%-44s %3d links x %4d blocks: %8.2f us total, %6.2f us/link\n", name, n_links, blocks, best * 1e3,
           best * 1e3 / n_links);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    if (ge) hipGraphExecDestroy(ge);
    if (g) hipGraphDestroy(g);
}

// two-stream fork inside a capture: K1 on s0, K2 on s1, no edge between them
static void fork_pair(hipStream_t s0, hipStream_t s1, unsigned long long *d_ts) {
    hipEvent_t ef, ej;
    CK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s0, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(ef, s0));
    CK(hipStreamWaitEvent(s1, ef, 0));
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s0, d_ts, 0, 2000);
    hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, s1, d_ts, 1);
    CK(hipEventRecord(ej, s1));
    CK(hipStreamWaitEvent(s0, ej, 0));
    CK(hipStreamEndCapture(s0, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    double best = 1e9, worst = -1e9;
    for (int r = 0; r < 20; ++r) {
        CK(hipGraphLaunch(ge, s0));
        CK(hipStreamSynchronize(s0));
        unsigned long long h[4];
        CK(hipMemcpy(h, d_ts, sizeof(h), hipMemcpyDeviceToHost));
        const double d = ((double)(long long)(h[2] - h[1])) / 100.0;
        if (r >= 2) { if (d < best) best = d; if (d > worst) worst = d; }
    }
    printf("%-44s K2.start-K1.end: min %7.2f us  max %7.2f us\n", "graph fork (2 streams, no edge)", best, worst);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
}

int main() {
    hipStream_t s, s1;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    unsigned long long *d_ts;
    CK(hipMalloc(&d_ts, 64 * sizeof(unsigned long long)));
    float *buf;
    CK(hipMalloc(&buf, 1 << 24));
    CK(hipMemset(buf, 0, 1 << 24));
    pair("plain launches", s, d_ts, 0, 0, false);
    pair("ext launch, flags 0", s, d_ts, 0, 0, false);
    pair("ext launch, K2 anyorder", s, d_ts, 0, hipExtAnyOrderLaunch, false);
    pair("ext launch, both anyorder", s, d_ts, hipExtAnyOrderLaunch, hipExtAnyOrderLaunch, false);
    pair("graph: ext launch, flags 0", s, d_ts, 0, 0, true);
    pair("graph: ext launch, K2 anyorder", s, d_ts, 0, hipExtAnyOrderLaunch, true);
    pair("graph: ext launch, both anyorder", s, d_ts, hipExtAnyOrderLaunch, hipExtAnyOrderLaunch, true);
    fork_pair(s, s1, d_ts);
    for (int blocks : {1, 256}) {
        chain("eager, flags 0", s, buf, 64, blocks, 0, false);
        chain("eager, anyorder", s, buf, 64, blocks, hipExtAnyOrderLaunch, false);
        chain("graph, flags 0", s, buf, 64, blocks, 0, true);
        chain("graph, anyorder", s, buf, 64, blocks, hipExtAnyOrderLaunch, true);
    }
    CK(hipDeviceSynchronize());
    printf("done\n");
    return 0;
}

// Diagnostic victim 3: the decode's own kernels (mp_decode.hip, compiled into
// this program) on fixed random inputs, launch after launch, every output
// compared bitwise with the first launch's on the device. Prints, per op, the
// launches and the differing elements. Run alone, then beside `garbage mfma`.
//   victim3 SECS [op]   op: ff1 ff1x ff2 qkv oproj sa xa all
#include "../../magpie-tts.cpp_amd/csrc/mp_decode.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

using namespace mp;

__global__ void cmp_kernel(const float *a, const float *b, size_t n, unsigned long long *bad) {
    unsigned long long nb = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
        nb += __float_as_uint(a[i]) != __float_as_uint(b[i]);
    if (nb) atomicAdd(bad, nb);
}

static float *dev_rand(size_t n, unsigned seed, float scale, float offset = 0.f) {
    std::vector<float> h(n);
    unsigned s = seed * 2654435761u + 12345u;
    for (size_t i = 0; i < n; ++i) {
        s = s * 1664525u + 1013904223u;
        h[i] = offset + scale * ((float)(s >> 8) / 16777216.0f - 0.5f);
    }
    float *d = nullptr;
    if (hipMalloc(&d, n * 4 + 256) != hipSuccess) exit(1);
    if (hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) exit(1);
    return d;
}
static int *dev_int(int v) {
    int *d = nullptr;
    if (hipMalloc(&d, 256) != hipSuccess || hipMemcpy(d, &v, 4, hipMemcpyHostToDevice) != hipSuccess) exit(1);
    return d;
}

int main(int argc, char **argv) {
    const double secs = argc > 1 ? atof(argv[1]) : 6.0;
    const std::string which = argc > 2 ? argv[2] : "all";
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    const int MS = 384, L = 1, T = 64, POS = 239;
    // inputs
    float *Wqkv = dev_rand(2304 * 768, 1, 0.04f), *Wo = dev_rand(768 * 768, 2, 0.04f);
    float *W1 = dev_rand(3072 * 768, 3, 0.04f), *W2 = dev_rand(768 * 3072, 4, 0.04f);
    float *x = dev_rand(768, 5, 2.f), *lnw = dev_rand(768, 6, 0.05f, 1.f), *h = dev_rand(3072, 7, 1.f);
    float *kc = dev_rand((size_t)MS * 768, 8, 1.f), *vc = dev_rand((size_t)MS * 768, 9, 1.f);
    float *kp = dev_rand((size_t)T * 768, 10, 1.f), *vp = dev_rand((size_t)T * 768, 11, 1.f);
    float *q = dev_rand(768, 12, 1.f);
    float *sa_part = nullptr, *xa_part = nullptr;
    {   // split states as the attention kernels leave them
        std::vector<float> sp((size_t)NH * SA_SPLITS * SA_PART), xp((size_t)XA_SPLITS * XA_PART);
        unsigned s = 77;
        auto r = [&]() { s = s * 1664525u + 1013904223u; return (float)(s >> 8) / 16777216.0f; };
        for (int g = 0; g < NH * SA_SPLITS; ++g) {
            float *p = sp.data() + (size_t)g * SA_PART;
            p[0] = 2.f * r(); p[1] = 1.f + 10.f * r(); p[2] = p[3] = 0.f;
            for (int i = 0; i < DH; ++i) p[4 + i] = r() - 0.5f;
        }
        for (int g = 0; g < XA_SPLITS; ++g) {
            float *p = xp.data() + (size_t)g * XA_PART;
            p[0] = 2.f * r(); p[1] = 1.f + 10.f * r(); p[2] = p[3] = 0.f;
            for (int i = 0; i < D; ++i) p[4 + i] = r() - 0.5f;
        }
        if (hipMalloc(&sa_part, sp.size() * 4) != hipSuccess || hipMalloc(&xa_part, xp.size() * 4) != hipSuccess) return 1;
        if (hipMemcpy(sa_part, sp.data(), sp.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
        if (hipMemcpy(xa_part, xp.data(), xp.size() * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
    }
    int *pos = dev_int(POS), *Tb = dev_int(T);
    float *out = nullptr, *ref = nullptr, *xres = nullptr, *part_out = nullptr;
    if (hipMalloc(&out, 3072 * 4 * 4) != hipSuccess || hipMalloc(&ref, 3072 * 4 * 4) != hipSuccess ||
        hipMalloc(&xres, 768 * 4) != hipSuccess || hipMalloc(&part_out, 65536 * 4) != hipSuccess)
        return 1;
    unsigned long long *bad = nullptr;
    if (hipMalloc(&bad, 8) != hipSuccess) return 1;

    struct Op { const char *name; size_t n; float *o; };
    GemvP g;
    memset(&g, 0, sizeof g);
    g.eps = 1e-5f; g.nlayers = L; g.max_seq = MS; g.pos = pos; g.lnw = lnw;
    auto run = [&](const std::string &op) -> Op {
        GemvP p = g;
        if (op == "ff1") {
            p.W = W1; p.N = 3072; p.src = x; p.src_ld = 768; p.out = out; p.out_ld = 3072;
            if (op_ff1_1(p, st) != hipSuccess) exit(2);
            return {"ff1 (PRO_LN, GELU)", 3072, out};
        }
        if (op == "ff1x") {
            p.W = W1; p.N = 3072; p.src = x; p.src_ld = 768; p.part = xa_part; p.xres = xres; p.out = out; p.out_ld = 3072;
            if (op_ff1x_1(p, st) != hipSuccess) exit(2);
            return {"ff1x (PRO_XA_LN, GELU)", 3072, out};
        }
        if (op == "ff2") {
            p.W = W2; p.N = 768; p.src = h; p.src_ld = 3072; p.out = out; p.out_ld = 768; p.addsrc = x;
            if (op_ff2_1(p, st) != hipSuccess) exit(2);
            return {"ff2 (PLAIN, ADD_STORE)", 768, out};
        }
        if (op == "qkv") {
            p.W = Wqkv; p.N = 2304; p.src = x; p.src_ld = 768; p.out = out; p.kc = kc; p.vc = vc; p.layer = 0;
            if (op_qkv_1(p, st) != hipSuccess) exit(2);
            return {"qkv (PRO_LN, QKV)", 768, out};
        }
        if (op == "oproj") {
            if (hipMemcpyAsync(out, x, 768 * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) exit(2);
            p.W = Wo; p.N = 768; p.part = sa_part; p.resid = out;
            if (op_oproj_1(p, st) != hipSuccess) exit(2);
            return {"oproj (PRO_SA_MERGE, RESID)", 768, out};
        }
        if (op == "sa") {
            AttnP a{};
            a.q = q; a.kc = kc; a.vc = vc; a.layer = 0; a.nlayers = 1; a.max_seq = MS; a.pos = pos; a.part = part_out;
            if (op_sa_attn(a, 1, st) != hipSuccess) exit(2);
            return {"sa_attn", (size_t)NH * SA_SPLITS * SA_PART, part_out};
        }
        if (op == "xa") {
            XaP a{};
            a.x = x; a.part = part_out; a.lnw = lnw; a.eps = 1e-5f; a.kp = kp; a.vp = vp; a.T = Tb; a.Tmax = T;
            a.layer = 0; a.nlayers = 1;
            if (op_xa(a, 1, st) != hipSuccess) exit(2);
            return {"xa_part", (size_t)XA_SPLITS * XA_PART, part_out};
        }
        exit(3);
    };
    std::vector<std::string> ops = which == "all" ? std::vector<std::string>{"ff1", "ff1x", "ff2", "oproj", "sa", "xa", "qkv"}
                                                 : std::vector<std::string>{which};
    for (const std::string &op : ops) {
        Op o = run(op);
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
        if (hipMemcpyAsync(ref, o.o, o.n * 4, hipMemcpyDeviceToDevice, st) != hipSuccess) return 1;
        if (hipMemsetAsync(bad, 0, 8, st) != hipSuccess) return 1;
        if (hipStreamSynchronize(st) != hipSuccess) return 1;
        long launches = 0;
        auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() < secs / ops.size()) {
            for (int k = 0; k < 64; ++k, ++launches) {
                run(op);
                hipLaunchKernelGGL(cmp_kernel, dim3(16), dim3(256), 0, st, ref, o.o, o.n, bad);
            }
            if (hipStreamSynchronize(st) != hipSuccess) return 1;
        }
        unsigned long long hb = 0;
        if (hipMemcpy(&hb, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("%-30s launches %7ld  differing elements %llu\n", o.name, launches, hb);
        fflush(stdout);
    }
    return 0;
}

// Device-side helpers shared by the gfx950 kernels (wave64 reductions, vector
// loads, block reductions). CDNA4 only: wave = 64 lanes, 256-thread workgroups.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define MP_WAVE 64
#define MP_BLOCK 256
#define MP_NWAVES (MP_BLOCK / MP_WAVE)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
    return v;
}
// sum over lanes that differ only in the low log2(W) bits (W = 2..64)
template <int W>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
    for (int o = W / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Block-wide reduction for 256 threads; `red` is an LDS scratch of >= 4 floats.
// Every thread returns the total. Contains two barriers.
__device__ __forceinline__ float block_sum(float v, float *red) {
    v = wave_sum(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    const float r = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return r;
}
__device__ __forceinline__ float block_max(float v, float *red) {
    v = wave_max(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    const float r = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    __syncthreads();
    return r;
}

// (value, index) argmax with the reference's tie rule: the FIRST maximal index
// wins (strict '>' scan from index 0, magpie.cpp:1250-1258).
__device__ __forceinline__ void argmax_merge(float &v, int &i, float v2, int i2) {
    if (v2 > v || (v2 == v && i2 < i)) { v = v2; i = i2; }
}
__device__ __forceinline__ void wave_argmax(float &v, int &i) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(i, o, 64);
        argmax_merge(v, i, v2, i2);
    }
}

__device__ __forceinline__ float gelu_tanh(float x) {
    // ggml_gelu: 0.5 x (1 + tanh(sqrt(2/pi) x (1 + 0.044715 x^2)))
    return 0.5f * x * (1.0f + tanhf(0.79788456080286535588f * x * (1.0f + 0.044715f * x * x)));
}

template <int VW> struct vecf;
template <> struct vecf<4> { using T = float4; };
template <> struct vecf<2> { using T = float2; };
template <> struct vecf<1> { using T = float; };

__device__ __forceinline__ float dotv(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
__device__ __forceinline__ float dotv(float2 a, float2 b) { return a.x * b.x + a.y * b.y; }
__device__ __forceinline__ float dotv(float a, float b) { return a * b; }

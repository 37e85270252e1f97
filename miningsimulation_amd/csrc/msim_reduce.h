// msim_reduce.h — workgroup reduction of per-run MinerStats terms (device code shared by the kernels).
#pragma once
#include <hip/hip_runtime.h>

#include "msim_kernels.h"

namespace msim {

// Wave-level (DPP/bpermute) reduction of 6*M 64-bit sums, then the workgroup's NT/64 waves through LDS.
template <int M, int NT = TPB>
__device__ __forceinline__ void block_reduce_store(const uint64_t (&v)[6 * M], uint64_t *__restrict__ out)
{
    static_assert(NT % 64 == 0 && NT <= 1024, "whole waves");
    constexpr int NW = NT / 64;
    __shared__ uint64_t red[NW][6 * M];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < 6 * M; ++i) {
        unsigned long long x = v[i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
        if (lane == 0) red[wv][i] = x;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < 6 * M; i += NT) {
        uint64_t t = 0;
#pragma unroll
        for (int w = 0; w < NW; ++w) t += red[w][i];
        out[i] = t;
    }
}

}  // namespace msim

// LDS access cost on gfx950 for the table-lookup shapes of the draw kernels (measurement tool, not
// shipped): each kernel does ITERS lookups per lane at random indices (xorshift per lane) into a table
// of E entries of B bytes, 8 waves per SIMD; wall time per wave-instruction relative to a
// conflict-free ds_read_b32 (lane-indexed).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 2048

template <int E, int MODE>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed)
{
    __shared__ uint4 tab[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) tab[i] = make_uint4(i, i * 3, i * 5, i * 7);
    __syncthreads();
    uint32_t x = (threadIdx.x + 1) * 2654435761u ^ seed, acc = 0;
    const uint32_t *t32 = (const uint32_t *)tab;
    const uint2 *t64 = (const uint2 *)tab;
    for (int i = 0; i < ITERS; ++i) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        const uint32_t j = (x >> 8) % E;
        if (MODE == 0) acc += t32[threadIdx.x & 63];                    // b32, lane-indexed (conflict-free)
        if (MODE == 1) acc += t32[j];                                   // b32 random over E dwords
        if (MODE == 2) { const uint2 v = t64[j]; acc += v.x ^ v.y; }    // b64 random over E entries
        if (MODE == 3) { const uint4 v = tab[j]; acc += v.x ^ v.y ^ v.z ^ v.w; }  // b128 random over E entries
        if (MODE == 4) acc += __builtin_amdgcn_ds_bpermute((int)(j & 63) << 2, (int)x);  // crossbar permute
        if (MODE == 5) { const uint4 v = tab[threadIdx.x & 63]; acc += v.x ^ v.y ^ v.z ^ v.w; }  // b128 lane-indexed
        if (MODE == 6) acc += 0;                                        // no LDS op: the xorshift alone
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

typedef void (*kfn)(uint32_t *, uint32_t);
struct K { const char *name; kfn f; };

int main()
{
    K ks[] = {{"none (xorshift only)", k<64, 6>}, {"b32 lane-indexed", k<64, 0>}, {"b32 rand/101", k<101, 1>},
              {"b32 rand/1024", k<1024, 1>}, {"b64 rand/64", k<64, 2>}, {"b64 rand/512", k<512, 2>},
              {"b128 rand/64", k<64, 3>}, {"b128 rand/100", k<100, 3>}, {"b128 rand/128", k<128, 3>},
              {"b128 rand/512", k<512, 3>}, {"b128 lane-indexed", k<64, 5>}, {"bpermute", k<64, 4>}};
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;
    uint32_t *out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float base = 0;
    printf("%-22s %10s %10s\n", "pattern", "ms", "ns/wave-op");
    for (auto &kk : ks) {
        hipLaunchKernelGGL(kk.f, dim3(blocks), dim3(256), 0, 0, out, 1u);
        (void)hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kk.f, dim3(blocks), dim3(256), 0, 0, out, 2u + r);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        if (base == 0) base = ms;
        // per CU: 32 waves x ITERS ops; report (ms - base) per wave-op per CU in ns
        printf("%-22s %10.4f %10.3f\n", kk.name, ms, (ms - base) * 1e6 / (32.0 * ITERS));
    }
    return 0;
}

// msim_common.hip — finalize kernel and the runtime miner-count dispatch (compiled once).
#include <hip/hip_runtime.h>

#include "msim_kernels.h"
#include "msim_sel_launch.h"
#include "msim_selseg.h"

namespace msim {

// One workgroup per summed value: the lanes stride over the workgroup partials, then a wave
// butterfly and the 4 waves through LDS (integer sums, so the result is order-independent). A single
// workgroup walking the partials serially spent ~64 us per launch on dependent loads.
__global__ __launch_bounds__(TPB) void msim_finalize(const uint64_t *__restrict__ partials, uint32_t nparts,
                                                     uint32_t nvals, uint64_t *__restrict__ out,
                                                     const uint32_t *__restrict__ retry_count,
                                                     const uint32_t *__restrict__ fail_count, const uint32_t retry_cap,
                                                     uint32_t *__restrict__ status)
{
    __shared__ uint64_t red[TPB / 64];
    const uint32_t i = blockIdx.x;
    if (i < nvals) {
        unsigned long long s = 0;
        for (uint32_t b = threadIdx.x; b < nparts; b += TPB) s += partials[(size_t)b * nvals + i];
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
        __syncthreads();
        if (threadIdx.x == 0) out[i] = red[0] + red[1] + red[2] + red[3];
    }
    if (i == 0 && threadIdx.x == 0 && status) {
        const uint32_t rc = *retry_count;
        status[0] = rc;
        status[1] = *fail_count + (rc > retry_cap ? rc - retry_cap : 0u);
    }
}

__global__ void msim_log1p_kernel(const double *__restrict__ x, double *__restrict__ out, uint64_t n)
{
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = glibc_log1p(x[i]);
}

hipError_t launch_log1p(const double *x, double *out, uint64_t n, hipStream_t s)
{
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(msim_log1p_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, out, n);
    return hipGetLastError();
}

hipError_t launch_finalize(const uint64_t *partials, uint32_t nparts, uint32_t nvals, uint64_t *out,
                           const uint32_t *retry_count, const uint32_t *fail_count, uint32_t retry_cap,
                           uint32_t *status, hipStream_t stream)
{
    hipLaunchKernelGGL(msim_finalize, dim3(nvals > 0 ? nvals : 1), dim3(TPB), 0, stream, partials, nparts, nvals, out, retry_count,
                       fail_count, retry_cap, status);
    return hipGetLastError();
}

hipError_t launch_runs(const LaunchArgs &a)
{
    switch (a.p.m) {
#define CASE(MM) \
    case MM:     \
        return launch_runs_m##MM(a);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

// Sweep sums: point p = fixed-order sum of its workgroups' partials + its retried runs.
__global__ void msim_sweep_finalize(const uint64_t *__restrict__ partials, uint32_t wpp, uint32_t nvals,
                                    const uint64_t *__restrict__ retry_sums, uint64_t *__restrict__ out,
                                    const uint32_t *__restrict__ counts, uint32_t retry_cap, uint32_t *__restrict__ status)
{
    const uint32_t p = blockIdx.x;
    for (uint32_t i = threadIdx.x; i < nvals; i += blockDim.x) {
        uint64_t s = retry_sums[(size_t)p * nvals + i];
        for (uint32_t b = 0; b < wpp; ++b) s += partials[((size_t)p * wpp + b) * nvals + i];
        out[(size_t)p * nvals + i] = s;
    }
    if (p == 0 && threadIdx.x == 0 && status) {
        const uint32_t rc = counts[0];
        status[0] = rc;
        status[1] = counts[1] + (rc > retry_cap ? rc - retry_cap : 0u);
    }
}

hipError_t launch_sweep_finalize(const SweepArgs &a)
{
    hipLaunchKernelGGL(msim_sweep_finalize, dim3(a.n_points), dim3(TPB), 0, a.stream, a.partials, a.wpp, 6 * a.m,
                       a.retry_sums, a.sums, a.err_count, a.err_cap, a.status);
    return hipGetLastError();
}

hipError_t launch_sweep(const SweepArgs &a)
{
    switch (a.m) {
#define CASE(MM) \
    case MM:     \
        return launch_sweep_m##MM(a);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_sel(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return launch_sel_m##MM(a, ns_class, s);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_segwork(const SelArgs &a, const SegArgs &g, uint32_t m, hipStream_t s)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return launch_segwork_m##MM(a, g, s);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

hipError_t launch_stitch(const SelArgs &a, const SegArgs &g, uint32_t m, hipStream_t s)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return launch_stitch_m##MM(a, g, s);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

size_t seg_rec_bytes(uint32_t m)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return sizeof(SegRec<MM>);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return 0;
    }
}
uint32_t seg_qcap(uint32_t cuts, uint32_t seg) { return (cuts + 1u) * (SEG_QWIN * 3u / 4u) + seg / SEG_QEVERY + 16u; }
size_t seg_qrec_bytes(uint32_t m)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return sizeof(SegQRec<MM>);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return 0;
    }
}

hipError_t launch_sel_retry(const SelArgs &a, uint32_t m, uint32_t ns_class, hipStream_t s)
{
    switch (m) {
#define CASE(MM) \
    case MM:     \
        return launch_sel_retry_m##MM(a, ns_class, s);
        MSIM_FOR_EACH_M(CASE)
#undef CASE
    default:
        return hipErrorInvalidValue;
    }
}

// F: one workgroup per (point, value); lanes stride over the point's workgroup partials.
__global__ __launch_bounds__(TPB) void msim_sel_finalize(const uint64_t *__restrict__ partials, uint32_t wpp,
                                                         uint32_t nvals, const uint64_t *__restrict__ retry_sums,
                                                         uint64_t *__restrict__ out, const uint32_t *__restrict__ counts,
                                                         uint32_t *__restrict__ status)
{
    __shared__ uint64_t red[TPB / 64];
    const uint32_t p = blockIdx.x / nvals, i = blockIdx.x % nvals;
    unsigned long long s = 0;
    for (uint32_t b = threadIdx.x; b < wpp; b += TPB) s += partials[((size_t)p * wpp + b) * nvals + i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) out[(size_t)p * nvals + i] = red[0] + red[1] + red[2] + red[3] + retry_sums[(size_t)p * nvals + i];
    if (blockIdx.x == 0 && threadIdx.x == 0 && status) {
        status[0] = counts[0];
        status[1] = counts[1];
    }
}

hipError_t launch_sel_finalize(const uint64_t *partials, uint32_t n_points, uint32_t wpp, uint32_t nvals,
                               const uint64_t *retry_sums, uint64_t *out, const uint32_t *counts, uint32_t *status,
                               hipStream_t s)
{
    hipLaunchKernelGGL(msim_sel_finalize, dim3(n_points * nvals), dim3(TPB), 0, s, partials, wpp, nvals, retry_sums, out,
                       counts, status);
    return hipGetLastError();
}

size_t partials_words(uint32_t m, uint32_t n, uint32_t err_cap)
{
    // one row per 64 runs: the pipeline's combine kernel K3 runs one-wave workgroups (msim_kernels.hip)
    const size_t nb = (n + 63) / 64, nbr = (err_cap + TPB - 1) / TPB;
    return (nb + nbr) * 6 * (size_t)m;
}

}  // namespace msim

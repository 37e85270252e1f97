// selkat_dev.hip — TEST INFRASTRUCTURE: the TestSelfishStrategy replay (selkat.h) as a gfx950 kernel, one lane
// per case, so the -m gpu test runs the product's state machines (msim_sel.h, msim_selm.h) as device code.
// Never part of the product path.
#include <hip/hip_runtime.h>

#include "selkat.h"

using namespace msim;

__global__ void selkat_kernel(const KatIn *in, KatOut *out, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    KatOut o;
    kat_sel(in[i], o);
    kat_macro(in[i], o);
    out[i] = o;
}

extern "C" uint32_t selkat_sizes(uint32_t *in_bytes, uint32_t *out_bytes)
{
    *in_bytes = (uint32_t)sizeof(KatIn);
    *out_bytes = (uint32_t)sizeof(KatOut);
    return (uint32_t)KAT_MAXB;
}

// Returns 0, or the failing HIP error code.
extern "C" int selkat_run_dev(const KatIn *in, KatOut *out, uint32_t n)
{
    KatIn *din = nullptr;
    KatOut *dout = nullptr;
    hipError_t e = hipMalloc((void **)&din, sizeof(KatIn) * n);
    if (e == hipSuccess) e = hipMalloc((void **)&dout, sizeof(KatOut) * n);
    if (e == hipSuccess) e = hipMemcpy(din, in, sizeof(KatIn) * n, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(selkat_kernel, dim3((n + 63) / 64), dim3(64), 0, 0, din, dout, n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(KatOut) * n, hipMemcpyDeviceToHost);
    (void)hipFree(din);
    (void)hipFree(dout);
    return (int)e;
}

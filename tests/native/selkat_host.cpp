// selkat_host.cpp — TEST INFRASTRUCTURE: host build of the TestSelfishStrategy replay (selkat.h) on the
// product's entity engine and settled form. Never part of the product path.
#include "selkat.h"

using namespace msim;

extern "C" uint32_t selkat_sizes(uint32_t *in_bytes, uint32_t *out_bytes)
{
    *in_bytes = (uint32_t)sizeof(KatIn);
    *out_bytes = (uint32_t)sizeof(KatOut);
    return (uint32_t)KAT_MAXB;
}

extern "C" void selkat_run(const KatIn *in, KatOut *out, uint32_t n)
{
    for (uint32_t i = 0; i < n; ++i) {
        kat_sel(in[i], out[i]);
        kat_macro(in[i], out[i]);
    }
}

// msim_jump.h — GF(2) jump-ahead for the reference's xoroshiro128++ streams.
//
// The reference draws every random number of a run sequentially from two RNG objects
// (/root/reference/main.cpp:134, xoroshiro128++.h:26-34). The state update of xoroshiro128 (not its
// "++" output function) is linear over GF(2)^128:
//     t = s1 ^ s0;  s0' = rotl(s0, 49) ^ t ^ (t << 21);  s1' = rotl(t, 28)
// so advancing a stream by n draws is one 128x128 bit-matrix product, T^n · s. The draw kernel uses
// this to start many workers of ONE run at different draw indices (segment j starts at draw j*S), and
// every worker then produces bit-identical draws to the reference's sequential loop.
//
// Matrix layout: column b (0..127) is T^n applied to basis vector e_b, where bits 0..63 are s0 and
// 64..127 are s1. Device layout: uint4 {s0.lo, s0.hi, s1.lo, s1.hi} per column, 2 KiB per matrix.
#pragma once
#include <stdint.h>

#include "msim_draws.h"

namespace msim {

struct Mat128 {
    uint64_t lo[128];  // column b, s0 half
    uint64_t hi[128];  // column b, s1 half
};

// One xoroshiro128 state step, without the output function (xoroshiro128++.h:30-33).
MSIM_HD void xoro_step(uint64_t &s0, uint64_t &s1)
{
    const uint64_t t = s1 ^ s0;
    s0 = rotl64(s0, 49) ^ t ^ (t << 21);
    s1 = rotl64(t, 28);
}

inline void mat_apply(const Mat128 &m, uint64_t s0, uint64_t s1, uint64_t &o0, uint64_t &o1)
{
    uint64_t a = 0, b = 0;
    for (int i = 0; i < 64; ++i)
        if ((s0 >> i) & 1u) {
            a ^= m.lo[i];
            b ^= m.hi[i];
        }
    for (int i = 0; i < 64; ++i)
        if ((s1 >> i) & 1u) {
            a ^= m.lo[64 + i];
            b ^= m.hi[64 + i];
        }
    o0 = a;
    o1 = b;
}

inline void mat_identity(Mat128 &m)
{
    for (int i = 0; i < 64; ++i) {
        m.lo[i] = 1ull << i;
        m.hi[i] = 0;
        m.lo[64 + i] = 0;
        m.hi[64 + i] = 1ull << i;
    }
}

inline void mat_step(Mat128 &m)  // T itself
{
    for (int b = 0; b < 128; ++b) {
        uint64_t s0 = b < 64 ? (1ull << b) : 0, s1 = b < 64 ? 0 : (1ull << (b - 64));
        xoro_step(s0, s1);
        m.lo[b] = s0;
        m.hi[b] = s1;
    }
}

// out = a ∘ b (apply b first, then a). out may alias neither input.
inline void mat_mul(const Mat128 &a, const Mat128 &b, Mat128 &out)
{
    for (int c = 0; c < 128; ++c) mat_apply(a, b.lo[c], b.hi[c], out.lo[c], out.hi[c]);
}

// out = T^n (square and multiply).
inline void mat_pow(uint64_t n, Mat128 &out)
{
    Mat128 base, acc, tmp;
    mat_step(base);
    mat_identity(acc);
    while (n) {
        if (n & 1u) {
            mat_mul(base, acc, tmp);
            acc = tmp;
        }
        n >>= 1;
        if (n) {
            mat_mul(base, base, tmp);
            base = tmp;
        }
    }
    out = acc;
}

// Host: matrices for draw offsets j*S, j = 0..nseg-1, packed as uint32 columns (4 words per column).
inline void build_jump_table(uint32_t nseg, uint32_t seg, uint32_t *out /* nseg*128*4 */)
{
    Mat128 step, cur, tmp;
    mat_pow(seg, step);
    mat_identity(cur);
    for (uint32_t j = 0; j < nseg; ++j) {
        for (int c = 0; c < 128; ++c) {
            uint32_t *w = out + ((size_t)j * 128 + c) * 4;
            w[0] = (uint32_t)cur.lo[c];
            w[1] = (uint32_t)(cur.lo[c] >> 32);
            w[2] = (uint32_t)cur.hi[c];
            w[3] = (uint32_t)(cur.hi[c] >> 32);
        }
        mat_mul(step, cur, tmp);
        cur = tmp;
    }
}

#if defined(__HIPCC__)
// Device: both RNG states of a lane advanced by the same jump matrix (128 wave-uniform columns, uint4 each, in
// the layout of build_jump_table): o ^= column & -bit, one v_bitop3_b32 per word.
__device__ __forceinline__ void jump2(const uint4 *__restrict__ cols, Rng &a, Rng &b)
{
    const uint32_t sa[4] = {(uint32_t)a.s0, (uint32_t)(a.s0 >> 32), (uint32_t)a.s1, (uint32_t)(a.s1 >> 32)};
    const uint32_t sb[4] = {(uint32_t)b.s0, (uint32_t)(b.s0 >> 32), (uint32_t)b.s1, (uint32_t)(b.s1 >> 32)};
    uint32_t oa0 = 0, oa1 = 0, oa2 = 0, oa3 = 0, ob0 = 0, ob1 = 0, ob2 = 0, ob3 = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
#pragma unroll 8
        for (int i = 0; i < 32; ++i) {
            const uint4 c = cols[w * 32 + i];
            const uint32_t ma = 0u - ((sa[w] >> i) & 1u), mb = 0u - ((sb[w] >> i) & 1u);
            // o ^= c & m as one v_bitop3_b32 (table of (src0 & src1) ^ src2: 0xF0 & 0xCC ^ 0xAA = 0x6A)
            oa0 = __builtin_amdgcn_bitop3_b32(c.x, ma, oa0, 0x6A);
            oa1 = __builtin_amdgcn_bitop3_b32(c.y, ma, oa1, 0x6A);
            oa2 = __builtin_amdgcn_bitop3_b32(c.z, ma, oa2, 0x6A);
            oa3 = __builtin_amdgcn_bitop3_b32(c.w, ma, oa3, 0x6A);
            ob0 = __builtin_amdgcn_bitop3_b32(c.x, mb, ob0, 0x6A);
            ob1 = __builtin_amdgcn_bitop3_b32(c.y, mb, ob1, 0x6A);
            ob2 = __builtin_amdgcn_bitop3_b32(c.z, mb, ob2, 0x6A);
            ob3 = __builtin_amdgcn_bitop3_b32(c.w, mb, ob3, 0x6A);
        }
    }
    a.s0 = (uint64_t)oa0 | ((uint64_t)oa1 << 32);
    a.s1 = (uint64_t)oa2 | ((uint64_t)oa3 << 32);
    b.s0 = (uint64_t)ob0 | ((uint64_t)ob1 << 32);
    b.s1 = (uint64_t)ob2 | ((uint64_t)ob3 << 32);
}
#endif

}  // namespace msim

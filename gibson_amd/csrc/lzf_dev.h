/*
 * lzf_dev.h -- device helpers shared by the compress kernels (lzf_cand.hip):
 * unaligned byte-window loads that never touch memory past a value's end,
 * and the reference's slot function.
 */
#ifndef GIBSON_AMD_LZF_DEV_H
#define GIBSON_AMD_LZF_DEV_H

#include "lzf_internal.h"

__device__ __forceinline__ uint4 dv_ld16(const uint8_t *p)          /* unaligned */
{
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__device__ __forceinline__ uint2 dv_ld8(const uint8_t *p)
{
    uint2 v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

__device__ __forceinline__ uint32_t dv_ld4(const uint8_t *p)
{
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

/* bytes [p, p + avail), avail < 16, zero beyond: never touches p + avail */
__device__ __forceinline__ uint4 dv_ld16_tail(const uint8_t *p, uint32_t avail)
{
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (uint32_t k = 0; k < 16u; k++)
        if (k < avail) w[k >> 2] |= (uint32_t)p[k] << (8u * (k & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint4 dv_ld16_safe(const uint8_t *p, uint32_t avail)
{
    return avail >= 16u ? dv_ld16(p) : dv_ld16_tail(p, avail);
}

/* 8 bytes at p, zero past avail (never touches p + avail) */
__device__ __forceinline__ uint2 dv_ld8_safe(const uint8_t *p, uint32_t avail)
{
    if (avail >= 8u) return dv_ld8(p);
    const uint4 t = dv_ld16_tail(p, avail);
    return make_uint2(t.x, t.y);
}

/* 8 bytes at src + pp, zero past n, with one unconditional 8-byte load
 * (needs n >= 8): near the end the load is moved back to n - 8 and the
 * bytes shifted into place; pp past n gives zeros.  Branch-free, so the
 * compiler can count such loads in flight instead of draining them. */
__device__ __forceinline__ uint2 dv_ld8_clamped(const uint8_t *src, uint32_t n, uint32_t pp)
{
    const uint32_t at = pp + 8u <= n ? pp : n - 8u;
    const uint2 v = dv_ld8(src + at);
    const uint32_t sh = pp - at;
    const uint64_t x = ((uint64_t)v.y << 32) | v.x;
    const uint64_t y = sh < 8u ? x >> (8u * sh) : 0ull;
    return make_uint2((uint32_t)y, (uint32_t)(y >> 32));
}

/* the 16-byte load address for bytes from pp in a value of n >= 16 bytes:
 * moved back to n - 16 near the end, so the load stays inside the value */
__device__ __forceinline__ uint32_t dv_at16(uint32_t n, uint32_t pp) { return pp + 16u <= n ? pp : n - 16u; }

/* v shifted down by sh (0 .. 15) bytes, zeros in */
__device__ __forceinline__ uint4 dv_shr16(uint4 v, uint32_t sh)
{
    uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    const bool big = sh >= 8u;
    lo = big ? hi : lo;
    hi = big ? 0ull : hi;
    const uint32_t b = 8u * (sh & 7u);
    lo = b ? (lo >> b) | (hi << (64u - b)) : lo;
    hi >>= b;
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

/* slot(p) of src/lzf_c.c:47-57 (VERY_FAST, HLOG 16) from b[p..p+2] = tri */
__device__ __forceinline__ uint32_t dv_slot(uint32_t tri)
{
    const uint32_t b0 = tri & 0xFFu, b1 = (tri >> 8) & 0xFFu, b2 = (tri >> 16) & 0xFFu;
    return (((b0 << 8) | b1) - 5u * ((b1 << 8) | b2)) & 0xFFFFu;
}

/* index of the first differing byte of two 16-byte pieces, 16 if equal */
__device__ __forceinline__ uint32_t dv_first_diff(uint4 a, uint4 b)
{
    uint32_t x;
    if ((x = a.x ^ b.x)) return (uint32_t)__builtin_ctz(x) >> 3;
    if ((x = a.y ^ b.y)) return 4u + ((uint32_t)__builtin_ctz(x) >> 3);
    if ((x = a.z ^ b.z)) return 8u + ((uint32_t)__builtin_ctz(x) >> 3);
    if ((x = a.w ^ b.w)) return 12u + ((uint32_t)__builtin_ctz(x) >> 3);
    return 16u;
}

__device__ __forceinline__ uint32_t dv_sel4(uint4 v, uint32_t i)
{
    return i == 0u ? v.x : i == 1u ? v.y : i == 2u ? v.z : v.w;
}

/* store exactly len (<= 16) bytes of v at p (unaligned) */
__device__ __forceinline__ void dv_st_exact(uint8_t *p, uint4 v, uint32_t len)
{
    if (len >= 16u) {
        __builtin_memcpy(p, &v, 16);
        return;
    }
    uint32_t a = v.x, b = v.y, c = v.z, d = v.w;
    if (len & 8u) {
        uint2 t = make_uint2(a, b);
        __builtin_memcpy(p, &t, 8);
        p += 8;
        a = c;
        b = d;
    }
    if (len & 4u) {
        __builtin_memcpy(p, &a, 4);
        p += 4;
        a = b;
    }
    if (len & 2u) {
        const uint16_t t = (uint16_t)a;
        __builtin_memcpy(p, &t, 2);
        p += 2;
        a >>= 16;
    }
    if (len & 1u) *p = (uint8_t)a;
}

#endif

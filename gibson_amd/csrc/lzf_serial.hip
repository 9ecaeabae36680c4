/*
 * lzf_serial.hip -- first-generation (single-lane) LZF kernels for gfx950.
 *
 * One workgroup of one wave per value; lane 0 runs the greedy parse / token
 * decode serially, the other lanes only stage input into LDS.  These kernels
 * are the simplest faithful device form of the reference and stay in the
 * library as the "serial" generation: selectable with LZF_GPU_KERNEL=serial,
 * cross-checked against the parallel generation by the GPU tests.
 *
 * Semantics follow src/lzf_c.c:98-294 and src/lzf_d.c:55-149 (see
 * oracle/lzf_oracle.c for the spec restatement); differences are only in
 * representation:
 *   - the slot table holds 16-bit positions in LDS (128 KiB) and is never
 *     cleared: output does not depend on its initial contents
 *      because every check the reference makes on a
 *     stale pointer (off < 8192, ref > start, 3 equal bytes) is kept;
 *   - nothing is written at or beyond out_cap (the reference can store one
 *     byte at out_end in a failing rollover case; output is unspecified on
 *     failure anyway).
 * Limits: compress takes values up to 65536 bytes (16-bit positions).
 */
#include "lzf_internal.h"

#define SER_STAGE_MAX 32768u

__device__ __forceinline__ uint32_t ser_slot(const uint8_t *b, uint32_t p)
{
    uint32_t hi = ((uint32_t)b[p] << 8) | b[p + 1];
    uint32_t lo = ((uint32_t)b[p + 1] << 8) | b[p + 2];
    return (hi - 5u * lo) & 0xFFFFu;
}

__global__ __launch_bounds__(64) void lzf_compress_serial_kernel(LzfBatch bt, uint32_t stage_cap)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint16_t *tab = (uint16_t *)smem;
    uint8_t *stage = smem + LZF_SLOTS * sizeof(uint16_t);

    const uint32_t v = blockIdx.x;
    const uint32_t n = bt.in_len[v];
    const uint8_t *src = bt.in + bt.in_off[v];
    const bool staged = n <= stage_cap;
    if (staged)
        for (uint32_t k = threadIdx.x; k < n; k += 64u) stage[k] = src[k];
    __syncthreads();
    if (threadIdx.x != 0) return;

    const uint8_t *b = staged ? (const uint8_t *)stage : src;
    uint8_t *out = bt.out + bt.out_off[v];
    const uint32_t cap = bt.out_cap[v];
    if (n == 0u || cap == 0u || n > 65536u) { bt.out_len[v] = 0u; return; }

    uint32_t o = 1u, run = 0u, p = 0u;
    bool ok = true;
    while (n >= 3u && p < n - 2u) {
        uint32_t s = ser_slot(b, p);
        uint32_t r = tab[s];
        tab[s] = (uint16_t)p;
        bool hit = r < p && (p - r - 1u) < LZF_WINDOW && p + 4u < n && r > 0u &&
                   b[r] == b[p] && b[r + 1] == b[p + 1] && b[r + 2] == b[p + 2];
        if (!hit) {
            if (o >= cap) { ok = false; break; }
            out[o++] = b[p++];
            if (++run == LZF_MAX_LIT) { out[o - 33u] = 31u; run = 0u; o++; }
            continue;
        }
        uint32_t maxlen = n - p - 2u;
        if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
        uint32_t lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
        uint32_t m = 3u;
        while (m < lim && b[r + m] == b[p + m]) m++;
        uint32_t off = p - r - 1u;
        if (run) out[o - run - 1u] = (uint8_t)(run - 1u);
        else o--;
        if (o + 4u >= cap) { ok = false; break; }
        uint32_t L = m - 2u;
        if (L < 7u) {
            out[o++] = (uint8_t)((off >> 8) | (L << 5));
        } else {
            out[o++] = (uint8_t)((off >> 8) | 0xE0u);
            out[o++] = (uint8_t)(L - 7u);
        }
        out[o++] = (uint8_t)off;
        run = 0u;
        o++;
        p += m;
        if (p >= n - 2u) break;
        tab[ser_slot(b, p - 2u)] = (uint16_t)(p - 2u);
        tab[ser_slot(b, p - 1u)] = (uint16_t)(p - 1u);
    }
    if (!ok || o + 3u > cap) { bt.out_len[v] = 0u; return; }
    while (p < n) {
        out[o++] = b[p++];
        if (++run == LZF_MAX_LIT) { out[o - 33u] = 31u; run = 0u; o++; }
    }
    if (run) out[o - run - 1u] = (uint8_t)(run - 1u);
    else o--;
    bt.out_len[v] = o;
}

__global__ __launch_bounds__(64) void lzf_decompress_serial_kernel(LzfBatch bt)
{
    if (threadIdx.x != 0) return;
    const uint32_t v = blockIdx.x;
    if (bt.skip && bt.skip[v]) return;
    const uint8_t *in = bt.in + bt.in_off[v];
    const uint32_t in_len = bt.in_len[v];
    uint8_t *out = bt.out + bt.out_off[v];
    const uint32_t cap = bt.out_cap[v];
    uint32_t i = 0, o = 0;
    int32_t err = 0;
    do {
        uint32_t c = in[i++];
        if (c < 32u) {
            uint32_t cnt = c + 1u;
            if ((uint64_t)o + cnt > cap) { err = 7; break; }        /* E2BIG */
            if ((uint64_t)i + cnt > in_len) { err = 22; break; }    /* EINVAL */
            for (uint32_t k = 0; k < cnt; k++) out[o + k] = in[i + k];
            o += cnt;
            i += cnt;
        } else {
            uint32_t len = c >> 5;
            if (i >= in_len) { err = 22; break; }
            if (len == 7u) {
                len += in[i++];
                if (i >= in_len) { err = 22; break; }
            }
            uint32_t back = ((c & 31u) << 8) + 1u + in[i++];
            if ((uint64_t)o + len + 2u > cap) { err = 7; break; }
            if (back > o) { err = 22; break; }
            for (uint32_t k = 0; k < len + 2u; k++) out[o + k] = out[o - back + k];
            o += len + 2u;
        }
    } while (i < in_len);
    bt.out_len[v] = err ? 0u : o;
    bt.err[v] = err;
}

hipError_t lzf_launch_compress_serial(const LzfBatch &b, hipStream_t s)
{
    uint32_t stage = b.max_len <= SER_STAGE_MAX ? b.max_len : 0u;
    size_t lds = LZF_SLOTS * sizeof(uint16_t) + ((stage + 15u) & ~15u);
    hipError_t e = hipFuncSetAttribute((const void *)lzf_compress_serial_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lzf_compress_serial_kernel, dim3(b.count), dim3(64), lds, s, b, stage);
    return hipGetLastError();
}

hipError_t lzf_launch_decompress_serial(const LzfBatch &b, hipStream_t s)
{
    hipLaunchKernelGGL(lzf_decompress_serial_kernel, dim3(b.count), dim3(64), 0, s, b);
    return hipGetLastError();
}

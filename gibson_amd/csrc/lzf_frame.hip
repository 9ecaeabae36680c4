/*
 * lzf_frame.hip -- the MGET / KEYS reply payload assembled in HBM, with the
 * LZF items decompressed straight into it.
 *
 * The reference builds the payload item by item on the host
 * (gbClientEnqueueKeyValueSet, src/net.c:1256-1342): a u32 element count,
 * then per non-null item [u32 key size][key][u8 encoding][u32 value size]
 * [value], where an LZF item is first decompressed into the shared
 * lzf_buffer (src/net.c:1301-1311) and then copied (src/net.c:1333-1335),
 * and framed again by gbClientEnqueueData (src/net.c:1162-1205) behind
 * [i16 code][u8 encoding][u32 size].  Here:
 *
 *   1. frame_size: per item its frame bytes; a block-local exclusive scan;
 *   2. frame_scan: exclusive scan of the block sums (one workgroup), the
 *      payload size and the max-response check (CHECK_SPACE, src/net.c:
 *      1272-1277: the per-write checks fail iff the final size exceeds);
 *   3. frame_write: one wave per item writes its headers and key, copies a
 *      PLAIN / NUMBER value, and describes an LZF item to the decoder: its
 *      output offset inside the frame and its recorded original length;
 *   4. the tokpar64 decoder over the same items (the others skipped)
 *      decodes every LZF value in place -- no lzf_buffer, no second copy;
 *   5. frame_check: every LZF item must decode to its recorded length.
 *
 * The decoded length of an LZF item must be known up front (the side table
 * of original lengths, §8(f) rank 3): the caller passes it in val_len.
 */
#include "lzf_internal.h"
#include "../../include/lzf_gpu.h"

#define FR_BLOCK 256u
#define FR_PER   4u
#define FR_TILE  (FR_BLOCK * FR_PER)

__device__ __forceinline__ uint64_t fr_item_bytes(const LzfFrameArgs &a, uint32_t i)
{
    const uint8_t e = a.enc[i];
    if (e == LZF_ENC_NULL) return 0;                      /* src/net.c:1287 */
    const uint32_t v = e == LZF_ENC_LZF ? a.val_len[i] : a.val_size[i];
    return 4ull + a.key_len[i] + 1ull + 4ull + v;
}

/* Block-wide exclusive scan of one u64 per thread (wave DPP scans would do;
 * this path is not the hot one, so plain LDS Hillis-Steele). */
__device__ uint64_t fr_block_excl(uint64_t x, uint64_t *sh, uint64_t *total)
{
    const uint32_t t = threadIdx.x;
    sh[t] = x;
    __syncthreads();
    for (uint32_t d = 1; d < FR_BLOCK; d <<= 1) {
        const uint64_t y = t >= d ? sh[t - d] : 0ull;
        __syncthreads();
        sh[t] += y;
        __syncthreads();
    }
    const uint64_t incl = sh[t];
    *total = sh[FR_BLOCK - 1];
    __syncthreads();
    return incl - x;
}

__global__ __launch_bounds__(FR_BLOCK) void lzf_frame_size_kernel(LzfFrameArgs a)
{
    __shared__ uint64_t sh[FR_BLOCK];
    const uint32_t base = blockIdx.x * FR_TILE + threadIdx.x * FR_PER;
    uint64_t sz[FR_PER], s = 0;
#pragma unroll
    for (uint32_t k = 0; k < FR_PER; k++) {
        sz[k] = base + k < a.count ? fr_item_bytes(a, base + k) : 0ull;
        s += sz[k];
    }
    uint64_t tot;
    uint64_t o = fr_block_excl(s, sh, &tot);
#pragma unroll
    for (uint32_t k = 0; k < FR_PER; k++) {
        if (base + k < a.count) a.w_off[base + k] = o;
        o += sz[k];
    }
    if (threadIdx.x == 0) a.w_bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(FR_BLOCK) void lzf_frame_scan_kernel(LzfFrameArgs a, uint32_t nblocks)
{
    __shared__ uint64_t sh[FR_BLOCK];
    uint64_t run = 0;
    for (uint32_t c = 0; c < nblocks; c += FR_BLOCK) {
        const uint32_t i = c + threadIdx.x;
        const uint64_t x = i < nblocks ? a.w_bsum[i] : 0ull;
        uint64_t tot;
        const uint64_t o = fr_block_excl(x, sh, &tot);
        if (i < nblocks) a.w_bsum[i] = run + o;
        run += tot;
    }
    if (threadIdx.x == 0) {
        const uint64_t payload = 4ull + run;              /* u32 element count + items */
        a.w_state[0] = payload;
        a.w_state[1] = payload > a.max_response ? 1ull : 0ull;   /* CHECK_SPACE */
    }
}

__device__ __forceinline__ void fr_put32(uint8_t *p, uint32_t x)
{
    p[0] = (uint8_t)x; p[1] = (uint8_t)(x >> 8); p[2] = (uint8_t)(x >> 16); p[3] = (uint8_t)(x >> 24);
}

/* one wave per item */
__global__ __launch_bounds__(64) void lzf_frame_write_kernel(LzfFrameArgs a)
{
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    const bool over = a.w_state[1] != 0ull;
    const uint64_t hdr = a.reply_header ? 7u : 0u;       /* [i16 code][u8 enc][u32 size] */
    if (i == 0 && lane == 0 && !over) {
        uint8_t *f = a.frame;
        if (a.reply_header) {
            f[0] = (uint8_t)LZF_REPL_KVAL; f[1] = (uint8_t)(LZF_REPL_KVAL >> 8);   /* src/net.c:1185 */
            f[2] = LZF_ENC_PLAIN;                                                 /* src/net.c:1339 */
            fr_put32(f + 3, (uint32_t)a.w_state[0]);
        }
        fr_put32(f + hdr, a.elements);                                            /* src/net.c:1282 */
    }
    const uint8_t e = a.enc[i];
    bool dec = false;
    if (!over && e != LZF_ENC_NULL) {
        const uint32_t kl = a.key_len[i];
        const uint32_t vl = e == LZF_ENC_LZF ? a.val_len[i] : a.val_size[i];
        uint8_t *f = a.frame + hdr + 4u + a.w_off[i] + a.w_bsum[i / FR_TILE];
        const uint8_t *key = a.keys + a.key_off[i];
        if (lane == 0) {
            fr_put32(f, kl);                                                      /* :1294 */
            f[4 + kl] = e == LZF_ENC_LZF ? LZF_ENC_PLAIN : e;                     /* :1313, :1331 */
            fr_put32(f + 5 + kl, vl);                                             /* :1332 */
        }
        for (uint32_t k = lane; k < kl; k += 64u) f[4 + k] = key[k];             /* :1295 */
        uint8_t *v = f + 9u + kl;
        if (e == LZF_ENC_LZF) {
            dec = true;
            if (lane == 0) a.w_voff[i] = (uint64_t)(v - a.frame);
        } else {
            const uint8_t *s = a.vals + a.val_off[i];
            for (uint32_t k = lane; k < vl; k += 64u) v[k] = s[k];               /* :1333 */
        }
    }
    if (lane == 0) a.w_skip[i] = dec ? 0u : 1u;
}

__global__ __launch_bounds__(FR_BLOCK) void lzf_frame_check_kernel(LzfFrameArgs a)
{
    __shared__ int bad;
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < a.count; i += FR_BLOCK)
        if (!a.w_skip[i] && (a.w_err[i] != 0 || a.w_len[i] != a.val_len[i])) bad = 1;
    __syncthreads();
    if (threadIdx.x == 0) {
        const bool ok = !bad && a.w_state[1] == 0ull;
        *a.frame_len = ok ? a.w_state[0] + (a.reply_header ? 7u : 0u) : 0ull;
    }
}

size_t lzf_frame_work_bytes(uint32_t count)
{
    const size_t nb = (count + FR_TILE - 1) / FR_TILE;
    /* off, voff (u64) | bsum (u64 per block) | state (2 x u64) | len, err (u32) | skip (u8) */
    return (size_t)count * (8 + 8 + 4 + 4 + 1) + nb * 8 + 16 + 64;
}

void lzf_frame_carve(LzfFrameArgs &a, void *work)
{
    const size_t nb = (a.count + FR_TILE - 1) / FR_TILE;
    uint8_t *w = (uint8_t *)(((uintptr_t)work + 7u) & ~(uintptr_t)7u);
    a.w_off = (uint64_t *)w;              w += (size_t)a.count * 8;
    a.w_voff = (uint64_t *)w;             w += (size_t)a.count * 8;
    a.w_bsum = (uint64_t *)w;             w += nb * 8;
    a.w_state = (uint64_t *)w;            w += 16;
    a.w_len = (uint32_t *)w;              w += (size_t)a.count * 4;
    a.w_err = (int32_t *)w;               w += (size_t)a.count * 4;
    a.w_skip = (uint8_t *)w;
}

hipError_t lzf_launch_frame(LzfFrameArgs &a, hipStream_t s,
                            hipError_t (*decode)(const LzfBatch &, hipStream_t))
{
    const uint32_t nb = (a.count + FR_TILE - 1) / FR_TILE;
    hipLaunchKernelGGL(lzf_frame_size_kernel, dim3(nb), dim3(FR_BLOCK), 0, s, a);
    hipLaunchKernelGGL(lzf_frame_scan_kernel, dim3(1), dim3(FR_BLOCK), 0, s, a, nb);
    hipLaunchKernelGGL(lzf_frame_write_kernel, dim3(a.count), dim3(64), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    LzfBatch b{};
    b.in = a.vals;
    b.in_off = a.val_off;
    b.in_len = a.val_size;
    b.out = a.frame;
    b.out_off = a.w_voff;
    b.out_cap = a.val_len;
    b.out_len = a.w_len;
    b.err = a.w_err;
    b.count = a.count;
    b.max_len = a.max_val_len;
    b.skip = a.w_skip;
    e = decode(b, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lzf_frame_check_kernel, dim3(1), dim3(FR_BLOCK), 0, s, a);
    return hipGetLastError();
}

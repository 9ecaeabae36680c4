/*
 * lzf_selfcheck.hip -- run-time check of the LDS behaviour the table, lane
 * and window compressor generations rely on.
 *
 * Their q1 step (lzf_cand.hip, lzf_lane.hip, lzf_wparse.hip) updates the
 * slot table with ONE ds_mskor_rtn_b32 per 64 positions: each lane replaces
 * the 16-bit half of its slot and gets the old dword back.  That is the
 * reference's sequential `ref = *hslot; *hslot = ip` (src/lzf_c.c:147-149)
 * only if the LDS executes a wave's same-address operations in lane order:
 * then every lane sees the nearest LOWER lane's write to its half (or the
 * table's value) and the highest lane's write is what stays.  gfx950 does
 * this (tools/lds_mskor_order.hip, profiles/r02/lds_mskor_order.txt), but it
 * is measured hardware behaviour, not a documented guarantee, so the library
 * re-checks it once per device before the first launch of those kernels and
 * routes compress batches to window64 (lzf_compress.hip, order-free
 * atomics only) when it does not hold.
 *
 * The probe: blocks of one wave, each lane one exchange on a 64-dword table
 * under 16 collision patterns (1 .. 128 halves, two lane -> half maps); every
 * lane checks its returned half and its table word against the lane-order
 * image it computes itself, and counts mismatches.
 */
#include <mutex>

#include "lzf_internal.h"

__device__ __forceinline__ uint32_t sc_half(uint32_t lane, uint32_t blk, uint32_t nhalf, uint32_t mode)
{
    return (mode == 0u ? (lane * 7u + blk) : ((lane * 2654435761u + blk * 40503u) >> 20)) % nhalf;
}

__global__ __launch_bounds__(64) void lzf_lds_order_probe_kernel(uint32_t *bad, uint32_t nhalf, uint32_t mode)
{
    __shared__ uint32_t T[64];
    const uint32_t lane = threadIdx.x, blk = blockIdx.x;
    T[lane] = 0xA5A5A5A5u;
    __syncthreads();
    const uint32_t h = sc_half(lane, blk, nhalf, mode), sh = (h & 1u) * 16u;
    const uint32_t addr = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint32_t *)&T[h >> 1];
    const uint32_t mask = 0xFFFFu << sh, data = (lane + 1u) << sh;
    uint32_t r;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(r) : "v"(addr), "v"(mask), "v"(data) : "memory");
    __syncthreads();
    /* lane order: the nearest lower lane on the same half, else the initial
     * value; the final word: per half, the highest lane writing it */
    uint32_t exp = 0xA5A5u, lo = 0xA5A5u, hi = 0xA5A5u;
    for (uint32_t l = 0; l < 64u; l++) {
        const uint32_t hl = sc_half(l, blk, nhalf, mode);
        if (l < lane && hl == h) exp = l + 1u;
        if (hl == 2u * lane) lo = l + 1u;
        if (hl == 2u * lane + 1u) hi = l + 1u;
    }
    uint32_t n = ((r >> sh) & 0xFFFFu) != exp ? 1u : 0u;
    n += T[lane] != (lo | (hi << 16)) ? 1u : 0u;
    if (n) atomicAdd(bad, n);
}

/* mismatch count over all patterns (0: lane order held), or a negative
 * LZF_GPU_E* code.  Runs on a non-blocking stream of its own with a counter
 * and a pinned result word made once per device, so it neither waits for
 * nor holds up the caller's streams (the device is not synchronised). */
int lzf_lds_order_check(int dev)
{
    static std::mutex mu;
    static hipStream_t st[64];
    static uint32_t *cnt[64], *res[64];
    if (dev < 0 || dev >= 64) return -2;
    std::lock_guard<std::mutex> lk(mu);
    if (!st[dev] && hipStreamCreateWithFlags(&st[dev], hipStreamNonBlocking) != hipSuccess) {
        st[dev] = nullptr;
        return -2;
    }
    if (!cnt[dev] && hipMalloc(&cnt[dev], sizeof(uint32_t)) != hipSuccess) {
        cnt[dev] = nullptr;
        return -4;
    }
    if (!res[dev] && hipHostMalloc(&res[dev], sizeof(uint32_t), hipHostMallocDefault) != hipSuccess) {
        res[dev] = nullptr;
        return -4;
    }
    int rc = hipMemsetAsync(cnt[dev], 0, sizeof(uint32_t), st[dev]) == hipSuccess ? 0 : -2;
    for (uint32_t mode = 0; mode < 2u && !rc; mode++)
        for (uint32_t nh = 1; nh <= 128u && !rc; nh *= 2u) {
            hipLaunchKernelGGL(lzf_lds_order_probe_kernel, dim3(1024), dim3(64), 0, st[dev], cnt[dev], nh, mode);
            if (hipGetLastError() != hipSuccess) rc = -2;
        }
    if (!rc && hipMemcpyAsync(res[dev], cnt[dev], sizeof(uint32_t), hipMemcpyDeviceToHost, st[dev]) != hipSuccess)
        rc = -2;
    if (!rc && hipStreamSynchronize(st[dev]) != hipSuccess) rc = -2;
    (void)hipGetLastError();
    return rc ? rc : (int)*res[dev];
}

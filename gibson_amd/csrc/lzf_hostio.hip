/*
 * lzf_hostio.hip -- value moves between caller host memory and the device
 * arenas of a host-memory batch, done by the GPU itself.
 *
 * The host-memory calls (lzf_host_compress_batch / lzf_host_decompress_batch,
 * include/lzf_gpu.h) start in the client's request buffer and end in the
 * trie-resident value (src/server.c:180, src/query.c:409, src/net.c:1229).
 * When the caller has registered those arenas (lzf_host_register: page-locked
 * and mapped into the device address space), no CPU copies a value byte: this
 * kernel reads each value from the mapped host arena into the packed device
 * arena (gather), and writes each stream, exactly out_len[k] bytes, from the
 * device arena into its slot of the mapped host arena (scatter).  Measured on
 * the MI355X box (tools/probe/pcie_probe.hip): mapped reads 55.9 GB/s, mapped
 * writes 54.7 GB/s, both at the pinned hipMemcpyAsync rate (57.6 / 57.0).
 *
 * One workgroup per value (grid-stride over values), 16-byte accesses in the
 * body; the host lays the device side out so that both ends of every move
 * have the same address mod 16 (a move whose ends do not is copied byte by
 * byte, so a wrong layout costs speed, never correctness).
 */
#include "lzf_internal.h"

__global__ __launch_bounds__(256) void lzf_move_kernel(const uint8_t *__restrict__ src,
                                                       const uint64_t *__restrict__ src_off,
                                                       uint8_t *__restrict__ dst,
                                                       const uint64_t *__restrict__ dst_off,
                                                       const uint32_t *__restrict__ len, uint32_t min_len,
                                                       uint32_t count)
{
    for (uint32_t k = blockIdx.x; k < count; k += gridDim.x) {
        const uint8_t *s = src + src_off[k];
        uint8_t *d = dst + dst_off[k];
        uint32_t n = len[k];
        if (n < min_len) n = min_len;
        if ((((uintptr_t)s ^ (uintptr_t)d) & 15u) != 0u) {
            for (uint32_t j = threadIdx.x; j < n; j += blockDim.x) d[j] = s[j];
            continue;
        }
        uint32_t head = (uint32_t)((16u - ((uintptr_t)s & 15u)) & 15u);
        if (head > n) head = n;
        if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
        const uint32_t body = (n - head) >> 4;
        const uint4 *s16 = (const uint4 *)(s + head);
        uint4 *d16 = (uint4 *)(d + head);
        /* four 16-byte loads in flight per lane before the stores: a PCIe
         * round trip is microseconds, so the loads are what must overlap */
        uint32_t j = threadIdx.x;
        for (; j + 768u < body; j += 1024u) {
            const uint4 a = s16[j], b = s16[j + 256u], c = s16[j + 512u], e = s16[j + 768u];
            d16[j] = a;
            d16[j + 256u] = b;
            d16[j + 512u] = c;
            d16[j + 768u] = e;
        }
        for (; j < body; j += 256u) d16[j] = s16[j];
        const uint32_t t0 = head + (body << 4);
        if (threadIdx.x < n - t0) d[t0 + threadIdx.x] = s[t0 + threadIdx.x];
    }
}

hipError_t lzf_launch_move(const uint8_t *src, const uint64_t *src_off, uint8_t *dst, const uint64_t *dst_off,
                           const uint32_t *len, uint32_t min_len, uint32_t count, hipStream_t s)
{
    if (!count) return hipSuccess;
    const uint32_t grid = count < 65536u ? count : 65536u;
    hipLaunchKernelGGL(lzf_move_kernel, dim3(grid), dim3(256), 0, s, src, src_off, dst, dst_off, len, min_len,
                       count);
    return hipGetLastError();
}

/* Registered decode: the slots of values whose outputs abut go back to the
 * caller as one DMA run of their whole capacity.  The bytes of a slot past
 * its decoded length (a short or failed decode) would then carry whatever an
 * earlier chunk or batch left in the device arena -- other requests' values.
 * They are zeroed first, so a DMA run writes only this value's bytes and
 * zeros.  One workgroup per value (grid-stride); most slots are full
 * (out_len == cap) and return at once. */
__global__ __launch_bounds__(256) void lzf_clear_tail_kernel(uint8_t *__restrict__ dst,
                                                             const uint64_t *__restrict__ dst_off,
                                                             const uint32_t *__restrict__ len,
                                                             const uint32_t *__restrict__ cap, uint32_t count)
{
    for (uint32_t k = blockIdx.x; k < count; k += gridDim.x) {
        const uint32_t lo = len[k], hi = cap[k];
        if (lo >= hi) continue;
        uint8_t *d = dst + dst_off[k];
        for (uint32_t j = lo + threadIdx.x; j < hi; j += blockDim.x) d[j] = 0u;
    }
}

hipError_t lzf_launch_clear_tail(uint8_t *dst, const uint64_t *dst_off, const uint32_t *len, const uint32_t *cap,
                                 uint32_t count, hipStream_t s)
{
    if (!count) return hipSuccess;
    const uint32_t grid = count < 65536u ? count : 65536u;
    hipLaunchKernelGGL(lzf_clear_tail_kernel, dim3(grid), dim3(256), 0, s, dst, dst_off, len, cap, count);
    return hipGetLastError();
}

/*
 * fetch_calib.hip -- calibrates rocprofv3 FETCH_SIZE for the access shape of
 * the lane parse kernel (every lane of a wave loads 16 bytes from its own
 * line) against a coalesced stream of the same byte count.  The guide's
 * doubling correction is calibrated only for coalesced streaming reads.
 *
 *   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o /tmp/fetch_calib
 *   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- /tmp/fetch_calib
 * Each kernel reads NLOADS x 16 B from a 4 GiB buffer (beyond the 256 MiB
 * Infinity Cache), every 128-byte line at most once.
 */
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define LINES (1u << 25)            /* 4 GiB of 128-byte lines */

__global__ void scattered16(const uint4 *buf, uint32_t nloads, uint32_t *out, uint32_t lmask)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nloads) return;
    const uint32_t line = (i * 2654435761u) & lmask;          /* odd multiplier: a permutation */
    const uint4 v = buf[(uint64_t)line * 8u];                 /* 16 B at the start of the line */
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = i;
}

__global__ void scattered16_mid(const uint4 *buf, uint32_t nloads, uint32_t *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nloads) return;
    const uint32_t line = (i * 2654435761u) & (LINES - 1u);
    const uint4 v = buf[(uint64_t)line * 8u + 5u];            /* 16 B at byte 80 of the line */
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = i;
}

__global__ void coalesced16(const uint4 *buf, uint32_t nloads, uint32_t *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nloads) return;
    const uint4 v = buf[i];
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) out[0] = i;
}

int main()
{
    const uint32_t nloads = 1u << 24;              /* 16 M loads = 256 MiB requested */
    uint4 *buf;
    uint32_t *out;
    if (hipMalloc(&buf, (size_t)LINES * 128u) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) {
        printf("alloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, (size_t)LINES * 128u);
    hipDeviceSynchronize();
    const dim3 g((nloads + 255u) / 256u), b(256);
    hipLaunchKernelGGL(coalesced16, g, b, 0, 0, buf + (size_t)LINES * 4u, nloads, out);
    hipLaunchKernelGGL(scattered16, g, b, 0, 0, buf, nloads, out, LINES - 1u);
    /* the same loads over 128 MiB (Infinity Cache) and 16 MiB (L2) of lines */
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(scattered16, g, b, 0, 0, buf, nloads, out, (1u << 20) - 1u);
        hipLaunchKernelGGL(scattered16, g, b, 0, 0, buf, nloads, out, (1u << 17) - 1u);
    }
    hipLaunchKernelGGL(scattered16_mid, g, b, 0, 0, buf, nloads, out);
    hipDeviceSynchronize();
    printf("loads per kernel %u, bytes requested %llu (16 B each)\n", nloads, (unsigned long long)nloads * 16ull);
    hipFree(buf);
    hipFree(out);
    return 0;
}

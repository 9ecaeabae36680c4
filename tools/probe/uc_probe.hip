/*
 * uc_probe.hip -- what a scattered one-line-per-lane access costs by memory
 * type (the record parse's bound at configs[2]'s size, DESIGN.md §4.1: ~21 k
 * scattered 128-byte line fetches per value at the one-line-per-lane ceiling).
 * A 4 GiB buffer (beyond the 256 MiB Infinity Cache) allocated three ways --
 * hipMalloc (coarse-grained, L2-cached), hipExtMallocWithFlags Finegrained and
 * Uncached -- and, for each, 64 M accesses at random lines (every lane its own
 * line) of 4, 16 and 64 bytes (loads) and 16-byte stores.  Prints G
 * accesses per second.
 *   hipcc --offload-arch=gfx950 -O3 tools/probe/uc_probe.hip -o tools/probe/uc_probe_bin
 */
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define LINES (1u << 25)            /* 4 GiB of 128-byte lines */

__device__ __forceinline__ uint32_t line_of(uint32_t i) { return (i * 2654435761u) & (LINES - 1u); }

template <int BYTES>
__global__ __launch_bounds__(256) void gather(const uint32_t *buf, uint32_t n, uint32_t *out)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t *p = buf + (uint64_t)line_of(i) * 32u + (i & 1u) * 16u;   /* either half of the line */
    uint32_t acc;
    if (BYTES == 4) {
        acc = p[3];
    } else if (BYTES == 16) {
        const uint4 v = *(const uint4 *)p;
        acc = v.x ^ v.y ^ v.z ^ v.w;
    } else {
        const uint4 a = ((const uint4 *)p)[0], b = ((const uint4 *)p)[1], c = ((const uint4 *)p)[2],
                    d = ((const uint4 *)p)[3];
        acc = a.x ^ b.y ^ c.z ^ d.w;
    }
    if (acc == 0x12345678u) out[0] = i;
}

__global__ __launch_bounds__(256) void scatter16(uint32_t *buf, uint32_t n)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint4 *p = (uint4 *)(buf + (uint64_t)line_of(i) * 32u + (i & 1u) * 16u);
    *p = make_uint4(i, i, i, i);
}

__global__ void fill(uint32_t *buf, uint64_t words)
{
    for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < words; k += (uint64_t)gridDim.x * blockDim.x)
        buf[k] = (uint32_t)(k * 0x9E3779B9u);
}

int main()
{
    const char *names[3] = {"hipMalloc (coarse)", "Finegrained", "Uncached"};
    const unsigned flags[3] = {0u, hipDeviceMallocFinegrained, hipDeviceMallocUncached};
    uint32_t *out;
    hipMalloc(&out, 64);
    const uint32_t n = 1u << 26;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int t = 0; t < 3; t++) {
        uint32_t *buf = nullptr;
        const hipError_t e = t == 0 ? hipMalloc(&buf, (size_t)LINES * 128u)
                                    : hipExtMallocWithFlags((void **)&buf, (size_t)LINES * 128u, flags[t]);
        if (e != hipSuccess) {
            printf("%-20s alloc failed: %s\n", names[t], hipGetErrorString(e));
            (void)hipGetLastError();
            continue;
        }
        hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, buf, (uint64_t)LINES * 32u);
        hipDeviceSynchronize();
        const dim3 g(n / 256u), b(256);
        float ms[4];
        for (int k = 0; k < 4; k++) {
            for (int rep = 0; rep < 2; rep++) {
                hipEventRecord(e0);
                if (k == 0) hipLaunchKernelGGL(gather<4>, g, b, 0, 0, buf, n, out);
                if (k == 1) hipLaunchKernelGGL(gather<16>, g, b, 0, 0, buf, n, out);
                if (k == 2) hipLaunchKernelGGL(gather<64>, g, b, 0, 0, buf, n, out);
                if (k == 3) hipLaunchKernelGGL(scatter16, g, b, 0, 0, buf, n);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                hipEventElapsedTime(&ms[k], e0, e1);
            }
        }
        printf("%-20s gather4 %6.1f  gather16 %6.1f  gather64 %6.1f  scatter16 %6.1f G/s\n", names[t],
               n / ms[0] / 1e6, n / ms[1] / 1e6, n / ms[2] / 1e6, n / ms[3] / 1e6);
        hipFree(buf);
    }
    return 0;
}

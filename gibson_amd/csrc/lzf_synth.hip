/*
 * lzf_synth.hip -- device-side synthetic value generation (synth.h), so
 * bench.py and the GPU tests build multi-GiB batches directly in HBM.
 * One thread per value: generation is setup, never inside a timed region.
 */
#include "lzf_internal.h"
#include "synth.h"

__global__ __launch_bounds__(256) void lzf_synth_kernel(int kind, uint64_t seed, uint64_t first,
                                                        uint64_t stride, uint32_t count,
                                                        uint32_t n, uint8_t *out)
{
    uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= count) return;
    syn_generate(kind, seed, first + (uint64_t)k * stride, out + (uint64_t)k * n, n);
}

hipError_t lzf_launch_synth(int kind, uint64_t seed, uint64_t first, uint64_t stride,
                            uint32_t count, uint32_t n, uint8_t *out, hipStream_t s)
{
    hipLaunchKernelGGL(lzf_synth_kernel, dim3((count + 255u) / 256u), dim3(256), 0, s,
                       kind, seed, first, stride, count, n, out);
    return hipGetLastError();
}

/*
 * lds_order2.hip -- does the LDS process a wave's same-address operations in
 * lane order? (1) ds_or_rtn_b64: each lane gets back the OR of the bits of
 * the lower lanes with the same address; (2) ds_write_b16: the highest lane's
 * value is the one left.  Prints mismatch counts (0 = lane order held).
 *   hipcc --offload-arch=gfx950 -O3 tools/lds_order2.hip -o tools/lds_order2_bin
 */
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ unsigned addr_of(unsigned lane, unsigned blk, int naddr, int mode)
{
    return (mode == 0) ? (lane * 7u + blk) % naddr : ((lane * 2654435761u + blk * 40503u) >> 26) % naddr;
}

__global__ void k(unsigned long long *rtn, unsigned short *fin, int naddr, int mode)
{
    __shared__ unsigned long long T[64];
    __shared__ unsigned short W[64];
    const unsigned lane = threadIdx.x;
    T[lane] = 0ull;
    W[lane] = 0xFFFFu;
    __syncthreads();
    const unsigned a = addr_of(lane, blockIdx.x, naddr, mode);
    rtn[blockIdx.x * 64 + lane] = __hip_atomic_fetch_or(&T[a], 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    W[a] = (unsigned short)lane;
    __syncthreads();
    fin[blockIdx.x * 64 + lane] = W[lane];
}

int main()
{
    const int B = 1024;
    unsigned long long *dr, *hr = new unsigned long long[B * 64];
    unsigned short *df, *hf = new unsigned short[B * 64];
    hipMalloc(&dr, sizeof(unsigned long long) * B * 64);
    hipMalloc(&df, sizeof(unsigned short) * B * 64);
    for (int mode = 0; mode < 2; mode++)
        for (int naddr = 1; naddr <= 64; naddr *= 2) {
            hipLaunchKernelGGL(k, dim3(B), dim3(64), 0, 0, dr, df, naddr, mode);
            hipMemcpy(hr, dr, sizeof(unsigned long long) * B * 64, hipMemcpyDeviceToHost);
            hipMemcpy(hf, df, sizeof(unsigned short) * B * 64, hipMemcpyDeviceToHost);
            long bad_or = 0, bad_w = 0;
            for (int b = 0; b < B; b++) {
                for (unsigned l = 0; l < 64; l++) {
                    unsigned long long exp = 0;
                    const unsigned a = (mode == 0) ? (l * 7u + b) % naddr : ((l * 2654435761u + b * 40503u) >> 26) % naddr;
                    for (unsigned m = 0; m < l; m++) {
                        const unsigned am = (mode == 0) ? (m * 7u + b) % naddr : ((m * 2654435761u + b * 40503u) >> 26) % naddr;
                        if (am == a) exp |= 1ull << m;
                    }
                    if (hr[b * 64 + l] != exp) bad_or++;
                }
                for (unsigned s = 0; s < 64; s++) {
                    unsigned last = 0xFFFFu;
                    for (unsigned m = 0; m < 64; m++) {
                        const unsigned am = (mode == 0) ? (m * 7u + b) % naddr : ((m * 2654435761u + b * 40503u) >> 26) % naddr;
                        if (am == s) last = m;
                    }
                    if (hf[b * 64 + s] != last) bad_w++;
                }
            }
            printf("mode %d naddr %2d: or_rtn mismatches %ld, write-last mismatches %ld (of %d)\n", mode, naddr,
                   bad_or, bad_w, B * 64);
        }
    return 0;
}

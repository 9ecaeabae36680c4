#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned *out, int naddr, int mode)
{
    __shared__ unsigned H[64];
    unsigned lane = threadIdx.x;
    H[lane] = 0;
    __syncthreads();
    unsigned a = (mode == 0) ? (lane * 7u + blockIdx.x) % naddr : ((lane * 2654435761u) >> 26) % naddr;
    unsigned key = (lane + 1u) << 16 | a;
    unsigned r = atomicMax(&H[a], key);
    out[blockIdx.x * 64 + lane] = r;
}
int main()
{
    unsigned *d, h[64 * 1024];
    hipMalloc(&d, sizeof(h));
    long bad = 0, tot = 0;
    for (int mode = 0; mode < 2; mode++)
    for (int naddr = 1; naddr <= 32; naddr *= 2) {
        hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, d, naddr, mode);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        for (int b = 0; b < 1024; b++)
            for (int l = 0; l < 64; l++) {
                unsigned a = (mode == 0) ? (l * 7u + b) % naddr : ((l * 2654435761u) >> 26) % naddr;
                unsigned exp = 0;
                for (int m = 0; m < l; m++) {
                    unsigned am = (mode == 0) ? (m * 7u + b) % naddr : ((m * 2654435761u) >> 26) % naddr;
                    if (am == a) exp = ((m + 1u) << 16) | am;
                }
                tot++;
                if (h[b * 64 + l] != exp) bad++;
            }
        printf("mode %d naddr %d: mismatches %ld / %ld\n", mode, naddr, bad, tot);
        bad = tot = 0;
    }
    return 0;
}

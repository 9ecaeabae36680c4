/*
 * lds_mskor_order.hip -- does gfx950's LDS process a wave's same-address
 * ds_mskor_rtn_b32 in lane order?  Each lane replaces one 16-bit half of a
 * dword (mask = the half, data = lane + 1 in that half) and gets the old
 * dword back.  Lane order means: the returned half is the value of the
 * nearest LOWER lane that wrote the same half (else the initial value), the
 * other half is never clobbered, and the final half is the highest lane's.
 * That is an exchange on 16-bit table entries -- the cand kernel's q1 in one
 * LDS instruction.  Prints mismatch counts (0 = lane order held).
 *   hipcc --offload-arch=gfx950 -O3 tools/lds_mskor_order.hip -o tools/lds_mskor_order_bin
 */
#include <hip/hip_runtime.h>
#include <stdio.h>

__host__ __device__ unsigned half_of(unsigned lane, unsigned blk, int nhalf, int mode)
{
    return (mode == 0) ? (lane * 7u + blk) % nhalf : ((lane * 2654435761u + blk * 40503u) >> 20) % nhalf;
}

__global__ void k(unsigned *rtn, unsigned *fin, int nhalf, int mode)
{
    __shared__ unsigned T[64];
    const unsigned lane = threadIdx.x;
    T[lane] = 0xA5A5A5A5u;
    __syncthreads();
    const unsigned h = half_of(lane, blockIdx.x, nhalf, mode);
    const unsigned sh = (h & 1u) * 16u;
    const unsigned addr = (unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned *)&T[h >> 1];
    const unsigned mask = 0xFFFFu << sh, data = (lane + 1u) << sh;
    unsigned r;
    asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(r) : "v"(addr), "v"(mask), "v"(data) : "memory");
    rtn[blockIdx.x * 64 + lane] = r;
    __syncthreads();
    fin[blockIdx.x * 64 + lane] = T[lane];
}

int main()
{
    const int nb = 1024;
    unsigned *dr, *df;
    static unsigned hr[64 * 1024], hf[64 * 1024];
    hipMalloc(&dr, sizeof(hr));
    hipMalloc(&df, sizeof(hf));
    long bad_r = 0, bad_f = 0, tot = 0;
    for (int mode = 0; mode < 2; mode++)
        for (int nhalf = 1; nhalf <= 128; nhalf *= 2) {
            hipLaunchKernelGGL(k, dim3(nb), dim3(64), 0, 0, dr, df, nhalf, mode);
            hipMemcpy(hr, dr, sizeof(hr), hipMemcpyDeviceToHost);
            hipMemcpy(hf, df, sizeof(hf), hipMemcpyDeviceToHost);
            long br = 0, bf = 0;
            for (int b = 0; b < nb; b++) {
                unsigned img[64];
                for (int i = 0; i < 64; i++) img[i] = 0xA5A5A5A5u;
                for (unsigned l = 0; l < 64; l++) {
                    const unsigned h = half_of(l, b, nhalf, mode), sh = (h & 1u) * 16u;
                    const unsigned got = (hr[b * 64 + l] >> sh) & 0xFFFFu, exp = (img[h >> 1] >> sh) & 0xFFFFu;
                    if (got != exp) br++;
                    img[h >> 1] = (img[h >> 1] & ~(0xFFFFu << sh)) | ((l + 1u) << sh);
                    tot++;
                }
                for (int i = 0; i < 64; i++)
                    if (hf[b * 64 + i] != img[i]) bf++;
            }
            printf("mode %d halves %3d: returned-half mismatches %ld, final-table mismatches %ld\n", mode, nhalf, br,
                   bf);
            bad_r += br;
            bad_f += bf;
        }
    printf("mskor lane order: %s (%ld / %ld lanes, %ld final words)\n", (bad_r || bad_f) ? "VIOLATED" : "held",
           bad_r, tot, bad_f);
    return (bad_r || bad_f) ? 1 : 0;
}

// Probe: unaligned 16-byte LDS reads/writes (ds_read_b128 / ds_write_b128 at
// any byte offset) on gfx950 -- the compiler emits them for unknown
// alignment; this checks the hardware result byte for byte.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
__global__ void k(uint8_t *out)
{
    __shared__ __attribute__((aligned(16))) uint8_t lds[4096 + 64];
    const uint32_t t = threadIdx.x;
    for (uint32_t i = t; i < 4096 + 64; i += 64) lds[i] = 0;
    __syncthreads();
    // lane t writes 16 bytes (t*16+1 .. ) at offset 17*t + (t % 16)
    const uint32_t wa = 40u * t + (t & 15u);
    uint4 v;
    uint8_t b[16];
    for (int i = 0; i < 16; i++) b[i] = (uint8_t)(t * 16 + i + 1);
    __builtin_memcpy(&v, b, 16);
    __builtin_memcpy(lds + wa, &v, 16);
    __syncthreads();
    uint4 r;
    __builtin_memcpy(&r, lds + wa, 16);
    __builtin_memcpy(out + 16 * t, &r, 16);
    // a read straddling two lanes' data at offset wa + 8
    uint4 r2;
    __builtin_memcpy(&r2, lds + wa + 3, 16);
    __builtin_memcpy(out + 1024 + 16 * t, &r2, 16);
}
int main()
{
    uint8_t *d, h[2048];
    hipMalloc(&d, 2048);
    k<<<1, 64>>>(d);
    hipMemcpy(h, d, 2048, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int t = 0; t < 64; t++)
        for (int i = 0; i < 16; i++) {
            if (h[16 * t + i] != (uint8_t)(t * 16 + i + 1)) bad++;
            uint8_t e = i + 3 < 16 ? (uint8_t)(t * 16 + i + 3 + 1) : 0;   // 40-byte spacing: zeros after
            if (h[1024 + 16 * t + i] != e) bad++;
        }
    printf("unaligned LDS b128: %s (%d bad bytes)\n", bad ? "WRONG" : "ok", bad);
    return bad != 0;
}

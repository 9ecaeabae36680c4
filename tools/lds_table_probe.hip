/*
 * lds_table_probe.hip -- cost of one table step on gfx950's LDS, per window of
 * 64 random 16-bit slots in a 65536-entry u16 table (the cand kernels' T):
 *   mode 0  ds_mskor_rtn_b32 exchange (the product's table step), 15 per step
 *   mode 1  plain ds_read_u16 + ds_write_b16 + ds_read_u16 read-back
 *   mode 2  plain ds_read_u16 + ds_write_b16
 *   mode 3  ds_read_u16 only
 * issued by one wave per CU, 15 windows per asm batch, one wait per batch
 * (as the table wave does), over `iters` steps; prints cycles per window.
 * Also checks the ordering the plain form would rely on: one ds_write_b16
 * whose lanes share addresses leaves the highest lane's value.
 *   hipcc --offload-arch=gfx950 -O3 tools/lds_table_probe.hip -o tools/lds_table_probe_bin
 */
#include <hip/hip_runtime.h>
#include <stdio.h>

__device__ __forceinline__ unsigned hsh(unsigned x)
{
    x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned lds_addr(const void *p)
{
    return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

#define X5(i) "ds_mskor_rtn_b32 %" #i ", %[a" #i "], %[m" #i "], %[d" #i "]\n\t"
#define P5(i) "ds_read_u16 %" #i ", %[h" #i "]\n\tds_write_b16 %[h" #i "], %[d" #i "]\n\t"

template <int MODE>
__global__ __launch_bounds__(256) void tk(unsigned long long *cyc, unsigned *sink, int iters, int dup, int dense)
{
    __shared__ __attribute__((aligned(16))) unsigned short T[65536 + 64];
    const unsigned lane = threadIdx.x & 63u, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (unsigned i = threadIdx.x; i < 65536u / 2u; i += blockDim.x) ((unsigned *)T)[i] = 0u;
    __syncthreads();
    const unsigned tb = lds_addr(T);
    unsigned acc = 0;
    /* slots precomputed per window; an iteration adds one uniform (even)
     * offset, so the timed loop spends ~2 VALU per window on addressing */
    unsigned hb[15];
#pragma unroll
    for (unsigned i = 0; i < 15u; i++) {
        const unsigned key = dup ? (lane >> 2) : lane;             /* dup: groups of 4 lanes share a slot */
        hb[i] = hsh(key * 131u + i * 31u + blockIdx.x * 7919u) & 0xFFFFu;
    }
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
        const unsigned off = (unsigned)__builtin_amdgcn_readfirstlane((int)(((unsigned)it * 2654435761u) >> 16)) & 0xFFFEu;
#pragma unroll
        for (unsigned g = 0; g < 15u; g += 5u) {
            unsigned h[5], a[5], m[5], d[5], r[5], t[5];
#pragma unroll
            for (unsigned u = 0; u < 5u; u++) {
                h[u] = (hb[g + u] + off) & 0xFFFFu;
                const unsigned sh = (h[u] & 1u) << 4;
                a[u] = tb + 4u * (h[u] >> 1);
                m[u] = 0xFFFFu << sh;
                d[u] = (((unsigned)it * 960u + (g + u) * 64u + lane) & 0xFFFFu) << sh;
                h[u] = tb + 2u * h[u];
            }
            if (MODE == 0) {
                /* per window, the lanes whose slot this wave owns (slot pair
                 * mod nw; nw = 1: all lanes), then one wait that "writes" the
                 * results, so nothing reads them before it */
#pragma unroll
                for (unsigned u = 0; u < 5u; u++) {
                    r[u] = 0u;
                    /* dense: whole windows dealt to the waves (the compacted
                     * slot-partition packets of a split table role); else
                     * every wave issues every window, exec-masked by slot */
                    if (dense ? ((g + u) % nw == wv) : ((h[u] >> 2) % nw == wv))
                        asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3" : "=&v"(r[u]) : "v"(a[u]), "v"(m[u]), "v"(d[u]) : "memory");
                }
                asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]) :: "memory");
                acc += r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4];
            } else if (MODE == 1 || MODE == 2) {
                unsigned dd[5];
#pragma unroll
                for (unsigned u = 0; u < 5u; u++) dd[u] = ((unsigned)it * 960u + (g + u) * 64u + lane) & 0xFFFFu;
                if (MODE == 1) {
                    asm volatile(P5(0) "ds_read_u16 %5, %[h0]\n\t" P5(1) "ds_read_u16 %6, %[h1]\n\t"
                                 P5(2) "ds_read_u16 %7, %[h2]\n\t" P5(3) "ds_read_u16 %8, %[h3]\n\t"
                                 P5(4) "ds_read_u16 %9, %[h4]\n\t" "s_waitcnt lgkmcnt(0)"
                                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4]),
                                   "=&v"(t[0]), "=&v"(t[1]), "=&v"(t[2]), "=&v"(t[3]), "=&v"(t[4])
                                 : [h0] "v"(h[0]), [d0] "v"(dd[0]), [h1] "v"(h[1]), [d1] "v"(dd[1]),
                                   [h2] "v"(h[2]), [d2] "v"(dd[2]), [h3] "v"(h[3]), [d3] "v"(dd[3]),
                                   [h4] "v"(h[4]), [d4] "v"(dd[4])
                                 : "memory");
                    acc += r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4] ^ t[0] ^ t[1] ^ t[2] ^ t[3] ^ t[4];
                } else {
                    asm volatile(P5(0) P5(1) P5(2) P5(3) P5(4) "s_waitcnt lgkmcnt(0)"
                                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
                                 : [h0] "v"(h[0]), [d0] "v"(dd[0]), [h1] "v"(h[1]), [d1] "v"(dd[1]),
                                   [h2] "v"(h[2]), [d2] "v"(dd[2]), [h3] "v"(h[3]), [d3] "v"(dd[3]),
                                   [h4] "v"(h[4]), [d4] "v"(dd[4])
                                 : "memory");
                    acc += r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4];
                }
            } else {
                asm volatile("ds_read_u16 %0, %5\n\tds_read_u16 %1, %6\n\tds_read_u16 %2, %7\n\t"
                             "ds_read_u16 %3, %8\n\tds_read_u16 %4, %9\n\ts_waitcnt lgkmcnt(0)"
                             : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
                             : "v"(h[0]), "v"(h[1]), "v"(h[2]), "v"(h[3]), "v"(h[4])
                             : "memory");
                acc += r[0] ^ r[1] ^ r[2] ^ r[3] ^ r[4];
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
    sink[blockIdx.x * 256 + threadIdx.x] = acc;
}

/* plain-store ordering: lanes grouped onto shared u16 addresses, one
 * ds_write_b16 of lane + 1; the final entry must be the highest lane's */
__global__ void ok(unsigned *bad, int ngrp)
{
    __shared__ unsigned short T[256];
    const unsigned lane = threadIdx.x;
    for (unsigned i = lane; i < 256u; i += 64u) T[i] = 0xFFFFu;
    __syncthreads();
    const unsigned g = hsh(lane * 2654435761u + blockIdx.x * 40503u) % (unsigned)ngrp;
    const unsigned a = lds_addr(&T[g]);
    const unsigned d = lane + 1u;
    asm volatile("ds_write_b16 %0, %1\n\ts_waitcnt lgkmcnt(0)" ::"v"(a), "v"(d) : "memory");
    __syncthreads();
    /* expected: the highest lane of group g */
    unsigned hi = 0;
    for (unsigned l = 0; l < 64u; l++)
        if (hsh(l * 2654435761u + blockIdx.x * 40503u) % (unsigned)ngrp == g) hi = l + 1u;
    if (T[g] != hi) atomicAdd(bad, 1u);
}

int main()
{
    int dev = 0, cus = 256;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    unsigned long long *dc;
    unsigned *ds, *db;
    hipMalloc(&dc, sizeof(unsigned long long) * cus);
    hipMalloc(&ds, sizeof(unsigned) * cus * 256);
    hipMalloc(&db, sizeof(unsigned));
    static unsigned long long hc[1024];
    const int iters = 2000;
    const char *nm[4] = {"mskor_rtn exchange", "read+write+readback", "read+write", "read only"};
    for (int dup = 0; dup < 2; dup++)
        for (int mode = 0; mode < 4; mode++) {
            for (int rep = 0; rep < 2; rep++) {
                if (mode == 0) hipLaunchKernelGGL(tk<0>, dim3(cus), dim3(64), 0, 0, dc, ds, iters, dup, 0);
                if (mode == 1) hipLaunchKernelGGL(tk<1>, dim3(cus), dim3(64), 0, 0, dc, ds, iters, dup, 0);
                if (mode == 2) hipLaunchKernelGGL(tk<2>, dim3(cus), dim3(64), 0, 0, dc, ds, iters, dup, 0);
                if (mode == 3) hipLaunchKernelGGL(tk<3>, dim3(cus), dim3(64), 0, 0, dc, ds, iters, dup, 0);
                hipDeviceSynchronize();
            }
            hipMemcpy(hc, dc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < cus; i++) s += (double)hc[i];
            /* s_memtime counts at 100 MHz on gfx9 parts: convert to 2.4 GHz shader cycles */
            printf("%-22s dup=%d: %8.1f memtime ticks per window (%.0f shader cycles at 2.4 GHz)\n", nm[mode], dup,
                   s / cus / iters / 15.0, s / cus / iters / 15.0 * 24.0);
        }
    for (int dense = 0; dense < 2; dense++)
    for (int dup = 0; dup < 2; dup++)
        for (int nw = 1; nw <= 4; nw *= 2) {
            for (int rep = 0; rep < 2; rep++) {
                hipLaunchKernelGGL(tk<0>, dim3(cus), dim3(64 * nw), 0, 0, dc, ds, iters, dup, dense);
                hipDeviceSynchronize();
            }
            hipMemcpy(hc, dc, sizeof(unsigned long long) * cus, hipMemcpyDeviceToHost);
            double s = 0;
            for (int i = 0; i < cus; i++) s += (double)hc[i];
            /* per window of the whole step: 15 windows per step whatever nw */
            printf("exchange split over %d waves (%s) dup=%d: %8.1f shader cycles per window of the step\n", nw,
                   dense ? "dense windows dealt per wave" : "by slot, exec-masked", dup, s / cus / iters / 15.0 * 24.0);
        }
    unsigned bad = 0, tot = 0;
    for (int ng = 1; ng <= 64; ng *= 2) {
        hipMemset(db, 0, sizeof(unsigned));
        hipLaunchKernelGGL(ok, dim3(4096), dim3(64), 0, 0, db, ng);
        unsigned b = 0;
        hipMemcpy(&b, db, sizeof(unsigned), hipMemcpyDeviceToHost);
        printf("plain ds_write_b16 order, %2d groups: %u of %u lanes see a non-highest winner\n", ng, b, 4096u * 64u);
        bad += b;
        tot += 4096u * 64u;
    }
    printf("plain store lane order: %s\n", bad ? "VIOLATED" : "held");
    return 0;
}

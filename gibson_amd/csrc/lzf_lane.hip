/*
 * lzf_lane.hip -- the "lane" generation of the LZF kernels for gfx950.
 *
 * Values are independent; the reference's loops over one value are serial
 * (the token decoder src/lzf_d.c:64-146, the greedy parse src/lzf_c.c:145-274).
 * This generation runs ONE LANE PER VALUE for the serial parts, so a wave
 * advances 64 values at once and one VALU instruction does the work of 64
 * scalar steps, instead of spending a whole wave on one value:
 *
 *   decompress  lzf_decompress_lane_kernel: one lane decodes one stream with
 *               the reference's checks in the reference's order; literal runs
 *               and back-references move as unaligned 16-byte pieces.
 *
 *   compress    two kernels per batch (chunked by the scratch size):
 *     1. lzf_cand_small_kernel (values <= 4 KiB, and <= 8 KiB with a 3-bit
 *        identity; lzf_cand_mid_kernel up to 64 KiB, opt-in), one wave per value, position-parallel: for every
 *        position p the nearest earlier position q with the same 16-bit slot
 *        (src/lzf_c.c:47-57, HLOG 16) -- whether or not the parse will insert
 *        q -- and how far the bytes at p and q agree (<= 8).  Packed into a
 *        u16 per position in HBM scratch ("cand").  Same-bucket and same-slot
 *        lanes of a window come from lane bitmaps in LDS; earlier positions
 *        from bucket heads and per-position skip links in LDS.
 *     2. lzf_parse_lane_kernel (one lane per value): the reference's greedy
 *        parse and emission, bit-exact.  The reference's ref at p is the
 *        latest INSERTED position of p's slot (src/lzf_c.c:147-149); every
 *        position the parse visits is inserted, plus the last two positions
 *        of each match (src/lzf_c.c:227-247), so ref(p) is the first
 *        position on the cand chain from p that is not inside an earlier
 *        match.  The lane keeps an inserted-bitmap of its value (the last 32
 *        words in LDS, older words in HBM scratch) and walks the chain only
 *        past skipped positions.  Every wave memory instruction touches one
 *        line per lane, so the kernel is shaped to issue few of them
 *        (DESIGN.md §4.0).
 *     lzf_parse_wave_kernel (opt-in): the same parse as one wave per value,
 *        64 positions per step over LDS-resident data.
 *
 * Scratch per value: 2 B/position (cand) + 1 bit/position (bitmap).
 */
#include <stdlib.h>
#include <string.h>

#include "lzf_internal.h"

/* ---- small helpers ------------------------------------------------------ */

__device__ __forceinline__ uint4 ln_ld16(const uint8_t *p)          /* unaligned */
{
    uint4 v;
    __builtin_memcpy(&v, p, 16);
    return v;
}

__device__ __forceinline__ uint2 ln_ld8(const uint8_t *p)
{
    uint2 v;
    __builtin_memcpy(&v, p, 8);
    return v;
}

__device__ __forceinline__ uint32_t ln_ld4(const uint8_t *p)
{
    uint32_t v;
    __builtin_memcpy(&v, p, 4);
    return v;
}

/* bytes [p, p + avail), avail < 16, zero beyond: never touches p + avail */
__device__ __forceinline__ uint4 ln_ld16_tail(const uint8_t *p, uint32_t avail)
{
    uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16u; k++) {
        const uint32_t b = k < avail ? (uint32_t)p[k] : 0u;
        const uint32_t s = 8u * (k & 3u);
        if (k < 4u) w0 |= b << s;
        else if (k < 8u) w1 |= b << s;
        else if (k < 12u) w2 |= b << s;
        else w3 |= b << s;
    }
    return make_uint4(w0, w1, w2, w3);
}

__device__ __forceinline__ uint4 ln_ld16_safe(const uint8_t *p, uint32_t avail)
{
    return avail >= 16u ? ln_ld16(p) : ln_ld16_tail(p, avail);
}

/* store exactly len (<= 16) bytes of v at p (unaligned) */
__device__ __forceinline__ void ln_st_exact(uint8_t *p, uint4 v, uint32_t len)
{
    if (len >= 16u) {
        __builtin_memcpy(p, &v, 16);
        return;
    }
    uint32_t a = v.x, b = v.y, c = v.z, d = v.w;
    if (len & 8u) {
        uint2 t = make_uint2(a, b);
        __builtin_memcpy(p, &t, 8);
        p += 8;
        a = c;
        b = d;
    }
    if (len & 4u) {
        __builtin_memcpy(p, &a, 4);
        p += 4;
        a = b;
    }
    if (len & 2u) {
        const uint16_t t = (uint16_t)a;
        __builtin_memcpy(p, &t, 2);
        p += 2;
        a >>= 16;
    }
    if (len & 1u) *p = (uint8_t)a;
}

__device__ __forceinline__ uint32_t ln_ab(uint32_t hi, uint32_t lo)    /* (hi:lo) >> 8 */
{
    return __builtin_amdgcn_alignbyte(hi, lo, 1u);
}

__device__ __forceinline__ uint32_t ln_sel4(uint4 v, uint32_t i)
{
    /* selects on the index bits: three v_cndmask, where an i == 0 / 1 / 2
     * chain may become branches around a divergent index */
    const uint32_t a = (i & 1u) ? v.y : v.x, b = (i & 1u) ? v.w : v.z;
    return (i & 2u) ? b : a;
}

__device__ __forceinline__ uint32_t ln_first_diff(uint4 a, uint4 b)   /* 16 if equal */
{
    uint32_t x;
    if ((x = a.x ^ b.x)) return (uint32_t)__builtin_ctz(x) >> 3;
    if ((x = a.y ^ b.y)) return 4u + ((uint32_t)__builtin_ctz(x) >> 3);
    if ((x = a.z ^ b.z)) return 8u + ((uint32_t)__builtin_ctz(x) >> 3);
    if ((x = a.w ^ b.w)) return 12u + ((uint32_t)__builtin_ctz(x) >> 3);
    return 16u;
}

__device__ __forceinline__ void ln_wave_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

/* slot(p) of src/lzf_c.c:47-57 (VERY_FAST, HLOG 16) from b[p..p+2] */
__device__ __forceinline__ uint32_t ln_slot(uint32_t tri)
{
    const uint32_t b0 = tri & 0xFFu, b1 = (tri >> 8) & 0xFFu, b2 = (tri >> 16) & 0xFFu;
    return (((b0 << 8) | b1) - 5u * ((b1 << 8) | b2)) & 0xFFFFu;
}

/* bijective 16-bit mix of the slot: bucket = high bits, identity = low bits */
__device__ __forceinline__ uint32_t ln_mix(uint32_t s) { return (s * 40503u) & 0xFFFFu; }

#ifdef LZF_DIAG   /* cross-check form, diagnostic build only */
/* ======================================================================== */
/* decompress: one lane per stream                                          */
/* ======================================================================== */

#define LD_THREADS 256u

/* Back-reference copy of L bytes from distance `back` (src/lzf_d.c:137-142
 * copies byte-serially, so an overlapping source replicates a period of
 * `back` bytes).  Pieces of up to 16 bytes; while the period is shorter than
 * 16 the copy distance doubles (any multiple of the period is a valid source
 * once that many bytes exist), so a run of 264 takes 5 + 16 pieces. */
__device__ __forceinline__ void ln_copy_back(uint8_t *out, uint32_t o, uint32_t back, uint32_t L,
                                             uint32_t cap)
{
    uint32_t D = back, t = 0;
    do {
        uint32_t c = L - t;
        if (c > 16u) c = 16u;
        if (c > D) c = D;
        const uint32_t s = o + t - D;
        const uint4 v = ln_ld16_safe(out + s, cap - s);
        ln_st_exact(out + o + t, v, c);
        t += c;
        if (D < 16u) D <<= 1;
    } while (t < L);
}

__global__ __launch_bounds__(LD_THREADS) void lzf_decompress_lane_kernel(LzfBatch bt)
{
    const uint32_t v = blockIdx.x * LD_THREADS + threadIdx.x;
    if (v >= bt.count) return;
    if (bt.skip && bt.skip[v]) return;
    const uint32_t in_len = bt.in_len[v];
    const uint32_t cap = bt.out_cap[v];
    const uint8_t *in = bt.in + bt.in_off[v];
    uint8_t *out = bt.out + bt.out_off[v];
    /* as the reference (do-while, src/lzf_d.c:64), a 0-length stream still
     * reads its first control byte */
    const uint32_t avail = in_len ? in_len : 1u;
    uint32_t i = 0, o = 0;
    int32_t err = 0;
    do {
        uint4 w0, w1;
        if (i + 32u <= avail) {
            w0 = ln_ld16(in + i);
            w1 = ln_ld16(in + i + 16u);
        } else {
            w0 = ln_ld16_safe(in + i, avail - i);
            w1 = i + 16u < avail ? ln_ld16_tail(in + i + 16u, avail - i - 16u) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t c = w0.x & 0xFFu;
        if (c < 32u) {                                               /* literal run */
            const uint32_t cnt = c + 1u;
            if ((uint64_t)o + cnt > cap) { err = 7; break; }         /* E2BIG  src/lzf_d.c:72 */
            if ((uint64_t)i + 1u + cnt > in_len) { err = 22; break; }/* EINVAL src/lzf_d.c:79 */
            const uint4 lo = make_uint4(ln_ab(w0.y, w0.x), ln_ab(w0.z, w0.y), ln_ab(w0.w, w0.z),
                                        ln_ab(w1.x, w0.w));
            ln_st_exact(out + o, lo, cnt);
            if (cnt > 16u) {
                const uint32_t b32 = cnt == 32u ? (uint32_t)in[i + 32u] : 0u;
                const uint4 hi = make_uint4(ln_ab(w1.y, w1.x), ln_ab(w1.z, w1.y), ln_ab(w1.w, w1.z),
                                            ln_ab(b32, w1.w));
                ln_st_exact(out + o + 16u, hi, cnt - 16u);
            }
            o += cnt;
            i += 1u + cnt;
        } else {                                                     /* back-reference */
            uint32_t len = c >> 5, ob = (w0.x >> 8) & 0xFFu, tsz = 2u;
            if (i + 1u >= in_len) { err = 22; break; }               /* src/lzf_d.c:101 */
            if (len == 7u) {
                len += ob;
                ob = (w0.x >> 16) & 0xFFu;
                tsz = 3u;
                if (i + 2u >= in_len) { err = 22; break; }           /* src/lzf_d.c:111 */
            }
            const uint32_t back = ((c & 31u) << 8) + 1u + ob;
            if ((uint64_t)o + len + 2u > cap) { err = 7; break; }    /* src/lzf_d.c:121 */
            if (back > o) { err = 22; break; }                       /* src/lzf_d.c:127 */
            ln_copy_back(out, o, back, len + 2u, cap);
            o += len + 2u;
            i += tsz;
        }
    } while (i < in_len);
    bt.out_len[v] = err ? 0u : o;
    bt.err[v] = err;
}

#endif /* LZF_DIAG */

/* Residency cap for the one-lane-per-value kernels: each lane streams its own
 * value, so the lines in use grow with the lanes in flight; past what the
 * XCD's L2 holds every access refetches its line.  Capping the blocks per CU
 * (through the LDS reservation of the launch) trades latency hiding for
 * L2 hits.  0 = no cap. */
static size_t lane_lds_for(const char *env, uint32_t dflt_blocks_per_cu)
{
    const char *e = getenv(env);
    const uint32_t b = e ? (uint32_t)atoi(e) : dflt_blocks_per_cu;
    if (b == 0u) return 0;
    size_t lds = (160u * 1024u) / b;
    if (lds > 64u * 1024u) lds = 64u * 1024u;
    return lds - 256u;
}

#ifdef LZF_DIAG
hipError_t lzf_launch_decompress_lane(const LzfBatch &b, hipStream_t s)
{
    const uint32_t grid = (b.count + LD_THREADS - 1u) / LD_THREADS;
    const size_t lds = lane_lds_for("LZF_LANE_DEC_BLOCKS", 0u);
    if (lds) {
        hipError_t e = hipFuncSetAttribute((const void *)lzf_decompress_lane_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(lzf_decompress_lane_kernel, dim3(grid), dim3(LD_THREADS), lds, s, b);
    return hipGetLastError();
}
#endif /* LZF_DIAG */

/* ======================================================================== */
/* compress, kernel 1: same-slot predecessor of every position              */
/* ======================================================================== */

/* cand word: bits 0-12 off = p - q - 1, bits 13-15 code:
 *   0  no earlier position with p's slot inside the window (or only q = 0,
 *      which is never a ref: src/lzf_c.c:155 `ref > in_data`)
 *   1  q has p's slot but its 3 bytes differ (slot collision)
 *   2..6  bytes agree for exactly code+1 bytes (3..7)
 *   7  bytes agree for >= 8 bytes                                         */
#define CAND_DIFF   1u
#define CAND_LONG   7u

#define K1_WIN      4u            /* windows of 64 positions resolved per step */
#ifndef KS_WIN
#define KS_WIN      4u            /* small class: windows per step (exchange form, json4k compress: 4: 48.6 ms, 3: 49.1, 2: 49.8, 1: 52.2) */
#endif
#ifndef KS8_WIN
#define KS8_WIN     2u            /* 8 KiB small class: windows per step */
#endif
#define KS_MAXN     4096u         /* small class: 12-bit bucket, 4-bit identity, positions + 1 fit 12 bits */
#define KS8_MAXN    8192u         /* small class, 8 KiB: 13-bit bucket, 3-bit identity, positions + 1 fit 13 bits */
#define KM_BUCKETS  2048u         /* mid class */
#define KM_MAXN     65536u        /* positions + 1 fit 16 bits */

__device__ __forceinline__ uint32_t k1_tri(const uint8_t *src, uint32_t n, uint32_t p)
{
    if (p + 4u <= n) return ln_ld4(src + p);
    return (uint32_t)src[p] | ((uint32_t)src[p + 1u] << 8) | ((uint32_t)src[p + 2u] << 16);
}

/* agreement of the bytes at p and q (q < p), at most 8 and at most n - p */
__device__ __forceinline__ uint32_t k1_agree(const uint8_t *src, uint32_t n, uint32_t p, uint32_t q)
{
    const uint32_t avail = n - p;
    uint32_t a0, a1, b0, b1;
    if (avail >= 8u) {
        const uint2 a = ln_ld8(src + p), b = ln_ld8(src + q);
        a0 = a.x; a1 = a.y; b0 = b.x; b1 = b.y;
    } else {
        const uint4 a = ln_ld16_tail(src + p, avail), b = ln_ld16_tail(src + q, avail);
        a0 = a.x; a1 = a.y; b0 = b.x; b1 = b.y;
    }
    uint32_t k;
    if (a0 != b0) k = (uint32_t)__builtin_ctz(a0 ^ b0) >> 3;
    else if (a1 != b1) k = 4u + ((uint32_t)__builtin_ctz(a1 ^ b1) >> 3);
    else k = 8u;
    return k < avail ? k : avail;
}

__device__ __forceinline__ uint32_t k1_code(uint32_t k)
{
    return k < 3u ? CAND_DIFF : (k >= 8u ? CAND_LONG : k - 1u);
}

#ifdef LZF_DIAG   /* used by the mid class only */
/* Lane-order check of the bucket-head atomics: a returned head from a later
 * position means the LDS did not serialise the wave's same-address atomics in
 * lane order; then the predecessors are rebuilt from the keys (the head before
 * the step is the smallest value any lane of the bucket got back). */
template <uint32_t BSHIFT>
__device__ __noinline__ void k1_fix_order(uint32_t (&r)[K1_WIN], const uint32_t (&key)[K1_WIN],
                                          const bool (&act)[K1_WIN])
{
    const uint32_t lane = threadIdx.x;
    uint32_t fixed[K1_WIN];
#pragma unroll
    for (uint32_t j = 0; j < K1_WIN; j++) {
        const uint32_t myb = (key[j] & 0xFFFFu) >> BSHIFT;
        uint32_t mn = 0xFFFFFFFFu, mx = 0u;
        for (uint32_t t = 0; t < 64u * K1_WIN; t++) {
            const uint32_t tj = t >> 6, tl = t & 63u;
            uint32_t kt = 0u, rt = 0u, at = 0u;
#pragma unroll
            for (uint32_t jj = 0; jj < K1_WIN; jj++) {
                const uint32_t kk = (uint32_t)__shfl((int)key[jj], (int)tl);
                const uint32_t rr = (uint32_t)__shfl((int)r[jj], (int)tl);
                const uint32_t aa = (uint32_t)__shfl(act[jj] ? 1 : 0, (int)tl);
                if (jj == tj) { kt = kk; rt = rr; at = aa; }
            }
            if (at && ((kt & 0xFFFFu) >> BSHIFT) == myb) {
                mn = rt < mn ? rt : mn;
                if (t < 64u * j + lane && kt > mx) mx = kt;
            }
        }
        fixed[j] = mn > mx ? mn : mx;
    }
#pragma unroll
    for (uint32_t j = 0; j < K1_WIN; j++)
        if (act[j]) r[j] = fixed[j];
}

#endif /* LZF_DIAG */

/* Small class (every value <= MAXN <= 8 KiB bytes: all positions inside one
 * 8 KiB window, so no window test).  Persistent workgroups of one wave walk the batch; the next
 * value's bytes are loaded into registers while the current one is
 * processed and then staged in LDS, so the position loop reads only LDS.
 *
 * Slot-mix m = mix(slot) (bijective): bucket = m >> IDB, identity = the low
 * IDB bits (IDB = 4 for values <= 4 KiB, 3 for values <= 8 KiB, so that an
 * entry [pos+1 | identity] fits 16 bits).
 * Per position the kernel keeps, in LDS, the bucket head (latest position of
 * the bucket) and a skip link: the latest earlier position of the bucket
 * with ANOTHER identity.  Per window of 64 positions one lane-ordered 16-bit
 * exchange on the heads (ds_mskor_rtn_b32) gives each lane its latest
 * earlier same-bucket position, the head's or an earlier lane's; the
 * same-slot predecessor follows the skip links from there until the
 * identity matches (one hop per change of identity, not per position).
 * Entries are [pos+1:16-IDB | identity:IDB].  LDS at 4 KiB: heads 8 KiB,
 * links 8 KiB, bytes 4 KiB; at 8 KiB: heads 16 KiB, links 16 KiB, bytes
 * 8 KiB. */
__device__ __forceinline__ uint32_t ks_rd4(const uint32_t *w, uint32_t x)
{
    return __builtin_amdgcn_alignbyte(w[(x >> 2) + 1u], w[x >> 2], x & 3u);
}

/* highest set bit of a 64-bit mask (mask != 0) */
__device__ __forceinline__ uint32_t ks_hibit(uint64_t m)
{
    return 63u - (uint32_t)__builtin_clzll(m);
}

/* WIN lane-ordered 16-bit exchanges (ds_mskor_rtn_b32), issued in order, one wait */
template <uint32_t WIN>
__device__ __forceinline__ void ks_xchg(uint32_t (&r)[WIN], const uint32_t (&a)[WIN], const uint32_t (&m)[WIN],
                                        const uint32_t (&d)[WIN])
{
    static_assert(WIN >= 1u && WIN <= 4u, "1..4 windows per step");
    if constexpr (WIN == 1u) {
        asm volatile("ds_mskor_rtn_b32 %0, %1, %2, %3\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r[0]) : "v"(a[0]), "v"(m[0]), "v"(d[0]) : "memory");
    } else if constexpr (WIN == 2u) {
        asm volatile("ds_mskor_rtn_b32 %0, %2, %3, %4\n\tds_mskor_rtn_b32 %1, %5, %6, %7\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r[0]), "=&v"(r[1])
                     : "v"(a[0]), "v"(m[0]), "v"(d[0]), "v"(a[1]), "v"(m[1]), "v"(d[1]) : "memory");
    } else if constexpr (WIN == 3u) {
        asm volatile("ds_mskor_rtn_b32 %0, %3, %4, %5\n\tds_mskor_rtn_b32 %1, %6, %7, %8\n\t"
                     "ds_mskor_rtn_b32 %2, %9, %10, %11\n\ts_waitcnt lgkmcnt(0)"
                     : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2])
                     : "v"(a[0]), "v"(m[0]), "v"(d[0]), "v"(a[1]), "v"(m[1]), "v"(d[1]), "v"(a[2]), "v"(m[2]),
                       "v"(d[2]) : "memory");
    } else {
        asm volatile("ds_mskor_rtn_b32 %0, %4, %5, %6\n\tds_mskor_rtn_b32 %1, %7, %8, %9\n\t"
                     "ds_mskor_rtn_b32 %2, %10, %11, %12\n\tds_mskor_rtn_b32 %3, %13, %14, %15\n\t"
                     "s_waitcnt lgkmcnt(0)"
                     : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3])
                     : "v"(a[0]), "v"(m[0]), "v"(d[0]), "v"(a[1]), "v"(m[1]), "v"(d[1]), "v"(a[2]), "v"(m[2]),
                       "v"(d[2]), "v"(a[3]), "v"(m[3]), "v"(d[3]) : "memory");
    }
}

template <uint32_t IDB, uint32_t MAXN, uint32_t WIN>
__global__ __launch_bounds__(64) void lzf_cand_small_kernel(LzfBatch bt, LzfLaneScratch sc)
{
    static_assert(MAXN <= LZF_WINDOW && ((MAXN - 1u) >> (16u - IDB)) == 0u, "entry [pos+1 | id] must fit 16 bits");
    constexpr uint32_t BUCKETS = 1u << (16u - IDB), IDM = (1u << IDB) - 1u;
    constexpr uint32_t PF = MAXN / 1024u;                /* 16-byte loads per lane per value */
    __shared__ __attribute__((aligned(16))) uint16_t H[BUCKETS + 64u];   /* + one dummy per lane */
    __shared__ uint16_t E[MAXN];
    __shared__ __attribute__((aligned(16))) uint32_t Bw[MAXN / 4u + 4u];
    const uint32_t lane = threadIdx.x;
    uint32_t v = blockIdx.x;
    if (v >= bt.count) return;
    uint4 pf[PF];
    uint32_t pn = bt.in_len[v];
    {
        const uint8_t *s0 = bt.in + bt.in_off[v];
#pragma unroll
        for (uint32_t k = 0; k < PF; k++) {
            const uint32_t at = 16u * (64u * k + lane);
            pf[k] = at < pn ? ln_ld16_safe(s0 + at, pn - at) : make_uint4(0, 0, 0, 0);
        }
    }
    while (v < bt.count) {
        const uint32_t n = pn;
        uint16_t *cand = sc.cand + (uint64_t)v * sc.cstride;
#pragma unroll
        for (uint32_t k = 0; k < PF; k++) ((uint4 *)Bw)[64u * k + lane] = pf[k];
        const uint32_t vn = v + gridDim.x;
        if (vn < bt.count) {                       /* next value's bytes, in flight */
            pn = bt.in_len[vn];
            const uint8_t *s1 = bt.in + bt.in_off[vn];
#pragma unroll
            for (uint32_t k = 0; k < PF; k++) {
                const uint32_t at = 16u * (64u * k + lane);
                pf[k] = at < pn ? ln_ld16_safe(s1 + at, pn - at) : make_uint4(0, 0, 0, 0);
            }
        }
        if (n >= 3u && n <= MAXN) {          /* a longer value: refused by the parse (n > max_len) */
            for (uint32_t k = lane; k < BUCKETS / 8u; k += 64u) ((uint4 *)H)[k] = make_uint4(0, 0, 0, 0);
            ln_wave_fence();
            const uint32_t np = n - 2u;               /* positions 0 .. n-3 */
            for (uint32_t P = 0; P < np; P += 64u * WIN) {
                uint32_t p[WIN], m[WIN], tri[WIN];
                bool act[WIN];
                /* the step's byte reads first, in one LDS round trip */
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    p[j] = P + 64u * j + lane;
                    act[j] = p[j] < np;
                    tri[j] = ks_rd4(Bw, act[j] ? p[j] : 0u);
                }
                /* one lane-ordered 16-bit exchange per window on the bucket's
                 * head (ds_mskor_rtn_b32, tools/lds_mskor_order.hip): each lane
                 * gets the latest earlier position of its bucket -- the
                 * head's or an earlier lane's of the window -- and the
                 * highest lane's key stays.  The skip link of p is that
                 * predecessor when its identity differs, else the
                 * predecessor's own link (an earlier lane's: resolved by
                 * pointer doubling over the window's lanes); the same-slot
                 * predecessor follows the links from it until the identity
                 * matches.  Windows go in order: window j's links are in E
                 * before window j+1 exchanges. */
                uint32_t q1[WIN], cur[WIN];
                bool need = false;
                const uint32_t hb = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)H;
                /* the windows' exchanges in window order, then one wait (the
                 * results are outputs of the same asm statement) */
                uint32_t xa[WIN], xm[WIN], xd[WIN], xr[WIN], xs[WIN];
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    m[j] = ln_mix(ln_slot(tri[j]));
                    const uint32_t h = act[j] ? (m[j] >> IDB) : BUCKETS + lane;
                    xs[j] = (h & 1u) << 4;
                    xa[j] = hb + 4u * (h >> 1);
                    xm[j] = 0xFFFFu << xs[j];
                    xd[j] = ((((p[j] + 1u) << IDB) | (m[j] & IDM)) & 0xFFFFu) << xs[j];
                }
                ks_xchg<WIN>(xr, xa, xm, xd);
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    const uint32_t id = m[j] & IDM;
                    const uint32_t sh = xs[j], rv = xr[j];
                    const uint32_t prev = act[j] ? (rv >> sh) & 0xFFFFu : 0u;
                    const uint32_t ppos = (prev >> IDB) - 1u;            /* prev != 0 */
                    const uint32_t w0 = P + 64u * j;                      /* the window's first position */
                    const bool same = prev && (prev & IDM) == id;
                    /* link entry: resolved (bit 16 | link) or pending (the lane of
                     * an earlier same-slot position of this window) */
                    const uint32_t lprev = same && ppos < w0 ? (uint32_t)E[ppos] : 0u;
                    uint32_t le = !same ? (0x10000u | prev) : ppos >= w0 ? (ppos - w0) : (0x10000u | lprev);
                    /* six doublings resolve any chain inside 64 lanes; the cap bounds
                     * the loop even if the lane order failed (then lzf_selfcheck.hip
                     * has already routed compress batches away from this kernel) */
                    for (uint32_t r_ = 0; r_ < 6u && __ballot(!(le & 0x10000u)); r_++)
                        le = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(((le & 0x10000u) ? lane : le) << 2), (int)le);
                    if (act[j]) E[p[j]] = (uint16_t)le;
                    ln_wave_fence();
                    /* same-slot predecessor: prev if its identity is mine, else
                     * along the links from prev's own link */
                    q1[j] = same ? (prev >> IDB) : 0u;                    /* pos+1 */
                    cur[j] = (prev && !same) ? (uint32_t)E[ppos] : 0u;
                    if (cur[j] && (cur[j] & IDM) == id) { q1[j] = cur[j] >> IDB; cur[j] = 0u; }
                    need |= cur[j] != 0u;
                }
                ln_wave_fence();
                while (__ballot(need)) {
                    need = false;
#pragma unroll
                    for (uint32_t j = 0; j < WIN; j++) {
                        if (cur[j]) {
                            /* links go to earlier positions; anything else ends the walk */
                            const uint32_t e0 = E[(cur[j] >> IDB) - 1u];
                            const uint32_t e = (e0 >> IDB) < (cur[j] >> IDB) ? e0 : 0u;
                            cur[j] = e;
                            if (e && (e & IDM) == (m[j] & IDM)) { q1[j] = e >> IDB; cur[j] = 0u; }
                            need |= cur[j] != 0u;
                        }
                    }
                }
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    if (!act[j]) continue;
                    uint32_t w = 0u;
                    if (q1[j] > 1u) {                    /* q = q1 - 1 > 0 */
                        const uint32_t q = q1[j] - 1u;
                        /* agreement of the bytes at p and q, <= 8, <= n - p:
                         * both dwords read at once (one LDS round trip) */
                        const uint32_t x0 = tri[j] ^ ks_rd4(Bw, q);
                        const uint32_t x1 = ks_rd4(Bw, p[j] + 4u) ^ ks_rd4(Bw, q + 4u);
                        const uint64_t xx = ((uint64_t)x1 << 32) | x0;
                        uint32_t k = xx ? (uint32_t)__builtin_ctzll(xx) >> 3 : 8u;
                        const uint32_t avail = n - p[j];
                        if (k > avail) k = avail;
                        w = (k1_code(k) << 13) | (p[j] - q - 1u);
                    }
                    cand[p[j]] = (uint16_t)w;
                }
            }
        }
        ln_wave_fence();
        v = vn;
    }
}

#ifdef LZF_DIAG   /* ring and mid classes: cross-check forms */
/* Small class, 16 KiB ("ring" form: values <= 16 KiB, so positions reach
 * 8 KiB past the window).  The value's bytes are staged whole as above; the
 * bucket heads are u32 [pos+1 | identity:4] (4096 buckets, 16 KiB) and the
 * skip links are kept only for the last 8192 positions, which is all a
 * candidate inside the window can reach, in a ring of u16 (16 KiB): a link
 * is [d:13 | identity bits 0-2], d = distance back to the target (0: none;
 * a target 8192 or more back is outside every later window).  A target whose
 * three stored identity bits match is confirmed from its bytes (its full slot
 * mix, read in the same LDS round trip as its own link).  A head or
 * link whose position is more than 8192 before p is outside p's window
 * (src/lzf_c.c:153 off < MAX_OFF) and ends the lookup: so is every older one.
 * The links of the step in flight go to S first and join the ring after the
 * step's walks, so that a walk never reads a ring slot the step overwrote.
 * LDS 50.6 KiB: 3 values per CU (u32 links: 66.8 KiB, 2 per CU).
 *
 * Against window64 at 1 M values of 16 KiB (tools/crossover.py): mixed
 * entropy (BASELINE configs[4]) 570 vs 648 ms, Zipf text 437 vs 938 ms,
 * sentence text 473 vs 676 ms.  With u32 links (2 values per CU) it was
 * 702 / 523 / 549 ms. */
#define KR_MAXN 16384u
#define KR64_MAXN 65536u
#ifndef KR_WIN
#define KR_WIN  2u
#endif
template <uint32_t MAXN, uint32_t WIN>
__global__ __launch_bounds__(64) void lzf_cand_ring_kernel(LzfBatch bt, LzfLaneScratch sc)
{
    constexpr uint32_t IDB = 4u, IDM = 15u, BUCKETS = 4096u, RING = LZF_WINDOW;
    constexpr uint32_t T0 = 0u, T1 = 64u, T2 = 128u, TN = 144u;   /* digits as at 4 KiB */
    /* values past 16 KiB stream their bytes through a 16 KiB LDS ring in 1 KiB
     * chunks, one chunk in flight in registers: a step reads positions from
     * P - 8192 (the window) to P + 64*WIN + 12, and a chunk is stored only
     * once P + 64*WIN + 16 passes the bytes staged, so it never overwrites a
     * byte the window still reaches */
    constexpr bool STREAM = MAXN > KR_MAXN;
    constexpr uint32_t RB = 16384u, WM = RB / 4u - 1u;
    constexpr uint32_t PF = STREAM ? 1u : MAXN / 1024u;
    __shared__ __attribute__((aligned(16))) uint32_t H[BUCKETS];
    __shared__ uint16_t E[RING];
    __shared__ uint16_t S[64u * WIN];
    __shared__ __attribute__((aligned(16))) uint32_t Bw[STREAM ? RB / 4u : MAXN / 4u + 4u];
    __shared__ unsigned long long T[WIN][TN];
    const auto rd4 = [&](uint32_t x) -> uint32_t {
        if constexpr (STREAM) {
            const uint32_t w = x >> 2;
            return __builtin_amdgcn_alignbyte(Bw[(w + 1u) & WM], Bw[w & WM], x & 3u);
        } else {
            return ks_rd4(Bw, x);
        }
    };
    const uint32_t lane = threadIdx.x;
    const unsigned long long mine = 1ull << lane, below = mine - 1ull;
    uint32_t v = blockIdx.x;
    if (v >= bt.count) return;
    for (uint32_t k = lane; k < WIN * TN; k += 64u) (&T[0][0])[k] = 0ull;
    uint4 pf[PF];
    uint32_t pn = bt.in_len[v];
    if (!STREAM) {
        const uint8_t *s0 = bt.in + bt.in_off[v];
#pragma unroll
        for (uint32_t k = 0; k < PF; k++) {
            const uint32_t at = 16u * (64u * k + lane);
            pf[k] = at < pn ? ln_ld16_safe(s0 + at, pn - at) : make_uint4(0, 0, 0, 0);
        }
    }
    while (v < bt.count) {
        const uint32_t n = pn;
        uint16_t *cand = sc.cand + (uint64_t)v * sc.cstride;
        const uint8_t *src = bt.in + bt.in_off[v];
        uint32_t L = 0u;                           /* STREAM: bytes staged in the ring */
        if (!STREAM) {
#pragma unroll
            for (uint32_t k = 0; k < PF; k++) ((uint4 *)Bw)[64u * k + lane] = pf[k];
        } else {                                   /* the first chunk */
            pf[0] = 16u * lane < n ? ln_ld16_safe(src + 16u * lane, n - 16u * lane) : make_uint4(0, 0, 0, 0);
        }
        const uint32_t vn = v + gridDim.x;
        if (vn < bt.count) pn = bt.in_len[vn];
        if (!STREAM && vn < bt.count) {            /* next value's bytes, in flight */
            pn = bt.in_len[vn];
            const uint8_t *s1 = bt.in + bt.in_off[vn];
#pragma unroll
            for (uint32_t k = 0; k < PF; k++) {
                const uint32_t at = 16u * (64u * k + lane);
                pf[k] = at < pn ? ln_ld16_safe(s1 + at, pn - at) : make_uint4(0, 0, 0, 0);
            }
        }
        if (n >= 3u) {
            for (uint32_t k = lane; k < BUCKETS / 4u; k += 64u) ((uint4 *)H)[k] = make_uint4(0, 0, 0, 0);
            ln_wave_fence();
            const uint32_t np = n - 2u;               /* positions 0 .. n-3 */
            for (uint32_t P = 0; P < np; P += 64u * WIN) {
                if (STREAM && L < n && L < P + 64u * WIN + 16u) {
                    ((uint4 *)Bw)[((L >> 4) + lane) & (RB / 16u - 1u)] = pf[0];
                    L += 1024u;
                    const uint32_t at = L + 16u * lane;
                    pf[0] = at < n ? ln_ld16_safe(src + at, n - at) : make_uint4(0, 0, 0, 0);
                    ln_wave_fence();
                }
                uint32_t p[WIN], m[WIN], tri[WIN];
                bool act[WIN];
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    p[j] = P + 64u * j + lane;
                    act[j] = p[j] < np;
                    tri[j] = rd4(act[j] ? p[j] : 0u);
                }
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    m[j] = ln_mix(ln_slot(tri[j]));
                    if (act[j]) {
                        __hip_atomic_fetch_or(&T[j][T0 + ((m[j] >> IDB) & 63u)], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_or(&T[j][T1 + (m[j] >> (IDB + 6u))], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        __hip_atomic_fetch_or(&T[j][T2 + (m[j] & IDM)], mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
                ln_wave_fence();
                unsigned long long MB[WIN], MS[WIN];
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    MB[j] = T[j][T0 + ((m[j] >> IDB) & 63u)] & T[j][T1 + (m[j] >> (IDB + 6u))];
                    MS[j] = MB[j] & T[j][T2 + (m[j] & IDM)];
                    if (!act[j]) MB[j] = MS[j] = 0ull;
                }
                ln_wave_fence();
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    if (act[j]) {
                        T[j][T0 + ((m[j] >> IDB) & 63u)] = 0ull;
                        T[j][T1 + (m[j] >> (IDB + 6u))] = 0ull;
                        T[j][T2 + (m[j] & IDM)] = 0ull;
                    }
                }
                /* a head x = [y+1 | id] is inside p's window iff y + 8192 >= p;
                 * the link of position y is in S while y belongs to this step */
#define KR_INW(x_, p_) ((x_) != 0u && ((x_) >> IDB) + (RING - 1u) >= (p_))
#define KR_LINK(y_) ((uint32_t)((y_) >= P ? S[(y_) - P] : E[(y_) & (RING - 1u)]))
                uint32_t q1[WIN], cp[WIN], ci[WIN];   /* candidate: pos+1 (0: none), id bits 0-2 */
                bool need = false;
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    const uint32_t bk = m[j] >> IDB, id = m[j] & IDM;
                    const uint32_t key = ((p[j] + 1u) << IDB) | id;
                    const unsigned long long ss = MS[j] & below, sb = MB[j] & ~MS[j] & below;
                    const uint32_t h0 = act[j] ? H[bk] : 0u;
                    const uint32_t h = KR_INW(h0, p[j]) ? h0 : 0u;
                    /* the head's link: target pos+1 (0: none or out of window), id bits */
                    uint32_t ey = 0u, ei = 0u;
                    if (h) {
                        const uint32_t e = KR_LINK((h >> IDB) - 1u);
                        ey = e ? (h >> IDB) - (e >> 3) : 0u;
                        if (ey + (RING - 1u) < p[j]) ey = 0u;
                        ei = e & 7u;
                    }
                    /* skip link: latest earlier bucket position with another identity */
                    const uint32_t lsb = sb ? ks_hibit(sb) : lane;
                    const uint32_t ksb = (uint32_t)__shfl((int)key, (int)lsb);
                    uint32_t ty, ti;                                  /* link target pos+1, id bits */
                    if (sb) { ty = ksb >> IDB; ti = ksb & 7u; }
                    else if (h && (h & IDM) != id) { ty = h >> IDB; ti = h & 7u; }
                    else { ty = ey; ti = ei; }
                    const uint32_t d = p[j] + 1u - ty;                /* >= 1 when ty != 0 */
                    if (act[j]) S[p[j] - P] = (uint16_t)((ty && d < RING) ? ((d << 3) | ti) : 0u);
                    if (act[j] && (MB[j] >> lane) == 1ull) H[bk] = key;
                    /* same-slot predecessor (pos+1), inside the window */
                    q1[j] = ss ? P + 64u * j + ks_hibit(ss) + 1u : 0u;
                    cp[j] = 0u;
                    ci[j] = ei;
                    if (act[j] && !ss && h) {
                        if ((h & IDM) == id) q1[j] = h >> IDB;
                        else cp[j] = ey;                              /* walk from the head's link */
                    }
                    need |= cp[j] != 0u;
                }
                ln_wave_fence();
                /* per hop: the candidate's link and bytes in one LDS round trip;
                 * it is the same-slot predecessor iff its slot mix equals mine */
                while (__ballot(need)) {
                    need = false;
#pragma unroll
                    for (uint32_t j = 0; j < WIN; j++) {
                        if (cp[j]) {
                            const uint32_t y = cp[j] - 1u;
                            const uint32_t e = KR_LINK(y);
                            const uint32_t ty = rd4(y);
                            if (ci[j] == (m[j] & 7u) && ln_mix(ln_slot(ty)) == m[j]) {
                                q1[j] = cp[j];
                                cp[j] = 0u;
                            } else {
                                uint32_t ny = e ? cp[j] - (e >> 3) : 0u;
                                if (ny + (RING - 1u) < p[j]) ny = 0u;
                                cp[j] = ny;
                                ci[j] = e & 7u;
                                need |= ny != 0u;
                            }
                        }
                    }
                }
#undef KR_INW
#undef KR_LINK
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++) {
                    if (!act[j]) continue;
                    uint32_t w = 0u;
                    if (q1[j] > 1u) {                    /* q = q1 - 1 > 0, p - q - 1 < 8192 */
                        const uint32_t q = q1[j] - 1u;
                        const uint32_t x0 = tri[j] ^ rd4(q);
                        const uint32_t x1 = rd4(p[j] + 4u) ^ rd4(q + 4u);
                        const uint64_t xx = ((uint64_t)x1 << 32) | x0;
                        uint32_t k = xx ? (uint32_t)__builtin_ctzll(xx) >> 3 : 8u;
                        const uint32_t avail = n - p[j];
                        if (k > avail) k = avail;
                        w = (k1_code(k) << 13) | (p[j] - q - 1u);
                    }
                    cand[p[j]] = (uint16_t)w;
                }
                /* the step's links join the ring (every walk of the step is done) */
#pragma unroll
                for (uint32_t j = 0; j < WIN; j++)
                    if (act[j]) E[p[j] & (RING - 1u)] = S[64u * j + lane];
                ln_wave_fence();
            }
        }
        ln_wave_fence();
        v = vn;
    }
}

/* Mid class (values <= 64 KiB).  LDS: bucket heads [pos+1:16 | mix:16]
 * (8 KiB), a ring of the head each position displaced (its bucket
 * predecessor's key) over the last 8192 positions (32 KiB), and the keys of
 * the step in flight, which join the ring only after the step's walks. */
__global__ __launch_bounds__(64) void lzf_cand_mid_kernel(LzfBatch bt, LzfLaneScratch sc)
{
    __shared__ __attribute__((aligned(16))) uint32_t H[KM_BUCKETS];
    __shared__ uint32_t R[LZF_WINDOW];
    __shared__ uint32_t S[64u * K1_WIN];
    const uint32_t lane = threadIdx.x, v = blockIdx.x;
    const uint32_t n = bt.in_len[v];
    const uint8_t *src = bt.in + bt.in_off[v];
    uint16_t *cand = sc.cand + (uint64_t)v * sc.cstride;
    if (n < 3u) return;
    for (uint32_t k = lane; k < KM_BUCKETS / 4u; k += 64u) ((uint4 *)H)[k] = make_uint4(0, 0, 0, 0);
    ln_wave_fence();
    const uint32_t np = n - 2u;
    for (uint32_t P = 0; P < np; P += 64u * K1_WIN) {
        uint32_t p[K1_WIN], m[K1_WIN], key[K1_WIN], r[K1_WIN];
        bool act[K1_WIN];
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++) {
            p[j] = P + 64u * j + lane;
            act[j] = p[j] < np;
            m[j] = act[j] ? ln_mix(ln_slot(k1_tri(src, n, p[j]))) : 0u;
            key[j] = ((p[j] + 1u) << 16) | m[j];
        }
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++)
            r[j] = act[j] ? atomicMax(&H[m[j] >> 5], key[j]) : 0u;
        bool bad = sc.force_fix != 0u;
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++) bad |= act[j] && (r[j] >> 16) > p[j];
        if (__ballot(bad)) k1_fix_order<5>(r, key, act);
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++) S[64u * j + lane] = r[j];
        ln_wave_fence();
        uint32_t cur[K1_WIN];
        bool fd[K1_WIN], need = false;
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++) {
            cur[j] = r[j];
            /* an entry is usable while inside the window: p - q - 1 < 8192 */
            if (cur[j] && p[j] - (cur[j] >> 16) >= LZF_WINDOW) cur[j] = 0u;
            fd[j] = cur[j] != 0u && (cur[j] & 0xFFFFu) == m[j];
            need |= act[j] && !fd[j] && cur[j] != 0u;
        }
        while (__ballot(need)) {
            need = false;
#pragma unroll
            for (uint32_t j = 0; j < K1_WIN; j++) {
                if (act[j] && !fd[j] && cur[j] != 0u) {
                    const uint32_t x = (cur[j] >> 16) - 1u;
                    uint32_t e = x >= P ? S[x - P] : R[x & (LZF_WINDOW - 1u)];
                    if (e && p[j] - (e >> 16) >= LZF_WINDOW) e = 0u;
                    cur[j] = e;
                    fd[j] = e != 0u && (e & 0xFFFFu) == m[j];
                    need |= !fd[j] && e != 0u;
                }
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++) {
            if (!act[j]) continue;
            uint32_t w = 0u;
            if (fd[j] && (cur[j] >> 16) > 1u) {
                const uint32_t q = (cur[j] >> 16) - 1u;
                w = (k1_code(k1_agree(src, n, p[j], q)) << 13) | (p[j] - q - 1u);
            }
            cand[p[j]] = (uint16_t)w;
        }
        ln_wave_fence();
#pragma unroll
        for (uint32_t j = 0; j < K1_WIN; j++)
            if (act[j]) R[p[j] & (LZF_WINDOW - 1u)] = r[j];
        ln_wave_fence();
    }
}

#endif /* LZF_DIAG */

/* ======================================================================== */
/* compress, kernel 2: the greedy parse and emission, one lane per value    */
/* ======================================================================== */

#ifndef K2_THREADS
#define K2_THREADS 256u
#endif
#ifndef K2_CB
#define K2_CB      32u          /* cand words per parse block: 8, 16 or 32 (16 B each 8) */
#endif
#ifndef K2_RW
#define K2_RW      32u          /* bitmap words kept in LDS per lane (power of two) */
#endif

/* Diagnostic build only (-DK2_COUNT_SITES): per-site event counts of the
 * parse kernel's global memory accesses, summed over all lanes. */
#if defined(K2_COUNT_SITES) || defined(KW_PHASES) || defined(K2_WAVE_SITES)
__device__ unsigned long long k2_sites[16];
extern "C" int lzf_gpu_debug_sites(unsigned long long *out16, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(k2_sites), sizeof(k2_sites));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(k2_sites), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : -2;
}
#endif
#ifdef K2_COUNT_SITES
#define K2_SITE(i) atomicAdd(&k2_sites[i], 1ull)
#else
#define K2_SITE(i) ((void)0)
#endif
/* -DK2_WAVE_SITES: how often the WAVE runs each section of the lane parse
 * (once per wave pass, whatever its active lanes), in k2_sites[0..15] */
#ifdef K2_WAVE_SITES
#define K2_WS(i)                                                                   \
    do {                                                                           \
        const uint64_t b_ = __ballot(1);                                           \
        if ((b_ & (~b_ + 1ull)) == (1ull << (threadIdx.x & 63u))) wsc_[i]++;       \
    } while (0)
#else
#define K2_WS(i) ((void)0)
#endif
/* -DKW_PHASES: cycles per phase of the wave-form parse, summed in k2_sites[0..7] */
#ifdef KW_PHASES
#define KW_PH(i) do { const uint64_t t_ = clock64(); ph_[i] += t_ - ph_t; ph_t = t_; } while (0)
#else
#define KW_PH(i) ((void)0)
#endif

/* m = min(first mismatch >= start, lim), bytes [0, start) known equal
 * (src/lzf_c.c:169-209; lim carries the 16-compare quirk) */

/* The lanes of a wave are at different points of their values, so the loop
 * is a state machine in which every lane does at most ONE unit of each kind
 * of work per iteration -- take the cand word of p, test one candidate for
 * insertion (or hop one link back), compare one 16-byte piece of a long
 * match, emit one literal or one back-reference -- and a long walk or match
 * of one lane costs the others only the small blocks it runs through. */
#ifndef K2_NRES
#define K2_NRES 1u
#endif
/* one trip taken when 6 lanes gain from it: with the persistent lanes, 2 trips
 * / 8 lanes cost json4k, mixed16k and text8k 1.6-2.7 % (profiles/r06/v) */
#ifndef K2_LITMIN
#define K2_LITMIN   6u       /* lanes of the wave that must take a free-literal trip for it to run */
#endif
#ifndef K2_LITX
#define K2_LITX 1u       /* free-literal trips after a literal in the same iteration (0: none) */
#endif
#ifndef K2_LITB
#define K2_LITB 1        /* a trip takes up to 4 free literals (0: one) */
#endif
enum { K2_STEP = 0, K2_RESOLVE = 1, K2_DECIDE = 2, K2_EXTEND = 3, K2_EMIT = 4, K2_DONE = 5 };

/* rel of p to the next link r of the chain from its rel to q and q's cand
 * code for r.  3-byte agreements combine (both agree => p~r agree, exactly one
 * => they differ); K2_EXACT: exact agreements too -- p~q exactly a bytes and
 * q~r exactly b != a give p~r exactly min(a, b), one exact and one >= 8 give
 * the exact one, both >= 8 give >= 8 (cand words are capped at their own
 * remaining bytes, more than p's, so the rule holds at the value's end; the
 * same rule as lzf_cand.hip's k3_comb) */
/* off by default: same-process A/B, output identical (profiles/r05/cand/ab_k2x*):
 * json4k 47.21 -> 47.49 ms, mixed16k 50.56 -> 50.96, text8k 48.03 -> 47.77 --
 * lane generation's chains are short and its agreement probes are LDS-cheap */
#ifndef K2_EXACT
#define K2_EXACT 0
#endif
__device__ __forceinline__ uint32_t k2_comb(uint32_t rel, uint32_t code)
{
    if (rel == 9u) return 9u;
    const bool e1 = rel >= 2u, e2 = code >= 2u;
    if (!(e1 && e2)) return (e1 != e2) ? CAND_DIFF : 9u;
    if (K2_EXACT && rel <= CAND_LONG) {
        if (rel != code) return rel < code ? rel : code;
        if (rel == CAND_LONG) return CAND_LONG;
    }
    return 8u;
}

__global__ __launch_bounds__(K2_THREADS) void lzf_parse_lane_kernel(LzfBatch bt, LzfLaneScratch sc)
{
    /* Persistent lanes: as many blocks as stay resident, lane l parsing
     * values l, l + G, l + 2G, ... (G lanes in the grid), so a wave stays
     * full while values remain: a wave's pass costs its instructions whatever
     * its active lanes, and one value's chain can be ~2x another's (mixed
     * data: 6.1 k wave passes for 3.4 k per value, profiles/r06/o).  A queue
     * handing out values as lanes finish balanced mixed data ~3 % better and
     * cost text and json 5-7 %: a load waits behind its lane's atomic
     * (profiles/r06/p-r). */
    uint32_t v = blockIdx.x * K2_THREADS + threadIdx.x;
    uint32_t n = 0u, cap = 0u;
    const uint8_t *src = nullptr;
    uint8_t *dst = nullptr;
    const uint16_t *cand = nullptr;
    uint32_t *bits = nullptr;

    /* output: aligned dwords at da; acc holds the bytes from dword fw on */
    uint32_t dm = 0u;
    uint8_t *da = nullptr;
    uint64_t acc = 0;
    uint32_t accn = 0u, fw = 0;
    uint32_t hx = 0u;                   /* header byte of the open run (index from da) */
    /* completed dwords [fs, fw) wait in pb0..2 and go out as one 16-byte
     * store: every store instruction of the wave touches 64 lines (one
     * per lane's value), so fewer, wider stores */
    uint32_t pb0 = 0u, pb1 = 0u, pb2 = 0u, fs = 0u;
    /* input: the 16 bytes from position wb; loaded at the first byte that
     * falls outside it (a literal, or a match extension's own piece) */
    uint32_t wb = 0xFFFFFFF0u;          /* none yet */
    uint4 W = make_uint4(0, 0, 0, 0);

    uint32_t o = 1u, run = 0u, p = 0u; /* o, run: the reference's op and lit */
    /* cand words [cb, cb+32): one 64-byte, line-aligned block.  A wave load
     * costs one line fetch per lane; the four loads of a block share it */
    uint32_t cb = 0xFFFFFFE0u;         /* none yet (p - cb >= 32 for every p) */
    uint4 C0 = W, C1 = W, C2 = W, C3 = W;
    uint32_t cw = 0u, curw = 0u;       /* inserted-bitmap word of p, in flight */
    /* the last K2_RW bitmap words of the value in LDS (word w at slot w % K2_RW,
     * lane-interleaved: conflict-free), older words in the scratch array;
     * only words [fl, cw) of the current value are ever read from it */
    __shared__ uint32_t k2_ring[K2_RW][K2_THREADS];
    uint32_t *const ring = &k2_ring[0][threadIdx.x];
#define K2_RING(w_) ring[((w_) & (K2_RW - 1u)) * K2_THREADS]
    /* words [0, fl) are in the scratch array: a word goes there, four at a
     * time in one 16-byte store, before its ring slot is reused */
    uint32_t fl = 0u;
#define K2_FLUSH_TO(w_)                                                            \
    do {                                                                           \
        while (fl + K2_RW <= (w_)) {                                               \
            *(uint4 *)(bits + fl) = make_uint4(K2_RING(fl), K2_RING(fl + 1u),      \
                                               K2_RING(fl + 2u), K2_RING(fl + 3u)); \
            fl += 4u;                                                              \
        }                                                                          \
    } while (0)
    uint32_t ms = 0u, me = 0u;         /* the last match: [ms, me) */
    uint32_t rel = 0u, q = 0u, k = 0u, lim = 0u, m = 0u;
    bool ok = true, live = false;
    uint32_t mode = K2_DONE;
    [[maybe_unused]] uint32_t fm = 0u, fmb = 0xFFFFFFE0u;   /* K2_LITB: candidate mask of block fmb */
    /* the lane's next value */
#define K2_NEXT() (v + gridDim.x * K2_THREADS)
    /* The value after this one: its lengths and offsets are loaded when the
     * parse of v passes 31/32 of it, so a lane that finishes rarely waits */
    uint32_t nv = v, nn = 0u, ncap = 0u, rsv = 2u, tr2 = 0u;
    uint64_t nio = 0u, noo = 0u;
#define K2_LOAD_AHEAD()                                                            \
    do {                                                                           \
        if (nv < bt.count) {                                                       \
            nn = bt.in_len[nv];                                                    \
            ncap = bt.out_cap[nv];                                                 \
            nio = bt.in_off[nv];                                                   \
            noo = bt.out_off[nv];                                                  \
        }                                                                          \
        rsv = 2u;                                                                  \
    } while (0)
    /* take the value ahead, or the first after it that the parse does not
     * refuse (src/lzf_c.c:131; past the stated max_len, the scratch stride),
     * with its state fresh; none left: the lane idles */
#define K2_START()                                                                 \
    do {                                                                           \
        live = false;                                                              \
        for (;;) {                                                                 \
            if (rsv != 2u) K2_LOAD_AHEAD();                                        \
            if (nv >= bt.count) break;                                             \
            v = nv;                                                                \
            n = nn;                                                                \
            cap = ncap;                                                            \
            src = bt.in + nio;                                                     \
            dst = bt.out + noo;                                                    \
            nv = K2_NEXT();                                                        \
            rsv = 0u;                                                              \
            if (n != 0u && cap != 0u && n <= bt.max_len) {                         \
                live = true;                                                       \
                break;                                                             \
            }                                                                      \
            bt.out_len[v] = 0u;                                                    \
        }                                                                          \
        if (live) {                                                                \
            cand = sc.cand + (uint64_t)v * sc.cstride;                             \
            bits = sc.bits + (uint64_t)v * sc.bstride;                             \
            dm = (uint32_t)((uintptr_t)dst & 3u);                                  \
            da = dst - dm;                                                         \
            acc = 0;                                                               \
            accn = dm;                                                             \
            fw = 0u;                                                               \
            hx = dm;                                                               \
            pb0 = pb1 = pb2 = fs = 0u;                                             \
            wb = 0xFFFFFFF0u;                                                      \
            o = 1u;                                                                \
            run = p = 0u;                                                          \
            cb = 0xFFFFFFE0u;                                                      \
            cw = curw = fl = 0u;                                                   \
            ms = me = 0u;                                                          \
            ok = true;                                                             \
            fmb = 0xFFFFFFE0u;                                                     \
            tr2 = n - (n >> 5);                                                    \
            mode = n >= 3u ? K2_STEP : K2_DONE;                                    \
        } else {                                                                   \
            mode = K2_DONE;                                                        \
        }                                                                          \
    } while (0)
#ifdef K2_WAVE_SITES
    uint32_t wsc_[16] = {0u};
#endif

/* completed dwords [fs, fw) wait in pb0..2 (slot fw - fs) and leave with
 * the fourth as one 16-byte store; slot and patch selects instead of
 * branches (lzf_cand.hip's parse has the same cursor) */
#define K2_STORE16(w_)                                                             \
    do {                                                                           \
        if (fs == 0u && dm != 0u) {        /* dst's first dword: bytes before dst are not ours */ \
            for (uint32_t t_ = dm; t_ < 4u; t_++) da[t_] = (uint8_t)(pb0 >> (8u * t_)); \
            const uint2 m_ = make_uint2(pb1, pb2);                                 \
            __builtin_memcpy(da + 4u, &m_, 8);                                     \
            const uint32_t l_ = (w_);                                              \
            __builtin_memcpy(da + 12u, &l_, 4);                                    \
        } else {                                                                   \
            const uint4 v_ = make_uint4(pb0, pb1, pb2, (w_));                      \
            __builtin_memcpy(da + 4u * fs, &v_, 16);                               \
        }                                                                          \
        K2_SITE(8);                                                                \
    } while (0)
#define K2_PUT(bytes_, cnt_)                                                       \
    do {                                                                           \
        acc |= (uint64_t)(bytes_) << (8u * accn);                                  \
        accn += (cnt_);                                                            \
        if (accn >= 4u) {                                                          \
            const uint32_t w_ = (uint32_t)acc, np_ = fw - fs;                      \
            pb0 = np_ == 0u ? w_ : pb0;                                            \
            pb1 = np_ == 1u ? w_ : pb1;                                            \
            pb2 = np_ == 2u ? w_ : pb2;                                            \
            if (np_ == 3u) {                                                       \
                K2_STORE16(w_);                                                    \
                fs = fw + 1u;                                                      \
            }                                                                      \
            fw++;                                                                  \
            acc >>= 32;                                                            \
            accn -= 4u;                                                            \
        }                                                                          \
    } while (0)
#define K2_PATCH(x_, byte_)                                                        \
    do {                                                                           \
        if ((x_) >= 4u * fw) {                                                     \
            const uint32_t sh_ = 8u * ((x_) - 4u * fw);                            \
            acc = (acc & ~(0xFFull << sh_)) | ((uint64_t)(byte_) << sh_);          \
        } else if ((x_) >= 4u * fs) {                                              \
            const uint32_t i_ = ((x_) >> 2) - fs, sh_ = 8u * ((x_) & 3u);          \
            const uint32_t mk_ = ~(0xFFu << sh_), b_ = (uint32_t)(byte_) << sh_;  \
            pb0 = i_ == 0u ? (pb0 & mk_) | b_ : pb0;                               \
            pb1 = i_ == 1u ? (pb1 & mk_) | b_ : pb1;                               \
            pb2 = i_ == 2u ? (pb2 & mk_) | b_ : pb2;                               \
        } else {                                                                   \
            da[(x_)] = (uint8_t)(byte_);                                           \
        }                                                                          \
    } while (0)
#define K2_BYTE(pos_, out_)                                                        \
    do {                                                                           \
        uint32_t d_ = (pos_) - wb;                                                 \
        if (d_ >= 16u) {                                                           \
            K2_SITE(6);                                                            \
            W = ln_ld16_safe(src + (pos_), n - (pos_));                            \
            wb = (pos_);                                                           \
            d_ = 0u;                                                               \
        }                                                                          \
        (out_) = (ln_sel4(W, d_ >> 2) >> (8u * (d_ & 3u))) & 0xFFu;               \
    } while (0)
#define K2_LITERAL(pos_)                                                           \
    do {                                                                           \
        uint32_t byte_;                                                            \
        K2_BYTE(pos_, byte_);                                                      \
        const bool first_ = run == 0u;             /* the run's header slot first */ \
        hx = first_ ? 4u * fw + accn : hx;                                         \
        K2_PUT(first_ ? byte_ << 8 : byte_, first_ ? 2u : 1u);                     \
        o++;                                                                       \
        if (++run == LZF_MAX_LIT) { K2_PATCH(hx, LZF_MAX_LIT - 1u); run = 0u; o++; } \
    } while (0)

    K2_LOAD_AHEAD();                   /* nv = v: the lane's first value */
    K2_START();
    while (__ballot(live)) {
        if (mode != K2_DONE) K2_SITE(0);
        K2_WS(0);
        /* the next value's lengths and offsets */
        if (live && rsv != 2u && p >= tr2) K2_LOAD_AHEAD();
        /* ---- the cand word of p ------------------------------------------ */
        if (mode == K2_STEP) {                                            /* src/lzf_c.c:145 */
            if (p >= n - 2u) {
                mode = K2_DONE;
            } else {
                uint32_t d = p - cb;
                K2_SITE(10);
                K2_WS(1);
                if (d >= K2_CB) {
                    K2_SITE(1);
                    K2_WS(2);
                    cb = p & ~(K2_CB - 1u);
                    d = p - cb;
                    const uint4 *cp = (const uint4 *)(cand + cb);
                    C0 = cp[0];
                    if (K2_CB >= 16u) C1 = cp[1];
                    if (K2_CB >= 32u) {
                        C2 = cp[2];
                        C3 = cp[3];
                    }
                }
                const uint32_t dw = d >> 1;
                const uint4 Cq = dw < 8u ? (dw < 4u ? C0 : C1) : (dw < 12u ? C2 : C3);
                const uint32_t c = (ln_sel4(Cq, dw & 3u) >> (16u * (d & 1u))) & 0xFFFFu;
                /* rel: 0 no ref; 1 ref with other bytes; 2..6 equal for rel+1
                 * bytes; 7 equal >= 8; 8 equal 3 bytes, length unknown; 9 unknown */
                rel = c >> 13;
                q = p - 1u - (c & 0x1FFFu);
                mode = rel ? K2_RESOLVE : K2_DECIDE;
            }
        }
        /* ---- is the candidate inserted? else one link back: up to K2_NRES
         * tests per iteration ---------------------------------------------- */
#pragma unroll
        for (uint32_t rt_ = 0; rt_ < K2_NRES; rt_++) {
            if (mode == K2_RESOLVE) {
                K2_WS(3);
                uint32_t word;
                if (q >= ms) {
                    word = (q > ms && q + 3u <= me) ? 0u : 0xFFFFFFFFu;         /* last match's interior */
                } else {
                    const uint32_t d = cw - (q >> 5);
                    if (d != 0u && (q >> 5) < fl) K2_SITE(3);
                    word = d == 0u ? curw : (q >> 5) >= fl ? K2_RING(q >> 5) : bits[q >> 5];
                }
                if ((word >> (q & 31u)) & 1u) {                              /* q is the ref */
                    if (rel == 9u) K2_SITE(5);
                    if (rel == 9u) {
                        /* one 4-byte load per side (q + 3 <= p + 2 < n, p >= 1):
                         * one memory wait instead of up to three */
                        const uint32_t x_ = ln_ld4(src + q) ^ (ln_ld4(src + p - 1u) >> 8);
                        rel = (x_ & 0xFFFFFFu) == 0u ? 8u : 1u;
                    }
                    mode = K2_DECIDE;
                } else {
                    K2_SITE(4);
                    const uint32_t c2 = cand[q];
                    const uint32_t r2 = c2 >> 13;
                    const uint32_t q2 = q - 1u - (c2 & 0x1FFFu);
                    if (!r2 || p - q2 - 1u >= LZF_WINDOW) {
                        rel = 0u;
                        mode = K2_DECIDE;
                    } else {
                        rel = k2_comb(rel, r2);
                        q = q2;
                    }
                }
            }
        }
        /* ---- literal, or the start of a back-reference ------------------- */
        if (mode == K2_DECIDE) {
            K2_WS(4);
            curw |= 1u << (p & 31u);                                     /* p is inserted */
            if (!(rel >= 2u && p + 4u < n)) {                            /* src/lzf_c.c:151-166 */
                K2_WS(5);
                if (o >= cap) {                                          /* src/lzf_c.c:263 */
                    ok = false;
                    mode = K2_DONE;
                } else {
                    K2_LITERAL(p);
                    p++;
                    if ((p & 31u) == 0u) {
                        K2_FLUSH_TO(cw);
                        K2_RING(cw) = curw;
                        cw++;
                        curw = 0u;
                    }
                    mode = K2_STEP;
#if K2_LITX
                    /* free literals: while the next positions have no
                     * candidate at all (cand code 0: no earlier position with
                     * their slot in the window, so no inserted one either,
                     * src/lzf_c.c:153-158), and their cand word and byte are
                     * already in registers, they are literals with no memory
                     * access -- up to K2_LITX more per iteration */
                    /* only when enough lanes of the wave are at a literal at
                     * all (one ballot of the branch's lanes): on text, where
                     * few are, the wave skips the path */
                    bool go = true;
#if K2_LITB
                    /* K2_LITB: up to 4 free literals per trip.  fm: bit j set
                     * when cand word cb + j has a candidate (code != 0), made
                     * once per block on the path's first use of it */
                    if ((uint32_t)__builtin_popcountll(__ballot(true)) >= K2_LITMIN) {
                        K2_WS(6);
                        if (fmb != cb) {
                            K2_WS(7);
                            fm = 0u;
#pragma unroll
                            for (uint32_t k_ = 0; k_ < 8u; k_++) {
                                const uint4 Ck_ = k_ < 2u ? C0 : k_ < 4u ? C1 : k_ < 6u ? C2 : C3;
                                const uint32_t lo_ = ln_sel4(Ck_, (2u * k_) & 3u), hi_ = ln_sel4(Ck_, (2u * k_ + 1u) & 3u);
                                /* the high bytes of cand words 4k..4k+3 (their codes in bits 5-7) */
                                const uint32_t x_ = __builtin_amdgcn_perm(hi_, lo_, 0x07050301u);
                                /* bit 7 of each byte: its code is nonzero; the multiply gathers
                                 * bits 7, 15, 23, 31 into bits 28-31 (no carries reach them) */
                                const uint32_t t_ = (x_ | (x_ << 1) | (x_ << 2)) & 0x80808080u;
                                fm |= ((t_ * 0x00204081u) >> 28) << (4u * k_);
                            }
                            fmb = cb;
                        }
#pragma unroll
                        for (uint32_t e_ = 0; e_ < K2_LITX; e_++) {
                            const uint32_t d_ = p - cb, x_ = p - wb;
                            uint32_t r_ = 0u;
                            if (go && p < n - 2u && d_ < K2_CB && x_ < 16u && o < cap) {
                                const uint32_t z_ = fm >> d_;
                                r_ = z_ ? (uint32_t)__builtin_ctz(z_) : 32u;
                                r_ = min(r_, min(K2_CB - d_, 16u - x_));
                                r_ = min(r_, min(n - 2u - p, cap - o));
                                r_ = min(r_, min(LZF_MAX_LIT - run, 32u - (p & 31u)));
                                r_ = min(r_, run == 0u ? 3u : 4u);     /* acc: at most 4 new bytes per put */
                            }
                            go = r_ != 0u;
                            if ((uint32_t)__builtin_popcountll(__ballot(go)) < K2_LITMIN) break;
                            K2_WS(8);
                            if (go) {
                                K2_SITE(9);
                                curw |= ((1u << r_) - 1u) << (p & 31u);
                                const uint32_t lo_ = ln_sel4(W, x_ >> 2), hi_ = ln_sel4(W, (x_ >> 2) + 1u);
                                const uint32_t by_ = __builtin_amdgcn_alignbit(hi_, lo_, 8u * (x_ & 3u)) &
                                                     (r_ == 4u ? 0xFFFFFFFFu : (1u << (8u * r_)) - 1u);
                                const bool first_ = run == 0u;
                                hx = first_ ? 4u * fw + accn : hx;
                                K2_PUT(first_ ? (uint64_t)by_ << 8 : (uint64_t)by_, first_ ? r_ + 1u : r_);
                                o += r_;
                                run += r_;
                                if (run == LZF_MAX_LIT) { K2_PATCH(hx, LZF_MAX_LIT - 1u); run = 0u; o++; }
                                p += r_;
                                if ((p & 31u) == 0u) {
                                    K2_FLUSH_TO(cw);
                                    K2_RING(cw) = curw;
                                    cw++;
                                    curw = 0u;
                                }
                            }
                        }
                    }
#else
                    if ((uint32_t)__builtin_popcountll(__ballot(true)) >= K2_LITMIN)
#pragma unroll
                    for (uint32_t e_ = 0; e_ < K2_LITX; e_++) {
                        const uint32_t d_ = p - cb, x_ = p - wb;
                        go = go && p < n - 2u && d_ < K2_CB && x_ < 16u && o < cap;
                        if (go) {
                            const uint32_t dw_ = d_ >> 1;
                            const uint4 Cq_ = dw_ < 8u ? (dw_ < 4u ? C0 : C1) : (dw_ < 12u ? C2 : C3);
                            go = ((ln_sel4(Cq_, dw_ & 3u) >> (16u * (d_ & 1u))) & 0xE000u) == 0u;
                        }
                        /* a trip the wave takes only when enough lanes gain
                         * from it: on text, where few do, the others would
                         * wait through it */
                        if ((uint32_t)__builtin_popcountll(__ballot(go)) < K2_LITMIN) break;
                        if (go) {
                            K2_SITE(9);
                            curw |= 1u << (p & 31u);
                            const uint32_t byte_ = (ln_sel4(W, x_ >> 2) >> (8u * (x_ & 3u))) & 0xFFu;
                            const bool first_ = run == 0u;
                            hx = first_ ? 4u * fw + accn : hx;
                            K2_PUT(first_ ? byte_ << 8 : byte_, first_ ? 2u : 1u);
                            o++;
                            if (++run == LZF_MAX_LIT) { K2_PATCH(hx, LZF_MAX_LIT - 1u); run = 0u; o++; }
                            p++;
                            if ((p & 31u) == 0u) {
                                K2_FLUSH_TO(cw);
                                K2_RING(cw) = curw;
                                cw++;
                                curw = 0u;
                            }
                        }
                    }
#endif  /* K2_LITB */
#endif
                }
            } else {
                K2_WS(9);
                uint32_t maxlen = n - p - 2u;                            /* src/lzf_c.c:169-170 */
                if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
                lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
                if (rel <= 6u) {
                    m = rel + 1u < lim ? rel + 1u : lim;
                    mode = K2_EMIT;
                } else {
                    k = rel == 7u ? 8u : 3u;
                    mode = K2_EXTEND;
                }
            }
        }
        /* ---- one 16-byte piece of a long match --------------------------- */
        if (mode == K2_EXTEND) {
            K2_WS(10);
            if (k < lim) {
                K2_SITE(7);
                const uint32_t avail = n - (p + k);
                const uint4 a = ln_ld16_safe(src + p + k, avail), b = ln_ld16_safe(src + q + k, avail);
                W = a;                                   /* literals after the match read it */
                wb = p + k;
                const uint32_t d = ln_first_diff(a, b);
                k += d;
                if (d < 16u) lim = k < lim ? k : lim;
            }
            if (k >= lim) {
                m = lim;
                mode = K2_EMIT;
            }
        }
        /* ---- the back-reference ------------------------------------------ */
        if (mode == K2_EMIT) {
            K2_WS(11);
            const uint32_t off = p - q - 1u;
            if (run) K2_PATCH(hx, run - 1u);                             /* close the run */
            else o--;                                                    /* undo empty run */
            if (o + 4u >= cap) {                                         /* src/lzf_c.c:176 */
                ok = false;
                mode = K2_DONE;
            } else {
                const uint32_t L = m - 2u;
                const bool two = L < 7u;
                K2_PUT(two ? ((off >> 8) | (L << 5)) | ((off & 0xFFu) << 8)
                           : (0xE0u | (off >> 8)) | ((L - 7u) << 8) | ((off & 0xFFu) << 16),
                       two ? 2u : 3u);
                o += two ? 2u : 3u;
                run = 0u;
                o++;                                                     /* reserve a header */
                ms = p;
                p += m;
                me = p;
                if (p >= n - 2u) {                                       /* src/lzf_c.c:229 */
                    mode = K2_DONE;
                } else {
                    /* the two last positions of the match are inserted, its interior not */
                    const uint32_t nw = p >> 5, t1 = p - 2u, t2 = p - 1u;
                    const uint32_t b1 = 1u << (t1 & 31u), b2 = 1u << (t2 & 31u);
                    if (nw == cw) {
                        curw |= b1 | b2;
                    } else {
                        K2_WS(12);
                        uint32_t wo = curw, wm = 0u, wn = 0u;
                        if ((t1 >> 5) == cw) wo |= b1; else if ((t1 >> 5) == nw) wn |= b1; else wm |= b1;
                        if ((t2 >> 5) == cw) wo |= b2; else if ((t2 >> 5) == nw) wn |= b2; else wm |= b2;
                        K2_FLUSH_TO(cw);
                        K2_RING(cw) = wo;
                        /* words cw+1 .. nw-2 are all interior (0), nw-1 holds tails */
                        for (uint32_t w = cw + 1u; w < nw; w++) {
                            K2_FLUSH_TO(w);
                            K2_RING(w) = w + 1u == nw ? wm : 0u;
                        }
                        curw = wn;
                        cw = nw;
                    }
                    mode = K2_STEP;
                }
            }
        }
        /* ---- a finished value: its tail (src/lzf_c.c:276-290), then the next */
        if (live && mode == K2_DONE) {
            if (!ok || o + 3u > cap) {                                    /* src/lzf_c.c:276 */
                bt.out_len[v] = 0u;
            } else {
                while (p < n) {                                           /* src/lzf_c.c:279-288 */
                    K2_LITERAL(p);
                    p++;
                }
                if (run) K2_PATCH(hx, run - 1u);
                else o--;
                for (uint32_t i = fs; i < fw; i++) {
                    const uint32_t wv = i == fs ? pb0 : i == fs + 1u ? pb1 : pb2;
                    if (i == 0u && dm != 0u)
                        for (uint32_t t = dm; t < 4u; t++) da[t] = (uint8_t)(wv >> (8u * t));
                    else
                        *(uint32_t *)(da + 4u * i) = wv;
                }
                for (uint32_t t = 0; t < accn; t++)
                    if (4u * fw + t >= dm) da[4u * fw + t] = (uint8_t)(acc >> (8u * t));
                bt.out_len[v] = o;
            }
            K2_START();
        }
    }
#ifdef K2_WAVE_SITES
    for (uint32_t i_ = 0; i_ < 16u; i_++)
        if (wsc_[i_]) atomicAdd(&k2_sites[i_], (unsigned long long)wsc_[i_]);
#endif
#undef K2_STORE16
#undef K2_PUT
#undef K2_PATCH
#undef K2_BYTE
#undef K2_LITERAL
#undef K2_RING
#undef K2_FLUSH_TO
#undef K2_NEXT
#undef K2_LOAD_AHEAD
#undef K2_START
}

#ifdef LZF_DIAG   /* wave-form parse: cross-check form */
/* ======================================================================== */
/* compress, kernel 2 (wave form): the parse 64 positions at a time         */
/* ======================================================================== */

/* One wave per value of the small class; the value's bytes, its cand words
 * and an inserted-bitmap live in LDS.  Per window of 64 positions from the
 * parse position P every lane decides its position as if the parse visited
 * it: its ref is the first inserted position on the cand chain, literal or
 * match, and the match length (cand agreement, else an 8-byte probe).  A
 * candidate before P is checked in the bitmap (decided); one inside the
 * window is assumed inserted.  The scalar unit then follows the parse's
 * orbit P -> P + step -> ... jumping over runs of literal lanes; lanes it
 * stops at that still need work get it there, so only visited positions pay
 * for it: a candidate found skipped is walked back along its cand chain, a
 * match longer than the probe is measured by the whole wave (256 bytes at
 * once).  A visited lane whose in-window candidate turns out to lie in a
 * match interior (not inserted: src/lzf_c.c:227-247) ends the window there,
 * so every emitted token is the reference's.  Emission is closed form over
 * the window's tokens (prefix sum of output sizes; a run's header is written
 * when the run closes) with the reference's out-of-space checks. */
#define KW_MAXN KS_MAXN

/* lane states of a window */
#define KW_LIT   0u    /* literal */
#define KW_MATCH 1u    /* match of length m */
#define KW_LONG  2u    /* match of length >= k (k < lim), to be measured */
#define KW_WALK  3u    /* candidate q not inserted: walk the chain first */

/* literal or match at x given the ref q and its rel code (src/lzf_c.c:151-209) */
__device__ __forceinline__ void kw_decide(const uint32_t *Bw, uint32_t n, uint32_t x, bool act, uint32_t rel,
                                          uint32_t q, uint32_t &st, uint32_t &m, uint32_t &k, uint32_t &lim)
{
    st = KW_LIT;
    m = 1u;
    if (!(act && rel >= 2u && x + 4u < n)) return;
    uint32_t maxlen = n - x - 2u;                                     /* src/lzf_c.c:169-170 */
    if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
    lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
    st = KW_MATCH;
    if (rel <= 6u) {
        m = rel + 1u < lim ? rel + 1u : lim;
        return;
    }
    k = rel == 7u ? 8u : 3u;
    const uint32_t d0 = ks_rd4(Bw, x + k) ^ ks_rd4(Bw, q + k);
    const uint32_t d1 = ks_rd4(Bw, x + k + 4u) ^ ks_rd4(Bw, q + k + 4u);
    if (d0) k += (uint32_t)__builtin_ctz(d0) >> 3;
    else if (d1) k += 4u + ((uint32_t)__builtin_ctz(d1) >> 3);
    else k += 8u;
    if (!(d0 | d1) && k < lim) st = KW_LONG;
    m = k < lim ? k : lim;
}

/* one link back along the cand chain from a skipped q */
__device__ __forceinline__ bool kw_hop(const uint16_t *Cw, uint32_t x, uint32_t &rel, uint32_t &q)
{
    K2_SITE(12);
    const uint32_t c2 = Cw[q], r2 = c2 >> 13, q2 = q - 1u - (c2 & 0x1FFFu);
    if (!r2 || x - q2 - 1u >= LZF_WINDOW) {
        rel = 0u;
        return false;
    }
    const bool e1 = rel >= 2u && rel <= 8u, e2 = r2 >= 2u;
    rel = rel == 9u ? 9u : (e1 && e2) ? 8u : (e1 != e2) ? 1u : 9u;
    q = q2;
    return true;
}

/* first inserted position on the cand chain from q (q < P: the bitmap is
 * final there); rel follows it: 8 equal (length unknown), 1 differ, 0 none.
 * A skipped position below P is never visited, so its cand word serves only
 * walks through it: the walk's start q0 is pointed straight at the result
 * (path compression; code 2 = 3 bytes equal, 1 = differ, 0 = none). */
__device__ __forceinline__ void kw_walk(const uint32_t *Bw, uint16_t *Cw, const uint32_t *IB, uint32_t x,
                                        uint32_t &rel, uint32_t &q, uint32_t q0)
{
    while (!((IB[q >> 5] >> (q & 31u)) & 1u)) {
        if (!kw_hop(Cw, x, rel, q)) {
            Cw[q0] = 0u;
            return;
        }
    }
    if (q != q0) {
        const bool eq = ((ks_rd4(Bw, q0) ^ ks_rd4(Bw, q)) & 0xFFFFFFu) == 0u;
        Cw[q0] = (uint16_t)(((eq ? 2u : 1u) << 13) | (q0 - q - 1u));
    }
    if (rel == 9u) rel = ((ks_rd4(Bw, x) ^ ks_rd4(Bw, q)) & 0xFFFFFFu) == 0u ? 8u : 1u;
}
__device__ __forceinline__ unsigned long long kw_range(uint32_t a, uint32_t b)   /* bits [a, b), a < 64 */
{
    const unsigned long long hi = b >= 64u ? ~0ull : (1ull << b) - 1ull;
    return hi & ~((1ull << a) - 1ull);
}

__global__ __launch_bounds__(64) void lzf_parse_wave_kernel(LzfBatch bt, LzfLaneScratch sc)
{
    __shared__ __attribute__((aligned(16))) uint32_t Bw[KW_MAXN / 4u + 8u];
    __shared__ __attribute__((aligned(16))) uint16_t Cw[KW_MAXN + 64u];
    __shared__ uint32_t IB[KW_MAXN / 32u + 4u];
    const uint32_t lane = threadIdx.x, v = blockIdx.x;
    const unsigned long long mine = 1ull << lane, lt = mine - 1ull;
    const uint32_t n = bt.in_len[v], cap = bt.out_cap[v];
    if (n == 0u || cap == 0u) {                                       /* src/lzf_c.c:131 */
        if (lane == 0u) bt.out_len[v] = 0u;
        return;
    }
    const uint8_t *src = bt.in + bt.in_off[v];
    uint8_t *dst = bt.out + bt.out_off[v];
    const uint32_t np = n >= 3u ? n - 2u : 0u;                        /* positions 0 .. n-3 */
#ifdef KW_PHASES
    uint64_t ph_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ph_t = clock64();
#endif
    {
        const uint4 *cand = (const uint4 *)(sc.cand + (uint64_t)v * sc.cstride);
        for (uint32_t k = lane; k < (KW_MAXN / 4u + 8u) / 4u; k += 64u) {
            const uint32_t at = 16u * k;
            ((uint4 *)Bw)[k] = at < n ? ln_ld16_safe(src + at, n - at) : make_uint4(0, 0, 0, 0);
        }
        for (uint32_t k = lane; k < (np + 7u) / 8u; k += 64u) ((uint4 *)Cw)[k] = cand[k];
        for (uint32_t k = lane; k < KW_MAXN / 32u + 4u; k += 64u) IB[k] = 0u;
    }
    __syncthreads();
    KW_PH(0);
#define KW_BYTE(x_) ((Bw[(x_) >> 2] >> (8u * ((x_) & 3u))) & 0xFFu)
    uint32_t P = 0u, o = 1u, run = 0u;                                /* op, lit of the reference */
    bool ok = true;
    while (P < np) {
        if (lane == 0u) K2_SITE(11);
        const uint32_t x = P + lane;
        const bool act = x < np;
        const uint32_t c = act ? (uint32_t)Cw[x] : 0u;
        /* rel: 0 no ref; 1 ref with other bytes; 2..6 equal for rel+1 bytes;
         * 7 equal >= 8; 8 equal 3 bytes, length unknown; 9 unknown */
        uint32_t rel = c >> 13;
        uint32_t q = x - 1u - (c & 0x1FFFu);
        const bool spec = rel != 0u && q >= P;                        /* assumed inserted */
        uint32_t st = KW_LIT, m = 1u, k = 0u, lim = 0u;
        const uint32_t q1 = q;
        bool walk = rel != 0u && !spec && !((IB[q >> 5] >> (q & 31u)) & 1u);
        if (walk) {                                                   /* one link back, all lanes */
            walk = kw_hop(Cw, x, rel, q) && !((IB[q >> 5] >> (q & 31u)) & 1u);
            if (!walk && rel == 9u) rel = ((ks_rd4(Bw, x) ^ ks_rd4(Bw, q)) & 0xFFFFFFu) == 0u ? 8u : 1u;
        }
        if (walk) st = KW_WALK;
        else kw_decide(Bw, n, x, act, rel, q, st, m, k, lim);
        KW_PH(1);
        /* the orbit of the parse through the window: runs of literal lanes
         * are taken at once, the scalar loop stops at the other lanes */
        const uint32_t end = np - P < 64u ? np - P : 64u;             /* lanes that are positions */
        unsigned long long STOP = __ballot(st != KW_LIT), V = 0ull;
        uint32_t t = 0u;
        while (true) {
            const unsigned long long rest = STOP & ~((1ull << t) - 1ull);
            const uint32_t u = rest ? (uint32_t)__builtin_ctzll(rest) : 64u;
            if (u >= end) {
                V |= kw_range(t, end);
                t = end;
                break;
            }
            V |= kw_range(t, u + 1u);
            if (lane == 0u) K2_SITE(15);
            uint32_t su = (uint32_t)__builtin_amdgcn_readlane((int)st, (int)u);
            if (su == KW_WALK) {                                      /* skipped candidate */
                KW_PH(2);
                if (lane == 0u) K2_SITE(10);
                if (lane == u) {
                    kw_walk(Bw, Cw, IB, x, rel, q, q1);
                    kw_decide(Bw, n, x, act, rel, q, st, m, k, lim);
                }
                su = (uint32_t)__builtin_amdgcn_readlane((int)st, (int)u);
                KW_PH(6);
            }
            if (su == KW_LONG) {                                      /* the wave measures it */
                KW_PH(2);
                if (lane == 0u) K2_SITE(13);
                const uint32_t xu = P + u;
                const uint32_t qu = (uint32_t)__builtin_amdgcn_readlane((int)q, (int)u);
                const uint32_t ku = (uint32_t)__builtin_amdgcn_readlane((int)k, (int)u);
                const uint32_t lu = (uint32_t)__builtin_amdgcn_readlane((int)lim, (int)u);
                const uint32_t at = ku + 4u * lane;
                const uint32_t dd = at < lu ? ks_rd4(Bw, xu + at) ^ ks_rd4(Bw, qu + at) : 0xFFu;
                const unsigned long long dm = __ballot(dd != 0u);
                uint32_t mu = lu;
                if (dm) {
                    const uint32_t j = (uint32_t)__builtin_ctzll(dm);
                    const uint32_t dj = (uint32_t)__builtin_amdgcn_readlane((int)dd, (int)j);
                    const uint32_t e = ku + 4u * j + ((uint32_t)__builtin_ctz(dj) >> 3);
                    mu = e < lu ? e : lu;
                }
                if (lane == u) {
                    m = mu;
                    st = KW_MATCH;
                }
                su = KW_MATCH;
                KW_PH(7);
            }
            t = su == KW_LIT ? u + 1u : u + (uint32_t)__builtin_amdgcn_readlane((int)m, (int)u);
            if (t >= end) break;
        }
        KW_PH(2);
        const bool hit = st != KW_LIT;                                /* every visited lane is final */
        const unsigned long long HITm = __ballot(hit);
        const bool isv = (V >> lane) & 1ull;
        const uint32_t s = ks_hibit(V & (lt | mine));                 /* latest token <= lane */
        const uint32_t m_s = (uint32_t)__shfl((int)m, (int)s);
        const bool inm = !isv && ((HITm >> s) & 1ull);                /* inside s's match */
        const unsigned long long IM = __ballot(inm && lane + 2u < s + m_s);
        const unsigned long long INV = V & __ballot(spec && ((IM >> (q - P)) & 1ull));
        const uint32_t f = INV ? (uint32_t)__builtin_ctzll(INV) : 64u;
        if (lane == 0u && f < 64u) K2_SITE(14);
        const unsigned long long keep = f < 64u ? (1ull << f) - 1ull : ~0ull;
        const unsigned long long TK = V & keep;
        const unsigned long long INS = __ballot(isv || (inm && lane + 2u >= s + m_s)) & keep;
        KW_PH(3);

        /* emission (src/lzf_c.c:172-224, 258-273) */
        const bool tok = (TK >> lane) & 1ull;
        const unsigned long long Mb = TK & HITm, Lb = TK & ~HITm, mlt = Mb & lt;
        const unsigned long long seg = mlt ? lt & ~((2ull << ks_hibit(mlt)) - 1ull) : lt;
        const uint32_t lb = (uint32_t)__builtin_popcountll(Lb & seg);
        const uint32_t r0 = (mlt ? 0u : run) + lb;                    /* open run before lane */
        const uint32_t rl = r0 & 31u;
        /* output bytes of a token: literal 1 (+1 on a rollover); match 3
         * (+1 long form, -1 when it undoes an empty run): prefix sums as
         * lane-mask popcounts */
        const unsigned long long RL = __ballot(tok && !hit && ((r0 + 1u) & 31u) == 0u);
        const unsigned long long BG = __ballot(tok && hit && m - 2u >= 7u);
        const unsigned long long UD = __ballot(tok && hit && rl == 0u);
#define KW_MB(M_) __builtin_amdgcn_mbcnt_hi((uint32_t)((M_) >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)(M_), 0u))
        const uint32_t ob = o + KW_MB(TK) + KW_MB(RL) + 2u * KW_MB(Mb) + KW_MB(BG) - KW_MB(UD);
#undef KW_MB
        const uint32_t osum = (uint32_t)(__builtin_popcountll(TK) + __builtin_popcountll(RL) +
                                         2 * __builtin_popcountll(Mb) + __builtin_popcountll(BG) -
                                         __builtin_popcountll(UD));
        const uint32_t om = ob - (rl == 0u ? 1u : 0u);
        const bool bad = tok && (hit ? om + 4u >= cap : ob >= cap);   /* src/lzf_c.c:176, 263 */
        KW_PH(4);
        if (__ballot(bad)) {
            ok = false;
            break;
        }
        if (tok) {
            if (!hit) {
                dst[ob] = (uint8_t)KW_BYTE(x);
                if (((r0 + 1u) & 31u) == 0u) dst[ob - LZF_MAX_LIT] = (uint8_t)(LZF_MAX_LIT - 1u);
            } else {
                const uint32_t off = x - q - 1u, L = m - 2u;
                if (rl) dst[ob - rl - 1u] = (uint8_t)(rl - 1u);       /* close the run */
                if (L < 7u) {
                    dst[om] = (uint8_t)((off >> 8) | (L << 5));
                    dst[om + 1u] = (uint8_t)off;
                } else {
                    dst[om] = (uint8_t)(0xE0u | (off >> 8));
                    dst[om + 1u] = (uint8_t)(L - 7u);
                    dst[om + 2u] = (uint8_t)off;
                }
            }
        }
        /* inserted positions of the window; a match past the window inserts
         * its two last positions (src/lzf_c.c:227-247) */
        if (lane < 3u) {
            const uint32_t sh = P & 31u;
            const unsigned long long lo = INS << sh;
            const uint32_t w = lane == 0u ? (uint32_t)lo : lane == 1u ? (uint32_t)(lo >> 32)
                                                                      : (sh ? (uint32_t)(INS >> (64u - sh)) : 0u);
            if (w) IB[(P >> 5) + lane] |= w;
        }
        const uint32_t last = ks_hibit(TK);
        if (f == 64u && lane == last && hit && lane + m > 64u) {
            const uint32_t t1 = x + m - 2u, t2 = t1 + 1u;
            if (lane + m - 2u >= 64u) IB[t1 >> 5] |= 1u << (t1 & 31u);
            IB[t2 >> 5] |= 1u << (t2 & 31u);
        }
        o += osum;
        run = ((HITm >> last) & 1ull) ? 0u : (((uint32_t)__builtin_amdgcn_readlane((int)r0, (int)last) + 1u) & 31u);
        P = f < 64u ? P + f : P + t;
        KW_PH(5);
        ln_wave_fence();
    }
#ifdef KW_PHASES
    if (lane == 0u)
        for (uint32_t i = 0; i < 8u; i++) atomicAdd(&k2_sites[i], (unsigned long long)ph_[i]);
#endif
    if (lane == 0u) {
        if (!ok || o + 3u > cap) {                                    /* src/lzf_c.c:276 */
            bt.out_len[v] = 0u;
        } else {
            for (uint32_t p = P; p < n; p++) {                        /* src/lzf_c.c:279-288 */
                dst[o++] = (uint8_t)KW_BYTE(p);
                if (++run == LZF_MAX_LIT) {
                    dst[o - LZF_MAX_LIT - 1u] = (uint8_t)(LZF_MAX_LIT - 1u);
                    run = 0u;
                    o++;
                }
            }
            if (run) dst[o - run - 1u] = (uint8_t)(run - 1u);
            else o--;
            bt.out_len[v] = o;
        }
    }
#undef KW_BYTE
}

#endif /* LZF_DIAG */

/* ---- launcher ------------------------------------------------------------ */

/* cand words per value: a multiple of 64 (128 bytes), so the parse's 64-byte
 * blocks never straddle a line, plus slack for the last block */
static uint64_t lane_cstride(uint32_t max_len) { return (((uint64_t)max_len + 63u) & ~63ull) + 64u; }
static uint64_t lane_bstride(uint32_t max_len) { return ((((uint64_t)max_len + 31u) >> 5) + 3u) & ~3ull; }

size_t lzf_lane_scratch_per_value(uint32_t max_len)
{
    return (size_t)(lane_cstride(max_len) * 2u + lane_bstride(max_len) * 4u);
}

/* The default lane path takes the small and ring classes (values <= 64 KiB;
 * LZF_GPU_LANE_RING=0 stops it at 8 KiB, and LZF_GPU_LANE_MID=1 then routes
 * values up to 64 KiB through the mid-class kernels). */
#ifdef LZF_DIAG
static bool lane_ring_enabled()
{
    const char *r = getenv("LZF_GPU_LANE_RING");     /* "0" turns the ring class off */
    return !(r && *r == '0');
}
#endif

/* kernel 1 of the lane generation: the stream form (lzf_stream.hip: the
 * exact table, values back to back in one pipeline per CU; any value of at
 * most 64 KiB), or -- diagnostic build, LZF_GPU_CAND=small, read per launch,
 * a cross-check -- the small class (values of at most 4 KiB; the ring and
 * mid classes past that).  json4k 1 M x 4 KiB: 45.9 ms with the stream form,
 * 48.7 with the small class (cand 17.3 vs 19.9 ms, rocprof). */
static bool lane_cand_small()
{
#ifdef LZF_DIAG
    const char *e = getenv("LZF_GPU_CAND");
    return e && !strcmp(e, "small");
#else
    return false;
#endif
}

const char *lzf_lane_cand_name(void) { return lane_cand_small() ? "cand_small" : "cand_stream"; }

bool lzf_lane_compress_supported(uint32_t max_len)
{
#ifndef LZF_DIAG
    /* the stream form takes any value the parse's 13-bit offsets and 16-bit
     * positions cover */
    return max_len <= LZF_SLOTS;
#else
    if (!lane_cand_small()) return max_len <= LZF_SLOTS;
    if (max_len <= KS8_MAXN) return true;
    if (max_len <= KR64_MAXN && lane_ring_enabled()) return true;
    const char *e = getenv("LZF_GPU_LANE_MID");
    return max_len <= KM_MAXN && e && *e == '1';
#endif
}

/* blocks of the lane parse resident on the whole device at once (0: unknown);
 * LZF_GPU_PARSE_RESIDENT overrides it (diagnostics) */
static uint32_t parse_resident(size_t lds)
{
    if (const char *e = getenv("LZF_GPU_PARSE_RESIDENT")) return (uint32_t)strtoul(e, nullptr, 10);
    int dev = 0, cus = 0, per = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void *)lzf_parse_lane_kernel, (int)K2_THREADS,
                                                     lds) != hipSuccess ||
        cus <= 0 || per <= 0) {
        (void)hipGetLastError();
        return 0u;
    }
    return (uint32_t)cus * (uint32_t)per;
}

hipError_t lzf_launch_compress_lane(const LzfBatch &b, hipStream_t s, void *scratch,
                                    size_t scratch_bytes, uint32_t force_fix, hipStream_t aux,
                                    hipEvent_t *ev, uint32_t *chunks)
{
    if (!lzf_lane_compress_supported(b.max_len)) return hipErrorInvalidValue;
    const uint64_t cstride = lane_cstride(b.max_len), bstride = lane_bstride(b.max_len);
    /* with an aux stream: two scratch halves, kernel 1 of chunk i+1 on s
     * overlaps kernel 2 of chunk i on aux */
    const bool pipe = aux != nullptr && ev != nullptr &&
                      scratch_bytes / 2u >= lzf_lane_scratch_per_value(b.max_len) + 512u && b.count >= 4u;
    const size_t half = pipe ? (scratch_bytes / 2u) & ~(size_t)255 : scratch_bytes;
    uint64_t chunk = half / lzf_lane_scratch_per_value(b.max_len);
    const auto bits_at = [&](uint64_t ch) { return ((ch * cstride * 2u) + 255u) & ~255ull; };
    while (chunk && bits_at(chunk) + chunk * bstride * 4u > half) chunk--;
    if (chunk == 0) return hipErrorInvalidValue;
    if (pipe) {                       /* at least 4 chunks so the stages overlap */
        const uint64_t quarter = (b.count + 3u) / 4u;
        if (quarter < chunk) chunk = quarter < 1024u ? (b.count < 1024u ? b.count : 1024u) : quarter;
    }
    if (chunks) *chunks = (uint32_t)((b.count + chunk - 1u) / chunk);
    LzfLaneScratch sc[2];
    for (int h = 0; h < 2; h++) {
        uint8_t *base = (uint8_t *)scratch + (pipe ? h * half : 0);
        sc[h].cand = (uint16_t *)base;
        sc[h].bits = (uint32_t *)(base + bits_at(chunk));
        sc[h].cstride = cstride;
        sc[h].bstride = bstride;
        sc[h].force_fix = force_fix;
    }
    /* the small-class kernel (diagnostic) is persistent: as many one-wave
     * workgroups as stay resident (LDS-bound), each walking the batch */
#ifdef LZF_DIAG
    const bool ring = b.max_len > KS8_MAXN && b.max_len <= KR64_MAXN && lane_ring_enabled();
    const void *small_fn = b.max_len <= KS_MAXN    ? (const void *)lzf_cand_small_kernel<4u, KS_MAXN, KS_WIN>
                           : b.max_len <= KS8_MAXN ? (const void *)lzf_cand_small_kernel<3u, KS8_MAXN, KS8_WIN>
                           : b.max_len <= KR_MAXN  ? (const void *)lzf_cand_ring_kernel<KR_MAXN, KR_WIN>
                                                   : (const void *)lzf_cand_ring_kernel<KR64_MAXN, KR_WIN>;
    uint32_t small_grid = 256u * 8u;
    if (lane_cand_small()) {
        int dev = 0, cus = 0;
        hipFuncAttributes fa;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipFuncGetAttributes(&fa, small_fn) == hipSuccess && cus > 0 &&
            fa.sharedSizeBytes > 0) {
            uint32_t per = (uint32_t)(160u * 1024u / fa.sharedSizeBytes);   /* LDS-bound residency */
            const char *pe_ = getenv("LZF_LANE_CAND_PER");            /* residency override */
            if (pe_ && atoi(pe_) > 0) per = (uint32_t)atoi(pe_);
            if (per > 32u) per = 32u;
            if (per < 1u) per = 1u;
            small_grid = (uint32_t)cus * per;
        }
    }
#endif
    /* kernel 2: one lane per value; LZF_GPU_LANE_PARSE=wave selects the wave
     * form for the small class (slower today) */
#ifdef LZF_DIAG
    const char *pe = getenv("LZF_GPU_LANE_PARSE");
    const bool wave_parse = b.max_len <= KW_MAXN && pe && pe[0] == 'w';
#endif
    const size_t parse_lds = lane_lds_for("LZF_LANE_PARSE_BLOCKS", 0u);
    if (parse_lds) {
        hipError_t e = hipFuncSetAttribute((const void *)lzf_parse_lane_kernel,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)parse_lds);
        if (e != hipSuccess) return e;
    }
    const bool stream = !lane_cand_small();
    /* diagnostics: LZF_GPU_LANE_STAGE=1 runs kernel 1 only (its own time) */
    const char *stg = getenv("LZF_GPU_LANE_STAGE");
    const bool cand_only = stg && *stg == '1';
    hipError_t e;
    uint32_t i = 0;
    for (uint64_t first = 0; first < b.count; first += chunk, i++) {
        const uint32_t cnt = (uint32_t)((b.count - first) < chunk ? (b.count - first) : chunk);
        const int h = pipe ? (int)(i & 1u) : 0;
        LzfBatch c = b;
        c.in_off = b.in_off + first;
        c.in_len = b.in_len + first;
        c.out_off = b.out_off + first;
        c.out_cap = b.out_cap + first;
        c.out_len = b.out_len + first;
        c.count = cnt;
        /* scratch half h is free once kernel 2 of chunk i-2 is done */
        if (pipe && i >= 2u && (e = hipStreamWaitEvent(s, ev[2 + h], 0)) != hipSuccess) return e;
        if (stream) {
            if ((e = lzf_launch_cand_stream(c, sc[h], s)) != hipSuccess) return e;
        }
#ifdef LZF_DIAG
        else if (b.max_len <= KS_MAXN) {
            const uint32_t g = cnt < small_grid ? cnt : small_grid;
            hipLaunchKernelGGL((lzf_cand_small_kernel<4u, KS_MAXN, KS_WIN>), dim3(g), dim3(64), 0, s, c, sc[h]);
        } else if (b.max_len <= KS8_MAXN) {
            const uint32_t g = cnt < small_grid ? cnt : small_grid;
            hipLaunchKernelGGL((lzf_cand_small_kernel<3u, KS8_MAXN, KS8_WIN>), dim3(g), dim3(64), 0, s, c, sc[h]);
        } else if (ring) {
            const uint32_t g = cnt < small_grid ? cnt : small_grid;
            if (b.max_len <= KR_MAXN)
                hipLaunchKernelGGL((lzf_cand_ring_kernel<KR_MAXN, KR_WIN>), dim3(g), dim3(64), 0, s, c, sc[h]);
            else
                hipLaunchKernelGGL((lzf_cand_ring_kernel<KR64_MAXN, KR_WIN>), dim3(g), dim3(64), 0, s, c, sc[h]);
        } else {
            hipLaunchKernelGGL(lzf_cand_mid_kernel, dim3(cnt), dim3(64), 0, s, c, sc[h]);
        }
#endif
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (cand_only) continue;
        hipStream_t s2 = s;
        if (pipe) {
            if ((e = hipEventRecord(ev[h], s)) != hipSuccess) return e;
            if ((e = hipStreamWaitEvent(aux, ev[h], 0)) != hipSuccess) return e;
            s2 = aux;
        }
#ifdef LZF_DIAG
        if (wave_parse)
            hipLaunchKernelGGL(lzf_parse_wave_kernel, dim3(cnt), dim3(64), 0, s2, c, sc[h]);
        else
#endif
        {
            /* persistent lanes: as many blocks as stay resident */
            uint32_t grid = (cnt + K2_THREADS - 1u) / K2_THREADS;
            const uint32_t res = parse_resident(parse_lds);
            if (res && grid > res) grid = res;
            hipLaunchKernelGGL(lzf_parse_lane_kernel, dim3(grid), dim3(K2_THREADS), parse_lds, s2, c, sc[h]);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (pipe && (e = hipEventRecord(ev[2 + h], aux)) != hipSuccess) return e;
    }
    if (pipe) {                       /* join: s waits for the last kernel 2 of both halves */
        for (uint32_t h = 0; h < 2u && h < i; h++)
            if ((e = hipStreamWaitEvent(s, ev[2 + h], 0)) != hipSuccess) return e;
    }
    return hipSuccess;
}

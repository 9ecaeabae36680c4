/*
 * lzf_wparse.hip -- the "window" generation of the LZF compressor for gfx950
 * (values of at most 64 KiB).  Two kernels per batch:
 *
 *   1. lzf_cand_q1_kernel -- position-parallel, one value at a time per
 *      workgroup (one workgroup per CU: the table is 128 KiB of LDS).  For
 *      every position p it finds q1(p), the latest earlier position with p's
 *      16-bit slot, from an exact direct-mapped table T[slot] -> latest
 *      position (65536 x u16, the reference's own table size, src/lzfP.h:55)
 *      updated in position order by lane-ordered ds_mskor_rtn_b32 exchanges,
 *      and stores the u16 cand word [1:3 | p - q1 - 1 : 13] (0: none) in HBM.
 *
 *   2. lzf_wparse_kernel -- the greedy parse and emission, ONE WAVE PER
 *      VALUE, 64 positions per window.  The reference's ref at a visited p is
 *      the latest INSERTED position with p's slot (src/lzf_c.c:147-149);
 *      inserted = every visited position plus the last two positions of a
 *      match (src/lzf_c.c:227-247).  The wave keeps a ring R over the last
 *      8192 positions in LDS:
 *          R(x) = x                 if x is inserted,
 *               = R(q1(x))          otherwise,
 *      so the ref at a visited p is R(q1(p)) -- one LDS read, no chain walk
 *      (tools/rparse_model.c checks the identity on every visited position).
 *      Per window:
 *        a. links: x = q1(p); the window's same-slot lanes SM(p) and the
 *           chain's exit xo(p) (its first link out of the window) by pointer
 *           doubling; r_out = R(xo) from the ring;
 *        b. 16 bytes at p and at r_out (and at x, from lane x) -> matched
 *           lengths LB, LA, capped at 16;
 *        c. a scalar walk over the window's stop lanes (possible matches,
 *           and lanes whose ref depends on the window's own inserted mask);
 *           runs of literals between them are skipped by find-first-set; a
 *           match whose 16 bytes all agree is measured by the whole wave;
 *        d. emission: token sizes from lane masks (popcounts), output
 *           offsets as one prefix sum, run headers written when a run
 *           closes; the reference's out-of-space checks (src/lzf_c.c:176,
 *           263, 276) as final-position tests (the output cursor only grows);
 *        e. ring update: R of the window's positions.
 *      tools/wparse_sim.c is the executable CPU form of this kernel, checked
 *      against the oracle.
 */
#include <stdlib.h>

#include "lzf_dev.h"

#define WP_NONE  0xFFFFFFFFu
#define WP_RNONE 0xFFFFu

/* ======================================================================== */
/* kernel 1: q1 per position (exact table, lane-ordered exchanges)          */
/* ======================================================================== */

#ifndef KQ_WIN
#define KQ_WIN 15u                 /* windows of 64 positions per block = worker waves */
#endif
#define KQ_BLK (64u * KQ_WIN)
#define KQ_THREADS (64u * (KQ_WIN + 1u))
#ifndef KQ_PF
#define KQ_PF 4u                   /* blocks of input bytes in flight per worker lane */
#endif
#ifndef KQ_XCHG
/* 1: the table step by lane-ordered exchanges; 0: plain T reads and
 * last-writer writes with the window's same-slot lanes from 16 ballots in the
 * workers (no returning atomics: 29.5 vs 14.5 ms for 64 K x 64 KiB, kept as
 * an option) */
#define KQ_XCHG 1
#endif

__device__ __forceinline__ uint32_t kq_lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

/* the block's 15 exchanges, issued in window (= position) order with one
 * wait at the end.  The LDS runs one wave's same-address ds_mskor_rtn_b32
 * in lane order (tools/lds_mskor_order.hip; checked at run time by
 * lzf_selfcheck.hip), so each lane gets the latest earlier same-slot
 * position -- the table's or an earlier lane's -- and the highest lane's
 * position is what stays; and one wave's LDS operations execute in order,
 * so the table is updated in position order.  Three asm groups of five: the
 * later groups take the earlier results as in-out operands, so nothing reads
 * a result before the single wait. */
#define KQ_X(i_) "ds_mskor_rtn_b32 %" #i_ ", %[a" #i_ "], %[m" #i_ "], %[d" #i_ "]\n\t"
#define KQ_IN(i_, o_) [a##i_] "v"(a[(o_) + i_]), [m##i_] "v"(m[(o_) + i_]), [d##i_] "v"(d[(o_) + i_])
__device__ __forceinline__ void kq_xchg15(uint32_t (&r)[15], const uint32_t (&a)[15], const uint32_t (&m)[15],
                                          const uint32_t (&d)[15])
{
    asm volatile(KQ_X(0) KQ_X(1) KQ_X(2) KQ_X(3) KQ_X(4)
                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
                 : KQ_IN(0, 0), KQ_IN(1, 0), KQ_IN(2, 0), KQ_IN(3, 0), KQ_IN(4, 0)
                 : "memory");
    asm volatile(KQ_X(0) KQ_X(1) KQ_X(2) KQ_X(3) KQ_X(4)
                 : "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]), "=&v"(r[8]), "=&v"(r[9]),
                   "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4])
                 : KQ_IN(0, 5), KQ_IN(1, 5), KQ_IN(2, 5), KQ_IN(3, 5), KQ_IN(4, 5)
                 : "memory");
    asm volatile(KQ_X(0) KQ_X(1) KQ_X(2) KQ_X(3) KQ_X(4) "s_waitcnt lgkmcnt(0)"
                 : "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]),
                   "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]),
                   "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9])
                 : KQ_IN(0, 10), KQ_IN(1, 10), KQ_IN(2, 10), KQ_IN(3, 10), KQ_IN(4, 10)
                 : "memory");
}
#undef KQ_X
#undef KQ_IN
static_assert(KQ_WIN == 15u, "kq_xchg15 issues 15 windows");

/* bytes p, p+1, p+2 (p + 3 <= n) with one 4-byte load moved back inside the
 * value near its end */
__device__ __forceinline__ uint32_t kq_tri(const uint8_t *src, uint32_t n, uint32_t p)
{
    if (n >= 4u) {
        const uint32_t at = p + 4u <= n ? p : n - 4u;
        return dv_ld4(src + at) >> (8u * (p - at));
    }
    return (uint32_t)src[p] | ((uint32_t)src[p + 1u] << 8) | ((uint32_t)src[p + 2u] << 16);
}

template <uint32_t V> struct KqIc { static constexpr uint32_t value = V; };

/* Blocks of KQ_BLK positions through a pipeline with one barrier per step:
 *   step t   A(t)    worker j: window j of block t -> slot in S[t%2]
 *   step t   B(t-1)  table wave: window by window, exchange -> q1 in O[(t-1)%2]
 *   step t   C(t-2)  worker j: cand word of window j of block t-2 -> HBM */
__global__ __launch_bounds__(KQ_THREADS) void lzf_cand_q1_kernel(LzfBatch bt, uint16_t *cand, uint64_t cstride)
{
    __shared__ __attribute__((aligned(16))) uint16_t T[LZF_SLOTS + 64u];  /* slot -> latest position, 0: none; + dummies */
    /* S: per position, KQ_XCHG: the exchange operands [T dword address |
     * half bit, data]; else [slot:16 | last of its slot in the window:1 |
     * nearest earlier same-slot lane (127: none):7].  O: its q1 */
#if KQ_XCHG
    __shared__ uint2 S[2u * KQ_BLK];
#else
    __shared__ uint32_t S[2u * KQ_BLK];
#endif
    __shared__ uint16_t O[2u * KQ_BLK];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6, j = w - 1u;
    for (uint32_t v = blockIdx.x; v < bt.count; v += gridDim.x) {
        const uint32_t n = bt.in_len[v];
        if (n < 3u || n > LZF_SLOTS || n > bt.max_len) continue;      /* uniform per workgroup */
        const uint8_t *src = bt.in + bt.in_off[v];
        uint16_t *cw = cand + (uint64_t)v * cstride;
        const uint32_t np = n - 2u;                                    /* positions 0 .. n-3 */
        const uint32_t nb = (np + KQ_BLK - 1u) / KQ_BLK;
        uint32_t pf[KQ_PF];
#pragma unroll
        for (uint32_t d = 0; d < KQ_PF; d++) {
            const uint32_t p = KQ_BLK * d + 64u * j + lane;
            pf[d] = (w && p < np) ? kq_tri(src, n, p) : 0u;
        }
        for (uint32_t k = tid; k < LZF_SLOTS / 8u; k += KQ_THREADS) ((uint4 *)T)[k] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        const auto step = [&](auto ps, uint32_t t) {
            constexpr uint32_t PS = decltype(ps)::value;                  /* t % KQ_PF */
            if (w == 0u) {
#ifdef KQ_ABL_B     /* diagnostics: no table-wave work */
                if (false) {
#else
                if (t >= 1u && t <= nb) {                                  /* B(t-1) */
#endif
                    const uint32_t k = t - 1u;
                    uint16_t *Ok = O + KQ_BLK * (k & 1u);
#if KQ_XCHG
                    const uint2 *Sk = S + KQ_BLK * (k & 1u);
                    uint32_t xa[15], xm[15], xd[15], xr[15];
                    uint2 e[15];
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++) e[i] = Sk[64u * i + lane];
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++) {
                        xa[i] = e[i].x & ~1u;
                        xm[i] = (e[i].x & 1u) ? 0xFFFF0000u : 0x0000FFFFu;
                        xd[i] = e[i].y;
                    }
                    kq_xchg15(xr, xa, xm, xd);
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++)
                        Ok[64u * i + lane] = (uint16_t)(xr[i] >> ((e[i].x & 1u) << 4));
#else
                    /* window by window: read T at the slot, then the window's
                     * last lane of each slot writes its position (the others
                     * write their lane's dummy, so no two lanes share an
                     * address); a lane with an earlier same-slot lane in its
                     * window takes that lane's position instead of T's */
                    const uint32_t B = KQ_BLK * k, *Sk = S + KQ_BLK * (k & 1u);
                    uint32_t e[15], r[15];
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++) e[i] = Sk[64u * i + lane];
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++) {
                        r[i] = T[e[i] & 0xFFFFu];
                        T[(e[i] & 0x10000u) ? (e[i] & 0xFFFFu) : LZF_SLOTS + lane] =
                            (uint16_t)(B + 64u * i + lane);
                    }
#pragma unroll
                    for (uint32_t i = 0; i < 15u; i++) {
                        const uint32_t pl = (e[i] >> 17) & 127u;
                        Ok[64u * i + lane] = (uint16_t)(pl < 64u ? B + 64u * i + pl : r[i]);
                    }
#endif
                }
            } else {
                if (t >= 2u && t - 2u < nb) {                              /* C(t-2) */
                    const uint32_t k = t - 2u;
                    const uint32_t p = KQ_BLK * k + 64u * j + lane;
                    if (p < np) {
                        const uint32_t q = O[KQ_BLK * (k & 1u) + 64u * j + lane];   /* 0: none */
                        cw[p] = (uint16_t)((q != 0u && p - q <= LZF_WINDOW) ? ((1u << 13) | (p - q - 1u)) : 0u);
                    }
                }
                if (t < nb) {                                              /* A(t) */
                    const uint32_t p = KQ_BLK * t + 64u * j + lane;
                    const bool act = p < np;
#if KQ_XCHG
                    /* a position past the value exchanges in its lane's own dummy */
                    const uint32_t h = act ? dv_slot(pf[PS]) : LZF_SLOTS + lane;
                    S[KQ_BLK * (t & 1u) + 64u * j + lane] =
                        make_uint2((kq_lds_addr(T) + 4u * (h >> 1)) | (h & 1u), (p & 0xFFFFu) << ((h & 1u) << 4));
#else
                    /* the window's same-slot lanes from 16 ballots of the slot
                     * bits: the nearest earlier one (or none), and whether
                     * this lane is its slot's last in the window */
                    const uint32_t sl = act ? dv_slot(pf[PS]) : 0u;
                    uint64_t eq = __ballot(act);
#pragma unroll
                    for (uint32_t b = 0; b < 16u; b++) {
                        const uint64_t mb = __ballot((sl >> b) & 1u);
                        eq &= ((sl >> b) & 1u) ? mb : ~mb;
                    }
                    const uint64_t lo = eq & ((1ull << lane) - 1ull), hi = eq & ~((2ull << lane) - 1ull);
                    const uint32_t pl = lo ? 63u - (uint32_t)__builtin_clzll(lo) : 127u;
                    S[KQ_BLK * (t & 1u) + 64u * j + lane] =
                        act ? (sl | (hi ? 0u : 0x10000u) | (pl << 17)) : (127u << 17);
#endif
                }
                const uint32_t lp = KQ_BLK * (t + KQ_PF) + 64u * j + lane;
#ifdef KQ_ABL_L     /* diagnostics: no input loads */
                pf[PS] = lp * 2654435761u;
#else
                pf[PS] = lp < np ? kq_tri(src, n, lp) : 0u;
#endif
            }
#ifndef KQ_ABL_S    /* diagnostics: no barrier */
            __syncthreads();
#endif
        };
        for (uint32_t t = 0; t < nb + 2u; t += KQ_PF) {
            step(KqIc<0>{}, t);
            step(KqIc<1>{}, t + 1u);
            step(KqIc<2>{}, t + 2u);
            step(KqIc<3>{}, t + 3u);
        }
    }
}
static_assert(KQ_PF == 4u, "the step loop is unrolled 4x");

/* ======================================================================== */
/* kernel 2: the window parse, one wave per value                           */
/* ======================================================================== */

__device__ __forceinline__ uint32_t wp_bperm(uint32_t v, uint32_t from)
{
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(from << 2), (int)v);
}
__device__ __forceinline__ uint32_t wp_rl(uint32_t v, uint32_t lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)lane);
}
__device__ __forceinline__ uint64_t wp_from(uint32_t i) { return i >= 64u ? 0ull : (~0ull << i); }
__device__ __forceinline__ uint64_t wp_below(uint32_t i) { return i >= 64u ? ~0ull : ((1ull << i) - 1ull); }
__device__ __forceinline__ uint32_t wp_msb(uint64_t m) { return 63u - (uint32_t)__builtin_clzll(m); }
/* popcount of m's bits below this lane */
__device__ __forceinline__ uint32_t wp_mb(uint64_t m)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ void wp_put(uint8_t *dst, uint32_t cap, uint32_t i, uint32_t b)
{
    if (i < cap) dst[i] = (uint8_t)b;
}
/* 4 bytes at p, zero past avail (never touches p + avail) */
__device__ __forceinline__ uint32_t wp_ld4_safe(const uint8_t *p, uint32_t avail)
{
    if (avail >= 4u) return dv_ld4(p);
    uint32_t v = 0u;
    for (uint32_t k = 0; k < avail; k++) v |= (uint32_t)p[k] << (8u * k);
    return v;
}

/* -DWP_TIMING (diagnostic variant, tools/wp_timing.py): cycles per phase
 * summed over waves, each phase closed by a full wait: [0] cand words and
 * links, [1] ring read, [2] byte loads and lengths, [3] scalar walk, [4]
 * wave-wide extensions, [5] emission, [6] ring update; counts: [8] windows,
 * [9] active windows, [10] stops, [11] extensions, [12] doubling rounds */
#ifdef WP_TIMING
__device__ unsigned long long wp_times[16];
extern "C" int lzf_gpu_debug_wp(unsigned long long *out16, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(wp_times), sizeof(wp_times));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(wp_times), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : -2;
}
#define WP_T0() uint64_t wp_t = (__builtin_amdgcn_s_waitcnt(0), __builtin_amdgcn_s_memtime())
#define WP_TM(i_) do { __builtin_amdgcn_s_waitcnt(0); const uint64_t t_ = __builtin_amdgcn_s_memtime(); wp_acc[i_] += t_ - wp_t; wp_t = t_; } while (0)
#define WP_CNT(i_) (wp_acc[i_]++)
#else
#define WP_T0() ((void)0)
#define WP_TM(i_) ((void)0)
#define WP_CNT(i_) ((void)0)
#endif

/* One value; every lane runs it, scalar state is wave-uniform.  Returns the
 * compressed length or 0 (src/lzf_c.c:98-294). */
__device__ uint32_t wp_value(const uint8_t *src, uint32_t n, uint8_t *dst, uint32_t cap, const uint16_t *cw,
                             uint16_t *ring)
{
    const uint32_t lane = threadIdx.x;
    const uint32_t np = n >= 3u ? n - 2u : 0u;                     /* positions 0 .. n-3, src/lzf_c.c:145 */
    uint32_t c = 0u, S = 0u, j0 = 0u;                              /* parse position, output bytes, open run % 32 */
    uint32_t t1 = WP_NONE, t2 = WP_NONE;                           /* the last match's inserted tails */
    bool ok = true, done = np == 0u;
    /* cand words in blocks of 256 positions: lane l holds positions wb + 4l .. +3 */
    const auto cblock = [&](uint32_t wb) -> uint2 {
        const uint32_t at = wb + 4u * lane;
        return at < np ? *(const uint2 *)(cw + at) : make_uint2(0u, 0u);
    };
    uint2 cb_cur = cblock(0u), cb_next = cblock(256u);
    /* the 16 bytes at each lane's position, one window ahead */
    const auto pload = [&](uint32_t pp) -> uint4 {
        return pp < np ? dv_ld16_safe(src + pp, n - pp) : make_uint4(0u, 0u, 0u, 0u);
    };
    uint4 Pn = pload(lane);
#ifdef WP_TIMING
    uint64_t wp_acc[16] = {0};
#endif
    WP_T0();
    for (uint32_t w = 0; !done && w < np; w += 64u) {
        WP_CNT(8);
        const uint32_t kb = (w >> 6) & 3u;
        if (kb == 0u && w) {
            cb_cur = cb_next;
            cb_next = cblock(w + 256u);
        }
        const uint32_t p = w + lane;
        const bool act = p < np;
        const uint4 P = Pn;
        Pn = pload(p + 64u);
        uint32_t cwv;
        {
            const uint32_t sl = 16u * kb + (lane >> 2);
            const uint32_t dx = wp_bperm(cb_cur.x, sl), dy = wp_bperm(cb_cur.y, sl);
            const uint32_t d = (lane & 2u) ? dy : dx;
            cwv = act ? ((lane & 1u) ? d >> 16 : d & 0xFFFFu) : 0u;
        }
        const uint32_t x = cwv ? p - (cwv & 0x1FFFu) - 1u : WP_NONE;
        const bool D = x != WP_NONE && x >= w;                      /* q1 inside the window */
        /* ---- a. same-slot lanes of the window and the chain's exit ------- */
        uint32_t link = D ? x - w : 64u, xo = (x != WP_NONE && !D) ? x : WP_NONE;
        uint32_t SMlo = 0u, SMhi = 0u;
        while (__ballot(link < 64u)) {
            WP_CNT(12);
            const uint32_t t = link < 64u ? link : lane;
            const uint32_t ol = wp_bperm(link, t), ox = wp_bperm(xo, t);
            const uint32_t sl = wp_bperm(SMlo, t), sh = wp_bperm(SMhi, t);
            if (link < 64u) {
                SMlo |= (link < 32u ? 1u << link : 0u) | sl;
                SMhi |= (link >= 32u ? 1u << (link - 32u) : 0u) | sh;
                xo = ox;
                link = ol;
            }
        }
        const uint64_t SM = ((uint64_t)SMhi << 32) | SMlo;
        WP_TM(0);
        uint32_t r_out = WP_NONE;
        if (xo != WP_NONE) {
            const uint32_t e = ring[xo & (LZF_WINDOW - 1u)];
            r_out = e == WP_RNONE ? WP_NONE : xo - e;
        }
        WP_TM(1);
        /* the window's inserted mask: tails of the last match */
        uint64_t INS = 0ull;
        if (t1 != WP_NONE && t1 >= w && t1 < w + 64u) INS |= 1ull << (t1 - w);
        if (t2 != WP_NONE && t2 >= w && t2 < w + 64u) INS |= 1ull << (t2 - w);
        if (c < w + 64u) {
            /* ---- b. matched lengths against the candidate refs ------------- */
            const uint32_t avail = act ? n - p : 0u;
            const bool rv = act && r_out != WP_NONE;
            const uint4 QB = rv ? dv_ld16_safe(src + r_out, n - r_out) : make_uint4(0, 0, 0, 0);
            const uint32_t ta = D ? x - w : lane;
            const uint4 QA = make_uint4(wp_bperm(P.x, ta), wp_bperm(P.y, ta), wp_bperm(P.z, ta), wp_bperm(P.w, ta));
            const uint32_t LB = rv ? min(dv_first_diff(P, QB), avail) : 0u;
            const uint32_t LA = D ? min(dv_first_diff(P, QA), avail) : 0u;
            const uint32_t Lw = np - w < 64u ? np - w : 64u;
            const uint32_t i0 = c - w;
            const uint64_t INS0 = INS;
            uint32_t maxlen = act ? n - p - 2u : 0u;                    /* src/lzf_c.c:169-170 */
            if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
            /* the 16 unrolled compares run whenever maxlen > 16 (src/lzf_c.c:181-202) */
            const uint32_t lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
            const bool okp = act && p + 4u < n;                          /* src/lzf_c.c:156 */
            /* the guess for the window's own inserted mask: every position
             * from c on; the walk's result corrects it (c5) */
            uint64_t Ig = INS0 | wp_from(i0);
            uint64_t VIS = 0ull, VS = 0ull;
            uint32_t ref = WP_NONE, mlen = 0u, nxt = 0u, kref = 0u, kmlen = 0u, knxt = 0u;
            uint32_t istart = i0, iend = Lw;
            WP_CNT(9);
            WP_TM(2);
            for (uint32_t it = 0;; it++) {
                /* ---- c1. every lane's decision as if it were visited ---------- */
                const uint64_t cm = SM & Ig;
                uint32_t l16;
                {
                    const bool inw = D && cm != 0ull;                       /* the latest inserted same-slot lane */
                    const uint32_t jl = inw ? wp_msb(cm) : lane;
                    ref = inw ? w + jl : r_out;
                    l16 = inw ? LA : LB;
                    const bool deep = inw && jl != x - w;                   /* an earlier one than x */
                    if (__ballot(deep)) {
                        const uint32_t tj = deep ? jl : lane;
                        const uint4 Q = make_uint4(wp_bperm(P.x, tj), wp_bperm(P.y, tj), wp_bperm(P.z, tj),
                                                   wp_bperm(P.w, tj));
                        if (deep) l16 = min(dv_first_diff(P, Q), avail);
                    }
                    if (ref == WP_NONE) l16 = 0u;
                }
                /* src/lzf_c.c:151-166: off < 8192, ip + 4 < in_end, ref > in_data */
                const bool match = okp && ref != WP_NONE && ref > 0u && p - ref - 1u < LZF_WINDOW && l16 >= 3u;
                /* ---- c2. lengths past 16 bytes along diagonals: if lane l+1's
                 * ref is ref + 1, the match at l is one longer than its ------ */
                const uint32_t refn = wp_bperm(ref, lane < 63u ? lane + 1u : lane);
                const uint64_t SAME = __ballot(lane < 63u && l16 == 16u && ref != WP_NONE && refn == ref + 1u);
                const uint32_t de = (uint32_t)__builtin_ctzll(~SAME & wp_from(lane));
                const uint32_t l16de = wp_bperm(l16, de);
                const uint32_t lb = (de - lane) + l16de;                    /* exact when l16de < 16 */
                const bool exact = l16de < 16u || lb >= lim;
                mlen = lb < lim ? lb : lim;
                nxt = !match ? lane + 1u : exact ? lane + mlen : (lane + lb >= 64u ? 64u + lb : 250u);
                if (lane < istart) {                                        /* the walk's part that stands */
                    ref = kref;
                    mlen = kmlen;
                    nxt = knxt;
                }
                const uint64_t STOP = __ballot(match);
                uint64_t INEX = __ballot(match && !exact);
                /* ---- c3. the scalar walk: find-first-set over the matches ---- */
                uint32_t i = istart;
                VS &= wp_below(istart);
                for (;;) {
                    const uint64_t st = STOP & (~0ull << i);
                    if (!st) {
                        iend = Lw;
                        break;
                    }
                    const uint32_t m = (uint32_t)__builtin_ctzll(st);
                    WP_CNT(10);
                    VS |= 1ull << m;
                    i = wp_rl(nxt, m);
                    if (i >= Lw) {
                        if ((INEX >> m) & 1ull) {                           /* the whole wave measures it */
                            WP_CNT(11);
                            WP_TM(3);
                            INEX &= ~(1ull << m);
                            const uint32_t pm = w + m, rm = wp_rl(ref, m), lm = wp_rl(lim, m);
                            const uint32_t k = 16u + 4u * lane;
                            const bool in = k < lm;
                            const uint32_t a = in ? wp_ld4_safe(src + pm + k, n - pm - k) : 0u;
                            const uint32_t b = in ? wp_ld4_safe(src + rm + k, n - rm - k) : 0u;
                            const uint32_t dd = a ^ b;
                            const uint64_t bad = __ballot(in && dd != 0u);
                            uint32_t e = lm;
                            if (bad) {
                                const uint32_t f = (uint32_t)__builtin_ctzll(bad);
                                const uint32_t ee = 16u + 4u * f + ((uint32_t)__builtin_ctz(wp_rl(dd, f)) >> 3);
                                e = ee < lm ? ee : lm;
                            }
                            mlen = lane == m ? e : mlen;
                            nxt = lane == m ? m + e : nxt;
                            i = m + e;
                            WP_TM(4);
                            if (i < Lw) continue;
                        }
                        iend = i;
                        break;
                    }
                }
                /* ---- c4. visited lanes and the window's inserted mask -------- */
                const uint64_t vb = VS & wp_below(lane + 1u);
                const uint32_t lv = vb ? wp_msb(vb) : lane;
                const uint32_t e = wp_bperm(nxt, lv);
                const bool vis = act && lane >= i0 && (!vb || lane == lv || lane >= e);
                const bool tail = act && !vis && vb && w + e < np && (lane + 2u == e || lane + 1u == e);
                VIS = __ballot(vis);
                const uint64_t In = (INS0 & wp_below(i0)) | VIS | __ballot(tail);
                /* ---- c5. a visited lane whose in-window ref the guess got wrong
                 * restarts the walk there (everything before it stands) -------- */
                const uint64_t ca = SM & In;
                const bool bad = vis && D && (cm ? wp_msb(cm) : 64u) != (ca ? wp_msb(ca) : 64u);
                const uint64_t B = __ballot(bad);
                if (!B || it >= 64u) {
                    INS = In;
                    break;
                }
                istart = (uint32_t)__builtin_ctzll(B);
                Ig = In;
                kref = ref;
                kmlen = mlen;
                knxt = nxt;
            }
            const uint64_t MS = VS;
            const uint32_t toklen = mlen, tokoff = p - ref - 1u;
            c = w + iend;
            t1 = t2 = WP_NONE;
            if (c >= np) {
                done = true;                                                /* src/lzf_c.c:229 */
            } else if (MS && wp_rl(nxt, wp_msb(MS)) == iend) {
                t1 = c - 2u;                                                /* the last match's tails */
                t2 = c - 1u;
            }
            WP_TM(3);
            /* ---- d. emission ------------------------------------------------ */
            {
                const uint64_t LM = VIS & ~MS, below = wp_below(lane);
                const bool vis = (VIS >> lane) & 1ull, ism = (MS >> lane) & 1ull;
                const uint64_t pmb = MS & below;
                uint32_t rp;
                if (pmb) {
                    const uint32_t lm = wp_msb(pmb);
                    rp = wp_mb(LM) - (uint32_t)__builtin_popcountll(LM & wp_below(lm + 1u));
                } else {
                    rp = j0 + wp_mb(LM);
                }
                const uint32_t jj = rp & 31u;
                const uint32_t size = !vis ? 0u : ism ? (toklen - 2u < 7u ? 2u : 3u) : (jj == 0u ? 2u : 1u);
                const uint64_t B0 = __ballot(size & 1u), B1 = __ballot(size & 2u);
                const uint32_t off = S + wp_mb(B0) + 2u * wp_mb(B1);
                bool fail = false;
                if (vis) {
                    if (ism) {
                        if (jj) wp_put(dst, cap, off - jj - 1u, jj - 1u);   /* close the run */
                        fail = off + 4u >= cap;                             /* src/lzf_c.c:176 */
                        const uint32_t L = toklen - 2u, of = tokoff;
                        if (L < 7u) {
                            wp_put(dst, cap, off, (of >> 8) | (L << 5));
                            wp_put(dst, cap, off + 1u, of);
                        } else {
                            wp_put(dst, cap, off, (of >> 8) | (7u << 5));
                            wp_put(dst, cap, off + 1u, L - 7u);
                            wp_put(dst, cap, off + 2u, of);
                        }
                    } else {
                        const uint32_t bi = off + (jj == 0u ? 1u : 0u);
                        fail = bi >= cap;                                    /* src/lzf_c.c:263 */
                        wp_put(dst, cap, bi, P.x & 0xFFu);
                        if (jj == 31u) wp_put(dst, cap, bi - 32u, 31u);       /* rollover, src/lzf_c.c:268-272 */
                    }
                }
                if (__ballot(fail)) {
                    ok = false;
                    break;
                }
                S += (uint32_t)__builtin_popcountll(B0) + 2u * (uint32_t)__builtin_popcountll(B1);
                j0 = MS ? ((uint32_t)__builtin_popcountll(LM & wp_from(wp_msb(MS) + 1u)) & 31u)
                        : ((j0 + (uint32_t)__builtin_popcountll(LM)) & 31u);
            }
            WP_TM(5);
        }
        if (done) break;
        /* ---- e. ring update ------------------------------------------------- */
        {
            const uint64_t deeper = SM & INS;
            const uint32_t ref = deeper ? w + wp_msb(deeper) : r_out;
            const uint32_t e = ((INS >> lane) & 1ull) ? 0u
                               : (ref == WP_NONE || ref == 0u || p - ref >= LZF_WINDOW) ? WP_RNONE
                                                                                     : p - ref;
            __asm__ volatile("" ::: "memory");
            if (act) ring[p & (LZF_WINDOW - 1u)] = (uint16_t)e;
            __asm__ volatile("" ::: "memory");
        }
        WP_TM(6);
    }
#ifdef WP_TIMING
    if (lane == 0u)
        for (uint32_t k = 0; k < 16u; k++) atomicAdd(&wp_times[k], (unsigned long long)wp_acc[k]);
#endif
    if (!ok) return 0u;
    if (S + (j0 == 0u ? 1u : 0u) + 3u > cap) return 0u;               /* src/lzf_c.c:276 */
    if (lane == 0u) {
        for (uint32_t q = c; q < n; q++) {                             /* src/lzf_c.c:279-288 */
            const uint32_t bi = S + (j0 == 0u ? 1u : 0u);
            dst[bi] = src[q];
            S = bi + 1u;
            j0 = (j0 + 1u) & 31u;
            if (j0 == 0u) dst[S - 33u] = 31u;
        }
        if (j0) dst[S - j0 - 1u] = (uint8_t)(j0 - 1u);                 /* src/lzf_c.c:290-291 */
    }
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)S);
}

__global__ __launch_bounds__(64) void lzf_wparse_kernel(LzfBatch bt, const uint16_t *cand, uint64_t cstride)
{
    __shared__ uint16_t ring[LZF_WINDOW];
    for (uint32_t v = blockIdx.x; v < bt.count; v += gridDim.x) {
        const uint32_t n = bt.in_len[v], cap = bt.out_cap[v];
        uint32_t r = 0u;
        if (n != 0u && cap != 0u && n <= LZF_SLOTS && n <= bt.max_len)   /* src/lzf_c.c:131; past max_len: refused */
            r = wp_value(bt.in + bt.in_off[v], n, bt.out + bt.out_off[v], cap, cand + (uint64_t)v * cstride, ring);
        if (threadIdx.x == 0u) bt.out_len[v] = r;
    }
}

/* ---- launcher ------------------------------------------------------------ */

/* cand words per value: whole 256-position blocks plus one of slack */
static uint64_t wp_cstride(uint32_t max_len) { return (((uint64_t)max_len + 255u) & ~255ull) + 256u; }

size_t lzf_wtab_scratch_per_value(uint32_t max_len) { return (size_t)(wp_cstride(max_len) * 2u); }

bool lzf_wtab_compress_supported(uint32_t max_len) { return max_len <= LZF_SLOTS; }

hipError_t lzf_launch_compress_wtab(const LzfBatch &b, hipStream_t s, void *scratch, size_t scratch_bytes,
                                    uint32_t *chunks)
{
    if (b.max_len > LZF_SLOTS) return hipErrorInvalidValue;
    const uint64_t cstride = wp_cstride(b.max_len);
    uint64_t chunk = scratch_bytes / (cstride * 2u);
    if (chunk > b.count) chunk = b.count;
    if (chunk == 0) return hipErrorInvalidValue;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    /* diagnostics: LZF_GPU_TABLE_STAGE=1 runs kernel 1 only (its own time) */
    const char *stg = getenv("LZF_GPU_TABLE_STAGE");
    const bool cand_only = stg && *stg == '1';
    const char *wpb = getenv("LZF_GPU_WPARSE_PER_CU");              /* residency override */
    uint32_t per_cu = wpb && atoi(wpb) > 0 ? (uint32_t)atoi(wpb) : 9u;   /* 16 KiB ring each: 9 resident per CU (10 measured as two generations) */
    hipError_t e;
    uint32_t nch = 0;
    for (uint64_t first = 0; first < b.count; first += chunk, nch++) {
        const uint32_t cnt = (uint32_t)((b.count - first) < chunk ? (b.count - first) : chunk);
        LzfBatch c = b;
        c.in_off = b.in_off + first;
        c.in_len = b.in_len + first;
        c.out_off = b.out_off + first;
        c.out_cap = b.out_cap + first;
        c.out_len = b.out_len + first;
        c.count = cnt;
        const uint32_t g1 = cnt < (uint32_t)cus ? cnt : (uint32_t)cus;
        hipLaunchKernelGGL(lzf_cand_q1_kernel, dim3(g1), dim3(KQ_THREADS), 0, s, c, (uint16_t *)scratch, cstride);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        if (cand_only) continue;
        const uint32_t g2 = cnt < (uint32_t)cus * per_cu ? cnt : (uint32_t)cus * per_cu;
        hipLaunchKernelGGL(lzf_wparse_kernel, dim3(g2), dim3(64), 0, s, c, (const uint16_t *)scratch, cstride);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    if (chunks) *chunks = nch;
    return hipSuccess;
}

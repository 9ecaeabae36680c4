/*
 * lzf_cand.hip -- the "table" generation of the LZF compressor for gfx950
 * (values of at most 64 KiB; larger values go to window64, lzf_compress.hip).
 *
 * The reference's greedy parse (src/lzf_c.c:145-274) is serial per value and
 * its ref at a visited position p is the latest INSERTED position with p's
 * 16-bit slot (src/lzf_c.c:147-149).  Inserted = every visited position plus
 * the last two positions of each match (src/lzf_c.c:227-247); so the ref is
 * the first position on the "same-slot chain" of p (p's nearest earlier
 * same-slot position q1(p), then q1(q1(p)), ...) that the parse did not skip.
 * Two kernels per batch:
 *
 *   1. lzf_cand_table_kernel -- position-parallel, one value at a time per
 *      workgroup of 16 waves (one workgroup per CU: the table is 128 KiB of
 *      LDS).  For every position p: q1(p) and q2(p) = q1(q1(p)), each with
 *      how far its bytes agree with p's (<= 8), packed in a u32 record in
 *      HBM scratch.  q1 comes from an exact direct-mapped table T[slot] ->
 *      latest position (65536 x u16, the reference's own table size,
 *      src/lzfP.h:55), so there are no bucket chains to walk on any data; q2
 *      from a ring Q of q1 over the last 8192 positions (a candidate farther
 *      back is outside every window, src/lzf_c.c:153).  Blocks of 15
 *      windows of 64 positions run through a pipeline (kt_value below):
 *        A  worker wave j takes window j: bytes and slot;
 *        B  the table wave exchanges each window's positions into T, window
 *           by window: ds_mskor_rtn_b32 replaces the slot's 16-bit half and
 *           returns the old dword, and the LDS runs a wave's same-address
 *           operations in lane order, so each lane gets the latest earlier
 *           same-slot position -- the table's or an earlier lane's -- and one
 *           wave's LDS operations execute in order, so T is updated in
 *           position order without cross-wave ordering;
 *        C  each worker takes its window again: q1, q2, agreement, record.
 *
 *   2. lzf_parse_rec_kernel -- the greedy parse and emission, ONE LANE PER
 *      VALUE (a wave advances 64 values at once).  It keeps an inserted-
 *      bitmap of its value (32 words in LDS, older words in HBM scratch) and
 *      walks the chain only past skipped positions.  A record holds two
 *      chain links, so a walk loads one record per two skipped candidates.
 *
 * Scratch per value: 4 B/position (records) + 1 bit/position (bitmap).
 */
#include <stdlib.h>
#include <string.h>

#include "lzf_dev.h"

/* record of position p: bits 0-12 off1 = p - q1 - 1, 13-15 code1,
 * bits 16-28 off2 = p - q2 - 1, 29-31 code2.  Codes:
 *   0     none (no earlier position with p's slot inside p's window, or only
 *         position 0, which is never a ref: src/lzf_c.c:155 `ref > in_data`)
 *   1     same slot, the three bytes differ (slot collision)
 *   2..6  the bytes agree for exactly code + 1 bytes (3..7)
 *   7     the bytes agree for >= 8 bytes                                   */
#define RC_DIFF 1u
#define RC_LONG 7u

#ifndef KT_WIN
#define KT_WIN 15u                /* windows of 64 positions per block = worker waves: 15 + the table wave = 4 per SIMD */
#endif
#define KT_BLK (64u * KT_WIN)
#define KT_THREADS (64u * (KT_WIN + 1u))
#ifndef KT_PF
#define KT_PF 4u                /* blocks of input bytes in flight per lane */
#endif
#ifndef KT_CL
#define KT_CL 2u                /* steps from C1 (agreement loads issued) to C2 (consumed); divides KT_PF */
#endif

/* v_ffbl_b32: the lowest set bit's index, 0xFFFFFFFF for 0 (defined here,
 * unlike __builtin_ctz) */
__device__ __forceinline__ uint32_t kt_ffbl(uint32_t x)
{
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
__device__ __forceinline__ uint32_t kt_code(uint32_t k)
{
    return k < 3u ? RC_DIFF : (k >= 8u ? RC_LONG : k - 1u);
}


static_assert(KT_WIN % 5u == 0u, "the exchanges go in groups of 5 windows");
/* LDS byte address of a __shared__ object */
__device__ __forceinline__ uint32_t kt_lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}
/* five windows' exchanges, issued in window (= position) order, then one
 * wait: the LDS writes the results after issue, so they are outputs of the
 * same asm statement (early-clobber: no result shares an input's register)
 * and nothing reads them before the wait.  Groups of five keep the table
 * wave's live registers inside the workers' budget (15 at once spills) */
#define KT_X(i_) "ds_mskor_rtn_b32 %" #i_ ", %[a" #i_ "], %[m" #i_ "], %[d" #i_ "]\n\t"
#define KT_IN(i_) [a##i_] "v"(a[i_]), [m##i_] "v"(m[i_]), [d##i_] "v"(d[i_])
__device__ __forceinline__ void kt_xchg5(uint32_t (&r)[5], const uint32_t (&a)[5], const uint32_t (&m)[5],
                                         const uint32_t (&d)[5])
{
    asm volatile(KT_X(0) KT_X(1) KT_X(2) KT_X(3) KT_X(4) "s_waitcnt lgkmcnt(0)"
                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
                 : KT_IN(0), KT_IN(1), KT_IN(2), KT_IN(3), KT_IN(4)
                 : "memory");
}
#undef KT_X
#undef KT_IN
/* S entry of a position of the block: its slot and whether it is active */
#define KS_ACT  (1u << 16)

/* the 8 bytes at pp: one branch-free 8-byte load for values of >= 8 bytes
 * (the compiler then counts the loads in flight instead of draining them) */
template <bool SMALL>
__device__ __forceinline__ uint2 kt_ld8(const uint8_t *src, uint32_t n, uint32_t pp)
{
    if constexpr (SMALL) return pp < n ? dv_ld8_safe(src + pp, n - pp) : make_uint2(0u, 0u);
    else return dv_ld8_clamped(src, n, pp);
}

/* how far the bytes at q agree with p's 8 bytes a (at most 8, at most
 * avail = n - p); q < p */
template <bool SMALL>
__device__ __forceinline__ uint32_t kt_agree(uint2 a, const uint8_t *src, uint32_t n, uint32_t q,
                                             uint32_t avail)
{
    const uint2 b = kt_ld8<SMALL>(src, n, q);
    const uint64_t x = ((uint64_t)(a.y ^ b.y) << 32) | (uint64_t)(a.x ^ b.x);
    const uint32_t k = x ? (uint32_t)__builtin_ctzll(x) >> 3 : 8u;
    return k < avail ? k : avail;
}

/* Pipelined over blocks of KT_BLK = KT_WIN windows (960 positions): wave 0 is
 * the table wave, waves 1..KT_WIN are workers (16 waves: 4 per SIMD), and
 * each step ends with ONE workgroup barrier.  Block k goes through
 *   step k         A(k)   worker j: window j -- bytes, slot -> S[k%2]
 *   step k+1       B(k)   table wave: exchanges of the windows in order -> O[k%3]
 *   step k+2       C1(k)  worker j: q1, q2 (O[k%3], O[(k-1)%3], Q); agreement loads issued
 *   step k+3       Q <- O[k%3]
 *   step k+2+KT_CL C2(k)  worker j: agreement, record stored
 * Q(k) is written in step k+3: the slots it overwrites belong to positions
 * 8192 before block k, which no C1 of block k+1 or later can reach
 * (off < 8192).  The kernel is bound by chains of dependent LDS round trips
 * and the per-step barrier. */
/* -DKT_TIMING (diagnostic build): cycles per phase, summed over waves in
 * kt_times[]: [0] table wave B, [1] table wave barrier, [2] C2, [3] C1,
 * [4] A, [5] worker loads, [6] worker barrier, [7] steps */
#ifdef KT_TIMING
__device__ unsigned long long kt_times[16];
extern "C" int lzf_gpu_debug_kt(unsigned long long *out16, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(kt_times), sizeof(kt_times));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(kt_times), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : -2;
}
#define KT_T0() uint64_t kt_t = __builtin_amdgcn_s_memtime()
#ifdef KT_LITE
/* -DKT_LITE: each wave's busy cycles per step (step start to the barrier),
 * written to kt_trace for the first KT_LW workgroups and KT_LS steps; no
 * per-phase sums (the per-phase form spills ~95 VGPRs and runs the kernel
 * ~3.5x slower, which skews its phase figures) */
#define KT_LW 64u
#define KT_LS 4096u
__device__ uint32_t kt_trace[KT_LW * KT_LS * 16u];
extern "C" int lzf_gpu_debug_kt_trace(uint32_t *out)
{
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(kt_trace), sizeof(kt_trace)) == hipSuccess ? 0 : -2;
}
#define KT_TM(i) ((void)0)
#else
#define KT_TM(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); kt_loc[i] += t_ - kt_t; kt_t = t_; } while (0)
#endif
#else
#define KT_T0() ((void)0)
#define KT_TM(i) ((void)0)
#endif

struct KtLds {
    uint16_t *T, *Q, *O;                 /* O: 3 buffers of KT_BLK */
    uint32_t *S;                         /* S: 2 buffers of KT_BLK */
};

template <uint32_t V> struct KtIc { static constexpr uint32_t value = V; };
/* KT_INTERIOR (round 5): the main loop's steps with their block and position
 * tests dropped (they hold there); the first KT_PF steps keep them */
#ifndef KT_INTERIOR
#define KT_INTERIOR 1
#endif
/* KT_SPRE (round 5): workers store the table wave's exchange address */
#ifndef KT_SPRE
#define KT_SPRE 1
#endif
/* round 5: C2's agreements without 64-bit compares, C1's q2 index by selects */
#ifndef KT_AGREE2
#define KT_AGREE2 1
#endif
#ifndef KT_IQSEL
#define KT_IQSEL 1
#endif

#ifdef KT_TIMING
#define KT_ACC_ARG , uint64_t *kt_acc, uint32_t *kt_busy
#define KT_ACC_PASS , kt_acc, kt_busy
#else
#define KT_ACC_ARG
#define KT_ACC_PASS
#endif
template <bool SMALL>
__device__ __forceinline__ void kt_value(const KtLds &L, const uint8_t *src, uint32_t n, uint32_t *rec KT_ACC_ARG)
{
    uint16_t *const T = L.T, *const Q = L.Q, *const O = L.O;
    uint32_t *const S = L.S;
#ifdef KT_WREV
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = KT_WIN - (tid >> 6);   /* experiment: table wave last */
#else
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
#endif
#ifdef KT_JREV
    const uint32_t j = KT_WIN - w;                             /* experiment: windows in reverse wave order */
#else
    const uint32_t j = w - 1u;                                 /* worker's window (w >= 1) */
#endif
    const uint32_t np = n - 2u;                                /* positions 0 .. n-3, src/lzf_c.c:145 */
    const uint32_t nb = (np + KT_BLK - 1u) / KT_BLK;
    /* worker: the 8 bytes of its position in the next KT_PF blocks are in
     * flight; slot d holds the blocks = d (mod KT_PF), so the step loop is
     * unrolled KT_PF times and no register rotates (a rotation would copy a
     * register whose load is in flight, i.e. wait for it) */
    uint2 pf[KT_PF], ak[KT_PF];
#pragma unroll
    for (uint32_t d = 0; d < KT_PF; d++) {
        pf[d] = make_uint2(0u, 0u);
        ak[d] = make_uint2(0u, 0u);
    }
    if (w) {
        if (!SMALL && KT_BLK * KT_PF + 8u <= n) {                /* the first blocks need no clamp */
#pragma unroll
            for (uint32_t d = 0; d < KT_PF; d++) pf[d] = dv_ld8(src + KT_BLK * d + 64u * j + lane);
        } else {
#pragma unroll
            for (uint32_t d = 0; d < KT_PF; d++) pf[d] = kt_ld8<SMALL>(src, n, KT_BLK * d + 64u * j + lane);
        }
    }
    /* the table starts empty for every value (position 0 = none: it is
     * never a ref, and a candidate 0 decides like no candidate) */
    for (uint32_t k = tid; k < LZF_SLOTS / 8u; k += KT_THREADS) ((uint4 *)T)[k] = make_uint4(0, 0, 0, 0);
    __syncthreads();
    /* C1 -> C2 state of the worker's window: KT_CL sets, so the agreement
     * loads C1 issues are consumed KT_CL steps later (one step of slack puts
     * a load latency on every step's critical path) */
    uint32_t c_p[KT_CL], c_q1[KT_CL], c_q2[KT_CL], c_avail[KT_CL];
    uint2 c_a[KT_CL], c_b1[KT_CL], c_b2[KT_CL];
#pragma unroll
    for (uint32_t i = 0; i < KT_CL; i++) {
        c_p[i] = 0xFFFFFFFFu;
        c_q1[i] = c_q2[i] = c_avail[i] = 0u;
        c_a[i] = c_b1[i] = c_b2[i] = make_uint2(0u, 0u);
    }
#ifdef KT_TIMING
    uint64_t kt_loc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    /* m3 = t % 3 (the O buffer of block t), kept by the caller: the three
     * k % 3 of a step are selects of it, not three scalar divisions */
    const auto step = [&](auto ps, auto clamp, uint32_t t, uint32_t m3) {
        constexpr uint32_t PS = decltype(ps)::value;             /* t % KT_PF */
        constexpr uint32_t CS = PS % KT_CL;                      /* C1 -> C2 set of this step */
        /* CLAMP: the step's loads may reach past the value (its last
         * blocks); otherwise they are plain 8-byte loads */
        constexpr bool CLAMP = SMALL || decltype(clamp)::value == 1u;
        /* INTERIOR (clamp 2, KT_INTERIOR): t >= KT_PF and blocks t-3 .. t +
         * KT_PF + 3 lie inside the value, so every block and position test
         * of the step holds; they are dropped (no exec-mask branches) */
        constexpr bool INTERIOR = !SMALL && decltype(clamp)::value == 2u;
        const uint32_t m3_1 = m3 == 0u ? 2u : m3 - 1u;          /* (t - 1) % 3 */
        const uint32_t m3_2 = m3 == 2u ? 0u : m3 + 1u;          /* (t - 2) % 3 */
        const auto ld8 = [&](uint32_t pp) { return CLAMP ? kt_ld8<SMALL>(src, n, pp) : dv_ld8(src + pp); };
        KT_T0();
#ifdef KT_TIMING
        const uint64_t kt_s = kt_t;
#endif
        /* this step's global loads are issued unconditionally, by every
         * wave, at the end: a load inside a branch leaves a register merge
         * behind that waits for it */
        uint32_t l1 = 0u, l2 = 0u;                               /* agreement loads of C1 */
        const uint32_t lp = KT_BLK * (t + KT_PF) + 64u * j + lane;   /* input of block t + KT_PF */
        if (w == 0u) {
            /* ---- B(t-1): the table wave ------------------------------------- */
            /* one lane-ordered exchange per window, in window (= position)
             * order, five windows per asm group; no exec masking */
            if (INTERIOR || (t >= 1u && t <= nb)) {
                const uint32_t k = t - 1u, B = KT_BLK * k;
                const uint32_t *Sk = S + KT_BLK * (k & 1u);
                uint16_t *Ok = O + KT_BLK * m3_1;
                /* a position past the value exchanges in its lane's own
                 * dummy half (T[65536 + lane]) */
                const uint32_t tb = kt_lds_addr(T);
#pragma unroll
                for (uint32_t g = 0; g < KT_WIN; g += 5u) {
                    uint32_t xa[5], xm[5], xd[5], xr[5], xs[5];
#pragma unroll
                    for (uint32_t u = 0; u < 5u; u++) {
                        const uint32_t i = g + u;
                        const uint32_t e = Sk[64u * i + lane];
#if KT_SPRE
                        /* the worker stored the exchange's dword address and
                         * the slot's half (bit 0) */
                        (void)tb;
                        xs[u] = (e & 1u) << 4;
                        xa[u] = e & ~3u;
#else
                        const uint32_t h = (e & KS_ACT) ? (e & 0xFFFFu) : LZF_SLOTS + lane;
                        xs[u] = (h & 1u) << 4;
                        xa[u] = tb + 4u * (h >> 1);
#endif
                        xm[u] = 0xFFFFu << xs[u];
                        xd[u] = (((B + 64u * i) & 0xFFFFu) | lane) << xs[u];   /* B + 64 i: a multiple of 64 */
                    }
                    kt_xchg5(xr, xa, xm, xd);
#pragma unroll
                    for (uint32_t u = 0; u < 5u; u++) Ok[64u * (g + u) + lane] = (uint16_t)(xr[u] >> xs[u]);
                }
            }
        } else {
            /* ---- C2(t-2-KT_CL): agreement and record ------------------------ */
            if (INTERIOR || c_p[CS] < np) {
                const uint32_t cp = c_p[CS], cq1 = c_q1[CS], cq2 = c_q2[CS], cav = c_avail[CS];
                const uint2 ca = c_a[CS], cb1 = c_b1[CS], cb2 = c_b2[CS];
                /* branch-free: both agreements always, the record by selects */
                const uint64_t x1 = ((uint64_t)(ca.y ^ cb1.y) << 32) | (uint64_t)(ca.x ^ cb1.x);
                const uint64_t x2 = ((uint64_t)(ca.y ^ cb2.y) << 32) | (uint64_t)(ca.x ^ cb2.x);
#if KT_AGREE2
                /* first differing byte of 8 (8: none), without the 64-bit compare
                 * and select: v_ffbl gives the lowest set bit or ~0 for none, so
                 * min3(ffbl(lo), ffbl(hi) | 32, 64) is the first differing bit */
                const uint32_t k1 = min(min(min(kt_ffbl((uint32_t)x1), kt_ffbl((uint32_t)(x1 >> 32)) | 32u), 64u) >> 3, cav);
                const uint32_t k2 = min(min(min(kt_ffbl((uint32_t)x2), kt_ffbl((uint32_t)(x2 >> 32)) | 32u), 64u) >> 3, cav);
#else
                const uint32_t k1 = min(x1 ? (uint32_t)__builtin_ctzll(x1) >> 3 : 8u, cav);
                const uint32_t k2 = min(x2 ? (uint32_t)__builtin_ctzll(x2) >> 3 : 8u, cav);
#endif
                const uint32_t r1 = (cp - cq1 - 1u) | (kt_code(k1) << 13);
                const uint32_t r2 = ((cp - cq2 - 1u) | (kt_code(k2) << 13)) << 16;
                rec[cp] = cq1 ? (r1 | (cq2 ? r2 : 0u)) : 0u;
            }
            /* ---- Q <- O of block t-3 ---------------------------------------- */
            if (INTERIOR || (t >= 3u && t - 3u < nb)) {
                const uint32_t k = t - 3u;
                const uint32_t x = KT_BLK * k + 64u * j + lane;
                if (INTERIOR || x < np) Q[x & (LZF_WINDOW - 1u)] = O[KT_BLK * m3 + 64u * j + lane];
            }
            KT_TM(2);
            /* ---- C1(t-2): q1, q2; their agreement loads below ---------------- */
            c_p[CS] = 0xFFFFFFFFu;
            c_q1[CS] = c_q2[CS] = 0u;
            if (INTERIOR || (t >= 2u && t - 2u < nb)) {
                const uint32_t k = t - 2u, B = KT_BLK * k;
                const uint32_t p = B + 64u * j + lane;
                /* branch-free: the Q..O read at a clamped index for every lane,
                 * validity by selects */
                const bool act = INTERIOR || p < np;
                const uint16_t *Ok = O + KT_BLK * m3_2;
                const uint32_t q1r = Ok[64u * j + lane];
                const uint32_t q1 = act && p - q1r <= LZF_WINDOW ? q1r : 0u;   /* q1r = 0: none */
                const uint32_t ik = LZF_WINDOW + KT_BLK * m3_2, ip = LZF_WINDOW + KT_BLK * m3;   /* (k + 2) % 3 = t % 3 */
#if KT_IQSEL
                /* all three indices, then selects (the nested ternary compiled to
                 * exec-mask branches: ~20 SALU per step) */
                const uint32_t iq0 = ik + (q1 - B), iq1 = ip + (q1 + KT_BLK - B), iq2 = q1 & (LZF_WINDOW - 1u);
                const uint32_t iq01 = q1 + KT_BLK >= B ? iq1 : iq2;
                const uint32_t iq = q1 >= B ? iq0 : iq01;
#else
                const uint32_t iq = q1 >= B ? ik + (q1 - B)
                                  : q1 + KT_BLK >= B ? ip + (q1 + KT_BLK - B)
                                                     : (q1 & (LZF_WINDOW - 1u));
#endif
                const uint32_t q2r = Q[iq];
                const uint32_t q2 = q1 && q2r != 0u && p - q2r <= LZF_WINDOW ? q2r : 0u;
                c_p[CS] = act ? p : 0xFFFFFFFFu;
                c_avail[CS] = n - p;
                c_a[CS] = ak[(PS + KT_PF - 2u) % KT_PF];              /* A's bytes of block t-2 */
                c_q1[CS] = l1 = q1;
                c_q2[CS] = l2 = q2;
            }
            KT_TM(3);
            /* ---- A(t): the worker's window of block t ----------------------- */
            if (INTERIOR || t < nb) {
                const uint32_t p = KT_BLK * t + 64u * j + lane;
                const bool act = INTERIOR || p < np;
                const uint2 a = pf[PS];
                ak[PS] = a;
                const uint32_t s = dv_slot(a.x);
#if KT_SPRE
                {
                    /* the table wave's exchange address (T's dword of the slot,
                     * or the lane's dummy past the value) and half, so it does
                     * not compute them: it shares its SIMD with three workers
                     * and sets the step's pace there (tools/kt_trace.py) */
                    const uint32_t h = act ? s : LZF_SLOTS + lane;
                    S[KT_BLK * (t & 1u) + 64u * j + lane] = kt_lds_addr(T) + 4u * (h >> 1) + (h & 1u);
                }
#else
                S[KT_BLK * (t & 1u) + 64u * j + lane] = act ? (s | KS_ACT) : 0u;
#endif
            }
        }
        if (w) KT_TM(4);
        else KT_TM(0);
        /* the step's loads: agreement bytes of C1 first, then the input of
         * block t + KT_PF, so a wait for the former never waits for it */
        c_b1[CS] = ld8(l1);
        c_b2[CS] = ld8(l2);
        pf[PS] = ld8(lp);
        if (w) KT_TM(5);
#if defined(KT_TIMING) && defined(KT_LITE)
        if (lane == 0u && blockIdx.x < KT_LW && kt_loc[7] < KT_LS)
            kt_trace[(blockIdx.x * KT_LS + (uint32_t)kt_loc[7]) * 16u + w] =
                (uint32_t)(__builtin_amdgcn_s_memtime() - kt_s);
#elif defined(KT_TIMING)
        /* each wave's busy cycles this step; after the barrier the table wave
         * sums the slowest worker's (kt_acc[8]) and the mean worker's (9) */
        if (lane == 0u) kt_busy[16u * (t & 1u) + w] = (uint32_t)(kt_t - kt_s);
#endif
        __syncthreads();
        if (w) KT_TM(6);
        else KT_TM(1);
#ifdef KT_TIMING
        kt_loc[7]++;
#ifndef KT_LITE
        if (w == 0u && lane == 0u) {
            uint32_t mx = 0u, sm = 0u;
            for (uint32_t i = 1; i <= KT_WIN; i++) {
                const uint32_t b = kt_busy[16u * (t & 1u) + i];
                mx = b > mx ? b : mx;
                sm += b;
            }
            kt_loc[8] += mx;
            kt_loc[9] += sm / KT_WIN;
        }
#endif
#endif
    };
    /* steps whose loads all stay inside the value -- the input of block
     * t + KT_PF and agreement bytes of positions before block t - 1 -- skip
     * the end-of-value clamp (the last group of steps keeps it) */
    uint32_t t = 0, m3 = 0;                                    /* m3 = t % 3 */
    const auto next3 = [](uint32_t x) { return x == 2u ? 0u : x + 1u; };
    if (!SMALL) {
        if (KT_INTERIOR && KT_BLK * (KT_PF + 3u + KT_PF + 1u) + 8u <= n) {
            /* the first KT_PF steps test their blocks (t - 3 < 0 ...) */
            step(KtIc<0>{}, KtIc<0>{}, 0u, 0u);
            step(KtIc<1>{}, KtIc<0>{}, 1u, 1u);
            step(KtIc<2>{}, KtIc<0>{}, 2u, 2u);
            step(KtIc<3>{}, KtIc<0>{}, 3u, 0u);
            t = KT_PF;
            m3 = KT_PF % 3u;
            for (; t < nb + 2u + KT_CL && KT_BLK * (t + 3u + KT_PF + 1u) + 8u <= n; t += KT_PF) {
                step(KtIc<0>{}, KtIc<2>{}, t, m3);
                m3 = next3(m3);
                step(KtIc<1>{}, KtIc<2>{}, t + 1u, m3);
                m3 = next3(m3);
                step(KtIc<2>{}, KtIc<2>{}, t + 2u, m3);
                m3 = next3(m3);
                step(KtIc<3>{}, KtIc<2>{}, t + 3u, m3);
                m3 = next3(m3);
            }
        }
        for (; t < nb + 2u + KT_CL && KT_BLK * (t + 3u + KT_PF + 1u) + 8u <= n; t += KT_PF) {
            step(KtIc<0>{}, KtIc<0>{}, t, m3);
            m3 = next3(m3);
            step(KtIc<1>{}, KtIc<0>{}, t + 1u, m3);
            m3 = next3(m3);
            step(KtIc<2>{}, KtIc<0>{}, t + 2u, m3);
            m3 = next3(m3);
            step(KtIc<3>{}, KtIc<0>{}, t + 3u, m3);
            m3 = next3(m3);
        }
    }
    /* (a per-step tail, to run no empty steps past the last, measured
     * slower: its switch costs more than the steps it saves) */
    for (; t < nb + 2u + KT_CL; t += KT_PF) {
        step(KtIc<0>{}, KtIc<1>{}, t, m3);
        m3 = next3(m3);
        step(KtIc<1>{}, KtIc<1>{}, t + 1u, m3);
        m3 = next3(m3);
        step(KtIc<2>{}, KtIc<1>{}, t + 2u, m3);
        m3 = next3(m3);
        step(KtIc<3>{}, KtIc<1>{}, t + 3u, m3);
        m3 = next3(m3);
    }
#ifdef KT_TIMING
#pragma unroll
    for (uint32_t i = 0; i < 10u; i++) kt_acc[i] += kt_loc[i];
#endif
}

__global__ __launch_bounds__(KT_THREADS) void lzf_cand_table_kernel(LzfBatch bt, LzfRecScratch sc)
{
    __shared__ __attribute__((aligned(16))) uint16_t T[LZF_SLOTS + 64u];  /* slot -> latest position, 0: none; + dummies */
    /* Q: q1 of position x at x % 8192; O (right behind it, one array, so a
     * q2 lookup is one read at a selected index): q1 of the blocks' positions */
    __shared__ uint16_t QO[LZF_WINDOW + 3u * KT_BLK];
    uint16_t *const Q = QO, *const O = QO + LZF_WINDOW;
    __shared__ uint32_t S[2u * KT_BLK];
    const KtLds L{T, Q, O, S};
#ifdef KT_PMAP
    {
        /* per-wave issue priority, 2 bits per wave index (experiment) */
        const uint32_t pw = (uint32_t)((KT_PMAP >> (4u * (threadIdx.x >> 6))) & 3u);
        if (pw == 1u) __builtin_amdgcn_s_setprio(1);
        else if (pw == 2u) __builtin_amdgcn_s_setprio(2);
        else if (pw == 3u) __builtin_amdgcn_s_setprio(3);
    }
#endif
#ifdef KT_PRIO
    if (threadIdx.x < 64u) __builtin_amdgcn_s_setprio(KT_PRIO);   /* the table wave */
#endif
#ifdef KT_TIMING
    /* summed per wave over its values, added once at the end (per-value
     * atomics on one line serialised and skewed the timings) */
    uint64_t kt_acc[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    __shared__ uint32_t kt_busy[32];
#endif
    for (uint32_t v = blockIdx.x; v < bt.count; v += gridDim.x) {
        const uint32_t n = bt.in_len[v];
        /* no positions, or past the stated max_len (the record stride): the
         * parse refuses such a value (uniform per workgroup) */
        if (n < 3u || n > LZF_SLOTS || n > bt.max_len) continue;
        const uint8_t *src = bt.in + bt.in_off[v];
        uint32_t *rec = sc.rec + (uint64_t)v * sc.rstride;
        if (n >= 8u) kt_value<false>(L, src, n, rec KT_ACC_PASS);
        else kt_value<true>(L, src, n, rec KT_ACC_PASS);
    }
#ifdef KT_TIMING
    if ((threadIdx.x & 63u) == 0u)
        for (uint32_t i = 0; i < 10u; i++) atomicAdd(&kt_times[i], (unsigned long long)kt_acc[i]);
#endif
}

/* ======================================================================== */
/* kernel 2: the greedy parse and emission, one lane per value              */
/* ======================================================================== */

#ifndef K3_THREADS
#define K3_THREADS 256u
#endif
#define K3_CB      16u          /* records per parse block: 64 bytes of one line (32, the whole line: no gain) */
#ifndef K3_NRES
#define K3_NRES    2u           /* candidate tests per loop iteration (2: 206.2 vs 210.8 ms for 1 + a memory-free one) */
#endif
#ifndef K3_RW
#define K3_RW      32u          /* bitmap words kept in LDS per lane (a multiple of 4) */
#endif
#ifndef K3_LITMIN
#define K3_LITMIN   8u       /* lanes of the wave that must take a free-literal trip for it to run */
#endif
#ifndef K3_LITX
#define K3_LITX    3u           /* free literals taken after a literal in the same iteration (0: none) */
#endif

/* rel codes of the walk, relative to p: the record codes 0..7, plus
 * 8 (the first 3 bytes agree, length unknown) and 9 (unknown).
 * K3_EXACT (round 5): exact agreements combine too.  If p~q agree in exactly
 * a bytes and q~r in exactly b != a, then p~r agree in exactly min(a, b) (the
 * first mismatch of the shorter one is a mismatch of p~r, the bytes before
 * it agree in all three); with one of them exact (a < 8) and the other
 * >= 8, exactly the exact one; both >= 8, >= 8.  A deeper candidate's match
 * length then often needs no extension load (a record's agreements are capped
 * at its own remaining bytes, which are more than p's: the cap binds p's
 * first, so the rule holds at the value's end too). */
#ifndef K3_EXACT
#define K3_EXACT 1
#endif
__device__ __forceinline__ uint32_t k3_comb(uint32_t rel, uint32_t code)
{
    /* p~q agree in 3 bytes and q~r agree in 3 bytes => p~r agree in 3;
     * exactly one of them => p~r differ in the first 3 bytes */
    if (rel == 9u) return 9u;
    const bool e1 = rel >= 2u, e2 = code >= 2u;
    if (!(e1 && e2)) return (e1 != e2) ? RC_DIFF : 9u;
    if (K3_EXACT && rel <= RC_LONG) {              /* rel exact (2..6) or >= 8 (7); code is 2..7 */
        if (rel != code) return rel < code ? rel : code;   /* min: an exact one below the other */
        if (rel == RC_LONG) return RC_LONG;        /* both >= 8 */
    }
    return 8u;
}

enum { K3_STEP = 0, K3_RESOLVE = 1, K3_DECIDE = 2, K3_EXTEND = 3, K3_EMIT = 4, K3_DONE = 5 };

/* A value shorter than 16 bytes, whole: the reference's loop
 * (src/lzf_c.c:145-290) over the bytes in registers, the table replaced by
 * a search of the inserted positions (at most 13).  Keeps the main loop's
 * 16-byte loads inside every value. */
__device__ __noinline__ uint32_t k3_small(const uint8_t *src, uint32_t n, uint8_t *dst, uint32_t cap)
{
    const uint4 V = dv_ld16_tail(src, n);
#define K3S_B(i_) ((dv_sel4(V, (i_) >> 2) >> (8u * ((i_) & 3u))) & 0xFFu)
#define K3S_SLOT(i_) dv_slot(K3S_B(i_) | (K3S_B((i_) + 1u) << 8) | (K3S_B((i_) + 2u) << 16))
    uint32_t op = 1u, lit = 0u, ins = 0u, p = 0u;
    while (p + 2u < n) {                                           /* src/lzf_c.c:145 */
        const uint32_t s = K3S_SLOT(p);
        uint32_t q = 0u;
        for (uint32_t t = p; t-- > 0u;)                            /* the latest inserted, same slot */
            if (((ins >> t) & 1u) && K3S_SLOT(t) == s) { q = t; break; }
        ins |= 1u << p;
        if (q > 0u && p + 4u < n && K3S_B(q) == K3S_B(p) && K3S_B(q + 1u) == K3S_B(p + 1u) &&
            K3S_B(q + 2u) == K3S_B(p + 2u)) {                      /* src/lzf_c.c:151-158 */
            const uint32_t maxlen = n - p - 2u;
            uint32_t len = 3u;
            while (len < maxlen && K3S_B(q + len) == K3S_B(p + len)) len++;
            if (op - (lit ? 0u : 1u) + 4u >= cap) return 0u;     /* src/lzf_c.c:172-176 */
            if (lit) dst[op - lit - 1u] = (uint8_t)(lit - 1u);
            else op--;
            const uint32_t off = p - q - 1u, L = len - 2u;
            if (L < 7u) {
                dst[op++] = (uint8_t)((off >> 8) | (L << 5));
            } else {
                dst[op++] = (uint8_t)((off >> 8) | (7u << 5));
                dst[op++] = (uint8_t)(L - 7u);
            }
            dst[op++] = (uint8_t)off;
            lit = 0u;
            op++;
            p += len;
            if (p >= n - 2u) break;                                 /* src/lzf_c.c:229 */
            ins |= (1u << (p - 2u)) | (1u << (p - 1u));
        } else {
            if (op >= cap) return 0u;                               /* src/lzf_c.c:263 */
            lit++;
            dst[op++] = (uint8_t)K3S_B(p);
            p++;
            if (lit == LZF_MAX_LIT) { dst[op - lit - 1u] = (uint8_t)(lit - 1u); lit = 0u; op++; }
        }
    }
    if (op + 3u > cap) return 0u;                                   /* src/lzf_c.c:276 */
    while (p < n) {                                                 /* src/lzf_c.c:279-288 */
        lit++;
        dst[op++] = (uint8_t)K3S_B(p);
        p++;
        if (lit == LZF_MAX_LIT) { dst[op - lit - 1u] = (uint8_t)(lit - 1u); lit = 0u; op++; }
    }
    if (lit) dst[op - lit - 1u] = (uint8_t)(lit - 1u);
    else op--;
    return op;
#undef K3S_B
#undef K3S_SLOT
}

/* The lanes of a wave are at different points of their values, so the loop
 * is a state machine in which every lane does at most ONE unit of each kind
 * of work per iteration -- take the record of p, test one candidate for
 * insertion (or load one record of the chain), compare one 16-byte piece of
 * a long match, emit one literal or one back-reference.  Every wave memory
 * instruction touches one line per lane (64 values), so the kernel is shaped
 * to issue few of them: records in 64-byte blocks, output in 16-byte stores,
 * the input in 16-byte windows, the bitmap's recent words in LDS. */
#ifndef K3_MINB
#define K3_MINB 1
#endif
__global__ __launch_bounds__(K3_THREADS, K3_MINB) void lzf_parse_rec_kernel(LzfBatch bt, LzfRecScratch sc)
{
    const uint32_t v = blockIdx.x * K3_THREADS + threadIdx.x;
    if (v >= bt.count) return;
    const uint32_t n = bt.in_len[v], cap = bt.out_cap[v];
    if (n == 0u || cap == 0u || n > LZF_SLOTS || n > bt.max_len) {  /* src/lzf_c.c:131; past max_len: refused */
        bt.out_len[v] = 0u;
        return;
    }
    const uint8_t *src = bt.in + bt.in_off[v];
    uint8_t *dst = bt.out + bt.out_off[v];
    if (n < 16u) {                     /* below one 16-byte window: whole, in registers */
        bt.out_len[v] = k3_small(src, n, dst, cap);
        return;
    }
    const uint32_t *rec = sc.rec + (uint64_t)v * sc.rstride;
    uint32_t *bits = sc.bits + (uint64_t)v * sc.bstride;

    /* output: aligned dwords at da; acc holds the bytes from dword fw on;
     * completed dwords [fs, fw) wait in pb0..2 and leave as one 16-byte store */
    const uint32_t dm = (uint32_t)((uintptr_t)dst & 3u);
    uint8_t *const da = dst - dm;
    uint64_t acc = 0;
    uint32_t accn = dm, fw = 0;
    uint32_t hx = dm;                   /* header byte of the open run (index from da) */
    uint32_t pb0 = 0u, pb1 = 0u, pb2 = 0u, fs = 0u;
    /* input: the 16 bytes from position wb */
    uint32_t wb = 0xFFFFFFF0u;
    uint4 W = make_uint4(0, 0, 0, 0);

    uint32_t o = 1u, run = 0u, p = 0u; /* o, run: the reference's op and lit (src/lzf_c.c:113-143) */
    uint32_t cb = 0xFFFFFFE0u;         /* records [cb, cb + K3_CB) in C0..C3 (C4..C7) */
    uint4 C0 = W, C1 = W, C2 = W, C3 = W;
    /* record d of the block: a select tree over the block's words (a dynamic
     * index would put the block in scratch memory) */
    const auto pick = [&](uint32_t d) -> uint32_t {
        const bool b0 = d & 1u, b1 = d & 2u;
        const uint32_t c0 = b1 ? (b0 ? C0.w : C0.z) : (b0 ? C0.y : C0.x);
        const uint32_t c1 = b1 ? (b0 ? C1.w : C1.z) : (b0 ? C1.y : C1.x);
        const uint32_t c2 = b1 ? (b0 ? C2.w : C2.z) : (b0 ? C2.y : C2.x);
        const uint32_t c3 = b1 ? (b0 ? C3.w : C3.z) : (b0 ? C3.y : C3.x);
        const uint32_t lo = (d & 8u) ? ((d & 4u) ? c3 : c2) : ((d & 4u) ? c1 : c0);
        return lo;
    };
    uint32_t cw = 0u, curw = 0u;       /* inserted-bitmap word of p, in flight */
    __shared__ uint32_t k3_ring[K3_RW][K3_THREADS];
    uint32_t *const ring = &k3_ring[0][threadIdx.x];
#define K3_RING(w_) ring[((w_) % K3_RW) * K3_THREADS]
    uint32_t fl = 0u;                  /* bitmap words [0, fl) are in scratch */
#define K3_FLUSH_TO(w_)                                                            \
    do {                                                                           \
        while (fl + K3_RW <= (w_)) {                                               \
            *(uint4 *)(bits + fl) = make_uint4(K3_RING(fl), K3_RING(fl + 1u),      \
                                               K3_RING(fl + 2u), K3_RING(fl + 3u)); \
            fl += 4u;                                                              \
        }                                                                          \
    } while (0)
    uint32_t ms = 0u, me = 0u;         /* the last match: [ms, me) */
    uint32_t rel = 0u, q = 0u, k = 0u, lim = 0u, m = 0u;
    uint32_t reln = 0u, qn = 0u;       /* the next chain link from the same record (reln 0: none) */
    bool ok = true;
    uint32_t mode = n >= 3u ? K3_STEP : K3_DONE;
#ifdef KT_TIMING
    /* [8] wave iterations [9] wave cycles [10] steps [11] resolve tests
     * [12] bitmap words from scratch [13] record hops [14] extend pieces [15] block loads */
    uint64_t k3c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint64_t k3t0 = __builtin_amdgcn_s_memtime();
#define K3_CNT(i) (k3c[(i) - 8]++)
#else
#define K3_CNT(i) ((void)0)
#endif

/* completed dwords [fs, fw) wait in pb0..2 (slot fw - fs) and leave with
 * the fourth as one 16-byte store; slot and patch selects instead of
 * branches (every branch costs the wave its exec-mask juggling) */
#define K3_STORE16(w_)                                                             \
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
    } while (0)
#define K3_PUT(bytes_, cnt_)                                                       \
    do {                                                                           \
        acc |= (uint64_t)(bytes_) << (8u * accn);                                  \
        accn += (cnt_);                                                            \
        if (accn >= 4u) {                                                          \
            const uint32_t w_ = (uint32_t)acc, np_ = fw - fs;                      \
            pb0 = np_ == 0u ? w_ : pb0;                                            \
            pb1 = np_ == 1u ? w_ : pb1;                                            \
            pb2 = np_ == 2u ? w_ : pb2;                                            \
            if (np_ == 3u) {                                                       \
                K3_STORE16(w_);                                                    \
                fs = fw + 1u;                                                      \
            }                                                                      \
            fw++;                                                                  \
            acc >>= 32;                                                            \
            accn -= 4u;                                                            \
        }                                                                          \
    } while (0)
#define K3_PATCH(x_, byte_)                                                        \
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
#define K3_BYTE(pos_, out_)                                                        \
    do {                                                                           \
        uint32_t d_ = (pos_) - wb;                                                 \
        if (d_ >= 16u) {                   /* 16 bytes inside the value (n >= 16) */ \
            wb = dv_at16(n, (pos_));                                               \
            W = dv_ld16(src + wb);                                                 \
            d_ = (pos_) - wb;                                                      \
        }                                                                          \
        (out_) = (dv_sel4(W, d_ >> 2) >> (8u * (d_ & 3u))) & 0xFFu;               \
    } while (0)
#define K3_LITERAL(pos_)                                                           \
    do {                                                                           \
        uint32_t byte_;                                                            \
        K3_BYTE(pos_, byte_);                                                      \
        const bool first_ = run == 0u;             /* the run's header slot first */ \
        hx = first_ ? 4u * fw + accn : hx;                                         \
        K3_PUT(first_ ? byte_ << 8 : byte_, first_ ? 2u : 1u);                     \
        o++;                                                                       \
        if (++run == LZF_MAX_LIT) { K3_PATCH(hx, LZF_MAX_LIT - 1u); run = 0u; o++; } \
    } while (0)

    while (__ballot(mode != K3_DONE)) {
        K3_CNT(8);
        /* ---- the record of p ---------------------------------------------- */
        if (mode == K3_STEP) {                                            /* src/lzf_c.c:145 */
            if (p >= n - 2u) {
                mode = K3_DONE;
            } else {
                K3_CNT(10);
                uint32_t d = p - cb;
                if (d >= K3_CB) {
                    K3_CNT(15);
                    cb = p & ~(K3_CB - 1u);
                    d = p - cb;
                    const uint4 *cp = (const uint4 *)(rec + cb);
                    C0 = cp[0];
                    C1 = cp[1];
                    C2 = cp[2];
                    C3 = cp[3];
                }
                const uint32_t c = pick(d);
                rel = (c >> 13) & 7u;
                q = p - 1u - (c & 0x1FFFu);
                reln = c >> 29;
                qn = p - 1u - ((c >> 16) & 0x1FFFu);
                mode = rel ? K3_RESOLVE : K3_DECIDE;
            }
        }
        /* ---- is the candidate inserted? else the next chain link: up to
         * K3_NRES tests per iteration (a walk past a skipped candidate then
         * rarely costs the wave an iteration) ------------------------------ */
#pragma unroll
        for (uint32_t rt_ = 0; rt_ < K3_NRES; rt_++) {
            if (mode == K3_RESOLVE) {
                K3_CNT(11);
                uint32_t word;
                if (q >= ms) {
                    word = (q > ms && q + 3u <= me) ? 0u : 0xFFFFFFFFu;         /* last match's interior */
                } else {
                    const uint32_t d = cw - (q >> 5);
                    word = d == 0u ? curw : (q >> 5) >= fl ? K3_RING(q >> 5) : bits[q >> 5];
#ifdef KT_TIMING
                    if (d && (q >> 5) < fl) K3_CNT(12);
#endif
                }
                if ((word >> (q & 31u)) & 1u) {                              /* q is the ref */
                    if (rel == 9u) {
                        /* bytes q..q+2 against p..p+2 with one 4-byte load per side
                         * (q + 3 <= p + 2 < n and p >= 1: both inside the value),
                         * one memory wait instead of up to three */
                        const uint32_t x_ = dv_ld4(src + q) ^ (dv_ld4(src + p - 1u) >> 8);
                        rel = (x_ & 0xFFFFFFu) == 0u ? 8u : RC_DIFF;
                    }
                    mode = K3_DECIDE;
                } else if (reln) {                                           /* the record's second link */
                    q = qn;
                    rel = reln;
                    reln = 0u;
                    /* the link after it needs q's own record: mark with reln 0 and
                     * qn = q (a load below on the next failure) */
                    qn = 0xFFFFFFFFu;
                } else if (qn == 0xFFFFFFFFu) {                              /* load q's record: two more links */
                    K3_CNT(13);
                    const uint32_t c2 = rec[q];
                    const uint32_t r1 = (c2 >> 13) & 7u, r2 = c2 >> 29;
                    const uint32_t y1 = q - 1u - (c2 & 0x1FFFu), y2 = q - 1u - ((c2 >> 16) & 0x1FFFu);
                    if (!r1 || p - y1 - 1u >= LZF_WINDOW) {                  /* the chain leaves p's window */
                        rel = 0u;
                        mode = K3_DECIDE;
                    } else {
                        const uint32_t rq = rel;
                        rel = k3_comb(rq, r1);
                        q = y1;
                        if (r2 && p - y2 - 1u < LZF_WINDOW) {
                            reln = k3_comb(rq, r2);
                            qn = y2;
                        } else {
                            reln = 0u;
                            qn = 0u;                                         /* nothing after y1 */
                        }
                    }
                } else {                                                     /* no further link */
                    rel = 0u;
                    mode = K3_DECIDE;
                }
            }
        }
        /* ---- literal, or the start of a back-reference --------------------- */
        if (mode == K3_DECIDE) {
            curw |= 1u << (p & 31u);                                     /* p is inserted */
            if (!(rel >= 2u && p + 4u < n)) {                            /* src/lzf_c.c:151-166 */
                if (o >= cap) {                                          /* src/lzf_c.c:263 */
                    ok = false;
                    mode = K3_DONE;
                } else {
                    K3_LITERAL(p);
                    p++;
                    if ((p & 31u) == 0u) {
                        K3_FLUSH_TO(cw);
                        K3_RING(cw) = curw;
                        cw++;
                        curw = 0u;
                    }
                    mode = K3_STEP;
#if K3_LITX
                    /* free literals (lzf_lane.hip's parse has the same path):
                     * positions whose record has no candidate at all (code1
                     * 0, src/lzf_c.c:153-158), with the record and the byte in
                     * registers, up to K3_LITX more per iteration */
                    /* only when enough lanes of the wave are at a literal at
                     * all (one ballot of the branch's lanes): on text, where
                     * few are, the wave skips the path */
                    bool go = true;
                    if ((uint32_t)__builtin_popcountll(__ballot(true)) >= K3_LITMIN)
#pragma unroll
                    for (uint32_t e_ = 0; e_ < K3_LITX; e_++) {
                        const uint32_t d_ = p - cb, x_ = p - wb;
                        go = go && p < n - 2u && d_ < K3_CB && x_ < 16u && o < cap;
                        if (go) {
                            const uint32_t c_ = pick(d_);
                            go = (c_ & 0xE000u) == 0u;
                        }
                        /* a trip the wave takes only when enough lanes gain
                         * from it: on text, where few do, the others would
                         * wait through it */
                        if ((uint32_t)__builtin_popcountll(__ballot(go)) < K3_LITMIN) break;
                        if (go) {
                            curw |= 1u << (p & 31u);
                            const uint32_t byte_ = (dv_sel4(W, x_ >> 2) >> (8u * (x_ & 3u))) & 0xFFu;
                            const bool first_ = run == 0u;
                            hx = first_ ? 4u * fw + accn : hx;
                            K3_PUT(first_ ? byte_ << 8 : byte_, first_ ? 2u : 1u);
                            o++;
                            if (++run == LZF_MAX_LIT) { K3_PATCH(hx, LZF_MAX_LIT - 1u); run = 0u; o++; }
                            p++;
                            if ((p & 31u) == 0u) {
                                K3_FLUSH_TO(cw);
                                K3_RING(cw) = curw;
                                cw++;
                                curw = 0u;
                            }
                        }
                    }
#endif
                }
            } else {
                uint32_t maxlen = n - p - 2u;                            /* src/lzf_c.c:169-170 */
                if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
                /* the 16 unrolled compares run whenever maxlen > 16 (src/lzf_c.c:181-202) */
                lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
                if (rel <= 6u) {
                    m = rel + 1u < lim ? rel + 1u : lim;
                    mode = K3_EMIT;
                } else {
                    k = rel == RC_LONG ? 8u : 3u;
                    mode = K3_EXTEND;
                }
            }
        }
        /* ---- one 16-byte piece of a long match ----------------------------- */
        if (mode == K3_EXTEND) {
            if (k < lim) {
                K3_CNT(14);
                const uint32_t avail = n - (p + k);
                const uint4 a = dv_ld16_safe(src + p + k, avail);
                const uint4 b = dv_ld16_safe(src + q + k, avail);
                W = a;                                   /* literals after the match read it */
                wb = p + k;
                const uint32_t d = dv_first_diff(a, b);
                k += d;
                if (d < 16u) lim = k < lim ? k : lim;
            }
            if (k >= lim) {
                m = lim;
                mode = K3_EMIT;
            }
        }
        /* ---- the back-reference -------------------------------------------- */
        if (mode == K3_EMIT) {
            const uint32_t off = p - q - 1u;
            if (run) K3_PATCH(hx, run - 1u);                             /* close the run */
            else o--;                                                    /* undo empty run */
            if (o + 4u >= cap) {                                         /* src/lzf_c.c:176 */
                ok = false;
                mode = K3_DONE;
            } else {
                const uint32_t L = m - 2u;
                const bool two = L < 7u;
                K3_PUT(two ? ((off >> 8) | (L << 5)) | ((off & 0xFFu) << 8)
                           : (0xE0u | (off >> 8)) | ((L - 7u) << 8) | ((off & 0xFFu) << 16),
                       two ? 2u : 3u);
                o += two ? 2u : 3u;
                run = 0u;
                o++;                                                     /* reserve a header */
                ms = p;
                p += m;
                me = p;
                if (p >= n - 2u) {                                       /* src/lzf_c.c:229 */
                    mode = K3_DONE;
                } else {
                    /* the two last positions of the match are inserted, its interior not */
                    const uint32_t nw = p >> 5, t1 = p - 2u, t2 = p - 1u;
                    const uint32_t b1 = 1u << (t1 & 31u), b2 = 1u << (t2 & 31u);
                    if (nw == cw) {
                        curw |= b1 | b2;
                    } else {
                        const uint32_t w1 = t1 >> 5, w2 = t2 >> 5;
                        const uint32_t wo = curw | (w1 == cw ? b1 : 0u) | (w2 == cw ? b2 : 0u);
                        const uint32_t wn = (w1 == nw ? b1 : 0u) | (w2 == nw ? b2 : 0u);
                        const uint32_t wm = (w1 != cw && w1 != nw ? b1 : 0u) | (w2 != cw && w2 != nw ? b2 : 0u);
                        K3_FLUSH_TO(cw);
                        K3_RING(cw) = wo;
                        /* words cw+1 .. nw-2 are all interior (0), nw-1 holds tails */
                        for (uint32_t w = cw + 1u; w < nw; w++) {
                            K3_FLUSH_TO(w);
                            K3_RING(w) = w + 1u == nw ? wm : 0u;
                        }
                        curw = wn;
                        cw = nw;
                    }
                    mode = K3_STEP;
                }
            }
        }
#ifdef KT_ENDMODE   /* diagnostics: lanes that end an iteration mid-step, by mode */
        k3c[4] += mode == K3_RESOLVE;
        k3c[5] += mode == K3_DECIDE;
        k3c[6] += mode == K3_EXTEND;
        k3c[7] += mode == K3_EMIT;
#endif
    }
#ifdef KT_TIMING
    k3c[1] = __builtin_amdgcn_s_memtime() - k3t0;
    if ((threadIdx.x & 63u) != 0u) k3c[0] = k3c[1] = 0u;   /* wave figures once */
    for (uint32_t i = 0; i < 8u; i++) atomicAdd(&kt_times[8u + i], (unsigned long long)k3c[i]);
#endif
#undef K3_CNT
    if (!ok || o + 3u > cap) { bt.out_len[v] = 0u; return; }          /* src/lzf_c.c:276 */
    while (p < n) {                                                   /* src/lzf_c.c:279-288 */
        K3_LITERAL(p);
        p++;
    }
    if (run) K3_PATCH(hx, run - 1u);
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
#undef K3_PUT
#undef K3_STORE16
#undef K3_PATCH
#undef K3_BYTE
#undef K3_LITERAL
#undef K3_RING
#undef K3_FLUSH_TO
}

/* ---- launcher ------------------------------------------------------------ */

/* records per value: a multiple of 16 (64 bytes) plus one block of slack, so
 * the parse's 64-byte blocks never straddle a line and never leave the value */
static uint64_t rec_stride(uint32_t max_len)
{
    return (((uint64_t)max_len + K3_CB - 1u) & ~(uint64_t)(K3_CB - 1u)) + (K3_CB < 16u ? 16u : K3_CB);
}
static uint64_t rec_bstride(uint32_t max_len) { return ((((uint64_t)max_len + 31u) >> 5) + 3u) & ~3ull; }

size_t lzf_table_scratch_per_value(uint32_t max_len)
{
    return (size_t)(rec_stride(max_len) * 4u + rec_bstride(max_len) * 4u);
}

bool lzf_table_compress_supported(uint32_t max_len) { return max_len <= LZF_SLOTS; }

hipError_t lzf_launch_compress_table(const LzfBatch &b, hipStream_t s, void *scratch, size_t scratch_bytes,
                                     uint32_t *chunks, const LzfParts *parts)
{
    if (b.max_len > LZF_SLOTS) return hipErrorInvalidValue;
    const uint64_t rstride = rec_stride(b.max_len), bstride = rec_bstride(b.max_len);
    const size_t per = lzf_table_scratch_per_value(b.max_len);
    const auto bytes_for = [&](uint64_t ch) { return ((ch * rstride * 4u + 255u) & ~255ull) + ch * bstride * 4u; };
    uint64_t chunk = scratch_bytes / per;
    if (chunk > b.count) chunk = b.count;
    while (chunk && bytes_for(chunk) > scratch_bytes) chunk--;
    if (chunk == 0) return hipErrorInvalidValue;
    /* diagnostics: LZF_GPU_TABLE_STAGE=1 runs kernel 1 only (its own time) */
    const char *stg = getenv("LZF_GPU_TABLE_STAGE");
    const bool cand_only = stg && *stg == '1';
    /* kernel 1: the per-value pipeline (lzf_cand_table_kernel); in the
     * diagnostic build LZF_GPU_TCAND=stream takes the stream kernel's record
     * form instead (lzf_stream.hip, bit-exact, slower: DESIGN.md §4.2) */
#ifdef LZF_DIAG
    const char *tc = getenv("LZF_GPU_TCAND");
    const bool stream = tc && !strcmp(tc, "stream");
#else
    constexpr bool stream = false;
#endif
    LzfRecScratch sc;
    sc.rec = (uint32_t *)scratch;
    sc.bits = (uint32_t *)((uint8_t *)scratch + ((chunk * rstride * 4u + 255u) & ~255ull));
    sc.rstride = rstride;
    sc.bstride = bstride;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    hipError_t e;
    if (chunks) *chunks = (uint32_t)((b.count + chunk - 1u) / chunk);
    if (parts && parts->n) {
        if (chunk < b.count || stream || cand_only || parts->end[parts->n - 1u] != b.count) {
            /* not one chunk: every part in first, then the plain launch */
            for (uint32_t p = 0; p < parts->n; p++)
                if ((e = hipStreamWaitEvent(s, parts->ev[p], 0)) != hipSuccess) return e;
        } else {
            /* kernel 1 per part as its inputs arrive (its records go to the
             * part's own rows of the scratch), then one parse over the batch */
            uint32_t lo = 0;
            for (uint32_t p = 0; p < parts->n; p++) {
                const uint32_t hi = parts->end[p];
                if ((e = hipStreamWaitEvent(s, parts->ev[p], 0)) != hipSuccess) return e;
                if (hi <= lo) continue;
                LzfBatch c = b;
                c.in_off = b.in_off + lo;
                c.in_len = b.in_len + lo;
                c.out_off = b.out_off + lo;
                c.out_cap = b.out_cap + lo;
                c.out_len = b.out_len + lo;
                c.count = hi - lo;
                LzfRecScratch sp = sc;
                sp.rec = sc.rec + (uint64_t)lo * rstride;
                const uint32_t g = c.count < (uint32_t)cus ? c.count : (uint32_t)cus;
                hipLaunchKernelGGL(lzf_cand_table_kernel, dim3(g), dim3(KT_THREADS), 0, s, c, sp);
                if ((e = hipGetLastError()) != hipSuccess) return e;
                lo = hi;
            }
            hipLaunchKernelGGL(lzf_parse_rec_kernel, dim3((b.count + K3_THREADS - 1u) / K3_THREADS),
                               dim3(K3_THREADS), 0, s, b, sc);
            return hipGetLastError();
        }
    }
    for (uint64_t first = 0; first < b.count; first += chunk) {
        const uint32_t cnt = (uint32_t)((b.count - first) < chunk ? (b.count - first) : chunk);
        LzfBatch c = b;
        c.in_off = b.in_off + first;
        c.in_len = b.in_len + first;
        c.out_off = b.out_off + first;
        c.out_cap = b.out_cap + first;
        c.out_len = b.out_len + first;
        c.count = cnt;
        /* one 512-thread workgroup per CU (the table is 128 KiB), persistent */
        const uint32_t g = cnt < (uint32_t)cus ? cnt : (uint32_t)cus;
        if (stream) {
#ifdef LZF_DIAG
            if ((e = lzf_launch_cand_stream_rec(c, sc, s)) != hipSuccess) return e;
#endif
        } else {
            hipLaunchKernelGGL(lzf_cand_table_kernel, dim3(g), dim3(KT_THREADS), 0, s, c, sc);
            if ((e = hipGetLastError()) != hipSuccess) return e;
        }
        if (cand_only) continue;
        hipLaunchKernelGGL(lzf_parse_rec_kernel, dim3((cnt + K3_THREADS - 1u) / K3_THREADS), dim3(K3_THREADS),
                           0, s, c, sc);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

/*
 * lzf_compress.hip -- wave-parallel, bit-exact LZF compressor for gfx950.
 *
 * Replaces src/lzf_c.c:98-294 for batches of independent values: one
 * workgroup = one 64-lane wave per value.  The reference's greedy parse is
 * serial (the slot table it consults depends on which positions earlier
 * decisions inserted, src/lzf_c.c:147-149, 227-247); this kernel keeps that
 * exact semantics but resolves it 64 positions ("a window") at a time:
 *
 *   1. every lane i takes position p = P+i: slot(p) (src/lzf_c.c:47-57) and
 *      the exact sets of window lanes sharing its slot / its head bucket,
 *      from three small LDS lane bitmaps keyed by bits 0-5, 6-11, 12-15 of
 *      a bijective slot mix (ds_or_b64; same slot = all three agree, same
 *      bucket = bits 6-15 agree).  The nearest earlier same-slot lane (prevW) is the ref IF
 *      every window position were inserted;
 *   2. every lane also looks the slot up in the exact table of inserted
 *      positions < P: 1024 bucket heads (slot, pos) + a skip chain over the
 *      last 8192 positions (distance to the latest earlier inserted position
 *      of the bucket with a DIFFERENT slot).  The walk stops at the first
 *      entry with the same 16-bit slot -- exactly the pointer the
 *      reference's 65536-slot table holds -- or beyond the 8 KiB window,
 *      where the reference's `off < MAX_OFF` test fails too;
 *   3. match test and length per lane (src/lzf_c.c:151-209, including the 16
 *      unconditional compares: lim = maxlen>16 ? max(maxlen,19) : maxlen),
 *      probed up to 19 bytes per lane;
 *   4. the parse orbit: a minimal scalar loop over match lanes (s_ff1 on the
 *      ballot); a match on the orbit that reached the probe cap gets its
 *      exact length from a whole-wave 256-byte compare.  A visited lane
 *      whose prevW lies inside an earlier match (not inserted by the
 *      reference, src/lzf_c.c:227-247) is repaired in place: its ref becomes
 *      the latest inserted same-slot lane, else the table entry from step 2;
 *   5. emission: the reference's output cursor (reserved run header,
 *      32-literal rollover, undo of an empty run, out-of-space checks at
 *      src/lzf_c.c:176, 263, 276) is a function of per-lane run indices and
 *      one wave prefix sum (DPP) of per-token sizes; all lanes store their
 *      literal / header / back-reference bytes in parallel;
 *   6. the window's inserted positions go into heads / skip chain, the last
 *      one per bucket and each one's skip target read off the lane bitmaps.
 *
 * Nothing is ever written at or past out_cap; the return value (0 or the
 * stream length) and the stream are identical to the reference's.
 */
#include "lzf_internal.h"

#define CW_LANES     64u
#ifndef CW_HBITS
#define CW_HBITS     10
#endif
#define CW_HBUCKETS  (1u << CW_HBITS)
/* lane bitmaps keyed by slot-mix bits [0,16-HBITS), [16-HBITS,12), [12,16):
 * same slot = all three agree, same bucket = the last two agree */
#define CW_T1        (1u << (16 - CW_HBITS))
#define CW_T2        (1u << (CW_HBITS - 4))
#define CW_T3        16u
#define CW_TALL      (CW_T1 + CW_T2 + CW_T3)
#define CW_CHAIN     8192u
#define CW_RING_MAX  16384u
#define CW_EXT_CAP   19u          /* per-lane match length probe (3 + 4 x 4 bytes) */
#define CW_TBYTES    (CW_TALL * 8u)
#ifndef CW_HOPCAP
#define CW_HOPCAP    3u           /* chain hops in the wave-uniform lookup loop */
#endif

/* Diagnostic build only (make stats -> liblzf_hip_stats.so): per-phase
 * s_memtime cycles and event counts, summed over all waves. */
#ifdef LZF_CW_STATS
__device__ unsigned long long cw_stats[32];
enum { ST_WINDOWS, ST_TRUNC, ST_HOPS, ST_EXT, ST_ORBITM, ST_VALUES, ST_COOP, ST_PH0 = 8 };
#define CW_STAT_ADD(k, v) (st_##k += (v))
#define CW_PHASE(i)                                                       \
    do {                                                                  \
        unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
        st_ph[i] += t_ - t_last;                                          \
        t_last = t_;                                                      \
    } while (0)
#else
#define CW_STAT_ADD(k, v) ((void)0)
#define CW_PHASE(i) ((void)0)
#endif

__device__ __forceinline__ uint64_t lanemask_lt(uint32_t i)
{
    return i >= 64u ? ~0ull : ((1ull << i) - 1ull);
}

__device__ __forceinline__ uint64_t range_mask(uint32_t lo, uint32_t hi)   /* bits [lo, hi) */
{
    return lanemask_lt(hi) & ~lanemask_lt(lo);
}

__device__ __forceinline__ uint32_t slot_of(uint32_t tri)
{
    uint32_t b0 = tri & 0xFFu, b1 = (tri >> 8) & 0xFFu, b2 = (tri >> 16) & 0xFFu;
    return (((b0 << 8) | b1) - 5u * ((b1 << 8) | b2)) & 0xFFFFu;
}

/* Order-preserving LDS hand-off between the lanes of the (single-wave)
 * workgroup: LDS ops of one wave execute in order, so only the compiler
 * must not move memory operations across this point. */
__device__ __forceinline__ void wave_lds_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

/* Inclusive prefix sum over the 64 lanes (DPP row shifts + row broadcasts). */
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false); /* row_shr:1 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false); /* row_shr:2 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false); /* row_shr:4 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false); /* row_shr:8 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); /* row_bcast:15 */
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); /* row_bcast:31 */
    return x;
}

/* Bucket-head entry: position of the latest inserted position of the
 * bucket, its slot's identity within the bucket (slot-mix bits 0-5; the
 * bucket fixes the rest) and an 8-bit presence filter over the identities
 * ever inserted into the bucket (bit ident & 7).  A lookup whose filter bit
 * is clear has no same-slot entry to find and skips the chain walk.  Values
 * up to 64 KiB use 32-bit entries [pos:16 | ident:8 | filter:8]; longer
 * ones 64-bit [pos:32 | ident:8 | filter:8 | 0:16]. */
template <typename E> struct HeadOps;
template <> struct HeadOps<uint32_t> {
    typedef uint16_t PosT;
    static constexpr uint32_t EMPTY = 0x00FFFFFFu;      /* no position, empty filter */
    __device__ static uint32_t pos(uint32_t e) { return e & 0xFFFFu; }
    __device__ static bool empty(uint32_t e) { return (e & 0xFFFFu) == 0xFFFFu; }
    __device__ static uint32_t ident(uint32_t e) { return (e >> 16) & 0xFFu; }
    __device__ static uint32_t filter(uint32_t e) { return e >> 24; }
};
template <> struct HeadOps<unsigned long long> {
    typedef uint32_t PosT;
    static constexpr unsigned long long EMPTY = 0x000000FFFFFFFFFFull;
    __device__ static uint32_t pos(unsigned long long e) { return (uint32_t)e; }
    __device__ static bool empty(unsigned long long e) { return (uint32_t)e == 0xFFFFFFFFu; }
    __device__ static uint32_t ident(unsigned long long e) { return (uint32_t)(e >> 32) & 0xFFu; }
    __device__ static uint32_t filter(unsigned long long e) { return (uint32_t)(e >> 40) & 0xFFu; }
};

template <typename HeadT, bool WRAP>
struct CwLds {
    uint8_t *ring;        /* input ring, R bytes (power of two) */
    uint32_t rmask;       /* R - 1 */
    HeadT *head;          /* CW_HBUCKETS: latest inserted (slot, pos) of the bucket */
    uint16_t *chain;      /* per inserted position: distance to the latest earlier
                           * inserted position of its bucket with another slot */
    uint32_t cmask;       /* chain ring entries - 1 */
    unsigned long long *t1, *t2, *t3;   /* window lane bitmaps keyed by slot-mix bits
                                         * 0-5, 6-11, 12-15 */

    /* ring word / chain entry index: the ring and chain wrap only when the
     * value is longer than them (WRAP); otherwise indices are positions */
    __device__ __forceinline__ uint32_t wi(uint32_t w) const { return WRAP ? (w & (rmask >> 2)) : w; }
    __device__ __forceinline__ uint32_t ci(uint32_t x) const { return WRAP ? (x & cmask) : x; }
    __device__ __forceinline__ uint32_t rd4(uint32_t x) const
    {
        const uint32_t *w = (const uint32_t *)ring;
        uint32_t lo = w[wi(x >> 2)], hi = w[wi((x >> 2) + 1u)];
        return __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
    }
    __device__ __forceinline__ uint32_t rd1(uint32_t x) const { return ring[WRAP ? (x & rmask) : x]; }
};

/* Stream input bytes [from, to) of the value into the ring. */
template <typename HeadT, bool WRAP>
__device__ void cw_fill(const CwLds<HeadT, WRAP> &L, const uint8_t *src, uint32_t from, uint32_t to)
{
    const uint32_t lane = threadIdx.x;
    if (((uintptr_t)(src + from) & 15u) == 0u) {
        uint32_t nvec = (to - from) >> 4;
        for (uint32_t k = lane; k < nvec; k += CW_LANES) {
            uint4 v = *(const uint4 *)(src + from + 16u * k);
            uint32_t x = from + 16u * k;
            if ((x & 15u) == 0u) {
                *(uint4 *)(L.ring + (x & L.rmask)) = v;
            } else {
                const uint8_t *vb = (const uint8_t *)&v;
                for (int t = 0; t < 16; t++) L.ring[(x + t) & L.rmask] = vb[t];
            }
        }
        for (uint32_t x = from + (nvec << 4) + lane; x < to; x += CW_LANES) L.ring[x & L.rmask] = src[x];
    } else {
        for (uint32_t x = from + lane; x < to; x += CW_LANES) L.ring[x & L.rmask] = src[x];
    }
}

__device__ __forceinline__ uint32_t slot_mix(uint32_t s) { return (s * 40503u) & 0xFFFFu; }
__device__ __forceinline__ uint32_t bucket_of(uint32_t sm) { return sm >> (16 - CW_HBITS); }
__device__ __forceinline__ uint32_t ident_of(uint32_t sm) { return sm & (CW_T1 - 1u); }
__device__ __forceinline__ uint32_t filter_bit(uint32_t id) { return 1u << (id & 7u); }

/* Bucket-head updates.  The filter bit is OR-ed in (every inserted position);
 * position and identity are plain sub-word stores (the bucket's last one). */
template <typename HeadT>
__device__ __forceinline__ void head_mark(HeadT *head, uint32_t b, uint32_t id)
{
    uint32_t *w = (uint32_t *)(head + b) + (sizeof(HeadT) == 8 ? 1 : 0);
    atomicOr(w, filter_bit(id) << (sizeof(HeadT) == 8 ? 8 : 24));
}
template <typename HeadT>
__device__ __forceinline__ void head_set(HeadT *head, uint32_t b, uint32_t id, uint32_t x)
{
    typedef typename HeadOps<HeadT>::PosT PosT;
    *(PosT *)(head + b) = (PosT)x;
    *((uint8_t *)(head + b) + sizeof(PosT)) = (uint8_t)id;
}

/* Length of the match p/r whose first k0 bytes are known equal, up to lim:
 * the whole wave compares 256 bytes per step (uniform inputs and result). */
template <typename HeadT, bool WRAP>
__device__ __forceinline__ uint32_t cw_coop_len(const CwLds<HeadT, WRAP> &L, uint32_t p, uint32_t r,
                                                uint32_t k0, uint32_t lim)
{
    const uint32_t lane = threadIdx.x;
    uint32_t kb = k0;
    while (kb < lim) {
        const uint32_t kk = kb + 4u * lane;
        uint32_t x = 0;
        if (kk < lim) {
            x = L.rd4(p + kk) ^ L.rd4(r + kk);
            const uint32_t rem = lim - kk;
            if (rem < 4u) x |= 0xFFFFFFFFu << (8u * rem);
        }
        const uint64_t hit = __ballot(x != 0u);
        if (hit) {
            const uint32_t fl = (uint32_t)__builtin_ctzll(hit);
            const uint32_t xf = __builtin_amdgcn_readlane(x, fl);
            const uint32_t k = kb + 4u * fl + ((uint32_t)__builtin_ctz(xf) >> 3);
            return k < lim ? k : lim;
        }
        kb += 4u * CW_LANES;
    }
    return lim;
}

/* Latest inserted position < P with slot s (or none), from the bucket head
 * hv and the skip chain; exactly the reference's table entry when it is
 * within the 8 KiB window (src/lzf_c.c:147-155).  id = s's identity in its
 * bucket; a clear filter bit means s was never inserted. */
template <typename HeadT, bool WRAP>
__device__ __forceinline__ uint32_t cw_lookup(const CwLds<HeadT, WRAP> &L, HeadT hv, uint32_t hch, uint32_t s,
                                              uint32_t id, uint32_t p)
{
    typedef HeadOps<HeadT> H;
    if (!(H::filter(hv) & filter_bit(id))) return 0xFFFFFFFFu;   /* never inserted (or empty) */
    uint32_t q = H::pos(hv);
    bool same = H::ident(hv) == id;
    uint32_t d = hch;                             /* the head's chain entry, read early */
    while (p - q <= LZF_WINDOW) {
        if (same) return q;
        if (d == 0u) break;                       /* skip q's run of its slot */
        q -= d;
        same = slot_of(L.rd4(q) & 0xFFFFFFu) == s;
        d = L.chain[L.ci(q)];
    }
    return 0xFFFFFFFFu;
}

/* First mismatch index in [3, kc) of p vs r (kc <= 19), or kc: five aligned
 * dwords per side, no loop. */
template <typename HeadT, bool WRAP>
__device__ __forceinline__ uint32_t cw_probe(const CwLds<HeadT, WRAP> &L, uint32_t p, uint32_t r, uint32_t kc)
{
    const uint32_t *w = (const uint32_t *)L.ring;
    const uint32_t pa = (p + 3u) >> 2, ra = (r + 3u) >> 2;
    const uint32_t ps = (p + 3u) & 3u, rs = (r + 3u) & 3u;
    uint32_t pw[5], rw[5];
#pragma unroll
    for (int t = 0; t < 5; t++) {
        pw[t] = w[L.wi(pa + t)];
        rw[t] = w[L.wi(ra + t)];
    }
    uint32_t k = kc;
#pragma unroll
    for (int t = 3; t >= 0; t--) {
        const uint32_t x = __builtin_amdgcn_alignbyte(pw[t + 1], pw[t], ps) ^
                           __builtin_amdgcn_alignbyte(rw[t + 1], rw[t], rs);
        if (x) k = 3u + 4u * (uint32_t)t + ((uint32_t)__builtin_ctz(x) >> 3);
    }
    return k < kc ? k : kc;
}

/* Inclusive max over the 64 lanes (DPP). */
__device__ __forceinline__ uint32_t cd_incl_max(uint32_t x)
{
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
    return x;
}

/* One wave-uniform round of the table walk (cw_lookup) for every lane still
 * active: skip q's run of its slot, check the next entry.  Finished lanes
 * re-read their own entry. */
template <typename HeadT, bool WRAP>
__device__ __forceinline__ void cw_walk_step(const CwLds<HeadT, WRAP> &L, uint32_t p, uint32_t s, bool &act,
                                             uint32_t &q, uint32_t &d, uint32_t &T)
{
    act = act && d != 0u;
    q = act ? q - d : q;
    const uint32_t sq = slot_of(L.rd4(q) & 0xFFFFFFu);
    d = L.chain[L.ci(q)];
    act = act && p - q <= LZF_WINDOW;
    if (act && sq == s) T = q;
    act = act && sq != s;
}

__device__ __forceinline__ uint32_t match_lim(uint32_t n, uint32_t p)
{
    uint32_t maxlen = n - p - 2u;
    if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
    return (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;   /* src/lzf_c.c:181-206 */
}

__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, uint32_t l)
{
    return ((uint64_t)readlane_u32((uint32_t)(v >> 32), l) << 32) | readlane_u32((uint32_t)v, l);
}

/* one instance per ring size, with static LDS: the compiler folds the LDS
 * base into every address (with dynamic LDS it adds the base, 0, with one
 * VALU per LDS address) */
#define CW_LDS(HeadT, RING) ((RING) + CW_HBUCKETS * sizeof(HeadT) + CW_TBYTES + \
                             ((RING) < CW_CHAIN ? (RING) : CW_CHAIN) * sizeof(uint16_t))
template <typename HeadT, bool WRAP, uint32_t RING>
__global__ __launch_bounds__(64) void lzf_compress_window_kernel(LzfBatch bt, uint32_t ring_bytes)
{
    typedef HeadOps<HeadT> H;
    __shared__ __attribute__((aligned(16))) uint8_t smem[CW_LDS(HeadT, RING)];
    ring_bytes = RING;
    CwLds<HeadT, WRAP> L;
    L.ring = smem;
    L.rmask = ring_bytes - 1u;
    uint8_t *cur = smem + ring_bytes;
    L.head = (HeadT *)cur;                   cur += CW_HBUCKETS * sizeof(HeadT);
    L.t1 = (unsigned long long *)cur;
    L.t2 = L.t1 + CW_T1;
    L.t3 = L.t2 + CW_T2;
    cur += CW_TBYTES;
    L.chain = (uint16_t *)cur;
    L.cmask = (ring_bytes < CW_CHAIN ? ring_bytes : CW_CHAIN) - 1u;

    const uint32_t lane = threadIdx.x;
#ifdef LZF_CW_STATS
    unsigned long long st_hops = 0, st_ext = 0, st_windows = 0, st_trunc = 0, st_orbitm = 0,
                       st_coop = 0;
    unsigned long long st_ph[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t v = blockIdx.x;
    const uint32_t n = bt.in_len[v];
    const uint32_t cap = bt.out_cap[v];
    const uint8_t *src = bt.in + bt.in_off[v];
    uint8_t *dst = bt.out + bt.out_off[v];
    /* src/lzf_c.c:131; a value past the batch's stated max_len (the LDS plan
     * was sized from it) is refused the same way, never overrun */
    if (n == 0u || cap == 0u || n > bt.max_len) {
        if (lane == 0) bt.out_len[v] = 0u;
        return;
    }

    {
        for (uint32_t k = lane; k < CW_HBUCKETS; k += CW_LANES) L.head[k] = H::EMPTY;
        uint32_t *z = (uint32_t *)(L.head + CW_HBUCKETS);      /* lane bitmaps = 0 */
        for (uint32_t k = lane; k < CW_TBYTES / 4u; k += CW_LANES) z[k] = 0u;
    }
    uint32_t loaded = n < ring_bytes ? n : ring_bytes;
    cw_fill(L, src, 0u, loaded);
    __syncthreads();
    CW_PHASE(0);

    uint32_t P = 0;          /* next parse position (window start) */
    uint32_t H0 = 0;         /* output index of the open run's header */
    uint32_t c0 = 0;         /* literals in the open run (< 32) */
    bool fail = false;

    while (P + 2u < n) {     /* main loop: src/lzf_c.c:145 */
        /* keep the ring ahead of the window and its match extensions; the
         * ring also still holds the 8 KiB back-reference span */
        uint32_t need = P + CW_LANES + LZF_MAX_REF + 16u;
        if (need > n) need = n;
        if (__builtin_expect(loaded < need, 0)) {
            uint32_t to = loaded + 4096u;
            if (to < need) to = (need + 15u) & ~15u;
            if (to > n) to = n;
            cw_fill(L, src, loaded, to);
            loaded = to;
            __syncthreads();
        }
        CW_PHASE(1);
        CW_STAT_ADD(windows, 1);

        /* ---- 1. slots and same-slot / same-bucket lane sets ---------- */
        const uint32_t lim_lane = (n - 2u - P) < CW_LANES ? (n - 2u - P) : CW_LANES;
        const uint32_t p = P + lane;
        const bool valid = lane < lim_lane;
        const uint32_t tri = L.rd4(p) & 0xFFFFFFu;
        const uint32_t s = slot_of(tri);
        const uint32_t sm = slot_mix(s);          /* bijective 16-bit mix of the slot */
        const uint32_t b = bucket_of(sm);
        const uint32_t k1 = ident_of(sm);
        /* Lanes past lim_lane take part unconditionally (no exec-mask
         * regions): their bits only ever land above every valid lane, where
         * prevW (lanes below), `other` and `last` (masked by INS) never look,
         * and their lookups are switched off below. */
        const HeadT hv = L.head[b];
        const uint32_t hch = L.chain[L.ci(H::empty(hv) ? 0u : H::pos(hv))];   /* head's chain entry */
        const uint32_t k2 = (sm >> (16 - CW_HBITS)) & (CW_T2 - 1u), k3 = sm >> 12;
        const unsigned long long me = 1ull << lane;
        atomicOr(&L.t1[k1], me);
        atomicOr(&L.t2[k2], me);
        atomicOr(&L.t3[k3], me);
        wave_lds_fence();
        const uint64_t M1 = L.t1[k1], M2 = L.t2[k2], M3 = L.t3[k3];
        wave_lds_fence();
        L.t1[k1] = 0ull;
        L.t2[k2] = 0ull;
        L.t3[k3] = 0ull;
        const uint64_t Mb = M2 & M3;              /* lanes with my bucket (mix bits 6-15) */
        const uint64_t Ms = M1 & Mb;              /* lanes with my slot (all 16 bits) */
        const uint64_t msb = Ms & lanemask_lt(lane);
        int prevW = msb ? (int)(63u - (uint32_t)__builtin_clzll(msb)) : -1;
        CW_PHASE(2);

        /* ---- 2. exact table lookup among positions < P (cw_lookup for
         * the lanes without prevW, as one wave-uniform loop: every lane
         * steps each round, the finished ones re-read their own entry) --- */
        uint32_t T = 0xFFFFFFFFu;
        bool act = valid && prevW < 0 && (H::filter(hv) & filter_bit(k1)) && p - H::pos(hv) <= LZF_WINDOW;
        uint32_t wq = act ? H::pos(hv) : 0u, wd = hch;           /* walk state */
        if (act && H::ident(hv) == k1) T = wq;
        act = act && H::ident(hv) != k1;
        /* walks are cut off at CW_HOPCAP hops (unrolled: no loop branch);
         * their lanes count as literals for now and are finished (all at
         * once) only if the orbit visits one of them */
#pragma unroll
        for (uint32_t it = 0; it < CW_HOPCAP; it++) cw_walk_step(L, p, s, act, wq, wd, T);
        uint64_t U = __ballot(act);
        CW_PHASE(3);

        /* ---- 3. match test (src/lzf_c.c:151-166), probed length ------ */
        /* (every lane runs the test and the probe: no exec-mask regions;
         * a lane without a candidate reads its own position) */
        uint32_t ref = prevW >= 0 ? P + (uint32_t)prevW : T;
        const uint32_t lim0 = match_lim(n, p);
        const uint32_t kc = lim0 < CW_EXT_CAP ? lim0 : CW_EXT_CAP;
        bool match, exact;
        uint32_t lim, m;
        auto match_test = [&]() {
            const bool cand = valid & (ref != 0xFFFFFFFFu) & (ref > 0u) &
                              ((p - ref - 1u) < LZF_WINDOW) & (p + 4u < n);
            const uint32_t rr = cand ? ref : p;
            match = cand & ((L.rd4(rr) & 0xFFFFFFu) == tri);
            const uint32_t mp = cw_probe(L, p, rr, kc);   /* bytes [3, kc) in one go */
            lim = match ? lim0 : 0u;
            m = match ? mp : 1u;
            exact = !match | (mp < kc) | (kc == lim0);
        };
        match_test();
        CW_PHASE(4);

        /* ---- 4. the parse orbit -----------------------------------------
         * Literal lanes advance by one, so the orbit is fixed by the match
         * lanes on it: nm(i) = first match lane >= i+m (i+1 for a
         * literal), precomputed by every lane; a scalar walk follows nm
         * through the match lanes only (v_readlane), a long match on it
         * gets its exact length by a whole-wave compare, and the visited
         * lanes follow from one prefix max of the matches' reach.  A lane
         * whose prevW turns out to lie inside a match (never inserted by the
         * reference) is repaired in place and the walk resumes there. */
        uint64_t MMc = __ballot(match) & lanemask_lt(lim_lane);
        uint64_t NXc = __ballot(!exact) & MMc;
        uint64_t MMV = 0, V = 0;
        uint32_t end = lim_lane, mexit = 0, j0 = 0;
        int exitLane = -1;
        for (;;) {
            /* per-lane successor on the orbit */
            const bool isMatch = (MMc >> lane) & 1ull;
            const uint32_t tgt = lane + (isMatch ? m : 1u);
            const uint64_t after = tgt >= CW_LANES ? 0ull : (MMc & ~lanemask_lt(tgt));
            uint32_t nm = after ? (uint32_t)__builtin_ctzll(after) : CW_LANES;
            if (isMatch && tgt >= lim_lane) nm = 255u;                /* leaves the window */
            /* walk the match lanes of the orbit from j0 */
            const uint64_t first = MMc & ~lanemask_lt(j0);
            uint32_t j = first ? (uint32_t)__builtin_ctzll(first) : CW_LANES;
            exitLane = -1;
            uint32_t jl = 0;                      /* the last orbit match lane so far */
            for (;;) {
                /* the common steps: match lanes of exact length follow nm */
                /* seven scalar instructions per orbit match (s_bitcmp1 /
                 * s_bitset1 / v_readlane; the nop covers the readlane's
                 * lane-select hazard on the next step), unrolled 4x so the
                 * loop takes one backward branch per four matches */
                asm volatile(
                    "L%=_top:\n\t"
                    "s_cmp_lt_u32 %0, %4\n\t"
                    "s_cbranch_scc0 L%=_end\n\t"
                    "s_bitcmp1_b64 %3, %0\n\t"
                    "s_cbranch_scc1 L%=_end\n\t"
                    "s_bitset1_b64 %2, %0\n\t"
                    "s_mov_b32 %1, %0\n\t"
                    "v_readlane_b32 %0, %5, %0\n\t"
                    "s_nop 4\n\t"
                    "s_cmp_lt_u32 %0, %4\n\t"
                    "s_cbranch_scc0 L%=_end\n\t"
                    "s_bitcmp1_b64 %3, %0\n\t"
                    "s_cbranch_scc1 L%=_end\n\t"
                    "s_bitset1_b64 %2, %0\n\t"
                    "s_mov_b32 %1, %0\n\t"
                    "v_readlane_b32 %0, %5, %0\n\t"
                    "s_nop 4\n\t"
                    "s_cmp_lt_u32 %0, %4\n\t"
                    "s_cbranch_scc0 L%=_end\n\t"
                    "s_bitcmp1_b64 %3, %0\n\t"
                    "s_cbranch_scc1 L%=_end\n\t"
                    "s_bitset1_b64 %2, %0\n\t"
                    "s_mov_b32 %1, %0\n\t"
                    "v_readlane_b32 %0, %5, %0\n\t"
                    "s_nop 4\n\t"
                    "s_cmp_lt_u32 %0, %4\n\t"
                    "s_cbranch_scc0 L%=_end\n\t"
                    "s_bitcmp1_b64 %3, %0\n\t"
                    "s_cbranch_scc1 L%=_end\n\t"
                    "s_bitset1_b64 %2, %0\n\t"
                    "s_mov_b32 %1, %0\n\t"
                    "v_readlane_b32 %0, %5, %0\n\t"
                    "s_nop 4\n\t"
                    "s_branch L%=_top\n"
                    "L%=_end:"
                    : "+s"(j), "+s"(jl), "+s"(MMV)
                    : "s"(NXc), "s"(lim_lane), "v"(nm)
                    : "scc");
                /* the walk stopped: past the window (j == 255 after a match
                 * that leaves it, CW_LANES after a literal) -- or at a match
                 * that reached the probe cap, whose exact length the whole
                 * wave computes; then it goes on (one exit, no flow flags) */
                if (__builtin_expect(j >= lim_lane, 1)) break;
                CW_STAT_ADD(coop, 1);
                MMV |= 1ull << j;
                jl = j;
                const uint32_t mj = cw_coop_len(L, P + j, readlane_u32(ref, j),
                                                readlane_u32(m, j), readlane_u32(lim, j));
                if (lane == j) m = mj;
                NXc &= ~(1ull << j);
                const uint64_t a = j + mj >= lim_lane ? 0ull : MMc & ~lanemask_lt(j + mj);
                j = j + mj >= lim_lane ? 255u : (a ? (uint32_t)__builtin_ctzll(a) : CW_LANES);
            }
            exitLane = j == 255u ? (int)jl : -1;
            mexit = readlane_u32(m, jl);
            end = exitLane >= 0 ? (uint32_t)exitLane + 1u : lim_lane;
            /* visited = not strictly inside the reach of an earlier orbit match */
            /* (orbit match lanes are visited; their own reach is > lane) */
            const uint32_t reach = ((MMV >> lane) & 1ull) ? lane + m : 0u;
            const uint32_t rmax = cd_incl_max(reach);
            V = (__ballot(rmax <= lane) | MMV) & lanemask_lt(end);
            /* speculation check: prevW must be an inserted position */
            const uint64_t INTR = ~V & ~(V >> 1) & ~(V >> 2);    /* inside a match */
            const bool vis = (V >> lane) & 1ull;
            const uint64_t BADC = __ballot(vis && prevW >= 0 && ((INTR >> (uint32_t)prevW) & 1ull));
            const uint64_t BADU = U & V;
            if (__builtin_expect(!(BADC | BADU), 1)) break;
            if (BADU && (!BADC || __builtin_ctzll(BADU) < __builtin_ctzll(BADC))) {
                /* a visited lane's table walk was cut off: finish every cut-off
                 * walk (one wave-uniform loop); if some of them now match,
                 * redo their match tests and, when one of those is visited,
                 * walk the orbit again from it */
                CW_STAT_ADD(hops, 1);
                const bool was = (U >> lane) & 1ull;
                while (__ballot(act)) cw_walk_step(L, p, s, act, wq, wd, T);
                const bool cu = was & (T != 0xFFFFFFFFu) & (T > 0u) & ((p - T - 1u) < LZF_WINDOW) &
                                (p + 4u < n) & ((L.rd4(was && T != 0xFFFFFFFFu ? T : p) & 0xFFFFFFu) == tri);
                const uint64_t newM = __ballot(cu);
                if (newM) {
                    const bool om = match, oe = exact;
                    const uint32_t oref = ref, olim = lim, omm = m;
                    if (was) ref = T;
                    match_test();
                    if (!was) { match = om; exact = oe; ref = oref; lim = olim; m = omm; }
                    MMc |= newM;
                    NXc |= __ballot(!exact) & newM;
                }
                U = 0;
                const uint64_t chg = newM & V;
                if (chg) {
                    const uint32_t f = (uint32_t)__builtin_ctzll(chg);
                    MMV &= lanemask_lt(f);
                    j0 = f;
                    continue;
                }
                if (!BADC) break;
            }
            /* lane f read an entry the reference never inserted (or its table
             * walk was cut off): its ref is the latest INSERTED same-slot lane,
             * else the table entry */
            CW_STAT_ADD(trunc, 1);
            const uint32_t f = (uint32_t)__builtin_ctzll(BADC);
            const uint64_t alt = readlane_u64(Ms, f) & lanemask_lt(f) & ~INTR;
            const uint32_t pf = P + f;
            uint32_t rf;
            if (alt) {
                rf = P + 63u - (uint32_t)__builtin_clzll(alt);
            } else {
                HeadT hf;
                if constexpr (sizeof(HeadT) == 8) hf = (HeadT)readlane_u64((uint64_t)hv, f);
                else hf = (HeadT)readlane_u32((uint32_t)hv, f);
                rf = cw_lookup<HeadT, WRAP>(L, hf, readlane_u32(hch, f), readlane_u32(s, f),
                                            readlane_u32(k1, f), pf);
            }
            bool ok = rf != 0xFFFFFFFFu && rf > 0u && (pf - rf - 1u) < LZF_WINDOW && pf + 4u < n;
            if (ok) ok = readlane_u32(L.rd4(rf) & 0xFFFFFFu, 0) == readlane_u32(tri, f);
            const uint64_t fb = 1ull << f;
            if (ok) {
                const uint32_t mf = cw_coop_len(L, pf, rf, 3u, match_lim(n, pf));
                MMc |= fb;
                if (lane == f) { m = mf; ref = rf; }
            } else {
                MMc &= ~fb;
            }
            NXc &= ~fb;
            if (lane == f) prevW = -1;
            MMV &= lanemask_lt(f);
            j0 = f;
        }
        const uint64_t ACC = lanemask_lt(end);
        const bool byMatch = exitLane >= 0;
        CW_STAT_ADD(orbitm, (unsigned long long)__builtin_popcountll(MMV));
        CW_PHASE(5);

        /* ---- 5. emission.  A segment = the visited lanes after one match
         * up to and including the next; its literals are consecutive. ---- */
        const bool visited = (V >> lane) & 1ull;
        const bool isM = (MMV >> lane) & 1ull;
        const uint64_t NVb = ~V & lanemask_lt(lane);
        const uint32_t segStart = NVb ? 64u - (uint32_t)__builtin_clzll(NVb) : 0u;
        const bool seg0 = (MMV & lanemask_lt(lane)) == 0ull;
        const uint32_t R = (seg0 ? c0 : 0u) + lane - segStart;   /* literal index in run */
        const uint32_t tlen = (m - 2u < 7u) ? 2u : 3u;
        const uint32_t nf = 1u + R + (R >> 5);                    /* relative to H0 of seg */
        const uint32_t Tr = nf - ((R & 31u) == 0u ? 1u : 0u);
        const uint32_t delta = (visited && isM) ? Tr + tlen : 0u;
        const uint32_t incl = wave_incl_sum(delta);
        const uint32_t myH0 = H0 + incl - delta;
        /* Each visited lane stores up to four bytes, as four unconditional
         * stores under one exec mask: an unused store repeats the lane's
         * previous (address, byte).  Literal: [rollover header 31 at pos-32]
         * + the byte.  Match: [run header] + 2 or 3 back-reference bytes.
         * Out of space (src/lzf_c.c:176, 263): nothing of the lane is stored. */
        const uint32_t lit = L.rd1(p);
        asm volatile("" ::"v"(lit));              /* load for every lane: no branch around it */
        const uint32_t off = p - ref - 1u;
        const uint32_t Lc = m - 2u;
        const uint32_t pos = myH0 + (isM ? Tr : nf);
        const bool lfail = visited & (pos + (isM ? 4u : 0u) >= cap);
        const uint32_t b0 = isM ? ((off >> 8) | (Lc < 7u ? Lc << 5 : 0xE0u)) : lit;
        const bool h1 = isM ? (R & 31u) != 0u : (R & 31u) == 31u;
        const uint32_t hpos = myH0 + 33u * (R >> 5);              /* the run's header */
        asm volatile("" ::"v"(hpos));
        const uint32_t a1 = h1 ? (isM ? hpos : pos - 32u) : pos;
        const uint32_t v1 = h1 ? (isM ? (R & 31u) - 1u : 31u) : b0;
        const uint32_t a3 = isM ? pos + 1u : pos;
        const uint32_t v3 = isM ? (Lc < 7u ? off : Lc - 7u) : b0;
        const bool long3 = isM & (Lc >= 7u);
        const uint32_t a4 = long3 ? pos + 2u : a3;
        const uint32_t v4 = long3 ? off : v3;
        if (visited & !lfail) {
            dst[a1] = (uint8_t)v1;
            dst[pos] = (uint8_t)b0;
            dst[a3] = (uint8_t)v3;
            dst[a4] = (uint8_t)v4;
        }
        if (__builtin_expect(__ballot(lfail) != 0, 0)) { fail = true; break; }
        CW_PHASE(6);

        /* ---- carry the cursor state to the next window ---------------- */
        uint32_t Pn;
        uint64_t INS = (V | (~V & ((V >> 1) | (V >> 2)))) & ACC;   /* visited + match tails */
        uint32_t tx0 = 0xFFFFFFFFu, tx1 = 0xFFFFFFFFu;           /* tails beyond the window */
        if (byMatch) {
            const uint32_t j = (uint32_t)exitLane;
            H0 = H0 + readlane_u32(incl, j);
            c0 = 0u;
            Pn = P + j + mexit;
            if (Pn + 2u < n) {                 /* src/lzf_c.c:229-247 */
                const uint32_t a = j + mexit - 2u, c = j + mexit - 1u;
                if (a < CW_LANES) INS |= 1ull << a; else tx0 = P + a;
                if (c < CW_LANES) INS |= 1ull << c; else tx1 = P + c;
            }
        } else {
            const uint32_t e = end;            /* == lim_lane: first lane of the next window */
            const uint64_t nvb = ~V & lanemask_lt(e);
            const uint32_t ss = nvb ? 64u - (uint32_t)__builtin_clzll(nvb) : 0u;
            const uint32_t Re = (MMV ? 0u : c0) + e - ss;
            H0 = H0 + readlane_u32(incl, e - 1u) + 33u * (Re >> 5);
            c0 = Re & 31u;
            Pn = P + e;
        }

        /* ---- 6. insert the window's inserted positions --------------- */
        {
            /* skip target of every lane, branch-free: the latest earlier
             * inserted window lane of the bucket with another slot, else the
             * bucket head (or the head's own target when it has my slot) */
            const bool ins = (INS >> lane) & 1ull;
            const bool last = (Mb & INS & ~lanemask_lt(lane + 1u)) == 0ull;
            const uint64_t other = Mb & ~Ms & INS & lanemask_lt(lane);
            const uint32_t hp = H::pos(hv);
            const bool hok = !H::empty(hv) & (p - hp <= LZF_WINDOW);
            const uint32_t yh = H::ident(hv) != k1 ? hp : (hch ? hp - hch : 0xFFFFFFFFu);
            const uint32_t y = other ? P + 63u - (uint32_t)__builtin_clzll(other)
                                     : (hok ? yh : 0xFFFFFFFFu);
            const uint32_t cv = (y != 0xFFFFFFFFu && p - y <= LZF_WINDOW) ? p - y : 0u;
            if (ins) {
                L.chain[L.ci(p)] = (uint16_t)cv;
                head_mark(L.head, b, k1);
                if (last) head_set(L.head, b, k1, p);
            }
        }
        wave_lds_fence();
        if (tx0 != 0xFFFFFFFFu || tx1 != 0xFFFFFFFFu) {
            /* the exit match's tails past the window: lane 0 inserts tx0,
             * lane 1 tx1 (after tx0: when both hit one bucket, tx0 is tx1's
             * head) */
            const uint32_t t = lane == 0 ? tx0 : tx1;
            const bool act = lane < 2u && t != 0xFFFFFFFFu;
            uint32_t bt = 0xFFFFFFFFu, idt = 0, y = 0xFFFFFFFFu;
            if (act) {
                const uint32_t smt = slot_mix(slot_of(L.rd4(t) & 0xFFFFFFu));
                bt = bucket_of(smt);
                idt = ident_of(smt);
                const HeadT ht = L.head[bt];
                if (!H::empty(ht) && t - H::pos(ht) <= LZF_WINDOW) {
                    const uint32_t hp = H::pos(ht);
                    if (H::ident(ht) != idt) {
                        y = hp;
                    } else {
                        const uint32_t d = L.chain[L.ci(hp)];
                        if (d) y = hp - d;
                    }
                }
            }
            const uint32_t b0t = readlane_u32(bt, 0), b1t = readlane_u32(bt, 1);
            const uint32_t id0 = readlane_u32(idt, 0), y0 = readlane_u32(y, 0);
            if (lane == 1 && tx0 != 0xFFFFFFFFu && bt == b0t) y = id0 != idt ? tx0 : y0;
            if (act) {
                L.chain[L.ci(t)] = (uint16_t)((y != 0xFFFFFFFFu && t - y <= LZF_WINDOW) ? t - y : 0u);
                head_mark(L.head, bt, idt);
                if (lane == 1 || tx1 == 0xFFFFFFFFu || b1t != bt) head_set(L.head, bt, idt, t);
            }
            wave_lds_fence();
        }
        CW_PHASE(7);
        P = Pn;
    }
#ifdef LZF_CW_STATS
    if (lane == 0) {
        atomicAdd(&cw_stats[ST_HOPS], st_hops);
        atomicAdd(&cw_stats[ST_EXT], st_ext);
        atomicAdd(&cw_stats[ST_WINDOWS], st_windows);
        atomicAdd(&cw_stats[ST_TRUNC], st_trunc);
        atomicAdd(&cw_stats[ST_ORBITM], st_orbitm);
        atomicAdd(&cw_stats[ST_COOP], st_coop);
        atomicAdd(&cw_stats[ST_VALUES], 1ull);
        for (int k = 0; k < 12; k++) atomicAdd(&cw_stats[ST_PH0 + k], st_ph[k]);
    }
#endif

    /* tail: src/lzf_c.c:276-293 */
    if (!fail && H0 + 1u + c0 + 3u > cap) fail = true;
    if (fail) {
        if (lane == 0) bt.out_len[v] = 0u;
        return;
    }
    const uint32_t ntail = n > P ? n - P : 0u;      /* 0..2 */
    if (lane < ntail) {
        const uint32_t R = c0 + lane;
        const uint32_t pos = H0 + 1u + R + (R >> 5);
        dst[pos] = (uint8_t)L.rd1(P + lane);
        if ((R & 31u) == 31u) dst[pos - 32u] = 31u;
    }
    if (lane == 0) {
        const uint32_t R = c0 + ntail;
        if (R & 31u) dst[H0 + 33u * (R >> 5)] = (uint8_t)((R & 31u) - 1u);
        bt.out_len[v] = H0 + 1u + R + (R >> 5) - ((R & 31u) == 0u ? 1u : 0u);
    }
}

static uint32_t ring_for(uint32_t max_len)
{
    uint32_t r = 256u;
    while (r < max_len && r < CW_RING_MAX) r <<= 1;
    return r;
}

template <typename HeadT, bool WRAP, uint32_t RING>
static hipError_t launch_window(const LzfBatch &b, hipStream_t s)
{
    lzf_compress_window_kernel<HeadT, WRAP, RING><<<dim3(b.count), dim3(CW_LANES), 0, s>>>(b, RING);
    return hipGetLastError();
}

hipError_t lzf_launch_compress(const LzfBatch &b, hipStream_t s)
{
    /* values that fit the chain (8 KiB) never wrap the ring or the chain */
    static_assert(CW_CHAIN == 8192u && CW_RING_MAX == 16384u, "the instances below");
    switch (b.max_len <= CW_CHAIN ? ring_for(b.max_len) : 0u) {
    case 256u: return launch_window<uint32_t, false, 256u>(b, s);
    case 512u: return launch_window<uint32_t, false, 512u>(b, s);
    case 1024u: return launch_window<uint32_t, false, 1024u>(b, s);
    case 2048u: return launch_window<uint32_t, false, 2048u>(b, s);
    case 4096u: return launch_window<uint32_t, false, 4096u>(b, s);
    case 8192u: return launch_window<uint32_t, false, 8192u>(b, s);
    default: break;
    }
    if (b.max_len <= 65536u) return launch_window<uint32_t, true, CW_RING_MAX>(b, s);
    return launch_window<unsigned long long, true, CW_RING_MAX>(b, s);
}

const char *lzf_compress_kernel_name(void) { return "window64"; }

#ifdef LZF_CW_STATS
extern "C" int lzf_gpu_debug_stats(unsigned long long *out32, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(out32, HIP_SYMBOL(cw_stats), sizeof(cw_stats));
    if (e == hipSuccess && reset) {
        unsigned long long z[32] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(cw_stats), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : -2;
}
#endif

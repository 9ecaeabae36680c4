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
 *      the nearest earlier lane with the same slot (prevW), found through a
 *      256-key LDS bitmask (ds_or_b64) -- the ref IF every window position
 *      were inserted;
 *   2. lanes without prevW look the slot up in the exact table of inserted
 *      positions < P: 4096 bucket heads + a skip chain over the last 8192
 *      positions (entry = slot << 16 | distance to the latest earlier
 *      inserted position of the bucket with a DIFFERENT slot).  The walk
 *      stops at the first entry with the same 16-bit slot -- exactly the
 *      pointer the reference's 65536-slot table holds -- or beyond the 8 KiB
 *      window, where the reference's `off < MAX_OFF` test fails too;
 *   3. match test and length per lane (src/lzf_c.c:151-209, including the 16
 *      unconditional compares: lim = maxlen>16 ? max(maxlen,19) : maxlen),
 *      probed up to 11 bytes per lane;
 *   4. the parse orbit: a minimal scalar loop over match lanes (s_ff1 on the
 *      ballot); a match on the orbit that reached the probe cap gets its
 *      exact length from a whole-wave 256-byte compare;
 *   5. validation: a visited lane whose prevW lies inside a match (not
 *      inserted by the reference, src/lzf_c.c:227-247) would have read an
 *      older entry -- the window is accepted up to that lane only;
 *   6. emission: the reference's output cursor (reserved run header,
 *      32-literal rollover, undo of an empty run, out-of-space checks at
 *      src/lzf_c.c:176, 263, 276) is a function of per-lane run indices and
 *      one wave prefix sum (DPP) of per-token sizes; all lanes store their
 *      literal / header / back-reference bytes in parallel;
 *   7. the window's inserted positions go into heads / skip chain.
 *
 * Nothing is ever written at or past out_cap; the return value (0 or the
 * stream length) and the stream are identical to the reference's.
 */
#include "lzf_internal.h"

#define CW_LANES     64u
#define CW_HBUCKETS  4096u
#define CW_KEYS      256u
#define CW_CHAIN     8192u
#define CW_RING_MAX  16384u
#define CW_EXT_CAP   11u          /* per-lane match length probe (3 + 2 x 4 bytes) */

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

__device__ __forceinline__ uint32_t hbucket(uint32_t slot)
{
    return ((slot * 40503u) >> 4) & (CW_HBUCKETS - 1u);
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

template <typename HeadT>
struct CwLds {
    uint8_t *ring;        /* input ring, R bytes (power of two) */
    uint32_t rmask;       /* R - 1 */
    HeadT *head;          /* CW_HBUCKETS: latest inserted position of the bucket */
    uint32_t *chain;      /* per inserted position: slot << 16 | skip distance */
    uint32_t cmask;       /* chain ring entries - 1 */
    unsigned long long *keymask; /* CW_KEYS: window lanes per bucket key */
    uint32_t *sb;         /* 64 x (bucket << 16 | slot) of the window */

    __device__ __forceinline__ uint32_t rd4(uint32_t x) const
    {
        const uint32_t *w = (const uint32_t *)ring;
        uint32_t m = rmask >> 2;
        uint32_t lo = w[(x >> 2) & m], hi = w[((x >> 2) + 1u) & m];
        return __builtin_amdgcn_alignbyte(hi, lo, x & 3u);
    }
    __device__ __forceinline__ uint32_t rd1(uint32_t x) const { return ring[x & rmask]; }
};

/* Stream input bytes [from, to) of the value into the ring. */
template <typename HeadT>
__device__ void cw_fill(const CwLds<HeadT> &L, const uint8_t *src, uint32_t from, uint32_t to)
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

/* Insert position x (slot sx) after every earlier position (one lane). */
template <typename HeadT>
__device__ __forceinline__ void cw_insert_one(const CwLds<HeadT> &L, uint32_t x, uint32_t sx)
{
    const HeadT NONE = (HeadT)~(HeadT)0;
    uint32_t bx = hbucket(sx);
    uint32_t h = (uint32_t)L.head[bx];
    uint32_t y = 0xFFFFFFFFu;
    if (h != (uint32_t)NONE && x - h <= LZF_WINDOW) {
        uint32_t eh = L.chain[h & L.cmask];
        if ((eh >> 16) != sx) y = h;
        else if (eh & 0xFFFFu) y = h - (eh & 0xFFFFu);
    }
    L.chain[x & L.cmask] = (sx << 16) | ((y != 0xFFFFFFFFu && x - y <= LZF_WINDOW) ? x - y : 0u);
    L.head[bx] = (HeadT)x;
}

template <typename HeadT>
__global__ __launch_bounds__(64) void lzf_compress_window_kernel(LzfBatch bt, uint32_t ring_bytes)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const HeadT NONE = (HeadT)~(HeadT)0;
    CwLds<HeadT> L;
    L.ring = smem;
    L.rmask = ring_bytes - 1u;
    uint8_t *cur = smem + ring_bytes;
    L.keymask = (unsigned long long *)cur;  cur += CW_KEYS * 8u;
    L.sb = (uint32_t *)cur;                 cur += CW_LANES * 4u;
    L.head = (HeadT *)cur;                  cur += CW_HBUCKETS * sizeof(HeadT);
    L.chain = (uint32_t *)cur;
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
    if (n == 0u || cap == 0u) {                 /* src/lzf_c.c:131 */
        if (lane == 0) bt.out_len[v] = 0u;
        return;
    }

    for (uint32_t k = lane; k < CW_KEYS; k += CW_LANES) L.keymask[k] = 0ull;
    {
        uint32_t *h32 = (uint32_t *)L.head;
        for (uint32_t k = lane; k < CW_HBUCKETS * sizeof(HeadT) / 4u; k += CW_LANES) h32[k] = ~0u;
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
        if (loaded < need) {
            uint32_t to = loaded + 4096u;
            if (to < need) to = (need + 15u) & ~15u;
            if (to > n) to = n;
            cw_fill(L, src, loaded, to);
            loaded = to;
            __syncthreads();
        }
        CW_PHASE(1);
        CW_STAT_ADD(windows, 1);

        const uint32_t lim_lane = (n - 2u - P) < CW_LANES ? (n - 2u - P) : CW_LANES;
        const uint32_t p = P + lane;
        const bool valid = lane < lim_lane;
        const uint32_t tri = L.rd4(p) & 0xFFFFFFu;
        const uint32_t s = valid ? slot_of(tri) : 0xFFFFFFFFu;
        const uint32_t b = valid ? hbucket(s) : 0u;
        const uint32_t key = b & (CW_KEYS - 1u);
        L.sb[lane] = (b << 16) | (s & 0xFFFFu);
        if (valid) atomicOr(&L.keymask[key], 1ull << lane);
        wave_lds_fence();
        const uint64_t M = valid ? L.keymask[key] : 0ull;
        const uint32_t head_old = valid ? (uint32_t)L.head[b] : (uint32_t)NONE;
        wave_lds_fence();
        if (valid) L.keymask[key] = 0ull;
        CW_PHASE(2);

        /* 1. nearest earlier window lane with the same slot */
        int prevW = -1;
        for (uint64_t cand = M & lanemask_lt(lane); cand;) {
            uint32_t j = 63u - __builtin_clzll(cand);
            cand &= ~(1ull << j);
            if ((L.sb[j] & 0xFFFFu) == s) { prevW = (int)j; break; }
        }
        CW_PHASE(3);

        /* 2. exact table lookup for positions < P */
        uint32_t ref = 0xFFFFFFFFu;
        if (prevW >= 0) {
            ref = P + (uint32_t)prevW;
        } else if (head_old != (uint32_t)NONE) {
            uint32_t q = head_old;
            while (p - q <= LZF_WINDOW) {
                CW_STAT_ADD(hops, 1);
                uint32_t e = L.chain[q & L.cmask];
                if ((e >> 16) == s) { ref = q; break; }
                uint32_t d = e & 0xFFFFu;     /* skip q's whole run of its slot */
                if (d == 0u) break;
                q -= d;
            }
        }
        CW_PHASE(4);

        /* 3. match test (src/lzf_c.c:151-166) and probed length (169-209) */
        const bool match = valid && ref != 0xFFFFFFFFu && ref > 0u &&
                           (p - ref - 1u) < LZF_WINDOW && p + 4u < n &&
                           (L.rd4(ref) & 0xFFFFFFu) == tri;
        uint32_t lim = 0, m = 1;
        bool exact = true;
        if (match) {
            uint32_t maxlen = n - p - 2u;
            if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
            lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
            const uint32_t kc = lim < CW_EXT_CAP ? lim : CW_EXT_CAP;
            uint32_t k = 3u;
            while (k < kc) {
                CW_STAT_ADD(ext, 1);
                uint32_t x = L.rd4(p + k) ^ L.rd4(ref + k);
                uint32_t rem = kc - k;
                if (rem < 4u) x |= 0xFFFFFFFFu << (8u * rem);
                if (x) { k += (uint32_t)__builtin_ctz(x) >> 3; break; }
                k += 4u;
            }
            m = k < kc ? k : kc;
            exact = (m < kc) || (kc == lim);
        }
        CW_PHASE(5);

        /* 4. the parse orbit: one scalar step per match on it */
        const uint64_t MM = __ballot(match) & lanemask_lt(lim_lane);
        const uint64_t NX = __ballot(!exact);
        uint64_t V = 0, MMV = 0;
        uint32_t i0 = 0, end = lim_lane, mexit = 0;
        int exitLane = -1;
        for (;;) {
            const uint64_t rest = MM & ~lanemask_lt(i0);
            if (!rest) {
                V |= range_mask(i0, lim_lane);
                break;
            }
            const uint32_t j = (uint32_t)__builtin_ctzll(rest);
            V |= range_mask(i0, j + 1u);
            MMV |= 1ull << j;
            uint32_t mj = __builtin_amdgcn_readlane(m, j);
            if ((NX >> j) & 1ull) {
                /* exact length of a long match on the orbit, 256 B per step */
                CW_STAT_ADD(coop, 1);
                const uint32_t pj = P + j;
                const uint32_t rj = __builtin_amdgcn_readlane(ref, j);
                const uint32_t limj = __builtin_amdgcn_readlane(lim, j);
                uint32_t kb = mj;
                mj = limj;
                while (kb < limj) {
                    const uint32_t kk = kb + 4u * lane;
                    uint32_t x = 0;
                    if (kk < limj) {
                        x = L.rd4(pj + kk) ^ L.rd4(rj + kk);
                        const uint32_t rem = limj - kk;
                        if (rem < 4u) x |= 0xFFFFFFFFu << (8u * rem);
                    }
                    const uint64_t hit = __ballot(x != 0u);
                    if (hit) {
                        const uint32_t fl = (uint32_t)__builtin_ctzll(hit);
                        const uint32_t xf = __builtin_amdgcn_readlane(x, fl);
                        mj = kb + 4u * fl + ((uint32_t)__builtin_ctz(xf) >> 3);
                        break;
                    }
                    kb += 4u * CW_LANES;
                }
                if (mj > limj) mj = limj;
                if (lane == j) m = mj;
            }
            if (j + mj >= lim_lane) {
                exitLane = (int)j;
                mexit = mj;
                end = j + 1u;
                break;
            }
            i0 = j + mj;
        }
        CW_PHASE(6);

        /* 5. speculation check: prevW must be an inserted position */
        const uint64_t INTR = ~V & ~(V >> 1) & ~(V >> 2);    /* inside a match */
        const bool visited = (V >> lane) & 1ull;
        const bool bad = visited && prevW >= 0 && ((INTR >> (uint32_t)prevW) & 1ull);
        const uint64_t BAD = __ballot(bad);
        uint32_t acc_end = end;            /* lanes [0, acc_end) are accepted */
        bool byMatch = exitLane >= 0;
        if (BAD) {
            CW_STAT_ADD(trunc, 1);
            acc_end = (uint32_t)__builtin_ctzll(BAD);
            byMatch = false;
        }
        const uint64_t ACC = lanemask_lt(acc_end);
        CW_STAT_ADD(orbitm, (unsigned long long)__builtin_popcountll(MMV & ACC));
        CW_PHASE(7);

        /* 6. emission.  A segment = the visited lanes after one match up to
         * and including the next; its literals are consecutive lanes. */
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
        bool lfail = false;
        if (visited && ((ACC >> lane) & 1ull)) {
            if (!isM) {
                const uint32_t pos = myH0 + nf;
                if (pos >= cap) {
                    lfail = true;                                   /* src/lzf_c.c:263 */
                } else {
                    dst[pos] = (uint8_t)L.rd1(p);
                    if ((R & 31u) == 31u) dst[pos - 32u] = 31u;     /* rollover header */
                }
            } else {
                const uint32_t T = myH0 + Tr;
                if (T + 4u >= cap) {
                    lfail = true;                                   /* src/lzf_c.c:176 */
                } else {
                    if (R & 31u) dst[myH0 + 33u * (R >> 5)] = (uint8_t)((R & 31u) - 1u);
                    const uint32_t off = p - ref - 1u;
                    const uint32_t Lc = m - 2u;
                    if (Lc < 7u) {
                        dst[T] = (uint8_t)((off >> 8) | (Lc << 5));
                        dst[T + 1u] = (uint8_t)off;
                    } else {
                        dst[T] = (uint8_t)((off >> 8) | 0xE0u);
                        dst[T + 1u] = (uint8_t)(Lc - 7u);
                        dst[T + 2u] = (uint8_t)off;
                    }
                }
            }
        }
        if (__ballot(lfail)) { fail = true; break; }
        CW_PHASE(8);

        /* carry the cursor state to the next window */
        uint32_t Pn;
        uint64_t INS = (V | (~V & ((V >> 1) | (V >> 2)))) & ACC;   /* visited + match tails */
        uint32_t tx0 = 0xFFFFFFFFu, tx1 = 0xFFFFFFFFu;           /* tails beyond the window */
        if (byMatch) {
            const uint32_t j = (uint32_t)exitLane;
            H0 = H0 + __builtin_amdgcn_readlane(incl, j);
            c0 = 0u;
            Pn = P + j + mexit;
            if (Pn + 2u < n) {                 /* src/lzf_c.c:229-247 */
                const uint32_t a = j + mexit - 2u, c = j + mexit - 1u;
                if (a < CW_LANES) INS |= 1ull << a; else tx0 = P + a;
                if (c < CW_LANES) INS |= 1ull << c; else tx1 = P + c;
            }
        } else {
            const uint32_t e = acc_end;        /* first lane of the next window */
            const uint64_t nvb = ~V & lanemask_lt(e);
            const uint32_t ss = nvb ? 64u - (uint32_t)__builtin_clzll(nvb) : 0u;
            const uint32_t Re = ((MMV & lanemask_lt(e)) ? 0u : c0) + e - ss;
            H0 = H0 + __builtin_amdgcn_readlane(incl, e - 1u) + 33u * (Re >> 5);
            c0 = Re & 31u;
            Pn = P + e;
        }

        /* 7. insert the window's inserted positions, in position order */
        if ((INS >> lane) & 1ull) {
            const uint64_t same = M & INS & ~(1ull << lane);
            const uint32_t myb = b << 16;
            bool last = true;
            int y = -1;        /* nearest earlier inserted lane, same bucket, other slot */
            for (uint64_t c = same; c; c &= c - 1ull) {
                const uint32_t j = (uint32_t)__builtin_ctzll(c);
                const uint32_t e = L.sb[j];
                if ((e & 0xFFFF0000u) != myb) continue;
                if (j > lane) last = false;
                else if ((e & 0xFFFFu) != s) y = (int)j;
            }
            uint32_t yp = 0xFFFFFFFFu;
            if (y >= 0) {
                yp = P + (uint32_t)y;
            } else if (head_old != (uint32_t)NONE && p - head_old <= LZF_WINDOW) {
                const uint32_t eh = L.chain[head_old & L.cmask];
                if ((eh >> 16) != s) yp = head_old;
                else if (eh & 0xFFFFu) yp = head_old - (eh & 0xFFFFu);
            }
            L.chain[p & L.cmask] = (s << 16) | ((yp != 0xFFFFFFFFu && p - yp <= LZF_WINDOW) ? p - yp : 0u);
            if (last) L.head[b] = (HeadT)p;
        }
        wave_lds_fence();
        if (tx0 != 0xFFFFFFFFu || tx1 != 0xFFFFFFFFu) {
            if (lane == 0) {
                if (tx0 != 0xFFFFFFFFu) cw_insert_one(L, tx0, slot_of(L.rd4(tx0) & 0xFFFFFFu));
                if (tx1 != 0xFFFFFFFFu) cw_insert_one(L, tx1, slot_of(L.rd4(tx1) & 0xFFFFFFu));
            }
            wave_lds_fence();
        }
        CW_PHASE(9);
        P = Pn;
    }
#ifdef LZF_CW_STATS
    atomicAdd(&cw_stats[ST_HOPS], st_hops);
    atomicAdd(&cw_stats[ST_EXT], st_ext);
    if (lane == 0) {
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

template <typename HeadT>
static hipError_t launch_window(const LzfBatch &b, hipStream_t s)
{
    const uint32_t ring = ring_for(b.max_len);
    const uint32_t chain = ring < CW_CHAIN ? ring : CW_CHAIN;
    const size_t lds = ring + CW_KEYS * 8u + CW_LANES * 4u + CW_HBUCKETS * sizeof(HeadT) +
                       chain * sizeof(uint32_t);
    hipError_t e = hipFuncSetAttribute((const void *)lzf_compress_window_kernel<HeadT>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lzf_compress_window_kernel<HeadT>, dim3(b.count), dim3(CW_LANES), lds, s, b,
                       ring);
    return hipGetLastError();
}

hipError_t lzf_launch_compress(const LzfBatch &b, hipStream_t s)
{
    if (b.max_len <= 65536u) return launch_window<uint16_t>(b, s);
    return launch_window<uint32_t>(b, s);
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

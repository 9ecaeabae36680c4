/*
 * lzf_compress.hip -- wave-parallel, bit-exact LZF compressor for gfx950.
 *
 * Replaces src/lzf_c.c:98-294 for batches of independent values: one
 * workgroup = one 64-lane wave per value.  The reference's greedy parse is
 * inherently serial (the slot table it consults depends on which positions
 * earlier decisions inserted, src/lzf_c.c:147-149, 227-247); this kernel
 * keeps that exact semantics but resolves it 64 positions at a time:
 *
 *   window  lanes i = 0..63 take positions p = P+i of the current window.
 *   1. slot(p) (src/lzf_c.c:47-57), and the nearest earlier lane with the
 *      same slot (prevW), found through a 256-entry LDS bucket bitmask
 *      (ds_or_b64) -- i.e. the ref if every window position were inserted.
 *   2. lanes without prevW look the slot up in the exact table of inserted
 *      positions < P: a 4096-bucket head array + a delta chain ring over
 *      the last 8192 positions (the reference's 65536-slot table restated
 *      compactly; a walk stops at the first entry with the SAME 16-bit slot,
 *      i.e. exactly the pointer the reference would read, or when the
 *      distance exceeds the 8 KiB window, where the reference also fails).
 *   3. match test + length, per lane (src/lzf_c.c:151-209 incl. the 16
 *      unconditional compares: lim = maxlen>16 ? max(maxlen,19) : maxlen),
 *      4 bytes per step from the LDS input ring via v_alignbyte.
 *   4. the parse orbit through the window: a scalar loop over match lanes
 *      (s_ff1 on the ballot mask), one iteration per match.
 *   5. validation: a visited lane whose prevW is a skipped match interior
 *      (not inserted by the reference, src/lzf_c.c:227-247) would have read
 *      an older entry -- the window is cut right before it and re-done.
 *   6. emission: output positions of literals / run headers / back-refs
 *      from per-segment records (v_writelane) + the reference's cursor rules
 *      (reserved run header, 32-literal rollover, undo of an empty run,
 *      out-of-space checks at src/lzf_c.c:176, 263, 276) -- all lanes store
 *      their bytes in parallel.
 *   7. insertion of the window's inserted positions into head/chain, the
 *      last writer per bucket resolved through the same bucket bitmask.
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

template <typename HeadT>
struct CwLds {
    uint8_t *ring;        /* input ring, R bytes (power of two) */
    uint32_t rmask;       /* R - 1 */
    HeadT *head;          /* CW_HBUCKETS */
    uint16_t *chain;      /* CW_CHAIN: delta to previous inserted pos of the bucket */
    unsigned long long *keymask; /* CW_KEYS */
    uint32_t *sl;         /* 64 slots of the window */
    uint32_t *bl;         /* 64 buckets of the window */

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
    if (((uintptr_t)(src + from) & 15u) == 0u && (from & 15u) == 0u) {
        uint32_t nvec = (to - from) >> 4;
        for (uint32_t k = lane; k < nvec; k += CW_LANES) {
            uint4 v = *(const uint4 *)(src + from + 16u * k);
            uint32_t x = from + 16u * k;
            *(uint4 *)(L.ring + (x & L.rmask)) = v;
        }
        for (uint32_t x = from + (nvec << 4) + lane; x < to; x += CW_LANES) L.ring[x & L.rmask] = src[x];
    } else {
        for (uint32_t x = from + lane; x < to; x += CW_LANES) L.ring[x & L.rmask] = src[x];
    }
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
    L.sl = (uint32_t *)cur;                 cur += CW_LANES * 4u;
    L.bl = (uint32_t *)cur;                 cur += CW_LANES * 4u;
    L.head = (HeadT *)cur;                  cur += CW_HBUCKETS * sizeof(HeadT);
    L.chain = (uint16_t *)cur;

    const uint32_t lane = threadIdx.x;
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
    for (uint32_t k = lane; k < CW_HBUCKETS; k += CW_LANES) L.head[k] = NONE;
    uint32_t loaded = n < ring_bytes ? n : ring_bytes;
    cw_fill(L, src, 0u, loaded);
    __syncthreads();

    uint32_t P = 0;          /* next parse position (window start) */
    uint32_t H0 = 0;         /* output index of the open run's header */
    uint32_t c0 = 0;         /* literals in the open run (< 32) */
    bool fail = false;

    while (P + 2u < n) {     /* main loop: src/lzf_c.c:145 */
        /* keep the ring ahead: the window, its match extensions and the
         * 8 KiB back-reference span must be resident */
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

        const uint32_t lim_lane = (n - 2u - P) < CW_LANES ? (n - 2u - P) : CW_LANES;
        const uint32_t p = P + lane;
        const bool valid = lane < lim_lane;
        const uint32_t tri = L.rd4(p) & 0xFFFFFFu;
        const uint32_t s = valid ? slot_of(tri) : 0xFFFFFFFFu;
        const uint32_t b = valid ? hbucket(s) : 0u;
        const uint32_t key = b & (CW_KEYS - 1u);
        L.sl[lane] = s;
        L.bl[lane] = b;
        if (valid) atomicOr(&L.keymask[key], 1ull << lane);
        __syncthreads();
        const uint64_t M = valid ? L.keymask[key] : 0ull;
        const uint32_t head_old = valid ? (uint32_t)L.head[b] : 0u;
        __syncthreads();
        if (valid) L.keymask[key] = 0ull;

        /* 1. nearest earlier window lane with the same slot */
        int prevW = -1;
        {
            uint64_t cand = M & lanemask_lt(lane);
            while (cand) {
                uint32_t j = 63u - __builtin_clzll(cand);
                if (L.sl[j] == s) { prevW = (int)j; break; }
                cand &= ~(1ull << j);
            }
        }
        /* 2. exact table lookup for positions < P */
        uint32_t ref = 0xFFFFFFFFu;
        if (prevW >= 0) {
            ref = P + (uint32_t)prevW;
        } else if (valid && head_old != (uint32_t)NONE) {
            uint32_t q = head_old;
            while (p - q <= LZF_WINDOW) {
                if (slot_of(L.rd4(q) & 0xFFFFFFu) == s) { ref = q; break; }
                uint32_t d = L.chain[q & (CW_CHAIN - 1u)];
                if (d == 0u) break;
                q -= d;
            }
        }
        /* 3. match test (src/lzf_c.c:151-166) and length (169-209) */
        bool match = valid && ref != 0xFFFFFFFFu && ref > 0u && (p - ref - 1u) < LZF_WINDOW &&
                     p + 4u < n && (L.rd4(ref) & 0xFFFFFFu) == tri;
        uint32_t lim = 0, kcap = 0, m = 1;
        bool exact = true;
        if (match) {
            uint32_t maxlen = n - p - 2u;
            if (maxlen > LZF_MAX_REF) maxlen = LZF_MAX_REF;
            lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
            uint32_t room = lim_lane - lane;       /* a jump >= room leaves the window */
            kcap = lim < room ? lim : room;
            uint32_t k = 3u;
            while (k < kcap) {
                uint32_t x = L.rd4(p + k) ^ L.rd4(ref + k);
                uint32_t rem = kcap - k;
                if (rem < 4u) x |= 0xFFFFFFFFu << (8u * rem);
                if (x) { k += (uint32_t)__builtin_ctz(x) >> 3; break; }
                k += 4u;
            }
            if (k > kcap) k = kcap;
            m = k;
            exact = (kcap == lim) || (k < kcap);
        }

        /* 4. the parse orbit: scalar walk over match lanes */
        const uint64_t MM = __ballot(match) & lanemask_lt(lim_lane);
        const uint64_t NX = __ballot(!exact);
        uint64_t V = 0, MMV = 0, INTR = 0, TAIL = 0;
        uint32_t seg = 0, i0 = 0;
        uint32_t segH0 = H0;
        int segBase = (int)c0;
        uint32_t recH0 = segH0;          /* lane k holds segment k's record */
        int recBase = segBase;
        int exitLane = -1;
        uint32_t end = lim_lane;
        for (;;) {
            uint64_t rest = MM & ~lanemask_lt(i0);
            if (!rest) {
                V |= range_mask(i0, lim_lane);
                end = lim_lane;
                break;
            }
            uint32_t j = (uint32_t)__builtin_ctzll(rest);
            V |= range_mask(i0, j + 1u);
            MMV |= 1ull << j;
            uint32_t mj = __builtin_amdgcn_readlane(m, j);
            if (j + mj >= lim_lane || ((NX >> j) & 1ull)) {
                exitLane = (int)j;
                end = j;
                break;
            }
            uint32_t R = (uint32_t)(segBase + (int)j);
            uint32_t nf = segH0 + 1u + R + (R >> 5);
            uint32_t T = nf - ((R & 31u) == 0u ? 1u : 0u);
            uint32_t t = (mj - 2u < 7u) ? 2u : 3u;
            if (mj > 3u) INTR |= range_mask(j + 1u, j + mj - 2u);
            TAIL |= (3ull << (j + mj - 2u));
            segH0 = T + t;
            i0 = j + mj;
            segBase = -(int)i0;
            seg++;
            if (lane == seg) { recH0 = segH0; recBase = segBase; }
        }

        /* 5. speculation check: prevW must not be a skipped interior */
        const bool visited = (V >> lane) & 1ull;
        const bool bad = visited && prevW >= 0 && ((INTR >> (uint32_t)prevW) & 1ull);
        const uint64_t BAD = __ballot(bad);
        uint32_t acc_end;           /* lanes [0, acc_end) of the parse are accepted */
        bool byMatch = false;
        uint32_t mfull = 0;
        if (BAD) {
            acc_end = (uint32_t)__builtin_ctzll(BAD);
        } else if (exitLane >= 0) {
            acc_end = (uint32_t)exitLane + 1u;
            byMatch = true;
            /* full length of the exiting match, whole wave, 256 B per step */
            const uint32_t j = (uint32_t)exitLane;
            const uint32_t pj = P + j;
            const uint32_t rj = __builtin_amdgcn_readlane(ref, j);
            const uint32_t limj = __builtin_amdgcn_readlane(lim, j);
            uint32_t kb = __builtin_amdgcn_readlane(m, j);
            mfull = limj;
            if (kb < limj) {
                for (;;) {
                    uint32_t kk = kb + 4u * lane;
                    uint32_t x = 0;
                    if (kk < limj) {
                        x = L.rd4(pj + kk) ^ L.rd4(rj + kk);
                        uint32_t rem = limj - kk;
                        if (rem < 4u) x |= 0xFFFFFFFFu << (8u * rem);
                    }
                    uint64_t hit = __ballot(x != 0u);
                    if (hit) {
                        uint32_t fl = (uint32_t)__builtin_ctzll(hit);
                        uint32_t xf = __builtin_amdgcn_readlane(x, fl);
                        mfull = kb + 4u * fl + ((uint32_t)__builtin_ctz(xf) >> 3);
                        break;
                    }
                    kb += 4u * CW_LANES;
                    if (kb >= limj) break;
                }
            } else {
                mfull = kb;
            }
            if (mfull > limj) mfull = limj;
        } else {
            acc_end = end;
        }
        const uint64_t ACC = lanemask_lt(acc_end);

        /* 6. emission of the accepted lanes */
        const uint32_t segOf = __builtin_amdgcn_mbcnt_hi((uint32_t)(MMV >> 32),
                                                         __builtin_amdgcn_mbcnt_lo((uint32_t)MMV, 0u));
        const uint32_t myH0 = (uint32_t)__shfl((int)recH0, (int)segOf);
        const int myBase = __shfl(recBase, (int)segOf);
        bool lfail = false;
        if ((ACC >> lane) & 1ull & (V >> lane)) {
            const uint32_t R = (uint32_t)(myBase + (int)lane);
            if (!((MMV >> lane) & 1ull)) {
                uint32_t pos = myH0 + 1u + R + (R >> 5);
                if (pos >= cap) {
                    lfail = true;                                   /* src/lzf_c.c:263 */
                } else {
                    dst[pos] = L.ring[p & L.rmask];
                    if ((R & 31u) == 31u) dst[pos - 32u] = 31u;     /* rollover header */
                }
            } else {
                uint32_t ml = (byMatch && (int)lane == exitLane) ? mfull : m;
                uint32_t nf = myH0 + 1u + R + (R >> 5);
                uint32_t T = nf - ((R & 31u) == 0u ? 1u : 0u);
                if (T + 4u >= cap) {
                    lfail = true;                                   /* src/lzf_c.c:176 */
                } else {
                    if (R & 31u) dst[myH0 + 33u * (R >> 5)] = (uint8_t)((R & 31u) - 1u);
                    uint32_t off = p - ref - 1u;
                    uint32_t Lc = ml - 2u;
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

        /* carry the cursor state to the next window */
        uint32_t Pn;
        uint64_t INS;
        uint32_t t0 = 0xFFFFFFFFu, t1 = 0xFFFFFFFFu;   /* out-of-window tail inserts */
        if (byMatch) {
            const uint32_t j = (uint32_t)exitLane;
            const uint32_t sj = __builtin_amdgcn_readlane(segOf, j);
            const uint32_t h0 = __builtin_amdgcn_readlane(recH0, sj);
            const int bs = __builtin_amdgcn_readlane(recBase, sj);
            const uint32_t R = (uint32_t)(bs + (int)j);
            const uint32_t nf = h0 + 1u + R + (R >> 5);
            const uint32_t T = nf - ((R & 31u) == 0u ? 1u : 0u);
            H0 = T + ((mfull - 2u < 7u) ? 2u : 3u);
            c0 = 0u;
            Pn = P + j + mfull;
            INS = (V | TAIL) & ACC;
            if (Pn + 2u < n) {                 /* src/lzf_c.c:229-247 */
                uint32_t a = j + mfull - 2u, c = j + mfull - 1u;
                if (a < CW_LANES) INS |= 1ull << a; else t0 = P + a;
                if (c < CW_LANES) INS |= 1ull << c; else t1 = P + c;
            }
        } else {
            const uint32_t sE = (uint32_t)__builtin_popcountll(MMV & ACC);
            const uint32_t h0 = __builtin_amdgcn_readlane(recH0, sE);
            const int bs = __builtin_amdgcn_readlane(recBase, sE);
            const uint32_t R = (uint32_t)(bs + (int)acc_end);
            H0 = h0 + 33u * (R >> 5);
            c0 = R & 31u;
            Pn = P + acc_end;
            INS = (V | TAIL) & ACC;
        }

        /* 7. insert the window's inserted positions (increasing order) */
        const bool ins = (INS >> lane) & 1ull;
        if (ins) {
            const uint64_t same = M & INS & ~(1ull << lane);
            int prevI = -1;
            bool last = true;
            for (uint64_t c = same; c;) {
                uint32_t j = (uint32_t)__builtin_ctzll(c);
                c &= c - 1ull;
                if (L.bl[j] != b) continue;
                if (j < lane) prevI = (int)j;
                else { last = false; break; }
            }
            uint32_t d;
            if (prevI >= 0) d = lane - (uint32_t)prevI;
            else if (head_old != (uint32_t)NONE && p - head_old <= LZF_WINDOW) d = p - head_old;
            else d = 0u;
            L.chain[p & (CW_CHAIN - 1u)] = (uint16_t)d;
            if (last) L.head[b] = (HeadT)p;
        }
        __syncthreads();
        if (t0 != 0xFFFFFFFFu || t1 != 0xFFFFFFFFu) {
            if (lane == 0) {
                for (int k = 0; k < 2; k++) {
                    uint32_t x = k ? t1 : t0;
                    if (x == 0xFFFFFFFFu) continue;
                    uint32_t bx = hbucket(slot_of(L.rd4(x) & 0xFFFFFFu));
                    uint32_t h = (uint32_t)L.head[bx];
                    L.chain[x & (CW_CHAIN - 1u)] =
                        (uint16_t)((h != (uint32_t)NONE && x - h <= LZF_WINDOW) ? x - h : 0u);
                    L.head[bx] = (HeadT)x;
                }
            }
            __syncthreads();
        }
        P = Pn;
    }

    /* tail: src/lzf_c.c:276-293 */
    if (!fail) {
        uint32_t o = H0 + 1u + c0;
        if (o + 3u > cap) fail = true;
    }
    if (fail) {
        if (lane == 0) bt.out_len[v] = 0u;
        return;
    }
    const uint32_t ntail = n > P ? n - P : 0u;      /* 0..2 */
    if (lane < ntail) {
        uint32_t R = c0 + lane;
        uint32_t pos = H0 + 1u + R + (R >> 5);
        uint32_t byte = loaded > P + lane ? L.rd1(P + lane) : src[P + lane];
        dst[pos] = (uint8_t)byte;
        if ((R & 31u) == 31u) dst[pos - 32u] = 31u;
    }
    if (lane == 0) {
        uint32_t R = c0 + ntail;
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
    uint32_t ring = ring_for(b.max_len);
    size_t lds = ring + CW_KEYS * 8u + 2u * CW_LANES * 4u + CW_HBUCKETS * sizeof(HeadT) +
                 CW_CHAIN * sizeof(uint16_t);
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

/*
 * lzf_stream.hip -- the "stream" cand kernel of the LZF compressor for gfx950:
 * the same-slot predecessor q1(p) of every position p (the latest earlier
 * position with p's 16-bit slot, src/lzf_c.c:147-149) and how far p's bytes
 * agree with q1's, as the u16 cand words the lane parse reads
 * (lzf_parse_lane_kernel, lzf_lane.hip).
 *
 * Like lzf_cand_table_kernel (lzf_cand.hip) it keeps the reference's exact
 * table T[65536] in LDS and updates it by lane-ordered ds_mskor_rtn_b32
 * exchanges, one value position per lane, 15 windows of 64 positions per
 * step.  The difference is that a workgroup runs its values as ONE STREAM:
 * value k's windows follow value k-1's in the same pipeline, so a value
 * costs its own windows only -- no table clear and no pipeline fill and
 * drain per value, which for 4 KiB values is more than half the steps.
 *
 * T holds stream positions mod 65536 and is never cleared after the start.
 * A lane at stream position g reads the old entry r and takes
 * q = g - ((g - r) mod 65536), the latest position below g with those low
 * bits.  q is p's true same-slot predecessor exactly when q's own slot is
 * p's: if the latest same-slot position L lies within 65536 positions, the
 * entry is L and q = L; if L is older (or absent), no position in the last
 * 65536 has p's slot, so whatever q the stale entry names has another slot.
 * A q outside p's value or window, or at the value's first position (never
 * a ref, src/lzf_c.c:155 `ref > in_data`), gives no candidate.  The slot
 * test reads the 8 bytes at q that the agreement needs anyway.
 */
#include <type_traits>

#include "lzf_dev.h"

#define KS_WINS   15u                        /* worker waves = windows per block */
#define KS_BLK    (64u * KS_WINS)
#define KS_THR    (64u * (KS_WINS + 1u))
#define KS_PF     4u                         /* blocks of input in flight (the step loop's unroll) */
#define KS_CL     2u                         /* steps from the agreement load to its use */

__device__ __forceinline__ uint32_t ks_lds_addr(const void *p)
{
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void *)p;
}

/* the block's 15 exchanges in window (= stream position) order, one wait at
 * the end; later groups take earlier results as in-out operands so nothing
 * reads a result before the wait (lzf_wparse.hip has the same step) */
#define KSX(i_) "ds_mskor_rtn_b32 %" #i_ ", %[a" #i_ "], %[m" #i_ "], %[d" #i_ "]\n\t"
#define KSI(i_, o_) [a##i_] "v"(a[(o_) + i_]), [m##i_] "v"(m[(o_) + i_]), [d##i_] "v"(d[(o_) + i_])
__device__ __forceinline__ void ks_xchg15(uint32_t (&r)[15], const uint32_t (&a)[15], const uint32_t (&m)[15],
                                          const uint32_t (&d)[15])
{
    asm volatile(KSX(0) KSX(1) KSX(2) KSX(3) KSX(4)
                 : "=&v"(r[0]), "=&v"(r[1]), "=&v"(r[2]), "=&v"(r[3]), "=&v"(r[4])
                 : KSI(0, 0), KSI(1, 0), KSI(2, 0), KSI(3, 0), KSI(4, 0)
                 : "memory");
    asm volatile(KSX(0) KSX(1) KSX(2) KSX(3) KSX(4)
                 : "=&v"(r[5]), "=&v"(r[6]), "=&v"(r[7]), "=&v"(r[8]), "=&v"(r[9]),
                   "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4])
                 : KSI(0, 5), KSI(1, 5), KSI(2, 5), KSI(3, 5), KSI(4, 5)
                 : "memory");
    asm volatile(KSX(0) KSX(1) KSX(2) KSX(3) KSX(4) "s_waitcnt lgkmcnt(0)"
                 : "=&v"(r[10]), "=&v"(r[11]), "=&v"(r[12]), "=&v"(r[13]), "=&v"(r[14]),
                   "+v"(r[0]), "+v"(r[1]), "+v"(r[2]), "+v"(r[3]), "+v"(r[4]),
                   "+v"(r[5]), "+v"(r[6]), "+v"(r[7]), "+v"(r[8]), "+v"(r[9])
                 : KSI(0, 10), KSI(1, 10), KSI(2, 10), KSI(3, 10), KSI(4, 10)
                 : "memory");
}
#undef KSX
#undef KSI

/* windows of a value: positions 0 .. n-3 in windows of 64.  A value the
 * parse refuses gets none, and so does one of fewer than 8 bytes (its few
 * words come from ks_tiny): every window's loads are then plain clamped
 * 8-byte loads inside its value, with no branch for the compiler to drain */
__device__ __forceinline__ uint32_t ks_windows(uint32_t n, uint32_t max_len)
{
    return (n >= 8u && n <= max_len) ? (n - 2u + 63u) >> 6 : 0u;
}

/* cand words of a value of 3..7 bytes, directly: per position the latest
 * earlier position with its slot, and the agreement of their bytes */
__device__ __noinline__ void ks_tiny(const uint8_t *src, uint32_t n, uint16_t *cand)
{
    uint32_t b[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    for (uint32_t i = 0; i < n; i++) b[i] = src[i];
    for (uint32_t p = 0; p + 2u < n; p++) {
        const uint32_t sp = dv_slot(b[p] | (b[p + 1u] << 8) | (b[p + 2u] << 16));
        uint32_t q = 0xFFFFFFFFu;
        for (uint32_t x = 0; x < p; x++)
            if (dv_slot(b[x] | (b[x + 1u] << 8) | (b[x + 2u] << 16)) == sp) q = x;
        uint32_t word = 0u;
        if (q != 0xFFFFFFFFu && q > 0u) {                   /* position 0 is never a ref */
            uint32_t k = 0u;
            while (k < 8u && p + k < n && b[q + k] == b[p + k]) k++;
            word = ((k < 3u ? 1u : k >= 8u ? 7u : k - 1u) << 13) | (p - q - 1u);
        }
        cand[p] = (uint16_t)word;
    }
}

/* a window of the stream: which value, where (uniform per wave and block);
 * a window past the stream keeps a real value's src and n (so its loads
 * stay inside that value) with live 0 */
struct KsWin {
    uint32_t v;          /* the value */
    uint32_t off_lo, off_hi;   /* its input offset */
    uint32_t n;          /* its length (>= 8) */
    uint32_t lb;         /* the window's first position in the value */
    uint32_t g0;         /* stream position of the value's position 0 */
    uint32_t live;       /* 0: past the stream */
};
__device__ __forceinline__ uint32_t ks_u(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ const uint8_t *ks_src(const LzfBatch &bt, const KsWin &d)
{
    return bt.in + (((uint64_t)d.off_hi << 32) | d.off_lo);
}

/* 8 bytes for position pp of a value of n >= 8 bytes: the raw load from
 * min(pp, n - 8) (inside the value) -- and, where it is used, ks_fix shifts
 * the bytes into place.  The shift stays out of the load's step, so the
 * compiler counts the load in flight instead of waiting for it there. */
__device__ __forceinline__ uint2 ks_ld(const uint8_t *src, uint32_t n, uint32_t pp)
{
    return dv_ld8(src + (pp + 8u <= n ? pp : n - 8u));
}
__device__ __forceinline__ uint2 ks_fix(uint2 v, uint32_t n, uint32_t pp)
{
    const uint32_t sh = pp + 8u <= n ? 0u : pp - (n - 8u);
    const uint64_t x = ((uint64_t)v.y << 32) | v.x;
    const uint64_t y = sh < 8u ? x >> (8u * sh) : 0ull;
    return make_uint2((uint32_t)y, (uint32_t)(y >> 32));
}

template <uint32_t V> struct KsIc { static constexpr uint32_t value = V; };

/* -DKS_TIMING (diagnostic builds): cycles per phase summed over waves in
 * ks_times[]: [0] table wave B, [1] table wave loads, [2] table wave
 * barrier, [3] C2, [4] C1 (with Q), [5] A, [6] worker loads + cursor,
 * [7] worker barrier, [8] steps (every wave) */
#ifdef KS_TIMING
__device__ unsigned long long ks_times[16];
extern "C" int lzf_gpu_debug_ks(unsigned long long *out16, int reset)
{
    hipError_t e = hipMemcpyFromSymbol(out16, HIP_SYMBOL(ks_times), sizeof(ks_times));
    if (e == hipSuccess && reset) {
        unsigned long long z[16] = {0};
        e = hipMemcpyToSymbol(HIP_SYMBOL(ks_times), z, sizeof(z));
    }
    return e == hipSuccess ? 0 : -2;
}
#define KS_T0() uint64_t ks_t = __builtin_amdgcn_s_memtime()
#define KS_TM(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); ks_acc[i] += t_ - ks_t; ks_t = t_; } while (0)
#else
#define KS_T0() ((void)0)
#define KS_TM(i) ((void)0)
#endif

/* agreement code of k equal bytes (src/lzf_c.c:151-158 and the parse's
 * walk): 1 differ within 3, 2..6 exactly k (3..7), 7 at least 8 */
__device__ __forceinline__ uint32_t ks_code(uint32_t k) { return k < 3u ? 1u : (k >= 8u ? 7u : k - 1u); }

/* agreement of 8 bytes a (at p) and b (at q), at most avail = n - p */
#ifndef KS_FFBL
#define KS_FFBL 1
#endif
__device__ __forceinline__ uint32_t ks_agree(uint2 a, uint2 b, uint32_t avail)
{
#if KS_FFBL
    /* v_ffbl gives the lowest set bit or ~0 for none: min3(ffbl(lo),
     * ffbl(hi) | 32, 64) is the first differing bit, 64 for none (round 5:
     * no 64-bit compare and select) */
    uint32_t fl, fh;
    asm("v_ffbl_b32 %0, %1" : "=v"(fl) : "v"(a.x ^ b.x));
    asm("v_ffbl_b32 %0, %1" : "=v"(fh) : "v"(a.y ^ b.y));
    const uint32_t k = min(min(fl, fh | 32u), 64u) >> 3;
#else
    const uint64_t x = ((uint64_t)(a.y ^ b.y) << 32) | (uint64_t)(a.x ^ b.x);
    const uint32_t k = x ? (uint32_t)__builtin_ctzll(x) >> 3 : 8u;
#endif
    return k < avail ? k : avail;
}

/* the latest stream position below g whose low 16 bits are r (g itself when
 * r == g mod 65536: no candidate) */
__device__ __forceinline__ uint32_t ks_back(uint32_t g, uint32_t r) { return g - ((g - r) & 0xFFFFu); }

/* One workgroup per CU, persistent over the values blockIdx.x + k * gridDim.x.
 * Wave 0 is the table wave, waves 1..15 are workers; window w of the
 * workgroup's stream is worker 1 + w % 15's in block w / 15.  Block t goes
 * through
 *   step t      A(t)   worker: slot of its window's positions -> S[t%2]
 *   step t+1    B(t)   table wave: the 15 exchanges in order -> O
 *   step t+2    C1(t)  worker: q1 (and, REC, q2 = q1's own old entry) from
 *                      O / Q, window and value tests; agreement loads issued
 *   step t+3    (REC) Q <- O of block t
 *   step t+4    C2(t)  worker: slot tests, agreements, the cand word (u16,
 *                      lzf_parse_lane_kernel) or (REC) the two-link record
 *                      (u32, lzf_parse_rec_kernel) stored
 * with one workgroup barrier per step.
 * REC: q2 of p is q1's same-slot predecessor.  q1's old entry lies in O
 * (blocks t and t-1, three O buffers) or in the ring Q of the last 8192
 * stream positions' entries, and q2 passes the same tests as q1 plus its
 * own slot test (its slot must be q1's, which is p's). */
template <bool REC>
__global__ __launch_bounds__(KS_THR) void lzf_cand_stream_kernel(LzfBatch bt, uint8_t *out, uint64_t ostride)
{
    constexpr uint32_t NO = REC ? 3u : 2u;      /* O buffers */
    __shared__ __attribute__((aligned(16))) uint16_t T[LZF_SLOTS + 64u];   /* + one dummy slot per lane */
    /* S: REC [slot | active << 16] (the table wave makes the operands: LDS
     * is short); else the exchange operands [T dword address | half, data] */
    __shared__ std::conditional_t<REC, uint32_t, uint2> S[2u * KS_BLK];
    /* O: old entry returned to each position of a block; REC: Q, the ring of
     * the last 8192 positions' old entries, right in front of it */
    __shared__ uint16_t QO[(REC ? LZF_WINDOW : 0u) + NO * KS_BLK];
    uint16_t *const O = QO + (REC ? LZF_WINDOW : 0u);
    uint16_t *const Q = QO;
    __shared__ __attribute__((aligned(16))) uint32_t D[KS_PF][KS_WINS][8];   /* windows of blocks in flight, for C1 */
    /* the wave index through readfirstlane: branches on it are scalar, so the
     * windows' fields stay in scalar registers */
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6)), j = w - 1u;
    const uint32_t G = gridDim.x;

    for (uint32_t k = tid; k < (LZF_SLOTS + 64u) / 8u; k += KS_THR) ((uint4 *)T)[k] = make_uint4(0, 0, 0, 0);

    /* the stream's length in windows (every wave computes it: uniform) */
    uint32_t nw_lane = 0u;
    for (uint32_t v = blockIdx.x + lane * G; v < bt.count; v += 64u * G) {
        const uint32_t n = bt.in_len[v];
        nw_lane += ks_windows(n, bt.max_len);
        /* the record parse takes values below 16 bytes whole (k3_small) */
        if (!REC && w == 0u && n >= 3u && n < 8u && n <= bt.max_len)
            ks_tiny(bt.in + bt.in_off[v], n, (uint16_t *)out + (uint64_t)v * ostride);
    }
#pragma unroll
    for (uint32_t o = 32u; o >= 1u; o >>= 1) nw_lane += (uint32_t)__shfl_xor((int)nw_lane, (int)o);
    const uint32_t nwin = (uint32_t)__builtin_amdgcn_readfirstlane((int)nw_lane);
    const uint32_t nb = (nwin + KS_WINS - 1u) / KS_WINS;
    __syncthreads();
    if (nwin == 0u) return;

    /* worker cursor over the stream's values: the current value cv covers
     * windows [wbeg, wend); the next one's length and offset are read one
     * value ahead with scalar loads (constant address space: the kernel
     * never writes them), so advancing rarely waits */
    const __attribute__((address_space(4))) uint32_t *cin_len =
        (const __attribute__((address_space(4))) uint32_t *)bt.in_len;
    const __attribute__((address_space(4))) uint64_t *cin_off =
        (const __attribute__((address_space(4))) uint64_t *)bt.in_off;
    const uint32_t vlast = bt.count - 1u;
    uint32_t cv = 0u, cn = 0u, wbeg = 0u, wend = 0u;
    uint64_t coff = 0u;
    uint32_t nv = blockIdx.x;
    uint32_t nn = cin_len[nv];
    uint64_t noff = cin_off[nv];
    /* the window w_ of the stream (w_ < nwin), advancing the cursor */
    const auto window = [&](uint32_t w_) {
        KsWin d;
        while (w_ >= wend) {
            cv = nv;
            cn = nn;
            coff = noff;
            wbeg = wend;
            wend += ks_windows(cn, bt.max_len);
            nv = cv + G;
            const uint32_t vi = nv < vlast ? nv : vlast;
            nn = nv <= vlast ? cin_len[vi] : 0u;
            noff = cin_off[vi];
        }
        d.v = cv;
        d.off_hi = (uint32_t)(coff >> 32);
        d.off_lo = (uint32_t)coff;
        d.n = cn;
        d.lb = 64u * (w_ - wbeg);
        d.g0 = 64u * wbeg;
        d.live = 1u;
        return d;
    };
    /* the window w_, or (past the stream) the last real one, not live */
    KsWin last{};
    const auto window_or_none = [&](uint32_t w_) {
        if (w_ < nwin) last = window(w_);
        else last.live = 0u;
        return last;
    };

    /* Every wave runs a cursor and issues the step's loads -- the table wave
     * shadows worker 1 -- so the loads sit after the role branch, where no
     * register holding one in flight is merged (a merge copy would wait for
     * it).  Prefetched windows: block t at slot t % KS_PF, in scalar
     * registers; the windows of blocks t-1 and t-2 for C1 in LDS (D). */
    const uint32_t jj = w ? j : 0u;
    /* the stream's first window (nwin > 0) stands in for windows past the
     * stream until a later one is taken (its loads stay inside a value of
     * at least 8 bytes); then the cursor starts over */
    last = window(0u);
    cv = cn = wbeg = wend = 0u;
    coff = 0u;
    nv = blockIdx.x;
    nn = cin_len[nv];
    noff = cin_off[nv];
    KsWin pw[KS_PF];
    uint2 pa[KS_PF], aa[KS_PF];
    [[maybe_unused]] uint32_t as_[KS_PF] = {0u, 0u, 0u, 0u};   /* slot of p, with aa (KS_OPT) */
#pragma unroll
    for (uint32_t s = 0; s < KS_PF; s++) {
        pw[s] = window_or_none(KS_WINS * s + jj);
        pa[s] = ks_ld(ks_src(bt, pw[s]), pw[s].n, pw[s].lb + lane);
        aa[s] = make_uint2(0u, 0u);
    }
    /* C1 -> C2 state, KS_CL sets (q2: REC only) */
    uint32_t c_v[KS_CL], c_n[KS_CL];
    uint32_t c_p[KS_CL], c_q[KS_CL], c_q2[KS_CL];
    uint2 c_a[KS_CL], c_b[KS_CL], c_b2[KS_CL];
    [[maybe_unused]] uint32_t c_s[KS_CL] = {0u, 0u};
#pragma unroll
    for (uint32_t i = 0; i < KS_CL; i++) {
        c_v[i] = c_n[i] = 0u;
        c_p[i] = 0xFFFFFFFFu;
        c_q[i] = c_q2[i] = 0u;
        c_a[i] = c_b[i] = c_b2[i] = make_uint2(0u, 0u);
    }
    const uint32_t tb = ks_lds_addr(T);

#ifdef KS_TIMING
    uint64_t ks_acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#endif
    const auto step = [&](auto ps, uint32_t t) {
        constexpr uint32_t PS = decltype(ps)::value;             /* t % KS_PF */
        constexpr uint32_t CS = PS % KS_CL;
        constexpr uint32_t S2 = (PS + KS_PF - 2u) % KS_PF;        /* block t-2 */
        KS_T0();
        /* the agreement loads' addresses: a harmless default inside block t's
         * value, replaced by C1's candidates */
        const uint8_t *lsrc = ks_src(bt, pw[PS]);
        uint32_t ln = pw[PS].n, lq = 0u, lq2 = 0u;
        if (w == 0u) {
            /* ---- B(t-1): the table wave ----------------------------------- */
            if (t >= 1u && t <= nb) {
                const uint32_t k = t - 1u;
                const auto *Sk = S + KS_BLK * (k & 1u);
                uint16_t *Ok = O + KS_BLK * (k % NO);
                uint32_t xa[15], xm[15], xd[15], xr[15], hs[15];
#pragma unroll
                for (uint32_t i = 0; i < 15u; i++) {
                    if constexpr (REC) {
                        /* a position past its value exchanges in its lane's dummy slot */
                        const uint32_t e = Sk[64u * i + lane];
                        const uint32_t h = (e >> 16) ? (e & 0xFFFFu) : LZF_SLOTS + lane;
                        hs[i] = (h & 1u) << 4;
                        xa[i] = tb + 4u * (h >> 1);
                        xm[i] = 0xFFFFu << hs[i];
                        xd[i] = ((KS_BLK * k + 64u * i + lane) & 0xFFFFu) << hs[i];
                    } else {
                        const uint2 e = Sk[64u * i + lane];
                        hs[i] = (e.x & 1u) << 4;
                        xa[i] = e.x & ~1u;
                        xm[i] = 0xFFFFu << hs[i];
                        xd[i] = e.y;
                    }
                }
                ks_xchg15(xr, xa, xm, xd);
#pragma unroll
                for (uint32_t i = 0; i < 15u; i++) Ok[64u * i + lane] = (uint16_t)(xr[i] >> hs[i]);
            }
            KS_TM(0);
        } else {
            /* ---- C2(t-2-KS_CL): slot tests, agreements, the output -------- */
            if (c_p[CS] != 0xFFFFFFFFu) {
                const uint32_t p = c_p[CS], q = c_q[CS], n = c_n[CS];
                const uint2 a = c_a[CS];
                /* no lane within 8 bytes of its value's end: every q < p too,
                 * so the loads were not moved back and need no shift */
                const bool near_end = __ballot(p + 8u > n) != 0ull;
                const uint2 b = near_end ? ks_fix(c_b[CS], n, q) : c_b[CS];
                const uint32_t sp = c_s[CS];
                /* branch-free (every branch costs the wave its exec-mask
                 * juggling): both tests always, the word by selects.  q1: a
                 * stale table entry names a position of another slot */
                const uint32_t k1 = ks_agree(a, b, n - p);
                const bool v1 = q != 0u && (k1 >= 3u || dv_slot(b.x) == sp);
                uint32_t word = v1 ? (ks_code(k1) << 13) | (p - q - 1u) : 0u;
                if constexpr (REC) {
                    const uint32_t q2 = c_q2[CS];
                    const uint2 b2 = near_end ? ks_fix(c_b2[CS], n, q2) : c_b2[CS];
                    const uint32_t k2 = ks_agree(a, b2, n - p);
                    const bool v2 = v1 && q2 != 0u && (k2 >= 3u || dv_slot(b2.x) == sp);
                    word |= v2 ? ((ks_code(k2) << 13) | (p - q2 - 1u)) << 16 : 0u;
                }
                if constexpr (REC)
                    ((uint32_t *)out)[(uint64_t)c_v[CS] * ostride + p] = word;
                else
                    ((uint16_t *)out)[(uint64_t)c_v[CS] * ostride + p] = (uint16_t)word;
            }
            KS_TM(3);
            /* ---- REC: Q <- O of block t-3 ------------------------------ */
            if constexpr (REC) {
                if (t >= 3u && t - 3u < nb) {
                    const uint32_t x = KS_BLK * (t - 3u) + 64u * j + lane;
                    Q[x & (LZF_WINDOW - 1u)] = O[KS_BLK * ((t - 3u) % NO) + 64u * j + lane];
                }
            }
            /* ---- C1(t-2): the candidates from the table's old entries ----- */
            c_p[CS] = 0xFFFFFFFFu;
            if (t >= 2u && t - 2u < nb) {
                const uint4 d0 = *(const uint4 *)&D[S2][j][0];
                const uint4 d1 = *(const uint4 *)&D[S2][j][4];
                const uint32_t r = O[KS_BLK * ((t - 2u) % NO) + 64u * j + lane];
                const uint32_t dv = ks_u(d0.x), dn = ks_u(d0.w), dlb = ks_u(d1.x), dg0 = ks_u(d1.y);
                const uint32_t dlive = ks_u(d1.z);
                const uint8_t *dsrc = bt.in + (((uint64_t)ks_u(d0.z) << 32) | ks_u(d0.y));
                const uint32_t p = dlb + lane;
                if (dlive && p < dn - 2u) {
                    const uint32_t g = dg0 + p;
                    const uint32_t qg = ks_back(g, r);
                    /* inside the value, not its position 0, inside p's window */
                    const bool ok = qg != g && qg > dg0 && g - qg <= LZF_WINDOW;
                    c_p[CS] = p;
                    c_q[CS] = ok ? qg - dg0 : 0u;
                    c_a[CS] = aa[S2];
                    c_s[CS] = as_[S2];
                    lq = ok ? qg - dg0 : p;
                    if constexpr (REC) {
                        /* q1's own old entry: block t-2 or t-3 in O, else Q */
                        const uint32_t B = KS_BLK * (t - 2u);   /* stream position of block t-2 */
                        const uint32_t iq = qg >= B ? KS_BLK * ((t - 2u) % NO) + (qg - B)
                                          : qg + KS_BLK >= B ? KS_BLK * ((t + NO - 3u) % NO) + (qg + KS_BLK - B)
                                                             : 0xFFFFFFFFu;
                        const uint32_t r2 = iq != 0xFFFFFFFFu ? O[iq] : Q[qg & (LZF_WINDOW - 1u)];
                        const uint32_t q2g = ks_back(qg, r2);
                        const bool ok2 = ok && q2g != qg && q2g > dg0 && g - q2g <= LZF_WINDOW;
                        c_q2[CS] = ok2 ? q2g - dg0 : 0u;
                        lq2 = ok2 ? q2g - dg0 : p;
                    }
                }
                c_n[CS] = dn;
                c_v[CS] = dv;
                lsrc = dsrc;
                ln = dn;
            }
            KS_TM(4);
            /* ---- A(t): slots of the worker's window of block t ------------ */
            if (t < nb) {
                const KsWin &d = pw[PS];
                const uint32_t p = d.lb + lane;
                const bool act = d.live && p < d.n - 2u;
                const uint2 pb = d.lb + 64u + 8u <= d.n ? pa[PS] : ks_fix(pa[PS], d.n, p);
                const uint32_t sl = dv_slot(pb.x);
                if constexpr (REC) {
                    /* the stream position of this lane is the block's (the
                     * table wave's data), which is d.g0 + p for a live lane */
                    S[KS_BLK * (t & 1u) + 64u * j + lane] = act ? (sl | (1u << 16)) : 0u;
                } else {
                    const uint32_t h = act ? sl : LZF_SLOTS + lane;
                    const uint32_t data = act ? ((d.g0 + p) & 0xFFFFu) : 0u;
                    S[KS_BLK * (t & 1u) + 64u * j + lane] =
                        make_uint2((tb + 4u * (h >> 1)) | (h & 1u), data << ((h & 1u) << 4));
                }
                if (lane == 0u) {
                    *(uint4 *)&D[PS][j][0] = make_uint4(d.v, d.off_lo, d.off_hi, d.n);
                    *(uint4 *)&D[PS][j][4] = make_uint4(d.lb, d.g0, d.live, 0u);
                }
                aa[PS] = pb;
                as_[PS] = sl;
            }
            KS_TM(5);
        }
        /* ---- the step's loads, every wave: the agreement bytes of C1, then
         * the window of block t + KS_PF --------------------------------------- */
        c_b[CS] = ks_ld(lsrc, ln, lq);
        if constexpr (REC) c_b2[CS] = ks_ld(lsrc, ln, lq2);
        pw[PS] = window_or_none(KS_WINS * (t + KS_PF) + jj);
        pa[PS] = ks_ld(ks_src(bt, pw[PS]), pw[PS].n, pw[PS].lb + lane);
        if (w) KS_TM(6);
        else KS_TM(1);
        __syncthreads();
        if (w) KS_TM(7);
        else KS_TM(2);
#ifdef KS_TIMING
        ks_acc[8]++;
#endif
    };
    for (uint32_t t = 0; t < nb + 2u + KS_CL; t += KS_PF) {
        step(KsIc<0>{}, t);
        step(KsIc<1>{}, t + 1u);
        step(KsIc<2>{}, t + 2u);
        step(KsIc<3>{}, t + 3u);
    }
#ifdef KS_TIMING
    if (lane == 0u)
        for (uint32_t i = 0; i < 9u; i++) atomicAdd(&ks_times[i], (unsigned long long)ks_acc[i]);
#endif
}
static_assert(KS_PF == 4u && KS_CL == 2u, "the step loop is unrolled 4x; C2 runs KS_CL steps after C1");

static uint32_t ks_grid(uint32_t count)
{
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    return count < (uint32_t)cus ? count : (uint32_t)cus;
}

hipError_t lzf_launch_cand_stream(const LzfBatch &b, const LzfLaneScratch &sc, hipStream_t s)
{
    hipLaunchKernelGGL(lzf_cand_stream_kernel<false>, dim3(ks_grid(b.count)), dim3(KS_THR), 0, s, b,
                       (uint8_t *)sc.cand, sc.cstride);
    return hipGetLastError();
}

#ifdef LZF_DIAG   /* the record form: a cross-check of the table generation's kernel 1 */
hipError_t lzf_launch_cand_stream_rec(const LzfBatch &b, const LzfRecScratch &sc, hipStream_t s)
{
    hipLaunchKernelGGL(lzf_cand_stream_kernel<true>, dim3(ks_grid(b.count)), dim3(KS_THR), 0, s, b,
                       (uint8_t *)sc.rec, sc.rstride);
    return hipGetLastError();
}
#endif

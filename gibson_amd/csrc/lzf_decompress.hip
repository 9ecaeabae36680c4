/*
 * lzf_decompress.hip -- token-parallel LZF decoder for gfx950.
 *
 * Replaces src/lzf_d.c:55-149 for batches of independent streams.  A stream
 * is consumed in rounds; a round starts at a token boundary and covers the
 * tokens that START in the next 128 input bytes (CD_ROUND):
 *
 *   1. token boundaries: every lane sizes the tokens that would start at its
 *      two positions of the round (literal c<32: c+2 bytes; back-ref: 2, or 3
 *      when c>>5 == 7); the chain of boundaries is found by pointer doubling
 *      (ds_bpermute) or by a scalar walk over runs of 2-byte tokens, and lane
 *      l ends up holding the start of token l (<= 64 per round);
 *   2. lane l decodes token l (src/lzf_d.c:66-119) and the output offsets
 *      follow from one wave prefix sum (DPP) of the token output lengths;
 *   3. the reference's error checks, in its order (literal: E2BIG then
 *      EINVAL, src/lzf_d.c:72-84; back-ref: EINVAL on a truncated token,
 *      E2BIG, EINVAL on a reference before the output start,
 *      src/lzf_d.c:100-131) -- the first failing token decides errno;
 *   4. the output bytes are produced 64 at a time, one per lane: the owning
 *      token comes from a ballot of token-start marks, the byte from the
 *      LDS input ring (literal) or the LDS output window (back-ref); a
 *      back-ref byte whose source lies in the same 64-byte group (runs,
 *      src/lzf_d.c:137-142 copies byte-serially so overlap replicates) is
 *      resolved by pointer doubling over the group's lanes.  Every group is
 *      stored to HBM as it completes.
 *
 * Steps 1-3 depend on the input alone, step 4 on the output of the rounds
 * before.  Each wave's round is a chain of dependent LDS round trips, and a
 * stream's LDS (the 8 KiB output window) allows ~4 streams per SIMD, so one
 * wave per stream leaves the SIMDs waiting on LDS latency.  `pipe` (the
 * product form) gives a stream two waves: a producer runs steps 1-3 one round
 * ahead and hands the round's token table over in LDS (double-buffered, one
 * workgroup barrier per round); a consumer runs step 4.  `tokpar64` (one wave
 * does everything) stays as the single-wave form.
 */
#include "lzf_internal.h"

#define CD_LANES   64u
#define CD_ROUND   128u             /* input bytes whose token starts one round covers */
/* input ring: a round reads [base, base + CD_ROUND + 33); staging runs in
 * CD_STAGE-byte pieces (one 16-byte load per lane) when the round's reach
 * passes base + 2 * CD_ROUND (loaded < base + 2 * CD_ROUND), so a piece
 * overwrites only bytes before loaded - in_ring + CD_STAGE.  Single wave:
 * ring 512, piece 256, which is < base.  Pipe: the consumer still reads
 * round k's literals, [base_k, base_k + 161), while the producer stages for
 * round k + 1 (base_{k+1} <= base_k + 160): ring 1024, piece 512, so a piece
 * overwrites only bytes before base_{k+1} - 256 < base_k */
#define CD_IN_RING1 512u
#define CD_IN_RING2 1024u
/* output window ring: back-references reach at most 8192 bytes back
 * (src/lzf_d.c:95, off < 8192), and a group reads all its sources before it
 * writes its 64 bytes, so a ring of 8 KiB suffices: the slots a group
 * overwrites (o - 8192) are read, if at all, by that group alone */
#ifndef CD_OUT_MAX
#define CD_OUT_MAX 8192u
#endif
/* Measured and removed (same-process A/Bs, all bit-exact):
 * a scalar walk over size-2 runs for token discovery (no faster); groups
 * inside one long token copied without the owner search (slower on every
 * shape: the per-round check and per-group readlanes sit on the consumer's
 * critical path); the next group's owner search overlapped with the current
 * group's byte reads (slower: the consumer is issue-bound at 8 waves per
 * SIMD).  Kept: completed output leaves the LDS window in 16-byte pieces per
 * lane, a flush unit (1 KiB, or half the window) at a time. */
/* decoder form: 1 = pipe (producer + consumer wave per stream), 0 = tokpar64 */
#ifndef CD_PIPE
#define CD_PIPE    1
#endif

/* 16 bytes from p, of which `avail` (< 16: the rest reads as zero) exist */
__device__ __forceinline__ uint4 cd_ld16(const uint8_t *p, uint32_t avail)
{
    uint4 v;
    if (avail >= 16u) {
        __builtin_memcpy(&v, p, 16);
        return v;
    }
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; k < avail; k++) w[k >> 2] |= (uint32_t)p[k] << (8u * (k & 3u));
    return make_uint4(w[0], w[1], w[2], w[3]);
}

/* v shifted down by d bytes (0 < d < 16), zeros in from the top */
__device__ __forceinline__ uint4 cd_shr16(uint4 v, uint32_t d)
{
    uint64_t lo = ((uint64_t)v.y << 32) | v.x, hi = ((uint64_t)v.w << 32) | v.z;
    if (d >= 8u) {
        lo = hi >> (8u * (d - 8u));
        hi = 0u;
    } else {
        lo = (lo >> (8u * d)) | (hi << (64u - 8u * d));
        hi >>= 8u * d;
    }
    return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

/* the wave's lane mask of a predicate, straight from the compare (HIP's
 * __ballot takes an int, which can cost a select and a compare per use) */
__device__ __forceinline__ uint64_t cd_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ void cd_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

#ifdef CD_TIMING
/* diagnostic build: per role, cycles working and cycles waiting at the
 * pipe's barriers, summed over waves (lzf_gpu_dec_tstat) */
/* 1024 rows of 8 counters, a workgroup adding to row blockIdx.x % 1024: one
 * row for all would serialise ~6 atomics per workgroup at one L2 channel
 * (1 M values of 8 KiB: 88 ms instead of 15) */
#define CD_TROWS 1024u
__device__ unsigned long long cd_tstat[CD_TROWS * 8u];
#endif

/* workgroup barrier with LDS release/acquire (the pipe's hand-over); tw[0]
 * accumulates working cycles, tw[1] waiting ones (CD_TIMING builds) */
__device__ __forceinline__ void cd_barrier(uint64_t *tw = nullptr)
{
#ifdef CD_TIMING
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
#endif
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef CD_TIMING
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    if (tw) {
        tw[0] += t0 - tw[2];
        tw[1] += t1 - t0;
        tw[2] = t1;
    }
#else
    (void)tw;
#endif
}

__device__ __forceinline__ uint32_t cd_incl_sum(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
    return x;
}

__device__ __forceinline__ uint32_t cd_rl(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__device__ __forceinline__ uint32_t cd_tsz(uint32_t c)
{
    return c < 32u ? c + 2u : ((c >> 5) == 7u ? 3u : 2u);
}

/* stage input [base, base + 2 * CD_ROUND) (tokens starting in the round and
 * their literal payloads, <= CD_ROUND - 1 + 33 bytes) into the input ring */
template <uint32_t IN_RING>
__device__ __forceinline__ void cd_stage(uint8_t *inr, const uint8_t *src, uint32_t base, uint32_t avail,
                                         uint32_t &loaded, uint32_t lane)
{
    constexpr uint32_t STAGE = IN_RING / 2u;
    static_assert(STAGE >= 2u * CD_ROUND && STAGE <= 16u * CD_LANES, "one staging piece per round");
    uint32_t need = base + 2u * CD_ROUND;
    if (need > avail) need = avail;
    if (loaded < need) {                 /* need - loaded <= CD_ROUND + 33 <= STAGE */
        uint32_t to = loaded + STAGE;
        if (to > avail) to = avail;
        const uint32_t x = loaded + 16u * lane;   /* loaded is a multiple of 16 here */
        if (x < to) *(uint4 *)(inr + (x & (IN_RING - 1u))) = cd_ld16(src + x, to - x);
        loaded = to;
        cd_fence();
    }
}

/* step 1: lane l gets the round-relative start of token l (CD_ROUND: none).
 * The jump table lives in LDS: jt holds 256 bytes,
 * J(p) for the round's positions p < 128 and 255 ("leaves the round") at
 * [128, 256), so a jump is one ds_read_u8 at the entry itself.  Level b's
 * table is read at J_b(p) to make J_{b+1} and at the lane's rank walk x, and
 * overwritten in place: one wave's LDS operations execute in order, so every
 * lane's reads of level b precede the write.  The rank walk applies level b
 * as the table reaches it (the levels are powers of one map, so they commute):
 * four LDS operations per level (round 3 held the tables in registers, two
 * per lane: two ds_bpermute and their byte extraction per table level plus
 * one per rank level). */
#ifndef CD_PREF
#define CD_PREF 1
#endif
/* the pipe producer's input pieces two rounds ahead (round 5; the kernel) */
#ifndef CD_PREF2
#define CD_PREF2 1
#endif
/* tokpar64: the next staging piece prefetched into registers (round 5) */
#ifndef CD_TPREF
#define CD_TPREF 1
#endif
template <uint32_t V> struct CdPar { static constexpr uint32_t value = V; };
__device__ uint4 cd_dummy16;    /* the idle lanes' load address */
/* CD_CPRIO: issue priority of the pipe's consumer wave (s_setprio).  VALU
 * issue is arbitrated by priority, then age; with the consumer first: Zipf
 * 16.14 -> 15.57 ms, sentence text 12.79 -> 12.10, mixed 7.93 -> 7.99 (the
 * same at 1, 2 or 3; the producer first: 17.23 / 13.52 / 8.07) */
#ifndef CD_CPRIO
#define CD_CPRIO 1
#endif
/* the jump table's 255s above position 127, and token sizes from a 256-byte
 * table, tszt[c] = cd_tsz(c), at jt + 256 (one LDS read instead of six VALU) */
template <bool TSZT = true>
__device__ __forceinline__ void cd_jt_init(uint8_t *jt, uint32_t lane)
{
    *(uint16_t *)(jt + CD_ROUND + 2u * lane) = 0xFFFFu;
    const uint32_t c = 4u * lane;
    if (TSZT)
        *(uint32_t *)(jt + 256u + c) = cd_tsz(c) | (cd_tsz(c + 1u) << 8) | (cd_tsz(c + 2u) << 16) | (cd_tsz(c + 3u) << 24);
}
template <bool TSZT = true>
__device__ __forceinline__ uint32_t cd_discover_lds(const uint8_t *inr, uint32_t imask, uint8_t *jt, uint32_t base,
                                                    uint32_t in_len, uint32_t lane)
{
    const uint32_t pa = 2u * lane, pb = pa + 1u;
    const uint32_t ca = inr[(base + pa) & imask], cb = inr[(base + pb) & imask];
    const uint32_t ta = TSZT ? jt[256u + ca] : cd_tsz(ca), tb = TSZT ? jt[256u + cb] : cd_tsz(cb);
    /* J0 = the next token's start: any entry >= 128 leaves the round (the
     * table holds 255 there, so its first jump gives 255); away from the
     * stream's end no token crosses in_len, so only near it are entries
     * clamped (a round's last token ends at most 127 + 33 bytes in) */
    uint32_t na = pa + ta, nb = pb + tb;
    if (base + CD_ROUND + 33u > in_len) {
        const uint32_t ipa = base + pa;
        if (ipa + ta >= in_len) na = 255u;
        if (ipa + 1u + tb >= in_len) nb = 255u;
    }
    *(uint16_t *)(jt + pa) = (uint16_t)(na | (nb << 8));
    cd_fence();
    uint32_t x = 0;
#pragma unroll
    for (uint32_t b = 0; b < 6u; b++) {
        const uint32_t jx = jt[x];
        if (b < 5u) {
            na = jt[na];
            nb = jt[nb];
            cd_fence();
            *(uint16_t *)(jt + pa) = (uint16_t)__builtin_amdgcn_perm(nb, na, 0x0c0c0400u);   /* na | nb << 8 */
            cd_fence();
        }
        x = ((lane >> b) & 1u) ? jx : x;
    }
    return x >= CD_ROUND ? CD_ROUND : x;
}

/* steps 2-3 for lane l's token: its output offset within the round (rel),
 * the owner info of its output bytes (tinfo: literal -> input ring index
 * o - tinfo, flagged in bit 31; back-ref -> distance), the round's output
 * bytes, and errno of the first failing token (0: none) */
#ifndef CD_PER_RATIO
#define CD_PER_RATIO 4u
#endif
struct CdRound {
    uint32_t rel, tinfo, total;
    uint32_t nbase;          /* the input offset after the round's last token */
    int32_t err;
    uint64_t overlap;        /* lanes whose back-reference repeats its distance CD_PER_RATIO times */
    uint32_t ntok;           /* tokens of the round (lanes 0 .. ntok - 1) */
};

__device__ __forceinline__ CdRound cd_decode(const uint8_t *inr, uint32_t imask, uint32_t base, uint32_t x,
                                             uint32_t O, uint32_t in_len, uint32_t cap)
{
    const bool tok = x < CD_ROUND;
    const uint32_t ip = base + (tok ? x : 0u);
    const uint32_t c = inr[ip & imask];
    const uint32_t b1 = inr[(ip + 1u) & imask], b2 = inr[(ip + 2u) & imask];
    const bool lit = c < 32u;
    const bool l7 = (c >> 5) == 7u;                     /* length in the next byte */
    const uint32_t back = ((c & 31u) << 8) + (l7 ? b2 : b1) + 1u;   /* back-refs only */
    const uint32_t olen = lit ? c + 1u : (c >> 5) + (l7 ? b1 : 0u) + 2u;
    const uint32_t lsrc = ip + 1u;                      /* literals only */
    const uint32_t ol = tok ? olen : 0u;
    const uint32_t incl = cd_incl_sum(ol);
    CdRound r;
    r.rel = incl - ol;
    const uint32_t Ot = O + r.rel;                      /* output offset of my token */
    /* literal: Ot - lsrc, so the consumer's o - tinfo is the input offset
     * of output byte o for both kinds (the flag, 2^31, leaves the ring's
     * low bits alone) */
    r.tinfo = lit ? (((Ot - lsrc) & 0x7FFFFFFFu) | 0x80000000u) : back;
    r.total = cd_rl(incl, 63u);
    /* the round's last token (lane ntok - 1: tokens fill the low lanes) ends the round */
    r.ntok = (uint32_t)__builtin_popcountll(cd_ballot(tok));
    r.nbase = base + cd_rl(x + (lit ? c + 2u : (l7 ? 3u : 2u)), r.ntok - 1u);
    /* away from the stream's end (every token byte of the round, at most
     * base + CD_ROUND + 32, lies inside the input) and with the round's output
     * inside the cap, only a back-reference before the output start can fail */
    int32_t e = 0;
    if (base + CD_ROUND + 33u <= in_len && (uint64_t)O + r.total <= cap) {
        e = (tok && !lit && back > Ot) ? 22 : 0;                            /* :127 */
    } else if (tok) {
        if (lit) {
            if ((uint64_t)Ot + olen > cap) e = 7;                           /* E2BIG  :72 */
            else if ((uint64_t)ip + 1u + olen > in_len) e = 22;             /* EINVAL :79 */
        } else {
            if (ip + 1u >= in_len) e = 22;                                  /* :101 */
            else if ((c >> 5) == 7u && ip + 2u >= in_len) e = 22;          /* :111 */
            else if ((uint64_t)Ot + olen > cap) e = 7;                      /* :121 */
            else if (back > Ot) e = 22;                                     /* :127 */
        }
    }
    const uint64_t EB = cd_ballot(e != 0);
    r.err = EB ? (int32_t)cd_rl((uint32_t)e, (uint32_t)__builtin_ctzll(EB)) : 0;
    /* a run long enough that the shortcut saves doubling steps (CD_PER_RATIO
     * periods or more) */
    r.overlap = cd_ballot(tok && !lit && olen >= CD_PER_RATIO * back);
    return r;
}

/* output bytes [F, E) of the LDS window (ring offset outr_off, mask omask)
 * to dst: 16 bytes per lane, at most `unit` bytes per pass (unit <= 1024,
 * a multiple of 16), then the last < 16 bytes one per lane.  The window
 * still holds every byte of [F, E): E - F stays below half the window */
__device__ __forceinline__ void cd_flush(const uint8_t *lds, uint32_t outr_off, uint32_t omask, uint8_t *dst,
                                         uint32_t &F, uint32_t E, uint32_t lane)
{
    while (E - F >= 16u) {
        const uint32_t x = F + 16u * lane;
        if (x + 16u <= E) {
            uint4 v;
            __builtin_memcpy(&v, lds + outr_off + (x & omask), 16);
            __builtin_memcpy(dst + x, &v, 16);
        }
        const uint32_t nfull = (E - F) & ~15u;
        F += nfull < 16u * CD_LANES ? nfull : 16u * CD_LANES;
    }
    if (F + lane < E) dst[F + lane] = lds[outr_off + ((F + lane) & omask)];
    F = E;
}

/* step 4: the round's output [O, O + total), 64 bytes per step.  Tokens sit
 * in lanes in output order, so the owner of output byte b of a group is
 * (tokens started before the group) + (token starts in the group at or below
 * b) - 1: the starts are marked in LDS with the group's tag (gb + 1, never
 * reused, so the marks need no clearing) and read back as one ballot.  Byte
 * sources are selected without branches (each branch costs the wave its
 * exec-mask juggling); a byte's state is one word -- resolved (bit 16 |
 * value) or the group lane holding its source (bits 8-13, a back-reference
 * into the same group: src/lzf_d.c:137-142 copies byte-serially, so overlap
 * replicates); a doubling step takes over the pointed-to lane's word (a
 * resolved source resolves it, a pending one doubles the pointer).  Idle
 * lanes store their byte to a sink slot; every group goes to HBM as it
 * completes */
/* CD_PERIOD: in a round whose producer flagged a self-overlapping
 * back-reference (distance d < length, a run: src/lzf_d.c:137-142 copies
 * byte-serially, so its bytes repeat with period d), a byte at offset x >= d
 * of such a token takes its source in the token's first period,
 * Ot - d + (x mod d), which lies before the token: a run that started in an
 * earlier group resolves in one read instead of log2(64) doubling steps */
#ifndef CD_PERIOD
#define CD_PERIOD 1
#endif
/* CD_MARKAHEAD: the next group's start marks are written and read while this
 * group's owner lookup is in flight, taking one LDS round trip off the
 * per-group chain: -2.2 % on json4k (tokpar64, latency-bound); the pipe's
 * consumer is issue-bound and gains nothing */
#ifndef CD_MARKAHEAD
#define CD_MARKAHEAD 1
#endif
#ifndef CD_ENTGUARD                 /* the doubling loop's guard read off the entries */
#define CD_ENTGUARD 1
#endif
#ifndef CD_FARB
#define CD_FARB 1
#endif
#ifndef CD_FAR2                     /* FAR's one-compare test, its wait on its own path */
#define CD_FAR2 1
#endif
#ifndef CD_MARKAHEAD_PIPE           /* the pipe's consumer */
#define CD_MARKAHEAD_PIPE 0
#endif
/* FAR (round 5): the window is a ring smaller than the 8 KiB that
 * back-references reach (src/lzf_d.c:95); a source more than a window behind
 * the group is read back from the output in HBM, where the flush put it (the
 * flush lags the group by at most a unit + 64 bytes, less than a window; a
 * workgroup-scope release after each flush makes the stores visible to the
 * wave's own later loads) */
template <uint32_t IN_RING, bool PER = false, bool MA = CD_MARKAHEAD, typename MT = uint32_t, bool FAR = false>
__device__ __forceinline__ void cd_output(uint8_t *lds, uint32_t outr_off, uint32_t omask, MT *mark,
                                             uint32_t sink_off, uint8_t *dst, uint32_t O, uint32_t total, bool tok,
                                             uint32_t Ot, uint32_t tinfo, uint32_t lane, uint32_t &F)
{
    /* a flush unit of the window's completed bytes goes out as soon
     * as it is complete (half the window at most, so no byte is overwritten
     * before it is stored) */
    const uint32_t unit = (omask + 1u) / 2u < 1024u ? (omask + 1u) / 2u : 1024u;
    constexpr uint32_t imask = IN_RING - 1u;
    uint32_t tbase = 0;          /* tokens started before the group */
#ifdef LZF_CD_ABLATE_OUTPUT           /* diagnostic builds only: time discovery alone */
    total = 0u;
#endif
    /* lanes without a token mark slot 64 (never read): their start lies 2^31 away */
    const uint32_t Otm = tok ? Ot : Ot + 0x80000000u;
    uint32_t farb = 0u - (lane + omask + 2u);         /* FAR: tInf - lane - (window + 1) */
#if CD_FARB
    if (FAR) asm volatile("" : "+v"(farb));          /* kept whole: one add per group, not a subtract and an add */
#endif
    /* a start mark holds the token's own start, so it matches only in its
     * group (no per-group tag; position 0, the unwritten marks' 0, always
     * starts a token) */
    uint32_t m = 0u;
    if (MA && total) {
        mark[min(Otm - O, CD_LANES)] = (MT)Otm;       /* without a branch */
        cd_fence();
        m = mark[lane];
    }
    for (uint32_t g = 0; g < total; g += CD_LANES) {
        const uint32_t gb = O + g;                     /* group's first output offset */
        const uint32_t o = gb + lane;
        if (!MA) {
            mark[min(Otm - gb, CD_LANES)] = (MT)Otm;
            cd_fence();
            m = mark[lane];
        }
        const bool mine = (MT)m == (MT)o;   /* 16-bit marks: a stream's output stays below 65536 */
        const uint64_t S = cd_ballot(mine);
        const uint32_t le = __builtin_amdgcn_mbcnt_hi((uint32_t)(S >> 32),
                                                      __builtin_amdgcn_mbcnt_lo((uint32_t)S, 0u)) +
                            (mine ? 1u : 0u);
        const uint32_t k = tbase + le - 1u;
        tbase += (uint32_t)__builtin_popcountll(S);
        const uint32_t tInf = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)tinfo);
        if (MA) {
            /* the next group's marks, in the shadow of this group's LDS
             * chain (they depend on nothing it writes; a group past the
             * round marks slot 64 only: no token starts there) */
            cd_fence();
            mark[min(Otm - (gb + CD_LANES), CD_LANES)] = (MT)Otm;
            cd_fence();
            m = mark[lane];
        }
        const bool lit = (int32_t)tInf < 0;
        uint32_t so = o - tInf;
        if (PER) {                                     /* a round the producer flagged */
            const uint32_t ot = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)Ot);
            const uint32_t x = o - ot;
            if (!lit && x >= tInf) {
                /* x mod d: a float quotient, off by at most one, corrected */
                const uint32_t qf = (uint32_t)((float)x * __builtin_amdgcn_rcpf((float)tInf));
                int32_t r = (int32_t)(x - qf * tInf);
                r = r < 0 ? r + (int32_t)tInf : r;
                r = r >= (int32_t)tInf ? r - (int32_t)tInf : r;
                so = ot - tInf + (uint32_t)r;
            }
        }
        /* the input ring lies right after the window */
        const uint32_t li = IN_RING <= omask + 1u ? (so & imask) | (omask + 1u) : (so & imask) + (omask + 1u);
        const uint32_t a = outr_off + (lit ? li : so & omask);
        const uint32_t q = so - gb;
        uint32_t b = lds[a];
        if (FAR) {
            /* a source more than a window behind the group's start: out of the ring */
#if CD_FAR2
            /* gb - so = tInf - lane for a back-reference (a periodic source
             * only exists for distances < 264); literals carry bit 31 and
             * in-group sources wrap, so one add and one compare decide it.
             * The load's wait stays on this path: a wait after the join
             * would hold every group for the flush's outstanding stores */
            const bool far = tInf + farb < 8191u - omask;
            if (far) {
                b = dst[so];
                asm volatile("" ::"v"(b));
            }
#else
            const bool far = !lit && so < gb && gb - so > omask + 1u;
            if (cd_ballot(far)) {
                if (far) b = dst[so];
            }
#endif
        }
        /* resolved: bit 31 | the byte; pending: the source lane's ds_bpermute
         * address (lane × 4) in bits 10-15 */
        const bool pend = !lit && q < CD_LANES;
        int32_t ent = pend ? (int32_t)(q << 10) : (int32_t)(0x80000000u | b);
        /* FAR: the guard read off the entries' sign (== pend, one compare
         * instead of a select and a compare); measured slower on the pipe and
         * the plain tokpar64 (instruction placement), so FAR only */
        if (FAR && CD_ENTGUARD ? cd_ballot(ent >= 0) : cd_ballot(pend)) {
            const int32_t me = (int32_t)(lane << 2);
            do
                ent = __builtin_amdgcn_ds_bpermute(ent < 0 ? me : ent >> 8, ent);
            while (cd_ballot(ent >= 0));
        }
        const bool live = lane < total - g;
        lds[outr_off + (live ? o & omask : sink_off - outr_off)] = (uint8_t)ent;   /* the sink lies past the window */
        cd_fence();
        {
            const uint32_t done = g + CD_LANES <= total ? gb + CD_LANES : O + total;
            if (done - F >= unit) {
                /* one unit: unit / 16 lanes, 16 bytes each */
                const uint32_t x = F + 16u * lane;
                if (16u * lane < unit) {
                    uint4 v;
                    __builtin_memcpy(&v, lds + outr_off + (x & omask), 16);
                    __builtin_memcpy(dst + x, &v, 16);
                }
                F += unit;
                if (FAR) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            }
        }
    }
}

/* the pipe's input ring: the consumer reads round k's literals,
 * [base_k, base_k + 161), while the producer stages for round k + 1: staging
 * runs when fewer than 192 bytes are ahead of base and fills up to base + 320
 * (16-byte aligned), so it overwrites only bytes before
 * base_{k+1} + 320 - 512 <= base_k - 32 (base_{k+1} <= base_k + 160) */
#define CD_IN_RINGP 512u
/* Round 4 measured and removed: a token-granular output stage (one lane
 * per token, 16-byte unaligned LDS copies, a pass per in-round reference
 * chain: Zipf 1 M x 8 KiB 20.27 -> 102.30 ms, DESIGN.md §4.4,
 * profiles/r04/dab_*_tok.txt), and the input ring's first 32 bytes mirrored
 * past its end for single unaligned token reads in steps 1-2 (slower:
 * 11.14 -> 11.85 ms mixed16k, 21.75 -> 24.00 Zipf, 17.33 -> 18.88 text64k,
 * profiles/r04/dab_*_noper_nomir.txt). */

/* a value past the batch's stated max_out_cap is refused, never overrun.
 * The 16-bit start marks of tokpar64's windows of <= 4 KiB rely on this:
 * with out_cap <= max_len <= the window, a stream's output positions stay
 * below 65536, so a stale mark never matches a later group */
/* a stream's fields, every load issued before any is used (CD_META, round
 * 5: the skip flag, the refusal test and the offsets were four dependent
 * memory waits before the first input load) */
#ifndef CD_META
#define CD_META 1
#endif
struct CdMeta {
    uint32_t in_len, cap, max_len;
    const uint8_t *src;
    uint8_t *dst;
    bool skip;
};
__device__ __forceinline__ CdMeta cd_meta(const LzfBatch &bt, uint32_t v)
{
    CdMeta m;
    const uint8_t *sp = bt.skip ? bt.skip + v : (const uint8_t *)&cd_dummy16;   /* zero when there is no skip list */
    m.in_len = __builtin_amdgcn_readfirstlane(bt.in_len[v]);
    m.cap = __builtin_amdgcn_readfirstlane(bt.out_cap[v]);
    const uint64_t io = bt.in_off[v], oo = bt.out_off[v];
    const uint32_t sk = *sp;
    m.max_len = bt.max_len;
    /* all of them used here, before the skip and refusal branches: the
     * compiler would otherwise sink loads past them (one more wait each) */
    asm volatile("" ::"s"(io), "s"(oo), "v"(sk), "s"(m.max_len));
    m.src = bt.in + io;
    m.dst = bt.out + oo;
    m.skip = __builtin_amdgcn_readfirstlane(sk) != 0u;
    return m;
}
/* a value whose out_cap exceeds the batch's max_len is refused (EINVAL) */
__device__ __forceinline__ bool cd_refuse_cap(const LzfBatch &bt, uint32_t v, uint32_t cap, uint32_t max_len,
                                              uint32_t lane)
{
    if (cap <= max_len) return false;
    if (lane == 0) {
        bt.out_len[v] = 0u;
        bt.err[v] = 22;             /* EINVAL */
    }
    return true;
}
__device__ __forceinline__ bool cd_refused(const LzfBatch &bt, uint32_t v, uint32_t lane)
{
    if (bt.out_cap[v] <= bt.max_len) return false;
    if (lane == 0) {
        bt.out_len[v] = 0u;
        bt.err[v] = 22;             /* EINVAL */
    }
    return true;
}

/* CD_TP_SMALL: windows up to 4 KiB (the output stays below 65536, so 16-bit
 * start marks match only in their group: cd_refused holds out_cap to the
 * batch's max_len, and lzf_launch_decompress picks no window below max_len;
 * the FAR route runs the 4 KiB instance past its window only while max_len
 * <= 65536, checked at its launch) keep 16-bit marks and compute token
 * sizes instead of reading the 256-byte table: 5008 bytes of LDS for a 4 KiB
 * window, 32 streams per CU (the wave limit) instead of 30 */
#ifndef CD_TP_SMALL
#define CD_TP_SMALL 1
#endif
#ifndef CD_TP_TSZT
#define CD_TP_TSZT 0
#endif
template <bool B> struct CdMark { typedef uint32_t T; };
template <> struct CdMark<true> { typedef uint16_t T; };
/* one instance per window size, with static LDS (as the pipe) */
template <uint32_t RING, bool FAR = false>
__global__ __launch_bounds__(64) void lzf_decompress_tokpar_kernel(LzfBatch bt, uint32_t out_ring)
{
    constexpr bool SMALL = CD_TP_SMALL && RING <= 4096u;
    constexpr bool TSZT = !SMALL || CD_TP_TSZT;
    typedef typename CdMark<SMALL>::T MT;
    constexpr uint32_t MARKB = SMALL ? 2u * CD_LANES + 16u : 5u * CD_LANES;   /* marks + slot 64 and the sink */
    __shared__ __attribute__((aligned(16))) uint8_t smem[CD_IN_RING1 + RING + MARKB +
                                                         (TSZT ? 512u : 256u)];   /* + jump (and token-size) tables */
    out_ring = RING;
    uint8_t *outr = smem;                              /* out_ring (power of two) */
    uint8_t *inr = outr + out_ring;                    /* CD_IN_RING1, right after the window (cd_output) */
    MT *mark = (MT *)(inr + CD_IN_RING1);              /* 64 token-start marks */
    uint8_t *sink = (uint8_t *)(mark + CD_LANES);      /* the idle lanes' byte sink (and mark slot 64; both write-only) */
    uint8_t *jt = inr + CD_IN_RING1 + MARKB;           /* the jump table (+ token sizes) */
    const uint32_t imask = CD_IN_RING1 - 1u, omask = out_ring - 1u;

    const uint32_t lane = threadIdx.x;
    const uint32_t v = blockIdx.x;
#if CD_META
    const CdMeta md = cd_meta(bt, v);
    if (md.skip || cd_refuse_cap(bt, v, md.cap, md.max_len, lane)) return;
    const uint32_t in_len = md.in_len;
    const uint32_t cap = md.cap;
    const uint8_t *src = md.src;
    uint8_t *dst = md.dst;
#else
    if ((bt.skip && bt.skip[v]) || cd_refused(bt, v, lane)) return;
    const uint32_t in_len = bt.in_len[v];
    const uint32_t cap = bt.out_cap[v];
    const uint8_t *src = bt.in + bt.in_off[v];
    uint8_t *dst = bt.out + bt.out_off[v];
#endif
    /* as the reference, a 0-length stream still reads its first control byte */
    const uint32_t avail = in_len ? in_len : 1u;

    mark[lane] = 0u;            /* position 0 always starts a token */
    cd_jt_init<TSZT>(jt, lane);
    uint32_t loaded = 0, base = 0, O = 0;
    uint32_t F = 0;             /* output [0, F) stored */
    int32_t err = 0;
    bool first = true;
    /* CD_TPREF: the next staging piece in registers, loaded when the one
     * before it is written (one 16-byte load per lane, the stream's last piece
     * from avail - 16, idle lanes from a dummy: no byte loop, no branch), so a
     * staging waits for no load (streams of < 16 bytes stage synchronously) */
    uint4 pv = make_uint4(0u, 0u, 0u, 0u);
    uint32_t pf = 0u, pt = 0u;                        /* pv holds [pf, pt) */
    while (first || base < in_len) {                     /* src/lzf_d.c:64, 146 */
        first = false;
        if (CD_TPREF && avail >= 16u) {
            constexpr uint32_t STAGE = CD_IN_RING1 / 2u;
            uint32_t need = base + 2u * CD_ROUND;
            if (need > avail) need = avail;
            if (loaded < need) {
                const uint32_t to = min(loaded + STAGE, avail);
                const uint32_t x = loaded + 16u * lane;
                if (pt > pf) {                       /* the prefetched piece: [loaded, to) */
                    if (x < pt) {
                        const uint32_t d = pt - x < 16u ? 16u - (pt - x) : 0u;
                        uint4 w = pv;
                        if (d) w = cd_shr16(w, d);
                        *(uint4 *)(inr + (x & (CD_IN_RING1 - 1u))) = w;
                    }
                } else if (x < to) {
                    *(uint4 *)(inr + (x & (CD_IN_RING1 - 1u))) = cd_ld16(src + x, to - x);
                }
                loaded = to;
                cd_fence();
                /* the piece after it */
                const uint32_t to2 = min(loaded + STAGE, avail);
                const uint32_t x2 = loaded + 16u * lane;
                const uint8_t *pa = x2 < to2 ? src + (to2 - x2 >= 16u ? x2 : avail - 16u) : (const uint8_t *)&cd_dummy16;
                __builtin_memcpy(&pv, pa, 16);
                pf = loaded;
                pt = to2;
            }
        } else {
            cd_stage<CD_IN_RING1>(inr, src, base, avail, loaded, lane);
        }
#ifdef CD_DISC_TWICE                 /* diagnostics: the discovery's marginal cost (run twice, same result) */
        {
            const uint32_t x0 = cd_discover_lds<TSZT>(inr, imask, jt, base, in_len, lane);
            asm volatile("" ::"v"(x0));
        }
#endif
        const uint32_t x = cd_discover_lds<TSZT>(inr, imask, jt, base, in_len, lane);
        const CdRound r = cd_decode(inr, imask, base, x, O, in_len, cap);
        if (r.err) {
            err = r.err;
            break;
        }
        cd_output<CD_IN_RING1, false, CD_MARKAHEAD, MT, FAR>(smem, 0u, omask, mark, (uint32_t)(sink - smem), dst, O, r.total,
                               x < CD_ROUND, O + r.rel, r.tinfo, lane, F);
        O += r.total;
        base = r.nbase;
    }
    cd_flush(smem, 0u, omask, dst, F, O, lane);   /* the rounds before a failing one, as the reference */
    if (lane == 0) {
        bt.out_len[v] = err ? 0u : O;
        bt.err[v] = err;
    }
}

/* the pipe's hand-over of one round: token table + header, double-buffered.
 * tok[l] = rel (bits 0-15: <= 64 * 264) | literal flag (16) | info (17-31:
 * back-ref distance <= 8192, or the low bits of the literal's input offset
 * minus its output offset, all the input ring's mask keeps) */
struct CdSlot {
    uint32_t tok[CD_LANES];
    uint32_t ntok, total, last;
    int32_t err;
};

__device__ __forceinline__ void cd_stage_pipe(uint8_t *inr, const uint8_t *src, uint32_t base, uint32_t avail,
                                              uint32_t &loaded, uint32_t lane)
{
    const uint32_t need = min(avail, base + 192u);
    if (loaded < need) {
        const uint32_t to = min(avail, (base + 320u) & ~15u);
        const uint32_t x = loaded + 16u * lane;       /* loaded is a multiple of 16 here */
        if (x < to) {
            const uint4 v = cd_ld16(src + x, to - x);
            *(uint4 *)(inr + (x & (CD_IN_RINGP - 1u))) = v;
        }
        loaded = to;
        cd_fence();
    }
}

/* the pipe's window is always CD_OUT_MAX (values over 4 KiB), so its LDS is
 * static: the compiler folds the LDS base into every address (with dynamic
 * LDS it adds the base, 0, with one VALU per LDS address) */
#define CD_PIPE_LDS (CD_IN_RINGP + 2u * sizeof(CdSlot) + 5u * CD_LANES + 16u + CD_OUT_MAX + \
                     512u)   /* + jump and token-size tables */
__global__ __launch_bounds__(128) void lzf_decompress_pipe_kernel(LzfBatch bt, uint32_t out_ring)
{
    __shared__ __attribute__((aligned(16))) uint8_t smem[CD_PIPE_LDS];
    out_ring = CD_OUT_MAX;
    CdSlot *slot = (CdSlot *)smem;                     /* 2 */
    uint32_t *mark = (uint32_t *)(slot + 2);           /* the consumer's 64 token-start marks */
    uint8_t *mark64 = (uint8_t *)(mark + CD_LANES);    /* mark slot 64 (write-only) and spare */
    uint8_t *outr = mark64 + CD_LANES;                 /* out_ring (power of two) */
    uint8_t *inr = outr + out_ring;                    /* CD_IN_RINGP, right after the window (cd_output) */
    uint8_t *jt = inr + CD_IN_RINGP;                   /* the jump table (+ token sizes) */
    uint8_t *sink = jt + 512u;                         /* the consumer's idle-lane byte sink, past the window */
    const uint32_t imask = CD_IN_RINGP - 1u, omask = out_ring - 1u;

    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64u;
    const uint32_t v = blockIdx.x;
#if CD_META
    const CdMeta md = cd_meta(bt, v);
    if (md.skip || cd_refuse_cap(bt, v, md.cap, md.max_len, threadIdx.x)) return;
    const uint32_t in_len = md.in_len;   /* scalar: no load wait in the loop */
    const uint32_t cap = md.cap;
#else
    if ((bt.skip && bt.skip[v]) || cd_refused(bt, v, threadIdx.x)) return;
    const uint32_t in_len = __builtin_amdgcn_readfirstlane(bt.in_len[v]);   /* scalar: no load wait in the loop */
    const uint32_t cap = __builtin_amdgcn_readfirstlane(bt.out_cap[v]);
#endif

    uint64_t tw[6] = {0ull, 0ull, 0ull, 0ull, 0ull, 0ull};
#ifdef CD_TIMING
    tw[2] = __builtin_amdgcn_s_memtime();
#endif
    if (producer) {
        /* steps 1-3, one round ahead of the consumer; round k's table goes to
         * slot k & 1, published by the barrier that ends round k */
#if CD_META
        const uint8_t *src = md.src;
#else
        const uint8_t *src = bt.in + bt.in_off[v];
#endif
        const uint32_t avail = in_len ? in_len : 1u;   /* a 0-length stream still reads one byte */
        uint32_t loaded = 0, base = 0, O = 0;
        cd_jt_init(jt, lane);
        /* CD_PREF: the input the next round needs is loaded at the start of
         * this round and written to the ring when the next round starts, so
         * its load latency is off the producer's chain (the synchronous stage
         * then runs in round 0 only) */
        uint4 pv = make_uint4(0u, 0u, 0u, 0u);
        uint32_t pto = 0u;
        bool pend = false;
        /* CD_PREF2: two rounds ahead.  The piece issued in round k lands in
         * register set k & 1 and is written at round k + 2's start, so a load
         * has two rounds to land.  It reaches base_k + 608, whose ring slot is
         * base_k + 96 < base_{k+1}: the consumer, then in round k + 1, has
         * left it (bases advance >= 128 per round but the last).  The loop is
         * unrolled by two so each set is its own registers: a select between
         * the sets would wait for the one in flight */
        uint4 pq0 = make_uint4(0u, 0u, 0u, 0u), pq1 = pq0;
        uint32_t pf0 = 0u, pt0 = 0u, pf1 = 0u, pt1 = 0u, iss = 0u;
        auto round = [&](auto par, uint32_t k) -> bool {
            constexpr uint32_t P = decltype(par)::value;
#ifdef CD_TIMING
            const uint64_t ts0 = __builtin_amdgcn_s_memtime();
#endif
            if (CD_PREF2) {
                uint4 &q = P ? pq1 : pq0;
                uint32_t &qf = P ? pf1 : pf0, &qt = P ? pt1 : pt0;
                {
                    /* no uniform branch around the write or the load below: the
                     * compiler's wait counting then sees one load per set per
                     * two rounds and waits for this set's alone */
                    const uint32_t px = qf + 16u * lane;
                    if (px < qt) {
                        /* the stream's last piece was loaded from avail - 16:
                         * its bytes move down by d, zeros above avail */
                        const uint32_t d = qt - px < 16u ? 16u - (qt - px) : 0u;
                        uint4 w = q;
                        if (d) w = cd_shr16(w, d);
                        *(uint4 *)(inr + (px & (CD_IN_RINGP - 1u))) = w;
                    }
                    loaded = max(loaded, qt);
                    qf = qt = 0u;
                    cd_fence();
                }
            } else if (CD_PREF && pend) {
                const uint32_t px = loaded + 16u * lane;
                if (px < pto) {
                    *(uint4 *)(inr + (px & (CD_IN_RINGP - 1u))) = pv;
                }
                loaded = pto;
                pend = false;
                cd_fence();
            }
            cd_stage_pipe(inr, src, base, avail, loaded, lane);
            if (CD_PREF2) {
                uint4 &q = P ? pq1 : pq0;
                uint32_t &qf = P ? pf1 : pf0, &qt = P ? pt1 : pt0;
                iss = max(iss, loaded);
                const uint32_t lim = min(avail, (base + 608u) & ~15u);
                const bool go = iss < lim && base + 128u < in_len;
                /* one 16-byte load per lane every round, the last piece's from
                 * avail - 16 (in_len > 128 when go), idle lanes' from a dummy:
                 * no byte loop and no branch, so the load stays in flight for
                 * two rounds */
                const uint32_t px = iss + 16u * lane;
                const uint8_t *pa = (go && px < lim) ? src + (lim - px >= 16u ? px : avail - 16u)
                                                     : (const uint8_t *)&cd_dummy16;
                __builtin_memcpy(&q, pa, 16);
                qf = go ? iss : 0u;
                qt = go ? lim : 0u;
                iss = go ? lim : iss;
            } else if (CD_PREF && loaded < min(avail, base + 448u) && base + 128u < in_len) {
                /* the next round starts at >= base + 128 (tokens start in
                 * [base, base + 128) and the last one ends past it) and at most
                 * base + 160: the ring may take up to base + 448 at its start
                 * (the consumer then reads round k's [base, base + 161), and
                 * offset y overwrites y - 512), and needs base_{k+1} + 192 */
                pto = min(avail, (base + 448u) & ~15u);
                const uint32_t px = loaded + 16u * lane;
                if (px < pto) pv = cd_ld16(src + px, pto - px);
                pend = true;
            }
#ifdef CD_TIMING
            const uint64_t td0 = __builtin_amdgcn_s_memtime();
#endif
            const uint32_t x = cd_discover_lds(inr, imask, jt, base, in_len, lane);
#ifdef CD_TIMING
            const uint64_t td1 = __builtin_amdgcn_s_memtime();
#endif
            const CdRound r = cd_decode(inr, imask, base, x, O, in_len, cap);
#ifdef CD_TIMING
            /* the producer's parts: staging, token discovery, token decode (the
             * latter ends at a use of its results, so its waits are in it) */
            tw[3] += td1 - td0;
            tw[5] += td0 - ts0;
            tw[4] += __builtin_amdgcn_s_memtime() - td1;
#endif
            const uint32_t ntok = r.ntok;
            const uint32_t total = r.total;
            CdSlot &s = slot[P];
            s.tok[lane] = (r.tinfo << 17) | ((r.tinfo >> 31) << 16) | r.rel;   /* rel < 65536 */
            const bool last = r.err != 0 || r.nbase >= in_len;   /* src/lzf_d.c:146 */
            if (lane == 0) {
                s.ntok = ntok;
                s.total = total;
                s.last = (last ? 1u : 0u) | (r.overlap != 0ull ? 2u : 0u);
                s.err = r.err;
            }
            O += total;
            base = r.nbase;
            cd_barrier(tw);
            (void)k;
            return last;
        };
        for (uint32_t k = 0;; k += 2u) {
            if (round(CdPar<0>(), k)) break;
            if (round(CdPar<1>(), k + 1u)) break;
        }
    } else {
#if CD_META
        uint8_t *dst = md.dst;
#else
        uint8_t *dst = bt.out + bt.out_off[v];
#endif
        if (CD_CPRIO) __builtin_amdgcn_s_setprio(CD_CPRIO);
        uint32_t O = 0, F = 0;  /* output [0, F) stored */
        int32_t err = 0;
        mark[lane] = 0u;        /* group tags are >= 1 */
        cd_barrier();
        for (uint32_t k = 0;; k++) {
            const CdSlot &s = slot[k & 1u];
            const uint32_t total = __builtin_amdgcn_readfirstlane(s.total);
            const uint32_t lastw = __builtin_amdgcn_readfirstlane(s.last);
            const uint32_t last = lastw & 1u;
            const bool per = (lastw & 2u) != 0u;
            const uint32_t ntok = __builtin_amdgcn_readfirstlane(s.ntok);
            err = __builtin_amdgcn_readfirstlane(s.err);
            if (err) break;      /* the failing round writes nothing */
            const uint32_t w = s.tok[lane];
            if (CD_PERIOD && per)   /* its own copy of the loop: the other rounds run the plain one */
                cd_output<CD_IN_RINGP, true, CD_MARKAHEAD_PIPE>(smem, (uint32_t)(outr - smem), omask, mark, (uint32_t)(sink - smem), dst,
                                             O, total, lane < ntok, O + (w & 0xFFFFu),
                                             (w >> 17) | ((w & 0x10000u) << 15), lane, F);
            else
                cd_output<CD_IN_RINGP, false, CD_MARKAHEAD_PIPE>(smem, (uint32_t)(outr - smem), omask, mark, (uint32_t)(sink - smem), dst, O,
                                       total, lane < ntok, O + (w & 0xFFFFu), (w >> 17) | ((w & 0x10000u) << 15),
                                       lane, F);
            O += total;
            if (last) break;
            cd_barrier(tw);
        }
        cd_flush(smem, (uint32_t)(outr - smem), omask, dst, F, O, lane);   /* also before a failing round */
#ifdef CD_TIMING
        tw[0] += __builtin_amdgcn_s_memtime() - tw[2];
#endif
        if (lane == 0) {
            bt.out_len[v] = err ? 0u : O;
            bt.err[v] = err;
        }
    }
#ifdef CD_TIMING
    if (lane == 0) {
        const uint32_t tr = (blockIdx.x % CD_TROWS) * 8u;
        atomicAdd(&cd_tstat[tr + (producer ? 0 : 2)], (unsigned long long)tw[0]);
        atomicAdd(&cd_tstat[tr + (producer ? 1 : 3)], (unsigned long long)tw[1]);
        if (producer) {
            atomicAdd(&cd_tstat[tr + 4], (unsigned long long)tw[3]);
            atomicAdd(&cd_tstat[tr + 5], (unsigned long long)tw[4]);
            atomicAdd(&cd_tstat[tr + 6], (unsigned long long)tw[5]);
        }
    }
#endif
}

/* the pipe for 8 KiB windows (values over 4 KiB); smaller windows leave
 * room for twice the streams per CU as single waves, which the pipe's two
 * waves per stream cannot use (32 waves per CU) */
#ifndef CD_PIPE_MIN_RING
#define CD_PIPE_MIN_RING 8192u
#endif

/* CD_FAR_MAX (round 5): values over 4 KiB and up to this size decode with
 * tokpar64's 4 KiB window (16-bit marks: outputs < 65536) and far sources
 * read back from HBM, one wave per stream (32 streams per CU), instead of the
 * pipe (0: off).  16 KiB: Zipf 8 KiB and mixed 16 KiB gain 6-10 %, json
 * 16 KiB and sentence text 64 KiB lose on their far groups */
#ifndef CD_FAR_MAX
#define CD_FAR_MAX 16384u
#endif
hipError_t lzf_launch_decompress(const LzfBatch &b, hipStream_t s)
{
    uint32_t ring = 256u;
    while (ring < b.max_len && ring < CD_OUT_MAX) ring <<= 1;
    if (CD_FAR_MAX && b.max_len > 4096u && b.max_len <= CD_FAR_MAX && b.max_len <= 65536u) {
        hipLaunchKernelGGL((lzf_decompress_tokpar_kernel<4096u, true>), dim3(b.count), dim3(CD_LANES), 0, s, b, 4096u);
        return hipGetLastError();
    }
    if (CD_PIPE && ring >= CD_PIPE_MIN_RING) {
        if (ring != CD_OUT_MAX) return hipErrorInvalidValue;   /* static LDS for the 8 KiB window */
        hipLaunchKernelGGL(lzf_decompress_pipe_kernel, dim3(b.count), dim3(2u * CD_LANES), 0, s, b, ring);
    } else {
        /* LDS: the input ring, the window, the 64 marks and token starts.
         * A window of <= 4 KiB covers max_len (its 16-bit marks need every
         * output below 65536, CD_TP_SMALL); the 8 KiB one is a ring */
        if (ring <= 4096u && b.max_len > ring) return hipErrorInvalidValue;
        switch (ring) {
        case 256u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<256u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        case 512u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<512u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        case 1024u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<1024u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        case 2048u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<2048u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        case 4096u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<4096u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        case 8192u: hipLaunchKernelGGL(lzf_decompress_tokpar_kernel<8192u>, dim3(b.count), dim3(CD_LANES), 0, s, b, ring); break;
        default: return hipErrorInvalidValue;
        }
    }
    return hipGetLastError();
}

#ifdef CD_TIMING
/* producer busy, producer waiting, consumer busy, consumer waiting (cycles,
 * summed over waves since the last call) */
extern "C" int lzf_gpu_dec_tstat(unsigned long long *out)
{
    static unsigned long long rows[CD_TROWS * 8u];
    if (hipMemcpyFromSymbol(rows, HIP_SYMBOL(cd_tstat), sizeof(rows)) != hipSuccess) return -1;
    for (uint32_t i = 0; i < 8u; i++) {
        out[i] = 0;
        for (uint32_t r = 0; r < CD_TROWS; r++) out[i] += rows[8u * r + i];
    }
    static const unsigned long long z[CD_TROWS * 8u] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(cd_tstat), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

const char *lzf_decompress_kernel_name(void)
{
    if (!CD_PIPE) return "tokpar64";
    return CD_FAR_MAX ? (CD_FAR_MAX >= 16384u ? "tokpar64 up to 4 KiB, tokpar64-far up to 16 KiB, pipe past"
                                              : "tokpar64 up to 4 KiB, tokpar64-far up to 8 KiB, pipe past")
                      : "tokpar64 up to 4 KiB, pipe past";
}

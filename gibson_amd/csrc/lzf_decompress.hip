/*
 * lzf_decompress.hip -- token-parallel LZF decoder for gfx950.
 *
 * Replaces src/lzf_d.c:55-149 for batches of independent streams: one
 * workgroup = one 64-lane wave per stream.  The stream is consumed in
 * rounds; a round starts at a token boundary and covers the tokens that
 * START in the next 128 input bytes (CD_ROUND):
 *
 *   1. token boundaries: every lane takes two input bytes and their token
 *      sizes (literal c<32: c+2 bytes; back-ref: 2, or 3 when c>>5 == 7);
 *      the chain of boundaries is found by pointer doubling (ds_bpermute),
 *      and lane l ends up holding the start of token l (<= 64 per round);
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
 */
#include "lzf_internal.h"

#define CD_LANES   64u
#ifndef CD_ROUND
#define CD_ROUND   128              /* input bytes whose token starts one round covers: 64 or 128 */
#endif
/* input ring: a round reads [base, base + CD_ROUND + 33); staging runs in
 * CD_STAGE-byte pieces (one 16-byte load per lane) when the round's reach
 * passes base + 2 * CD_ROUND (loaded < base + 2 * CD_ROUND), so a piece
 * overwrites only bytes before loaded - CD_IN_RING + CD_STAGE < base, which
 * no later round reads.  A small ring keeps the kernel's LDS small:
 * residency, not bandwidth, bounds this decoder */
#ifndef CD_IN_RING
#define CD_IN_RING 512u
#endif
#define CD_STAGE   (CD_IN_RING / 2u)
static_assert(CD_STAGE >= 2u * CD_ROUND && CD_STAGE <= 16u * CD_LANES, "one staging piece per round");
/* output window ring: back-references reach at most 8192 bytes back
 * (src/lzf_d.c:95, off < 8192), and a group reads all its sources before it
 * writes its 64 bytes, so a ring of 8 KiB suffices: the slots a group
 * overwrites (o - 8192) are read, if at all, by that group alone */
#ifndef CD_OUT_MAX
#define CD_OUT_MAX 8192u
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

__device__ __forceinline__ uint64_t cd_lt(uint32_t i)
{
    return i >= 64u ? ~0ull : ((1ull << i) - 1ull);
}

__device__ __forceinline__ void cd_fence()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
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

/* J(J(i)) for a jump table J whose exits are CD_LANES (= stay) */
__device__ __forceinline__ uint32_t cd_jump(uint32_t j)
{
    const uint32_t t = (uint32_t)__shfl((int)j, (int)(j & 63u));
    return j >= 64u ? 64u : t;
}

__device__ __forceinline__ uint32_t cd_rl(uint32_t v, uint32_t l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

__global__ __launch_bounds__(64) void lzf_decompress_tokpar_kernel(LzfBatch bt, uint32_t out_ring)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint8_t *inr = smem;                               /* CD_IN_RING */
    uint8_t *outr = smem + CD_IN_RING;                 /* out_ring (power of two) */
    uint32_t *mark = (uint32_t *)(outr + out_ring);    /* 64 token-start marks (group tags) */
    const uint32_t imask = CD_IN_RING - 1u, omask = out_ring - 1u;

    const uint32_t lane = threadIdx.x;
    const uint32_t v = blockIdx.x;
    if (bt.skip && bt.skip[v]) return;
    const uint32_t in_len = bt.in_len[v];
    const uint32_t cap = bt.out_cap[v];
    const uint8_t *src = bt.in + bt.in_off[v];
    uint8_t *dst = bt.out + bt.out_off[v];
    if (cap > bt.max_len) {          /* past the batch's stated max_out_cap: refused, never overrun */
        if (lane == 0) {
            bt.out_len[v] = 0u;
            bt.err[v] = 22;         /* EINVAL */
        }
        return;
    }
    /* as the reference, a 0-length stream still reads its first control byte */
    const uint32_t avail = in_len ? in_len : 1u;

    mark[lane] = 0u;            /* group tags are >= 1 */
    uint32_t loaded = 0;
    uint32_t base = 0;          /* input offset of the round's first token */
    uint32_t O = 0;             /* output bytes produced so far */
    int32_t err = 0;
    bool first = true;

    while (first || base < in_len) {                     /* src/lzf_d.c:64, 146 */
        first = false;
        /* stage input [base, base + 2 * CD_ROUND) (tokens starting in the
         * round and their literal payloads, <= CD_ROUND - 1 + 33 bytes) */
        uint32_t need = base + 2u * CD_ROUND;
        if (need > avail) need = avail;
        if (loaded < need) {                 /* need - loaded <= CD_ROUND + 33 <= CD_STAGE */
            uint32_t to = loaded + CD_STAGE;
            if (to > avail) to = avail;
            const uint32_t x = loaded + 16u * lane;   /* loaded is a multiple of 16 here */
            if (x < to) *(uint4 *)(inr + (x & imask)) = cd_ld16(src + x, to - x);
            loaded = to;
            cd_fence();
        }

        /* ---- 1. token boundaries -------------------------------------- */
#if CD_ROUND == 128
        /* two input bytes per lane; jump tables J0..J5 over the round's 128
         * positions packed two per lane (16 bits each; 128 = leaves the round).
         * A round holds <= 64 tokens (each takes >= 2 bytes): lane l finds the
         * start of token l with six doubling levels */
        uint32_t PJ[6];
        {
            const uint32_t ipa = base + 2u * lane, ipb = ipa + 1u;
            const uint32_t ca = inr[ipa & imask], cb = inr[ipb & imask];
            const uint32_t ta = ca < 32u ? ca + 2u : ((ca >> 5) == 7u ? 3u : 2u);
            const uint32_t tb = cb < 32u ? cb + 2u : ((cb >> 5) == 7u ? 3u : 2u);
            uint32_t na = 2u * lane + ta, nb = 2u * lane + 1u + tb;
            if (ipa + ta >= in_len || na > 128u) na = 128u;
            if (ipb + tb >= in_len || nb > 128u) nb = 128u;
            PJ[0] = na | (nb << 16);
        }
#pragma unroll
        for (uint32_t k = 1; k < 6u; k++) {
            const uint32_t ja = PJ[k - 1u] & 0xFFFFu, jb = PJ[k - 1u] >> 16;
            const uint32_t wa = (uint32_t)__shfl((int)PJ[k - 1u], (int)((ja >> 1) & 63u));
            const uint32_t wb = (uint32_t)__shfl((int)PJ[k - 1u], (int)((jb >> 1) & 63u));
            const uint32_t va = ja >= 128u ? 128u : ((ja & 1u) ? wa >> 16 : wa & 0xFFFFu);
            const uint32_t vb = jb >= 128u ? 128u : ((jb & 1u) ? wb >> 16 : wb & 0xFFFFu);
            PJ[k] = va | (vb << 16);
        }
        uint32_t x = 0;
#pragma unroll
        for (uint32_t b = 0; b < 6u; b++) {
            const uint32_t w = (uint32_t)__shfl((int)PJ[b], (int)((x >> 1) & 63u));
            const uint32_t y = (x & 1u) ? w >> 16 : w & 0xFFFFu;
            if (((lane >> b) & 1u) && x < 128u) x = y;
        }
        /* lane l now holds token l (tokens compacted in order): its bytes */
        const bool tok = x < 128u;
#else
        const uint32_t ip0 = base + lane;
        const uint32_t c0 = inr[ip0 & imask];
        const uint32_t tsz0 = c0 < 32u ? c0 + 2u : ((c0 >> 5) == 7u ? 3u : 2u);
        uint32_t nx = lane + tsz0;
        if (ip0 + tsz0 >= in_len || nx > CD_LANES) nx = CD_LANES;  /* loop ends / next round */
        /* every token takes >= 2 input bytes, so a round has <= 32 tokens:
         * lane l < 32 finds the start of token l with 5 doubling levels */
        /* every lane takes part in every shuffle: a shuffle under a partial
         * exec mask reads nothing from the inactive source lanes */
        uint32_t J0 = nx, J1, J2, J3, J4;
        J1 = cd_jump(J0);
        J2 = cd_jump(J1);
        J3 = cd_jump(J2);
        J4 = cd_jump(J3);
        uint32_t x = 0, y;
        y = (uint32_t)__shfl((int)J0, (int)(x & 63u)); if ((lane & 1u) && x < CD_LANES) x = y;
        y = (uint32_t)__shfl((int)J1, (int)(x & 63u)); if ((lane & 2u) && x < CD_LANES) x = y;
        y = (uint32_t)__shfl((int)J2, (int)(x & 63u)); if ((lane & 4u) && x < CD_LANES) x = y;
        y = (uint32_t)__shfl((int)J3, (int)(x & 63u)); if ((lane & 8u) && x < CD_LANES) x = y;
        y = (uint32_t)__shfl((int)J4, (int)(x & 63u)); if ((lane & 16u) && x < CD_LANES) x = y;
        if (lane >= 32u) x = CD_LANES;
        /* lane l now holds token l (tokens compacted in order): its bytes */
        const bool tok = x < CD_LANES;
#endif
        const uint32_t ntok = (uint32_t)__builtin_popcountll(__ballot(tok));
        const uint32_t ip = base + (tok ? x : 0u);
        const uint32_t c = inr[ip & imask];
        const uint32_t b1 = inr[(ip + 1u) & imask], b2 = inr[(ip + 2u) & imask];
        const uint32_t tsz = c < 32u ? c + 2u : ((c >> 5) == 7u ? 3u : 2u);

        /* ---- 2. decode + output offsets ------------------------------- */
        const bool lit = c < 32u;
        uint32_t olen, back = 0, lsrc = 0;
        int32_t e = 0;
        if (lit) {
            olen = c + 1u;
            lsrc = ip + 1u;
        } else {
            uint32_t len = c >> 5, offb = b1;
            if (len == 7u) { len += b1; offb = b2; }
            olen = len + 2u;
            back = ((c & 31u) << 8) + offb + 1u;
        }
        /* the owner's info for an output byte o: literal -> input ring index
         * o + (lsrc - Ot), flagged in bit 31; back-ref -> distance */
        const uint32_t ol = tok ? olen : 0u;
        const uint32_t incl = cd_incl_sum(ol);
        const uint32_t Ot = O + incl - ol;                 /* output offset of my token */
        const uint32_t tinfo = lit ? (((lsrc - Ot) & 0x7FFFFFFFu) | 0x80000000u) : back;
        /* ---- 3. the reference's checks, in its order ------------------ */
        if (tok) {
            if (lit) {
                if ((uint64_t)Ot + olen > cap) e = 7;                       /* E2BIG  :72 */
                else if ((uint64_t)ip + 1u + olen > in_len) e = 22;         /* EINVAL :79 */
            } else {
                if (ip + 1u >= in_len) e = 22;                              /* :101 */
                else if ((c >> 5) == 7u && ip + 2u >= in_len) e = 22;      /* :111 */
                else if ((uint64_t)Ot + olen > cap) e = 7;                  /* :121 */
                else if (back > Ot) e = 22;                                 /* :127 */
            }
        }
        const uint64_t EB = __ballot(e != 0);
        if (EB) {
            err = (int32_t)cd_rl((uint32_t)e, (uint32_t)__builtin_ctzll(EB));
            break;
        }
        const uint32_t total = cd_rl(incl, 63u);           /* round output bytes */

        /* ---- 4. output bytes, 64 per step ------------------------------ */
        /* tokens sit in lanes in output order, so the owner of output byte b
         * of a group is (tokens started before the group) + (token starts in
         * the group at or below b) - 1: the starts are marked in LDS with the
         * group's tag (gb + 1, never reused, so the marks need no clearing)
         * and read back as one ballot */
        uint32_t tbase = 0;          /* tokens started before the group */
#ifdef LZF_CD_ABLATE_OUTPUT           /* diagnostic builds only: time discovery alone */
        for (uint32_t g = 0; g < 0u; g += CD_LANES) {
#else
        for (uint32_t g = 0; g < total; g += CD_LANES) {
#endif
            const uint32_t gb = O + g;                     /* group's first output offset */
            if (tok && Ot >= gb && Ot < gb + CD_LANES) mark[Ot - gb] = gb + 1u;
            cd_fence();
            const uint64_t S = __ballot(mark[lane] == gb + 1u);
            const uint32_t le = __builtin_amdgcn_mbcnt_hi((uint32_t)(S >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)S, 0u)) +
                                (uint32_t)((S >> lane) & 1ull);
            const uint32_t k = tbase + le - 1u;
            tbase += (uint32_t)__builtin_popcountll(S);
            const uint32_t o = gb + lane;
            const bool live = g + lane < total;
            const uint32_t tInf = (uint32_t)__shfl((int)tinfo, (int)k);
            uint32_t val = 0;
            int ptr = -1;
            if (live) {
                if (tInf >> 31) {
                    val = inr[(o + tInf) & imask];
                } else {
                    const uint32_t so = o - tInf;
                    if (so >= gb) ptr = (int)(so - gb);
                    else val = outr[so & omask];
                }
            }
            /* in-group back-references (runs): pointer doubling */
            while (__ballot(ptr >= 0)) {
                const int pi = ptr >= 0 ? ptr : (int)lane;
                const uint32_t pv = (uint32_t)__shfl((int)val, pi);
                const int pp = __shfl(ptr, pi);
                if (ptr >= 0) { val = pv; ptr = pp; }
            }
            if (live) {
                outr[o & omask] = (uint8_t)val;
                dst[o] = (uint8_t)val;
            }
            cd_fence();
        }
        O += total;
        /* next round: the token after the last one of this round */
        base = base + cd_rl(x + tsz, ntok - 1u);
    }
    if (lane == 0) {
        bt.out_len[v] = err ? 0u : O;
        bt.err[v] = err;
    }
}

hipError_t lzf_launch_decompress(const LzfBatch &b, hipStream_t s)
{
    uint32_t ring = 256u;
    while (ring < b.max_len && ring < CD_OUT_MAX) ring <<= 1;
    const size_t lds = CD_IN_RING + ring + CD_LANES * 4u;     /* + the 64 marks */
    hipError_t e = hipFuncSetAttribute((const void *)lzf_decompress_tokpar_kernel,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lzf_decompress_tokpar_kernel, dim3(b.count), dim3(CD_LANES), lds, s, b, ring);
    return hipGetLastError();
}

const char *lzf_decompress_kernel_name(void) { return "tokpar64"; }

/*
 * wparse_sim.c -- CPU simulation of the window-parallel parse (design aid and
 * the executable spec of lzf_wparse.hip; not part of the product or tests).
 *
 * One wave per value, 64 positions per window.  Per position p the only
 * precomputed input is q1(p), the latest earlier position with p's slot
 * (all positions; kernel 1).  The parse keeps a ring R over the last 8192
 * positions: R(x) = x if x is inserted, else the latest inserted earlier
 * position with x's slot.  The reference's ref at a visited p
 * (src/lzf_c.c:147-149) is then R(q1(p)) -- for q1(p) outside the window
 * one ring read; inside the window the same-slot lanes are resolved against
 * the window's inserted mask.  Per window:
 *   1. links: x = q1(p); same-slot lanes of the window SM(p) and the chain's
 *      exit xo(p) by pointer doubling; r_out = R(xo) from the ring;
 *   2. 16 bytes at p, at r_out (and at x through lane x) -> LCP, capped 16;
 *   3. a scalar walk over the window's stop lanes (possible matches, and
 *      lanes whose ref depends on the window's inserted mask), literals
 *      between them skipped by find-first-set;
 *   4. emission: sizes by masks and popcounts, one prefix sum;
 *   5. ring update for the window's positions.
 * Checked against oracle_lzf_compress on the synthetic generators.
 *
 *   gcc -O2 -I gibson_amd/csrc tools/wparse_sim.c oracle/lzf_oracle.c -o /tmp/wparse_sim
 *   /tmp/wparse_sim <kind> <n> <count> <seed>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "synth.h"

unsigned int oracle_lzf_compress(const void *in_data, unsigned int in_len, void *out_data, unsigned int out_len);

#define NONE 0xFFFFFFFFu
#define RNONE 0xFFFFu

static inline uint32_t slot(const uint8_t *b, uint32_t p)
{
    uint32_t hi = ((uint32_t)b[p] << 8) | b[p + 1];
    uint32_t lo = ((uint32_t)b[p + 1] << 8) | b[p + 2];
    return (hi - 5u * lo) & 0xFFFFu;
}
static inline int msb64(uint64_t m) { return 63 - __builtin_clzll(m); }
static inline uint64_t bits_from(uint32_t i) { return i >= 64 ? 0 : (~0ull << i); }
static inline uint64_t bits_below(uint32_t i) { return i >= 64 ? ~0ull : ((1ull << i) - 1); }

static uint32_t lcp_cap(const uint8_t *b, uint32_t n, uint32_t p, uint32_t r, uint32_t cap)
{
    uint32_t k = 0;
    while (k < cap && p + k < n && b[p + k] == b[r + k]) k++;
    return k;
}

/* statistics */
static uint64_t st_orbits, st_long, st_maxorb;
static uint64_t st_windows, st_active, st_iters, st_rounds, st_slow, st_ext, st_dstop;

static void put(uint8_t *out, uint32_t cap, uint32_t i, uint8_t v)
{
    if (i < cap) out[i] = v;
}

static uint32_t wparse(const uint8_t *b, uint32_t n, const uint16_t *rec, uint8_t *out, uint32_t cap)
{
    if (n == 0 || cap == 0) return 0;
    static uint16_t ring[8192];
    const uint32_t np = n >= 3 ? n - 2 : 0;
    uint32_t c = 0, S = 0, j0 = 0;
    int ok = 1, done = 0;
    uint32_t t1 = NONE, t2 = NONE;              /* tails of the last match */
    for (uint32_t w = 0; w < np; w += 64) {
        st_windows++;
        const uint32_t L = np - w < 64 ? np - w : 64;
        uint32_t x[64], xo[64], r_out[64], LA[64], LB[64];
        int link[64];
        uint64_t SM[64];
        int D[64], dA[64], dB[64];
        for (uint32_t l = 0; l < L; l++) {
            const uint32_t p = w + l;
            x[l] = rec[p] == RNONE ? NONE : p - rec[p] - 1u;
            D[l] = x[l] != NONE && x[l] >= w;
            link[l] = D[l] ? (int)(x[l] - w) : -1;
            xo[l] = (x[l] != NONE && x[l] < w) ? x[l] : NONE;
            SM[l] = 0;
        }
        for (;;) {                                  /* pointer doubling */
            int any = 0;
            for (uint32_t l = 0; l < L; l++) any |= link[l] >= 0;
            if (!any) break;
            st_rounds++;
            int olink[64];
            uint32_t oxo[64];
            uint64_t oSM[64];
            memcpy(olink, link, sizeof link);
            memcpy(oxo, xo, sizeof xo);
            memcpy(oSM, SM, sizeof SM);
            for (uint32_t l = 0; l < L; l++)
                if (olink[l] >= 0) {
                    const int t = olink[l];
                    SM[l] |= (1ull << t) | oSM[t];
                    xo[l] = oxo[t];
                    link[l] = olink[t];
                }
        }
        for (uint32_t l = 0; l < L; l++) {
            const uint32_t p = w + l;
            r_out[l] = NONE;
            if (xo[l] != NONE) {
                const uint16_t e = ring[xo[l] & 8191u];
                r_out[l] = e == RNONE ? NONE : xo[l] - e;
            }
#define REFVALID(p_, r_) ((r_) != NONE && (r_) > 0u && (p_) - (r_) - 1u < 8192u && (p_) + 4u < n)
            LA[l] = D[l] ? lcp_cap(b, n, p, x[l], 16) : 0;
            LB[l] = r_out[l] != NONE ? lcp_cap(b, n, p, r_out[l], 16) : 0;
            dA[l] = D[l] && REFVALID(p, x[l]) && LA[l] >= 3;
            dB[l] = REFVALID(p, r_out[l]) && LB[l] >= 3;
        }
        uint64_t STOP = 0;
        for (uint32_t l = 0; l < L; l++)
            if (D[l] || dB[l]) STOP |= 1ull << l;
        /* inserted mask of the window: tails of the last match */
        uint64_t INS = 0, VIS = 0, MS = 0;
        if (t1 != NONE && t1 >= w && t1 < w + 64) INS |= 1ull << (t1 - w);
        if (t2 != NONE && t2 >= w && t2 < w + 64) INS |= 1ull << (t2 - w);
        uint32_t toklen[64], tokoff[64];
        if (!done && c < w + L) {
            st_active++;
            {   /* model: VALU orbit by fixed-point iteration over the window's inserted mask */
                uint64_t G = ~0ull;                   /* guess: in-window nodes >= c inserted */
                const uint64_t known = INS;           /* nodes < c: tails only */
                int iters = 0, nlong = 0;
                for (;;) {
                    iters++;
                    uint64_t Ig = (known & bits_below(c - w)) | (G & bits_from(c - w));
                    uint32_t nx[64];
                    for (uint32_t l = 0; l < L; l++) {
                        const uint32_t p = w + l;
                        uint32_t ref = r_out[l], len = LB[l];
                        int mt = dB[l];
                        if (D[l]) {
                            const uint64_t cand = SM[l] & Ig & bits_below(l);
                            if (cand) {
                                ref = w + (uint32_t)msb64(cand);
                                len = lcp_cap(b, n, p, ref, 16);
                                mt = REFVALID(p, ref) && len >= 3;
                            }
                        }
                        uint32_t maxlen = n - p - 2u; if (maxlen > 264u) maxlen = 264u;
                        const uint32_t lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
                        if (mt && len >= 16u && lim > 16u) { len = 16u + lcp_cap(b, n, p + 16u, ref + 16u, lim - 16u); if (l + 16 < 64) nlong++; }
                        nx[l] = mt ? (len < lim ? len : lim) : 1u;
                    }
                    uint64_t V2 = 0, I2 = known & bits_below(c - w);
                    uint32_t cc = c;
                    while (cc < w + L) {
                        const uint32_t l = cc - w;
                        V2 |= 1ull << l; I2 |= 1ull << l;
                        const uint32_t e = cc + nx[l];
                        if (nx[l] > 1u && e < np) {
                            if (e - 2u < w + 64) I2 |= 1ull << (e - 2u - w);
                            if (e - 1u < w + 64) I2 |= 1ull << (e - 1u - w);
                        }
                        if (nx[l] > 1u && e >= np) break;
                        cc = e;
                    }
                    if (((I2 ^ Ig) & bits_below(L)) == 0 || iters > 64) break;
                    G = I2;
                }
                st_orbits += iters;
                st_long += nlong;
                if (iters > st_maxorb) st_maxorb = iters;
            }
            while (c < w + L) {
                st_iters++;
                const uint32_t i = c - w;
                const uint64_t s = STOP & bits_from(i) & bits_below(L);
                if (!s) {
                    VIS |= bits_from(i) & bits_below(L);
                    INS |= bits_from(i) & bits_below(L);
                    c = w + L;
                    break;
                }
                const uint32_t m = (uint32_t)__builtin_ctzll(s);
                const uint64_t run = bits_from(i) & bits_below(m + 1);
                VIS |= run;
                INS |= run;
                const uint32_t p = w + m;
                uint32_t ref, len;
                int match;
                if (D[m]) {
                    st_dstop++;
                    const uint32_t xl = x[m] - w;
                    if ((INS >> xl) & 1u) {
                        ref = x[m];
                        len = LA[m];
                        match = dA[m];
                    } else {
                        const uint64_t deeper = SM[m] & INS;
                        if (deeper) {
                            st_slow++;
                            ref = w + (uint32_t)msb64(deeper);
                            len = lcp_cap(b, n, p, ref, 16);
                            match = REFVALID(p, ref) && len >= 3;
                        } else {
                            ref = r_out[m];
                            len = LB[m];
                            match = dB[m];
                        }
                    }
                } else {
                    ref = r_out[m];
                    len = LB[m];
                    match = dB[m];
                }
                if (!match) {
                    c = p + 1;
                    continue;
                }
                uint32_t maxlen = n - p - 2u;
                if (maxlen > 264u) maxlen = 264u;
                const uint32_t lim = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
                if (len >= 16u && lim > 16u) {
                    st_ext++;
                    len = 16u + lcp_cap(b, n, p + 16u, ref + 16u, lim - 16u);
                }
                const uint32_t mlen = len < lim ? len : lim;
                MS |= 1ull << m;
                toklen[m] = mlen;
                tokoff[m] = p - ref - 1u;
                c = p + mlen;
                t1 = t2 = NONE;
                if (c >= np) {
                    done = 1;
                    break;
                }
                t1 = c - 2u;
                t2 = c - 1u;
                if (t1 < w + 64) INS |= 1ull << (t1 - w);
                if (t2 < w + 64) INS |= 1ull << (t2 - w);
            }
            if (c >= np) done = 1;
            /* emission: sizes by masks, offsets by a prefix sum */
            const uint64_t LM = VIS & ~MS;
            uint32_t size[64], jj[64];
            for (uint32_t l = 0; l < 64; l++) {
                size[l] = 0;
                if (!((VIS >> l) & 1u)) continue;
                const uint64_t below = bits_below(l);
                const uint64_t pm = MS & below;
                uint32_t rp;
                if (pm) {
                    const int lm = msb64(pm);
                    rp = (uint32_t)__builtin_popcountll(LM & below & bits_from((uint32_t)lm + 1u));
                } else {
                    rp = j0 + (uint32_t)__builtin_popcountll(LM & below);
                }
                jj[l] = rp & 31u;
                if ((MS >> l) & 1u) size[l] = toklen[l] - 2u < 7u ? 2u : 3u;
                else size[l] = jj[l] == 0u ? 2u : 1u;
            }
            uint32_t off = S;
            for (uint32_t l = 0; l < 64; l++) {
                if (!((VIS >> l) & 1u)) continue;
                const uint32_t p = w + l;
                if ((MS >> l) & 1u) {
                    if (jj[l]) put(out, cap, off - jj[l] - 1u, (uint8_t)(jj[l] - 1u));
                    if (off + 4u >= cap) ok = 0;                    /* src/lzf_c.c:176 */
                    const uint32_t Lm = toklen[l] - 2u, of = tokoff[l];
                    if (Lm < 7u) {
                        put(out, cap, off, (uint8_t)((of >> 8) | (Lm << 5)));
                        put(out, cap, off + 1u, (uint8_t)of);
                    } else {
                        put(out, cap, off, (uint8_t)((of >> 8) | (7u << 5)));
                        put(out, cap, off + 1u, (uint8_t)(Lm - 7u));
                        put(out, cap, off + 2u, (uint8_t)of);
                    }
                } else {
                    const uint32_t bi = off + (jj[l] == 0u ? 1u : 0u);
                    if (bi >= cap) ok = 0;                          /* src/lzf_c.c:263 */
                    put(out, cap, bi, b[p]);
                    if (jj[l] == 31u) put(out, cap, bi - 32u, 31u);
                }
                off += size[l];
            }
            /* carry: literals of the open chunk */
            if (MS) {
                const int lm = msb64(MS);
                j0 = (uint32_t)__builtin_popcountll(LM & bits_from((uint32_t)lm + 1u)) & 31u;
            } else {
                j0 = (j0 + (uint32_t)__builtin_popcountll(LM)) & 31u;
            }
            S = off;
        }
        /* ring update */
        for (uint32_t l = 0; l < L; l++) {
            const uint32_t p = w + l;
            uint16_t e;
            if ((INS >> l) & 1u) {
                e = 0;
            } else {
                const uint64_t deeper = SM[l] & INS;
                const uint32_t ref = deeper ? w + (uint32_t)msb64(deeper) : r_out[l];
                e = (ref == NONE || ref == 0u || p - ref > 8191u) ? RNONE : (uint16_t)(p - ref);
            }
            ring[p & 8191u] = e;
        }
    }
    if (!ok) return 0;
    if (S + (j0 == 0u ? 1u : 0u) + 3u > cap) return 0;              /* src/lzf_c.c:276 */
    for (uint32_t p = c; p < n; p++) {                              /* src/lzf_c.c:279-288 */
        const uint32_t bi = S + (j0 == 0u ? 1u : 0u);
        put(out, cap, bi, b[p]);
        S = bi + 1u;
        j0 = (j0 + 1u) & 31u;
        if (j0 == 0u) put(out, cap, S - 33u, 31u);
    }
    if (j0) put(out, cap, S - j0 - 1u, (uint8_t)(j0 - 1u));
    return S;
}


/* ---- v2: per-lane decisions (VALU), lean scalar walk, fixed-point check --- */
static uint64_t v2_iters, v2_windows, v2_needext, v2_lastext, v2_stops, v2_maxit;

static uint32_t wparse2(const uint8_t *b, uint32_t n, const uint16_t *rec, uint8_t *out, uint32_t cap)
{
    if (n == 0 || cap == 0) return 0;
    static uint16_t ring[8192];
    const uint32_t np = n >= 3 ? n - 2 : 0;
    uint32_t c = 0, S = 0, j0 = 0;
    int ok = 1, done = np == 0;
    uint32_t t1 = NONE, t2 = NONE;
    for (uint32_t w = 0; !done && w < np; w += 64) {
        const uint32_t L = np - w < 64 ? np - w : 64;
        uint32_t x[64], xo[64], r_out[64], LA[64], LB[64], lim[64];
        int link[64], D[64];
        uint64_t SM[64];
        for (uint32_t l = 0; l < 64; l++) {
            const uint32_t p = w + l;
            x[l] = (l < L && rec[p] != RNONE) ? p - rec[p] - 1u : NONE;
            D[l] = x[l] != NONE && x[l] >= w;
            link[l] = D[l] ? (int)(x[l] - w) : -1;
            xo[l] = (x[l] != NONE && x[l] < w) ? x[l] : NONE;
            SM[l] = 0;
        }
        for (;;) {
            int any = 0;
            for (uint32_t l = 0; l < 64; l++) any |= link[l] >= 0;
            if (!any) break;
            int olink[64]; uint32_t oxo[64]; uint64_t oSM[64];
            memcpy(olink, link, sizeof link); memcpy(oxo, xo, sizeof xo); memcpy(oSM, SM, sizeof SM);
            for (uint32_t l = 0; l < 64; l++)
                if (olink[l] >= 0) { const int t = olink[l]; SM[l] |= (1ull << t) | oSM[t]; xo[l] = oxo[t]; link[l] = olink[t]; }
        }
        for (uint32_t l = 0; l < 64; l++) {
            const uint32_t p = w + l;
            r_out[l] = NONE;
            if (l < L && xo[l] != NONE) { const uint16_t e = ring[xo[l] & 8191u]; r_out[l] = e == RNONE ? NONE : xo[l] - e; }
            const uint32_t avail = l < L ? n - p : 0;
            LA[l] = D[l] ? lcp_cap(b, n, p, x[l], 16) : 0;
            LB[l] = (l < L && r_out[l] != NONE) ? lcp_cap(b, n, p, r_out[l], 16) : 0;
            (void)avail;
            uint32_t maxlen = l < L ? n - p - 2u : 0; if (maxlen > 264u) maxlen = 264u;
            lim[l] = (maxlen > 16u && maxlen < 19u) ? 19u : maxlen;
        }
        uint64_t INS0 = 0;
        if (t1 != NONE && t1 >= w && t1 < w + 64) INS0 |= 1ull << (t1 - w);
        if (t2 != NONE && t2 >= w && t2 < w + 64) INS0 |= 1ull << (t2 - w);
        uint64_t INS = INS0;
        if (c < w + 64) {
            v2_windows++;
            const uint32_t i0 = c - w;
            uint64_t Ig = INS0 | bits_from(i0), Ig_prev = 0;
            uint32_t refsel[64], l16[64], mlen[64], nxt[64], exact[64];
            uint32_t kref[64], kmlen[64], knxt[64], istart = i0;
            uint64_t VS = 0, V = 0;
            uint32_t iend = 0;
            int it = 0;
            for (;;) {
                it++;
                v2_iters++;
                /* per-lane decisions under Ig */
                Ig_prev = Ig;
                int match[64];
                for (uint32_t l = 0; l < 64; l++) {
                    const uint32_t p = w + l;
                    refsel[l] = NONE; l16[l] = 0; match[l] = 0;
                    if (l >= L) continue;
                    uint32_t ref = r_out[l], len = LB[l];
                    if (D[l]) {
                        const uint64_t cm = SM[l] & Ig;
                        if (cm) {
                            const uint32_t jl = (uint32_t)msb64(cm);
                            ref = w + jl;
                            len = (jl == x[l] - w) ? LA[l] : lcp_cap(b, n, p, ref, 16);
                        }
                    }
                    refsel[l] = ref; l16[l] = ref != NONE ? len : 0;
                    match[l] = REFVALID(p, ref) && len >= 3;
                }
                /* exact lengths by diagonals */
                uint64_t SAME = 0, STOP = 0;
                for (uint32_t l = 0; l + 1 < 64; l++)
                    if (l16[l] == 16 && refsel[l] != NONE && refsel[l + 1] == refsel[l] + 1) SAME |= 1ull << l;
                for (uint32_t l = 0; l < 64; l++) {
                    nxt[l] = l + 1; mlen[l] = 0; exact[l] = 1;
                    if (!match[l]) continue;
                    STOP |= 1ull << l;
                    const uint32_t de = (uint32_t)__builtin_ctzll(~SAME & bits_from(l));
                    const uint32_t lb = (de - l) + l16[de];          /* exact if l16[de] < 16 */
                    const int ex = l16[de] < 16 || lb >= lim[l];
                    mlen[l] = lb < lim[l] ? lb : lim[l];
                    exact[l] = ex;
                    nxt[l] = l + mlen[l];
                    if (!ex) { if (l + lb >= 64) nxt[l] = 64 + l + lb; else { nxt[l] = 250; v2_needext++; } }
                }
                /* the lean scalar walk, from the first lane the last pass got wrong */
                if (it > 1) {
                    for (uint32_t l = 0; l < istart; l++) { refsel[l] = kref[l]; mlen[l] = kmlen[l]; nxt[l] = knxt[l]; }
                }
                uint32_t i = istart;
                VS &= bits_below(istart);
                for (;;) {
                    const uint64_t s = STOP & (i < 64 ? (~0ull << i) : 0) & bits_below(L);
                    if (!s) { iend = L; break; }
                    const uint32_t m = (uint32_t)__builtin_ctzll(s);
                    v2_stops++;
                    VS |= 1ull << m;
                    i = nxt[m];
                    if (i >= L) {
                        if (!exact[m]) {                              /* the wave measures it */
                            const uint32_t p = w + m;
                            uint32_t len = 16u + lcp_cap(b, n, p + 16u, refsel[m] + 16u, lim[m] - 16u);
                            if (len > lim[m]) len = lim[m];
                            mlen[m] = len; exact[m] = 1; nxt[m] = m + len; i = nxt[m];
                            if (nxt[m] < 64) v2_lastext++;
                            if (i < L) continue;
                        }
                        iend = i;
                        break;
                    }
                }
                /* visited lanes and inserted mask from the walk */
                V = 0;
                uint64_t In = INS0 & bits_below(i0);
                for (uint32_t l = i0; l < L; l++) {
                    const uint64_t vb = VS & bits_below(l + 1);
                    int vis;
                    uint32_t e = 0;
                    if (!vb) vis = 1;
                    else { const uint32_t lv = (uint32_t)msb64(vb); e = nxt[lv]; vis = l == lv || l >= e; }
                    if (vis) { V |= 1ull << l; In |= 1ull << l; }
                    else if (w + e < np + 0 && (l + 2 == e || l + 1 == e)) In |= 1ull << l;
                }
                /* consistency of the visited in-window refs */
                int bad = 0;
                for (uint32_t l = 0; l < L; l++) {
                    if (!((V >> l) & 1) || !D[l]) continue;
                    const uint64_t a = SM[l] & Ig, bb = SM[l] & In;
                    const int ma = a ? msb64(a) : -1, mb = bb ? msb64(bb) : -1;
                    if (ma != mb) bad = 1;
                }
                if (!bad || it >= 64) { INS = In; break; }
                Ig = In | bits_from(L);
                istart = 64;
                for (uint32_t l = 0; l < L; l++) {
                    if (!((V >> l) & 1) || !D[l]) continue;
                    const uint64_t a = SM[l] & Ig, bb = SM[l] & In;
                    (void)a; (void)bb;
                }
                {
                    uint64_t Bm = 0;
                    const uint64_t Igp = Ig_prev;
                    for (uint32_t l = 0; l < L; l++) {
                        if (!((V >> l) & 1) || !D[l]) continue;
                        const uint64_t a = SM[l] & Igp, bb = SM[l] & In;
                        if ((a ? msb64(a) : -1) != (bb ? msb64(bb) : -1)) Bm |= 1ull << l;
                    }
                    istart = (uint32_t)__builtin_ctzll(Bm);
                }
                memcpy(kref, refsel, sizeof kref); memcpy(kmlen, mlen, sizeof kmlen); memcpy(knxt, nxt, sizeof knxt);
            }
            if ((uint64_t)it > v2_maxit) v2_maxit = it;
            /* c, tails */
            const uint32_t ce = w + iend;
            c = ce;
            t1 = t2 = NONE;
            if (c >= np) done = 1;
            else if (VS && nxt[msb64(VS)] == iend) {
                t1 = c - 2; t2 = c - 1;
                /* tails past the window stay in t1/t2; INS already has those inside */
            }
            /* emission (as v1) */
            const uint64_t MS = VS, LM = V & ~MS;
            uint32_t size[64], jj[64];
            for (uint32_t l = 0; l < 64; l++) {
                size[l] = 0;
                if (!((V >> l) & 1u)) continue;
                const uint64_t below = bits_below(l), pm = MS & below;
                uint32_t rp;
                if (pm) { const int lm = msb64(pm); rp = (uint32_t)__builtin_popcountll(LM & below & bits_from((uint32_t)lm + 1u)); }
                else rp = j0 + (uint32_t)__builtin_popcountll(LM & below);
                jj[l] = rp & 31u;
                if ((MS >> l) & 1u) size[l] = mlen[l] - 2u < 7u ? 2u : 3u;
                else size[l] = jj[l] == 0u ? 2u : 1u;
            }
            uint32_t off = S;
            for (uint32_t l = 0; l < 64; l++) {
                if (!((V >> l) & 1u)) continue;
                const uint32_t p = w + l;
                if ((MS >> l) & 1u) {
                    if (jj[l]) put(out, cap, off - jj[l] - 1u, (uint8_t)(jj[l] - 1u));
                    if (off + 4u >= cap) ok = 0;
                    const uint32_t Lm = mlen[l] - 2u, of = p - refsel[l] - 1u;
                    if (Lm < 7u) { put(out, cap, off, (uint8_t)((of >> 8) | (Lm << 5))); put(out, cap, off + 1u, (uint8_t)of); }
                    else { put(out, cap, off, (uint8_t)((of >> 8) | (7u << 5))); put(out, cap, off + 1u, (uint8_t)(Lm - 7u)); put(out, cap, off + 2u, (uint8_t)of); }
                } else {
                    const uint32_t bi = off + (jj[l] == 0u ? 1u : 0u);
                    if (bi >= cap) ok = 0;
                    put(out, cap, bi, b[p]);
                    if (jj[l] == 31u) put(out, cap, bi - 32u, 31u);
                }
                off += size[l];
            }
            if (MS) { const int lm = msb64(MS); j0 = (uint32_t)__builtin_popcountll(LM & bits_from((uint32_t)lm + 1u)) & 31u; }
            else j0 = (j0 + (uint32_t)__builtin_popcountll(LM)) & 31u;
            S = off;
            if (!ok) return 0;
        }
        if (done) break;
        for (uint32_t l = 0; l < L; l++) {
            const uint32_t p = w + l;
            uint16_t e;
            if ((INS >> l) & 1u) e = 0;
            else {
                const uint64_t deeper = SM[l] & INS;
                const uint32_t ref = deeper ? w + (uint32_t)msb64(deeper) : r_out[l];
                e = (ref == NONE || ref == 0u || p - ref > 8191u) ? RNONE : (uint16_t)(p - ref);
            }
            ring[p & 8191u] = e;
        }
    }
    if (!ok) return 0;
    if (S + (j0 == 0u ? 1u : 0u) + 3u > cap) return 0;
    for (uint32_t p = c; p < n; p++) {
        const uint32_t bi = S + (j0 == 0u ? 1u : 0u);
        put(out, cap, bi, b[p]);
        S = bi + 1u;
        j0 = (j0 + 1u) & 31u;
        if (j0 == 0u) put(out, cap, S - 33u, 31u);
    }
    if (j0) put(out, cap, S - j0 - 1u, (uint8_t)(j0 - 1u));
    return S;
}

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 2;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
    uint32_t count = argc > 3 ? (uint32_t)atoi(argv[3]) : 20;
    uint64_t seed = argc > 4 ? strtoull(argv[4], 0, 0) : 0x5EED0003ull;
    uint8_t *b = malloc(n + 64), *o1 = malloc(n + 1024), *o2 = malloc(n + 1024);
    uint16_t *rec = malloc((size_t)n * 2 + 2);
    uint32_t *last = malloc(65536 * 4);
    uint64_t bad = 0, cases = 0;
    for (uint32_t v = 0; v < count; v++) {
        uint32_t nn = n;
        if (kind == 99) nn = 1u + (uint32_t)((v * 2654435761u) % n);   /* ragged sizes, mixed kinds */
        int kd = kind == 99 ? (int)(v % 6u) : kind;
        syn_generate(kd, seed, v, b, nn);
        memset(b + nn, 0xAB, 64);
        for (uint32_t s = 0; s < 65536; s++) last[s] = NONE;
        for (uint32_t p = 0; p + 2 < nn; p++) {
            uint32_t s = slot(b, p);
            rec[p] = (last[s] != NONE && p - last[s] - 1u < 8192u) ? (uint16_t)(p - last[s] - 1u) : RNONE;
            last[s] = p;
        }
        const uint32_t caps[4] = {nn > 4 ? nn - 4 : 0, nn + nn / 16 + 64, nn / 2, (uint32_t)(v * 7919u) % (nn + 8)};
        for (int k = 0; k < 4; k++) {
            memset(o1, 0xCD, nn + 1024);
            memset(o2, 0xCD, nn + 1024);
            uint32_t r1 = oracle_lzf_compress(b, nn, o1, caps[k]);
            uint32_t r2 = wparse(b, nn, rec, o2, caps[k]);
            {
                static uint8_t o3[1 << 21];
                memset(o3, 0xCD, nn + 1024);
                uint32_t r3 = wparse2(b, nn, rec, o3, caps[k]);
                if (r1 != r3 || memcmp(o1, o3, r1)) {
                    if (bad < 5) fprintf(stderr, "V2 MISMATCH v %u n %u kind %d cap %u: oracle %u v2 %u\n", v, nn, kd, caps[k], r1, r3);
                    bad++;
                }
            }
            cases++;
            if (r1 != r2 || memcmp(o1, o2, r1)) {
                if (bad < 5) fprintf(stderr, "MISMATCH v %u n %u kind %d cap %u: oracle %u sim %u\n", v, nn, kd, caps[k], r1, r2);
                bad++;
            }
        }
    }
    printf("kind %d n %u count %u: cases %llu mismatches %llu\n", kind, n, count, (unsigned long long)cases,
           (unsigned long long)bad);
    printf("windows %llu active %.1f%% iters/active %.2f doubling rounds/window %.2f slow/active %.3f ext/active %.3f "
           "Dstops/active %.2f\n",
           (unsigned long long)st_windows, 100.0 * st_active / st_windows, (double)st_iters / st_active,
           (double)st_rounds / st_windows, (double)st_slow / st_active, (double)st_ext / st_active,
           (double)st_dstop / st_active);
    printf("VALU-orbit model: orbits/active window %.2f (max %llu), long lanes (<48) per active window %.2f\n",
           (double)st_orbits / st_active, (unsigned long long)st_maxorb, (double)st_long / st_active);
    printf("v2: iterations/active window %.3f (max %llu) stops/active %.2f needext/iter %.4f lastext/active %.3f\n",
           (double)v2_iters / v2_windows, (unsigned long long)v2_maxit, (double)v2_stops / v2_iters,
           (double)v2_needext / v2_iters, (double)v2_lastext / v2_windows);
    return bad != 0;
}

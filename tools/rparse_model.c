/*
 * rparse_model.c -- CPU statistics model for the redirect formulation of the
 * greedy parse (design aid, not part of the product or the tests).
 *
 * Claim checked here on every visited position: with q1(x) = the latest
 * earlier position with x's slot (all positions) and
 *     R(x) = x            if x is inserted (visited, or one of a match's
 *                          last two positions, src/lzf_c.c:227-247)
 *          = R(q1(x))     otherwise,
 * the reference's ref at a visited p (src/lzf_c.c:147-149) is R(q1(p)).
 *
 * Reports, per value, the quantities that size a window-parallel parse
 * (one wave per value, 64 positions per window): active windows, matches per
 * active window, how often ref == q1, match lengths, in-window q1 links.
 *
 *   gcc -O2 -I gibson_amd/csrc tools/rparse_model.c -o /tmp/rparse_model
 *   /tmp/rparse_model <kind> <n> <count> <seed>
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "synth.h"

static inline uint32_t slot(const uint8_t *b, uint32_t p)
{
    uint32_t hi = ((uint32_t)b[p] << 8) | b[p + 1];
    uint32_t lo = ((uint32_t)b[p + 1] << 8) | b[p + 2];
    return (hi - 5u * lo) & 0xFFFFu;
}

#define NONE 0xFFFFFFFFu

static uint32_t lcp(const uint8_t *b, uint32_t n, uint32_t p, uint32_t r, uint32_t cap)
{
    uint32_t k = 0;
    while (k < cap && p + k < n && b[p + k] == b[r + k]) k++;
    return k;
}

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 2;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
    uint32_t count = argc > 3 ? (uint32_t)atoi(argv[3]) : 100;
    uint64_t seed = argc > 4 ? strtoull(argv[4], 0, 0) : 0x5EED0003ull;
    uint8_t *b = malloc(n + 64);
    uint32_t *last = malloc(65536 * 4), *tab = malloc(65536 * 4);
    uint32_t *q1 = malloc((size_t)n * 4), *R = malloc((size_t)n * 4);
    uint8_t *ins = malloc(n), *vis = malloc(n), *mst = malloc(n);
    uint32_t *mlen = malloc((size_t)n * 4);
    uint64_t visited = 0, lits = 0, matches = 0, refq1 = 0, bad = 0, wins = 0, actwins = 0;
    uint64_t lhist[8] = {0};       /* match length: <=7, <=16, <=32, <=64, <=128, <=264 */
    uint64_t mpw_hist[10] = {0};   /* matches per active window */
    uint64_t inwin_q1_vis = 0, l1_ge32_vis = 0, long_spec = 0, win_long_spec = 0;
    uint64_t refne_l1lt = 0, refne_eq = 0;
    for (uint32_t v = 0; v < count; v++) {
        syn_generate(kind, seed, v, b, n);
        memset(b + n, 0, 64);
        memset(last, 0xFF, 65536 * 4);
        for (uint32_t p = 0; p + 2 < n; p++) {
            uint32_t s = slot(b, p);
            q1[p] = last[s];
            last[s] = p;
        }
        /* the reference parse */
        memset(tab, 0xFF, 65536 * 4);
        memset(ins, 0, n);
        memset(vis, 0, n);
        memset(mst, 0, n);
        uint32_t p = 0, rdone = 0;
        while (n >= 3 && p < n - 2) {
            for (; rdone < p; rdone++) R[rdone] = ins[rdone] ? rdone : (q1[rdone] == NONE ? NONE : R[q1[rdone]]);
            uint32_t s = slot(b, p), r = tab[s];
            tab[s] = p;
            ins[p] = vis[p] = 1;
            visited++;
            int hit = r != NONE && (p - r - 1) < 8192 && p + 4 < n && r > 0 && b[r] == b[p] &&
                      b[r + 1] == b[p + 1] && b[r + 2] == b[p + 2];
            /* R formulation */
            uint32_t x = q1[p];
            uint32_t rr = x == NONE ? NONE : R[x];
            if (rr != r) {
                /* the table may hold an entry the R chain does not: same slot */
                bad++;
            }
            if (!hit) { lits++; p++; continue; }
            uint32_t maxlen = n - p - 2; if (maxlen > 264) maxlen = 264;
            uint32_t lim = maxlen; if (maxlen > 16 && lim < 19) lim = 19;
            uint32_t k = 3; while (k < lim && b[r + k] == b[p + k]) k++;
            matches++;
            refq1 += (r == x);
            mst[p] = 1; mlen[p] = k;
            lhist[k <= 7 ? 0 : k <= 16 ? 1 : k <= 32 ? 2 : k <= 64 ? 3 : k <= 128 ? 4 : 5]++;
            if (r != x) {
                uint32_t a = lcp(b, n, p, x, 300), d = lcp(b, n, x, r, 300);
                if (a != d) refne_l1lt++; else refne_eq++;
            }
            p += k;
            if (p >= n - 2) break;
            ins[p - 2] = ins[p - 1] = 1;
            tab[slot(b, p - 2)] = p - 2;
            tab[slot(b, p - 1)] = p - 1;
            continue;
        }
        /* R: in position order */
        for (uint32_t t = 0; t + 2 < n; t++) R[t] = ins[t] ? t : (q1[t] == NONE ? NONE : R[q1[t]]);
        /* re-check the claim with the final R (R[x] for x < p is final when p is visited) */
        /* window statistics */
        uint32_t entry = 0;
        for (uint32_t w = 0; w + 2 < n; w += 64) {
            wins++;
            uint32_t we = w + 64 < n - 2 ? w + 64 : n - 2;
            int act = 0, mc = 0;
            for (uint32_t t = w; t < we; t++) {
                if (vis[t]) act = 1;
                if (mst[t]) mc++;
                if (vis[t] && q1[t] != NONE && q1[t] >= w) inwin_q1_vis++;
            }
            if (act) {
                actwins++;
                mpw_hist[mc < 9 ? mc : 9]++;
                /* speculative lanes from the first visited position on: LCP(p, R(q1(p))) > 32 */
                int any = 0;
                uint32_t first = w; while (first < we && !vis[first]) first++;
                for (uint32_t t = first; t < we; t++) {
                    uint32_t x = q1[t];
                    if (x == NONE) continue;
                    uint32_t r = R[x];
                    if (r == NONE || r == 0 || t - r - 1 >= 8192) continue;
                    if (lcp(b, n, t, r, 40) > 32) { long_spec++; any = 1; }
                }
                win_long_spec += any;
            }
            (void)entry;
        }
        for (uint32_t t = 0; t + 2 < n; t++)
            if (vis[t] && q1[t] != NONE && lcp(b, n, t, q1[t], 40) >= 32) l1_ge32_vis++;
    }
    printf("kind %d n %u count %u\n", kind, n, count);
    printf("per value: visited %.0f literals %.0f matches %.0f (ref==q1 %.1f%%) claim-mismatch %llu\n",
           (double)visited / count, (double)lits / count, (double)matches / count,
           100.0 * refq1 / (matches ? matches : 1), (unsigned long long)bad);
    printf("ref!=q1 matches: LCP(p,q1)!=LCP(q1,ref) %.1f%%, equal %.1f%%\n",
           100.0 * refne_l1lt / (refne_l1lt + refne_eq + 1e-9), 100.0 * refne_eq / (refne_l1lt + refne_eq + 1e-9));
    printf("windows %.0f active %.0f (%.1f%%)\n", (double)wins / count, (double)actwins / count,
           100.0 * actwins / wins);
    printf("match len hist <=7 %.1f%% <=16 %.1f%% <=32 %.1f%% <=64 %.1f%% <=128 %.1f%% <=264 %.1f%%\n",
           100.0 * lhist[0] / matches, 100.0 * lhist[1] / matches, 100.0 * lhist[2] / matches,
           100.0 * lhist[3] / matches, 100.0 * lhist[4] / matches, 100.0 * lhist[5] / matches);
    printf("matches per active window:");
    for (int i = 0; i < 10; i++) printf(" %d:%.1f%%", i, 100.0 * mpw_hist[i] / actwins);
    printf("\nvisited with in-window q1 %.2f%%; visited with LCP(p,q1)>=32 %.1f%%\n",
           100.0 * inwin_q1_vis / visited, 100.0 * l1_ge32_vis / visited);
    printf("speculative lanes (>= first visited) with LCP(p,ref)>32: %.2f per active window; windows with any %.1f%%\n",
           (double)long_spec / actwins, 100.0 * win_long_spec / actwins);
    return 0;
}

/*
 * parse_model.c -- CPU statistics model of the lane-generation compressor
 * (DESIGN.md §4.1).  A design aid, not part of the product or the tests.
 *
 * For synthetic values it runs the reference parse (oracle semantics,
 * src/lzf_c.c:98-294) and beside it the cand-chain formulation of
 * lzf_lane.hip, checks that both choose the same ref everywhere, and reports
 * per value: parse steps, literals, matches, chain walks past skipped
 * positions, how far back the candidate lies (which decides whether the
 * inserted-bitmap word is in registers), match lengths, and the bucket-chain
 * hops kernel 1 needs for a given bucket count.
 *
 *   gcc -O2 -I gibson_amd/csrc tools/parse_model.c -o /tmp/parse_model
 *   /tmp/parse_model <kind> <n> <count> [bucket_bits]
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

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 1;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 4096;
    uint32_t count = argc > 3 ? (uint32_t)atoi(argv[3]) : 1000;
    uint32_t bbits = argc > 4 ? (uint32_t)atoi(argv[4]) : 12;
    uint8_t *b = malloc(n + 64);
    uint32_t *tab = malloc(65536 * 4), *last = malloc(65536 * 4), *bhead = malloc(65536 * 4);
    uint32_t *cand = malloc((size_t)n * 4), *bprev = malloc((size_t)n * 4), *link = malloc((size_t)n * 4);
    uint8_t *ins = malloc(n);
    uint64_t steps = 0, lits = 0, matches = 0, walks = 0, hops = 0, maxhop = 0, mism = 0;
    uint64_t dist_hist[6] = {0}, mlen_hist[8] = {0}, backd[6] = {0};
    uint64_t sk_hops = 0, sk_max_win = 0, wins = 0, truncs = 0, k1hops = 0, k1max_win = 0, k1first = 0, maxsteps = 0;
    for (uint32_t v = 0; v < count; v++) {
        syn_generate(kind, 0x5EED0002ull + kind, v, b, n);
        memset(tab, 0xFF, 65536 * 4);
        memset(last, 0xFF, 65536 * 4);
        memset(bhead, 0xFF, 65536 * 4);
        memset(ins, 0, n);
        /* kernel 1: cand + bucket-chain hops (mix = slot*40503, bucket = top bits) */
        for (uint32_t P = 0; P + 2 < n; P += 64) {
            uint64_t wmax = 0, swmax = 0;
            for (uint32_t p = P; p < P + 64 && p + 2 < n; p++) {
                uint32_t s = slot(b, p);
                uint32_t m = (s * 40503u) & 0xFFFFu, bk = m >> (16 - bbits);
                cand[p] = last[s];
                last[s] = p;
                bprev[p] = bhead[bk];
                bhead[bk] = p;
                uint32_t h = 0, e = bprev[p];
                while (e != NONE && slot(b, e) != s && p - e <= 8192) { e = bprev[e]; h++; }
                k1hops += h;
                if (h > wmax) wmax = h;
                /* skip links: link(p) = latest earlier bucket position with another slot */
                {
                    uint32_t r = bprev[p];
                    link[p] = r == NONE ? NONE : (slot(b, r) != s ? r : link[r]);
                    uint32_t hs = 0, c = r;
                    while (c != NONE && slot(b, c) != s) { c = link[c]; hs++; }
                    sk_hops += hs;
                    if (hs > swmax) swmax = hs;
                }
            }
            k1max_win += wmax;
            sk_max_win += swmax;
            k1first++;
        }
        uint32_t p = 0, vs = 0, ms = 0, me = 0;
        while (n >= 3 && p < n - 2) {
            vs++;
            uint32_t s = slot(b, p);
            uint32_t r = tab[s];
            tab[s] = p;
            uint32_t q = cand[p], h = 0;
            if (q != NONE && p - q - 1 < 8192) {
                uint32_t d = (p >> 5) - (q >> 5);
                dist_hist[q >= ms ? 0 : d <= 4 ? 1 : d <= 16 ? 2 : d <= 64 ? 3 : 4]++;
            }
            if (q != NONE && !ins[q]) walks++;
            while (q != NONE && !ins[q] && p - q - 1 < 8192) { q = cand[q]; h++; }
            if (q != NONE && p - q - 1 >= 8192) q = NONE;
            if (h > maxhop) maxhop = h;
            hops += h;
            uint32_t rr = (r != NONE && p - r - 1 < 8192) ? r : NONE;
            if (rr != q) mism++;
            ins[p] = 1;
            int hit = r != NONE && r < p && (p - r - 1u) < 8192 && p + 4 < n && r > 0 &&
                      b[r] == b[p] && b[r + 1] == b[p + 1] && b[r + 2] == b[p + 2];
            if (!hit) { lits++; p++; continue; }
            uint32_t maxlen = n - p - 2;
            if (maxlen > 264) maxlen = 264;
            uint32_t lim = maxlen > 16 && maxlen < 19 ? 19 : maxlen;
            uint32_t m = 3;
            while (m < lim && b[r + m] == b[p + m]) m++;
            matches++;
            uint32_t off = p - r;
            backd[off <= 16 ? 0 : off <= 256 ? 1 : off <= 1024 ? 2 : off <= 4096 ? 3 : 4]++;
            mlen_hist[m < 4 ? 0 : m < 5 ? 1 : m < 8 ? 2 : m < 16 ? 3 : m < 32 ? 4 : m < 64 ? 5 : m < 264 ? 6 : 7]++;
            ms = p;
            p += m;
            me = p;
            if (p >= n - 2) break;
            tab[slot(b, p - 2)] = p - 2; ins[p - 2] = 1;
            tab[slot(b, p - 1)] = p - 1; ins[p - 1] = 1;
        }
        (void)me;
        /* window-parse model: replay the parse in 64-position windows; a window
         * ends at its first token >= P+64 or early at the first token whose
         * same-slot predecessor lies inside the window but in a match interior */
        {
            uint8_t *ins2 = calloc(n, 1);
            uint32_t *tab2 = malloc(65536 * 4);
            memset(tab2, 0xFF, 65536 * 4);
            uint32_t pp = 0, P = 0;
            wins++;
            while (n >= 3 && pp < n - 2) {
                if (pp >= P + 64) { P = pp; wins++; }
                uint32_t q1 = cand[pp];
                if (q1 != NONE && q1 >= P && pp > P && !ins2[q1]) { P = pp; wins++; truncs++; }
                uint32_t s = slot(b, pp), r = tab2[s];
                tab2[s] = pp; ins2[pp] = 1;
                int hit = r != NONE && (pp - r - 1u) < 8192 && pp + 4 < n && r > 0 &&
                          b[r] == b[pp] && b[r + 1] == b[pp + 1] && b[r + 2] == b[pp + 2];
                if (!hit) { pp++; continue; }
                uint32_t maxlen = n - pp - 2;
                if (maxlen > 264) maxlen = 264;
                uint32_t lim = maxlen > 16 && maxlen < 19 ? 19 : maxlen, m = 3;
                while (m < lim && b[r + m] == b[pp + m]) m++;
                pp += m;
                if (pp >= n - 2) break;
                tab2[slot(b, pp - 2)] = pp - 2; ins2[pp - 2] = 1;
                tab2[slot(b, pp - 1)] = pp - 1; ins2[pp - 1] = 1;
            }
            free(ins2); free(tab2);
        }
        steps += vs;
        if (vs > maxsteps) maxsteps = vs;
    }
    double c = count;
    printf("kind %d n %u count %u bucket_bits %u\n", kind, n, count, bbits);
    printf("steps/value %.1f (max %llu)  literals %.1f  matches %.1f\n", steps / c,
           (unsigned long long)maxsteps, lits / c, matches / c);
    printf("walks/value %.2f  hops/walk %.2f  max hops %llu  ref mismatches %llu\n", walks / c,
           walks ? (double)hops / walks : 0.0, (unsigned long long)maxhop, (unsigned long long)mism);
    printf("candidate: >= last match start %.1f | <=4 words %.1f | <=16 %.1f | <=64 %.1f | older %.1f\n",
           dist_hist[0] / c, dist_hist[1] / c, dist_hist[2] / c, dist_hist[3] / c, dist_hist[4] / c);
    printf("match len [3,4,5-7,8-15,16-31,32-63,64-263,264]:");
    for (int i = 0; i < 8; i++) printf(" %.1f", mlen_hist[i] / c);
    printf("\nmatch distance [<=16, <=256, <=1K, <=4K, more]:");
    for (int i = 0; i < 5; i++) printf(" %.1f", backd[i] / c);
    printf("\nkernel-1 bucket hops/position %.3f, max-over-window %.2f per 64-window\n",
           (double)k1hops / (steps ? (double)n * count : 1.0), (double)k1max_win / k1first);
    printf("kernel-1 skip-link hops/position %.3f, max-over-window %.2f\n",
           (double)sk_hops / ((double)n * count), (double)sk_max_win / k1first);
    printf("window parse: windows/value %.1f  truncated %.1f\n", wins / c, truncs / c);
    return 0;
}

/*
 * len_model.c -- CPU model of the table generation's extension loads (a
 * design aid, not product or test code).  Runs the reference parse (oracle
 * semantics, src/lzf_c.c:98-294) over synthetic values and, at every match,
 * notes which candidate of the same-slot chain was the ref (q1, q2, deeper)
 * and the agreement length k of p and the ref.  Then counts the 16-byte
 * extension pieces the record parse (lzf_cand.hip) loads when the record
 * gives exact agreement up to E bytes for q1 and q2 (E = 8 today: codes
 * "exactly 3..7" and ">= 8"), for deeper refs from 8 on.
 *
 *   gcc -O2 -I gibson_amd/csrc tools/len_model.c -o /tmp/len_model
 *   /tmp/len_model KIND N COUNT
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

/* pieces compared from offset `from` (16 bytes each) until the first
 * mismatch at k or the reach `m` (the matched length) */
static uint32_t pieces(uint32_t k, uint32_t m, uint32_t from)
{
    if (m <= from && k < from) return 0;
    uint32_t end = k < m ? k + 1 : m;         /* bytes that must be seen */
    if (end <= from) return 0;
    return (end - from + 15) / 16;
}

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 2;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 65536;
    uint32_t count = argc > 3 ? (uint32_t)atoi(argv[3]) : 200;
    uint64_t seed = kind == 0 ? 0x5EED0004ull : kind == 2 ? 0x5EED0003ull : kind == 3 ? 0x5EED0005ull : 0x5EED0002ull;
    uint8_t *b = malloc(n + 300);
    uint32_t *last = malloc(65536 * 4), *q1 = malloc((size_t)n * 4), *tab = malloc(65536 * 4);
    uint8_t *ins = malloc(n);
    const uint32_t E[] = {8, 12, 16, 20, 24, 32, 48, 64, 265};
    const int NE = sizeof E / sizeof E[0];
    uint64_t pc[16] = {0}, matches = 0, depth[4] = {0}, steps = 0, khist[8] = {0};
    for (uint32_t v = 0; v < count; v++) {
        syn_generate(kind, seed, v, b, n);
        memset(b + n, 0, 300);
        memset(last, 0xFF, 65536 * 4);
        for (uint32_t p = 0; p + 2 < n; p++) {
            uint32_t s = slot(b, p);
            q1[p] = last[s];
            last[s] = p;
        }
        memset(ins, 0, n);
        memset(tab, 0xFF, 65536 * 4);
        uint32_t ip = 0;
        while (ip + 2 < n) {
            steps++;
            uint32_t s = slot(b, ip);
            uint32_t ref = tab[s];
            tab[s] = ip;
            ins[ip] = 1;
            int ok = ref != 0xFFFFFFFFu && ip - ref - 1 < 8192u && ip + 4 < n && ref > 0 && b[ref] == b[ip] &&
                     b[ref + 1] == b[ip + 1] && b[ref + 2] == b[ip + 2];
            if (!ok) {
                ip++;
                continue;
            }
            /* depth of ref on the same-slot chain */
            uint32_t c = q1[ip], d = 1;
            while (c != ref && c != 0xFFFFFFFFu && d < 3) {
                c = q1[c];
                d++;
            }
            if (c != ref) d = 3;
            depth[d]++;
            uint32_t maxlen = n - ip - 2;
            maxlen = maxlen > 264 ? 264 : maxlen;
            uint32_t k = 0;
            while (ip + k < n && b[ref + k] == b[ip + k] && k < 300) k++;
            uint32_t m;
            if (maxlen <= 16) m = k < maxlen ? k : maxlen;
            else if (k <= 18) m = k;
            else m = k < (maxlen > 19 ? maxlen : 19) ? k : (maxlen > 19 ? maxlen : 19);
            khist[k < 8 ? 0 : k < 16 ? 1 : k < 24 ? 2 : k < 32 ? 3 : k < 64 ? 4 : k < 128 ? 5 : k < 264 ? 6 : 7]++;
            matches++;
            for (int e = 0; e < NE; e++) {
                const uint32_t from = d <= 2 ? E[e] : 8u;
                pc[e] += (d <= 2 && k < E[e]) ? 0 : pieces(k, m, from);
            }
            /* the reference's advance and tail inserts (src/lzf_c.c:211-247) */
            uint32_t np = ip + m;
            if (np >= n - 2) break;
            for (uint32_t x = np - 2; x < np; x++) {
                tab[slot(b, x)] = x;
                ins[x] = 1;
            }
            ip = np;
        }
    }
    printf("kind %d n %u values %u: steps %.1f, matches %.1f per value; ref depth q1 %.1f%% q2 %.1f%% deeper %.1f%%\n",
           kind, n, count, (double)steps / count, (double)matches / count, 100.0 * depth[1] / matches,
           100.0 * depth[2] / matches, 100.0 * depth[3] / matches);
    printf("agreement k: <8 %.1f%%, 8-15 %.1f%%, 16-23 %.1f%%, 24-31 %.1f%%, 32-63 %.1f%%, 64-127 %.1f%%, 128-263 %.1f%%, >=264 %.1f%%\n",
           100.0 * khist[0] / matches, 100.0 * khist[1] / matches, 100.0 * khist[2] / matches,
           100.0 * khist[3] / matches, 100.0 * khist[4] / matches, 100.0 * khist[5] / matches,
           100.0 * khist[6] / matches, 100.0 * khist[7] / matches);
    for (int e = 0; e < NE; e++)
        printf("exact agreement up to %3u bytes in the record (q1, q2): %.0f extension pieces per value\n", E[e],
               (double)pc[e] / count);
    return 0;
}

/*
 * dist_model.c -- CPU model for the decoder's output window (a design aid,
 * not product or test code).  Compresses synthetic values with the oracle's
 * restatement of src/lzf_c.c, decodes the token stream, and reports how far
 * back-reference bytes reach: the share of output bytes and of 64-byte output
 * groups that read a byte more than W bytes back, for W = 1, 2, 4, 8 KiB
 * (a decoder with a W-byte LDS window would read those from global memory).
 *
 *   gcc -O2 -I gibson_amd/csrc tools/dist_model.c oracle/lzf_oracle.c -o /tmp/dist_model
 *   /tmp/dist_model KIND N COUNT
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "synth.h"

unsigned int oracle_lzf_compress(const void *in, unsigned int in_len, void *out, unsigned int out_len);

int main(int argc, char **argv)
{
    int kind = argc > 1 ? atoi(argv[1]) : 0;
    uint32_t n = argc > 2 ? (uint32_t)atoi(argv[2]) : 8192;
    uint32_t count = argc > 3 ? (uint32_t)atoi(argv[3]) : 2000;
    uint64_t seed = kind == 0 ? 0x5EED0004ull : kind == 2 ? 0x5EED0003ull : kind == 3 ? 0x5EED0005ull : 0x5EED0002ull;
    uint8_t *b = malloc(n + 64), *c = malloc(n + 64);
    uint32_t *dist = malloc((size_t)n * 4);
    const uint32_t W[] = {1024, 2048, 4096, 8192};
    uint64_t far_b[4] = {0}, far_g[4] = {0}, bytes = 0, groups = 0, toks = 0;
    for (uint32_t v = 0; v < count; v++) {
        syn_generate(kind, seed, v, b, n);
        const uint32_t cl = oracle_lzf_compress(b, n, c, n - 4);
        if (!cl) continue;
        uint32_t ip = 0, op = 0;
        while (ip < cl) {
            const uint32_t ctrl = c[ip++];
            toks++;
            if (ctrl < 32) {
                for (uint32_t k = 0; k <= ctrl; k++) dist[op++] = 0;
                ip += ctrl + 1;
            } else {
                uint32_t len = ctrl >> 5;
                if (len == 7) len += c[ip++];
                const uint32_t d = ((ctrl & 31u) << 8) + c[ip++] + 1u;
                for (uint32_t k = 0; k < len + 2; k++) dist[op++] = d;
            }
        }
        bytes += op;
        for (uint32_t g = 0; g < op; g += 64) {
            groups++;
            for (int w = 0; w < 4; w++) {
                int any = 0;
                for (uint32_t x = g; x < g + 64 && x < op; x++)
                    if (dist[x] > W[w]) {
                        far_b[w]++;
                        any = 1;
                    }
                far_g[w] += any;
            }
        }
    }
    printf("kind %d n %u: %.2f output bytes per token\n", kind, n, (double)bytes / toks);
    for (int w = 0; w < 4; w++)
        printf("window %5u: bytes reaching past it %.2f%%, 64-byte groups with one %.2f%%\n", W[w],
               100.0 * far_b[w] / bytes, 100.0 * far_g[w] / groups);
    return 0;
}

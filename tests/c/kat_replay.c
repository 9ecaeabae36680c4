/*
 * kat_replay.c -- a C99 caller of the drop-in, as Gibson's src/query.c:32
 * and src/net.c:36 are: it includes "lzf.h" (include/lzf.h), links
 * liblzf_hip.so and calls lzf_compress / lzf_decompress with host buffers.
 * TEST INFRASTRUCTURE (tests/test_dropin.py feeds it the known answers of
 * tests/golden/kat.json and decoder cases at the server's out_len).
 *
 * stdin, one case per line:
 *   C <in_hex|-> <out_len> <result> <out_hex|->
 *   D <in_hex|-> <out_len> <result> <errno> <out_hex|->
 * prints "ok N" or the first mismatch and exits 0 / 1.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lzf.h"

static size_t unhex(const char *h, unsigned char *out)
{
    size_t n = 0;
    if (!strcmp(h, "-")) return 0;
    while (h[0] && h[1]) {
        unsigned int b;
        if (sscanf(h, "%2x", &b) != 1) break;
        out[n++] = (unsigned char)b;
        h += 2;
    }
    return n;
}

int main(void)
{
    static char line[1 << 20], a[1 << 19], o[1 << 19];
    unsigned char *in = malloc(1 << 19), *want = malloc(1 << 19), *out;
    unsigned long cases = 0;
    char op;
    unsigned int out_len, result;
    int err;
    if (!in || !want) return 2;
    while (fgets(line, sizeof line, stdin)) {
        if (line[0] == 'C') {
            if (sscanf(line, "%c %s %u %u %s", &op, a, &out_len, &result, o) != 5) return 2;
        } else if (line[0] == 'D') {
            if (sscanf(line, "%c %s %u %u %d %s", &op, a, &out_len, &result, &err, o) != 6) return 2;
        } else {
            continue;
        }
        size_t n = unhex(a, in), wn = unhex(o, want);
        out = malloc(out_len + 16);
        if (!out) return 2;
        memset(out, 0, out_len + 16);
        if (op == 'C') {
            unsigned int r = lzf_compress(in, (unsigned int)n, out, out_len);
            if (r != result || (r && (r != wn || memcmp(out, want, r)))) {
                printf("compress mismatch at case %lu: got %u want %u\n", cases, r, result);
                return 1;
            }
        } else {
            errno = 0;
            unsigned int r = lzf_decompress(in, (unsigned int)n, out, out_len);
            int e = r ? 0 : errno;
            if (r != result || e != err || (r && (r != wn || memcmp(out, want, r)))) {
                printf("decompress mismatch at case %lu: got %u/%d want %u/%d\n", cases, r, e, result, err);
                return 1;
            }
        }
        free(out);
        cases++;
    }
    printf("ok %lu (LZF_VERSION 0x%04x)\n", cases, LZF_VERSION);
    return 0;
}

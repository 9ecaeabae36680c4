/*
 * cpu_bench.c -- CPU-baseline harness for bench.py (TEST INFRASTRUCTURE).
 *
 * Times the CPU LZF codec on a bounded sample of the bench workload:
 * the same synthetic values (gibson_amd/csrc/synth.h), compress with
 * out_len = n-4 (server policy, src/query.c:385), decompress the successes
 * with out_len = n.  One value per OpenMP thread, schedule(static),
 * 1 warm-up + median of `reps`.
 *
 * Built twice by oracle/Makefile:
 *   oracle/cpu_bench            -> times oracle_lzf_* (kind "port")
 *   oracle/_ref/cpu_bench_ref   -> times the compiled reference (kind "reference")
 *
 * usage: cpu_bench KIND N COUNT THREADS SEED REPS
 * prints one JSON object.
 */
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "synth.h"

unsigned int oracle_lzf_compress(const void *, unsigned int, void *, unsigned int);
unsigned int oracle_lzf_decompress(const void *, unsigned int, void *, unsigned int);
#ifdef USE_REF
unsigned int ref_lzf_compress(const void *, unsigned int, void *, unsigned int);
unsigned int ref_lzf_decompress(const void *, unsigned int, void *, unsigned int);
#define CODEC_C ref_lzf_compress
#define CODEC_D ref_lzf_decompress
#define KIND_NAME "reference"
#else
#define CODEC_C oracle_lzf_compress
#define CODEC_D oracle_lzf_decompress
#define KIND_NAME "port"
#endif

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static int cmp_d(const void *a, const void *b)
{
    double x = *(const double *)a, y = *(const double *)b;
    return (x > y) - (x < y);
}

int main(int argc, char **argv)
{
    if (argc < 7) {
        fprintf(stderr, "usage: %s KIND N COUNT THREADS SEED REPS\n", argv[0]);
        return 2;
    }
    int kind = atoi(argv[1]);
    uint32_t n = (uint32_t)strtoul(argv[2], 0, 0);
    uint32_t count = (uint32_t)strtoul(argv[3], 0, 0);
    int threads = atoi(argv[4]);
    uint64_t seed = strtoull(argv[5], 0, 0);
    int reps = atoi(argv[6]);
    if (reps < 1) reps = 1;
    if (reps > 31) reps = 31;
    omp_set_num_threads(threads);

    uint8_t *in = (uint8_t *)malloc((size_t)n * count);
    uint8_t *cmp = (uint8_t *)malloc((size_t)n * count + 8);
    uint8_t *dec = (uint8_t *)malloc((size_t)n * count);
    uint32_t *clen = (uint32_t *)calloc(count, sizeof(uint32_t));
    uint32_t *dlen = (uint32_t *)calloc(count, sizeof(uint32_t));
    if (!in || !cmp || !dec || !clen || !dlen) { fprintf(stderr, "oom\n"); return 1; }

#pragma omp parallel for schedule(static)
    for (uint32_t i = 0; i < count; i++)
        syn_generate(kind, seed, i, in + (size_t)i * n, n);

    double tc[32], td[32];
    for (int r = 0; r <= reps; r++) {          /* r == 0 is the warm-up */
        double t0 = now_s();
#pragma omp parallel for schedule(static)
        for (uint32_t i = 0; i < count; i++)
            clen[i] = CODEC_C(in + (size_t)i * n, n, cmp + (size_t)i * n, n - 4u);
        double t1 = now_s();
#pragma omp parallel for schedule(static)
        for (uint32_t i = 0; i < count; i++)
            dlen[i] = clen[i] ? CODEC_D(cmp + (size_t)i * n, clen[i], dec + (size_t)i * n, n) : 0u;
        double t2 = now_s();
        if (r) { tc[r - 1] = t1 - t0; td[r - 1] = t2 - t1; }
    }
    qsort(tc, (size_t)reps, sizeof(double), cmp_d);
    qsort(td, (size_t)reps, sizeof(double), cmp_d);

    uint64_t in_bytes = (uint64_t)n * count, comp_bytes = 0, ok = 0, bad = 0;
    for (uint32_t i = 0; i < count; i++) {
        if (clen[i]) {
            ok++;
            comp_bytes += clen[i];
            if (dlen[i] != n || memcmp(dec + (size_t)i * n, in + (size_t)i * n, n)) bad++;
        }
    }
    double c = tc[reps / 2], d = td[reps / 2];
    printf("{\"kind\": \"%s\", \"threads\": %d, \"n\": %u, \"count\": %u, "
           "\"in_bytes\": %llu, \"comp_bytes\": %llu, \"compressed\": %llu, \"roundtrip_bad\": %llu, "
           "\"compress_s\": %.6f, \"decompress_s\": %.6f, \"roundtrip_GBps\": %.4f, "
           "\"compress_GBps\": %.4f, \"decompress_GBps\": %.4f}\n",
           KIND_NAME, threads, n, count, (unsigned long long)in_bytes,
           (unsigned long long)comp_bytes, (unsigned long long)ok, (unsigned long long)bad,
           c, d, (double)in_bytes / (c + d) / 1e9, (double)in_bytes / c / 1e9,
           d > 0 ? (double)in_bytes / d / 1e9 : 0.0);
    return bad ? 1 : 0;
}

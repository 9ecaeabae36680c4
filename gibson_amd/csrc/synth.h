/*
 * synth.h -- deterministic synthetic value generators.
 *
 * One value = one block of n bytes, a pure function of (kind, seed, index, n):
 * per-block PRNG state = seed ^ index * 0x9E3779B97F4A7C15, stepped with
 * splitmix64.  The same source compiles for the device (hipcc: bench.py and
 * the GPU tests generate batches in HBM) and for the host (gcc: the CPU
 * baseline and the fixture tooling regenerate the identical bytes).
 *
 * Gibson has no corpus of its own; these stand in for the value sizes the
 * configs in BASELINE.json name.  Kinds:
 *   SYN_TEXT      Zipf-skewed words from a fixed 140-word vocabulary,
 *                 separated by ' ' (15/16) or '\n' (1/16)      configs 1, 4
 *   SYN_JSON      {"id":..,"user":"w_u16","score":a.bb,"tags":["w","w"],
 *                 "active":bool}, records, truncated to n        config 2
 *   SYN_SENTENCE  sentences drawn uniformly from a per-seed bank of
 *                 SYN_BANK sentences of 6-20 Zipf words          config 3
 *                 (SURVEY.md §8(d) names a bank of 64 and a measured
 *                 ratio of ~0.365; with this vocabulary a bank of 64
 *                 gives 0.218, so the bank size is the one that
 *                 reproduces the survey's ratio: 168 -> 0.363)
 *   SYN_MIXED     segments of U[256,2304) bytes: uniform random bytes, a
 *                 single-byte run, or Zipf text                 config 5
 *   SYN_RANDOM    uniform random bytes (incompressible edge case)
 *   SYN_SMALLALPHA bytes from a 2..5 letter alphabet (quirk-heavy edge case)
 */
#ifndef GIBSON_AMD_SYNTH_H
#define GIBSON_AMD_SYNTH_H

#include <stdint.h>

#ifdef __HIPCC__
#define SYN_TABLE static __device__ __constant__ const
#define SYN_FN static __device__ __forceinline__
#else
#define SYN_TABLE static const
#define SYN_FN static inline
#endif

enum {
    SYN_TEXT = 0,
    SYN_JSON = 1,
    SYN_SENTENCE = 2,
    SYN_MIXED = 3,
    SYN_RANDOM = 4,
    SYN_SMALLALPHA = 5,
    SYN_KINDS = 6
};

#define SYN_NWORDS 140
#define SYN_BANK 168u
#define SYN_ZIPF_TOTAL 5790626u
SYN_TABLE char syn_words[SYN_NWORDS][8] = {
    {'t','h','e'}, {'o','f'}, {'a','n','d'}, {'t','o'}, {'i','n'}, {'i','s'},
    {'y','o','u'}, {'t','h','a','t'}, {'i','t'}, {'h','e'}, {'w','a','s'}, {'f','o','r'},
    {'o','n'}, {'a','r','e'}, {'a','s'}, {'w','i','t','h'}, {'h','i','s'}, {'t','h','e','y'},
    {'a','t'}, {'b','e'}, {'t','h','i','s'}, {'h','a','v','e'}, {'f','r','o','m'}, {'o','r'},
    {'o','n','e'}, {'h','a','d'}, {'b','y'}, {'w','o','r','d'}, {'b','u','t'}, {'n','o','t'},
    {'w','h','a','t'}, {'a','l','l'}, {'w','e','r','e'}, {'w','e'}, {'w','h','e','n'}, {'y','o','u','r'},
    {'c','a','n'}, {'s','a','i','d'}, {'t','h','e','r','e'}, {'u','s','e'}, {'a','n'}, {'e','a','c','h'},
    {'w','h','i','c','h'}, {'s','h','e'}, {'d','o'}, {'h','o','w'}, {'t','h','e','i','r'}, {'i','f'},
    {'w','i','l','l'}, {'u','p'}, {'o','t','h','e','r'}, {'a','b','o','u','t'}, {'o','u','t'}, {'m','a','n','y'},
    {'t','h','e','n'}, {'t','h','e','m'}, {'t','h','e','s','e'}, {'s','o'}, {'s','o','m','e'}, {'h','e','r'},
    {'w','o','u','l','d'}, {'m','a','k','e'}, {'l','i','k','e'}, {'h','i','m'}, {'i','n','t','o'}, {'t','i','m','e'},
    {'h','a','s'}, {'l','o','o','k'}, {'t','w','o'}, {'m','o','r','e'}, {'w','r','i','t','e'}, {'g','o'},
    {'s','e','e'}, {'n','u','m','b','e','r'}, {'n','o'}, {'w','a','y'}, {'c','o','u','l','d'}, {'p','e','o','p','l','e'},
    {'m','y'}, {'t','h','a','n'}, {'f','i','r','s','t'}, {'w','a','t','e','r'}, {'b','e','e','n'}, {'c','a','l','l'},
    {'w','h','o'}, {'o','i','l'}, {'i','t','s'}, {'n','o','w'}, {'f','i','n','d'}, {'l','o','n','g'},
    {'d','o','w','n'}, {'d','a','y'}, {'d','i','d'}, {'g','e','t'}, {'c','o','m','e'}, {'m','a','d','e'},
    {'m','a','y'}, {'p','a','r','t'}, {'o','v','e','r'}, {'n','e','w'}, {'s','o','u','n','d'}, {'t','a','k','e'},
    {'o','n','l','y'}, {'l','i','t','t','l','e'}, {'w','o','r','k'}, {'k','n','o','w'}, {'p','l','a','c','e'}, {'y','e','a','r'},
    {'l','i','v','e'}, {'m','e'}, {'b','a','c','k'}, {'g','i','v','e'}, {'m','o','s','t'}, {'v','e','r','y'},
    {'a','f','t','e','r'}, {'t','h','i','n','g'}, {'o','u','r'}, {'j','u','s','t'}, {'n','a','m','e'}, {'g','o','o','d'},
    {'s','e','n','t','e','n','c','e'}, {'m','a','n'}, {'t','h','i','n','k'}, {'s','a','y'}, {'g','r','e','a','t'}, {'w','h','e','r','e'},
    {'h','e','l','p'}, {'t','h','r','o','u','g','h'}, {'m','u','c','h'}, {'b','e','f','o','r','e'}, {'l','i','n','e'}, {'r','i','g','h','t'},
    {'t','o','o'}, {'m','e','a','n'}, {'o','l','d'}, {'a','n','y'}, {'s','a','m','e'}, {'t','e','l','l'},
    {'b','o','y'}, {'f','o','l','l','o','w'},
};
SYN_TABLE unsigned char syn_wlen[SYN_NWORDS] = {
    3, 2, 3, 2, 2, 2, 3, 4, 2, 2, 3, 3, 2, 3, 2, 4, 3, 4, 2, 2,
    4, 4, 4, 2, 3, 3, 2, 4, 3, 3, 4, 3, 4, 2, 4, 4, 3, 4, 5, 3,
    2, 4, 5, 3, 2, 3, 5, 2, 4, 2, 5, 5, 3, 4, 4, 4, 5, 2, 4, 3,
    5, 4, 4, 3, 4, 4, 3, 4, 3, 4, 5, 2, 3, 6, 2, 3, 5, 6, 2, 4,
    5, 5, 4, 4, 3, 3, 3, 3, 4, 4, 4, 3, 3, 3, 4, 4, 3, 4, 4, 3,
    5, 4, 4, 6, 4, 4, 5, 4, 4, 2, 4, 4, 4, 4, 5, 5, 3, 4, 4, 4,
    8, 3, 5, 3, 5, 5, 4, 7, 4, 6, 4, 5, 3, 4, 3, 3, 4, 4, 3, 6,
};
SYN_TABLE unsigned int syn_zipf_cum[SYN_NWORDS] = {
    1048576u, 1572864u, 1922389u, 2184533u, 2394248u, 2569010u, 2718806u, 2849878u,
    2966386u, 3071243u, 3166568u, 3253949u, 3334608u, 3409506u, 3479411u, 3544947u,
    3606627u, 3664881u, 3720069u, 3772497u, 3822429u, 3870091u, 3915681u, 3959371u,
    4001314u, 4041643u, 4080479u, 4117928u, 4154085u, 4189037u, 4222862u, 4255630u,
    4287405u, 4318245u, 4348204u, 4377331u, 4405670u, 4433264u, 4460150u, 4486364u,
    4511939u, 4536905u, 4561290u, 4585121u, 4608422u, 4631217u, 4653527u, 4675372u,
    4696771u, 4717742u, 4738302u, 4758466u, 4778250u, 4797668u, 4816733u, 4835457u,
    4853853u, 4871931u, 4889703u, 4907179u, 4924368u, 4941280u, 4957924u, 4974308u,
    4990439u, 5006326u, 5021976u, 5037396u, 5052592u, 5067571u, 5082339u, 5096902u,
    5111266u, 5125435u, 5139416u, 5153213u, 5166830u, 5180273u, 5193546u, 5206653u,
    5219598u, 5232385u, 5245018u, 5257501u, 5269837u, 5282029u, 5294081u, 5305996u,
    5317777u, 5329427u, 5340949u, 5352346u, 5363621u, 5374776u, 5385813u, 5396735u,
    5407545u, 5418244u, 5428835u, 5439320u, 5449701u, 5459981u, 5470161u, 5480243u,
    5490229u, 5500121u, 5509920u, 5519629u, 5529248u, 5538780u, 5548226u, 5557588u,
    5566867u, 5576065u, 5585183u, 5594222u, 5603184u, 5612070u, 5620881u, 5629619u,
    5638284u, 5646878u, 5655403u, 5663859u, 5672247u, 5680569u, 5688825u, 5697017u,
    5705145u, 5713210u, 5721214u, 5729157u, 5737041u, 5744866u, 5752633u, 5760343u,
    5767996u, 5775594u, 5783137u, 5790626u,
};

#define SYN_GOLDEN 0x9E3779B97F4A7C15ull

SYN_FN uint64_t syn_next(uint64_t *s)
{
    uint64_t z = (*s += SYN_GOLDEN);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

typedef struct {
    uint8_t *out;
    uint32_t pos;
    uint32_t n;
} syn_writer;

SYN_FN int syn_full(const syn_writer *w) { return w->pos >= w->n; }

SYN_FN void syn_putc(syn_writer *w, uint8_t c)
{
    if (w->pos < w->n) w->out[w->pos] = c;
    w->pos++;
}

SYN_FN void syn_puts(syn_writer *w, const char *s)
{
    while (*s) syn_putc(w, (uint8_t)*s++);
}

SYN_FN void syn_putu(syn_writer *w, uint32_t v, int min_digits)
{
    char tmp[12];
    int k = 0;
    do { tmp[k++] = (char)('0' + v % 10u); v /= 10u; } while (v);
    while (k < min_digits) tmp[k++] = '0';
    while (k) syn_putc(w, (uint8_t)tmp[--k]);
}

SYN_FN uint32_t syn_zipf(uint64_t *s)
{
    uint32_t u = (uint32_t)((syn_next(s) >> 32) % SYN_ZIPF_TOTAL);
    uint32_t lo = 0, hi = SYN_NWORDS - 1;     /* first r with cum[r] > u */
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (syn_zipf_cum[mid] > u) hi = mid; else lo = mid + 1;
    }
    return lo;
}

SYN_FN void syn_word(syn_writer *w, uint32_t r, int capital)
{
    for (uint32_t k = 0; k < syn_wlen[r]; k++) {
        uint8_t c = (uint8_t)syn_words[r][k];
        if (capital && k == 0) c = (uint8_t)(c - 32);
        syn_putc(w, c);
    }
}

SYN_FN void syn_text(syn_writer *w, uint64_t *s, uint32_t limit)
{
    while (w->pos < limit) {
        syn_word(w, syn_zipf(s), 0);
        syn_putc(w, (syn_next(s) & 15u) == 0u ? '\n' : ' ');
    }
}

SYN_FN void syn_json(syn_writer *w, uint64_t *s)
{
    while (!syn_full(w)) {
        uint64_t a = syn_next(s), b = syn_next(s);
        syn_puts(w, "{\"id\":");
        syn_putu(w, (uint32_t)(a % 1000000u), 1);
        syn_puts(w, ",\"user\":\"");
        syn_word(w, syn_zipf(s), 0);
        syn_putc(w, '_');
        syn_putu(w, (uint32_t)(a >> 48), 1);
        syn_puts(w, "\",\"score\":");
        syn_putu(w, (uint32_t)(b % 100u), 1);
        syn_putc(w, '.');
        syn_putu(w, (uint32_t)((b >> 8) % 100u), 2);
        syn_puts(w, ",\"tags\":[\"");
        syn_word(w, syn_zipf(s), 0);
        syn_puts(w, "\",\"");
        syn_word(w, syn_zipf(s), 0);
        syn_puts(w, "\"],\"active\":");
        syn_puts(w, ((b >> 20) & 1u) ? "true" : "false");
        syn_puts(w, "},");
    }
}

/* sentence j of the bank belonging to `seed` */
SYN_FN void syn_sentence(syn_writer *w, uint64_t seed, uint32_t j)
{
    uint64_t s = seed ^ (0xD1B54A32D192ED03ull * (uint64_t)(j + 1u));
    uint32_t words = 6u + (uint32_t)(syn_next(&s) % 15u);
    for (uint32_t k = 0; k < words && !syn_full(w); k++) {
        syn_word(w, syn_zipf(&s), k == 0);
        syn_putc(w, k + 1u == words ? '.' : ' ');
    }
    syn_putc(w, ' ');
}

SYN_FN void syn_mixed(syn_writer *w, uint64_t *s)
{
    while (!syn_full(w)) {
        uint64_t a = syn_next(s);
        uint32_t len = 256u + (uint32_t)(a % 2048u);
        uint32_t end = w->pos + len;
        uint32_t type = (uint32_t)((a >> 32) % 3u);
        if (type == 0u) {
            while (w->pos < end) {
                uint64_t r = syn_next(s);
                for (int k = 0; k < 8 && w->pos < end; k++) syn_putc(w, (uint8_t)(r >> (8 * k)));
            }
        } else if (type == 1u) {
            uint8_t c = (uint8_t)(a >> 48);
            while (w->pos < end) syn_putc(w, c);
        } else {
            syn_text(w, s, end);
        }
    }
}

/* Fill out[0..n) with value `index` of generator `kind` under `seed`. */
SYN_FN void syn_generate(int kind, uint64_t seed, uint64_t index, uint8_t *out, uint32_t n)
{
    uint64_t s = seed ^ (index * SYN_GOLDEN);
    syn_writer w = { out, 0u, n };
    switch (kind) {
    case SYN_JSON:
        syn_json(&w, &s);
        break;
    case SYN_SENTENCE:
        while (!syn_full(&w)) syn_sentence(&w, seed, (uint32_t)(syn_next(&s) % SYN_BANK));
        break;
    case SYN_MIXED:
        syn_mixed(&w, &s);
        break;
    case SYN_RANDOM:
        while (!syn_full(&w)) {
            uint64_t r = syn_next(&s);
            for (int k = 0; k < 8; k++) syn_putc(&w, (uint8_t)(r >> (8 * k)));
        }
        break;
    case SYN_SMALLALPHA: {
        uint32_t alpha = 2u + (uint32_t)(syn_next(&s) % 4u);
        while (!syn_full(&w)) {
            uint64_t r = syn_next(&s);
            for (int k = 0; k < 8; k++) syn_putc(&w, (uint8_t)('a' + (uint32_t)((r >> (8 * k)) & 0xFFu) % alpha));
        }
        break;
    }
    case SYN_TEXT:
    default:
        syn_text(&w, &s, n);
        break;
    }
}

#endif /* GIBSON_AMD_SYNTH_H */

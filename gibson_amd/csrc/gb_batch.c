/*
 * gb_batch.c -- Gibson's SET/MSET/MGET codec call sites as device batches
 * (include/gb_batch.h).  Host C on top of lzf_host_compress_batch /
 * lzf_host_decompress_batch; the semantics follow src/query.c:374-425,
 * :479-502 and src/net.c:1256-1342.
 */
#include <stdlib.h>
#include <string.h>

#include "../../include/gb_batch.h"
#include "../../include/lzf_gpu.h"

/* src/query.c:400-405, applied once per value stored LZF, in request order */
static void gb_stats_add(gb_stats *s, uint32_t comprlen, uint32_t vlen)
{
    if (!s) return;
    const double rate = 100.0 - ((comprlen * 100.0) / vlen);
    if (s->compravg == 0)
        s->compravg = rate;
    else
        s->compravg = (s->compravg + rate) / 2.0;
    s->ncompressed++;
}

/* out_len of src/query.c:384-391: size_t needcompr = vlen - 4, passed as
 * unsigned int, so a value of fewer than 4 bytes gets a wrapped, huge cap.
 * No LZF stream of vlen bytes exceeds vlen + vlen/32 + 1 bytes, so a cap
 * past vlen + vlen/16 + 8 decides exactly like the wrapped one. */
static uint32_t gb_needcompr(uint32_t vlen)
{
    const uint32_t c = (uint32_t)(vlen - 4u), most = vlen + vlen / 16u + 8u;
    return c < most ? c : most;
}

int gb_set_batch(const uint8_t *v, const uint64_t *v_off, const uint32_t *v_len, uint32_t n,
                 uint32_t compression, uint8_t *out, const uint64_t *out_off, gb_stored *st,
                 gb_stats *stats)
{
    if (!n || !v || !v_off || !v_len || !out || !out_off || !st) return LZF_GPU_EARG;
    uint32_t m = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (!v_len[i]) return LZF_GPU_EARG;                  /* src/query.c:377 asserts vlen > 0 */
        if (v_len[i] > compression) m++;                      /* src/query.c:389 */
    }
    uint32_t *idx = NULL, *len = NULL, *cap = NULL, *res = NULL;
    uint64_t *ioff = NULL, *ooff = NULL;
    int rc = LZF_GPU_OK;
    if (m) {
        idx = malloc(m * sizeof *idx);
        len = malloc(m * sizeof *len);
        cap = malloc(m * sizeof *cap);
        res = malloc(m * sizeof *res);
        ioff = malloc(m * sizeof *ioff);
        ooff = malloc(m * sizeof *ooff);
        if (!idx || !len || !cap || !res || !ioff || !ooff) {
            rc = LZF_GPU_ENOMEM;
            goto done;
        }
        uint32_t k = 0;
        for (uint32_t i = 0; i < n; i++) {
            if (v_len[i] <= compression) continue;
            idx[k] = i;
            ioff[k] = v_off[i];
            len[k] = v_len[i];
            ooff[k] = out_off[i];
            cap[k] = gb_needcompr(v_len[i]);
            k++;
        }
        rc = lzf_host_compress_batch(v, ioff, len, out, ooff, cap, res, m);
        if (rc) goto done;
    }
    /* the stores, and the running mean, in request order */
    for (uint32_t i = 0, k = 0; i < n; i++) {
        st[i].orig_len = v_len[i];
        if (k < m && idx[k] == i) {
            if (res[k]) {
                st[i].encoding = GB_ENC_LZF;
                st[i].size = res[k];
                gb_stats_add(stats, res[k], v_len[i]);
            } else {
                st[i].encoding = GB_ENC_PLAIN;               /* not enough compression */
                st[i].size = v_len[i];
            }
            k++;
        } else {
            st[i].encoding = GB_ENC_PLAIN;
            st[i].size = v_len[i];
        }
    }
done:
    free(idx);
    free(len);
    free(cap);
    free(res);
    free(ioff);
    free(ooff);
    return rc;
}

int gb_mset(const uint8_t *v, uint32_t vlen, uint32_t nkeys, uint32_t compression, uint8_t *out,
            gb_stored *st, gb_stats *stats)
{
    if (!v || !vlen || !nkeys || !out || !st) return LZF_GPU_EARG;
    const uint64_t zero = 0;
    int rc = gb_set_batch(v, &zero, &vlen, 1, compression, out, &zero, st, NULL);
    if (rc) return rc;
    /* every matched key stores the same stream: the STATS mean moves once per
     * key (src/query.c:500 -> gbSingleSet per key) */
    if (st->encoding == GB_ENC_LZF)
        for (uint32_t k = 0; k < nkeys; k++) gb_stats_add(stats, st->size, vlen);
    return LZF_GPU_OK;
}

/* ---- MGET payload ---------------------------------------------------------- */

/* SAFE_MEMCPY / CHECK_SPACE of src/net.c:1270-1277 */
static int gb_put(uint8_t **p, uint64_t *space, const void *src, uint64_t n)
{
    if (n > *space) return -1;
    memcpy(*p, src, n);
    *p += n;
    *space -= n;
    return 0;
}

/* bytes of the decode arena of the calling thread's last gb_mget_payload */
static _Thread_local uint64_t g_mget_staged;
uint64_t gb_mget_last_staged(void) { return g_mget_staged; }

long gb_mget_payload(const uint8_t *keys, const uint64_t *key_off, const uint32_t *key_len,
                     const uint8_t *vals, const uint64_t *val_off, const uint32_t *val_size,
                     const uint8_t *enc, const uint32_t *orig_len, uint32_t count, uint32_t elements,
                     uint32_t maxrequestsize, uint64_t max_response, int reply_header, uint8_t *out)
{
    if (!out || (count && (!keys || !key_off || !key_len || !vals || !val_off || !val_size || !enc)))
        return LZF_GPU_EARG;
    g_mget_staged = 0;
    /* One decode batch for the LZF items, each into a slot of its decoded
     * size.  The reference decodes with out_len = maxrequestsize
     * (src/net.c:1309-1315): a side-table length caps at that, and an item
     * with no entry is sized first by the device pre-pass
     * (lzf_host_decoded_size_batch) at that out_len -- no slot of
     * maxrequestsize bytes per item. */
    uint32_t m = 0;
    for (uint32_t i = 0; i < count; i++)
        if (enc[i] == GB_ENC_LZF) m++;
    uint32_t *len = NULL, *cap = NULL, *dl = NULL, *ul = NULL, *us = NULL;
    int32_t *er = NULL;
    uint64_t *ioff = NULL, *ooff = NULL, *pos = NULL, *uo = NULL;
    uint8_t *dec = NULL, *exact = NULL;
    long ret = 0;
    if (m) {
        len = malloc(m * sizeof *len);
        cap = malloc(m * sizeof *cap);
        dl = malloc(m * sizeof *dl);
        er = malloc(m * sizeof *er);
        ioff = malloc(m * sizeof *ioff);
        ooff = malloc(m * sizeof *ooff);
        exact = malloc(m);
        pos = malloc(count * sizeof *pos);
        uo = malloc(m * sizeof *uo);
        ul = malloc(m * sizeof *ul);
        us = malloc(m * sizeof *us);
        if (!len || !cap || !dl || !er || !ioff || !ooff || !exact || !pos || !uo || !ul || !us) {
            ret = LZF_GPU_ENOMEM;
            goto done;
        }
        uint32_t nu = 0;
        for (uint32_t i = 0, k = 0; i < count; i++) {
            if (enc[i] != GB_ENC_LZF) continue;
            ioff[k] = val_off[i];
            len[k] = val_size[i];
            pos[i] = k;
            if (orig_len && orig_len[i]) {
                cap[k] = orig_len[i] < maxrequestsize ? orig_len[i] : maxrequestsize;
                exact[k] = 0;
            } else {
                uo[nu] = val_off[i];
                ul[nu] = val_size[i];
                nu++;
                cap[k] = 0;
                exact[k] = 1;
            }
            k++;
        }
        if (nu) {
            const int rc = lzf_host_decoded_size_batch(vals, uo, ul, us, er, nu, maxrequestsize);
            if (rc) {
                ret = rc;
                goto done;
            }
            for (uint32_t k = 0, u = 0; k < m; k++)
                if (exact[k]) cap[k] = us[u++];                   /* 0: the item does not decode */
        }
        /* when every size is exact, a payload past max_response fails the
         * reference's CHECK_SPACE (src/net.c:1272-1277) whatever the order:
         * nothing is decoded then */
        {
            uint64_t need = 4;
            int all_exact = 1;
            for (uint32_t i = 0; i < count; i++) {
                if (enc[i] == GB_ENC_NULL) continue;
                uint64_t v = val_size[i];
                if (enc[i] == GB_ENC_LZF) {
                    v = cap[pos[i]];
                    all_exact &= exact[pos[i]];
                }
                need += 4u + (uint64_t)key_len[i] + 1u + 4u + v;
            }
            if (all_exact && need > max_response) goto done;
        }
        uint64_t total = 0;
        for (uint32_t k = 0; k < m; k++) {
            ooff[k] = total;
            total += cap[k];
        }
        dec = malloc(total ? total : 1);
        if (!dec) {
            ret = LZF_GPU_ENOMEM;
            goto done;
        }
        g_mget_staged = total;
        for (uint32_t k = 0; k < m; k++) dl[k] = 0;
        /* an item of size 0 (does not decode) keeps cap 0: it fails again
         * in the batch, and the frame below stops there as the reference does */
        int rc = lzf_host_decompress_batch(vals, ioff, len, dec, ooff, cap, dl, er, m);
        if (rc) {
            ret = rc;
            goto done;
        }
        /* side-table lengths that were too small (stale): every such item is
         * sized by ONE pre-pass batch and decoded by ONE batch into slots
         * appended to the arena (uo / ul / us are free to reuse now; sk maps
         * them back to their items) */
        uint32_t ns = 0;
        for (uint32_t k = 0; k < m; k++)
            if (!dl[k] && !exact[k]) ns++;
        if (ns) {
            int32_t *se = malloc(ns * sizeof *se);
            uint64_t *so = malloc(ns * sizeof *so);
            uint32_t *sl = malloc(ns * sizeof *sl), *sk = malloc(ns * sizeof *sk);
            /* any failure here fails the call (ret), as the first pass does:
             * the reply is never built from a half-failed retry */
            int rc2 = se && so && sl && sk ? LZF_GPU_OK : LZF_GPU_ENOMEM;
            for (uint32_t k = 0, j = 0; rc2 == LZF_GPU_OK && k < m; k++) {
                if (dl[k] || exact[k]) continue;
                uo[j] = ioff[k];
                ul[j] = len[k];
                sk[j++] = k;
            }
            if (rc2 == LZF_GPU_OK) rc2 = lzf_host_decoded_size_batch(vals, uo, ul, us, se, ns, maxrequestsize);
            uint64_t add = 0;
            for (uint32_t j = 0; rc2 == LZF_GPU_OK && j < ns; j++) {
                so[j] = total + add;
                add += us[j];
            }
            if (rc2 == LZF_GPU_OK && add) {
                uint8_t *b = realloc(dec, total + add);
                if (!b) {
                    rc2 = LZF_GPU_ENOMEM;
                } else {
                    dec = b;
                    /* items that do not decode at all keep size 0 (us == 0) */
                    rc2 = lzf_host_decompress_batch(vals, uo, ul, dec, so, us, sl, se, ns);
                    if (rc2 == LZF_GPU_OK) {
                        for (uint32_t j = 0; j < ns; j++) {
                            if (!us[j] || !sl[j]) continue;
                            dl[sk[j]] = sl[j];
                            er[sk[j]] = 0;
                            ooff[sk[j]] = so[j];
                        }
                        total += add;
                        g_mget_staged = total;
                    }
                }
            }
            if (rc2 != LZF_GPU_OK) {
                free(se);
                free(so);
                free(sl);
                free(sk);
                ret = rc2;
                goto done;
            }
            free(se);
            free(so);
            free(sl);
            free(sk);
        }
    }
    {
        uint8_t *data = out + (reply_header ? 7 : 0), *p = data;
        uint64_t space = max_response;
        if (gb_put(&p, &space, &elements, 4)) goto done;             /* memrev32ifbe: LE host */
        for (uint32_t i = 0; i < count; i++) {
            if (enc[i] == GB_ENC_NULL) continue;                   /* src/net.c:1287 */
            uint32_t sz = key_len[i], vsize = val_size[i];
            uint8_t e = enc[i];
            const uint8_t *vp = vals + val_off[i];
            if (gb_put(&p, &space, &sz, 4) || gb_put(&p, &space, keys + key_off[i], sz)) goto done;
            if (e == GB_ENC_LZF) {                                 /* src/net.c:1306-1318 */
                const uint32_t k = (uint32_t)pos[i];
                /* an item that does not decode goes out with size 0: the
                 * release build (-DNDEBUG, CMakeLists.txt:20) compiles the
                 * assert of src/net.c:1331 out */
                e = GB_ENC_PLAIN;
                vsize = dl[k];
                vp = dl[k] ? dec + ooff[k] : vals;
            }
            if (gb_put(&p, &space, &e, 1) || gb_put(&p, &space, &vsize, 4) || gb_put(&p, &space, vp, vsize))
                goto done;
        }
        ret = (long)(p - data);
        if (reply_header) {                                        /* src/net.c:1162-1205 */
            const int16_t code = 7;                                /* REPL_KVAL, src/query.h:71 */
            const uint8_t pe = GB_ENC_PLAIN;
            const uint32_t size = (uint32_t)ret;
            memcpy(out, &code, 2);
            memcpy(out + 2, &pe, 1);
            memcpy(out + 3, &size, 4);
            ret += 7;
        }
    }
done:
    free(len);
    free(cap);
    free(dl);
    free(er);
    free(ioff);
    free(ooff);
    free(exact);
    free(pos);
    free(uo);
    free(ul);
    free(us);
    free(dec);
    return ret;
}

/* ---- the original-length side table ---------------------------------------- */

struct gb_lentab {
    uint64_t *key;
    uint32_t *val;
    uint8_t *state;            /* 0 empty, 1 used, 2 deleted */
    size_t cap, used, filled;  /* filled = used + deleted */
};

static size_t gb_hash(uint64_t k, size_t mask)
{
    k ^= k >> 33;
    k *= 0xff51afd7ed558ccdull;
    k ^= k >> 33;
    return (size_t)k & mask;
}

static int gb_lentab_grow(gb_lentab *t, size_t ncap)
{
    uint64_t *key = calloc(ncap, sizeof *key);
    uint32_t *val = calloc(ncap, sizeof *val);
    uint8_t *state = calloc(ncap, 1);
    if (!key || !val || !state) {
        free(key);
        free(val);
        free(state);
        return LZF_GPU_ENOMEM;
    }
    for (size_t i = 0; i < t->cap; i++) {
        if (t->state[i] != 1) continue;
        size_t h = gb_hash(t->key[i], ncap - 1);
        while (state[h]) h = (h + 1) & (ncap - 1);
        key[h] = t->key[i];
        val[h] = t->val[i];
        state[h] = 1;
    }
    free(t->key);
    free(t->val);
    free(t->state);
    t->key = key;
    t->val = val;
    t->state = state;
    t->cap = ncap;
    t->filled = t->used;
    return 0;
}

gb_lentab *gb_lentab_new(void)
{
    gb_lentab *t = calloc(1, sizeof *t);
    if (!t) return NULL;
    if (gb_lentab_grow(t, 64)) {
        free(t);
        return NULL;
    }
    return t;
}

void gb_lentab_free(gb_lentab *t)
{
    if (!t) return;
    free(t->key);
    free(t->val);
    free(t->state);
    free(t);
}

static size_t gb_find(const gb_lentab *t, uint64_t item, int *found)
{
    size_t h = gb_hash(item, t->cap - 1), tomb = (size_t)-1;
    for (;;) {
        if (t->state[h] == 0) {
            *found = 0;
            return tomb != (size_t)-1 ? tomb : h;
        }
        if (t->state[h] == 1 && t->key[h] == item) {
            *found = 1;
            return h;
        }
        if (t->state[h] == 2 && tomb == (size_t)-1) tomb = h;
        h = (h + 1) & (t->cap - 1);
    }
}

int gb_lentab_put(gb_lentab *t, uint64_t item, uint32_t orig_len)
{
    if (!t) return LZF_GPU_EARG;
    if ((t->filled + 1) * 2 > t->cap && gb_lentab_grow(t, t->used * 4 > t->cap ? t->cap * 2 : t->cap))
        return LZF_GPU_ENOMEM;
    int found;
    const size_t h = gb_find(t, item, &found);
    if (!found) {
        if (t->state[h] == 0) t->filled++;
        t->state[h] = 1;
        t->key[h] = item;
        t->used++;
    }
    t->val[h] = orig_len;
    return 0;
}

int gb_lentab_get(const gb_lentab *t, uint64_t item, uint32_t *orig_len)
{
    if (!t) return 0;
    int found;
    const size_t h = gb_find(t, item, &found);
    if (found && orig_len) *orig_len = t->val[h];
    return found;
}

int gb_lentab_del(gb_lentab *t, uint64_t item)
{
    if (!t) return 0;
    int found;
    const size_t h = gb_find(t, item, &found);
    if (!found) return 0;
    t->state[h] = 2;
    t->used--;
    return 1;
}

size_t gb_lentab_size(const gb_lentab *t) { return t ? t->used : 0; }

/*
 * gb_batch.h -- Gibson's LZF call sites, batched (SURVEY.md §8(f) ranks 1
 * and 3), on top of the host-memory batch API of liblzf_hip.so.
 *
 * The reference calls the codec once per key: SET and every key an MSET
 * matches go through gbSingleSet (src/query.c:374-425, MSET via
 * gbMultiSetCallback src/query.c:479-502), and the MGET reply decodes its
 * LZF items one by one into lzf_buffer (src/net.c:1256-1342).  These helpers
 * keep the reference's semantics -- which values are compressed, what is
 * stored, the STATS running mean in request order, the reply payload byte
 * for byte -- while the codec work of a whole request is one device batch:
 *
 *   gb_set_batch        the store decision of gbSingleSet for N values, one
 *                       lzf_host_compress_batch for every value above the
 *                       compression threshold;
 *   gb_mset             one value under K keys: compressed ONCE (the stream
 *                       is a pure function of (bytes, length, out_len),
 *                       SURVEY.md §8(a) a8), the STATS update applied K
 *                       times, as K gbSingleSet calls would;
 *   gb_mget_payload     the MGET/KEYS payload of gbClientEnqueueKeyValueSet
 *                       with every LZF item decoded by one
 *                       lzf_host_decompress_batch, in request order;
 *   gb_lentab_*         the original-length side table: the reference keeps
 *                       only the compressed size (item->size, src/query.c:408;
 *                       META size returns it, src/query.c:1263-1266), so a
 *                       decoder must assume maxrequestsize.  The table maps
 *                       an item (any stable 64-bit key, e.g. its data
 *                       pointer) to its original length, so decode batches
 *                       are sized exactly and lzf_gpu_kv_frame gets val_len.
 *
 * Encodings and reply codes are the reference's (src/net.h:274-278,
 * src/query.h:71).  All pointers are host memory.  Return values: 0 (or a
 * length where stated) or a negative LZF_GPU_E* code of lzf_gpu.h.
 */
#ifndef GB_BATCH_H
#define GB_BATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GB_ENC_PLAIN  0x00   /* src/net.h:274 */
#define GB_ENC_LZF    0x01   /* src/net.h:276 */
#define GB_ENC_NUMBER 0x02   /* src/net.h:278 */
#define GB_ENC_NULL   0xFF   /* an expired / missing MGET item: skipped (src/net.c:1287) */

/* the STATS fields the store path maintains (src/query.c:400-405) */
typedef struct {
    double compravg;          /* server->stats.compravg */
    uint64_t ncompressed;     /* values stored GB_ENC_LZF by these helpers */
} gb_stats;

/* what gbSingleSet stores for one value */
typedef struct {
    uint8_t encoding;         /* GB_ENC_PLAIN or GB_ENC_LZF */
    uint32_t size;            /* item->size: the stream length for LZF, vlen for plain */
    uint32_t orig_len;        /* vlen (the side table's entry) */
} gb_stored;

/*
 * Store decision of gbSingleSet for values i = 0..n-1 (v + v_off[i], v_len[i]
 * bytes, v_len[i] > 0), in request order:
 *   v_len[i] > compression  -> lzf_compress(v, vlen, out, vlen - 4);
 *                              0 -> stored plain, else stored LZF with the
 *                              stream at out + out_off[i] (room for vlen-4
 *                              bytes; 8 for a value shorter than 8: the
 *                              reference's size_t vlen - 4 wraps there);
 *   otherwise               -> stored plain.
 * stats (optional) gets the reference's running mean per LZF value, in
 * request order.  st[i] receives the decision.
 */
int gb_set_batch(const uint8_t *v, const uint64_t *v_off, const uint32_t *v_len, uint32_t n,
                 uint32_t compression, uint8_t *out, const uint64_t *out_off, gb_stored *st,
                 gb_stats *stats);

/*
 * MSET: one value under nkeys keys.  Compressed once; *st describes what
 * every key stores (the same stream, at out, room vlen - 4); stats updated as
 * nkeys consecutive gbSingleSet calls would.
 */
int gb_mset(const uint8_t *v, uint32_t vlen, uint32_t nkeys, uint32_t compression, uint8_t *out,
            gb_stored *st, gb_stats *stats);

/*
 * MGET / KEYS payload (src/net.c:1256-1342): u32 elements, then per item
 * whose enc is not GB_ENC_NULL: [u32 key size][key][u8 encoding][u32 value
 * size][value], LZF items as GB_ENC_PLAIN with their decoded bytes; with
 * reply_header != 0 the [i16 REPL_KVAL][u8 GB_ENC_PLAIN][u32 size] header of
 * gbClientEnqueueData (src/net.c:1162-1205) in front.  Item i: key
 * keys + key_off[i] (key_len[i] bytes), stored bytes vals + val_off[i]
 * (val_size[i] bytes; for an LZF item the stream), enc[i]; orig_len (may be
 * NULL) gives an LZF item's decoded length (0 = unknown: sized by the
 * device pre-pass at out_len = maxrequestsize, as src/net.c:1309-1315, then
 * decoded into a slot of that size).  out holds
 * (reply_header ? 7 : 0) + max_response bytes.
 * An LZF item that does not decode at maxrequestsize goes out as PLAIN with
 * size 0, as the release build does (its assert, src/net.c:1331, is compiled
 * out by -DNDEBUG, CMakeLists.txt:20).  Returns the frame length, 0 when the
 * payload exceeds max_response (the reference's CHECK_SPACE,
 * src/net.c:1272-1277), or a negative error.
 */
long gb_mget_payload(const uint8_t *keys, const uint64_t *key_off, const uint32_t *key_len,
                     const uint8_t *vals, const uint64_t *val_off, const uint32_t *val_size,
                     const uint8_t *enc, const uint32_t *orig_len, uint32_t count, uint32_t elements,
                     uint32_t maxrequestsize, uint64_t max_response, int reply_header, uint8_t *out);
/* bytes of decode arena the calling thread's last gb_mget_payload staged:
 * the LZF items' decoded sizes (side table, capped at maxrequestsize, or the
 * device pre-pass lzf_host_decoded_size_batch), never maxrequestsize per
 * item; 0 when the payload was known to exceed max_response up front */
uint64_t gb_mget_last_staged(void);

/* the original-length side table (open addressing, grows; not thread-safe,
 * like the reference's single-threaded store) */
typedef struct gb_lentab gb_lentab;
gb_lentab *gb_lentab_new(void);
void gb_lentab_free(gb_lentab *t);
int gb_lentab_put(gb_lentab *t, uint64_t item, uint32_t orig_len);   /* 0 or LZF_GPU_ENOMEM */
int gb_lentab_get(const gb_lentab *t, uint64_t item, uint32_t *orig_len);   /* 1 found, 0 not */
int gb_lentab_del(gb_lentab *t, uint64_t item);                       /* 1 removed, 0 not */
size_t gb_lentab_size(const gb_lentab *t);

#ifdef __cplusplus
}
#endif

#endif /* GB_BATCH_H */

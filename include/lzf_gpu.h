/*
 * lzf_gpu.h -- batched, device-resident LZF API of liblzf_hip.so.
 *
 * The reference has no batch entry point: it calls lzf_compress once per
 * SET/MSET key (src/query.c:391, reached from src/query.c:453 and :500) and
 * lzf_decompress once per GET/MGET item (src/net.c:1229, src/net.c:1309).
 * These calls take a whole batch of independent values at once; each value
 * gets exactly the single-call semantics of src/lzf_c.c / src/lzf_d.c
 * (results bit-identical to the reference, per-value return value and
 * errno), so the single-call drop-in in lzf.h is a batch of one.
 *
 * Layout: values are addressed by (offset, length) pairs into one byte
 * arena per direction.  Every pointer passed to lzf_gpu_* is DEVICE memory
 * (hipMalloc'd, or torch CUDA tensors); `stream` is a hipStream_t (NULL =
 * the legacy default stream).  Calls are asynchronous on `stream`.
 *
 * Return value of every call: LZF_GPU_OK or a negative LZF_GPU_E* code
 * (the launch was not made).  Failures are returned, never aborted on.
 *
 * Bounds: a value longer than max_in_len (compress) or with an out_cap past
 * max_out_cap (decompress) -- a caller that under-states the bound -- gets
 * out_len 0 (and err EINVAL on decompress); nothing outside its own output
 * range is written.
 */
#ifndef LZF_GPU_H
#define LZF_GPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LZF_GPU_OK          0
#define LZF_GPU_EARG       -1   /* bad argument (NULL pointer, count 0 ...) */
#define LZF_GPU_ELAUNCH    -2   /* HIP launch / copy failed */
#define LZF_GPU_ENODEV     -3   /* no usable gfx950 device */
#define LZF_GPU_ENOMEM     -4   /* device / pinned allocation failed */

/* Largest value the batch kernels take in one piece (bytes).  Gibson's
 * default max_value_size is far below it (src/default.h:52) and the shipped
 * config's 2 MiB (debian/etc/gibson/gibson.conf:33) too. */
#define LZF_GPU_MAX_VALUE  (64u << 20)

/*
 * Compress `count` values.  Value i is in[in_off[i] .. +in_len[i]); its
 * stream is written to out[out_off[i] .. +out_cap[i]) and its length to
 * out_len[i] (0 = does not fit, exactly when src/lzf_c.c returns 0; the
 * bytes at out then are unspecified, and nothing is ever written at or past
 * out_cap[i]).  max_in_len is an upper bound on every in_len[i] (selects the
 * kernel's LDS plan without reading device memory); max_in_len 0 declares an
 * all-empty batch (every out_len 0, src/lzf_c.c:131).
 * The server policy of src/query.c:385 is out_cap[i] = in_len[i] - 4.
 */
int lzf_gpu_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                           uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                           uint32_t *out_len, uint32_t count, uint32_t max_in_len,
                           void *stream);

/*
 * Decompress `count` streams.  Stream i is in[in_off[i] .. +in_len[i]);
 * the decoded bytes go to out[out_off[i] .. +out_cap[i]); out_len[i] gets
 * the decoded length or 0, err[i] gets 0, E2BIG or EINVAL exactly as the
 * reference sets errno (src/lzf_d.c:72-131).  As in the reference, a stream
 * with in_len 0 still reads its first control byte, so in[in_off[i]] must be
 * readable.  max_out_cap bounds every out_cap[i].
 */
int lzf_gpu_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                             uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                             uint32_t *out_len, int32_t *err, uint32_t count,
                             uint32_t max_out_cap, void *stream);

/*
 * Decoded-size pre-pass: out_size[i] gets the length lzf_decompress would
 * return for stream i with out_len = out_limit (0 on failure) and err[i]
 * its errno (0, E2BIG or EINVAL in the reference's check order,
 * src/lzf_d.c:64-146); nothing is decoded.  For MGET items without an
 * original-length side-table entry: size them at out_limit = maxrequestsize
 * (src/net.c:1309-1315), then decode into exact slots (gb_mget_payload, or
 * val_len for lzf_gpu_kv_frame).  As for decompress, in[in_off[i]] must be
 * readable even when in_len[i] is 0.
 */
int lzf_gpu_decoded_size_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                               uint32_t *out_size, int32_t *err, uint32_t count, uint32_t out_limit,
                               void *stream);
int lzf_host_decoded_size_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                                uint32_t *out_size, int32_t *err, uint32_t count, uint32_t out_limit);

/*
 * Fill `count` values of n bytes each, value k at out[k*n], with synthetic
 * generator `kind` (gibson_amd/csrc/synth.h) at indices first + k*stride.
 * Bench/test data generation directly in HBM.
 */
int lzf_gpu_synth_fill(int kind, uint64_t seed, uint64_t first, uint64_t stride,
                       uint32_t count, uint32_t n, uint8_t *out, void *stream);

/*
 * Host-memory batch (the north star's PCIe-inclusive path): the same as the
 * device calls, but every pointer is host memory, and the call returns after
 * the results are back in host memory.
 *
 * Devices: with LZF_GPU_DEVICES set ("0,1,2,3", "all"; an index may repeat),
 * value i goes to entry i mod G of that list, each entry served by its own
 * worker thread (bound to its device's NUMA node), streams and staging; the
 * results land at index i.  A failure on any entry makes the call return
 * that entry's LZF_GPU_E* code.  Unset: the one device LZF_GPU_DEVICE
 * (default 0), on the calling thread.
 *
 * Moving bytes: when both arenas' spans lie in ranges given to
 * lzf_host_register, no CPU copies a value byte (the GPU and its DMA engines
 * move them; the bytes of an output slot past out_len[i] are then either
 * left as they were or zeroed -- never bytes of another value).  Otherwise
 * the library stages values through its own pinned buffers.  Results are
 * identical either way.
 *
 * LZF_GPU_SPLIT=block gives entry g a contiguous span of the values instead
 * of every G-th one (lzf_host_split_block below).
 */
int lzf_host_compress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                            uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                            uint32_t *out_len, uint32_t count);
int lzf_host_decompress_batch(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len,
                              uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                              uint32_t *out_len, int32_t *err, uint32_t count);

/*
 * Register [ptr, ptr+len) of caller memory (an arena of request buffers, the
 * store's values) for the host-memory batches: page-locked and mapped into
 * every device of the plan (hipHostRegister, portable + mapped).  The range
 * must stay allocated until lzf_host_unregister(ptr).  Returns LZF_GPU_OK,
 * LZF_GPU_EARG (NULL, empty, or overlapping a registered range) or the HIP
 * failure's code.  Registration costs about 15 ms per GiB (measured).
 */
int lzf_host_register(const void *ptr, uint64_t len);
/* (LZF_GPU_ENODEV: some device of the plan gave no device address for the
 * range; it is then left unregistered.) */
int lzf_host_unregister(const void *ptr);

/*
 * The device plan of the host-memory calls: returns G, the number of
 * entries, and fills (for k < max) device[k] (HIP device index),
 * numa_node[k] (the device's node from sysfs, -1 unknown) and bound[k]
 * (1 when entry k's worker thread runs on that node's CPUs with its memory
 * preferred there).  A negative LZF_GPU_E* code when the plan is invalid.
 */
int lzf_gpu_device_plan(int *device, int *numa_node, int *bound, int max);
/* The calling thread's last host-memory call: values each plan entry took
 * and its wall time in ms (the per-device spread).  Returns G. */
int lzf_host_last_spread(uint32_t *values, double *ms, int max);
/* The partition rule: entry g of `groups` takes values first + k * stride,
 * k < the returned count (first = g, stride = groups): value i to entry
 * i mod G, the default. */
uint32_t lzf_host_split(uint32_t count, uint32_t groups, uint32_t g, uint32_t *first, uint32_t *stride);
/* The contiguous split (LZF_GPU_SPLIT=block): entry g takes the values
 * [first, first + returned count), first = floor(count * g / groups), so
 * every entry's share is one span of the caller's arena and its values keep
 * the registered path's DMA runs. */
uint32_t lzf_host_split_block(uint32_t count, uint32_t groups, uint32_t g, uint32_t *first);
/* The split the host-memory calls use: 0 round-robin (default), 1 block. */
int lzf_host_split_policy(void);
/* The LZF_GPU_DEVICES grammar ("all", or comma-separated indices below
 * `visible`): fills dev[] and returns the count, or a negative code. */
int lzf_gpu_parse_device_list(const char *spec, int visible, int *dev, int max);

/*
 * MGET / KEYS reply assembled on the device.
 *
 * Builds exactly the payload of gbClientEnqueueKeyValueSet
 * (src/net.c:1256-1342) -- u32 `elements`, then per item that is not
 * LZF_ENC_NULL: [u32 key size][key][u8 encoding][u32 value size][value],
 * little-endian, LZF items emitted as PLAIN with their decoded bytes -- and,
 * with reply_header != 0, the [i16 REPL_KVAL][u8 PLAIN][u32 size] reply
 * header of gbClientEnqueueData (src/net.c:1162-1205) in front.
 *
 * Item i: key keys[key_off[i] .. +key_len[i]); encoding enc[i]; stored
 * bytes vals[val_off[i] .. +val_size[i]) (the LZF stream for an LZF item,
 * the 8-byte little-endian number for a NUMBER item, src/net.c:1321-1329).
 * val_len[i] is the decoded length of an LZF item -- the original length
 * recorded at SET time (the side table of §8(f) rank 3); max_val_len bounds
 * it.  LZF items are decoded straight into the frame (no bounce buffer).
 *
 * frame must hold (reply_header ? 7 : 0) + max_response bytes.  On the
 * device, *frame_len receives the frame's byte count, or 0 when the payload
 * exceeds max_response (the reference's CHECK_SPACE, src/net.c:1272-1277)
 * or an LZF item did not decode to val_len[i].  `work` is device scratch of
 * lzf_gpu_kv_frame_work_size(count) bytes.
 */
#define LZF_ENC_PLAIN   0x00   /* GB_ENC_PLAIN,  src/net.h:274 */
#define LZF_ENC_LZF     0x01   /* GB_ENC_LZF,    src/net.h:276 */
#define LZF_ENC_NUMBER  0x02   /* GB_ENC_NUMBER, src/net.h:278 */
#define LZF_ENC_NULL    0xFF   /* expired / missing item: skipped (src/net.c:1287) */
#define LZF_REPL_KVAL   7      /* src/query.h:71 */

uint64_t lzf_gpu_kv_frame_work_size(uint32_t count);
int lzf_gpu_kv_frame(const uint8_t *keys, const uint64_t *key_off, const uint32_t *key_len,
                     const uint8_t *vals, const uint64_t *val_off, const uint32_t *val_size,
                     const uint8_t *enc, const uint32_t *val_len, uint32_t count,
                     uint32_t elements, uint32_t max_val_len, int reply_header,
                     uint8_t *frame, uint64_t max_response, uint64_t *frame_len, void *work,
                     void *stream);

/* Free the library's device scratch (all devices), the calling thread's and
 * the device workers' staging buffers; later calls allocate them again.
 * Each thread's staging buffers are also freed when the thread exits. */
void lzf_gpu_release(void);

/* One-time self-check of the current device (run lazily before the first
 * compress launch, or here): the table / lane / window compressor kernels
 * need the LDS to execute a wave's same-address ds_mskor_rtn_b32 in lane
 * order (gibson_amd/csrc/lzf_selfcheck.hip).  Returns 1 when that held (the
 * measured routing is used), 0 when it did not (compress batches then run
 * window64, which needs no ordering), or a negative LZF_GPU_E* code.  The
 * result also appears in lzf_gpu_kernel_info() as lds_order=... */
int lzf_gpu_selfcheck(void);
/* The probe itself, run again: mismatching lanes over 16 collision patterns
 * of 1024 waves (0 = lane order held), or a negative LZF_GPU_E* code. */
int lzf_gpu_lds_order_probe(void);

/* Which kernel generation the batch calls dispatch to (diagnostics):
 * returns a static string such as "compress=window64 decompress=tokpar". */
const char *lzf_gpu_kernel_info(void);

#ifdef __cplusplus
}
#endif

#endif /* LZF_GPU_H */

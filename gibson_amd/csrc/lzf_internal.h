/*
 * lzf_internal.h -- shared definitions between the HIP kernels and the
 * C-ABI layer (lzf_api.cpp).  Not installed; the public boundary is
 * include/lzf.h and include/lzf_gpu.h.
 */
#ifndef GIBSON_AMD_LZF_INTERNAL_H
#define GIBSON_AMD_LZF_INTERNAL_H

#include <hip/hip_runtime.h>
#include <stdint.h>

/* LZF format constants (reference src/lzf_c.c:74-76, src/lzfP.h:55) */
#define LZF_MAX_LIT   32u
#define LZF_WINDOW    8192u
#define LZF_MAX_REF   264u
#define LZF_SLOTS     65536u

/* one batch, device pointers */
struct LzfBatch {
    const uint8_t *in;
    const uint64_t *in_off;
    const uint32_t *in_len;
    uint8_t *out;
    const uint64_t *out_off;
    const uint32_t *out_cap;
    uint32_t *out_len;
    int32_t *err;          /* decompress only */
    uint32_t count;
    uint32_t max_len;      /* max in_len (compress) / max out_cap (decompress) */
    const uint8_t *skip;   /* decompress: values with skip[i] != 0 are left alone (NULL: none) */
};

/* the MGET reply frame (lzf_frame.hip); device pointers */
struct LzfFrameArgs {
    const uint8_t *keys;
    const uint64_t *key_off;
    const uint32_t *key_len;
    const uint8_t *vals;
    const uint64_t *val_off;
    const uint32_t *val_size;
    const uint8_t *enc;
    const uint32_t *val_len;
    uint32_t count, elements;
    uint32_t max_val_len;
    int reply_header;
    uint64_t max_response;
    uint8_t *frame;
    uint64_t *frame_len;
    /* work area (lzf_frame_carve) */
    uint64_t *w_off, *w_voff, *w_bsum, *w_state;
    uint32_t *w_len;
    int32_t *w_err;
    uint8_t *w_skip;
};

/* compress scratch of the lane generation (lzf_lane.hip), device pointers:
 * per value cstride u16 cand words and bstride u32 inserted-bitmap words */
struct LzfLaneScratch {
    uint16_t *cand;
    uint32_t *bits;
    uint64_t cstride;
    uint64_t bstride;
    uint32_t force_fix;    /* diagnostics: take the atomic-order repair path */
};

/* compress scratch of the table generation (lzf_cand.hip), device pointers:
 * per value rstride u32 records and bstride u32 inserted-bitmap words */
struct LzfRecScratch {
    uint32_t *rec;
    uint32_t *bits;
    uint64_t rstride;
    uint64_t bstride;
};

/* a batch whose inputs arrive in parts (the registered host path): part p is
 * values [end[p-1], end[p]) (end[-1] = 0), in once ev[p] has fired on its
 * stream; kernel 1 of a part may start then, the parse after all of them */
struct LzfParts {
    uint32_t n;
    const uint32_t *end;
    const hipEvent_t *ev;
};

/* launchers, defined next to their kernels; return hipSuccess or the error */
hipError_t lzf_launch_compress_table(const LzfBatch &b, hipStream_t s, void *scratch, size_t scratch_bytes,
                                     uint32_t *chunks, const LzfParts *parts = nullptr);
size_t lzf_table_scratch_per_value(uint32_t max_len);
bool lzf_table_compress_supported(uint32_t max_len);
hipError_t lzf_launch_compress_wtab(const LzfBatch &b, hipStream_t s, void *scratch, size_t scratch_bytes,
                                    uint32_t *chunks);
size_t lzf_wtab_scratch_per_value(uint32_t max_len);
bool lzf_wtab_compress_supported(uint32_t max_len);
hipError_t lzf_launch_decompress_lane(const LzfBatch &b, hipStream_t s);
hipError_t lzf_launch_dsize(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint32_t *out_size,
                            int32_t *err, uint32_t count, uint32_t limit, hipStream_t s);
/* aux / ev (4 events) optional: chunks pipelined over s (kernel 1) and aux
 * (kernel 2); s is joined with aux before returning */
hipError_t lzf_launch_compress_lane(const LzfBatch &b, hipStream_t s, void *scratch,
                                    size_t scratch_bytes, uint32_t force_fix, hipStream_t aux,
                                    hipEvent_t *ev, uint32_t *chunks);
size_t lzf_lane_scratch_per_value(uint32_t max_len);
hipError_t lzf_launch_cand_stream(const LzfBatch &b, const LzfLaneScratch &sc, hipStream_t s);
hipError_t lzf_launch_cand_stream_rec(const LzfBatch &b, const LzfRecScratch &sc, hipStream_t s);
const char *lzf_lane_cand_name(void);
bool lzf_lane_compress_supported(uint32_t max_len);
hipError_t lzf_launch_compress(const LzfBatch &b, hipStream_t s);
hipError_t lzf_launch_decompress(const LzfBatch &b, hipStream_t s);
hipError_t lzf_launch_synth(int kind, uint64_t seed, uint64_t first, uint64_t stride,
                            uint32_t count, uint32_t n, uint8_t *out, hipStream_t s);
hipError_t lzf_launch_frame(LzfFrameArgs &a, hipStream_t s,
                            hipError_t (*decode)(const LzfBatch &, hipStream_t));
size_t lzf_frame_work_bytes(uint32_t count);
void lzf_frame_carve(LzfFrameArgs &a, void *work);
const char *lzf_compress_kernel_name(void);
/* value moves between mapped host memory and device arenas (lzf_hostio.hip):
 * len[k] (at least min_len) bytes from src + src_off[k] to dst + dst_off[k] */
hipError_t lzf_launch_move(const uint8_t *src, const uint64_t *src_off, uint8_t *dst, const uint64_t *dst_off,
                           const uint32_t *len, uint32_t min_len, uint32_t count, hipStream_t s);
/* zero bytes [len[k], cap[k]) of every value's slot at dst + dst_off[k] (the
 * bytes past a decoded value that a DMA of abutting slots would carry) */
hipError_t lzf_launch_clear_tail(uint8_t *dst, const uint64_t *dst_off, const uint32_t *len, const uint32_t *cap,
                                 uint32_t count, hipStream_t s);
/* lzf_api.cpp, for the host-memory paths of lzf_host.cpp: the routed
 * launches, the routing's batch threshold, the device check, the scratch */
hipError_t lzf_route_compress(const LzfBatch &b, hipStream_t s);
hipError_t lzf_route_decompress(const LzfBatch &b, hipStream_t s);
uint32_t lzf_route_min_count(uint32_t max_len);
bool lzf_device_ok(int dev);
void lzf_scratch_release_all(void);
/* compress with the routed generations whatever the batch size, on a private
 * scratch (lzf_scratch_create): the host pipeline's side-by-side chunks */
hipError_t lzf_route_compress_bulk(const LzfBatch &b, hipStream_t s, void *scratch,
                                   const LzfParts *parts = nullptr);
/* window64 (one wave per value), and whether the default routing is in
 * force (no LZF_GPU_KERNEL override, the LDS lane order held) */
hipError_t lzf_route_compress_window(const LzfBatch &b, hipStream_t s);
bool lzf_route_default(void);
/* a private scratch holding 1/share of the cap (the host pipeline's slots) */
void *lzf_scratch_create(unsigned share);
void lzf_scratch_release(void *scratch);
void lzf_scratch_destroy(void *scratch);
const char *lzf_decompress_kernel_name(void);

#endif

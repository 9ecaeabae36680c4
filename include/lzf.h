/*
 * lzf.h -- drop-in replacement for Gibson's src/lzf.h (reference
 * src/lzf.h:49, 76-78, 95-97), served by liblzf_hip.so on MI355X.
 *
 * The prototypes, LZF_VERSION, argument meaning, return values and errno
 * conventions are the reference's:
 *   lzf_compress   returns the number of bytes written to out_data, or 0 if
 *                  the stream does not fit in out_len (or in_len/out_len is
 *                  0); errno untouched.  Output is bit-identical to the
 *                  reference src/lzf_c.c.
 *   lzf_decompress returns the decoded length, or 0 with errno = E2BIG
 *                  (out_len too small) or EINVAL (corrupt stream), checked in
 *                  the order of src/lzf_d.c.
 * Buffers are host memory owned by the caller and must not overlap.
 *
 * Unlike the reference header this one carries an extern "C" guard, so the
 * same header serves C callers (src/query.c, src/net.c) and C++ code.
 * The calls are thread-safe; the library initialises HIP lazily on first use,
 * on the device named by LZF_GPU_DEVICE (default 0), and restores the
 * caller's current device before returning.
 */
#ifndef LZF_H
#define LZF_H

#define LZF_VERSION 0x0105 /* 1.5, API version (src/lzf.h:49) */

#ifdef __cplusplus
extern "C" {
#endif

/* replaces src/lzf_c.c:98 (prototype src/lzf.h:76-78) */
unsigned int
lzf_compress (const void *const in_data,  unsigned int in_len,
              void             *out_data, unsigned int out_len);

/* replaces src/lzf_d.c:55 (prototype src/lzf.h:95-97) */
unsigned int
lzf_decompress (const void *const in_data,  unsigned int in_len,
                void             *out_data, unsigned int out_len);

#ifdef __cplusplus
}
#endif

#endif /* LZF_H */

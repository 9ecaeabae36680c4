/*
 * lzf_dsize.hip -- decoded-size pre-pass: for every stream, the length
 * lzf_decompress would return with a given out_len, and its errno, without
 * writing any output.
 *
 * Gibson stores only the compressed length of an LZF item (src/net.h:285,
 * src/query.c:408) and decodes into one maxrequestsize buffer per item
 * (src/net.c:1306-1311, src/gibson.c:246).  A device batch of MGET items
 * needs an output slot per item, so items without an original-length
 * side-table entry (gb_lentab_*) are sized by this kernel first and then
 * decoded into exact slots -- nothing is staged at maxrequestsize.
 *
 * One lane per stream walks the tokens with the reference's checks in its
 * order (src/lzf_d.c:64-146): literal E2BIG (:72-76) before input EINVAL
 * (:78-84); back-reference input EINVAL (:100-117), then E2BIG (:121-125),
 * then the reference-before-output EINVAL (:127-131); the do-while reads one
 * control byte even for in_len 0 (:64-66).  MGET batches are small (tens to
 * thousands of items), so a lane per stream keeps a wave busy with 64 of
 * them; the decoder itself (lzf_decompress.hip) is the throughput path.
 */
#include <errno.h>

#include "lzf_internal.h"

__global__ __launch_bounds__(256) void lzf_dsize_kernel(const uint8_t *in, const uint64_t *in_off,
                                                      const uint32_t *in_len, uint32_t *out_size, int32_t *err,
                                                      uint32_t count, uint32_t limit)
{
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint8_t *ip = in + in_off[i];
    const uint32_t n = in_len[i];
    uint64_t k = 0, o = 0;
    int32_t e = 0;
    do {
        const uint32_t c = ip[k++];
        if (c < 32u) {                                              /* literal run of c + 1 */
            const uint32_t cnt = c + 1u;
            if (o + cnt > limit) { e = E2BIG; break; }
            if (k + cnt > n) { e = EINVAL; break; }
            o += cnt;
            k += cnt;
        } else {                                                    /* back-reference */
            uint32_t len = c >> 5;
            if (k >= n) { e = EINVAL; break; }
            if (len == 7u) {
                len += ip[k++];
                if (k >= n) { e = EINVAL; break; }
            }
            const uint64_t back = (((uint64_t)(c & 31u)) << 8) + 1u + ip[k++];
            if (o + len + 2u > limit) { e = E2BIG; break; }
            if (back > o) { e = EINVAL; break; }
            o += len + 2u;
        }
    } while (k < n);
    out_size[i] = e ? 0u : (uint32_t)o;
    err[i] = e;
}

hipError_t lzf_launch_dsize(const uint8_t *in, const uint64_t *in_off, const uint32_t *in_len, uint32_t *out_size,
                            int32_t *err, uint32_t count, uint32_t limit, hipStream_t s)
{
    hipLaunchKernelGGL(lzf_dsize_kernel, dim3((count + 255u) / 256u), dim3(256), 0, s, in, in_off, in_len, out_size,
                       err, count, limit);
    return hipGetLastError();
}

// decompress parallel generation: placeholder (serial kernel serves) until it lands
#include "lzf_internal.h"
hipError_t lzf_launch_decompress(const LzfBatch &, hipStream_t) { return hipErrorNotSupported; }
const char *lzf_decompress_kernel_name(void) { return nullptr; }

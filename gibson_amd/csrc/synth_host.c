/*
 * synth_host.c -- host build of the synthetic value generators (synth.h),
 * so tests and fixture tooling regenerate exactly the bytes the device
 * generator (lzf_synth_fill in liblzf_hip.so) writes into HBM.
 */
#include <stdint.h>
#include "synth.h"

void synth_fill(int kind, uint64_t seed, uint64_t first, uint32_t count,
                uint32_t n, uint8_t *out)
{
    for (uint32_t i = 0; i < count; i++)
        syn_generate(kind, seed, first + i, out + (uint64_t)i * n, n);
}

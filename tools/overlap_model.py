#!/usr/bin/env python3
"""Schedule model for the table generation's two kernels on configs[2]
(262 144 x 64 KiB text values, 256 CUs): can cand (lzf_cand_table_kernel)
and the record parse (lzf_parse_rec_kernel) overlap?  A design aid, not
product or test code ("model first").

Measured inputs:
  - cand: 82.8 ms for 262 144 values on 256 CUs, one value per CU at a time
    -> tau_c = 80.9 us per value per CU; a cand workgroup takes 157 KiB of the
    CU's 160 KiB LDS, so no parse block can share its CU;
  - parse: one lane per value, 256-lane blocks, 4 blocks (1024 lanes, 32 KiB
    LDS each block) per CU; one value's chain is ~68 ms however few values
    run (parse_scaling: 8 K values 67.9 ms ... 64 K 71.4); it ends line-bound
    at ~21 k one-line-per-lane fetches per value, ~50 G lines/s for the whole
    device (tools/fetch_calib.hip: 46-55 G/s from HBM / the Infinity Cache,
    so a device-wide limit; 241 G/s from L2).

Schedules, makespan lower bounds:
  sequential        cand on all CUs, then the parse: cand + max(chain, lines)
  CU partition(x)   cand on x CUs, the parse on the other 256 - x (stream CU
                    masks), records streamed from one to the other:
                    >= cand(x) + chain            (the last value's chain)
                    >= ceil(N / (1024 (256 - x))) chains (lanes in flight)
                    >= lines / rate               (rate device-wide, or
                                                   scaled by the parse CUs)
  co-resident       both on every CU (needs cand's table and 4 parse blocks
                    in one CU's LDS: 157 + 4 x 32 KiB > 160 KiB, so not
                    buildable): >= max(cand + chain, lines / rate)
"""
import math

N = 262144            # values (configs[2])
CUS = 256
TAU_C = 82.8e-3 * CUS / N          # s per value per CU (cand)
CHAIN = 68e-3                      # s, one value's parse chain
LANES_PER_CU = 1024
LINES = 21000 * N                  # parse line fetches
RATE = 50e9                        # lines/s, device-wide


def cand_time(cus):
    return N * TAU_C / cus


def main():
    seq = cand_time(CUS) + max(CHAIN, LINES / RATE)
    print("configs[2], 262 144 x 64 KiB values, 256 CUs -- makespan lower bounds (ms)")
    print(f"  sequential (measured: 82.8 + 107.4 = 190.2): model {1e3 * seq:.1f}")
    best = {}
    print("  CU partition, cand on x CUs / parse on 256 - x:")
    print("      x   cand+chain  lane gens x chain   lines (device)   lines (per CU)   bound (device / per CU)")
    for x in range(32, 256, 16):
        y = CUS - x
        a = cand_time(x) + CHAIN
        b = math.ceil(N / (LANES_PER_CU * y)) * CHAIN
        c_dev = LINES / RATE
        c_cu = LINES / (RATE * y / CUS)
        bd, bc = max(a, b, c_dev), max(a, b, c_cu)
        best.setdefault("dev", (bd, x))
        best.setdefault("cu", (bc, x))
        best["dev"] = min(best["dev"], (bd, x))
        best["cu"] = min(best["cu"], (bc, x))
        print(f"    {x:3d}   {1e3 * a:9.1f}   {1e3 * b:16.1f}   {1e3 * c_dev:14.1f}   {1e3 * c_cu:14.1f}"
              f"   {1e3 * bd:7.1f} / {1e3 * bc:7.1f}")
    print(f"  best CU partition: {1e3 * best['dev'][0]:.1f} ms at x = {best['dev'][1]} (device-wide line rate), "
          f"{1e3 * best['cu'][0]:.1f} ms at x = {best['cu'][1]} (per-CU line rate)")
    co = max(cand_time(CUS) + CHAIN, LINES / RATE)
    print(f"  co-resident (not buildable: LDS): {1e3 * co:.1f}")
    print("A CU partition cannot beat the sequential schedule: the parse needs all 262 144 values in")
    print("flight at once (1024 lanes on every CU) to pay its ~68 ms chain once, and every CU given to")
    print("cand takes 1024 of those lanes.  Only co-residency (both kernels on every CU) would reach ~151 ms.")


if __name__ == "__main__":
    main()

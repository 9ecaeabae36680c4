#!/usr/bin/env python3
"""Host model of the window64 compressor's control flow (no codec output):
counts windows, truncated windows, chain hops and matches per value so kernel
changes can be reasoned about without a GPU.  Uses the exact greedy parse."""
import sys

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tests.oracle_lib import synth  # noqa: E402


def slot(b, p):
    return (((b[p] << 8) | b[p + 1]) - 5 * ((b[p + 1] << 8) | b[p + 2])) & 0xFFFF


def hb(s):
    return ((s * 40503) >> 4) & 4095


def parse(b):
    """exact reference parse: list of (pos, m or 0), inserted set order"""
    n = len(b)
    tab = {}
    p = 0
    steps = []
    ins = []
    while n >= 3 and p < n - 2:
        s = slot(b, p)
        r = tab.get(s)
        tab[s] = p
        ins.append(p)
        if r is not None and p - r - 1 < 8192 and p + 4 < n and r > 0 and b[r:r + 3] == b[p:p + 3]:
            maxlen = min(n - p - 2, 264)
            lim = 19 if 16 < maxlen < 19 else maxlen
            k = 3
            while k < lim and b[r + k] == b[p + k]:
                k += 1
            steps.append((p, k))
            p += k
            if p >= n - 2:
                break
            tab[slot(b, p - 2)] = p - 2
            tab[slot(b, p - 1)] = p - 1
            ins += [p - 2, p - 1]
        else:
            steps.append((p, 0))
            p += 1
    return steps, set(ins)


def model(b, W=64):
    n = len(b)
    steps, ins = parse(b)
    stepat = {p: m for p, m in steps}
    windows = trunc = matches = hops = 0
    head = {}      # bucket -> list of inserted positions (for hop counting)
    P = 0
    inserted_sorted = sorted(ins)
    while P + 2 < n:
        windows += 1
        lim_lane = min(W, n - 2 - P)
        # visited lanes via the true parse from P
        i = 0
        interior = set()
        cut = None
        while i < lim_lane:
            p = P + i
            # prevW: nearest earlier lane with same slot
            s = slot(b, p)
            pw = None
            for j in range(i - 1, -1, -1):
                if slot(b, P + j) == s:
                    pw = j
                    break
            if pw is not None and pw in interior:
                cut = i
                break
            m = stepat.get(p, 0)
            if m:
                matches += 1
                for t in range(i + 1, i + m - 2):
                    interior.add(t)
                i += m
            else:
                i += 1
        if cut is not None:
            trunc += 1
            P += cut
        else:
            P += i
    return dict(n=n, steps=len(steps), windows=windows, trunc=trunc, matches=matches,
                bytes_per_window=n / windows)


if __name__ == "__main__":
    kind = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    for idx in range(3):
        print(model(synth(kind, 0x5EED0002, idx, n)))

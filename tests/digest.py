"""Full-batch digest of a compress batch, the record of
tests/golden/digests.json: sha256 over the values in order of
(u32 little-endian length || stream), length 0 = the value does not fit."""
import hashlib


def batch_digest(comp, n, lens):
    """comp: numpy uint8 array, value k's stream at k*n; lens: numpy ints."""
    h = hashlib.sha256()
    for k, ln in enumerate(lens.tolist()):
        h.update(int(ln).to_bytes(4, "little"))
        if ln:
            h.update(comp[k * n:k * n + ln].data)
    return h.hexdigest()

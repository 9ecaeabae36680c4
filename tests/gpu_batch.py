"""Helpers to run lists of byte strings through the device batch API."""
import numpy as np
import torch

import gibson_amd


def _pack(values, align=16):
    offs, pos = [], 0
    for v in values:
        offs.append(pos)
        pos += (max(len(v), 1) + align - 1) // align * align
    arena = np.zeros(max(pos, 16), np.uint8)
    for o, v in zip(offs, values):
        arena[o:o + len(v)] = np.frombuffer(v, np.uint8)
        if not v:
            arena[o] = 0xFF          # the phantom control byte of a 0-length stream
    return arena, np.array(offs, np.int64)


def _caps_layout(caps, align=16):
    offs, pos = [], 0
    for c in caps:
        offs.append(pos)
        pos += (max(c, 1) + align - 1) // align * align
    return np.array(offs, np.int64), max(pos, 16)


def gpu_compress(values, out_caps, dev="cuda", align=16):
    arena, in_off = _pack(values, align)
    out_off, out_size = _caps_layout(out_caps, align)
    d_in = torch.from_numpy(arena).to(dev)
    d_in_off = torch.from_numpy(in_off).to(dev)
    d_in_len = torch.tensor([len(v) for v in values], dtype=torch.int32, device=dev)
    d_out = torch.zeros(out_size, dtype=torch.uint8, device=dev)
    d_out_off = torch.from_numpy(out_off).to(dev)
    d_cap = torch.tensor(out_caps, dtype=torch.int32, device=dev)
    d_len = torch.full((len(values),), -1, dtype=torch.int32, device=dev)
    gibson_amd.compress_batch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_cap, d_len,
                              max(len(v) for v in values))
    torch.cuda.synchronize()
    lens = d_len.cpu().numpy().astype(np.int64)
    out = d_out.cpu().numpy()
    res = []
    for o, l in zip(out_off, lens):
        res.append(bytes(out[o:o + l]) if l > 0 else None)
    return res


def gpu_decompress(streams, out_caps, dev="cuda", align=16):
    arena, in_off = _pack(streams, align)
    out_off, out_size = _caps_layout(out_caps, align)
    d_in = torch.from_numpy(arena).to(dev)
    d_in_off = torch.from_numpy(in_off).to(dev)
    d_in_len = torch.tensor([len(v) for v in streams], dtype=torch.int32, device=dev)
    d_out = torch.zeros(out_size, dtype=torch.uint8, device=dev)
    d_out_off = torch.from_numpy(out_off).to(dev)
    d_cap = torch.tensor(out_caps, dtype=torch.int32, device=dev)
    d_len = torch.full((len(streams),), -1, dtype=torch.int32, device=dev)
    d_err = torch.full((len(streams),), -1, dtype=torch.int32, device=dev)
    gibson_amd.decompress_batch(d_in, d_in_off, d_in_len, d_out, d_out_off, d_cap, d_len, d_err,
                                max(out_caps))
    torch.cuda.synchronize()
    lens = d_len.cpu().numpy().astype(np.int64)
    errs = d_err.cpu().numpy()
    out = d_out.cpu().numpy()
    res = []
    for o, l, e in zip(out_off, lens, errs):
        res.append((bytes(out[o:o + l]) if l > 0 else None, int(e)))
    return res

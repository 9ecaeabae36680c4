"""Multi-process sharding on CPU (gloo, world_size 2): round-robin value
ownership covers every value exactly once, and the max/sum reductions used
by bench.py combine per-rank results.  The per-rank codec work here is the
CPU oracle (test infrastructure), standing in for the GPU batch."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gibson_amd.shard import global_indices, reduce_stats, spread_stats
    from tests.oracle_lib import Oracle, synth
    per = total // world
    idx = global_indices(rank, world, per)
    o = Oracle()
    in_bytes = comp = 0
    for i in idx:
        v = synth(1, 0x5EED0002, i, 512)
        c = o.compress(v, 508)
        in_bytes += len(v)
        comp += len(c) if c else 0
    (tmax,), (b, cb, nv) = reduce_stats([float(rank + 1)], [in_bytes, comp, len(idx)])
    (lo, clo), (hi, chi) = spread_stats([10.0 * (rank + 1), comp])
    q.put((rank, idx, tmax, b, cb, nv, comp, lo, hi, clo, chi))
    dist.destroy_process_group()


def test_round_robin_two_ranks():
    world, total = 2, 64
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    owned = sorted(i for r in res for i in r[1])
    assert owned == list(range(total))                 # each value exactly once
    assert res[0][1] == list(range(0, total, 2))       # value i -> rank i mod N
    for r in res:
        assert r[2] == world                           # max over ranks
        assert r[3] == total * 512                     # summed bytes
        assert r[5] == total
    assert res[0][4] == res[0][6] + res[1][6]          # summed compressed bytes
    for r in res:                                      # per-rank spread: min / max over ranks
        assert (r[7], r[8]) == (10.0, 20.0)
        assert (r[9], r[10]) == (min(res[0][6], res[1][6]), max(res[0][6], res[1][6]))

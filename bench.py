#!/usr/bin/env python3
"""Headline benchmark: device-resident LZF compress+decompress over batched
value blocks (BASELINE.json "metric"), on N GPUs of one node.

A *step* is one pass of the hot path over one batch of synthetic values
already resident in HBM: lzf_gpu_compress_batch (out_len = n-4, the server
policy of src/query.c:385) followed by lzf_gpu_decompress_batch of the
results (out_len = n).  Values that do not compress are not decoded (as in
the server, src/query.c:393-397).

Default workload = BASELINE.json configs[2]: 256 K x 64 KiB sentence-bank
text values per GPU (the north star's 64 KiB target and the largest
single-GPU compress+decompress config).  Multi-GPU: one process per GPU,
values sharded round-robin (value i -> rank i mod N); no
data-path collective, only a barrier and a max-over-ranks of the timings.
Weak scaling by default (every rank owns `count` values); `--total T` is the
strong-scaling mode (T values over all ranks, e.g. BASELINE configs[4]:
--workload mixed16k --total 4194304).

`--gpus N` with N > 1 and no torchrun environment re-launches this script
under torch.distributed.run with N ranks (a child process, started before
any GPU call); under torchrun, --gpus must equal WORLD_SIZE.

Prints ONE JSON line on rank 0 (contract in the task statement), including
"roofline" for the dominant kernel (HIP events on the launch stream) and
"cpu_baseline" (the reference codec compiled from /root/reference by
oracle/Makefile, timed on this host's cores on a bounded sample; rank 0,
N=1 only).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
import gibson_amd  # noqa: E402
from gibson_amd.shard import reduce_stats, shard, spread_stats  # noqa: E402

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
CHUNK_BYTES = 16 << 30  # codec chunk of a batch past this many input bytes
RED_DEV = "cpu"         # device of the cross-rank reduction tensors (set in main)

WORKLOADS = {
    # name: (BASELINE config index, synth kind, seed, value bytes, values per GPU)
    "json4k": (1, 1, 0x5EED0002, 4096, 1 << 20),
    "text64k": (2, 2, 0x5EED0003, 65536, 1 << 18),
    "text8k": (3, 0, 0x5EED0004, 8192, 1 << 20),
    "mixed16k": (4, 3, 0x5EED0005, 16384, 1 << 20),
}
DESCR = {
    "json4k": "1M x 4 KiB JSON-like values per GPU (BASELINE configs[1])",
    "text64k": "256K x 64 KiB sentence-bank text per GPU (BASELINE configs[2])",
    "text8k": "8 KiB Zipf text values (BASELINE configs[3] value shape)",
    "mixed16k": "16 KiB mixed-entropy values (BASELINE configs[4] value shape)",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (ranks) on this node; default 1")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", default="roundtrip", choices=("roundtrip", "decompress"),
                    help="roundtrip = the headline (compress+decompress); decompress = "
                         "BASELINE configs[3], decode of pre-compressed blocks only")
    ap.add_argument("--workload", default="", choices=[""] + sorted(WORKLOADS),
                    help="default: text64k (roundtrip, BASELINE configs[2]), text8k (decompress)")
    ap.add_argument("--count", type=int, default=0, help="values per GPU (default: workload's)")
    ap.add_argument("--total", type=int, default=0,
                    help="strong scaling: values over all ranks (rank r takes values r, r+N, ...)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--config4", action="store_true",
                    help="also measure BASELINE configs[4] (4M x 16 KiB over the ranks) into a config4 "
                         "block; on by default when N > 1 on the default workload")
    ap.add_argument("--no-config4", action="store_true", help="skip the configs[4] block at N > 1")
    ap.add_argument("--config4-total", type=int, default=4 << 20,
                    help="values of the configs[4] block over all ranks (default 4194304, BASELINE configs[4])")
    ap.add_argument("--cpu-count", type=int, default=0, help="CPU baseline sample values")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU baseline threads (default: the cores this process may run on)")
    a = ap.parse_args()
    a.workload_given = bool(a.workload)
    return a


def launch_ranks(a):
    """--gpus N without a torchrun environment: run N ranks as a child
    torch.distributed.run (this process has not touched the GPU) and exit
    with its status.  Under torchrun, --gpus must match WORLD_SIZE."""
    world = os.environ.get("WORLD_SIZE")
    if world is not None:
        if a.gpus is not None and a.gpus != int(world):
            sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
        return
    if a.gpus is None or a.gpus <= 1:
        return
    import socket
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    sys.exit(subprocess.call(cmd))


def cpu_cores():
    """(cores, note): the CPUs this process may run on -- its affinity set,
    capped by the cgroup CPU quota (cpu.max) where one is set: on the GPU box
    the affinity lists the whole machine (256) while the quota grants 16."""
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    cores = min(aff, quota) if quota else aff
    return cores, f"affinity {aff} CPUs, cgroup quota {quota if quota else 'none'}"


def _cpu_run(kind, seed, n, count, threads, reps):
    ref = os.path.join(ROOT, "oracle", "_ref", "cpu_bench_ref")
    port = os.path.join(ROOT, "oracle", "cpu_bench")
    exe = ref if os.path.exists(ref) else port
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, str(kind), str(n), str(count), str(threads), hex(seed), str(reps)],
                         capture_output=True, text=True, timeout=900,
                         env=dict(os.environ, OMP_NUM_THREADS=str(threads)))
    if out.returncode != 0:
        return {"error": out.stderr.strip()[-200:]}
    return json.loads(out.stdout)


def cpu_baseline(kind, seed, n, count, threads, decode_only=False):
    """Time the CPU codec (the reference compiled by oracle/Makefile) on
    bounded samples of the workload (checker/baseline only): on all the
    cores this process may run on (`threads`, one value per OpenMP thread)
    and on one core."""
    key = "decompress_GBps" if decode_only else "roundtrip_GBps"
    r = _cpu_run(kind, seed, n, count, threads, 5)
    if r is None or "error" in r:
        return r
    cnt1 = max(16, min(count, (96 << 20) // n))
    r1 = _cpu_run(kind, seed, n, cnt1, 1, 3)
    what = "decompress of the reference-compressed values" if decode_only else "compress+decompress"
    out = {
        "value": round(r[key], 4),
        "unit": "GB/s",
        "cores": threads,
        "kind": r["kind"],
        "sample": f"{count} values x {n} B (the workload's first {count} value indices), {what}, "
                  f"median of 5 after 1 warm-up, one value per OpenMP thread on {threads} threads; "
                  f"compress {r['compress_GBps']:.3f} GB/s, decompress {r['decompress_GBps']:.3f} GB/s, "
                  f"ratio {r['comp_bytes'] / r['in_bytes']:.4f}",
        "cpu": _cpu_model(),
    }
    if r1 and "error" not in r1:
        out["value_1core"] = round(r1[key], 4)
        out["sample_1core"] = (f"{cnt1} values x {n} B, median of 3 after 1 warm-up, 1 thread; "
                               f"compress {r1['compress_GBps']:.4f} GB/s, "
                               f"decompress {r1['decompress_GBps']:.4f} GB/s")
    return out


def _traffic(workload, kernel, count):
    """(HBM bytes per launch of `kernel`, where they come from) from the
    committed PMC summary (profiles/traffic_<workload>.json, tools/traffic.py:
    2*FETCH_SIZE + WRITE_SIZE, KiB -> B; the x2 read correction is calibrated
    for both the streaming and the one-line-per-lane loads, profiles/r03/
    fetch_calib.txt), stamped with the commit the counters were taken at --
    a per-value figure times this launch's count, not a counter of this run;
    (None, None) when there is none."""
    f = os.path.join(ROOT, "profiles", f"traffic_{workload}.json")
    try:
        t = json.load(open(f))
        return (int(t["kernels"][kernel]["bytes_per_value"] * count),
                {"file": os.path.relpath(f, ROOT), "profile_commit": t.get("profile_commit"),
                 "bytes_per_value": round(t["kernels"][kernel]["bytes_per_value"], 1),
                 "read_correction": (t.get("calibration") or {}).get("read_correction", 2.0)})
    except (OSError, KeyError, ValueError):
        return None, None


def _spread(world, steps, k_lo, k_hi, w_lo, w_hi):
    """min / max over ranks of the per-step device time (HIP events around
    the rank's launches) and of the timed wall region: the imbalance the
    max-over-ranks `ms_per_step` hides"""
    return {"ranks": world,
            "kernel_ms_min": round(k_lo * 1e3, 3), "kernel_ms_max": round(k_hi * 1e3, 3),
            "wall_ms_per_step_min": round(w_lo / steps * 1e3, 3),
            "wall_ms_per_step_max": round(w_hi / steps * 1e3, 3),
            "kernel_imbalance": round(k_hi / k_lo, 4) if k_lo > 0 else None}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main():
    a = parse()
    launch_ranks(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # the ranks meet only at the timing barriers and one reduction of timings
    # and counts: RCCL by default; LZF_BENCH_BACKEND=gloo does both on the host
    # (LZF_BENCH_SHARE_GPU=1 puts every rank on device local % count: a
    # rehearsal of the N-rank path on a one-GPU box, not a measurement)
    backend = os.environ.get("LZF_BENCH_BACKEND", "nccl")
    if world > 1:
        share = os.environ.get("LZF_BENCH_SHARE_GPU") == "1"
        local_dev = local % torch.cuda.device_count() if share else local
        torch.cuda.set_device(local_dev)
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    global RED_DEV
    RED_DEV = "cpu" if backend == "gloo" else dev
    if not a.workload:
        a.workload = "text8k" if a.mode == "decompress" else "text64k"
    cfg_idx, kind, seed, n, count = WORKLOADS[a.workload]
    if a.mode == "decompress" and a.workload == "text8k":
        count = 8 << 20                                  # BASELINE configs[3]: 8 M blocks
    if a.count:
        count = a.count
    if a.total:                                          # strong scaling: rank's round-robin share
        if a.total < world:
            sys.exit(f"bench.py: --total {a.total} gives rank {world - 1} no value (fewer values than ranks)")
        count = (a.total - rank + world - 1) // world
    if a.mode == "decompress":
        return main_decompress(a, world, rank, dev, cfg_idx, kind, seed, n, count)

    rt = run_roundtrip(a, world, rank, dev, kind, seed, n, count)
    line = roundtrip_line(a, world, rank, rt, cfg_idx, kind, seed, n, count)
    # N > 1 on the default workload: the driver's 1 -> 8 curve stays on
    # configs[2] (weak scaling, the `value` every N reports), and the line also
    # carries configs[4] -- 4 M x 16 KiB split over the ranks, the config the
    # north star's >= 0.9x per-GPU efficiency target is stated on
    #  -- measured in the same job, with its per-GPU
    # efficiency against the committed N = 1 figure
    if wants_config4(a, world):
        del rt
        gibson_amd.release()
        torch.cuda.empty_cache()
        c_idx, c_kind, c_seed, c_n, _ = WORKLOADS["mixed16k"]
        c_total = a.config4_total
        c_count = (c_total - rank + world - 1) // world
        r4 = run_roundtrip(a, world, rank, dev, c_kind, c_seed, c_n, c_count)
        if rank == 0:
            line["config4"] = config4_block(world, r4, c_total, c_n)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


CONFIG4_TOTAL = 4 << 20          # BASELINE configs[4]: 4 M x 16 KiB values over all ranks
CONFIG4_N1 = os.path.join(ROOT, "profiles", "r06", "config4_n1.json")


def wants_config4(a, world):
    """whether the line carries the configs[4] block: asked for (--config4),
    or N > 1 on the default round-trip workload (the driver's scaling runs),
    unless --no-config4"""
    if a.no_config4 or a.mode != "roundtrip":
        return False
    return a.config4 or (world > 1 and not (a.workload_given or a.total or a.count))


def config4_block(world, r4, total, n):
    """configs[4]'s strong split measured beside the headline: aggregate
    GB/s over all ranks, and per-GPU efficiency = value / (N x the N = 1
    figure committed in profiles/r06/config4_n1.json, `bench.py --workload
    mixed16k --total 4194304` on one MI355X)"""
    sec = r4["wall"] / r4["steps"]
    value = r4["in_bytes_all"] / sec / 1e9
    blk = {"config": "BASELINE configs[4]: 4M x 16 KiB mixed-entropy values sharded round-robin over "
                     f"{world} rank(s) (strong scaling; the north star's >= 0.9x per-GPU efficiency target)",
           "baseline_config": 4, "total_values": total, "values_per_gpu_max": -(-total // world),
           "value": round(value, 3), "unit": "GB/s", "ms_per_step": round(sec * 1e3, 3),
           "roundtrip_ok": r4["bad_ranks"] == 0, "chunks_per_rank": r4["nch"],
           "per_kernel_ms_rank0": {"lzf_compress": round(r4["t_comp"] * 1e3, 3),
                                   "lzf_decompress": round(r4["t_dec"] * 1e3, 3)}}
    try:
        ref = json.load(open(CONFIG4_N1))
        v1 = float(ref["value"])
        blk["n1_value"] = v1
        blk["n1_source"] = os.path.relpath(CONFIG4_N1, ROOT)
        # only against the figure of the same configuration
        blk["per_gpu_efficiency"] = round(value / (world * v1), 4) if total == ref.get("total_values") else None
    except (OSError, KeyError, ValueError):
        blk["n1_value"] = None
        blk["per_gpu_efficiency"] = None
    return blk


def run_roundtrip(a, world, rank, dev, kind, seed, n, count):
    """One workload's timed round trips on this rank: value k of this rank is
    global value rank + k*world, generated into HBM; a step compresses every
    value (out_len n-4) and decodes every success.  Returns this rank's
    timings and counts and the job-wide reductions."""
    # A batch past CHUNK_BYTES (BASELINE configs[4] at N = 1: 4 M x 16 KiB =
    # 64 GiB) keeps every input and stream resident but runs the codec in
    # chunks of <= 16 GiB (SURVEY.md §8(d) timing rules): the kernels' scratch
    # and the decode arena are per chunk; a step is all chunks in order.
    chunk = count if count * n <= CHUNK_BYTES else max(1, CHUNK_BYTES // n)
    nch = (count + chunk - 1) // chunk
    src = torch.empty(count * n, dtype=torch.uint8, device=dev)
    first, stride = shard(rank, world)
    gibson_amd.synth_fill(kind, seed, first, stride, count, n, src)
    off = torch.arange(chunk, dtype=torch.int64, device=dev) * n
    in_len = torch.full((chunk,), n, dtype=torch.int32, device=dev)
    ccap = torch.full((chunk,), n - 4, dtype=torch.int32, device=dev)
    comp = torch.empty(count * n, dtype=torch.uint8, device=dev)
    clen = torch.zeros(count, dtype=torch.int32, device=dev)
    dcap = torch.full((chunk,), n, dtype=torch.int32, device=dev)
    dec = torch.empty(chunk * n, dtype=torch.uint8, device=dev)
    dlen = torch.zeros(chunk, dtype=torch.int32, device=dev)
    derr = torch.zeros(chunk, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    torch.cuda.synchronize()

    ev = []
    good = True

    def verify(c0, m):
        """every compressed value of chunk [c0, c0 + m) decoded back (untimed)"""
        ok = clen[c0:c0 + m] > 0
        g = bool(((dlen[:m] == n) | ~ok).all())
        dv, sv = dec[:m * n].view(m, n), src[c0 * n:(c0 + m) * n].view(m, n)
        for r0 in range(0, m, 1 << 16):
            r1 = min(m, r0 + (1 << 16))
            g = g and not bool(((dv[r0:r1] != sv[r0:r1]).any(dim=1) & ok[r0:r1]).any())
        return g

    def step(record, check):
        nonlocal good
        for ci in range(nch):
            c0 = ci * chunk
            m = min(chunk, count - c0)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e2 = torch.cuda.Event(enable_timing=True)
            sv, cv = src[c0 * n:(c0 + m) * n], comp[c0 * n:(c0 + m) * n]
            e0.record(stream)
            gibson_amd.compress_batch(sv, off[:m], in_len[:m], cv, off[:m], ccap[:m], clen[c0:c0 + m], n, stream)
            e1.record(stream)
            # failed values (clen == 0) decode a 0-length stream: one control
            # byte and an immediate error, i.e. they are skipped as in the server
            gibson_amd.decompress_batch(cv, off[:m], clen[c0:c0 + m], dec, off[:m], dcap[:m], dlen[:m], derr[:m],
                                        n, stream)
            e2.record(stream)
            if record:
                ev.append((e0, e1, e2))
            if check:
                torch.cuda.synchronize()
                good = verify(c0, m) and good

    for w_ in range(a.warmup):
        step(False, w_ == 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True, False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0

    t_comp = sum(e0.elapsed_time(e1) for e0, e1, _ in ev) / a.steps / 1e3
    t_dec = sum(e1.elapsed_time(e2) for _, e1, e2 in ev) / a.steps / 1e3
    ok = clen > 0
    n_ok = int(ok.sum())
    c_bytes = int(clen.to(torch.int64).sum())
    # sanity (outside the timed region): the last chunk of the last step, and
    # every chunk in the first warm-up step
    c0 = (nch - 1) * chunk
    good = verify(c0, count - c0) and good

    (k_lo, w_lo), (k_hi, w_hi) = spread_stats([t_comp + t_dec, wall], device=RED_DEV)
    (wall, t_comp_max, t_dec_max), (in_bytes_all, n_ok_all, c_bytes_all, bad_ranks) = reduce_stats(
        [wall, t_comp, t_dec], [count * n, n_ok, c_bytes, 0 if good else 1], device=RED_DEV)
    return {"wall": wall, "steps": a.steps, "t_comp": t_comp, "t_dec": t_dec, "n_ok": n_ok, "c_bytes": c_bytes,
            "in_bytes_all": in_bytes_all, "n_ok_all": n_ok_all, "c_bytes_all": c_bytes_all,
            "bad_ranks": bad_ranks, "nch": nch, "chunk": chunk,
            "spread": (k_lo, k_hi, w_lo, w_hi)}


def roundtrip_line(a, world, rank, rt, cfg_idx, kind, seed, n, count):
    """rank 0's JSON line for a round-trip run (None on other ranks)"""
    if rank != 0:
        return None
    wall, t_comp, t_dec = rt["wall"], rt["t_comp"], rt["t_dec"]
    n_ok, c_bytes = rt["n_ok"], rt["c_bytes"]
    sec_per_step = wall / a.steps
    value = rt["in_bytes_all"] / sec_per_step / 1e9
    # algorithmic bytes per launch, this rank
    comp_bytes = count * n + c_bytes + 4 * count          # read N, write C + 4
    dec_bytes = c_bytes + n_ok * n                          # read C, write N
    kern = {
        "lzf_compress": (comp_bytes, t_comp),
        "lzf_decompress": (dec_bytes, t_dec),
    }
    dom = max(kern, key=lambda k: kern[k][1])
    ach = kern[dom][0] / kern[dom][1] / 1e9
    # the north star's compress + decompress at once: 2N + 2C + 4 per value
    # over all ranks (compress reads N, writes C + 4; decode reads C, writes N)
    # over the step's wall time, per GPU, against the per-GPU peak
    rt_bytes_all = 2 * rt["in_bytes_all"] + 2 * rt["c_bytes_all"] + 4 * count * world
    roundtrip_frac = rt_bytes_all / sec_per_step / 1e9 / (HBM_PEAK_GBPS * world)
    k_lo, k_hi, w_lo, w_hi = rt["spread"]
    line = {
        "metric": "LZF GB/s (device-resident) over batched value blocks, compress+decompress",
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(sec_per_step * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if a.total else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {
            "workload": DESCR[a.workload] if not a.total else
                        f"{a.total} x {n // 1024} KiB values over all ranks ({DESCR[a.workload]})",
            "baseline_config": cfg_idx,
            "values_per_gpu": count,
            "value_bytes": n,
            "out_len_policy": "n-4 (src/query.c:385)",
            "sharding": "round-robin value i -> rank i mod N, no collective",
            "compressed_fraction": round(rt["n_ok_all"] / (count * world), 4),
            "ratio": round(rt["c_bytes_all"] / max(1.0, rt["n_ok_all"] * n), 4),
            "kernels": gibson_amd.kernel_info(),
            "roundtrip_ok": rt["bad_ranks"] == 0,
            "chunks": rt["nch"],
            "chunk_values": rt["chunk"],
        },
        "rank_spread": _spread(world, a.steps, k_lo, k_hi, w_lo, w_hi),
        "roofline": {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(ach, 2),
            "peak": HBM_PEAK_GBPS,
            "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBPS, 5),
            "roundtrip_frac": round(roundtrip_frac, 5),
            "roundtrip_bytes_per_value": "2N + 2C + 4 (compress reads N, writes C + 4; decode reads C, writes N)",
            "traffic": _traffic(a.workload, dom, count)[0],
            "traffic_source": _traffic(a.workload, dom, count)[1],
            "algorithmic_bytes": kern[dom][0],
            "per_kernel_ms": {k: round(v[1] * 1e3, 3) for k, v in kern.items()},
            "per_kernel_GBps": {k: round(v[0] / v[1] / 1e9, 2) for k, v in kern.items()},
            # the round trip's read-only fraction, sum(N + C) / t / peak
            "read_only_frac": round((count * n + c_bytes) / (t_comp + t_dec) / 1e9 / HBM_PEAK_GBPS, 5),
        },
    }
    if world == 1 and not a.no_cpu:
        cores, note = cpu_cores()
        threads = a.cpu_threads or cores
        cnt = a.cpu_count or min(count, max(4 * threads, (4 << 30) // n))
        line["cpu_baseline"] = cpu_baseline(kind, seed, n, cnt, threads)
        if line["cpu_baseline"] and "error" not in line["cpu_baseline"]:
            line["cpu_baseline"]["cores_note"] = note
    return line


def main_decompress(a, world, rank, dev, cfg_idx, kind, seed, n, count):
    """BASELINE configs[3]: decode-path throughput.  Setup (untimed): values
    are generated and compressed (out_len = n-4) in chunks of 1 M, into slots
    of n bytes; the generator buffer is then freed.  A step is one
    lzf_gpu_decompress_batch over all `count` streams with out_len = n.
    Values that did not compress (clen == 0) would decode a 0-length stream
    and fail at once; they are excluded from the bytes counted."""
    chunk = min(count, 1 << 20)
    first, stride = shard(rank, world)
    off = torch.arange(count, dtype=torch.int64, device=dev) * n
    comp = torch.empty(count * n, dtype=torch.uint8, device=dev)
    clen = torch.zeros(count, dtype=torch.int32, device=dev)
    src = torch.empty(chunk * n, dtype=torch.uint8, device=dev)
    coff = torch.arange(chunk, dtype=torch.int64, device=dev) * n
    cin = torch.full((chunk,), n, dtype=torch.int32, device=dev)
    ccap = torch.full((chunk,), n - 4, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream()
    for c0 in range(0, count, chunk):
        m = min(chunk, count - c0)
        gibson_amd.synth_fill(kind, seed, first + c0 * stride, stride, m, n, src)
        gibson_amd.compress_batch(src, coff[:m], cin[:m], comp[c0 * n:], coff[:m], ccap[:m],
                                  clen[c0:c0 + m], n, stream)
    torch.cuda.synchronize()
    dcap = torch.full((count,), n, dtype=torch.int32, device=dev)
    dec = torch.empty(count * n, dtype=torch.uint8, device=dev)
    dlen = torch.zeros(count, dtype=torch.int32, device=dev)
    derr = torch.zeros(count, dtype=torch.int32, device=dev)
    ev = []

    def step(record):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        gibson_amd.decompress_batch(comp, off, clen, dec, off, dcap, dlen, derr, n, stream)
        e1.record(stream)
        if record:
            ev.append((e0, e1))

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    t_dec = sum(e0.elapsed_time(e1) for e0, e1 in ev) / a.steps / 1e3

    # sanity (outside the timed region): every compressed value decodes back
    ok = clen > 0
    n_ok = int(ok.sum())
    c_bytes = int(clen.to(torch.int64).sum())
    good = bool(((dlen == n) | ~ok).all()) and not bool((derr[ok] != 0).any())
    for c0 in range(0, count, chunk):
        m = min(chunk, count - c0)
        gibson_amd.synth_fill(kind, seed, first + c0 * stride, stride, m, n, src)
        diff = (dec[c0 * n:(c0 + m) * n].view(m, n) != src[:m * n].view(m, n)).any(dim=1)
        good = good and not bool((diff & ok[c0:c0 + m]).any())
    del src

    (k_lo, w_lo), (k_hi, w_hi) = spread_stats([t_dec, wall], device=RED_DEV)
    (wall, t_dec), (n_ok_all, c_bytes_all, bad_ranks) = reduce_stats(
        [wall, t_dec], [n_ok, c_bytes, 0 if good else 1], device=RED_DEV)
    if rank == 0:
        sec_per_step = wall / a.steps
        out_bytes_all = n_ok_all * n
        dec_bytes = c_bytes + n_ok * n                          # read C, write N (this rank)
        ach = dec_bytes / t_dec / 1e9
        line = {
            "metric": "LZF GB/s (device-resident) decompress-only over pre-compressed value blocks",
            "value": round(out_bytes_all / sec_per_step / 1e9, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(sec_per_step * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if a.total else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {
                "workload": (f"{a.total} x {n // 1024} KiB pre-compressed blocks over all ranks, decompress only"
                             if a.total else
                             f"{count // (1 << 20)}M x {n // 1024} KiB pre-compressed blocks per GPU, "
                             f"decompress only (BASELINE configs[3])" if count >= (1 << 20) else
                             f"{count} x {n} B pre-compressed blocks per GPU, decompress only"),
                "baseline_config": 3,
                "values_per_gpu": count,
                "value_bytes": n,
                "out_len_policy": f"compressed at n-4 (src/query.c:385), decoded with out_len = {n}",
                "sharding": "round-robin value i -> rank i mod N, no collective",
                "compressed_fraction": round(n_ok_all / (count * world), 4),
                "ratio": round(c_bytes_all / max(1.0, out_bytes_all), 4),
                "kernels": gibson_amd.kernel_info(),
                "roundtrip_ok": bad_ranks == 0,
            },
            "rank_spread": _spread(world, a.steps, k_lo, k_hi, w_lo, w_hi),
            "roofline": {
                "bound": "hbm",
                "kernel": "lzf_decompress",
                "achieved": round(ach, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBPS, 5),
                "traffic": _traffic(f"{a.workload}_decode", "lzf_decompress", count)[0],
                "traffic_source": _traffic(f"{a.workload}_decode", "lzf_decompress", count)[1],
                "algorithmic_bytes": dec_bytes,
                "per_kernel_ms": {"lzf_decompress": round(t_dec * 1e3, 3)},
            },
        }
        if world == 1 and not a.no_cpu:
            cores, note = cpu_cores()
            threads = a.cpu_threads or cores
            cnt = a.cpu_count or min(count, max(4 * threads, (4 << 30) // n))
            line["cpu_baseline"] = cpu_baseline(kind, seed, n, cnt, threads, decode_only=True)
            if line["cpu_baseline"] and "error" not in line["cpu_baseline"]:
                line["cpu_baseline"]["cores_note"] = note
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

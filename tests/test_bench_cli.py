"""bench.py's command line: the driver's contract flags and the decode-only
mode parse on CPU (--help starts no GPU work); short runs on the GPU."""
import os
import subprocess
import sys

import pytest

from tests.oracle_lib import ROOT


def test_bench_help_lists_contract_flags():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-500:]
    for flag in ("--gpus", "--steps", "--warmup", "--mode", "--workload"):
        assert flag in r.stdout
    assert "decompress" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ["--count", "8192"],
    ["--mode", "decompress", "--count", "8192"],
    ["--workload", "text64k", "--count", "512"],
])
def test_bench_small_run(args):
    # a short bench.py run on the GPU prints one JSON line whose round trip
    # checked out (the driver's own runs use the full sizes)
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1",
                        "--warmup", "0", "--no-cpu"] + args,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-800:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["roundtrip_ok"] is True
    assert line["value"] > 0 and line["roofline"]["peak"] == 8000.0


def test_bench_gpus_must_match_world_size():
    # under torchrun, --gpus N that disagrees with WORLD_SIZE is refused
    # before any GPU work
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0
    assert "WORLD_SIZE" in r.stderr


@pytest.mark.gpu
def test_bench_default_is_configs2_with_cpu_baseline():
    # the driver's N=1 command on the default workload: BASELINE configs[2]
    # (256K x 64 KiB text), the CPU baseline on every core this process may
    # use plus a 1-core figure
    import json
    sys.path.insert(0, ROOT)
    import bench
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "1",
                        "--warmup", "0", "--cpu-count", "64"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-800:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["baseline_config"] == 2
    assert line["config"]["workload"].startswith("256K x 64 KiB") and line["n_gpus"] == 1
    assert line["config"]["roundtrip_ok"] is True
    cb = line["cpu_baseline"]
    assert cb["cores"] == bench.cpu_cores()[0]
    assert cb["value_1core"] > 0 and cb["value"] > 0


@pytest.mark.gpu
@pytest.mark.parametrize("args", [
    ["--count", "4096"],                                          # weak scaling, round trip
    ["--workload", "mixed16k", "--total", "8192"],                # strong scaling (configs[4] shape)
])
def test_bench_two_ranks_rehearsal(args):
    # the N-rank path end to end on one GPU: --gpus 2 starts two ranks as a
    # child torch.distributed.run, both on device 0 (LZF_BENCH_SHARE_GPU),
    # meeting through gloo; rank 0 prints one line for the whole job
    import json
    env = dict(os.environ, LZF_BENCH_BACKEND="gloo", LZF_BENCH_SHARE_GPU="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "0", "--no-cpu"] + args,
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-800:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-800:]
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["config"]["roundtrip_ok"] is True
    assert line["scaling"] == ("strong" if "--total" in args else "weak")
    if "--total" in args:
        assert line["config"]["values_per_gpu"] == 4096

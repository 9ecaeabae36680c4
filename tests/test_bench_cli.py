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

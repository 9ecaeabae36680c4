"""bench.py's command line on CPU: the driver's contract flags and the
decode-only mode parse (no GPU work is started by --help)."""
import os
import subprocess
import sys

from tests.oracle_lib import ROOT


def test_bench_help_lists_contract_flags():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-500:]
    for flag in ("--gpus", "--steps", "--warmup", "--mode", "--workload"):
        assert flag in r.stdout
    assert "decompress" in r.stdout

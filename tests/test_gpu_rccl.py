"""The one-process-per-GPU deployment path on the MI355X: bench.py under torch.distributed.run with
the RCCL communicator (world size 1 on a one-GPU box: RCCL communicator creation, all-gather of
pivot records, RCCL all-reduce of the timing/residual maxima; broadcasts are rank-local)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_under_torchrun_with_rccl():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29657", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--size", "4096", "--force-rccl"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    rep = json.loads(line)
    assert rep["status"] == 0 and rep["n_gpus"] == 1
    assert rep["residual_inf"] < 1e-6
    assert rep["value"] > 0 and rep["ms_per_step"] > 0


def test_cli_with_rccl_communicator():
    """`gj --comm rccl`: the in-process (one host thread per GPU) RCCL path of the CLI."""
    gj = os.path.join(ROOT, "build", "gj")
    out = subprocess.run([gj, "--comm", "rccl", "--gen", "random", "--json", "2048", "128"], cwd=ROOT,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "glob_time:" in out.stdout and "residual:" in out.stdout
    rep = json.loads([l for l in out.stderr.splitlines() if l.startswith("{")][-1])
    assert rep["status"] == 0 and rep["comm"].startswith("rccl") and rep["residual"] < 1e-6

"""The driver's multi-GPU command, rehearsed on the CPU: `bench.py` itself under
`torch.distributed.run --nproc-per-node N` with `--device cpu` (native host executor, gloo
collectives), so the exact script the round driver launches on 8 GPUs runs here at world size 8.

Also the collective failure agreement of the reference (main.cpp:366-381, :428-436): an allocation
that fails on ONE rank makes every rank exit with status 2, without a hang."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _torchrun(nproc, *args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--device", "cpu", *args]
    return subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout)


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("nproc,bcast", [(8, "auto"), (8, "direct"), (3, "ring")])
def test_bench_script_world(nproc, bcast):
    r = _torchrun(nproc, "--steps", "2", "--warmup", "1", "--size", "200", "--block", "8",
                  "--bcast", bcast)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == nproc and d["steps"] == 2 and d["warmup"] == 1
    assert d["status"] == 0
    assert d["residual_inf"] < 1e-8
    assert d["config"]["bcast"] == ("direct" if bcast == "direct" else "ring")
    assert d["value"] > 0 and d["ms_per_step"] > 0


@pytest.mark.parametrize("stage,status", [("matrix", None), ("block", 7)])
def test_bench_alloc_failure_on_one_rank(stage, status):
    # rank 0 owns the extra block row when Nr % p != 0: exactly the rank that fails alone near the
    # HBM limit.  Every rank must leave with status 2 (no hang: the subprocess timeout would fire).
    r = _torchrun(4, "--steps", "1", "--warmup", "1", "--size", "90", "--block", "8",
                  env_extra={"GJ_TEST_ALLOC_FAIL": f"0:{stage}"}, timeout=180)
    assert r.returncode != 0
    for rank in range(4):
        assert f"bench.py: rank {rank}:" in r.stderr, r.stderr[-3000:]
    if status is None:
        assert "peer rank" in r.stderr and "injected" in r.stderr
    else:
        assert f"status {status}" in r.stderr
    assert "exitcode  : 2" in r.stderr or "exitcode: 2" in r.stderr.replace(" ", ""), r.stderr[-2000:]

"""The one-process-per-GPU deployment path on the MI355X: bench.py with the RCCL communicator.

* world size 1 under torch.distributed.run (RCCL communicator creation, all-gather of pivot
  records, all-reduce of the timing/residual maxima; broadcasts are rank-local);
* world size 2 / 3 on the one GPU (`--same-gpu`: every rank its own RCCL "host", connected by
  RCCL's socket transport): the engine's real RCCL schedule at p > 1 — grouped ncclBroadcast of
  pivot-row chunks (ring, or the direct scatter + exchange over ncclSend/ncclRecv), ncclAllGather
  of pivot records, the grouped point-to-point final exchange — must give the p = 1 inverse.
  (profiles/rccl_same_gpu_r3.md)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def _verify(monkeypatch):
    """Every RCCL run of this tier hashes each broadcast buffer where it is consumed and compares
    the ranks' hashes after the solve (GJ_VERIFY, Engine::verify_hashes)."""
    monkeypatch.setenv("GJ_VERIFY", "1")


def test_bench_under_torchrun_with_rccl():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", "29657", os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--steps", "1", "--warmup", "1", "--size", "4096", "--force-rccl"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
    rep = json.loads(line)
    assert rep["status"] == 0 and rep["n_gpus"] == 1
    assert isinstance(rep["rccl_transport"], dict)  # one rank: no channel connections to report
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


def _self_launch(*args, timeout=300):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.parametrize("ranks,bcast", [(2, "ring"), (3, "direct")])
def test_rccl_multi_rank_same_gpu(ranks, bcast):
    common = ("--steps", "1", "--warmup", "1", "--size", "2048", "--block", "128", "--comm-timeout", "60")
    one = _self_launch("--gpus", "1", "--force-rccl", *common)
    rep = _self_launch("--gpus", str(ranks), "--same-gpu", "--bcast", bcast, *common)
    assert rep["status"] == 0 and rep["ranks"] == ranks
    assert rep["comm"].startswith("rccl(") and rep["comm"].endswith(f"{ranks} ranks)")
    assert rep["config"]["bcast"] == ("direct" if ranks > 2 and bcast == "direct" else "ring")
    assert rep["residual_inf"] < 1e-6  # random 2048 x 2048: 2.7e-8
    assert abs(rep["residual_inf"] - one["residual_inf"]) <= 1e-3 * one["residual_inf"]
    assert len(rep["rank_solve_seconds_max"]) == ranks
    # the rehearsal's ranks are separate RCCL "hosts": RCCL must have connected them over sockets
    assert any(k.startswith("NET") for k in rep["rccl_transport"]), rep["rccl_transport"]


def test_rccl_one_comm_same_gpu_matches_two_comms():
    """The one-communicator schedule (GJ_ONE_COMM=1: SIDE and COMM collectives in one RCCL
    communicator, one issue order) gives the same inverse bits as the two-communicator run, and
    the p > 1 record carries its untimed profiled solve."""
    common = ("--gpus", "2", "--same-gpu", "--steps", "1", "--warmup", "1", "--size", "2048", "--block", "128",
              "--comm-timeout", "60")
    two = _self_launch(*common)
    os.environ["GJ_ONE_COMM"] = "1"
    try:
        one = _self_launch(*common)
    finally:
        os.environ.pop("GJ_ONE_COMM", None)
    assert two["comm_mode"]["one_comm"] is False and one["comm_mode"]["one_comm"] is True
    assert "one communicator" in one["comm"]
    assert one["residual_inf"] == two["residual_inf"] and one["residual_inf"] < 1e-6
    assert one["phases_ms_max"]["trailing_update"] > 0 and one["profiled_solve"]["timed"] is False


def _cli(nproc, *args, timeout=300):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env["PYTHONPATH"] = ROOT
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "--local-ranks-filter", "0",
           "-m", "mpi_jordan_crazy_acceleration_amd.cli", "--device", "gpu", "--comm-timeout", "60", *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-3000:]
    return [l for l in out.stdout.splitlines() if not l.startswith("glob_time")]


def test_torchrun_cli_two_ranks_same_gpu():
    """The user-facing torchrun CLI at p = 2 (torch's RCCL process group + the engine's two RCCL
    communicators, both ranks on GPU 0 as separate RCCL hosts): the reference's stdout contract
    with the p = 1 corners and a small residual."""
    one = _cli(1, "1024", "64")
    two = _cli(2, "--same-gpu", "1024", "64")
    assert two[:-1] == one[:-1]  # A and inverse corners (2 decimals), "inverse matrix:"
    r1, r2 = float(one[-1].split()[1]), float(two[-1].split()[1])
    assert two[-1].startswith("residual: ") and r2 < 1e-6 and r2 <= 10 * r1 + 1e-12


def test_hw_queue_shortfall_after_early_hip_init():
    """Deadlock-freedom of TWO communicators needs 16 hardware queues per process (README
    "Progress of the two communicators").  A program that initialises HIP through torch before it
    imports the package runs with HIP's default 4: both ranks must agree on the one-communicator
    schedule and then complete a real RCCL solve on those 4 queues (no refusal, no hang)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "_hwq_early_init.py")]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout + out.stderr[-3000:]
    for r in (0, 1):
        assert f"rank {r}: effective queues 4" in out.stdout, out.stdout + out.stderr[-2000:]
        assert f"rank {r}: one_comm True (rank(s) [0, 1] run with 4" in out.stdout, out.stdout
        assert f"rank {r}: status 0 residual" in out.stdout and "one communicator" in out.stdout, out.stdout

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


def _ranks(world, *args, env_extra=None, timeout=180):
    """bench.py as `world` independent processes (the environment torchrun would give them), so
    every rank's own exit status is observed (torchrun stops the others after the first failure)."""
    port = str(_free_port())
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port, OMP_NUM_THREADS="1", **(env_extra or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                                       "--device", "cpu", *args], cwd="/tmp", env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    out = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            out.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    return out


@pytest.mark.parametrize("stage,status", [("matrix", None), ("block", 7)])
def test_bench_alloc_failure_on_one_rank(stage, status):
    # rank 0 owns the extra block row when Nr % p != 0: exactly the rank that fails alone near the
    # HBM limit.  Every rank must exit with status 2 on its own (a hang would hit the timeout).
    out = _ranks(4, "--steps", "1", "--warmup", "1", "--size", "90", "--block", "8",
                 env_extra={"GJ_TEST_ALLOC_FAIL": f"0:{stage}"})
    for rank, (rc, o, e) in enumerate(out):
        assert rc == 2, (rank, rc, e[-2000:])
        assert f"bench.py: rank {rank}:" in e
        if status is None:
            assert ("injected" if rank == 0 else "peer rank") in e
        else:
            assert f"status {status}" in e


def _self_launch(nproc, *args, env_extra=None, timeout=240):
    """`python bench.py --gpus N` with no torchrun environment: bench.py starts its own ranks."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    env.setdefault("OMP_NUM_THREADS", "1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(nproc), "--device", "cpu", *args]
    return subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout)


def test_bench_self_launch_matches_torchrun():
    args = ("--steps", "2", "--warmup", "1", "--size", "200", "--block", "8", "--bcast", "direct")
    a = _self_launch(8, *args)
    assert a.returncode == 0, a.stderr[-3000:]
    b = _torchrun(8, *args)
    assert b.returncode == 0, b.stderr[-3000:]
    da, db = _json_line(a.stdout), _json_line(b.stdout)
    assert set(da) == set(db)
    for k in ("n_gpus", "ranks", "steps", "warmup", "status", "offdiag_pivots", "config", "policy", "comm"):
        assert da[k] == db[k], k
    assert da["n_gpus"] == 8 and da["ranks"] == 8
    assert da["residual_inf"] < 1e-8 and abs(da["residual_inf"] - db["residual_inf"]) < 1e-12
    assert len(da["rank_solve_seconds_max"]) == 8
    assert da["policy"]["depth"] == da["config"]["depth"]
    # achieved bandwidth per collective kind and rank, from the untimed profiled solve
    bw = da["comm_bandwidth"]["per_rank"]
    assert len(bw) == 8
    for r in bw:
        assert set(r) == {"pivot_rows", "panel_pieces", "pivot_records"}
        assert r["pivot_rows"]["bytes"] > 0 and r["pivot_records"]["calls"] > 0
        assert r["pivot_rows"]["GB_s"] is None or r["pivot_rows"]["GB_s"] > 0
    assert len(da["step_ms"]) == 2


def test_bench_self_launch_failure_exit_code():
    # one rank cannot allocate: the launcher's own exit status is the ranks' status 2
    r = _self_launch(3, "--steps", "1", "--warmup", "1", "--size", "90", "--block", "8",
                     env_extra={"GJ_TEST_ALLOC_FAIL": "1:matrix"})
    assert r.returncode == 2, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "rank exit codes [2, 2, 2]" in r.stderr


@pytest.mark.parametrize("launcher", ["self", "ranks"])
def test_bench_hang_fails_fast(launcher):
    """A rank that never joins the pivot exchange of step 3 (GJ_TEST_HANG): every rank exits
    non-zero within the communication timeout and names the step (reference: none; a hung MPI
    rank hangs the job)."""
    import time
    t0 = time.monotonic()
    args = ("--steps", "1", "--warmup", "1", "--size", "200", "--block", "8", "--comm-timeout", "6")
    env = {"GJ_TEST_HANG": "2:3"}
    if launcher == "self":
        r = _self_launch(4, *args, env_extra=env, timeout=120)
        assert r.returncode == 2, r.stderr[-3000:]
        errs = r.stderr
        for rank in range(4):
            assert f"bench.py: rank {rank}: rank {rank}/4, step 3 of 25" in errs, errs[-3000:]
    else:
        out = _ranks(4, *args, env_extra=env, timeout=120)
        for rank, (rc, o, e) in enumerate(out):
            assert rc == 2, (rank, rc, e[-2000:])
            assert f"rank {rank}/4, step 3 of 25, phase pivot search" in e, e[-2000:]
        assert "timed out after 6" in out[2][2]
    assert time.monotonic() - t0 < 90


def test_bench_wrong_inverse_fails():
    """A wrong inverse is a failure, not a fast success (reference: main.cpp:490-507 prints the
    residual, never fails on it).  GJ_TEST_CORRUPT=1:5 zeroes rank 1's copy of step 5's pivot row
    in one chunk: the run completes, the JSON line says residual_failed, every rank exits 2."""
    args = ("--steps", "1", "--warmup", "0", "--size", "200", "--block", "8")
    clean = _self_launch(4, *args)
    assert clean.returncode == 0, clean.stderr[-3000:]
    d = _json_line(clean.stdout)
    assert d["check"] == "residual_ok" and d["residual_inf"] < d["residual_bound"]
    bad = _self_launch(4, *args, env_extra={"GJ_TEST_CORRUPT": "1:5"})
    assert bad.returncode == 2, bad.stderr[-3000:]
    d = _json_line(bad.stdout)
    assert d["check"] == "residual_failed" and not d["residual_inf"] < d["residual_bound"]
    assert "rank exit codes [2, 2, 2, 2]" in bad.stderr
    assert "wrong inverse" in bad.stderr


def test_bench_gate_checks_a_timed_solve():
    """At p > 1 the bench runs one extra untimed solve with the phase timers after the timed loop
    (another schedule).  The residual gate must check a TIMED solve: here only the unprofiled
    solves are corrupted (GJ_TEST_CORRUPT=<rank>:<step>:unprofiled), the profiled one is clean,
    and the run must still fail."""
    args = ("--steps", "1", "--warmup", "0", "--size", "200", "--block", "8")
    bad = _self_launch(2, *args, env_extra={"GJ_TEST_CORRUPT": "1:5:unprofiled"})
    assert bad.returncode == 2, bad.stderr[-3000:]
    d = _json_line(bad.stdout)
    assert d["check"] == "residual_failed"
    assert "profiled_solve" in d  # the clean profiled solve did run after the gate's solve


def test_cli_check_residual(gj_bin):
    base = [gj_bin, "--device", "cpu", "-p", "3", "--gen", "random", "--check-residual", "1e-6", "200", "8"]
    assert subprocess.run(base, capture_output=True, text=True, timeout=120).returncode == 0
    r = subprocess.run(base, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, GJ_TEST_CORRUPT="0:2"))
    assert r.returncode == 2 and "residual check failed" in r.stderr, r.stderr
    assert "residual:" in r.stdout  # the reference's output is still printed in full


def test_bench_hw_queue_shortfall_degrades_to_one_comm():
    """One rank runs with too few hardware queues (HIP initialised before the package could raise
    GPU_MAX_HW_QUEUES; faked by GJ_TEST_HW_QUEUES=1:4): every rank agrees on the one-communicator
    schedule (parallel.dist.agree_comm_mode) and the run COMPLETES -- no refusal, no hang -- with
    the same residual bits as the two-communicator run; the JSON names the mode and its reason.
    Also the p > 1 record's extra untimed profiled solve (phases_ms_max, per-rank host waits)."""
    args = ("--steps", "1", "--warmup", "0", "--size", "90", "--block", "8")
    low = _ranks(4, *args, env_extra={"GJ_TEST_HW_QUEUES": "1:4"}, timeout=120)
    ok = _ranks(4, *args, timeout=120)
    for rank, (rc, o, e) in enumerate(low + ok):
        assert rc == 0, (rank, rc, e[-2000:])
    d_low, d_ok = _json_line(low[0][1]), _json_line(ok[0][1])
    assert d_low["comm_mode"]["one_comm"] is True and d_low["comm_mode"]["hw_queues"] == 4
    assert "rank(s) [1] run with 4 hardware queues" in d_low["comm_mode"]["reason"]
    assert d_ok["comm_mode"]["one_comm"] is False
    assert d_low["residual_inf"] == d_ok["residual_inf"] and d_low["residual_inf"] < 1e-8
    for d in (d_low, d_ok):
        assert d["profiled_solve"]["timed"] is False and len(d["profiled_solve"]["seconds_per_rank"]) == 4
        assert d["phases_ms_max"]["trailing_update"] > 0 and "pivot_search" in d["phases_ms_max"]


def test_one_comm_forced_by_env_on_any_rank():
    """GJ_ONE_COMM=1 on one rank is enough: the mode is agreed, so ranks never disagree on how many
    communicators to create (a collective)."""
    out = _ranks(3, "--steps", "1", "--warmup", "0", "--size", "60", "--block", "8",
                 env_extra={"GJ_ONE_COMM": "1"}, timeout=120)
    assert all(rc == 0 for rc, _, _ in out), [e[-1000:] for _, _, e in out]
    d = _json_line(out[0][1])
    assert d["comm_mode"]["one_comm"] is True and "GJ_ONE_COMM" in d["comm_mode"]["reason"]


def test_effective_hw_queues_after_early_hip_init():
    """The recorded queue count is the one HIP started with: a program that initialised HIP (here:
    faked by a torch whose cuda reports initialised) before the package keeps its old count."""
    code = (
        "import os, sys, types\n"
        "os.environ.pop('GPU_MAX_HW_QUEUES', None)\n"
        "fake = types.ModuleType('torch'); fake.cuda = types.SimpleNamespace(is_initialized=lambda: True)\n"
        "sys.modules['torch'] = fake\n"
        "sys.path.insert(0, %r)\n"
        "import importlib.util as u\n"
        "spec = u.spec_from_file_location('rt', %r); rt = u.module_from_spec(spec); spec.loader.exec_module(rt)\n"
        "rt.configure_runtime_env()\n"
        "print(rt.effective_hw_queues(), os.environ['GPU_MAX_HW_QUEUES'])\n"
    ) % (ROOT, os.path.join(ROOT, "mpi_jordan_crazy_acceleration_amd", "runtime_env.py"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.split() == ["4", "16"]

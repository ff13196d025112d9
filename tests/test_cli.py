"""`gj` CLI contract vs the reference's behaviour matrix, host backend."""
import os
import re
import subprocess

import numpy as np
import pytest

from mpi_jordan_crazy_acceleration_amd.utils import generate_matrix


def run(gj_bin, *args, cwd=None):
    p = subprocess.run([gj_bin, "--device", "cpu", *map(str, args)], capture_output=True, text=True,
                       cwd=cwd, timeout=120)
    return p.returncode, p.stdout, p.stderr


@pytest.mark.parametrize("args", [[], ["5"], ["0", "3"], ["5", "0"], ["4", "2", "a", "b"], ["abc", "2"], ["-5", "3"]])
def test_usage_errors(gj_bin, args):
    rc, out, _ = run(gj_bin, *args)
    assert rc == 1
    assert out == f"usage:{gj_bin} n m [<file>]\n"


def test_cannot_open(gj_bin, tmp_path):
    rc, out, _ = run(gj_bin, 5, 3, tmp_path / "nonexist.txt")
    assert rc == 2 and out == f"cannot open {tmp_path / 'nonexist.txt'}\n"


def test_cannot_read_short_file(gj_bin, tmp_path):
    f = tmp_path / "short.txt"
    f.write_text("1 2 3\n")
    rc, out, _ = run(gj_bin, 2, 1, f)
    assert rc == 2 and out == f"cannot read {f}\n"


def test_singular_zero_matrix(gj_bin, tmp_path):
    f = tmp_path / "zero.txt"
    f.write_text("0 0\n0 0\n")
    rc, out, _ = run(gj_bin, 2, 1, f)
    assert rc == 2
    assert out.endswith("singular matrix\n")
    assert out.startswith("A\n0.00\t0.00\t\n0.00\t0.00\t\n")


def test_two_by_two_exact_output(gj_bin, tmp_path):
    f = tmp_path / "two.txt"
    f.write_text("1 2\n3 4\n")
    rc, out, _ = run(gj_bin, 2, 1, f)
    assert rc == 0
    lines = out.split("\n")
    assert lines[0] == "A"
    assert lines[1] == "1.00\t2.00\t" and lines[2] == "3.00\t4.00\t"
    assert re.fullmatch(r"glob_time: \d+\.\d\d", lines[3])
    assert lines[4] == "inverse matrix:" and lines[5] == ""
    assert lines[6] == "-2.00\t1.00\t" and lines[7] == "1.50\t-0.50\t"
    assert re.fullmatch(r"residual: \d\.\d{6}e[+-]\d\d", lines[8])
    assert float(lines[8].split()[1]) < 1e-14
    assert lines[9] == ""


def test_default_generator_corner_and_residual(gj_bin):
    rc, out, _ = run(gj_bin, "-p", 3, 12, 3)
    assert rc == 0
    lines = out.split("\n")
    assert lines[1] == "".join(f"{abs(0 - j):.2f}\t" for j in range(10))
    res = float(out.strip().split("\n")[-1].split()[1])
    assert res < 5e-13  # reference: 4.56e-14 at p=3


def test_compat_residual_mode_prints_p_eq_1(gj_bin):
    rc, out, _ = run(gj_bin, "--residual", "compat", 12, 3)
    assert rc == 0 and out.endswith("p == 1!\n")
    rc, out, _ = run(gj_bin, "--residual", "compat", "-p", 2, 12, 3)
    assert rc == 0 and "residual:" in out


def test_hilbert_generator(gj_bin):
    rc, out, _ = run(gj_bin, "--gen", "hilbert", 8, 2)
    assert rc == 0
    assert float(out.strip().split("\n")[-1].split()[1]) < 1e-4  # reference: 3.7e-6


def test_file_input_matches_numpy_and_out_file(gj_bin, tmp_path):
    n = 23
    A = np.random.default_rng(4).standard_normal((n, n))
    f = tmp_path / "r.txt"
    np.savetxt(f, A, fmt="%.17g")
    out_f = tmp_path / "inv.txt"
    rc, out, err = run(gj_bin, "-p", 2, "--out", out_f, "--json", n, 4, f)
    assert rc == 0, err
    inv = np.loadtxt(out_f)
    assert np.abs(inv - np.linalg.inv(A)).max() < 1e-10
    assert '"status": 0' in err


def test_binary_input(gj_bin, tmp_path):
    n = 17
    A = generate_matrix(n, "random", 8)
    f = tmp_path / "a.bin"
    A.astype("<f8").tofile(f)
    out_f = tmp_path / "inv.bin"
    rc, out, _ = run(gj_bin, "--out", out_f, n, 5, f)
    assert rc == 0
    inv = np.fromfile(out_f, dtype="<f8").reshape(n, n)
    assert np.abs(inv - np.linalg.inv(A)).max() < 1e-10


def test_axb_plumbing_512(gj_bin, tmp_path):
    """BASELINE config 1: 512x512 random dense A x = b, one rank, CPU."""
    xf = tmp_path / "x.txt"
    rc, out, err = run(gj_bin, "--gen", "random", "--seed", 5, "--rhs", "random", "--out-x", xf, "--json", 512, 64)
    assert rc == 0, err
    assert "Ax-b residual:" in out
    res = float(out.strip().split("\n")[-1].split()[-1])
    assert res < 1e-9  # block Gauss-Jordan on a random 512 matrix: ~1e-10 (summation-order dependent)
    x = np.loadtxt(xf)
    A = generate_matrix(512, "random", 5)
    assert np.abs(A @ x).max() > 0
    assert '"axb_residual"' in err


def test_axb_rhs_file(gj_bin, tmp_path):
    n = 40
    A = generate_matrix(n, "random", 3)
    b = np.arange(n, dtype=float) - 7.5
    af, bf, xf = tmp_path / "a.txt", tmp_path / "b.txt", tmp_path / "x.bin"
    np.savetxt(af, A, fmt="%.17g")
    np.savetxt(bf, b, fmt="%.17g")
    rc, out, _ = run(gj_bin, "-p", 3, "--rhs", bf, "--out-x", xf, n, 6, af)
    assert rc == 0
    x = np.fromfile(xf, dtype="<f8")
    assert np.allclose(x, np.linalg.solve(A, b), rtol=1e-9, atol=1e-11)
    rc, out, _ = run(gj_bin, "--rhs", tmp_path / "missing.txt", n, 6, af)
    assert rc == 2 and out == f"cannot open {tmp_path / 'missing.txt'}\n"


def test_profile_json_phases(gj_bin):
    rc, out, err = run(gj_bin, "-p", 2, "--profile", "--json", 200, 16)
    assert rc == 0
    import json
    rep = json.loads(err.strip().split("\n")[-1])
    ph = rep["phases_ms"]
    assert set(ph) == {"column", "pivot_search", "pivot_exchange", "owner_edits", "panel_pieces",
                       "normalise_rows", "row_bcast", "trailing_update", "finalize"}
    assert ph["trailing_update"] > 0


@pytest.mark.parametrize("mode", ["ring", "direct"])
def test_bcast_flag(gj_bin, mode):
    # 4 virtual host ranks; every broadcast takes the chosen algorithm (GJ_BCAST_MIN=1 -> direct for
    # all sizes); the answer does not depend on it
    import os
    import subprocess

    env = dict(os.environ, GJ_BCAST_MIN="1")
    p = subprocess.run([str(gj_bin), "--device", "cpu", "--gpus", "4", "--bcast", mode, "--gen", "random",
                        "--residual", "always", "40", "6"], capture_output=True, text=True, env=env, timeout=120)
    assert p.returncode == 0, p.stderr
    assert float(p.stdout.strip().split("\n")[-1].split()[-1]) < 1e-10


def test_bcast_flag_rejects_unknown(gj_bin):
    rc, out, _ = run(gj_bin, "--bcast", "tree", 10, 3)
    assert rc == 1


def test_not_enough_memory_messages(gj_bin, monkeypatch):
    # the matrix itself (main.cpp:366-381): before any output; the work space (main.cpp:428-436):
    # after the A corner, like the reference's Jordan() failure
    monkeypatch.setenv("GJ_TEST_ALLOC_FAIL", "1:matrix")
    rc, out, _ = run(gj_bin, "-p", 3, 40, 8)
    assert rc == 2 and out == "Not enough memory!\n"
    monkeypatch.setenv("GJ_TEST_ALLOC_FAIL", "2:block")
    rc, out, _ = run(gj_bin, "-p", 3, 40, 8)
    assert rc == 2 and out.startswith("A\n") and out.endswith("not enough memory for block\n")


def test_fp32_refinement_json(gj_bin):
    import json
    rc, out, err = run(gj_bin, "--dtype", "fp32", "--gen", "randshift", "--rhs", "ones", "--refine", 5, "--json",
                       300, 16)
    assert rc == 0 and "Ax-b residual:" in out
    d = json.loads(err.strip().splitlines()[-1])
    assert d["residual_fp64"] is True and d["refine_converged"] is True
    assert d["axb_history"][-1] < 1e-12 and d["refine_steps"] >= 1

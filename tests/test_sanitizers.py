"""Host code under AddressSanitizer + UBSan: engine, loopback ranks, reader, CLI.

GPU sanitizers are not available on this platform; the device code is exercised by the GPU tests."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN_BIN = os.path.join(ROOT, "build", "gj_asan")


@pytest.fixture(scope="module")
def asan_bin():
    r = subprocess.run(["make", "-j8", "asan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        pytest.fail("asan build failed:\n" + r.stderr[-3000:])
    return ASAN_BIN


def _run(binary, *args):
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:detect_leaks=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    p = subprocess.run([binary, "--device", "cpu", *map(str, args)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert "ERROR: AddressSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "ERROR: LeakSanitizer" not in p.stderr, p.stderr[-4000:]
    assert "runtime error:" not in p.stderr, p.stderr[-4000:]
    return p


@pytest.mark.parametrize("args", [
    ("-p", 3, "--depth", 4, 200, 16),
    ("-p", 4, "--depth", 2, "--chunk-cols", 32, 150, 7),
    ("--gen", "random", "--rhs", "random", "--profile", "--json", 300, 64),
    ("-p", 5, 33, 10),            # more ranks than some block rows
    ("--dtype", "fp32", "-p", 2, 96, 12),
])
def test_asan_cli_runs(asan_bin, args):
    p = _run(asan_bin, *args)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    assert "residual:" in p.stdout


def test_asan_file_and_errors(asan_bin, tmp_path):
    f = tmp_path / "a.txt"
    np.savetxt(f, np.random.default_rng(0).standard_normal((50, 50)), fmt="%.17g")
    assert _run(asan_bin, "-p", 2, 50, 8, f).returncode == 0
    short = tmp_path / "s.txt"
    short.write_text("1 2 3")
    assert _run(asan_bin, 50, 8, short).returncode == 2
    z = tmp_path / "z.txt"
    z.write_text("0 0 0 0")
    assert _run(asan_bin, "-p", 2, 2, 1, z).returncode == 2  # singular

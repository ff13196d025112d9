"""Matrix file reader: the scanf("%lf") accept set (reference read_matrix, main.cpp:209-282)."""
import numpy as np
import pytest


def test_reader_accept_set(native, tmp_path):
    f = tmp_path / "m.txt"
    # hex floats, exponents, signs, tokens glued like "1.5-2" (scanf reads two numbers), tabs/newlines
    f.write_text("0x1p3 -2.5e0\t+3\n1.5-2   inf\n nan 7 8 9 trailing junk")
    A = native.read_matrix_file(str(f), 3)
    assert A[0, 0] == 8.0 and A[0, 1] == -2.5 and A[0, 2] == 3.0
    assert A[1, 0] == 1.5 and A[1, 1] == -2.0 and np.isinf(A[1, 2])
    assert np.isnan(A[2, 0]) and A[2, 1] == 7 and A[2, 2] == 8


def test_reader_errors(native, tmp_path):
    with pytest.raises(RuntimeError, match="cannot open"):
        native.read_matrix_file(str(tmp_path / "missing.txt"), 2)
    f = tmp_path / "bad.txt"
    f.write_text("1 2 x 4")
    with pytest.raises(RuntimeError, match="cannot read"):
        native.read_matrix_file(str(f), 2)
    g = tmp_path / "ok_after.txt"
    g.write_text("1 2 3 4 x")  # junk after the first n*n numbers is ignored
    assert native.read_matrix_file(str(g), 2).tolist() == [[1, 2], [3, 4]]


def test_reader_parallel_large(native, tmp_path):
    n = 400  # > 1 MiB of text -> multi-threaded chunked parse
    A = np.random.default_rng(0).standard_normal((n, n)) * 1e5
    f = tmp_path / "big.txt"
    np.savetxt(f, A, fmt="%.17g")
    assert f.stat().st_size > (1 << 20)
    B = native.read_matrix_file(str(f), n)
    assert np.array_equal(A, B)


def test_reader_rows_subset(native, tmp_path):
    # one rank's block rows (block-row-cyclic, m = 7, p = 3, rank 1), text and .bin, several threads
    n, m, p, k = 300, 7, 3, 1
    A = np.random.default_rng(1).standard_normal((n, n))
    f = tmp_path / "a.txt"
    np.savetxt(f, A, fmt="%.17g")
    rows = [r for r in range(n) if (r // m) % p == k]
    for nt in (1, 3, 8):
        B = native.read_matrix_rows(str(f), n, rows, nt)
        assert np.array_equal(B, A[rows])
    g = tmp_path / "a.bin"
    A.tofile(g)
    assert np.array_equal(native.read_matrix_rows(str(g), n, rows), A[rows])
    with pytest.raises(RuntimeError, match="cannot read"):
        native.read_matrix_rows(str(g), n + 1, [0])


@pytest.mark.parametrize("where", [0.3, 0.8])
def test_reader_bad_token_late_chunk(native, tmp_path, where):
    # > 1 MiB: chunked; an invalid token deep inside fails, an irregular glued pair ("1-2") before
    # it shifts every later index (exact sequential fallback), rows of another rank skip the check
    n = 400
    A = np.random.default_rng(2).standard_normal((n, n))
    toks = [f"{v:.17g}" for v in A.ravel()]
    bad = int(where * len(toks))
    toks_bad = list(toks)
    toks_bad[bad] = "zz"
    f = tmp_path / "bad.txt"
    f.write_text(" ".join(toks_bad))
    with pytest.raises(RuntimeError, match="cannot read"):
        native.read_matrix_file(str(f), n)
    # scanf stops at "zz" whichever rank keeps its row: every rank reports the failure
    r_bad = bad // n
    other = [r for r in range(n) if r != r_bad][:50]
    with pytest.raises(RuntimeError, match="cannot read"):
        native.read_matrix_rows(str(f), n, other)
    # irregular: tokens i and i+1 glued as "a-b" (b negative) -> same numbers, sequential scan
    i = next(j for j in range(bad // 2, len(toks) - 1) if toks[j + 1].startswith("-"))
    toks_irr = toks[:i] + [toks[i] + toks[i + 1]] + toks[i + 2:]
    g = tmp_path / "irr.txt"
    g.write_text(" ".join(toks_irr))
    assert np.array_equal(native.read_matrix_file(str(g), n), A)


@pytest.mark.parametrize("nt", [1, 4])
def test_reader_glued_token_outside_requested_rows(native, tmp_path, nt):
    # a glued "a-b" in a row another rank keeps shifts every later value under scanf;
    # a rank reading only OTHER rows must see the shift too (sequential fallback on every rank)
    n = 400
    A = np.random.default_rng(4).standard_normal((n, n))
    toks = [f"{v:.17g}" for v in A.ravel()]
    i = next(j for j in range(n * 10, len(toks) - 1) if toks[j + 1].startswith("-"))
    glued_row = i // n
    toks_irr = toks[:i] + [toks[i] + toks[i + 1]] + toks[i + 2:] + ["0.5"]
    g = tmp_path / "irr_other.txt"
    g.write_text(" ".join(toks_irr))
    later = [r for r in range(glued_row + 1, n, 7)]
    earlier = [r for r in range(0, glued_row, 3)]
    rows = earlier + later
    assert glued_row not in rows
    got = native.read_matrix_rows(str(g), n, rows, nt)
    assert np.array_equal(got, A[rows])

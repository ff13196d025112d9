"""Block-row-cyclic layout math vs the reference formulas (main.cpp:95-127, :521-532)."""
import itertools

import numpy as np

from mpi_jordan_crazy_acceleration_amd.parallel.layout import Layout, global_rows, last_owner, num_block_rows, rows_owned


def ref_rows_p_process(Nr, p, k):
    # main.cpp:101-116 literally
    sender = (Nr - 1) % p
    if Nr % p == 0:
        return Nr // p
    return Nr // p + 1 if k <= sender else Nr // p


def test_rows_owned_matches_reference():
    for Nr, p in itertools.product(range(1, 40), range(1, 10)):
        assert sum(rows_owned(Nr, p, k) for k in range(p)) == Nr
        for k in range(p):
            assert rows_owned(Nr, p, k) == ref_rows_p_process(Nr, p, k)


def test_last_owner_and_blocks():
    assert num_block_rows(10, 3) == 4
    assert num_block_rows(12, 3) == 4
    assert num_block_rows(10, 12) == 1
    assert last_owner(4, 3) == 0


def test_global_rows_partition():
    for n, m, p in [(10, 3, 2), (11, 4, 3), (37, 5, 4), (10, 12, 5), (64, 8, 8), (7, 1, 3)]:
        allr = np.concatenate([global_rows(n, m, p, k) for k in range(p)])
        assert sorted(allr.tolist()) == list(range(n))
        for k in range(p):
            L = Layout(n, m, p, k)
            g = global_rows(n, m, p, k)
            for i, gi in enumerate(g):
                assert L.global_row(i) == gi
                assert (gi // m) % p == k  # block row I lives on rank I mod p

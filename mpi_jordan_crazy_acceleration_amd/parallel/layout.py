"""Block-row-cyclic ownership math (Python mirror of csrc/include/gj/layout.hpp).

Reference: num_block_rows (main.cpp:124-127), rows_p_process (main.cpp:95-116),
find_sender (main.cpp:521-532), local_to_global (main.cpp:118-123).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


def num_block_rows(n: int, m: int) -> int:
    return (n + m - 1) // m


def rows_owned(Nr: int, p: int, k: int) -> int:
    return Nr // p + (1 if k < Nr % p else 0)


def last_owner(Nr: int, p: int) -> int:
    return (Nr - 1) % p


@dataclass(frozen=True)
class Layout:
    n: int
    m: int
    p: int = 1
    k: int = 0

    @property
    def Nr(self) -> int:
        return num_block_rows(self.n, self.m)

    @property
    def npad(self) -> int:
        return self.Nr * self.m

    @property
    def nblk(self) -> int:
        return rows_owned(self.Nr, self.p, self.k)

    def global_row(self, local_row: int) -> int:
        m, p, k = self.m, self.p, self.k
        return ((local_row // m) * p + k) * m + local_row % m


def global_rows(n: int, m: int, p: int, k: int) -> np.ndarray:
    """Global indices of the *real* rows rank k owns, in local storage order."""
    L = Layout(n, m, p, k)
    loc = np.arange(L.nblk * m)
    g = ((loc // m) * p + k) * m + loc % m
    return g[g < n]

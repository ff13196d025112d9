"""Distribution: block-row-cyclic layout math and the one-process-per-GPU engine driver."""
from .dist import DistributedGaussJordan, TorchDistComm  # noqa: F401
from .layout import Layout, global_rows, rows_owned  # noqa: F401

"""MI355X-native dense block Gauss-Jordan inversion framework.

Capabilities of ``yusupov1alik/MPI-Jordan-crazy-acceleration`` (an MPI/CPU block Gauss-Jordan
inverter, reference ``main.cpp``) re-designed for AMD Instinct MI355X (gfx950):

* native C++ engine (``csrc/solver``) driving hand-written CDNA4 HIP kernels (``csrc/kernels``):
  fp64/fp32 MFMA elimination GEMM, register-resident batched block inversion for the pivot search,
  look-ahead on a side stream, chunk-pipelined pivot-row broadcast;
* block-row-cyclic distribution over GPUs with RCCL over xGMI (one process per GPU through
  ``torch.distributed``, or one thread per GPU in the ``gj`` CLI);
* reference-compatible CLI ``build/gj n m [file]`` (stdout, file format, residual, exit codes).

Python entry points:

``inverse(A, block_size)``             invert a matrix (numpy / torch)          -> models.gauss_jordan
``solve(A, b, block_size)``            solve A x = b via the inverse             -> models.gauss_jordan
``run(n, m, ...)``                     the CLI flow in-process (report dict)     -> models.gauss_jordan
``DistributedGaussJordan``             one rank per process over torch.distributed -> parallel.dist
``ops``                                kernel-level wrappers (tests, profiling)
"""
from ._native import load_native, native_available, native_path  # noqa: F401
from .models.gauss_jordan import GaussJordan, inverse, run, solve  # noqa: F401
from .parallel.dist import DistributedGaussJordan  # noqa: F401

__version__ = "0.1.0"

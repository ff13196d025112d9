"""Helper of tests/test_gpu_rccl.py::test_hw_queue_shortfall_after_early_hip_init (run by torchrun,
two ranks on GPU 0): HIP is initialised by torch BEFORE the package is imported, with
GPU_MAX_HW_QUEUES unset (HIP's default, 4 queues).  The package must notice that it is too late to
raise it, and the hardware-queue agreement must fail on every rank with the same message, before
any RCCL communicator is created."""
import os
import sys

os.environ.pop("GPU_MAX_HW_QUEUES", None)
import torch  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")  # HIP initialised here, with the default queue count
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mpi_jordan_crazy_acceleration_amd.parallel.dist import agree_hw_queues  # noqa: E402
from mpi_jordan_crazy_acceleration_amd.runtime_env import effective_hw_queues  # noqa: E402

print(f"rank {dist.get_rank()}: effective queues {effective_hw_queues()}", flush=True)
try:
    agree_hw_queues()
except RuntimeError as e:
    print(f"rank {dist.get_rank()}: refused: {e}", flush=True)
    dist.destroy_process_group()
    sys.exit(3)
print(f"rank {dist.get_rank()}: accepted", flush=True)
dist.destroy_process_group()

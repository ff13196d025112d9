"""Helper of tests/test_gpu_rccl.py::test_hw_queue_shortfall_after_early_hip_init (run by torchrun,
two ranks on GPU 0): HIP is initialised by torch BEFORE the package is imported, with
GPU_MAX_HW_QUEUES unset (HIP's default, 4 queues).  The package must notice that it is too late to
raise it, every rank must agree on the one-communicator schedule before any RCCL communicator is
created, and a real RCCL solve must then complete on those 4 queues (ranks sharing GPU 0 connect
as separate "hosts" over loopback sockets, as bench.py --same-gpu)."""
import os
import sys

os.environ.pop("GPU_MAX_HW_QUEUES", None)
rank = int(os.environ["RANK"])
os.environ["NCCL_HOSTID"] = f"gj-hwq-rank{rank}"
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
os.environ.setdefault("NCCL_IB_DISABLE", "1")
import torch  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")  # HIP initialised here, with the default queue count
import torch.distributed as dist  # noqa: E402

dist.init_process_group("gloo")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import mpi_jordan_crazy_acceleration_amd as gj  # noqa: E402
from mpi_jordan_crazy_acceleration_amd.parallel.dist import agree_comm_mode  # noqa: E402
from mpi_jordan_crazy_acceleration_amd.runtime_env import effective_hw_queues  # noqa: E402

print(f"rank {rank}: effective queues {effective_hw_queues()}", flush=True)
mode = agree_comm_mode()
print(f"rank {rank}: one_comm {mode['one_comm']} ({mode['reason']})", flush=True)
C = gj.load_native()
ids = [[C.rccl_unique_id(), C.rccl_unique_id()] if rank == 0 else None]
dist.broadcast_object_list(ids, src=0)
comm = C.rccl_comm(ids[0], 2, rank, 0, one_comm=mode["one_comm"])
eng = C.Engine(C.hip_device(0), comm, 512, 64, "fp64", comm_timeout_s=60.0)
eng.generate("random", 5)
st = eng.solve()
norm_a, norm_inv = eng.input_norm_inf(), eng.result_norm_inf()
res = eng.residual_generated("random", 5)
print(f"rank {rank}: status {st['status']} residual {res:.3e} comm {eng.policy['comm']}", flush=True)
dist.destroy_process_group()
from mpi_jordan_crazy_acceleration_amd.utils.metrics import residual_ok  # noqa: E402

sys.exit(0 if st["status"] == 0 and residual_ok(res, 512, norm_a, norm_inv) else 4)

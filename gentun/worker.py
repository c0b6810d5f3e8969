"""Reference module path ``gentun.worker`` (gentun/worker.py): a worker is an
evaluator rank of the RCCL process group (gentun_amd.parallel.distributed)."""
from gentun_amd.parallel.distributed import GentunWorker  # noqa: F401

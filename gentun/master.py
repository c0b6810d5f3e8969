"""Reference module path ``gentun.master`` (gentun/master.py): the RabbitMQ
master becomes rank 0 of an RCCL process group (gentun_amd.parallel.distributed)."""
from gentun_amd.parallel.distributed import DistributedPopulation, DistributedGridPopulation  # noqa: F401

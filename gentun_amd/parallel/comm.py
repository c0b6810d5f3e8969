"""Communicators for population-level parallelism.

Replaces the reference's RabbitMQ/pika RPC (gentun/master.py:17-129,
gentun/worker.py:13-66) with collectives:

* :class:`DistComm` -- ``torch.distributed`` process group, one rank per GPU.
  Backend ``"nccl"`` is RCCL on ROCm and runs over xGMI between the 8
  MI355X of a node; ``"gloo"`` is used for CPU-only runs and CPU tests.
  Per-generation traffic is < 2 KB (SURVEY.md §2.5 "Sizing on xGMI"), so the
  exchange is latency-bound: one broadcast of the genome table and one
  all_gather of fold scores, both tiny device tensors.
* :class:`ThreadComm` -- in-process test double with the same interface
  (ranks are threads, collectives rendezvous through a barrier). It is not
  a second backend: production code paths only see ``DistComm``.
"""

import datetime
import os
import threading

import numpy as np
import torch


class Communicator(object):
    rank = 0
    world_size = 1

    def broadcast_array(self, arr, src=0):
        """Broadcast a numpy array from ``src`` (shape/dtype need not be known
        by receivers; pass ``None`` there)."""
        raise NotImplementedError

    def all_gather_array(self, arr):
        """Return a list of every rank's array (same shape on every rank)."""
        raise NotImplementedError

    def barrier(self):
        raise NotImplementedError

    def ticket(self, key):
        """Atomic fetch-and-increment of a job-wide counter named ``key``
        (0, 1, 2, ... across all ranks): the work-stealing queue of dynamic
        scheduling."""
        raise NotImplementedError

    def is_master(self):
        return self.rank == 0


class LocalComm(Communicator):
    """world_size == 1."""

    def __init__(self):
        self._tickets = {}

    def broadcast_array(self, arr, src=0):
        return np.array(arr, copy=True)

    def all_gather_array(self, arr):
        return [np.array(arr, copy=True)]

    def barrier(self):
        return None

    def ticket(self, key):
        v = self._tickets.get(key, 0)
        self._tickets[key] = v + 1
        return v


_DTYPES = [np.float64, np.float32, np.int64, np.int32, np.uint8]


def _attempt_store(timeout):
    """Under torchrun's static rendezvous the agent's TCPStore outlives a
    restart (``--max-restarts``); this returns that store under the key
    prefix ``gentun/attempt_<TORCHELASTIC_RESTART_COUNT>`` (None outside
    torchrun), so a restarted group never meets keys of the attempt before.

    torch 2.10's env rendezvous opens a fresh agent-store client per attempt
    as well, but measured here that is not enough for our restart path: with
    this function disabled (round 3), tests/test_dead_rank.py's killed / hung
    rank restarts hang until the test timeout instead of resuming, so the
    prefix stays."""
    import torch.distributed as dist
    if os.environ.get("TORCHELASTIC_USE_AGENT_STORE") != "True" or "TORCHELASTIC_RESTART_COUNT" not in os.environ:
        return None
    base = dist.TCPStore(os.environ["MASTER_ADDR"], int(os.environ["MASTER_PORT"]),
                         int(os.environ["WORLD_SIZE"]), is_master=False, timeout=timeout)
    return dist.PrefixStore("gentun/attempt_{}".format(os.environ["TORCHELASTIC_RESTART_COUNT"]), base)


class DistComm(Communicator):
    """``torch.distributed`` collectives on small numpy arrays.

    With the ``nccl`` (RCCL) backend arrays travel as device tensors on this
    rank's GPU; with ``gloo`` as CPU tensors. Headers (dtype, ndim, shape)
    are broadcast as a fixed 8-int64 vector first so receivers need no
    out-of-band shape knowledge.
    """

    def __init__(self, backend=None, timeout_s=1800, init=True, device=None):
        import torch.distributed as dist
        self.dist = dist
        if init and not dist.is_initialized():
            if backend is None:
                backend = "nccl" if torch.cuda.is_available() else "gloo"
            kwargs = {"backend": backend, "timeout": datetime.timedelta(seconds=timeout_s)}
            if backend == "nccl" and device is not None:
                kwargs["device_id"] = torch.device(device)
            store = _attempt_store(kwargs["timeout"])
            if store is not None:
                kwargs.update(store=store, rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
            dist.init_process_group(**kwargs)
        self.backend = dist.get_backend()
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        if self.backend == "nccl":
            self.device = torch.device(device) if device is not None else \
                torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")

    def _t(self, arr):
        return torch.from_numpy(np.ascontiguousarray(arr)).to(self.device)

    def broadcast_array(self, arr, src=0):
        hdr = np.zeros(8, np.int64)
        if self.rank == src:
            arr = np.ascontiguousarray(arr)
            code = [i for i, d in enumerate(_DTYPES) if np.dtype(d) == arr.dtype]
            if not code:
                raise TypeError("unsupported dtype {}".format(arr.dtype))
            if arr.ndim > 6:
                raise ValueError("at most 6 dims")
            hdr[0] = code[0]
            hdr[1] = arr.ndim
            hdr[2:2 + arr.ndim] = arr.shape
        th = self._t(hdr)
        self.dist.broadcast(th, src=src)
        hdr = th.cpu().numpy()
        dtype = _DTYPES[int(hdr[0])]
        shape = tuple(int(s) for s in hdr[2:2 + int(hdr[1])])
        if self.rank == src:
            payload = self._t(arr.astype(dtype, copy=False))
        else:
            payload = torch.empty(shape, dtype=torch.from_numpy(np.zeros(0, dtype)).dtype, device=self.device)
        if payload.numel():
            self.dist.broadcast(payload, src=src)
        return payload.cpu().numpy()

    def all_gather_array(self, arr):
        t = self._t(arr)
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        self.dist.all_gather(out, t)
        return [o.cpu().numpy() for o in out]

    def barrier(self):
        if self.backend == "nccl":
            self.dist.barrier(device_ids=[self.device.index])
        else:
            self.dist.barrier()

    def ticket(self, key):
        # the rendezvous TCPStore of the process group: one round trip to the
        # store host (rank 0's node), no collective, ranks proceed independently
        store = self.dist.distributed_c10d._get_default_store()
        return int(store.add("gentun/" + key, 1)) - 1

    def destroy(self):
        if self.dist.is_initialized():
            self.dist.destroy_process_group()


class _ThreadHub(object):
    def __init__(self, world_size, timeout_s):
        self.world_size = world_size
        self.timeout_s = timeout_s
        self.barrier = threading.Barrier(world_size, timeout=timeout_s)
        self.slots = [None] * world_size
        self.lock = threading.Lock()
        self.tickets = {}


class ThreadComm(Communicator):
    """Test double: ranks are threads sharing a :class:`_ThreadHub`."""

    def __init__(self, hub, rank):
        self.hub = hub
        self.rank = rank
        self.world_size = hub.world_size

    @staticmethod
    def group(world_size, timeout_s=60.0):
        hub = _ThreadHub(world_size, timeout_s)
        return [ThreadComm(hub, r) for r in range(world_size)]

    def _exchange(self, value):
        self.hub.slots[self.rank] = value
        self.hub.barrier.wait()
        vals = list(self.hub.slots)
        self.hub.barrier.wait()
        return vals

    def broadcast_array(self, arr, src=0):
        vals = self._exchange(np.array(arr, copy=True) if self.rank == src else None)
        return np.array(vals[src], copy=True)

    def all_gather_array(self, arr):
        return [np.array(v, copy=True) for v in self._exchange(np.array(arr, copy=True))]

    def barrier(self):
        self.hub.barrier.wait()

    def ticket(self, key):
        with self.hub.lock:
            v = self.hub.tickets.get(key, 0)
            self.hub.tickets[key] = v + 1
            return v


def from_env(backend=None, timeout_s=None, device=None):
    """DistComm when launched by torchrun (``WORLD_SIZE`` > 1), else LocalComm."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return LocalComm()
    if timeout_s is None:
        timeout_s = int(os.environ.get("GENTUN_COLLECTIVE_TIMEOUT_S", "1800"))
    return DistComm(backend=backend, timeout_s=timeout_s, device=device)

"""Population-level parallelism: communicators, scheduler, evaluators, master/worker."""

from .comm import Communicator, DistComm, LocalComm, ThreadComm, from_env  # noqa: F401
from .evaluators import LocalBatchEvaluator, SequentialEvaluator  # noqa: F401
from .scheduler import lpt_assign, make_units  # noqa: F401
from .distributed import (DistributedGridPopulation, DistributedPopulation, GenomeCodec,  # noqa: F401
                          GentunWorker)

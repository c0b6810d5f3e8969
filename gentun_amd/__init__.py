"""gentun_amd -- MI355X-native distributed genetic-algorithm search engine.

Same public API as the reference package (gentun/__init__.py:2-19):
``GeneticAlgorithm, RussianRouletteGA, Population, GridPopulation,
DistributedPopulation, DistributedGridPopulation, GentunWorker,
XgboostIndividual, XgboostModel, GeneticCnnIndividual, GeneticCnnModel``.

Unlike the reference, the model classes never degrade to a printed warning:
the GBDT engine is native C++/HIP code built in-tree and the Genetic-CNN
model runs on PyTorch-ROCm + hand-written HIP kernels; both are importable
whenever the package is.
"""

from .algorithms import GeneticAlgorithm, RussianRouletteGA
from .populations import Population, GridPopulation
from .individuals import Individual, XgboostIndividual, GeneticCnnIndividual, random_log_uniform
from .parallel.distributed import DistributedPopulation, DistributedGridPopulation, GentunWorker
from .parallel.evaluators import LocalBatchEvaluator, SequentialEvaluator
from .models.cnn import GeneticCnnModel
from .models.xgboost_models import XgboostModel
from .utils.rng import seed as set_seed

__version__ = "0.1.0"

__all__ = [
    "GeneticAlgorithm", "RussianRouletteGA", "Population", "GridPopulation", "DistributedPopulation",
    "DistributedGridPopulation", "GentunWorker", "Individual", "XgboostIndividual", "XgboostModel",
    "GeneticCnnIndividual", "GeneticCnnModel", "LocalBatchEvaluator", "SequentialEvaluator",
    "random_log_uniform", "set_seed",
]

"""Fitness models: Genetic-CNN (HIP kernels on MI355X) and GBDT (native C++/HIP engine)."""

from .generic_models import GentunModel  # noqa: F401

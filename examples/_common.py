"""Shared helpers of the example drivers (the reference's tests/*.py scripts)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))


def wine():
    """White-wine-quality regression fixture (reference tests/data/winequality-white.csv)."""
    from gentun_amd.utils.data import load_wine_quality
    return load_wine_quality()


def mnist_like(n=10000, seed=0):
    """10k 28x28x1 one-hot samples standing in for the reference's MNIST
    subsample (``fetch_mldata`` is gone and there is no network)."""
    from gentun_amd.utils.data import make_mnist_like
    return make_mnist_like(n=n, seed=seed)

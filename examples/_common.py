"""Shared helpers of the example drivers (the reference's tests/*.py scripts)."""
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

# GENTUN_EXAMPLE_SMALL=1: CI-sized run of the same script (tests/test_examples.py)
SMALL = os.environ.get("GENTUN_EXAMPLE_SMALL") == "1"


def wine():
    """White-wine-quality regression fixture (vendored tests/data/winequality-white.csv)."""
    from gentun_amd.utils.data import load_wine_quality
    x, y = load_wine_quality()
    return (x[:600], y[:600]) if SMALL else (x, y)


def mnist_like(n=10000, seed=0):
    """10k 28x28x1 one-hot samples standing in for the reference's MNIST
    subsample (``fetch_mldata`` is gone and there is no network)."""
    from gentun_amd.utils.data import make_mnist_like
    return make_mnist_like(n=240 if SMALL else n, seed=seed)


def cnn_schedule(epochs=(20, 4, 1), learning_rate=(1e-3, 1e-4, 1e-5), nfold=5):
    """The reference schedule, or a one-epoch two-fold one in small mode."""
    if SMALL:
        return {'nfold': 2, 'epochs': (1,), 'learning_rate': (1e-3,)}
    return {'nfold': nfold, 'epochs': epochs, 'learning_rate': learning_rate}

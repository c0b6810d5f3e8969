"""Reference module path ``gentun.algorithms`` (gentun/algorithms.py)."""
from gentun_amd.algorithms import GeneticAlgorithm, RussianRouletteGA  # noqa: F401

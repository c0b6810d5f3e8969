"""Reference module path ``gentun.populations`` (gentun/populations.py)."""
from gentun_amd.populations import Population, GridPopulation  # noqa: F401

"""Reference module path ``gentun.individuals`` (gentun/individuals.py)."""
from gentun_amd.individuals import (Individual, XgboostIndividual, GeneticCnnIndividual,  # noqa: F401
                                    random_log_uniform)

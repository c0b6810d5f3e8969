"""Reference module path ``gentun.models.keras_models``: the Keras/TF model is
the MI355X Genetic-CNN engine (gentun_amd.models.cnn)."""
from gentun_amd.models.cnn import GeneticCnnModel  # noqa: F401

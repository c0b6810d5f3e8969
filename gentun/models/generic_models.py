"""Reference module path ``gentun.models.generic_models``."""
from gentun_amd.models.generic_models import GentunModel  # noqa: F401

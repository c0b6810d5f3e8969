"""Reference module path ``gentun.models.xgboost_models``: xgb.cv is the native
C++ / HIP GBDT engine (gentun_amd.models.gbdt)."""
from gentun_amd.models.xgboost_models import XgboostModel  # noqa: F401

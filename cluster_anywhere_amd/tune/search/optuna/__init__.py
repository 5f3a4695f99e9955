"""``ray.tune.search.optuna`` import path; the searcher is native (model_based.py)."""
from ..model_based import OptunaSearch

__all__ = ["OptunaSearch"]

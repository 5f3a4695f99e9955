"""``ray.tune.search.hyperopt`` import path; the searcher is native (model_based.py)."""
from ..model_based import HyperOptSearch

__all__ = ["HyperOptSearch"]

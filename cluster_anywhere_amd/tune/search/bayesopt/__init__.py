"""``ray.tune.search.bayesopt`` import path; the searcher is native (model_based.py)."""
from ..model_based import BayesOptSearch

__all__ = ["BayesOptSearch"]

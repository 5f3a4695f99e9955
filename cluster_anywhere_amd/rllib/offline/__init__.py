"""Offline RL I/O: episode recording (``config.offline_data(output=...)``), streaming
offline input for BC / MARWIL / CQL (``OfflineData`` / ``OfflinePreLearner``) and
off-policy estimators (``config.evaluation(off_policy_estimation_methods=...)``).
Reference: ``rllib/offline/``."""
from .estimators import (DirectMethod, DoublyRobust, FQETorchModel, ImportanceSampling, OffPolicyEstimator,
                         WeightedImportanceSampling, make_estimator)
from .io import COLUMNS, EpisodeRecorder
from .offline_data import OfflineData, OfflinePreLearner, discounted_returns

__all__ = ["OfflineData", "OfflinePreLearner", "EpisodeRecorder", "COLUMNS", "OffPolicyEstimator",
           "ImportanceSampling", "WeightedImportanceSampling", "DirectMethod", "DoublyRobust", "FQETorchModel",
           "make_estimator", "discounted_returns"]

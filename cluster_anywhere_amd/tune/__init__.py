"""Hyperparameter tuning (reference: python/ray/tune/__init__.py)."""
from ..train.checkpoint import Checkpoint
from ..train.config import CheckpointConfig, FailureConfig, RunConfig
from .callback import Callback, CLIReporter, CSVLoggerCallback, JsonLoggerCallback, LoggerCallback, ProgressReporter
from .controller import Trial
from .schedulers import (PB2, AsyncHyperBandScheduler, ASHAScheduler, DistributeResources, FIFOScheduler,
                         HyperBandForBOHB, HyperBandScheduler, MedianStoppingRule, PopulationBasedTraining,
                         PopulationBasedTrainingReplay,
                         ResourceChangingScheduler, TrialScheduler)
from .search.bohb import TuneBOHB
from .search.model_based import BayesOptSearch, HyperOptSearch, OptunaSearch
from .search import (BasicVariantGenerator, ConcurrencyLimiter, RandomLocalSearch, Repeater, Searcher,
                     choice, grid_search, lograndint, loguniform, qlograndint, qloguniform, qrandint, qrandn,
                     quniform, randint, randn, sample_from, uniform)
from .session import get_checkpoint, get_context, get_trial_dir, get_trial_id, get_trial_resources, report
from .stopper import (CombinedStopper, ExperimentPlateauStopper, FunctionStopper, MaximumIterationStopper,
                      Stopper, TimeoutStopper, TrialPlateauStopper)
from .trainable import PlacementGroupFactory, Trainable, with_parameters, with_resources
from .tuner import ExperimentAnalysis, ResultGrid, TuneConfig, Tuner, run

from .registry import (Experiment, ResumeConfig, create_scheduler, create_searcher, register_env,
                       register_trainable, run_experiments)
from ..train.trainer import Result
from ..train.session import TrainContext as TuneContext

JupyterNotebookReporter = CLIReporter
TuneError = RuntimeError

__all__ = [n for n in dir() if not n.startswith("_")]

"""ConnectorV2 pipelines (reference role: rllib/connectors/)."""
from .connector_v2 import ConnectorPipelineV2, ConnectorV2, build_pipeline
from .env_to_module import FlattenObservations, FrameStackingEnvToModule, MeanStdFilter, PrevActionsPrevRewards
from .learner import ChunkSequences, FlattenTimeMajor, GeneralAdvantageEstimation, NumpyToTensor
from .module_to_env import GetActions, NormalizeAndClipActions

__all__ = ["ConnectorV2", "ConnectorPipelineV2", "build_pipeline", "FlattenObservations", "MeanStdFilter",
           "FrameStackingEnvToModule", "PrevActionsPrevRewards", "NumpyToTensor", "GeneralAdvantageEstimation",
           "FlattenTimeMajor", "ChunkSequences", "NormalizeAndClipActions", "GetActions"]

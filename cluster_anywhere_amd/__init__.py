"""cluster_anywhere_amd — an MI355X-native distributed AI runtime with Ray's
capabilities (tasks / actors / objects, Train, Data, Tune, Serve, RLlib),
built on PyTorch-ROCm, hand-written gfx950 HIP kernels and RCCL over xGMI.

``import cluster_anywhere_amd as ray`` gives the familiar API surface.
"""
__version__ = "0.1.0"

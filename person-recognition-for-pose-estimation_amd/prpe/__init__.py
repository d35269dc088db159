"""prpe — MI355X-native (gfx950) per-frame inference hot path of the
Person-Recognition-for-Pose-Estimation combined multi-task model.

    from prpe import CombinedModel, non_max_suppression, keypoints_from_heatmaps

Device work: hand-written HIP kernels in ../csrc behind the C ABI of include/prpe.h
(libprpe.so, loaded by prpe._lib). PyTorch-ROCm supplies device memory, streams and
torch.distributed (RCCL) only.
"""
from .arch import TASKS, state_dict_spec  # noqa: F401
from .model import CombinedModel, PoseOutput  # noqa: F401
from .postproc import keypoints_from_heatmaps, non_max_suppression, non_max_suppression_padded  # noqa: F401

__all__ = ["CombinedModel", "PoseOutput", "non_max_suppression", "non_max_suppression_padded",
           "keypoints_from_heatmaps", "state_dict_spec", "TASKS"]

"""orb_slam_fusion_amd -- MI355X (gfx950) ORB front-end and pose optimisation.

Drop-in for the hot path of J094/orb_slam_fusion:
``ORB_SLAM_FUSION::OrbExtractor::operator()``, ``Optimizer::PoseOptimization``,
``Optimizer::LocalBundleAdjustment``, ``Frame::ComputeStereoMatches`` and the
``ORBmatcher::SearchByProjection`` searches of tracking and DBoW2's
``transform`` (Frame / KeyFrame ``ComputeBoW``).  The compute runs in hand-written HIP kernels
(csrc/*.hip) behind the C ABI of include/orbgpu.h; this package is the host
mirror of the reference interface over that ABI.
"""
from ._lib import KEYPOINT_DTYPE, POSE_OBS_DTYPE, OrbGpuError, library_path
from .extractor import OrbExtractor
from .lba import LocalBundleAdjuster
from .matcher import MatchFrame, ORBmatcher
from .vocab import ORBVocabulary
from .optimizer import PoseFrame, PoseOptimizer
from .stereo import compute_stereo_matches

__all__ = [
    "LocalBundleAdjuster",
    "MatchFrame",
    "ORBmatcher",
    "ORBVocabulary",
    "KEYPOINT_DTYPE",
    "POSE_OBS_DTYPE",
    "OrbGpuError",
    "OrbExtractor",
    "PoseFrame",
    "PoseOptimizer",
    "compute_stereo_matches",
    "library_path",
]

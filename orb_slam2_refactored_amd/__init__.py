"""MI355X-native ORB-SLAM2 hot path: ORB front end + local bundle adjustment on gfx950.

Host mirrors of the reference's interfaces (tiantianxuabc/ORB_SLAM2_Refactored):
  ORBextractor        <- include/ORBextractor.h
  ORBmatcher          <- include/ORBmatcher.h (Hamming kernels)
  Optimizer.LocalBundleAdjustment <- include/Optimizer.h:47
  Optimizer.PoseOptimization      <- include/Optimizer.h:49
All compute runs in liborbslam2_amd.so (HIP kernels behind include/orbslam2_amd.h).
"""
from .extractor import ORBextractor, KP_DTYPE
from .matcher import ORBmatcher, ComputeStereoMatches
from . import optimizer
from .synth import synth_image, shifted_pair, stereo_pair, make_pose_batch

__all__ = ["ORBextractor", "ORBmatcher", "ComputeStereoMatches", "optimizer", "KP_DTYPE", "synth_image", "shifted_pair", "stereo_pair", "make_pose_batch"]

"""MI355X-native back end for the census / CBCA / SGM / WTA stereo pipeline of
xinge456/myStereoMatching (stereoMatching.cpp), behind the reference's StereoMatching API.

Compute lives in libsm_hip.so (hand-written gfx950 HIP kernels behind the C-ABI of
include/sm_capi.h).  This package holds the host-side mirror of the reference interface.
"""
from .stereo_matching import SolveAll, StereoBatch, StereoMatching, pyrDown, run_batch_multi  # noqa: F401

__all__ = ["StereoMatching", "SolveAll", "StereoBatch", "pyrDown", "run_batch_multi"]

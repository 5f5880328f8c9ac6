"""bad-t evaluator of the reference (calErr, stereoMatching.h:1748-1825).

A pixel counts when mask == 255; it is an error when DP < 0 or |DT - DP| > t.  The reference
reports t = errorThreshold = 1 (h:225); BASELINE.json asks for t = 2 as well.  RMS follows the
reference: the float sum adds pow(dif, 2) per valid pixel and 2 per invalid one, in raster order
— evaluated by sm_cal_err in libsm_hip.so with exactly that arithmetic.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi

REGIONS = ("nonocc", "all", "disc")   # I_mask order (cpp:2073-2075)


def cal_err(DP: np.ndarray, DT: np.ndarray, mask: np.ndarray, thres: float = 1.0):
    """Return (PBM, RMS) over mask == 255 (one region of calErr)."""
    dp = np.ascontiguousarray(DP, np.int16)
    dt = np.ascontiguousarray(DT, np.float32)
    m = np.ascontiguousarray(mask, np.uint8)
    if not (dp.shape == dt.shape == m.shape) or dp.ndim != 2:
        raise ValueError("DP, DT and mask must be H x W arrays of one shape")
    lib = _capi.load()
    pbm, rms = C.c_float(), C.c_float()
    st = lib.sm_cal_err(_capi.ptr(dp), _capi.ptr(dt), _capi.ptr(m), dp.shape[0], dp.shape[1], float(thres),
                        C.byref(pbm), C.byref(rms))
    _capi.check(lib, None, st, "sm_cal_err")
    return float(pbm.value), float(rms.value)


def cal_err_regions(DP, DT, masks: dict, thres: float = 1.0) -> dict:
    """calErr over every available region: {region: (PBM, RMS)} (h:1760-1799)."""
    return {r: cal_err(DP, DT, masks[r], thres) for r in REGIONS if masks.get(r) is not None}

"""bad-t evaluator of the reference (calErr, stereoMatching.h:1748-1825), vectorised in numpy.

A pixel counts when mask == 255; it is an error when DP < 0 or |DT - DP| > t.  The reference
reports t = errorThreshold = 1 (h:225); BASELINE.json asks for t = 2 as well.
RMS follows the reference: invalid pixels add 2 to the squared-error sum.
"""
from __future__ import annotations

import numpy as np


def cal_err(DP: np.ndarray, DT: np.ndarray, mask: np.ndarray, thres: float = 1.0):
    """Return (PBM, RMS) over mask == 255."""
    m = np.asarray(mask) == 255
    n = int(m.sum())
    if n == 0:
        return 0.0, 0.0
    dp = np.asarray(DP)[m].astype(np.float32)
    dt = np.asarray(DT, np.float32)[m]
    valid = dp >= 0
    dif = np.abs(dt - dp)
    err = int((~valid).sum() + ((dif > thres) & valid).sum())
    sq = float(np.sum((dif[valid].astype(np.float64)) ** 2)) + 2.0 * float((~valid).sum())
    return err / n, float(np.sqrt(sq / n))

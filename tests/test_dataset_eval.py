"""Evaluator (calErr, h:1748-1825) and dataset reader (main_.cpp:26-129), CPU only.

The evaluator lives in libsm_hip.so's host code (sm_cal_err, no device call); it is checked
against the oracle's restatement (smo_bad_ratio).  The reader is checked on PNG files written
here (no Middlebury data ships with the reference or this image).
"""
import os

import numpy as np
import pytest

from mystereomatching_amd import dataset, evaluate


def _case(seed, H=37, W=53, D=40):
    rng = np.random.default_rng(seed)
    gt = (rng.random((H, W)) * D).astype(np.float32) * np.float32(0.25)
    dp = (gt + rng.normal(0, 2.0, (H, W))).round().astype(np.int16)
    dp[rng.random((H, W)) < 0.1] = -1
    mask = np.where(rng.random((H, W)) < 0.8, 255, 0).astype(np.uint8)
    mask[0, :5] = 128                     # only 255 counts
    return dp, gt, mask


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
@pytest.mark.parametrize("thres", [1.0, 2.0, 0.5])
def test_cal_err_matches_oracle(oracle, seed, thres):
    import ctypes as C
    dp, gt, mask = _case(seed)
    pbm, rms = evaluate.cal_err(dp, gt, mask, thres)
    lib = oracle.load()
    r = C.c_float()
    ref = lib.smo_bad_ratio(dp.shape[0], dp.shape[1], oracle._p(dp), oracle._p(gt), oracle._p(mask), thres, C.byref(r))
    assert np.float32(pbm) == np.float32(ref)
    assert np.float32(rms) == np.float32(r.value)


def test_cal_err_edge_cases():
    dp = np.full((4, 5), -1, np.int16)
    gt = np.zeros((4, 5), np.float32)
    assert evaluate.cal_err(dp, gt, np.full((4, 5), 255, np.uint8)) == (1.0, pytest.approx(np.sqrt(2.0)))
    assert evaluate.cal_err(dp, gt, np.zeros((4, 5), np.uint8)) == (0.0, 0.0)
    with pytest.raises(ValueError):
        evaluate.cal_err(dp, gt[:3], np.zeros((4, 5), np.uint8))


def test_gray_formula():
    # libpng rgb_to_gray fixed point (OpenCV's PNG decoder, coefficients 0.299 / 0.587)
    bgr = np.array([[[0, 0, 255], [0, 255, 0], [255, 0, 0], [255, 255, 255], [10, 20, 30]]], np.uint8)
    np.testing.assert_array_equal(dataset.gray_from_bgr(bgr)[0], [76, 150, 29, 255, (30 * 9798 + 20 * 19235 + 10 * 3735 + 16384) >> 15])


def test_load_middlebury_layout(tmp_path):
    from PIL import Image
    rng = np.random.default_rng(7)
    H, W = 30, 41
    d = tmp_path / "teddy"
    d.mkdir()
    rgb_l = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    rgb_r = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    Image.fromarray(rgb_l).save(d / "im2.png")
    Image.fromarray(rgb_r).save(d / "im6.png")
    gt8 = rng.integers(0, 240, (H, W), dtype=np.uint8)
    Image.fromarray(gt8).save(d / "disp2.png")
    for m in ("nonocc", "all"):
        Image.fromarray(np.where(rng.random((H, W)) < 0.7, 255, 0).astype(np.uint8)).save(d / f"{m}.png")
    s = dataset.load(str(tmp_path), "teddy")
    assert s.max_disp == 59
    np.testing.assert_array_equal(s.lbgr, rgb_l[..., ::-1])
    np.testing.assert_array_equal(s.rgray, dataset.gray_from_bgr(rgb_r[..., ::-1]))
    np.testing.assert_array_equal(s.gt, gt8.astype(np.float32) * np.float32(0.25))   # teddy: disparity x 4 (main:40)
    assert s.masks["disc"] is None and s.masks["nonocc"].shape == (H, W)
    with pytest.raises(FileNotFoundError):
        dataset.load(str(tmp_path), "cones")

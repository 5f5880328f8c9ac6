"""Middlebury / KITTI-style dataset reader mirroring main_.cpp's input handling (main_.cpp:26-129).

Per object the reference reads (main_.cpp:78-107):
  I1_c / I2_c = imread(left/right .png, 1)   -> BGR u8
  I1 / I2     = imread(left/right .png, 0)   -> gray u8 (the PNG decoder's RGB -> gray)
  masks       = imread(all/nonocc/disc.png, 0)
  DT          = imread(disp .png, 0) converted to float and divided by the object's disparity
                scale (disp_reduceCoeffList, main_.cpp:40) for "MD", by 256 for "KT" (main:124-127)
The object tables below are main_.cpp:33-41's lists.  PNG decoding uses PIL; OpenCV's PNG
decoder turns colour into gray with libpng's fixed-point rgb_to_gray (coefficients 0.299 / 0.587
-> 9798 / 19235 / 3735 over 2^15), restated in `gray_from_bgr` (an assumption about the
reference's OpenCV build, which this repository cannot link).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np

# main_.cpp:33-41 (object, left, right, gt, disparity scale, maxdisp)
OBJECTS = ["tsukuba", "venus", "teddy", "cones", "Art", "Books", "Dolls", "Laundry", "Moebius", "Reindeer", "Aloe",
           "Baby1", "Baby2", "Baby3", "Bowling1", "Bowling2", "Cloth1", "Cloth2", "Cloth3", "Cloth4", "Flowerpots",
           "Lampshade1", "Lampshade2", "Midd1", "Midd2", "Monopoly", "Plastic", "Rocks1", "Rocks2", "Wood1", "Wood2",
           "Katzaa", "Michmoret"]
LEFT = ["scene1.row3.col3", "im2", "im2", "im2"] + ["view1"] * 27 + ["left_matlab_valid_resize"] * 2
RIGHT = ["scene1.row3.col4", "im6", "im6", "im6"] + ["view5"] * 27 + ["right_matlab_valid_resize"] * 2
DISP = ["truedisp.row3.col3", "disp2", "disp2", "disp2"] + ["disp1"] * 27 + ["all"] * 2
REDUCE = [16, 8, 4, 4] + [3] * 27 + [5, 5]
MAXDISP = [15, 19, 59, 59] + [85] * 27 + [80, 80]
MASKS = {"all": "all.png", "nonocc": "nonocc.png", "disc": "disc.png"}


@dataclass
class Sample:
    name: str
    lbgr: np.ndarray
    rbgr: np.ndarray
    lgray: np.ndarray
    rgray: np.ndarray
    gt: Optional[np.ndarray]
    masks: Dict[str, Optional[np.ndarray]]
    max_disp: int

    def pair(self) -> dict:
        return {"lbgr": self.lbgr, "rbgr": self.rbgr, "lgray": self.lgray, "rgray": self.rgray}


def gray_from_bgr(bgr: np.ndarray) -> np.ndarray:
    """libpng rgb_to_gray as OpenCV's PNG decoder sets it up: (R*9798 + G*19235 + B*3735 + 2^14) >> 15."""
    b = bgr[..., 0].astype(np.int64)
    g = bgr[..., 1].astype(np.int64)
    r = bgr[..., 2].astype(np.int64)
    return ((r * 9798 + g * 19235 + b * 3735 + 16384) >> 15).astype(np.uint8)


def _read_png(path: str) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        if im.mode in ("I;16", "I;16B", "I"):
            raise ValueError(f"{path}: 16-bit PNGs are read by imread(.., 0) as 8 bit; not supported")
        return np.asarray(im.convert("RGB") if im.mode not in ("L", "RGB") else im)


def imread_color(path: str) -> np.ndarray:
    """imread(path, 1): BGR u8."""
    a = _read_png(path)
    if a.ndim == 2:
        a = np.repeat(a[..., None], 3, axis=2)
    return np.ascontiguousarray(a[..., ::-1])


def imread_gray(path: str) -> np.ndarray:
    """imread(path, 0): gray u8 (single-channel files as stored, colour files via rgb_to_gray)."""
    a = _read_png(path)
    if a.ndim == 2:
        return np.ascontiguousarray(a)
    return gray_from_bgr(a[..., ::-1])


def load(root: str, obj: str, dataset: str = "MD") -> Sample:
    """One object of main_.cpp's Middlebury loop (main_.cpp:78-129); root = StereoMatching::root."""
    i = OBJECTS.index(obj)
    d = os.path.join(root, obj)
    left, right = os.path.join(d, LEFT[i] + ".png"), os.path.join(d, RIGHT[i] + ".png")
    if not (os.path.exists(left) and os.path.exists(right)):
        raise FileNotFoundError("can't read original img")   # main_.cpp:110
    lbgr, rbgr = imread_color(left), imread_color(right)
    lg, rg = imread_gray(left), imread_gray(right)
    masks = {}
    for k, f in MASKS.items():
        p = os.path.join(d, f)
        masks[k] = imread_gray(p) if os.path.exists(p) else None
    gt = None
    gp = os.path.join(d, DISP[i] + ".png")
    if os.path.exists(gp):
        raw = imread_gray(gp).astype(np.float32)
        gt = raw / np.float32(256.0) if dataset == "KT" else raw * np.float32(1.0 / REDUCE[i])  # convertTo(CV_32F, 1/scale)
    return Sample(obj, lbgr, rbgr, lg, rg, gt, masks, MAXDISP[i])

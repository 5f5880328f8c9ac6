"""Seeded synthetic stereo pairs with known ground truth.

Piecewise-planar scene: random-texture background (uniform u8 noise blurred 3x3 per channel) and
8-16 textured rectangles, each a fronto-parallel or slanted disparity plane.  The right image is
the left image forward-warped by the integer GT disparity with a z-buffer (nearer surface wins);
occlusion holes are filled with fresh noise.  Gray = (R*9798 + G*19235 + B*3735 + 16384) >> 15,
the libpng rgb->gray formula OpenCV's PNG decoder uses (documented assumption).
Images are BGR like cv::imread(..., 1).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 20250307


def _texture(rng, h, w):
    n = rng.integers(0, 256, (h + 2, w + 2, 3), dtype=np.int32)
    s = np.zeros((h, w, 3), np.int32)
    for dy in range(3):
        for dx in range(3):
            s += n[dy:dy + h, dx:dx + w]
    return ((s + 4) // 9).astype(np.uint8)


def bgr_to_gray(bgr: np.ndarray) -> np.ndarray:
    b = bgr[..., 0].astype(np.int32)
    g = bgr[..., 1].astype(np.int32)
    r = bgr[..., 2].astype(np.int32)
    return ((r * 9798 + g * 19235 + b * 3735 + 16384) >> 15).astype(np.uint8)


def make_pair(H: int, W: int, D: int, index: int = 0, seed: int | None = None) -> dict:
    """Return dict(lbgr, rbgr, lgray, rgray, gt(float32, px), nonocc(u8 mask), all(u8 mask))."""
    rng = np.random.default_rng(SEED_BASE + index if seed is None else seed)
    left = _texture(rng, H, W)
    dmax = max(D - 1, 0)
    disp = np.full((H, W), rng.uniform(0, 0.25 * dmax), np.float64)
    nrect = int(rng.integers(8, 17))
    vv, uu = np.mgrid[0:H, 0:W]
    rects = []
    for _ in range(nrect):
        h = int(rng.integers(max(2, H // 10), max(3, H // 2)))
        w = int(rng.integers(max(2, W // 10), max(3, W // 2)))
        v0 = int(rng.integers(0, max(1, H - h)))
        u0 = int(rng.integers(0, max(1, W - w)))
        d0 = rng.uniform(0.1 * dmax, dmax)
        slanted = rng.random() < 0.5
        gu = rng.uniform(-0.08, 0.08) if slanted else 0.0
        gv = rng.uniform(-0.08, 0.08) if slanted else 0.0
        rects.append((d0, v0, u0, h, w, gu, gv))
    rects.sort(key=lambda r: r[0])  # painter's order: nearer (larger d) drawn last
    for d0, v0, u0, h, w, gu, gv in rects:
        tex = _texture(rng, h, w)
        sl = (slice(v0, v0 + h), slice(u0, u0 + w))
        left[sl] = tex
        plane = d0 + gu * (uu[sl] - (u0 + w / 2)) + gv * (vv[sl] - (v0 + h / 2))
        disp[sl] = plane
    disp = np.clip(disp, 0, dmax)
    di = np.rint(disp).astype(np.int64)
    # forward warp with z-buffer
    right = _texture(rng, H, W)
    ur = uu - di
    ok = ur >= 0
    zbuf = np.full((H, W), -1, np.int64)
    np.maximum.at(zbuf, (vv[ok], ur[ok]), di[ok])
    win = ok.copy()
    win[ok] = di[ok] == zbuf[vv[ok], ur[ok]]
    right[vv[win], ur[win]] = left[vv[win], uu[win]]
    nonocc = np.where(win, 255, 0).astype(np.uint8)
    return {
        "lbgr": left, "rbgr": right,
        "lgray": bgr_to_gray(left), "rgray": bgr_to_gray(right),
        "gt": di.astype(np.float32), "nonocc": nonocc,
        "all": np.full((H, W), 255, np.uint8),
    }


def make_batch(n: int, H: int, W: int, D: int, first_index: int = 0):
    pairs = [make_pair(H, W, D, first_index + i) for i in range(n)]
    stack = lambda k: np.ascontiguousarray(np.stack([p[k] for p in pairs]))
    return {k: stack(k) for k in ("lbgr", "rbgr", "lgray", "rgray", "gt", "nonocc")}

"""ctypes wrapper of the CPU restatement (oracle/sm_oracle.c) — TEST INFRASTRUCTURE ONLY.

PARITY UNPINNED (see sm_oracle.h): the reference cannot be built here and ships no fixtures.
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libsm_oracle.so")

COST = {"censusGrad": 0, "Census": 1, "ADCensus": 2, "AD": 3}


class Config(C.Structure):
    """struct smo_config (oracle/sm_oracle.h)."""

    _fields_ = [
        ("H", C.c_int), ("W", C.c_int), ("D", C.c_int), ("cost_method", C.c_int),
        ("census_rv", C.c_int), ("census_ru", C.c_int), ("census_ring", C.c_int),
        ("lam_cen", C.c_float), ("lam_g", C.c_float), ("grad_trunc", C.c_float),
        ("grad_adaptive", C.c_int), ("lam_ad", C.c_float), ("lam_cen_adc", C.c_float),
        ("ad_trunc_adc", C.c_float), ("ad_trunc_ad", C.c_float),
        ("arm_L", C.c_int), ("arm_L_out", C.c_int), ("arm_cT", C.c_int), ("arm_cT_out", C.c_int),
        ("arm_minL", C.c_int), ("aggregation", C.c_int), ("cbca_iters", C.c_int),
        ("solve_all", C.c_int), ("reg_lambda", C.c_float), ("optimization", C.c_int),
        ("sgm_paths", C.c_int), ("sgm_p1", C.c_float), ("sgm_p2", C.c_float),
        ("sgm_cor_thres", C.c_int), ("sgm_redu", C.c_int),
        ("do_refine", C.c_int), ("lr_max_diff", C.c_float), ("do_region_vote", C.c_int),
        ("region_vote_nums", C.c_int), ("rv_ratio", C.c_float), ("rv_s", C.c_int),
        ("do_proper_ipol", C.c_int), ("disp_occ", C.c_int), ("do_last_median", C.c_int),
        ("gf_r", C.c_int), ("gf_eps", C.c_float), ("nl_sigma", C.c_double), ("gf_mode", C.c_int),
    ]


class Dumps(C.Structure):
    """struct smo_dumps (oracle/sm_oracle.h)."""

    _fields_ = [(k, C.c_void_p) for k in ("vol_cost", "vol_agg", "vol_final", "vol_right", "vol_agg_right",
                                           "disp_left_raw", "disp_right", "stage_ms")]


_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P = C.c_void_p
        lib.smo_default_config.argtypes = [C.POINTER(Config), C.c_int, C.c_int, C.c_int]
        lib.smo_run.argtypes = [C.POINTER(Config), P, P, P, P, P, P, P, P, P, P]
        lib.smo_run.restype = C.c_int
        lib.smo_run_ex.argtypes = [C.POINTER(Config), P, P, P, P, P, C.POINTER(Dumps)]
        lib.smo_run_ex.restype = C.c_int
        lib.smo_lr_check.argtypes = [C.POINTER(Config), P, P]
        lib.smo_region_vote.argtypes = [C.POINTER(Config), P, P, C.c_float, C.c_int]
        lib.smo_proper_ipol.argtypes = [C.POINTER(Config), P, P]
        lib.smo_median3.argtypes = [C.c_int, C.c_int, P]
        lib.smo_refine.argtypes = [C.POINTER(Config), P, P, P, P]
        lib.smo_pyr_down_u8.argtypes = [P, C.c_int, C.c_int, C.c_int, P]
        lib.smo_pyr_weights.argtypes = [C.c_int, C.c_float, P]
        lib.smo_pyr_weights.restype = C.c_int
        lib.smo_solve_all_pyr.argtypes = [P, P, C.c_int, C.c_float]
        lib.smo_solve_all_pyr.restype = C.c_int
        lib.smo_run_pyr.argtypes = [C.POINTER(Config), C.c_int, P, P, P, P, P]
        lib.smo_run_pyr.restype = C.c_int
        lib.smo_census.argtypes = [C.POINTER(Config), P, P]
        lib.smo_arms.argtypes = [C.POINTER(Config), P, P]
        lib.smo_cost_volume.argtypes = [C.POINTER(Config), P, P, P, P, C.c_int, P]
        lib.smo_census_nwords.argtypes = [C.POINTER(Config)]
        lib.smo_solve_all_weight.argtypes = [C.c_float]
        lib.smo_solve_all_weight.restype = C.c_float
        lib.smo_bad_ratio.argtypes = [C.c_int, C.c_int, P, P, P, C.c_float, C.POINTER(C.c_float)]
        lib.smo_bad_ratio.restype = C.c_float
        lib.smo_expf_range.argtypes = [C.c_uint32, C.c_uint32, P]
        lib.smo_box_filter.argtypes = [C.c_int, C.c_int, C.c_int, P, P, P]
        lib.smo_box_filter_cv.argtypes = [C.c_int, C.c_int, C.c_int, P, P, P]
        lib.smo_reflect.argtypes = [C.c_int, C.c_int]
        lib.smo_reflect.restype = C.c_int
        lib.smo_guided_filter.argtypes = [C.POINTER(Config), P, P]
        lib.smo_guided_filter.restype = C.c_int
        lib.smo_nl_median3.argtypes = [C.c_int, C.c_int, P, P]
        lib.smo_nl_tree.argtypes = [C.c_int, C.c_int, P, P, P, P, P, P]
        lib.smo_nl_tree.restype = C.c_int
        lib.smo_nl_table.argtypes = [C.c_double, P]
        lib.smo_nl_aggregate.argtypes = [C.POINTER(Config), P, P]
        lib.smo_nl_aggregate.restype = C.c_int
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def config(H, W, max_disp, cost="censusGrad", **kw) -> Config:
    lib = load()
    c = Config()
    lib.smo_default_config(C.byref(c), max_disp, H, W)
    c.cost_method = COST[cost] if isinstance(cost, str) else cost
    for k, v in kw.items():
        if not hasattr(c, k):
            raise AttributeError(k)
        setattr(c, k, v)
    return c


def run(pair: dict, cfg: Config, dumps: bool = False, right: bool = False):
    """Run the pipeline; returns dict(disp, [cost, agg, final], [right], stage_ms)."""
    lib = load()
    H, W, D = cfg.H, cfg.W, cfg.D
    arr = {k: np.ascontiguousarray(pair[k], np.uint8) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    disp = np.empty((H, W), np.int16)
    vols = {k: (np.empty((H, W, D), np.float32) if dumps else None) for k in ("cost", "agg", "final")}
    vr = np.empty((H, W, D), np.float32) if right else None
    ms = (C.c_double * 6)()
    st = lib.smo_run(C.byref(cfg), _p(arr["lbgr"]), _p(arr["rbgr"]), _p(arr["lgray"]), _p(arr["rgray"]),
                     _p(disp), _p(vols["cost"]), _p(vols["agg"]), _p(vols["final"]), _p(vr), ms)
    if st != 0:
        raise ValueError("oracle rejected the configuration")
    out = {"disp": disp, "stage_ms": list(ms)}
    if dumps:
        out.update(vols)
    if right:
        out["right"] = vr
    return out


def run_ex(pair: dict, cfg: Config, dumps=()):
    """smo_run_ex: returns dict(disp, stage_ms, and each requested dump:
    cost, agg, final, right, agg_right (H x W x D float32), disp_raw, disp_right (H x W int16))."""
    lib = load()
    H, W, D = cfg.H, cfg.W, cfg.D
    arr = {k: np.ascontiguousarray(pair[k], np.uint8) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    disp = np.empty((H, W), np.int16)
    names = {"cost": "vol_cost", "agg": "vol_agg", "final": "vol_final", "right": "vol_right",
             "agg_right": "vol_agg_right", "disp_raw": "disp_left_raw", "disp_right": "disp_right"}
    bufs = {}
    d = Dumps()
    for k in dumps:
        bufs[k] = np.empty((H, W), np.int16) if k.startswith("disp") else np.empty((H, W, D), np.float32)
        setattr(d, names[k], bufs[k].ctypes.data)
    ms = (C.c_double * 7)()
    d.stage_ms = C.cast(ms, C.c_void_p).value
    st = lib.smo_run_ex(C.byref(cfg), _p(arr["lbgr"]), _p(arr["rbgr"]), _p(arr["lgray"]), _p(arr["rgray"]),
                        _p(disp), C.byref(d))
    if st != 0:
        raise ValueError("oracle rejected the configuration")
    return {"disp": disp, "stage_ms": list(ms), **bufs}


def lr_check(d0: np.ndarray, d1: np.ndarray, cfg: Config) -> np.ndarray:
    out = np.ascontiguousarray(d0, np.int16).copy()
    load().smo_lr_check(C.byref(cfg), _p(out), _p(np.ascontiguousarray(d1, np.int16)))
    return out


def region_vote(dp: np.ndarray, arms_l: np.ndarray, cfg: Config) -> np.ndarray:
    out = np.ascontiguousarray(dp, np.int16).copy()
    load().smo_region_vote(C.byref(cfg), _p(out), _p(np.ascontiguousarray(arms_l, np.uint16)), cfg.rv_ratio, cfg.rv_s)
    return out


def proper_ipol(dp: np.ndarray, bgr: np.ndarray, cfg: Config) -> np.ndarray:
    out = np.ascontiguousarray(dp, np.int16).copy()
    load().smo_proper_ipol(C.byref(cfg), _p(out), _p(np.ascontiguousarray(bgr, np.uint8)))
    return out


def median3(dp: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(dp, np.int16).copy()
    load().smo_median3(out.shape[0], out.shape[1], _p(out))
    return out


def refine(d0, d1, arms_l, bgr, cfg: Config) -> np.ndarray:
    out = np.ascontiguousarray(d0, np.int16).copy()
    load().smo_refine(C.byref(cfg), _p(out), _p(np.ascontiguousarray(d1, np.int16)),
                      _p(np.ascontiguousarray(arms_l, np.uint16)), _p(np.ascontiguousarray(bgr, np.uint8)))
    return out


def pyr_down(img: np.ndarray) -> np.ndarray:
    """cv::pyrDown of a u8 H x W or H x W x C image (smo_pyr_down_u8)."""
    a = np.ascontiguousarray(img, np.uint8)
    rows, cols = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    out = np.empty(((rows + 1) // 2, (cols + 1) // 2) + a.shape[2:], np.uint8)
    load().smo_pyr_down_u8(_p(a), rows, cols, ch, _p(out))
    return out


def pyr_weights(py_lvl: int, reg_lambda: float = 0.3) -> np.ndarray:
    w = np.zeros(8, np.float32)
    if load().smo_pyr_weights(py_lvl, reg_lambda, _p(w)) != 0:
        raise ValueError("PY_LVL must be in [1, 8]")
    return w[:py_lvl]


def run_pyr(pair: dict, cfg: Config, py_lvl: int) -> np.ndarray:
    """smo_run_pyr: main_.cpp:131-166 with PY_LEV = py_lvl; returns DP[0]."""
    arr = {k: np.ascontiguousarray(pair[k], np.uint8) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    disp = np.empty((cfg.H, cfg.W), np.int16)
    st = load().smo_run_pyr(C.byref(cfg), py_lvl, _p(arr["lbgr"]), _p(arr["rbgr"]), _p(arr["lgray"]),
                            _p(arr["rgray"]), _p(disp))
    if st != 0:
        raise ValueError("oracle rejected the pyramid configuration")
    return disp


def census(gray: np.ndarray, cfg: Config) -> np.ndarray:
    lib = load()
    nw = lib.smo_census_nwords(C.byref(cfg))
    g = np.ascontiguousarray(gray, np.uint8)
    out = np.zeros((cfg.H, cfg.W, nw), np.uint64)
    lib.smo_census(C.byref(cfg), _p(g), _p(out))
    return out


def arms(bgr: np.ndarray, cfg: Config) -> np.ndarray:
    lib = load()
    b = np.ascontiguousarray(bgr, np.uint8)
    out = np.zeros((cfg.H, cfg.W, 4), np.uint16)
    lib.smo_arms(C.byref(cfg), _p(b), _p(out))
    return out


def cost_volume(pair: dict, cfg: Config, view: int = 0) -> np.ndarray:
    lib = load()
    arr = {k: np.ascontiguousarray(pair[k], np.uint8) for k in ("lbgr", "rbgr", "lgray", "rgray")}
    out = np.empty((cfg.H, cfg.W, cfg.D), np.float32)
    lib.smo_cost_volume(C.byref(cfg), _p(arr["lbgr"]), _p(arr["rbgr"]), _p(arr["lgray"]), _p(arr["rgray"]), view, _p(out))
    return out


def solve_all_weight(reg_lambda: float = 0.3) -> float:
    return load().smo_solve_all_weight(reg_lambda)


def expf_range(first_bits: int, n: int) -> np.ndarray:
    out = np.empty(n, np.float32)
    load().smo_expf_range(first_bits, n, _p(out))
    return out


def expf_libm(x: np.ndarray) -> np.ndarray:
    """Host libm expf on each element (via ctypes to libm; numpy's exp is not libm's)."""
    libm = C.CDLL("libm.so.6")
    libm.expf.restype = C.c_float
    libm.expf.argtypes = [C.c_float]
    return np.array([libm.expf(float(v)) for v in np.asarray(x, np.float32).ravel()], np.float32)


def box_filter(img: np.ndarray, r: int) -> np.ndarray:
    """BoxFilter (cpp:5151-5202) of a float32 H x W image."""
    a = np.ascontiguousarray(img, np.float32)
    H, W = a.shape
    out, tmp = np.empty_like(a), np.empty_like(a)
    load().smo_box_filter(H, W, r, _p(a), _p(out), _p(tmp))
    return out


def box_filter_cv(img: np.ndarray, r: int) -> np.ndarray:
    """OpenCV boxFilter (normalised, BORDER_REFLECT, double running sums) of a float32 H x W image."""
    a = np.ascontiguousarray(img, np.float32)
    H, W = a.shape
    out, rs = np.empty_like(a), np.empty((H, W), np.float64)
    load().smo_box_filter_cv(H, W, r, _p(a), _p(out), _p(rs))
    return out


def guided_filter(vm: np.ndarray, bgr: np.ndarray, cfg: Config) -> np.ndarray:
    """guideFilter on every slice of an H x W x D volume: cfg.gf_mode 0 = ximgproc::guidedFilter
    (the shipped build), 1 = guideFilterCore_matlab (the MY_GUIDE build)."""
    out = np.ascontiguousarray(vm, np.float32).copy()
    if load().smo_guided_filter(C.byref(cfg), _p(out), _p(np.ascontiguousarray(bgr, np.uint8))) != 0:
        raise ValueError("guided filter needs H, W >= 2 r + 1")
    return out


def nl_median3(bgr: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(bgr, np.uint8)
    out = np.empty_like(a)
    load().smo_nl_median3(a.shape[0], a.shape[1], _p(a), _p(out))
    return out


def nl_tree(bgr: np.ndarray) -> dict:
    """The MST / BFS tree of NLCCA (order, parent, weight, nchild, child[n, 4])."""
    a = np.ascontiguousarray(bgr, np.uint8)
    H, W = a.shape[:2]
    n = H * W
    t = {"order": np.empty(n, np.int32), "parent": np.empty(n, np.int32), "weight": np.empty(n, np.uint8),
         "nchild": np.empty(n, np.int32), "child": np.full((n, 4), -1, np.int32)}
    if load().smo_nl_tree(H, W, _p(a), *(_p(t[k]) for k in ("order", "parent", "weight", "nchild", "child"))) != 0:
        raise ValueError("tree construction failed")
    return t


def nl_table(sigma: float = 0.1) -> np.ndarray:
    t = np.empty(256, np.float64)
    load().smo_nl_table(sigma, _p(t))
    return t


def nl_aggregate(vm: np.ndarray, bgr: np.ndarray, cfg: Config) -> np.ndarray:
    out = np.ascontiguousarray(vm, np.float32).copy()
    if load().smo_nl_aggregate(C.byref(cfg), _p(out), _p(np.ascontiguousarray(bgr, np.uint8))) != 0:
        raise ValueError("NL aggregation failed")
    return out

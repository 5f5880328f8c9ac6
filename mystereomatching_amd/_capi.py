"""ctypes binding of the C-ABI in include/sm_capi.h (libsm_hip.so, built in-tree).

The HIP library is the only compute path: if it is missing or fails to load this module raises;
there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libsm_hip.so")

SM_OK, SM_EINVAL, SM_ENOMEM, SM_EHIP, SM_ESTATE = 0, 1, 2, 3, 4
COST_METHODS = {"censusGrad": 0, "Census": 1, "ADCensus": 2, "AD": 3}
AGGREGATIONS = {"": 0, "none": 0, "CBCA": 1, "GF": 2, "NL": 3}
OPTIMIZATIONS = {"": 0, "wta": 0, "sgm": 1, "so": 2}


class sm_params(C.Structure):
    """Mirror of struct sm_params (include/sm_capi.h); field order must match."""

    _fields_ = [
        ("struct_size", C.c_uint32),
        ("rows", C.c_int32), ("cols", C.c_int32), ("num_disparities", C.c_int32),
        ("cost_method", C.c_int32), ("aggregation", C.c_int32), ("optimization", C.c_int32),
        ("census_rv", C.c_int32), ("census_ru", C.c_int32), ("census_ring", C.c_int32),
        ("lam_cen", C.c_float), ("lam_g", C.c_float), ("grad_trunc", C.c_float),
        ("grad_adaptive", C.c_int32),
        ("lam_ad", C.c_float), ("lam_cen_adc", C.c_float), ("ad_trunc_adc", C.c_float),
        ("ad_trunc_ad", C.c_float),
        ("arm_l", C.c_int32), ("arm_l_out", C.c_int32), ("arm_c_thresh", C.c_int32),
        ("arm_c_thresh_out", C.c_int32), ("arm_min_l", C.c_int32),
        ("cbca_iterations", C.c_int32), ("sgm_paths", C.c_int32),
        ("sgm_p1", C.c_float), ("sgm_p2", C.c_float),
        ("sgm_cor_dif_thres", C.c_int32), ("sgm_redu_coeff", C.c_int32),
        ("compute_right_view", C.c_int32), ("keep_final_volume", C.c_int32),
        ("batch_capacity", C.c_int32),
        ("do_refine", C.c_int32), ("lr_max_diff", C.c_float), ("do_region_vote", C.c_int32),
        ("region_vote_nums", C.c_int32), ("rv_ratio", C.c_float), ("rv_s", C.c_int32),
        ("do_proper_ipol", C.c_int32), ("disp_occ", C.c_int32), ("do_last_median_blur", C.c_int32),
        ("sub_batch", C.c_int32), ("num_streams", C.c_int32), ("fuse_norm_scan", C.c_int32),
        ("gf_eps", C.c_float), ("gf_mode", C.c_int32), ("nl_sigma", C.c_double),
        ("lr_consis", C.c_int32),
        ("placement_trials", C.c_int32),
    ]


# Every SM_API symbol declared in include/sm_capi.h: (name, restype, argtypes).
_P = C.c_void_p
_u8p = C.POINTER(C.c_uint8)
SIGNATURES = [
    ("sm_params_default", None, [C.POINTER(sm_params), C.c_int32, C.c_int32, C.c_int32]),
    ("sm_create", C.c_int, [C.POINTER(_P), C.POINTER(sm_params), C.c_int32]),
    ("sm_destroy", C.c_int, [_P]),
    ("sm_last_error", C.c_char_p, [_P]),
    ("sm_status_string", C.c_char_p, [C.c_int]),
    ("sm_set_images", C.c_int, [_P, _P, _P, C.c_size_t, _P, _P, C.c_size_t]),
    ("sm_cost_calculate", C.c_int, [_P]),
    ("sm_solve_all", C.c_int, [_P, C.c_int32, C.c_float]),
    ("sm_disp_optimize", C.c_int, [_P, _P]),
    ("sm_solve_all_pyr", C.c_int, [C.POINTER(_P), C.c_int32, C.c_float]),
    ("sm_pyr_down", C.c_int, [C.c_int32, _P, C.c_int32, C.c_int32, C.c_int32, _P]),
    ("sm_pyr_down_f32", C.c_int, [C.c_int32, _P, C.c_int32, C.c_int32, _P]),
    ("sm_refine", C.c_int, [_P, _P]),
    ("sm_get_disp", C.c_int, [_P, C.c_int32, _P]),
    ("sm_set_disp", C.c_int, [_P, C.c_int32, _P]),
    ("sm_get_volume", C.c_int, [_P, C.c_int32, _P]),
    ("sm_get_arms", C.c_int, [_P, C.c_int32, _P]),
    ("sm_upload_batch", C.c_int, [_P, C.c_int32, _P, _P, _P, _P]),
    ("sm_run", C.c_int, [_P, C.c_int32, C.c_float, _P]),
    ("sm_download_disp", C.c_int, [_P, C.c_int32, _P]),
    ("sm_download_disp_async", C.c_int, [_P, C.c_int32, _P]),
    ("sm_upload_batch_async", C.c_int, [_P, C.c_int32, _P, _P, _P, _P]),
    ("sm_upload_wait", C.c_int, [_P]),
    ("sm_download_wait", C.c_int, [_P, C.c_int32]),
    ("sm_run_batch", C.c_int, [_P, C.c_int32, _P, _P, _P, _P, C.c_float, _P]),
    ("sm_run_batch_multi", C.c_int, [C.POINTER(_P), C.c_int32, C.c_int32, _P, _P, _P, _P, C.c_float, _P]),
    ("sm_set_schedule", C.c_int, [_P, C.c_int32, C.c_int32]),
    ("sm_placement_trials_ms", C.c_int32, [_P, C.POINTER(C.c_double), C.c_int32]),
    ("sm_placement_kept", C.c_int32, [_P]),
    ("sm_synchronize", C.c_int, [_P]),
    ("sm_stream", C.c_void_p, [_P]),
    ("sm_profile_enable", C.c_int, [_P, C.c_int32]),
    ("sm_profile_read", C.c_int, [_P, C.c_int32, _P, _P, _P, _P, C.POINTER(C.c_int32)]),
    ("sm_profile_reset", C.c_int, [_P]),
    ("sm_cal_err", C.c_int, [_P, _P, _P, C.c_int32, C.c_int32, C.c_float, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    ("sm_expf_host", C.c_float, [C.c_float]),
    ("sm_expf_device_range", C.c_int, [_P, C.c_uint32, C.c_uint32, _P]),
    ("sm_div_area_check", C.c_int, [_P, C.c_int32, C.c_int32, _P]),
    ("sm_copy_ceiling", C.c_int, [_P, C.c_uint64, C.c_int32, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("sm_get_census", C.c_int, [_P, C.c_int32, _P]),
]

_lib = None


def load() -> C.CDLL:
    """Load libsm_hip.so (raises OSError/FileNotFoundError when absent: no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    # SM_HIP_LIB: an alternative build of the same library (tuning sweeps, tools/build_variants.sh)
    path = os.environ.get("SM_HIP_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise FileNotFoundError(
            f"{path} is missing; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C mystereomatching_amd/csrc`")
    lib = C.CDLL(path)
    for name, res, args in SIGNATURES:
        if path != LIB_PATH and not hasattr(lib, name):
            continue  # an older tuning build may predate a diagnostic entry point
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class SMError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"sm status {status}: {msg}")
        self.status = status


def check(lib, ctx, status: int, what: str = ""):
    if status != SM_OK:
        msg = lib.sm_last_error(ctx).decode() if ctx else lib.sm_status_string(status).decode()
        raise SMError(status, f"{what}: {msg}" if what else msg)


def default_params(max_disp: int, rows: int, cols: int, **overrides) -> sm_params:
    lib = load()
    p = sm_params()
    lib.sm_params_default(C.byref(p), max_disp, rows, cols)
    for k, v in overrides.items():
        if k == "cost_method" and isinstance(v, str):
            v = COST_METHODS[v]
        elif k == "aggregation" and isinstance(v, str):
            v = AGGREGATIONS[v]
        elif k == "optimization" and isinstance(v, str):
            v = OPTIMIZATIONS[v]
        if not hasattr(p, k):
            raise AttributeError(f"sm_params has no field {k!r}")
        setattr(p, k, v)
    return p


def ptr(a):
    """Raw data pointer of a C-contiguous numpy array."""
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return C.c_void_p(a.ctypes.data)

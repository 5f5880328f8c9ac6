"""C-ABI boundary checks that need no GPU: the library loads, exports exactly what
include/*.h declares, the ctypes struct matches the C layout, and parameter validation
rejects bad configurations before touching the device."""
import ctypes as C
import glob
import os
import re

import numpy as np
import pytest

from mystereomatching_amd import _capi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        txt = open(h).read()
        names |= set(re.findall(r"SM_API\s+[\w\s\*]+?\b(sm_\w+)\s*\(", txt))
    return names


def test_library_exports_every_declared_symbol():
    lib = _capi.load()
    decl = declared_symbols()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), name
    # the ctypes table covers exactly the header
    assert decl == {n for n, _, _ in _capi.SIGNATURES}


def test_params_struct_layout_and_defaults():
    # struct sm_params: 4-byte fields and one double; the header's C layout must match ctypes
    txt = open(os.path.join(ROOT, "include", "sm_capi.h")).read()
    body = txt[txt.index("typedef struct sm_params {"):txt.index("} sm_params;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    off, align = 0, 4
    for ln in body.splitlines()[1:]:
        ln = ln.strip()
        if not ln:
            continue
        size = 8 if ln.startswith("double") else 4
        for _ in re.findall(r"\b\w+\s*(?:,|;)", ln):
            off = (off + size - 1) // size * size + size
            align = max(align, size)
    assert C.sizeof(_capi.sm_params) == (off + align - 1) // align * align
    p = _capi.default_params(59, 375, 450)
    assert p.num_disparities == 60
    assert (p.census_rv, p.census_ru, p.census_ring) == (3, 4, 1)
    assert (p.arm_l, p.arm_l_out, p.arm_c_thresh, p.arm_c_thresh_out, p.arm_min_l) == (17, 34, 20, 6, 1)
    assert (p.cbca_iterations, p.sgm_paths, p.sgm_cor_dif_thres, p.sgm_redu_coeff) == (2, 4, 15, 4)
    assert (p.lam_cen, p.lam_g, p.grad_trunc, p.sgm_p1, p.sgm_p2) == (13.0, 1.0, 500.0, 1.0, 3.0)
    # refine() switches and constants (h:70-80, 212, 216, 306; cpp:1400-1401)
    assert (p.do_refine, p.lr_max_diff, p.do_region_vote, p.region_vote_nums, p.rv_s) == (0, 0.0, 1, 2, 20)
    assert (p.do_proper_ipol, p.disp_occ, p.do_last_median_blur) == (1, -32, 1)
    assert np.float32(p.rv_ratio) == np.float32(0.4)
    assert (p.sub_batch, p.num_streams, p.fuse_norm_scan) == (0, 0, -1)
    assert np.float32(p.gf_eps) == np.float32(1e-4) and p.nl_sigma == 0.1
    assert p.gf_mode == 0   # SM_GF_XIMGPROC: the shipped build (`//#define MY_GUIDE`, h:38)
    assert p.struct_size == C.sizeof(_capi.sm_params)


@pytest.mark.parametrize("field,value,msg", [
    ("rows", 1, b"rows"), ("num_disparities", 0, b"num_disparities"), ("num_disparities", 2000, b"num_disparities"),
    ("census_rv", 7, b"census"), ("arm_l_out", 200, b"arm"), ("sgm_paths", 9, b"sgm_paths"),
    ("batch_capacity", 0, b"batch"), ("cost_method", 7, b"cost_method"), ("lam_cen", 0.0, b"lambda"),
    ("lam_g", -1.0, b"lambda"), ("grad_trunc", -5.0, b"truncation"), ("sgm_p2", -1.0, b"penalties"),
    ("sgm_redu_coeff", -4, b"penalties"), ("sgm_p2", -0.0, b"penalties"), ("sgm_p1", -0.0, b"penalties"),
    ("grad_trunc", -0.0, b"truncation"), ("ad_trunc_ad", -0.0, b"truncation"), ("num_streams", 5, b"num_streams"),
    ("sub_batch", -1, b"sub_batch"), ("aggregation", 4, b"aggregation"), ("struct_size", 4, b"struct_size"),
])
def test_validation_rejects_before_device(field, value, msg):
    lib = _capi.load()
    p = _capi.default_params(63, 32, 32)
    setattr(p, field, value)
    ctx = C.c_void_p()
    st = lib.sm_create(C.byref(ctx), C.byref(p), 0)
    try:
        assert st == _capi.SM_EINVAL
        assert msg in lib.sm_last_error(ctx)
    finally:
        lib.sm_destroy(ctx)


def test_null_arguments():
    lib = _capi.load()
    assert lib.sm_create(None, None, 0) == _capi.SM_EINVAL
    assert lib.sm_cost_calculate(None) == _capi.SM_EINVAL
    assert lib.sm_destroy(None) == _capi.SM_OK
    assert lib.sm_status_string(_capi.SM_ESTATE) == b"call out of order"


def test_host_expf_matches_libm_sample(oracle):
    """The device expf algorithm (evaluated on the host) equals libm expf on a strided sample of
    [-103.97, 0]; the exhaustive check runs on the GPU (test_device_expf_exhaustive)."""
    lib = _capi.load()
    first, last = 0x80000000, 0xC2D00000
    idx = np.arange(first, last, 9973, dtype=np.uint64).astype(np.uint32)
    xs = idx.view(np.float32)
    ref = np.empty_like(xs)
    for i in range(0, len(idx), 1):
        pass
    ref = np.concatenate([oracle.expf_range(int(b), 1) for b in idx[::50]])
    got = np.array([lib.sm_expf_host(float(x)) for x in xs[::50]], np.float32)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    # near the exp(-G) cut where the fusion stops depending on the gradient term
    xs2 = np.linspace(-18, 0, 20001, dtype=np.float32)
    got2 = np.array([lib.sm_expf_host(float(x)) for x in xs2], np.float32)
    ref2 = np.concatenate([oracle.expf_range(int(b), 1) for b in xs2.view(np.uint32)])
    assert np.array_equal(got2.view(np.uint32), ref2.view(np.uint32))


@pytest.mark.parametrize("field,value,msg", [("rv_ratio", 0.0, b"rv_ratio"), ("region_vote_nums", -1, b"region_vote_nums")])
def test_refine_validation(field, value, msg):
    lib = _capi.load()
    p = _capi.default_params(63, 32, 32, do_refine=1)
    setattr(p, field, value)
    ctx = C.c_void_p()
    st = lib.sm_create(C.byref(ctx), C.byref(p), 0)
    try:
        assert st == _capi.SM_EINVAL
        assert msg in lib.sm_last_error(ctx)
    finally:
        lib.sm_destroy(ctx)


def test_run_batch_multi_argument_checks():
    """sm_run_batch_multi rejects bad arguments before touching a device."""
    lib = _capi.load()
    buf = (C.c_uint8 * 16)()
    out = (C.c_int16 * 16)()
    p = C.cast(buf, C.c_void_p)
    assert lib.sm_run_batch_multi(None, 1, 1, p, p, p, p, 0.3, C.cast(out, C.c_void_p)) == _capi.SM_EINVAL
    arr = (C.c_void_p * 1)(None)
    assert lib.sm_run_batch_multi(arr, 1, 1, p, p, p, p, 0.3, C.cast(out, C.c_void_p)) == _capi.SM_EINVAL
    assert lib.sm_run_batch_multi(arr, 0, 1, p, p, p, p, 0.3, C.cast(out, C.c_void_p)) == _capi.SM_EINVAL
    assert lib.sm_run_batch_multi(arr, 1, 0, p, p, p, p, 0.3, C.cast(out, C.c_void_p)) == _capi.SM_EINVAL


@pytest.mark.parametrize("over,msg", [(dict(aggregation=2, rows=8), b"GF"), (dict(aggregation=2, gf_mode=1, rows=18), b"GF"),
                                      (dict(aggregation=2, optimization=2), b"GF"),
                                      (dict(aggregation=3, rows=2, cols=2), b"NL"), (dict(aggregation=3, rows=2), b"NL"),
                                      (dict(aggregation=3, cols=2), b"NL"), (dict(aggregation=2, gf_eps=0.0), b"gf_eps"),
                                      (dict(aggregation=2, gf_mode=2), b"gf_mode"),
                                      (dict(aggregation=3, nl_sigma=0.0), b"nl_sigma"),
                                      (dict(aggregation=3, rows=8192, cols=8192, batch_capacity=8), b"2^29")])
def test_alternative_aggregator_domain(over, msg):
    lib = _capi.load()
    p = _capi.default_params(15, 32, 32)
    for k, v in over.items():
        setattr(p, k, v)
    ctx = C.c_void_p()
    st = lib.sm_create(C.byref(ctx), C.byref(p), 0)
    try:
        assert st == _capi.SM_EINVAL
        assert msg in lib.sm_last_error(ctx)
    finally:
        lib.sm_destroy(ctx)


def test_aggregator_constants_checked_only_for_their_aggregator():
    """gf_eps / nl_sigma / gf_mode are read only by GF / NL: a CBCA struct with them zeroed passes
    validation (here, without a GPU, sm_create then fails at the device, not with EINVAL)."""
    lib = _capi.load()
    p = _capi.default_params(15, 32, 32, gf_eps=0.0, nl_sigma=0.0, gf_mode=7)
    ctx = C.c_void_p()
    st = lib.sm_create(C.byref(ctx), C.byref(p), 0)
    try:
        assert st != _capi.SM_EINVAL, lib.sm_last_error(ctx)
    finally:
        lib.sm_destroy(ctx)

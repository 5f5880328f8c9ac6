"""Host-side mirror of the reference's ``class StereoMatching`` interface (stereoMatching.h:46-2738).

Same names, argument meaning and call order as ``main_.cpp`` uses them (main_.cpp:138-172):

    StereoMatching.costcalculation = "censusGrad"      # static selectors (h:51-53, main:15-17)
    param = StereoMatching.Parameters(maxDisp, h, w, lamCen, lamG, M, lamc, ts, csvName, disSc)
    sm = StereoMatching(I1_c, I2_c, I1, I2, DT, all_mask, nonocc_mask, disc_mask, param)
    sm.costCalculate()                                  # cost + CBCA (cpp:945-1021)
    SolveAll([sm], 1, 0.3)                              # cpp:2142-2208
    sm.dispOptimize()                                   # SGM + WTA (cpp:1046-1136)
    if StereoMatching.Do_refine: sm.refine()            # cpp:1138-1511 (main:165-166)
    disparity = sm.DP[0]                                # int16 H x W, -1 = invalid

All compute runs in libsm_hip.so on the GPU (no CPU fallback).  Errors are raised as
``SMError`` (the reference threw cv::Exception / called exit()).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence

import numpy as np

from . import _capi
from .evaluate import cal_err


class StereoMatching:
    # static std::string selectors (h:51-54); process-global in the reference, read at ctor time here
    costcalculation: str = "censusGrad"
    aggregation: str = "CBCA"
    optimization: str = "sgm"
    object: str = ""

    # compile-time switches the hot path reads (h:57-83); like the reference's static consts they
    # are read when an object is constructed (set StereoMatching.Do_refine = True before it)
    Do_refine = False
    Do_LRConsis = True
    # `#define MY_GUIDE` (h:38, commented out in the shipped build): guideFilter's form, False =
    # cv::ximgproc::guidedFilter (cpp:4513), True = guideFilterCore_matlab (cpp:4509)
    MY_GUIDE = False
    Do_regionVote = True
    Do_properIpol = True
    Do_lastMedianBlur = True

    class Parameters:
        """StereoMatching::Parameters (h:85-351): the fields the hot path reads."""

        def __init__(self, maxDisp: int, h: int, w: int, lamCen: int = 13, lamG: int = 1, M: int = 2,
                     lamc: int = 109, ts: int = 10, errCsvName: str = "", disSc: int = 1):
            self.numDisparities = maxDisp + 1          # h:209
            self.W_U, self.W_V = 4, 3                  # h:206-207
            self.errorThreshold = 1                    # h:225
            self.census_channel = 1                    # h:229
            self.censusFunc = 3                        # h:244
            self.gradFuse_adpWgt = True                # h:245
            self.grad_use2direc = True                 # h:246
            self.cbca_minArmL = 1                      # h:259
            self.cbca_iterationNum = 2                 # h:260
            self.cbca_intersect = True                 # h:262
            self.cbca_crossL = [17, 23, 34]            # h:263-265
            self.cbca_crossL_out = [34, 23, 34]        # h:266-268
            self.cbca_cTresh = [20, 30, 30]            # h:269-271
            self.cbca_cTresh_out = [6, 0, 0]           # h:272-274
            self.sgm_scanNum = 4                       # h:236 (the reference hard-codes 4, cpp:6214)
            self.sgm_P1, self.sgm_P2 = 1.0, 3.0        # ctor override for CBCA (cpp:2089-2091)
            self.sgm_corDifThres = 15                  # h:239
            self.sgm_reduCoeffi1 = 4                   # h:240
            self.lamCen, self.lamG = lamCen, lamG      # h:340-341
            self.ts, self.disSc = ts, disSc
            self.errCsvName = errCsvName
            self.vmTop_Num = M
            self.vmTop_thres = lamc * 0.01
            self.rows, self.cols = h, w
            self.LRmaxDiff = 0.0                       # h:212
            self.DISP_OCC = -2 * 16                    # h:216
            self.region_vote_nums = 2                  # h:306
            self.rv_ratio, self.rv_s = 0.4, 20         # refine(): rv_ratio[] / rv_s[] (cpp:1400-1401)

        def to_c(self, cost: str, aggregation: str, optimization: str, batch: int = 1,
                 compute_right_view: bool = False, keep_final_volume: bool = False,
                 do_refine: bool = False, switches=(True, True, True), my_guide: bool = False,
                 lr_consis: bool = True) -> _capi.sm_params:
            if self.censusFunc not in (0, 3):
                raise ValueError("censusFunc must be 0 (plain census) or 3 (census + ring bits)")
            p = _capi.default_params(self.numDisparities - 1, self.rows, self.cols)
            p.cost_method = _capi.COST_METHODS[cost]
            p.aggregation = _capi.AGGREGATIONS[aggregation]
            p.optimization = _capi.OPTIMIZATIONS[optimization]
            p.census_ring = 1 if self.censusFunc == 3 else 0
            p.lam_cen, p.lam_g = float(self.lamCen), float(self.lamG)
            p.grad_adaptive = int(self.gradFuse_adpWgt)
            # calArms divides the arm limits by the level's scale (cpp:5367-5371)
            sc = self.disSc if self.disSc > 1 else 1
            p.arm_l, p.arm_l_out = int(self.cbca_crossL[0] / sc), int(self.cbca_crossL_out[0] / sc)
            p.arm_c_thresh, p.arm_c_thresh_out = self.cbca_cTresh[0], self.cbca_cTresh_out[0]
            p.arm_min_l = self.cbca_minArmL
            p.cbca_iterations = self.cbca_iterationNum
            p.sgm_paths = self.sgm_scanNum
            p.sgm_cor_dif_thres = self.sgm_corDifThres
            p.sgm_redu_coeff = self.sgm_reduCoeffi1
            p.batch_capacity = batch
            p.compute_right_view = int(compute_right_view)
            p.keep_final_volume = int(keep_final_volume)
            p.do_refine = int(do_refine)
            p.lr_max_diff = float(self.LRmaxDiff)
            p.disp_occ = int(self.DISP_OCC)
            p.region_vote_nums = int(self.region_vote_nums)
            p.rv_ratio, p.rv_s = float(self.rv_ratio), int(self.rv_s)
            p.do_region_vote, p.do_proper_ipol, p.do_last_median_blur = (int(x) for x in switches)
            p.gf_mode = 1 if my_guide else 0
            p.lr_consis = int(lr_consis)
            return p

    def __init__(self, I1_c, I2_c, I1_g, I2_g, DT=None, all_mask=None, nonocc_mask=None, disc_mask=None,
                 param: Optional["StereoMatching.Parameters"] = None, device: int = 0,
                 keep_final_volume: bool = False):
        """StereoMatching::StereoMatching (cpp:2058-2110).  Images: BGR u8 HxWx3, gray u8 HxW."""
        I1_c, I2_c = np.ascontiguousarray(I1_c, np.uint8), np.ascontiguousarray(I2_c, np.uint8)
        I1_g, I2_g = np.ascontiguousarray(I1_g, np.uint8), np.ascontiguousarray(I2_g, np.uint8)
        h, w = I1_c.shape[:2]
        for im, nd in ((I1_c, 3), (I2_c, 3), (I1_g, 2), (I2_g, 2)):
            if im.ndim != nd or im.shape[:2] != (h, w) or (nd == 3 and im.shape[2] != 3):
                raise ValueError("images must be HxWx3 (colour) and HxW (gray) of one size")
        if param is None:
            raise ValueError("param is required")
        self.h_, self.w_ = h, w
        self.d_ = param.numDisparities
        self.param_ = param
        self.DT = DT
        self.I_mask = [nonocc_mask, all_mask, disc_mask]   # cpp:2073-2075
        self.I_c, self.I_g = [I1_c, I2_c], [I1_g, I2_g]
        self.DP: List[Optional[np.ndarray]] = [None, None]
        self._lib = _capi.load()
        if self.Do_refine and not self.Do_LRConsis:
            raise ValueError("Do_refine needs Do_LRConsis (refine() starts with the LR check, cpp:1364)")
        p = param.to_c(self.costcalculation, self.aggregation, self.optimization, my_guide=self.MY_GUIDE,
                       compute_right_view=self.Do_LRConsis and self.Do_refine,
                       keep_final_volume=keep_final_volume, do_refine=self.Do_refine, lr_consis=self.Do_LRConsis,
                       switches=(self.Do_regionVote, self.Do_properIpol, self.Do_lastMedianBlur))
        self._refine_on = bool(self.Do_refine)
        self._so_views2 = self.optimization == "so" and bool(self.Do_LRConsis)   # as passed to sm_create
        p.rows, p.cols = h, w
        ctx = C.c_void_p()
        st = self._lib.sm_create(C.byref(ctx), C.byref(p), device)
        self._ctx = ctx
        _capi.check(self._lib, ctx, st, "sm_create")
        st = self._lib.sm_set_images(ctx, _capi.ptr(I1_c), _capi.ptr(I2_c), w * 3,
                                     _capi.ptr(I1_g), _capi.ptr(I2_g), w)
        _capi.check(self._lib, ctx, st, "sm_set_images")

    def __del__(self):
        ctx = getattr(self, "_ctx", None)
        if ctx is not None and ctx.value:
            self._lib.sm_destroy(ctx)
            self._ctx = None

    # -- pipeline stages ---------------------------------------------------------------
    def costCalculate(self):
        """Cost volume + aggregation (cpp:945-1021)."""
        _capi.check(self._lib, self._ctx, self._lib.sm_cost_calculate(self._ctx), "costCalculate")

    def dispOptimize(self):
        """SGM (or WTA only) -> DP[0], and DP[1] when Do_refine; "so" -> DP[0] and DP[1]
        (num = Do_LRConsis ? 2 : 1, cpp:1093) (cpp:1046-1136)."""
        dp = np.empty((self.h_, self.w_), np.int16)
        _capi.check(self._lib, self._ctx, self._lib.sm_disp_optimize(self._ctx, _capi.ptr(dp)), "dispOptimize")
        self.DP[0] = dp
        if self._refine_on or self._so_views2:
            d1 = np.empty((self.h_, self.w_), np.int16)
            _capi.check(self._lib, self._ctx, self._lib.sm_get_disp(self._ctx, 1, _capi.ptr(d1)), "DP[1]")
            self.DP[1] = d1
        return dp

    def refine(self):
        """refine() (cpp:1138-1511): LR check against DP[1], region votes, proper interpolation,
        3x3 median -> DP[0].  Needs Do_refine = True when the object was constructed."""
        dp = np.empty((self.h_, self.w_), np.int16)
        _capi.check(self._lib, self._ctx, self._lib.sm_refine(self._ctx, _capi.ptr(dp)), "refine")
        self.DP[0] = dp
        return dp

    def pipeline(self):
        """pipeline() (cpp:1950-1981): costCalculate -> dispOptimize (no SolveAll)."""
        self.costCalculate()
        return self.dispOptimize()

    # -- state readback ------------------------------------------------------------------
    @property
    def vm(self) -> List[np.ndarray]:
        out = []
        for view in (0, 1):
            a = np.empty((self.h_, self.w_, self.d_), np.float32)
            st = self._lib.sm_get_volume(self._ctx, view, _capi.ptr(a))
            if st == _capi.SM_OK:
                out.append(a)
            elif view == 0:
                _capi.check(self._lib, self._ctx, st, "vm[0]")
        return out

    @property
    def HVL(self) -> List[np.ndarray]:
        out = []
        for view in (0, 1):
            a = np.empty((self.h_, self.w_, 4), np.uint16)
            _capi.check(self._lib, self._ctx, self._lib.sm_get_arms(self._ctx, view, _capi.ptr(a)), "HVL")
            out.append(a)
        return out

    def census_codes(self, view: int) -> np.ndarray:
        a = np.empty((self.h_, self.w_, 2), np.uint64)
        _capi.check(self._lib, self._ctx, self._lib.sm_get_census(self._ctx, view, _capi.ptr(a)), "census")
        return a

    def calErr(self, DP=None, thres: Optional[float] = None):
        """bad-t ratio / RMS per mask region (h:1748-1825) -> {region: (PBM, RMS)}."""
        DP = self.DP[0] if DP is None else DP
        t = self.param_.errorThreshold if thres is None else thres
        res = {}
        for name, m in zip(("nonocc", "all", "disc"), self.I_mask):
            if m is not None and self.DT is not None:
                res[name] = cal_err(DP, self.DT, m, t)
        return res


def SolveAll(smPyr: Sequence[StereoMatching], PY_LVL: int, REG_LAMBDA: float):
    """SolveAll (cpp:2142-2208).  PY_LVL = 1 (main_.cpp:131) scales vm; PY_LVL in [2, 8] combines
    the pyramid levels smPyr[0..PY_LVL-1] (built with pyrDown, main_.cpp:134-156) into smPyr[0]."""
    sm = smPyr[0]
    if int(PY_LVL) == 1:
        st = sm._lib.sm_solve_all(sm._ctx, 1, float(REG_LAMBDA))
    else:
        arr = (C.c_void_p * int(PY_LVL))(*[s._ctx.value for s in smPyr[:int(PY_LVL)]])
        st = sm._lib.sm_solve_all_pyr(arr, int(PY_LVL), float(REG_LAMBDA))
    _capi.check(sm._lib, sm._ctx, st, "SolveAll")


def pyrDown(img, device: int = 0) -> np.ndarray:
    """cv::pyrDown (main_.cpp:145-154), on the GPU: u8 H x W or H x W x 3 images (the inputs and
    masks) or a float32 H x W image (the ground truth DT, main_.cpp:149)."""
    lib = _capi.load()
    if np.asarray(img).dtype == np.float32:
        a = np.ascontiguousarray(img, np.float32)
        if a.ndim != 2:
            raise ValueError("float pyrDown takes a 1-channel image")
        rows, cols = a.shape
        out = np.empty(((rows + 1) // 2, (cols + 1) // 2), np.float32)
        st = lib.sm_pyr_down_f32(device, _capi.ptr(a), rows, cols, _capi.ptr(out))
        _capi.check(lib, None, st, "pyrDown")
        return out
    a = np.ascontiguousarray(img, np.uint8)
    rows, cols = a.shape[:2]
    ch = 1 if a.ndim == 2 else a.shape[2]
    out = np.empty(((rows + 1) // 2, (cols + 1) // 2) + a.shape[2:], np.uint8)
    st = lib.sm_pyr_down(device, _capi.ptr(a), rows, cols, ch, _capi.ptr(out))
    _capi.check(lib, None, st, "pyrDown")
    return out


def _is_device_tensor(a) -> bool:
    return type(a).__module__.startswith("torch") and getattr(a, "is_cuda", False)


def _to_numpy(a):
    return a.numpy() if type(a).__module__.startswith("torch") else a


class StereoBatch:
    """n independent pairs of one size through the whole main_.cpp sequence in one set of launches."""

    def __init__(self, max_disp: int, rows: int, cols: int, batch: int, device: int = 0, **overrides):
        self._lib = _capi.load()
        overrides.setdefault("batch_capacity", batch)
        p = _capi.default_params(max_disp, rows, cols, **overrides)
        self.params = p
        self.shape = (rows, cols, p.num_disparities)
        ctx = C.c_void_p()
        st = self._lib.sm_create(C.byref(ctx), C.byref(p), device)
        self._ctx = ctx
        _capi.check(self._lib, ctx, st, "sm_create")
        self.n = 0
        self._async_out = []   # buffers of download_async copies still in flight

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self._lib.sm_destroy(self._ctx)   # (waits for the context's streams)
            self._ctx = None
        getattr(self, "_async_out", []).clear()

    def __del__(self):
        self.close()

    def upload(self, lbgr, rbgr, lgray, rgray):
        """Stacked numpy arrays (host) or uint8 torch tensors already on the GPU (copied
        device-to-device; the caller's stream is synchronized first)."""
        if all(_is_device_tensor(a) for a in (lbgr, rbgr, lgray, rgray)):
            import torch
            ts = [a.contiguous() for a in (lbgr, rbgr, lgray, rgray)]
            if any(t.dtype != torch.uint8 for t in ts):
                raise TypeError("device images must be uint8 tensors")
            torch.cuda.current_stream(ts[0].device).synchronize()
            ptrs = [C.c_void_p(t.data_ptr()) for t in ts]
            n = ts[0].shape[0]
        else:
            arrs = [np.ascontiguousarray(_to_numpy(a), np.uint8) for a in (lbgr, rbgr, lgray, rgray)]
            ptrs = [_capi.ptr(a) for a in arrs]
            n = arrs[0].shape[0]
        st = self._lib.sm_upload_batch(self._ctx, n, *ptrs)
        _capi.check(self._lib, self._ctx, st, "sm_upload_batch")
        self.n = n

    def upload_async(self, lbgr, rbgr, lgray, rgray):
        """sm_upload_batch_async: contiguous uint8 device tensors (or page-locked host tensors)
        copied in behind the previous pipelined call's groups, without a join or a host wait.
        The sources must stay unchanged until upload_wait() returns."""
        ts = [a.contiguous() for a in (lbgr, rbgr, lgray, rgray)]
        import torch
        if any(t.dtype != torch.uint8 for t in ts):
            raise TypeError("images must be uint8 tensors")
        if any(t.data_ptr() != a.data_ptr() for t, a in zip(ts, (lbgr, rbgr, lgray, rgray))):
            raise ValueError("upload_async needs contiguous tensors (a copy would be freed before the upload)")
        n = ts[2].shape[0]
        if tuple(ts[2].shape[1:]) != self.shape[:2] or tuple(ts[0].shape[1:]) != self.shape[:2] + (3,):
            raise ValueError("upload_async: image shape differs from the context's")
        st = self._lib.sm_upload_batch_async(self._ctx, n, *[C.c_void_p(t.data_ptr()) for t in ts])
        _capi.check(self._lib, self._ctx, st, "sm_upload_batch_async")
        self.n = n

    def upload_wait(self):
        _capi.check(self._lib, self._ctx, self._lib.sm_upload_wait(self._ctx), "upload_wait")

    def download_wait(self, back: int = 0):
        """Host wait for the copies of the last (back 0) or previous (back 1) download_async."""
        _capi.check(self._lib, self._ctx, self._lib.sm_download_wait(self._ctx, int(back)), "download_wait")
        # (buffers of copies known done are released; the later one may still be in flight)
        del self._async_out[:max(0, len(self._async_out) - int(back))]

    def run(self, reg_lambda: float = 0.3, download: bool = True) -> Optional[np.ndarray]:
        out = np.empty((self.n, self.shape[0], self.shape[1]), np.int16) if download else None
        st = self._lib.sm_run(self._ctx, self.n, float(reg_lambda), _capi.ptr(out) if download else None)
        _capi.check(self._lib, self._ctx, st, "sm_run")
        return out

    def _map_dst(self, out, what: str):
        """C pointer of `out` after checking it can take the n int16 maps: a C-contiguous int16
        numpy array or torch tensor (host or device) of at least n*H*W elements."""
        need = self.n * self.shape[0] * self.shape[1]
        if type(out).__module__.startswith("torch"):
            import torch
            if out.dtype != torch.int16 or not out.is_contiguous() or out.numel() < need:
                raise ValueError(f"{what}: out must be a contiguous int16 tensor of at least n*H*W = {need} elements")
            return C.c_void_p(out.data_ptr())
        if not isinstance(out, np.ndarray) or out.dtype != np.int16 or not out.flags["C_CONTIGUOUS"] \
                or out.size < need:
            raise ValueError(f"{what}: out must be a C-contiguous int16 array of at least n*H*W = {need} elements")
        return _capi.ptr(out)

    def download(self, out=None):
        """The n int16 maps into a new numpy array, or into `out` (numpy, or an int16 torch
        tensor on the GPU: device-to-device copy)."""
        if out is None:
            out = np.empty((self.n, self.shape[0], self.shape[1]), np.int16)
        dst = self._map_dst(out, "download")
        _capi.check(self._lib, self._ctx, self._lib.sm_download_disp(self._ctx, self.n, dst), "download")
        return out

    def get_disp(self, view: int = 0) -> np.ndarray:
        """DP[view] of the first pair (sm_get_disp): DP[1] exists with do_refine or optimization "so"."""
        out = np.empty((self.shape[0], self.shape[1]), np.int16)
        _capi.check(self._lib, self._ctx, self._lib.sm_get_disp(self._ctx, view, _capi.ptr(out)), "get_disp")
        return out

    def download_async(self, out):
        """sm_download_disp_async: the n maps into `out` (page-locked host memory, e.g. a
        pin_memory torch tensor's numpy view, or device memory) on the copy stream; complete after
        synchronize().  The next run's map-writing kernels wait for the copy.  `out` is checked like
        download()'s and kept referenced until synchronize() or close(), so the copy never writes
        into a freed buffer."""
        dst = self._map_dst(out, "download_async")
        _capi.check(self._lib, self._ctx, self._lib.sm_download_disp_async(self._ctx, self.n, dst), "download_async")
        self._async_out.append(out)
        return out

    def copy_ceiling(self, nbytes: int, reps: int = 5):
        """sm_copy_ceiling: (best, median) GB/s of a dwordx4 device copy of nbytes (read + write)."""
        best, med = C.c_double(), C.c_double()
        st = self._lib.sm_copy_ceiling(self._ctx, int(nbytes), int(reps), C.byref(best), C.byref(med))
        _capi.check(self._lib, self._ctx, st, "copy_ceiling")
        return best.value, med.value

    def set_schedule(self, num_streams: int = 0, sub_batch: int = 0):
        """sm_set_schedule: num_streams / sub_batch for the following runs on the same allocations
        (0 / 0 = the auto default); maps are identical under every schedule."""
        st = self._lib.sm_set_schedule(self._ctx, int(num_streams), int(sub_batch))
        _capi.check(self._lib, self._ctx, st, "set_schedule")
        self.params.num_streams, self.params.sub_batch = int(num_streams), int(sub_batch)

    def placement(self):
        """The first run's volume placement trials (sm_params.placement_trials): (pipeline ms of
        each candidate set, index of the set kept), or ([], -1) when none ran."""
        buf = (C.c_double * 8)()
        nt = self._lib.sm_placement_trials_ms(self._ctx, buf, 8)
        return [round(buf[i], 3) for i in range(max(0, min(nt, 8)))], int(self._lib.sm_placement_kept(self._ctx))

    def synchronize(self):
        _capi.check(self._lib, self._ctx, self._lib.sm_synchronize(self._ctx), "sync")
        self._async_out.clear()

    def profile(self, on: bool = True):
        self._lib.sm_profile_enable(self._ctx, int(on))

    def profile_reset(self):
        self._lib.sm_profile_reset(self._ctx)

    def profile_read(self):
        names = C.create_string_buffer(64 * 48)
        launches = (C.c_int64 * 64)()
        total = (C.c_double * 64)()
        byts = (C.c_double * 64)()
        cnt = C.c_int32()
        st = self._lib.sm_profile_read(self._ctx, 64, names, launches, total, byts, C.byref(cnt))
        _capi.check(self._lib, self._ctx, st, "profile_read")
        out = {}
        for i in range(min(cnt.value, 64)):
            nm = names.raw[i * 48:(i + 1) * 48].split(b"\0", 1)[0].decode()
            out[nm] = {"launches": launches[i], "total_ms": total[i], "bytes_per_launch": byts[i]}
        return out


def run_batch_multi(batches: Sequence[StereoBatch], lbgr, rbgr, lgray, rgray, reg_lambda: float = 0.3) -> np.ndarray:
    """sm_run_batch_multi: n host pairs split into contiguous blocks over the contexts of
    `batches` (one per GPU, or several on one), one host thread per context; returns [n,H,W] int16."""
    lib = _capi.load()
    arrs = [np.ascontiguousarray(_to_numpy(a), np.uint8) for a in (lbgr, rbgr, lgray, rgray)]
    n, H, W = arrs[2].shape
    out = np.empty((n, H, W), np.int16)
    ctxs = (C.c_void_p * len(batches))(*[b._ctx.value for b in batches])
    st = lib.sm_run_batch_multi(ctxs, len(batches), n, *[_capi.ptr(a) for a in arrs], float(reg_lambda), _capi.ptr(out))
    _capi.check(lib, batches[0]._ctx, st, "sm_run_batch_multi")
    for b in batches:
        b.n = 0   # each context now holds only its own block
    return out

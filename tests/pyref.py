"""Independent numpy restatement of the reference hot path, for SMALL inputs only.

Written directly from the reference text (stereoMatching.cpp / .h), separately from the C
oracle, and used to cross-check it (tests/test_oracle.py).  float32 numpy ufuncs round every
operation individually (no FMA contraction), and np.add.accumulate is a strictly sequential
float32 prefix sum, so this reproduces the reference's arithmetic.  expf is the host libm's.
"""
from __future__ import annotations

import ctypes

import numpy as np

f32 = np.float32
_libm = ctypes.CDLL("libm.so.6")
_libm.expf.restype = ctypes.c_float
_libm.expf.argtypes = [ctypes.c_float]
_expf_vec = np.frompyfunc(lambda x: _libm.expf(float(x)), 1, 1)


def expf(a):
    return np.asarray(_expf_vec(np.asarray(a, f32)), dtype=f32)


def reflect101(p, n):
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p if p < 0 else 2 * n - p - 2
    return p


def census(gray, rv=3, ru=4, ring=True):
    """genCensusCode_NC_Sur (h:867-934) -> list of per-pixel bit strings (as python ints + length)."""
    H, W = gray.shape
    bits = np.zeros((H, W), dtype=object)
    ring_v = [-1, -1, -1, 0, 1, 1, 1, 0, -1]
    ring_u = [-1, 0, 1, 1, 1, 0, -1, -1, -1]
    for v in range(H):
        for u in range(W):
            c = int(gray[v, u])
            s = []
            for dv in range(-rv, rv + 1):
                for du in range(-ru, ru + 1):
                    s.append(1 if c < int(gray[reflect101(v + dv, H), reflect101(u + du, W)]) else 0)
            if ring:
                for i in range(8):
                    a = int(gray[reflect101(v + ring_v[i], H), reflect101(u + ring_u[i], W)])
                    b = int(gray[reflect101(v + ring_v[i + 1], H), reflect101(u + ring_u[i + 1], W)])
                    s.append(1 if a < b else 0)
            bits[v, u] = s
    return bits


def census_words(bits):
    """Pack a bit list the way h:886-930 does: 64-bit words, MSB first, last word right-aligned."""
    H, W = bits.shape
    L = len(bits[0, 0])
    nw = (L + 63) // 64
    out = np.zeros((H, W, nw), np.uint64)
    for v in range(H):
        for u in range(W):
            s = bits[v, u]
            for k in range(nw):
                chunk = s[64 * k:64 * (k + 1)]
                val = 0
                for bit in chunk:
                    val = (val << 1) | bit
                out[v, u, k] = val
    return out


def census_cost(bitsL, bitsR, D, view=0):
    H, W = bitsL.shape
    L = len(bitsL[0, 0])
    out = np.empty((H, W, D), f32)
    for v in range(H):
        for u in range(W):
            for d in range(D):
                lp, rp = (u + d, u) if view == 1 else (u, u - d)
                if lp >= W or rp < 0:
                    out[v, u, d] = f32(L)
                else:
                    out[v, u, d] = f32(sum(a != b for a, b in zip(bitsL[v, lp], bitsR[v, rp])))
    return out


def grads(gray):
    g = gray.astype(np.int32)
    gx = np.empty(g.shape, f32)
    gx[:, 1:-1] = (0.5 * (g[:, 2:] - g[:, :-2])).astype(f32)
    gx[:, 0] = g[:, 1] - g[:, 0]
    gx[:, -1] = g[:, -1] - g[:, -2]
    gy = np.empty(g.shape, f32)
    gy[1:-1] = (0.5 * (g[2:] - g[:-2])).astype(f32)
    gy[0] = g[1] - g[0]
    gy[-1] = g[-1] - g[-2]
    return gx, gy


def arms(bgr, L=17, L_out=34, cT=20, cT_out=6, minL=1):
    H, W, _ = bgr.shape
    I = bgr.astype(np.int32)
    out = np.zeros((H, W, 4), np.uint16)
    dirs = [(0, -1), (0, 1), (-1, 0), (1, 0)]
    for k, (dv, du) in enumerate(dirs):
        for v in range(H):
            for u in range(W):
                n = 0
                for arm in range(1, L_out + 1):
                    va, ua = v + arm * dv, u + arm * du
                    if not (0 <= va < H and 0 <= ua < W):
                        break
                    prev = I[v + (arm - 1) * dv, u + (arm - 1) * du]
                    cur = I[va, ua]
                    thr = cT if arm <= L else cT_out
                    if np.any(np.abs(cur - prev) > cT) or np.any(np.abs(I[v, u] - cur) > thr):
                        break
                    n = arm
                if n < minL:
                    n = 0
                    for ln in range(minL, -1, -1):
                        if 0 <= u + ln * du < W and 0 <= v + ln * dv < H:
                            n = ln
                            break
                out[v, u, k] = n
    return out


def grad_cost(gx0, gx1, gy0, gy1, arm, D, view=0, trunc=f32(500)):
    H, W = gx0.shape
    oor = f32(np.sqrt(2.0 * float(trunc) ** 2))
    out = np.empty((H, W, D), f32)
    sH = np.minimum(arm[..., 0], arm[..., 1]).astype(f32)
    sV = np.minimum(arm[..., 2], arm[..., 3]).astype(f32)
    sH[sH == 0] = 1
    sV[sV == 0] = 1
    a = (sH / (sH + sV)).astype(f32)
    one_m_a = (f32(1) - a).astype(f32)
    for d in range(D):
        for u in range(W):
            u0, u1 = (u + d, u) if view == 1 else (u, u - d)
            if u0 >= W or u1 < 0:
                out[:, u, d] = oor
                continue
            dx = np.minimum(np.abs(gx0[:, u0] - gx1[:, u1]), trunc).astype(f32)
            dy = np.minimum(np.abs(gy0[:, u0] - gy1[:, u1]), trunc).astype(f32)
            out[:, u, d] = (a[:, u] * dx).astype(f32) + (one_m_a[:, u] * dy).astype(f32)
    return out


def ad_cost(bgrL, bgrR, D, trunc, view=0):
    H, W, _ = bgrL.shape
    out = np.empty((H, W, D), f32)
    L = bgrL.astype(f32)
    R = bgrR.astype(f32)
    for d in range(D):
        for u in range(W):
            uL, uR = (u + d, u) if view == 1 else (u, u - d)
            if uL >= W or uR < 0:
                out[:, u, d] = f32(trunc)
                continue
            s = np.abs(L[:, uL] - R[:, uR]).sum(axis=1, dtype=f32)
            out[:, u, d] = np.minimum((s / f32(3)).astype(f32), f32(trunc))
    return out


def fuse(vm0, vm1, lam0, lam1):
    e0 = expf((-vm0 / f32(lam0)).astype(f32))
    e1 = expf((-vm1 / f32(lam1)).astype(f32))
    return ((f32(2) - e0).astype(f32) - e1).astype(f32)


def isect(aL, aR, D, view=0):
    """HVL_INTERSECTION[view] (cpp:2794-2845): view 0 pairs left u with right u - d, view 1 left
    u + d with right u; pairs falling outside the image stay 0 (memset)."""
    H, W, _ = aL.shape
    out = np.zeros((H, W, D, 4), np.int32)
    for d in range(D):
        if d < W:
            if view == 0:
                out[:, d:, d, :] = np.minimum(aL[:, d:, :], aR[:, :W - d, :])
            else:
                out[:, :W - d, d, :] = np.minimum(aL[:, d:, :], aR[:, :W - d, :])
    return out


def cbca(vm, aL, aR, iters=2, view=0):
    H, W, D = vm.shape
    A = isect(aL, aR, D, view)
    vm = vm.copy()
    vv, uu, dd = np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij")

    def pass1d(vm, area, horiz):
        axis = 1 if horiz else 0
        S = np.add.accumulate(vm, axis=axis, dtype=f32)
        Ar = np.add.accumulate(area, axis=axis)
        tail = A[..., 0] if horiz else A[..., 2]
        head = A[..., 1] if horiz else A[..., 3]
        if horiz:
            hi = (vv, uu + head, dd)
            pt = uu - tail - 1
            ti = (vv, np.maximum(pt, 0), dd)
        else:
            hi = (vv + head, uu, dd)
            pt = vv - tail - 1
            ti = (np.maximum(pt, 0), uu, dd)
        inner = pt >= 0
        out = np.where(inner, (S[hi] - S[ti]).astype(f32), S[hi]).astype(f32)
        ao = np.where(inner, Ar[hi] - Ar[ti], Ar[hi])
        return out, ao

    for it in range(iters):
        area = np.ones((H, W, D), np.int64)
        order = (True, False) if it % 2 == 0 else (False, True)
        for horiz in order:
            vm, area = pass1d(vm, area, horiz)
        vm = (vm / area.astype(f32)).astype(f32)
    return vm


def solve_all(vm, lam=f32(0.3)):
    m = f32(f32(1) + f32(lam))
    w = f32(1.0 / float(m))
    return (f32(0) + (w * vm).astype(f32)).astype(f32)


def sgm(vm, bgrL, paths=4, P1=f32(1), P2=f32(3), thres=15, redu=4):
    H, W, D = vm.shape
    RV = [+1, -1, 0, 0, +1, +1, -1, -1]
    RU = [0, 0, +1, -1, -1, +1, +1, -1]
    I = bgrL.astype(np.int32)
    BIG = np.finfo(f32).max
    acc = np.zeros_like(vm)
    for i in range(paths):
        rv, ru = RV[i], RU[i]
        Lr = np.empty_like(vm)
        vs = range(H - 1, -1, -1) if (rv > 0 or (rv == 0 and ru > 0)) else range(H)
        us = list(range(W - 1, -1, -1)) if (rv > 0 or (rv == 0 and ru > 0)) else list(range(W))
        for v in vs:
            for u in us:
                pv, pu = v + rv, u + ru
                if not (0 <= pv < H and 0 <= pu < W):
                    Lr[v, u] = vm[v, u]
                    continue
                D1 = int(np.max(np.abs(I[v, u] - I[pv, pu])))
                p1, p2 = f32(P1), f32(P2)
                if D1 > thres:
                    p1, p2 = f32(p1 / f32(redu)), f32(p2 / f32(redu))
                fore = Lr[pv, pu]
                m = fore.min()
                p1 = f32(p1 - m)
                S1 = (fore - m).astype(f32)
                S2 = np.full(D, BIG, f32)
                S2[1:] = (fore[:-1] + p1).astype(f32)
                S3 = np.full(D, BIG, f32)
                S3[:-1] = (fore[1:] + p1).astype(f32)
                mm = np.minimum(np.minimum(S1, S2), np.minimum(S3, np.full(D, p2, f32)))
                Lr[v, u] = (vm[v, u] + mm).astype(f32)
        acc = (acc + Lr).astype(f32)
    return acc


def wta(vm):
    H, W, D = vm.shape
    out = np.full((H, W), -1, np.int16)
    BIG = np.finfo(f32).max
    for v in range(H):
        for u in range(W):
            best = BIG
            for d in range(D):
                if best > vm[v, u, d]:
                    best = vm[v, u, d]
                    out[v, u] = d
    return out


def lr_check(d0, d1, maxdiff=f32(0)):
    """LRConsistencyCheck_normal (cpp:2262-2282)."""
    H, W = d0.shape
    out = d0.copy()
    uu = np.broadcast_to(np.arange(W), (H, W))
    d = d0.astype(np.int64)
    src = uu - d
    ok = (d >= 0) & (src >= 0)
    partner = np.where(ok, np.take_along_axis(d1.astype(np.int64), np.clip(src, 0, W - 1), axis=1), 0)
    bad = ~ok | (np.abs(d - partner).astype(f32) > f32(maxdiff))
    out[bad] = -1
    return out


def region_vote(dp, aL, D, ratio=f32(0.4), s=20):
    """regionVote_my (cpp:7219-7277): histogram of the valid disparities in the cross region,
    first maximum, integer hist/validNum compared with the float ratio (cpp:7270)."""
    H, W = dp.shape
    res = dp.copy()
    for v in range(H):
        for u in range(W):
            if dp[v, u] >= 0:
                continue
            vals = []
            for vn in range(v - int(aL[v, u, 2]), v + int(aL[v, u, 3]) + 1):
                row = dp[vn, u - int(aL[vn, u, 0]): u + int(aL[vn, u, 1]) + 1]
                vals.append(row[row >= 0])
            vals = np.concatenate(vals).astype(np.int64)
            if vals.size <= s:
                continue
            hist = np.bincount(vals, minlength=D)
            most = int(np.argmax(hist))   # first maximum
            if f32(int(hist[most]) // int(vals.size)) >= f32(ratio):
                res[v, u] = most
    return res


def proper_ipol(dp, bgr, occ=-32, depth=20):
    """properIpol (cpp:7395-7490)."""
    DW = [0, 2, 2, 2, 0, -2, -2, -2, 1, 2, 2, 1, -1, -2, -2, -1]
    DH = [2, 2, 0, -2, -2, -2, 0, 2, 2, 1, -1, -2, -2, -1, 1, 2]
    tdiv = lambda a, b: int(a / b)   # C truncating division
    H, W = dp.shape
    I = bgr.astype(np.int64)
    out = dp.copy()
    for v in range(H):
        for u in range(W):
            if dp[v, u] >= 0:
                continue
            found = []   # (direction order) disparity, colour difference
            for k in range(16):
                pv, pu = v, u
                for dep in range(depth):
                    if dep % 2 == 0:
                        pu += tdiv(DW[k], 2)
                        pv += tdiv(DH[k], 2)
                    else:
                        pu += DW[k] - tdiv(DW[k], 2)
                        pv += DH[k] - tdiv(DH[k], 2)
                    if not (0 <= pu < W and 0 <= pv < H):
                        break
                    if dp[pv, pu] >= 0:
                        found.append((int(dp[pv, pu]), int(np.max(np.abs(I[v, u] - I[pv, pu])))))
                        break
            if dp[v, u] == occ:
                if found:
                    out[v, u] = min(f[0] for f in found)
            else:
                cand = [f for f in found if f[1] < 255]
                if cand:
                    best = min(range(len(cand)), key=lambda i: (cand[i][1], i))
                    out[v, u] = cand[best][0]
    return out


def median3(dp):
    """cv::medianBlur(src, dst, 3) with replicated borders."""
    H, W = dp.shape
    P = np.pad(dp, 1, mode="edge")
    stack = np.stack([P[i:i + H, j:j + W] for i in range(3) for j in range(3)])
    return np.sort(stack, axis=0)[4].astype(np.int16)


def refine(d0, d1, aL, bgrL, D, nums=2):
    """refine(), cpp:1347-1510 with the default stage switches (h:72-81)."""
    d = lr_check(d0, d1)
    for _ in range(nums):
        d = region_vote(d, aL, D)
    for _ in range(nums):
        d = proper_ipol(d, bgrL)
    return median3(d)


def pipeline(pair, max_disp, cost="censusGrad", aggregate=True, solve=True, optimize=True, paths=4,
             refine_on=False):
    """Default main_.cpp sequence; returns dict of stage volumes and the disparity map.
    refine_on: Do_refine = 1 (both views through CBCA / SolveAll / SGM / WTA, then refine())."""
    D = max_disp + 1
    lb, rb, lg, rg = pair["lbgr"], pair["rbgr"], pair["lgray"], pair["rgray"]
    out = {}
    if cost == "AD":
        vm = ad_cost(lb, rb, D, 20)
    else:
        bl, br = census(lg), census(rg)
        cen = census_cost(bl, br, D)
        if cost == "Census":
            vm = cen
        elif cost == "ADCensus":
            vm = fuse(ad_cost(lb, rb, D, 1000), cen, 10, 30)
        else:
            gx0, gy0 = grads(lg)
            gx1, gy1 = grads(rg)
            aL = arms(lb)
            vm = fuse(cen, grad_cost(gx0, gx1, gy0, gy1, aL, D), 13, 1)
    out["cost"] = vm
    if aggregate:
        vm = cbca(vm, arms(lb), arms(rb))
    out["agg"] = vm
    if solve:
        vm = solve_all(vm)
    if optimize:
        vm = sgm(vm, lb, paths=paths)
    out["final"] = vm
    out["disp"] = wta(vm)
    if refine_on:
        assert cost == "censusGrad"
        gx0, gy0 = grads(lg)
        gx1, gy1 = grads(rg)
        v1 = fuse(census_cost(census(lg), census(rg), D, view=1),
                  grad_cost(gx0, gx1, gy0, gy1, arms(rb), D, view=1), 13, 1)
        if aggregate:
            v1 = cbca(v1, arms(lb), arms(rb), view=1)
        out["agg_right"] = v1
        if solve:
            v1 = solve_all(v1)
        if optimize:
            v1 = sgm(v1, rb, paths=paths)
        out["disp_right"] = wta(v1)
        out["disp_raw"] = out["disp"]
        out["disp"] = refine(out["disp"], out["disp_right"], arms(lb), lb, D)
    return out


# ---- cross-scale pyramid (main_.cpp:131-158, SolveAll cpp:2142-2208 with PY_LVL > 1) ----------

def pyr_down(img):
    """cv::pyrDown (u8, BORDER_REFLECT_101): separable 1-4-6-4-1, (sum + 128) >> 8."""
    a = img.astype(np.int64)
    rows, cols = a.shape[:2]
    pad = [(2, 2), (2, 2)] + [(0, 0)] * (a.ndim - 2)
    P = np.pad(a, pad, mode="reflect")          # numpy 'reflect' == REFLECT_101
    k = [1, 4, 6, 4, 1]
    dr, dc = (rows + 1) // 2, (cols + 1) // 2
    rowsum = sum(k[j] * P[:, j:j + 2 * dc:2] for j in range(5))      # columns 2x + j - 2
    tot = sum(k[i] * rowsum[i:i + 2 * dr:2] for i in range(5))       # rows 2y + i - 2
    return ((tot + 128) >> 8).astype(np.uint8)


def pyr_weights(L, lam=f32(0.3)):
    """regInv(0, :) of SolveAll's float regularisation matrix via OpenCV's small-matrix invert."""
    lam = f32(lam)
    M = np.zeros((L, L), np.float32)
    for s in range(L):
        if s == 0:
            M[s, s] = f32(1) + lam
            if L > 1:
                M[s, s + 1] = -lam
        elif s == L - 1:
            M[s, s] = f32(1) + lam
            M[s, s - 1] = -lam
        else:
            M[s, s] = f32(1) + f32(f32(2) * lam)
            M[s, s - 1] = -lam
            M[s, s + 1] = -lam
    if L > 3:
        return _lu_inv_row0(M)
    m = M.astype(np.float64)
    if L == 1:
        return np.array([f32(1.0 / m[0, 0])], np.float32)
    if L == 2:
        d = 1.0 / (m[0, 0] * m[1, 1] - m[0, 1] * m[1, 0])
        return np.array([m[1, 1] * d, -m[0, 1] * d]).astype(np.float32)
    det = (m[0, 0] * (m[1, 1] * m[2, 2] - m[1, 2] * m[2, 1]) - m[0, 1] * (m[1, 0] * m[2, 2] - m[1, 2] * m[2, 0])
           + m[0, 2] * (m[1, 0] * m[2, 1] - m[1, 1] * m[2, 0]))
    d = 1.0 / det
    return np.array([(m[1, 1] * m[2, 2] - m[1, 2] * m[2, 1]) * d, (m[0, 2] * m[2, 1] - m[0, 1] * m[2, 2]) * d,
                     (m[0, 1] * m[1, 2] - m[0, 2] * m[1, 1]) * d]).astype(np.float32)


def _lu_inv_row0(M):
    """Row 0 of Mat::inv for n > 3 (DECOMP_LU): OpenCV's LUImpl<float> on a copy of M with the
    identity as right-hand side — partial pivoting, d = -1 / a_ii, row updates, back substitution,
    every float product and sum rounded on its own."""
    A = M.copy()
    n = A.shape[0]
    B = np.eye(n, dtype=np.float32)
    for i in range(n):
        k = i
        for j in range(i + 1, n):
            if abs(A[j, i]) > abs(A[k, i]):
                k = j
        if abs(A[k, i]) < f32(np.finfo(np.float32).eps * 10):
            raise ValueError("singular regularisation matrix")
        if k != i:
            A[[i, k], i:] = A[[k, i], i:]
            B[[i, k]] = B[[k, i]]
        d = f32(f32(-1) / A[i, i])
        for j in range(i + 1, n):
            alpha = f32(A[j, i] * d)
            for q in range(i + 1, n):
                A[j, q] = f32(A[j, q] + f32(alpha * A[i, q]))
            for q in range(n):
                B[j, q] = f32(B[j, q] + f32(alpha * B[i, q]))
    for i in range(n - 1, -1, -1):
        for j in range(n):
            s = B[i, j]
            for q in range(i + 1, n):
                s = f32(s - f32(A[i, q] * B[q, j]))
            B[i, j] = f32(s / A[i, i])
    return B[0].copy()


def solve_all_pyr(vms, lam=f32(0.3)):
    """vms[s]: level-s volume; returns the new level-0 volume."""
    L = len(vms)
    w = pyr_weights(L, lam)
    H, W, D = vms[0].shape
    yy, xx, dd = np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij")
    acc = np.zeros((H, W, D), np.float32)
    for s in range(L):
        acc = (acc + (w[s] * vms[s][yy, xx, dd]).astype(np.float32)).astype(np.float32)
        yy, xx, dd = yy // 2, xx // 2, (dd + 1) // 2
    return acc


def pipeline_pyr(pair, max_disp, L, paths=4):
    """main_.cpp:131-163 with PY_LEV = L (censusGrad + CBCA, no refine)."""
    lv = [dict(pair)]
    for _ in range(1, L):
        lv.append({k: pyr_down(v) for k, v in lv[-1].items() if k in ("lbgr", "rbgr", "lgray", "rgray")})
    vms, md, sc = [], max_disp, 1
    for p in lv:
        D = md + 1
        lb, rb, lg, rg = p["lbgr"], p["rbgr"], p["lgray"], p["rgray"]
        gx0, gy0 = grads(lg)
        gx1, gy1 = grads(rg)
        aL = arms(lb, L=17 // sc, L_out=34 // sc)
        aR = arms(rb, L=17 // sc, L_out=34 // sc)
        vm = fuse(census_cost(census(lg), census(rg), D), grad_cost(gx0, gx1, gy0, gy1, aL, D), 13, 1)
        vms.append(cbca(vm, aL, aR))
        md, sc = md // 2 + 1, sc * 2
    vm = solve_all_pyr(vms)
    vm = sgm(vm, pair["lbgr"], paths=paths)
    return wta(vm)


def so(vm, bgr):
    """so (cpp:6272-6394): row DP left to right with trace + backtracking; returns (vm, DP)."""
    H, W, D = vm.shape
    vm = vm.copy()
    I = bgr.astype(np.int64)
    BIG = np.finfo(f32).max
    trace = np.zeros((H, W, D), np.int64)
    dd = np.arange(D)
    for v in range(H):
        for u in range(1, W):
            s_ = f32(0)
            for ch in range(3):
                s_ = f32(s_ + f32(abs(int(I[v, u, ch]) - int(I[v, u - 1, ch]))))
            s_ = f32(s_ / f32(3))
            disc = s_ > 15
            Pn2 = f32(f32(1.2) / f32(2)) if disc else f32(1.2)
            Pn3 = f32(f32(3.6) / f32(2)) if disc else f32(3.6)
            pre = vm[v, u - 1]
            dc = int(np.argmin(pre))               # first minimum
            cm = f32(pre[dc] + Pn3)
            cminus = np.full(D, BIG, f32)
            cminus[1:] = (pre[:-1] + Pn2).astype(f32)
            cplus = np.full(D, BIG, f32)
            cplus[:-1] = (pre[1:] + Pn2).astype(f32)
            best = pre.copy()
            dmin = dd.copy()
            m = cminus < best
            best, dmin = np.where(m, cminus, best), np.where(m, dd - 1, dmin)
            m = cplus < best
            best, dmin = np.where(m, cplus, best), np.where(m, dd + 1, dmin)
            m = cm < best
            best, dmin = np.where(m, cm, best), np.where(m, dc, dmin)
            vm[v, u] = (vm[v, u] + best.astype(f32)).astype(f32)
            trace[v, u] = dmin
    DP = np.zeros((H, W), np.int16)
    for v in range(H):
        d = int(np.argmin(vm[v, W - 1]))
        DP[v, W - 1] = d
        for u in range(W - 1, 0, -1):
            d = int(trace[v, u, d])
            DP[v, u - 1] = d
    return vm, DP

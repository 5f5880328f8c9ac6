"""Independent numpy restatement of the GF (MY_GUIDE and ximgproc forms) and NL aggregators, written
from the reference text (ximgproc: from the published algorithm, see oracle/sm_oracle_agg.c), used to
cross-check oracle/sm_oracle_agg.c on small inputs (test infrastructure).

GF:  guideFilterCore_matlab (stereoMatching.cpp:4975-5104) with BoxFilter / CumSum
     (cpp:5107-5202), vectorised over the disparity axis in float32 / float64 as written.
NL:  NLCCA::aggreCV (NL/NLCCA.cpp:27-96): ctmf 3x3 median (clamped borders), 4-neighbour edge
     weights (max channel difference), stable sort, Kruskal, BFS from pixel 0, tree filter in float64.
"""
from __future__ import annotations

import numpy as np

F = np.float32


def box_filter(a: np.ndarray, r: int) -> np.ndarray:
    """BoxFilter(imSrc, r) over axes 0 (rows) and 1 (cols); extra trailing axes are independent."""
    a = a.astype(F)
    H, W = a.shape[:2]
    cy = np.empty_like(a)
    cy[0] = F(0) + a[0]
    for y in range(1, H):
        cy[y] = cy[y - 1] + a[y]
    t = np.empty_like(a)
    for y in range(H):
        plus = cy[y + r] if y < H - r else cy[H - 1]
        t[y] = plus if y < r + 1 else plus - cy[y - r - 1]
    cx = np.empty_like(a)
    cx[:, 0] = t[:, 0]
    for x in range(1, W):
        cx[:, x] = cx[:, x - 1] + t[:, x]
    out = np.empty_like(a)
    for x in range(W):
        plus = cx[:, x + r] if x < W - r else cx[:, W - 1]
        out[:, x] = plus if x < r + 1 else plus - cx[:, x - r - 1]
    return out


def guided_filter(vm: np.ndarray, bgr: np.ndarray, r: int = 9, eps: float = 1e-4) -> np.ndarray:
    H, W, D = vm.shape
    eps = F(eps)
    I = [bgr[..., c].astype(F) for c in range(3)]
    N = box_filter(np.ones((H, W), F), r)
    mI = [box_filter(I[c], r) / N for c in range(3)]
    var = []
    for c0 in range(3):
        for c1 in range(c0, 3):
            v = box_filter(I[c0] * I[c1], r) / N
            var.append(v - mI[c0] * mI[c1])
    a11, a12, a13 = (var[0] + eps).astype(np.float64), var[1].astype(np.float64), var[2].astype(np.float64)
    a21, a22, a23 = var[1].astype(np.float64), (var[3] + eps).astype(np.float64), var[4].astype(np.float64)
    a31, a32, a33 = var[2].astype(np.float64), var[4].astype(np.float64), (var[5] + eps).astype(np.float64)
    DET = a11 * (a33 * a22 - a32 * a23) - a21 * (a33 * a12 - a32 * a13) + a31 * (a23 * a12 - a22 * a13)
    DET = 1 / DET
    p = vm.astype(F)
    NN = N[..., None]
    mean_p = box_filter(p, r) / NN
    cov = [box_filter(I[c][..., None] * p, r) / NN - mI[c][..., None] * mean_p for c in range(3)]
    c0, c1, c2 = (x.astype(np.float64) for x in cov)
    e = lambda x: x[..., None]   # noqa: E731
    a = [
        (e(DET) * (c0 * e(a33 * a22 - a32 * a23) + c1 * e(a31 * a23 - a33 * a21) + c2 * e(a32 * a21 - a31 * a22))).astype(F),
        (e(DET) * (c0 * e(a32 * a13 - a33 * a12) + c1 * e(a33 * a11 - a31 * a13) + c2 * e(a31 * a12 - a32 * a11))).astype(F),
        (e(DET) * (c0 * e(a23 * a12 - a22 * a13) + c1 * e(a21 * a13 - a23 * a11) + c2 * e(a22 * a11 - a21 * a12))).astype(F),
    ]
    b = mean_p.copy()
    for c in range(3):
        b = b - a[c] * mI[c][..., None]
    q = box_filter(b, r) / NN
    for c in range(3):
        q = q + (box_filter(a[c], r) / NN) * I[c][..., None]
    return q.astype(F)


def _reflect(p: int, n: int) -> int:
    """OpenCV borderInterpolate(BORDER_REFLECT)."""
    if n == 1:
        return 0
    while p < 0 or p >= n:
        p = -p - 1 if p < 0 else 2 * n - 1 - p
    return p


def box_filter_cv(a: np.ndarray, r: int) -> np.ndarray:
    """OpenCV boxFilter(CV_32F, (2r+1)^2, normalize, BORDER_REFLECT) over axes 0 (rows) and 1 (cols),
    float64 running sums: RowSum (first window, then += S[i+k] - S[i]) and ColumnSum (k-1 rows, then
    s0 = SUM + Sp, out = float32(s0 * scale), SUM = s0 - Sm)."""
    a = a.astype(F)
    H, W = a.shape[:2]
    k = 2 * r + 1
    ext = a[:, [_reflect(j - r, W) for j in range(W + 2 * r)]].astype(np.float64)
    rs = np.empty(a.shape, np.float64)
    s = np.zeros(a.shape[:1] + a.shape[2:], np.float64)
    for i in range(k):
        s = s + ext[:, i]
    rs[:, 0] = s
    for i in range(W - 1):
        s = s + (ext[:, i + k] - ext[:, i])
        rs[:, i + 1] = s
    scale = 1.0 / (k * k)
    out = np.empty(a.shape, F)
    SUM = np.zeros(a.shape[1:], np.float64)
    for i in range(k - 1):
        SUM = SUM + rs[_reflect(i - r, H)]
    for y in range(H):
        s0 = SUM + rs[_reflect(y + r, H)]
        out[y] = (s0 * scale).astype(F)
        SUM = s0 - rs[_reflect(y - r, H)]
    return out


def guided_filter_cv(vm: np.ndarray, bgr: np.ndarray, r: int = 9, eps: float = 1e-4) -> np.ndarray:
    """cv::ximgproc::guidedFilter(I = BGR as float, p = every channel of vm, r, eps) in the structure
    of GuidedFilterImpl (float32 products and sums, the box filter above), written independently of
    oracle/sm_oracle_agg.c from the same description (its header)."""
    H, W, D = vm.shape
    eps = F(eps)
    I = [bgr[..., c].astype(F) for c in range(3)]
    mI = [box_filter_cv(I[c], r) for c in range(3)]
    sig = {}
    for i in range(3):
        for j in range(i, 3):
            v = box_filter_cv(I[i] * I[j], r) - mI[i] * mI[j]
            sig[i, j] = sig[j, i] = (v + eps) if i == j else v
    a = sig
    cof = {(0, 0): a[1, 1] * a[2, 2] - a[1, 2] * a[1, 2], (0, 1): a[0, 2] * a[1, 2] - a[0, 1] * a[2, 2],
           (0, 2): a[0, 1] * a[1, 2] - a[0, 2] * a[1, 1], (1, 1): a[0, 0] * a[2, 2] - a[0, 2] * a[0, 2],
           (1, 2): a[0, 1] * a[0, 2] - a[0, 0] * a[1, 2], (2, 2): a[0, 0] * a[1, 1] - a[0, 1] * a[0, 1]}
    det = (a[0, 0] * cof[0, 0] + a[0, 1] * cof[0, 1]) + a[0, 2] * cof[0, 2]
    inv = {}
    for (i, j), v in cof.items():
        inv[i, j] = inv[j, i] = v / det
    p = vm.astype(F)
    e = lambda x: x[..., None]   # noqa: E731
    mP = box_filter_cv(p, r)
    cov = [box_filter_cv(p * e(I[c]), r) - mP * e(mI[c]) for c in range(3)]
    al = []
    for gi in range(3):
        y = e(inv[gi, 0]) * cov[0]
        for k in (1, 2):
            y = y + e(inv[gi, k]) * cov[k]
        al.append(y)
    be = mP
    for gi in range(3):
        be = be - al[gi] * e(mI[gi])
    q = box_filter_cv(be, r)
    for gi in range(3):
        q = q + box_filter_cv(al[gi], r) * e(I[gi])
    return q.astype(F)


def nl_tree(bgr: np.ndarray):
    H, W = bgr.shape[:2]
    n = H * W
    pad = np.pad(bgr.astype(np.int32), ((1, 1), (1, 1), (0, 0)), mode="edge")
    win = np.stack([pad[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)])
    med = np.sort(win, axis=0)[4]
    flat = med.reshape(n, 3)
    eu, ev = [], []
    for y in range(H):
        for x in range(W - 1):
            eu.append(y * W + x)
            ev.append(y * W + x + 1)
    for x in range(W):
        for y in range(H - 1):
            eu.append(y * W + x)
            ev.append((y + 1) * W + x)
    eu, ev = np.array(eu), np.array(ev)
    w = np.abs(flat[ev] - flat[eu]).max(axis=1)
    order_e = np.argsort(w, kind="stable")
    comp = list(range(n))

    def find(x):
        while comp[x] != x:
            comp[x] = comp[comp[x]]
            x = comp[x]
        return x

    nbr = [[] for _ in range(n)]
    for e in order_e:
        u, v = int(eu[e]), int(ev[e])
        ru, rv = find(u), find(v)
        if ru != rv:
            comp[ru] = rv
            nbr[u].append((v, int(w[e])))
            nbr[v].append((u, int(w[e])))
    parent = [-1] * n
    weight = [0] * n
    children = [[] for _ in range(n)]
    parent[0] = 0
    order = [0]
    head = 0
    while head < len(order):
        p = order[head]
        head += 1
        for q, wq in nbr[p]:
            if parent[q] == -1:
                parent[q] = p
                weight[q] = wq
                children[p].append(q)
                order.append(q)
    assert len(order) == n
    return order, parent, weight, children


def nl_aggregate(vm: np.ndarray, bgr: np.ndarray, sigma: float = 0.1) -> np.ndarray:
    H, W, D = vm.shape
    n = H * W
    order, parent, weight, children = nl_tree(bgr)
    table = np.exp(-np.arange(256, dtype=np.float64) / (255 * max(0.01, sigma)))

    def filt(cost):
        up = cost.copy()
        for i in reversed(order):
            for ch in children[i]:
                up[i] = up[i] + up[ch] * table[weight[ch]]
        out = np.empty_like(cost)
        out[order[0]] = up[order[0]]
        for i in order[1:]:
            wv = table[weight[i]]
            out[i] = wv * (out[parent[i]] - wv * up[i]) + up[i]
        return out

    c = filt(vm.reshape(n, D).astype(np.float64))
    ones = filt(np.ones((n, 1), np.float64))
    res = c.astype(F) / ones.astype(F)
    return res.reshape(H, W, D).astype(F)

"""Diagnostic: checkpointed SGM (default build) vs the plain path sweeps (tools/abvar/libsm_hip_nock.so)
on the same inputs; prints where the kept final volumes differ (v, u, d) and by how much."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mystereomatching_amd import _capi, StereoBatch  # noqa: E402
from mystereomatching_amd import synthetic as S  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def final(lib, pair, md, paths):
    _capi._lib = None
    if lib:
        os.environ["SM_HIP_LIB"] = os.path.join(ROOT, "tools", "abvar", f"libsm_hip_{lib}.so")
    else:
        os.environ.pop("SM_HIP_LIB", None)
    H, W = pair["lgray"].shape
    sb = StereoBatch(md, H, W, 1, sgm_paths=paths, keep_final_volume=1)
    sb.upload(*(pair[k][None] for k in ("lbgr", "rbgr", "lgray", "rgray")))
    disp = sb.run(0.3)[0]
    vol = np.empty((H, W, md + 1), np.float32)
    _capi.check(sb._lib, sb._ctx, sb._lib.sm_get_volume(sb._ctx, 0, _capi.ptr(vol)), "get_volume")
    sb.close()
    return disp, vol


for (H, W, md, paths, idx) in [(41, 67, 23, 4, 11), (24, 32, 15, 4, 3), (29, 41, 15, 4, 530), (40, 300, 191, 8, 40)]:
    pair = S.make_pair(H, W, md + 1, idx)
    d0, v0 = final("", pair, md, paths)
    d1, v1 = final("nock", pair, md, paths)
    nd = int((d0 != d1).sum())
    print(f"H={H} W={W} D={md + 1} paths={paths}: map diffs {nd}", flush=True)
    if v0 is not None:
        b0, b1 = v0.view(np.uint32), v1.view(np.uint32)
        idxs = np.argwhere(b0 != b1)
        print(f"  volume diffs {len(idxs)}")
        for v, u, d in idxs[:12]:
            print(f"   v={v} u={u} d={d} ck={v0[v, u, d]!r} plain={v1[v, u, d]!r} (W-1-u={W - 1 - u}, H-1-v={H - 1 - v})")

"""End-to-end on a Middlebury-layout folder: PNG files -> dataset.load -> tools/sm_eval.run
(main_.cpp's sequence incl. refine / pyramid) -> calErr; maps bit-exact against the oracle."""
import importlib.util
import os

import numpy as np
import pytest

from mystereomatching_amd import dataset
from mystereomatching_amd import synthetic as S

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _tool():
    spec = importlib.util.spec_from_file_location("sm_eval", os.path.join(ROOT, "tools", "sm_eval.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


@pytest.mark.parametrize("refine,levels", [(False, 1), (True, 1), (False, 2)])
def test_eval_tool_on_png_folder(oracle, tmp_path, refine, levels):
    from PIL import Image
    H, W = 90, 120
    p = S.make_pair(H, W, 60, 17)
    d = tmp_path / "teddy"
    d.mkdir()
    Image.fromarray(p["lbgr"][..., ::-1]).save(d / "im2.png")
    Image.fromarray(p["rbgr"][..., ::-1]).save(d / "im6.png")
    Image.fromarray(np.clip(p["gt"] * 4, 0, 255).astype(np.uint8)).save(d / "disp2.png")
    Image.fromarray(p["nonocc"]).save(d / "nonocc.png")
    s = dataset.load(str(tmp_path), "teddy")
    dp, _ = _tool().run(s, refine, levels, 0)
    cfg = oracle.config(H, W, s.max_disp, do_refine=int(refine))
    ref = oracle.run_pyr(s.pair(), cfg, levels) if levels > 1 else oracle.run_ex(s.pair(), cfg)["disp"]
    np.testing.assert_array_equal(dp, ref)
    from mystereomatching_amd.evaluate import cal_err
    pbm, _ = cal_err(dp, s.gt, s.masks["nonocc"], 2.0)
    assert pbm < 0.2

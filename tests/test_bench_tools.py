"""Host logic of the measurement tools: how bench.py groups profile names into kernel symbols for
the roofline (the dominant kernel as rocprofv3 --stats ranks code objects) and how
tools/pmc_summary.py maps rocprofv3 kernel symbols back onto those profile names."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import bench  # noqa: E402
import pmc_summary  # noqa: E402


def test_kernel_symbol_groups():
    # middle plain SGM paths share one symbol (D > 128: one line per wave in every direction;
    # D <= 128: the vertical ones run k_sgm_rows); the checkpointed pairs' A passes share one too
    assert bench.kernel_symbol("sgm_path4", 192, 8) == bench.kernel_symbol("sgm_path5", 192, 8) == "k_sgm<mid>"
    assert bench.kernel_symbol("sgm_path1", 64, 8) == "k_sgm_rows<mid>"
    assert bench.kernel_symbol("sgm_path2", 64, 8) == "k_sgm<mid>"
    assert bench.kernel_symbol("sgm_ck_a01", 256, 4) == bench.kernel_symbol("sgm_ck_a23", 256, 4) == "k_sgm_ck<A>"
    assert bench.kernel_symbol("sgm_ck_a01_r", 256, 4) == "k_sgm_ck<A>"
    assert bench.kernel_symbol("sgm_ck_b01", 256, 4) == "sgm_ck_b01"
    assert bench.kernel_symbol("sgm_last_wta", 256, 4) == "sgm_last_wta"
    assert bench.kernel_symbol("cbca_v_norm_scan", 256, 4) == "cbca_v_norm_scan"
    assert bench.kernel_symbol("cbca_v_norm_scan_r", 256, 4) == "cbca_v_norm_scan_r"   # its own instantiation


def test_pmc_profile_names():
    seen = {}
    names = [pmc_summary.profile_name(s, seen) for s in (
        "void sm::k_cbca<true, 0, true, false, false, 0>(sm::CbcaArgs)",
        "void sm::k_cbca_nsv<false, false>(sm::CbcaArgs)",
        "void sm::k_cbca<true, 1, true, true, false, 0>(sm::CbcaArgs)",
        "void sm::k_sgm_ck<8, 16, 1, false, true>(sm::SgmArgs)",
        "void sm::k_sgm_ck<8, 32, 1, false, true>(sm::SgmArgs)",
        "void sm::k_sgm_ck<8, 16, 1, false, true>(sm::SgmArgs)",
        "void sm::k_sgm_ck<8, 34, 1, false, true>(sm::SgmArgs)",
        "void sm::k_cost<0, true, 3, false, true, 4>(sm::CostArgs)",
        # 8 paths' middle pair (CK_MID = 64)
        "void sm::k_sgm_ck<8, 96, 1, false, false>(sm::SgmArgs)")]
    assert names == ["cbca_h_scan", "cbca_v_norm_scan", "cbca_h_norm", "sgm_ck_a01", "sgm_ck_b01",
                     "sgm_ck_a23", "sgm_last_wta", "cost_volume", "sgm_ck_b23"]

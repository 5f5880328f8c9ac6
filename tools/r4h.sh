#!/bin/bash
# Round-4 GPU pass h: the checkpointed SGM with FLT_MAX in the checkpoint lanes past D: the
# diagnostic, the SGM parity tests, then the whole -m gpu suite.
set -o pipefail
O=gpurun_out/${1:-r4h}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u tools/ck_diag.py > $O/ck_diag.txt 2>&1; head -20 $O/ck_diag.txt
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py tests/test_gpu_agg.py -k "checkpointed or shapes_and_edge or fixture or golden or batch_maps or kitti or stages or prep_tiles" > $O/pytest_sgm.log 2>&1
rc=$?; tail -3 $O/pytest_sgm.log; grep -E "FAILED|ERROR" $O/pytest_sgm.log | head
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20

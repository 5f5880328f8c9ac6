set -o pipefail
# the diagonal SGM pair (4, 6) checkpointed (default) vs the three diagonal sweeps (nodiag)
O=gpurun_out/r6dg; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_agg.py tests/test_gpu_large_fixtures.py > $O/pytest.log 2>&1; rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/ab_inproc.py --workload kitti --rounds 6 --copies 2 base:num_streams=1,placement_trials=0 nodiag:num_streams=1,placement_trials=0 > $O/ab_kitti.txt 2>&1 || exit $?
grep -A3 "medians" $O/ab_kitti.txt | cut -c1-400

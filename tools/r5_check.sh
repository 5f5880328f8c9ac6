# parity of the CBCA sweeps first (small shapes), then the large fixtures
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "lag34 or golden" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/small.log 2>&1; rc=$?; tail -3 $O/small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_fixtures.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/large.log 2>&1; rc=$?; tail -3 $O/large.log; exit $rc

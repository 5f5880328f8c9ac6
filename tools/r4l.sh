#!/bin/bash
# Round-4 GPU pass l: the V NORM_SCAN sweep's scan stage reading at the norm stage's saved S1
# addresses (S2 at slot p mod R, one tile code copy): its parity tests first, then the whole -m gpu
# suite, same-process A/B against the previous sweep (noah) at full resolution and Teddy (one
# stream each, kernel times), the default bench (auto streams; per-kernel pass on one stream) and
# rocprofv3 kernel stats of `bench.py --streams 1` (the per-kernel pass's schedule).
set -o pipefail
O=gpurun_out/${1:-r4l}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_large_fixtures.py tests/test_gpu_parity.py -k "norm_scan or fixture or lag34 or golden" > $O/pytest_ns.log 2>&1
rc=$?; tail -2 $O/pytest_ns.log; grep -E "^FAILED|^ERROR" $O/pytest_ns.log | head; ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20; ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,step base:num_streams=1 noah:num_streams=1 > $O/ab_fr.txt 2>&1 && tail -3 $O/ab_fr.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels cbca,step base noah > $O/ab_teddy.txt 2>&1 && tail -3 $O/ab_teddy.txt \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cut -c1-300 $O/bench.json \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -12 $O/kt_kernel_stats.csv \
 && echo "r4l done"

#!/bin/bash
# Round-4 GPU pass b: the fast V NORM_SCAN sweep (NsV) and H NORM sweep (HNorm): the NORM_SCAN parity
# tests first, then the whole -m gpu suite, then same-process A/B against the generic sweeps
# (tools/abvar/libsm_hip_gen.so; nohn = NsV only)
# at full resolution and 1080p, then smoke + the default bench + rocprofv3 kernel stats.
set -o pipefail
O=gpurun_out/${1:-r4b}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT -m gpu tests/test_gpu_large_fixtures.py tests/test_gpu_parity.py -k "norm_scan or fixture" > $O/pytest_ns.log 2>&1 \
 ; tail -3 $O/pytest_ns.log; grep -E "FAILED|ERROR" $O/pytest_ns.log | head
grep -q " passed" $O/pytest_ns.log && ! grep -qE "FAILED|ERROR|Timeout" $O/pytest_ns.log || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1 ; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -q " passed" $O/pytest_gpu.log && ! grep -qE "FAILED|ERROR|Timeout" $O/pytest_gpu.log || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,cost,step base gen nohn expskip > $O/ab_fr.txt 2>&1 && tail -4 $O/ab_fr.txt \
 && $A --workload hd --rounds 4 --steps 2 --copies 1 --kernels cbca,step base gen nohn > $O/ab_hd.txt 2>&1 && tail -4 $O/ab_hd.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels cbca,step base base:fuse_norm_scan=1 gen > $O/ab_teddy.txt 2>&1 && tail -4 $O/ab_teddy.txt \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -14 $O/kt_kernel_stats.csv \
 && echo "r4b done"

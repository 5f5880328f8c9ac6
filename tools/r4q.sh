#!/bin/bash
# Round-4 GPU pass q: NsV with the pre-line zeroing hoisted into one uniform branch per tile
# (parity, the whole suite, A/B against the previous NsV = nsvprev), then two-stream pair groups
# at the smaller workloads (Teddy x16, KITTI x4).
set -o pipefail
O=gpurun_out/${1:-r4q}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_large_fixtures.py tests/test_gpu_parity.py -k "norm_scan or fixture or lag34 or golden" > $O/pytest_ns.log 2>&1
rc=$?; tail -2 $O/pytest_ns.log; grep -E "^FAILED" $O/pytest_ns.log | head; ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head -20; ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca_v,step base:num_streams=1 nsvprev:num_streams=1 rb:num_streams=1 > $O/ab_fr.txt 2>&1 && tail -3 $O/ab_fr.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels step base base:num_streams=2,sub_batch=8 base:num_streams=2,sub_batch=4 > $O/ab_teddy.txt 2>&1 && tail -4 $O/ab_teddy.txt \
 && $A --workload kitti --rounds 5 --steps 5 --copies 2 --kernels step base base:num_streams=2,sub_batch=2 > $O/ab_kitti.txt 2>&1 && tail -3 $O/ab_kitti.txt \
 && echo "r4q done"

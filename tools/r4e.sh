#!/bin/bash
# Round-4 GPU pass e: (1) the checkpointed SGM path pairs (k_sgm_ck, default for 4 paths with
# 128 < D <= 256) — their parity tests first, then the whole -m gpu suite; (2) exact vmcnt waits
# in the CBCA sweep loops.  Then same-process A/B at full resolution (nock = the four path sweeps,
# gen = generic H NORM, oldgen = the previous CBCA sources with the generic H NORM, hnp3 = HNorm
# with three tiles in flight), 1080p and Teddy, smoke, the default bench and kernel stats.
# Test failures (pytest exit 1) do not stop the timing runs; a crash or a time limit ends the call.
set -o pipefail
O=gpurun_out/${1:-r4e}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py -k "checkpointed or shapes_and_edge or fixture or golden" > $O/pytest_sgm.log 2>&1
rc=$?; tail -3 $O/pytest_sgm.log; grep -E "FAILED|ERROR" $O/pytest_sgm.log | head
ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
ok $rc || exit 1
A="timeout -k 10 500 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,sgm,step base nock gen oldgen hnp3 > $O/ab_fr.txt 2>&1 && tail -6 $O/ab_fr.txt \
 && $A --workload hd --rounds 4 --steps 2 --copies 1 --kernels cbca,sgm,step base nock gen oldgen > $O/ab_hd.txt 2>&1 && tail -4 $O/ab_hd.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels cbca,step base gen oldgen > $O/ab_teddy.txt 2>&1 && tail -4 $O/ab_teddy.txt \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -16 $O/kt_kernel_stats.csv \
 && echo "r4e done"

#!/bin/bash
# Round-4 GPU pass i: (1) the checkpointed SGM with FLT_MAX in the checkpoint lanes past D (the
# diagnostic against the plain sweeps, the SGM parity tests); (2) NL's pipelined front (prep and
# cost volume on the NL front stream into double-buffered cost volume / flags); the whole -m gpu
# suite; NL A/B (nopipe = the previous schedule) and the NL bench; smoke and the default bench.
set -o pipefail
O=gpurun_out/${1:-r4i}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 300 python -u tools/ck_diag.py > $O/ck_diag.txt 2>&1; rc=$?; head -12 $O/ck_diag.txt; ok $rc || exit 1
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py tests/test_gpu_agg.py -k "checkpointed or shapes_and_edge or fixture or golden or batch_maps or kitti or stages or prep_tiles or nl or NL" > $O/pytest_sgm.log 2>&1
rc=$?; tail -3 $O/pytest_sgm.log; grep -E "FAILED|ERROR" $O/pytest_sgm.log | head
ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
ok $rc || exit 1
timeout -k 10 400 python -u tools/ab_inproc.py --workload teddy --agg NL --rounds 6 --steps 10 --copies 2 --kernels nl_,step base nopipe > $O/ab_nl.txt 2>&1 && tail -3 $O/ab_nl.txt \
 && timeout -k 10 300 python bench.py --workload teddy --agg NL --no-cpu-baseline > $O/bench_nl.json 2> $O/bench_nl.err && cut -c1-300 $O/bench_nl.json \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cut -c1-400 $O/bench.json \
 && echo "r4i done"

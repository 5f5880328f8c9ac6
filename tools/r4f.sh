#!/bin/bash
# Round-4 GPU pass f: checkpointed SGM pairs in both layouts (one line per wave for D > 128, four
# lines per wave below) and with 8 paths: their parity tests first, then the whole -m gpu suite;
# same-process A/B against the plain sweeps (nock) at Teddy and KITTI size; the NL bench (map
# copies overlapped with the next step); PMC HBM traffic of the default bench (FETCH_SIZE and
# WRITE_SIZE in separate passes); smoke, the default bench and kernel stats.
# Test failures (pytest exit 1) do not stop the timing runs; a crash or a time limit ends the call.
set -o pipefail
O=gpurun_out/${1:-r4f}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py tests/test_gpu_agg.py -k "checkpointed or shapes_and_edge or fixture or golden or batch_maps or kitti" > $O/pytest_sgm.log 2>&1
rc=$?; tail -3 $O/pytest_sgm.log; grep -E "FAILED|ERROR" $O/pytest_sgm.log | head
ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels sgm,step base nock > $O/ab_teddy.txt 2>&1 && tail -3 $O/ab_teddy.txt \
 && $A --workload kitti --rounds 5 --steps 5 --copies 2 --kernels sgm,step base nock > $O/ab_kitti.txt 2>&1 && tail -3 $O/ab_kitti.txt \
 && timeout -k 10 300 python bench.py --workload teddy --agg NL --no-cpu-baseline > $O/bench_nl.json 2> $O/bench_nl.err && cat $O/bench_nl.json | cut -c1-400 \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pf -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pf.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pw -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pw.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -16 $O/kt_kernel_stats.csv \
 && python3 tools/pmc_summary.py $(find $O/pf -name "*counter_collection.csv" | head -1) $(find $O/pw -name "*counter_collection.csv" | head -1) $O/pmc_fullres_b2.json && head -c 1500 $O/pmc_fullres_b2.json \
 && echo "r4f done"

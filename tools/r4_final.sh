#!/bin/bash
# Round-4 final GPU round on the final tree: the whole -m gpu suite, smoke, the default bench
# (configs[3]) and every other workload's bench line on the same box, rocprofv3 kernel stats of
# the default bench, and its PMC HBM traffic (FETCH_SIZE and WRITE_SIZE in separate passes); the
# profiled runs use one stream (--streams 1), the launch shape of bench.py's per-kernel pass, so the
# rocprof averages and PMC bytes per launch match the roofline's HIP-event times.
set -o pipefail
O=gpurun_out/${1:-r4_final}
mkdir -p $O
export TMPDIR=/tmp
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
B="timeout -k 10 300 python bench.py"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cut -c1-300 $O/bench.json \
 && $B --workload hd --no-cpu-baseline > $O/bench_hd.json 2> $O/bench_hd.err \
 && $B --workload teddy > $O/bench_teddy.json 2> $O/bench_teddy.err \
 && $B --workload kitti --no-cpu-baseline > $O/bench_kitti.json 2> $O/bench_kitti.err \
 && $B --workload teddy --refine --no-cpu-baseline > $O/bench_refine.json 2> $O/bench_refine.err \
 && $B --workload teddy --opt so --no-cpu-baseline > $O/bench_so.json 2> $O/bench_so.err \
 && $B --workload teddy --agg GF --no-cpu-baseline > $O/bench_gf.json 2> $O/bench_gf.err \
 && $B --workload teddy --agg NL --no-cpu-baseline > $O/bench_nl.json 2> $O/bench_nl.err \
 && for f in hd teddy kitti refine so gf nl; do python3 -c "import json,sys; d=json.load(open('$O/bench_$f.json')); print('$f', d['value'], d['ms_per_step'], d.get('parity'))"; done \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pf -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pf.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pw -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pw.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -16 $O/kt_kernel_stats.csv \
 && python3 tools/pmc_summary.py $(find $O/pf -name "*counter_collection.csv" | head -1) $(find $O/pw -name "*counter_collection.csv" | head -1) $O/pmc_fullres_b2.json \
 && echo "r4 final done"

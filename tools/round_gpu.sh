#!/bin/bash
# Full GPU pass: parity suite, smoke, the default bench (full resolution, configs[3]), rocprofv3
# kernel-trace stats and the two HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs; no trace
# domains with --pmc), then the other workloads' bench lines.
# usage: tools/round_gpu.sh TAG [extra bench args...]   — every step time-limited, chained with &&.
set -o pipefail
TAG=${1:-r2}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 \
 && tail -3 $O/pytest.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err \
 && cat $O/bench.json \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $O/kt.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile "$@" > $O/pmc_fetch.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile "$@" > $O/pmc_write.log 2>&1 \
 && timeout -k 10 300 python bench.py --workload teddy > $O/bench_teddy.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload teddy --refine --no-cpu-baseline > $O/bench_refine.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload teddy --opt so --no-cpu-baseline > $O/bench_so.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload kitti --no-cpu-baseline > $O/bench_kitti.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload hd --no-cpu-baseline > $O/bench_hd.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload teddy --agg GF --no-cpu-baseline > $O/bench_gf.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload teddy --agg NL --no-cpu-baseline > $O/bench_nl.json 2>> $O/bench.err \
 && echo "round_gpu $TAG done"

#!/bin/bash
# Full GPU pass: parity suite, smoke, default bench, rocprofv3 kernel-trace stats and the two
# HBM PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs; no trace domains with --pmc).
# usage: tools/round_gpu.sh TAG [bench args...]   — every step time-limited, chained with &&.
set -o pipefail
TAG=${1:-r1}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 400 > $O/pytest.log 2>&1 \
 && tail -3 $O/pytest.log \
 && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 \
 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py "$@" > $O/bench.json 2> $O/bench.err \
 && cat $O/bench.json \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline "$@" > $O/kt.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile "$@" > $O/pmc_fetch.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile "$@" > $O/pmc_write.log 2>&1 \
 && timeout -k 10 300 python bench.py --refine --no-cpu-baseline "$@" > $O/bench_refine.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --opt so --no-cpu-baseline "$@" > $O/bench_so.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload kitti --no-cpu-baseline > $O/bench_kitti.json 2>> $O/bench.err \
 && timeout -k 10 300 python bench.py --workload fullres --batch 2 --steps 5 --warmup 1 --no-cpu-baseline > $O/bench_fullres_b2.json 2>> $O/bench.err \
 && echo "round_gpu $TAG done"

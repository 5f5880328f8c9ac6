#!/bin/bash
# Round-4 GPU check: the whole -m gpu suite (verbose, per-test time limit), smoke, the default
# bench line (full resolution, configs[3]) and a rocprofv3 kernel-trace summary of the same bench.
# usage: tools/r4_check.sh TAG   -- every GPU step time-limited and chained with &&.
set -o pipefail
TAG=${1:-r4a}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
 ; tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -q " passed" $O/pytest_gpu.log && ! grep -qE "FAILED|ERROR|Timeout" $O/pytest_gpu.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json \
 && cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -14 $O/kt_kernel_stats.csv \
 && echo "r4_check $TAG done"

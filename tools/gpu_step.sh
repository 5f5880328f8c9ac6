#!/bin/bash
# One GPU call: the parity suite (-v, so progress streams to the log), smoke, the default bench,
# then any extra command given as arguments (e.g. an in-process A/B).  Every step time-limited,
# chained with &&; output under gpurun_out/TAG.
# usage: tools/gpu_step.sh TAG [pytest -k expr | - | skip] [extra command...]
set -o pipefail
TAG=${1:-run}; K=${2:--}; shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "$K" = "-" ]; then KA=(); else KA=(-k "$K"); fi
if [ "$K" != "skip" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 400 --timeout-method thread "${KA[@]}" > $O/pytest.log 2>&1 \
   && tail -3 $O/pytest.log \
   && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
   && tail -1 $O/smoke.log || exit 1
fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err \
 && python tools/bench_summary.py $O/bench.json || exit 1
if [ $# -gt 0 ]; then
  timeout -k 10 900 "$@" > $O/extra.log 2>&1
  rc=$?
  tail -14 $O/extra.log
  exit $rc
fi

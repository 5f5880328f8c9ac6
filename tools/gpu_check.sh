#!/bin/bash
# One GPU round trip: parity tests (fast subset or all), then the default bench.
# usage: tools/gpu_check.sh TAG [pytest -k expr]
set -o pipefail
TAG=${1:-run}
K=${2:-}
mkdir -p gpurun_out
if [ -n "$K" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -k "$K" > gpurun_out/${TAG}_pytest.log 2>&1
else
  timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 > gpurun_out/${TAG}_pytest.log 2>&1
fi
rc=$?
tail -4 gpurun_out/${TAG}_pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?
python -c "
import json,sys
d=json.load(open('gpurun_out/${TAG}_bench.json'))
print('value', d['value'], 'ms/step', d['ms_per_step'], 'roof', d['roofline']['kernel'], d['roofline']['frac'])
for k,v in d['kernels'].items(): print('  %-20s %8.4f ms  %7.1f GB/s  share %.3f' % (k, v['avg_ms'], v['GB_s'], v['share']))
" 2>&1 || tail -20 gpurun_out/${TAG}_bench.err
exit $rc

#!/bin/bash
# Runs the default bench under several env settings; prints value + per-kernel ms.
# usage: tools/sweep_env.sh TAG "ENV1=a ENV2=b" "ENV1=c" ...  (bench args via BENCH_ARGS)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for cfg in "$@"; do
  out=gpurun_out/${TAG}_$(echo "$cfg" | tr ' =' '_-').json
  env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline $BENCH_ARGS > $out 2> $out.err || { echo "FAIL $cfg"; tail -5 $out.err; exit 1; }
  python -c "
import json
d=json.load(open('$out'))
print('%-40s value %9.1f  ms/step %.3f' % ('$cfg', d['value'], d['ms_per_step']))
print('   ' + '  '.join('%s=%.3f' % (k, v['avg_ms']) for k, v in d['kernels'].items()))
"
done

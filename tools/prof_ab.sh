#!/bin/bash
# usage: [BENCH_ARGS=...] tools/prof_ab.sh TAG v1 v2 ...  — rocprofv3 kernel-trace stats of bench.py per library variant
export TMPDIR=/tmp
TAG=$1; shift
for v in "$@"; do
  SM_HIP_LIB=tools/variants/libsm_hip_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$v -o kt -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-profile --no-parity $BENCH_ARGS > gpurun_out/${TAG}_$v.log 2>&1 || exit 1
done

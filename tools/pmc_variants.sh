#!/bin/bash
# One PMC counter pass per library variant (tools/build_variants.sh) on the default bench.
# usage: tools/pmc_variants.sh TAG COUNTER v1 v2 ...   (one counter group per pass, no trace domains)
set -o pipefail
TAG=$1; CTR=$2; shift 2
export TMPDIR=/tmp
for v in "$@"; do
  mkdir -p gpurun_out/$TAG/$v
  SM_HIP_LIB=tools/variants/libsm_hip_$v.so timeout -k 10 300 rocprofv3 --pmc $CTR --output-format csv -d gpurun_out/$TAG/$v -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > gpurun_out/$TAG/$v/bench.log 2>&1 || { echo "FAIL $v"; exit 1; }
done
echo "pmc_variants $TAG done"

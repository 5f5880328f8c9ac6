#!/bin/bash
# PMC passes on the default bench (one counter group per pass; no trace domains).
# usage: tools/prof_pmc.sh TAG "COUNTERS" [bench args]
set -o pipefail
TAG=$1; CTRS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/$TAG
timeout -k 10 300 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/$TAG -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile "$@" > gpurun_out/$TAG/bench.log 2>&1

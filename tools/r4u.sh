#!/bin/bash
# Round-4 profile pass on the final tree: rocprofv3 kernel stats and PMC HBM traffic (FETCH_SIZE,
# WRITE_SIZE in separate passes) of the default bench on one stream (--streams 1: the launch shape
# of bench.py's per-kernel pass, so the rocprof averages and PMC bytes per launch match the
# roofline's HIP-event times).
export TMPDIR=/tmp
set -o pipefail
O=gpurun_out/${1:-r4u}
mkdir -p $O
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/kt -o kt -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/kt.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pf -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pf.log 2>&1 \
 && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pw -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity > $GRAFT_REPO_ROOT/$O/pw.log 2>&1 \
 && cd $GRAFT_REPO_ROOT && find $O/kt -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kt_kernel_stats.csv && head -16 $O/kt_kernel_stats.csv \
 && python3 tools/pmc_summary.py $(find $O/pf -name "*counter_collection.csv" | head -1) $(find $O/pw -name "*counter_collection.csv" | head -1) $O/pmc_fullres_b2.json \
 && echo "r4 final done"

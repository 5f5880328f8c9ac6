#!/bin/bash
# NL: producer/consumer rounds with and without the front overlapping the filter (SM_NL_SERIAL_FRONT).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3p4}
mkdir -p $O
timeout -k 10 400 python tools/ab_inproc.py --workload teddy --agg NL --rounds 6 --steps 5 --copies 2 --kernels nl,step base nopc base:SM_NL_SERIAL_FRONT=1 nopc:SM_NL_SERIAL_FRONT=1 > $O/ab_nl.txt 2>&1 && tail -5 $O/ab_nl.txt \
 && SM_NL_SERIAL_FRONT=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload teddy --agg NL --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 \
 && echo done

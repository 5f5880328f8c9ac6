#!/bin/bash
# SQ counters of the NL bench (Teddy x16): issue / wait breakdown of the filter kernels.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3q}
mkdir -p $O
P="timeout -s KILL 120 rocprofv3 --output-format csv"
B="python3 bench.py --workload teddy --agg NL --steps 1 --warmup 1 --no-cpu-baseline --no-profile"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $O/p1 -o pmc -- $B > $O/p1.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS -d $O/p2 -o pmc -- $B > $O/p2.log 2>&1 \
 && echo sq done

#!/bin/bash
# Round-4 GPU pass ac: SQ issue / wait counters of every kernel of the full-resolution bench on the
# final tree (one stream; one counter group per rocprofv3 pass, no trace domains).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4ac}
mkdir -p $O
P="timeout -s KILL 150 rocprofv3 --output-format csv"
B="python3 bench.py --streams 1 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-parity"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $O/p1 -o pmc -- $B > $O/p1.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $O/p2 -o pmc -- $B > $O/p2.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM -d $O/p3 -o pmc -- $B > $O/p3.log 2>&1 \
 && python3 tools/sq_summary.py $O/sq_fullres.json "r4ac: bench fullres --streams 1, final round-4 tree" $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") \
 && echo "r4ac done"

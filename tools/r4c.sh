#!/bin/bash
# Round-4 GPU pass c: SQ issue / wait counters of the fast CBCA sweeps (NsV, HNorm) on the
# full-resolution bench (one counter group per pass, no trace domains), then a same-process A/B of
# the H NORM sweep's tile / prefetch depth against the generic sweep (tools/abvar/).
set -o pipefail
O=gpurun_out/${1:-r4c}
mkdir -p $O
export TMPDIR=/tmp
P="timeout -s KILL 150 rocprofv3 --output-format csv"
B="python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-parity"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $O/p1 -o pmc -- $B > $O/p1.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $O/p2 -o pmc -- $B > $O/p2.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM -d $O/p3 -o pmc -- $B > $O/p3.log 2>&1 \
 && python3 tools/sq_summary.py $O/sq_fullres.json "r4c: bench fullres, NsV + HNorm (T5 PF4)" $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") \
 && echo "sq done" || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,step base gen hnp2 hnp1 hnt4p2 > $O/ab_fr.txt 2>&1 && tail -7 $O/ab_fr.txt \
 && echo "r4c done"

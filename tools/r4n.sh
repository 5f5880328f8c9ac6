#!/bin/bash
# Round-4 GPU pass n: checkpointed SGM loops with exact vmcnt waits (every tile / segment issues the
# same vector-memory sequence; dead tiles store into the dummy area): SGM parity tests, the whole
# -m gpu suite, same-process A/B against the previous loops (noexact) at full resolution and Teddy
# (one stream), then SQ issue / wait counters of every kernel of the full-resolution bench.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r4n}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 600 $PT -m gpu tests/test_gpu_parity.py tests/test_gpu_large_fixtures.py tests/test_gpu_agg.py -k "checkpointed or shapes_and_edge or fixture or golden or batch_maps or kitti or stages" > $O/pytest_sgm.log 2>&1
rc=$?; tail -2 $O/pytest_sgm.log; grep -E "^FAILED|^ERROR" $O/pytest_sgm.log | head; ok $rc || exit 1
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20; ok $rc || exit 1
A="timeout -k 10 400 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels sgm,step base:num_streams=1 noexact:num_streams=1 > $O/ab_fr.txt 2>&1 && tail -3 $O/ab_fr.txt \
 && $A --workload teddy --rounds 6 --steps 10 --copies 2 --kernels sgm,step base noexact > $O/ab_teddy.txt 2>&1 && tail -3 $O/ab_teddy.txt || exit 1
P="timeout -s KILL 150 rocprofv3 --output-format csv"
B="python3 bench.py --streams 1 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-parity"
$P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d $O/p1 -o pmc -- $B > $O/p1.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d $O/p2 -o pmc -- $B > $O/p2.log 2>&1 \
 && $P --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM -d $O/p3 -o pmc -- $B > $O/p3.log 2>&1 \
 && python3 tools/sq_summary.py $O/sq_fullres.json "r4n: bench fullres --streams 1" $(find $O/p1 $O/p2 $O/p3 -name "*counter_collection.csv") \
 && echo "r4n done"

#!/bin/bash
# One parameterised GPU pass (replaces the per-session tools/r3*.sh / r4*.sh scripts).
# usage: tools/gpu_round.sh TAG STEP [STEP ...]     every step time-limited, chained with &&:
#   tests            the whole -m gpu suite (-x)
#   smoke            __graft_entry__.smoke()
#   bench[:ARGS]     python bench.py ARGS (":"-separated args, e.g. bench:--workload:hd) -> bench_<n>.json
#   ab:WL:ROUNDS:COPIES:V1,V2,..   tools/ab_inproc.py on workload WL (variants as ab_inproc takes them)
#   kt[:ARGS]        rocprofv3 --kernel-trace --stats of bench.py --streams 1 ARGS
#   pmc[:ARGS]       FETCH_SIZE and WRITE_SIZE passes (separate runs) -> pmc_fullres_b2.json
#   sq[:ARGS]        three SQ counter passes -> sq_fullres.json
set -o pipefail
TAG=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
[ -n "$GRAFT_REPO_ROOT" ] || O=$(pwd)/gpurun_out/$TAG
R=$(dirname "$O")/..
mkdir -p "$O"
export TMPDIR=/tmp
nb=0
for step in "$@"; do
  kind=${step%%:*}; rest=${step#*:}; [ "$rest" = "$step" ] && rest=""
  args=${rest//:/ }
  case $kind in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
      rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || exit $?
      tail -1 "$O/smoke.log" ;;
    bench)
      nb=$((nb + 1))
      timeout -k 10 400 python bench.py $args > "$O/bench_$nb.json" 2> "$O/bench_$nb.err" || exit $?
      cut -c1-400 "$O/bench_$nb.json" ;;
    ab)
      IFS=: read -r wl rounds copies vars <<< "$rest"
      timeout -k 10 900 python -u tools/ab_inproc.py --workload "$wl" --rounds "$rounds" --copies "$copies" ${vars//,/ } > "$O/ab_$wl.txt" 2>&1 || exit $?
      grep -v "^round" "$O/ab_$wl.txt" | tail -20 ;;
    kt)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o kt -- python3 "$R/bench.py" --streams 1 --steps 10 --warmup 2 --no-cpu-baseline $args > "$O/kt.log" 2>&1) || exit $?
      f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1); cp "$f" "$O/kt_kernel_stats.csv"; head -12 "$O/kt_kernel_stats.csv" | cut -c1-200 ;;
    pmc)
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pf" -o pmc -- python3 "$R/bench.py" --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity $args > "$O/pf.log" 2>&1 \
        && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pw" -o pmc -- python3 "$R/bench.py" --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-parity $args > "$O/pw.log" 2>&1) || exit $?
      python3 tools/pmc_summary.py $(find "$O/pf" -name "*counter_collection.csv" | head -1) $(find "$O/pw" -name "*counter_collection.csv" | head -1) "$O/pmc_fullres_b2.json" || exit $? ;;
    sq)
      B="python3 $R/bench.py --streams 1 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-parity $args"
      P="timeout -s KILL 150 rocprofv3 --output-format csv"
      (cd /tmp && $P --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS -d "$O/p1" -o pmc -- $B > "$O/p1.log" 2>&1 \
        && $P --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS -d "$O/p2" -o pmc -- $B > "$O/p2.log" 2>&1 \
        && $P --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM -d "$O/p3" -o pmc -- $B > "$O/p3.log" 2>&1) || exit $?
      python3 tools/sq_summary.py "$O/sq_fullres.json" "$TAG" $(find "$O/p1" "$O/p2" "$O/p3" -name "*counter_collection.csv") || exit $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_round $TAG done"

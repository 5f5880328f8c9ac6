#!/bin/bash
# round-3 GPU check: two-pass SGM and ximgproc GF tests, in-process A/B of the two-pass SGM
# (full resolution, Teddy), rocprofv3 kernel stats of the GF pipeline (Teddy x16).
set -o pipefail
O=gpurun_out/${1:-r3e}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgm2.py tests/test_gpu_agg.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
 && tail -2 $O/tests.log \
 && timeout -k 10 300 python tools/ab_inproc.py --workload fullres --rounds 4 --steps 3 base base:sgm_2pass=1 > $O/ab.txt 2>&1 \
 && tail -2 $O/ab.txt \
 && timeout -k 10 200 python tools/ab_inproc.py --workload teddy --rounds 6 --steps 10 base base:sgm_2pass=1 > $O/ab_teddy.txt 2>&1 \
 && tail -2 $O/ab_teddy.txt \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gf -o gf -- python3 bench.py --workload teddy --agg GF --steps 5 --warmup 1 --no-cpu-baseline > $O/gf.log 2>&1 \
 && (find $O/gf -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -14)

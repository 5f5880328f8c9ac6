#!/bin/bash
# Split prep (SM_PREP_SPLIT, default) against the three-kernel prep (variant prepold): the GPU
# suite on the default library, then same-process A/B at full resolution and Teddy x16.
set -o pipefail
O=gpurun_out/${1:-ab_prep}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep,step \
  base prepold > $O/fullres.txt 2>&1 && tail -3 $O/fullres.txt \
 && timeout -k 10 300 python tools/ab_inproc.py --workload teddy --rounds 8 --steps 10 --copies 2 --kernels prep \
  base prepold > $O/teddy.txt 2>&1 && tail -3 $O/teddy.txt \
 && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_fetch.log 2>&1 \
 && timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_write.log 2>&1

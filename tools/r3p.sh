#!/bin/bash
# Round-3 GPU pass p: NL producer/consumer rounds (few long paths): NL GPU tests, the suite, and a
# same-process A/B against the block kernels only (nopc) and a higher unit threshold (pc2k).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3p}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "nl or NL" > $O/pytest_nl.log 2>&1 \
  || { tail -40 $O/pytest_nl.log; exit 1; }
tail -1 $O/pytest_nl.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 400 python tools/ab_inproc.py --workload teddy --agg NL --rounds 6 --steps 5 --copies 2 --kernels nl,step base upsh dn512k > $O/ab_nl.txt 2>&1 && tail -4 $O/ab_nl.txt \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload teddy --agg NL --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 \
 && echo done

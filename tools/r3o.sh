#!/bin/bash
# Round-3 GPU pass o: NL with the tree walk on the GPU (records, path tables, ones channel in the
# filter): NL GPU tests first, the whole suite, NL bench (Teddy x16), kernel-trace stats of it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_agg.py -m gpu -x -q --timeout 120 --timeout-method thread -k "nl or NL" > $O/pytest_nl.log 2>&1 \
  || { tail -40 $O/pytest_nl.log; exit 1; }
tail -1 $O/pytest_nl.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --workload teddy --agg NL --no-cpu-baseline > $O/bench_nl.json 2> $O/bench_nl.err && cat $O/bench_nl.json | head -c 600 && echo \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 bench.py --workload teddy --agg NL --steps 5 --warmup 2 --no-cpu-baseline > $O/kt.log 2>&1 \
 && echo done

#!/bin/bash
# NL producer/consumer timing probes (wrong maps, timing only): p1 producers skip data loads,
# p2 consumer skips stores, p3 both; rocprof per-round trace of each variant.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r3p7}
mkdir -p $O
timeout -k 10 400 python tools/ab_inproc.py --workload teddy --agg NL --rounds 6 --steps 5 --copies 1 --kernels nl,step base p1 p2 p3 > $O/ab.txt 2>&1 && tail -5 $O/ab.txt
for v in p1 p3; do
  SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$v -o kt -- python3 bench.py --workload teddy --agg NL --steps 3 --warmup 1 --no-cpu-baseline --no-parity > $O/kt_$v.log 2>&1 || exit 1
done
echo done

#!/bin/bash
# usage: [BENCH_ARGS="--workload kitti"] tools/sweep_variants.sh TAG v1 v2 ...
# (variants from tools/build_variants.sh); prints ms/step and every kernel's average ms
TAG=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  SM_HIP_LIB=tools/variants/libsm_hip_$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-parity $BENCH_ARGS \
    > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err || { echo "FAIL $v"; tail -3 gpurun_out/${TAG}_$v.err; exit 1; }
  python - "$v" "gpurun_out/${TAG}_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[2])); k = d["kernels"]
print("%-8s %.3f " % (sys.argv[1], d["ms_per_step"]) + " ".join("%s=%.3f" % (n.replace("cbca_", ""), k[n]["avg_ms"]) for n in k))
PY
done

# SGM one-line-per-wave (D = 256) tile depth at full resolution: parity of each variant library on
# the SGM / large-fixture GPU tests, then interleaved same-process A/B (tools/ab_inproc.py).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_sgm; mkdir -p $O
for v in t4 t6 t12; do
  SM_HIP_LIB=$PWD/tools/variants/libsm_hip_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "large or sgm" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels sgm base t4 t6 t12 base t4 t6 t12 > $O/ab_fullres.txt 2>&1 && tail -8 $O/ab_fullres.txt

set -o pipefail
# async uploads that wait for the inputs' last reader (SM_UP_EARLY, in-tree) vs the group's end (late)
O=gpurun_out/r6up; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_batch.log 2>&1; rc=$?; tail -2 $O/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
L=$GRAFT_REPO_ROOT/tools/abvar/libsm_hip_late.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_$i.json 2> $O/res_$i.err || exit $?
  timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > $O/early_$i.json 2> $O/early_$i.err || exit $?
  SM_HIP_LIB=$L timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > $O/late_$i.json 2> $O/late_$i.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6up/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["parity"]["bit_exact"])
PY

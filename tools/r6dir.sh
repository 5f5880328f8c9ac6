set -o pipefail
# run_many's direct path (one rank, page-locked host batches: the library uploads them itself):
# batch-runner tests, 1080p x8 e2e vs resident
O=gpurun_out/r6dir; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_batch.log 2>&1; rc=$?; tail -1 $O/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_hd.json 2> $O/res_hd.err || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > $O/e2s_$i.json 2> $O/e2s_$i.err || exit $?
done
timeout -k 10 300 python bench.py --e2e --e2e-stream --e2e-input numpy --workload hd --steps 10 --warmup 2 > $O/e2s_numpy.json 2> $O/e2s_numpy.err || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6dir/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["parity"]["bit_exact"])
PY

set -o pipefail
# resident vs streamed end to end (1080p x8), three interleaved repetitions on one box
O=gpurun_out/r6e2r4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_batch.log 2>&1; rc=$?; tail -1 $O/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_$i.json 2> $O/res_$i.err || exit $?
  timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > $O/e2s_$i.json 2> $O/e2s_$i.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6e2r4/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["parity"]["bit_exact"])
PY

set -o pipefail
# early uploads on the null stream, the context's streams created as before: batch-runner tests,
# Teddy x16 timed loop (maps copied out every step) x3 processes, 1080p x8 e2e vs resident
O=gpurun_out/r6st3; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_batch.log 2>&1; rc=$?; tail -1 $O/pytest_batch.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload teddy --no-cpu-baseline --no-profile > $O/teddy_$i.json 2> $O/teddy_$i.err || exit $?
done
timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_hd.json 2> $O/res_hd.err || exit $?
for i in 1 2; do
  timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > $O/e2s_$i.json 2> $O/e2s_$i.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6st3/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d.get("schedule_ab", {}).get("default_ms"), d["parity"]["bit_exact"])
PY

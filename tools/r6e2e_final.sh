set -o pipefail
O=gpurun_out/r6e2e; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_batch.log 2>&1; tail -2 $O/pytest_batch.log
timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_hd.json 2> $O/res_hd.err || exit $?
timeout -k 10 300 python bench.py --e2e --workload hd --steps 10 --warmup 2 > "$O/e2e_0.json" 2> "$O/e2e_0.err" || exit $?
timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 > "$O/e2s_0.json" 2> "$O/e2s_0.err" || exit $?
timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 --e2e-sub-batch 4 > "$O/e2s_4.json" 2> "$O/e2s_4.err" || exit $?
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6e2e/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["config"].get("sub_blocks"), d["parity"]["bit_exact"])
PY

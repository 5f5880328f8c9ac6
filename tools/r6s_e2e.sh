set -o pipefail
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 300 python bench.py --workload hd --steps 10 --warmup 2 --no-cpu-baseline --no-profile > $O/res_hd.json 2> $O/res_hd.err || exit $?
for sb in 8 1,7; do
  timeout -k 10 300 python bench.py --e2e --e2e-stream --workload hd --steps 10 --warmup 2 --e2e-sub-batch $sb > "$O/e2s_$sb.json" 2> "$O/e2s_$sb.err" || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6s/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d["config"].get("sub_blocks"), d["parity"]["bit_exact"])
PY

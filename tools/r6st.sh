set -o pipefail
# download stream created lazily (in-tree) vs with the others at sm_create (eagercst): Teddy x16
# timed loop (maps copied out every step), three processes each, interleaved
O=gpurun_out/r6st2; mkdir -p $O
E=$GRAFT_REPO_ROOT/tools/abvar/libsm_hip_eagercst.so
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --workload teddy --no-cpu-baseline --no-profile > $O/lazy_$i.json 2> $O/lazy_$i.err || exit $?
  SM_HIP_LIB=$E timeout -k 10 300 python bench.py --workload teddy --no-cpu-baseline --no-profile > $O/eager_$i.json 2> $O/eager_$i.err || exit $?
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r6st2/*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], d["ms_per_step"], d.get("schedule_ab", {}).get("default_ms"), d["parity"]["bit_exact"])
PY

set -o pipefail
O=gpurun_out/r6p; mkdir -p $O
for wl in teddy kitti; do
  timeout -k 10 400 python -u tools/ab_inproc.py --workload $wl --rounds 8 --copies 3 base:placement_trials=3 nohn2:placement_trials=3 nopipe:placement_trials=3 > $O/ab_$wl.txt 2>&1 || exit $?
  grep -B12 -A4 "medians" $O/ab_$wl.txt | grep "step=" | cut -c1-60
done

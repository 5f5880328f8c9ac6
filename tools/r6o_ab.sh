set -o pipefail
O=gpurun_out/r6o; mkdir -p $O
for wl in teddy kitti hd; do
  timeout -k 10 400 python -u tools/ab_inproc.py --workload $wl --rounds 4 --copies 2 base:placement_trials=3 old:placement_trials=3 nohn2:placement_trials=3 nopipe:placement_trials=3 > $O/ab_$wl.txt 2>&1 || exit $?
  grep -A5 "medians" $O/ab_$wl.txt
done

set -o pipefail
O=gpurun_out/r6q; mkdir -p $O
for wl in teddy kitti hd; do
  c=3; [ $wl = hd ] && c=2
  timeout -k 10 400 python -u tools/ab_inproc.py --workload $wl --rounds 6 --copies $c base:num_streams=1,placement_trials=0 nohn2:num_streams=1,placement_trials=0 nopipe:num_streams=1,placement_trials=0 > $O/ab_$wl.txt 2>&1 || exit $?
  grep -A4 "medians" $O/ab_$wl.txt | cut -c1-250
done

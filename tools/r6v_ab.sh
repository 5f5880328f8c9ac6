set -o pipefail
# pipelined groups taking turns on their CBCA sweeps (SM_PIPE_CBCA_EXCL 1) or on the first
# NORM_SCAN sweep only (2) vs the free-running default, same process, default schedule with
# placement trials
O=gpurun_out/r6w; mkdir -p $O
timeout -k 10 600 python -u tools/ab_inproc.py --workload fullres --rounds 6 --steps 4 --copies 2 base vexcl excl > $O/ab_fullres.txt 2>&1 || exit $?
grep -A4 "medians" $O/ab_fullres.txt | cut -c1-60
timeout -k 10 300 python -u tools/ab_inproc.py --workload hd --rounds 5 --steps 3 --copies 1 base vexcl > $O/ab_hd.txt 2>&1 || exit $?
grep -A3 "medians" $O/ab_hd.txt | cut -c1-60

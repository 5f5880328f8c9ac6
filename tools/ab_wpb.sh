# Timing probes of the CBCA V sweeps' arm gathers (full resolution, interleaved same-process A/B,
# tools/ab_inproc.py; probes give wrong maps): p2 = every gather re-reads row 0, p3 = right rows
# but every wave reads columns 0..63, p4 = right rows, 16 distinct words per gather.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab4; mkdir -p $O
timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels cbca base p2 p5 p6 base p2 p5 p6 > $O/ab_fullres.txt 2>&1 && tail -8 $O/ab_fullres.txt

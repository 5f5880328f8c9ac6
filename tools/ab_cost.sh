# Cost kernel: compile-time unrolled element loop (SM_COST_ND, default on) against the runtime loop
# (variant nd0): GPU parity suite on the default library, then interleaved same-process A/B at full
# resolution (D = 256), KITTI (D = 192) and Teddy (D = 64, unchanged path).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_cost; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && tail -1 $O/pytest.log \
 && timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels cost base nd0 base nd0 > $O/ab_fullres.txt 2>&1 && tail -4 $O/ab_fullres.txt \
 && timeout -k 10 300 python -u tools/ab_inproc.py --workload kitti --rounds 8 --steps 5 --copies 2 --kernels cost base nd0 > $O/ab_kitti.txt 2>&1 && tail -3 $O/ab_kitti.txt

# CBCA normalising sweeps: area prefix step as v_dot2_u32_u16 (default) against shift/add/add3
# (variant nodot): GPU parity suite, then interleaved same-process A/B (full resolution, Teddy x16).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab_dot2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && tail -1 $O/pytest.log \
 && timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels norm base nodot base nodot > $O/ab_fullres.txt 2>&1 && tail -4 $O/ab_fullres.txt \
 && timeout -k 10 300 python -u tools/ab_inproc.py --workload teddy --rounds 8 --steps 5 --copies 3 --kernels norm base nodot > $O/ab_teddy.txt 2>&1 && tail -3 $O/ab_teddy.txt

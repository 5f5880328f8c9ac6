# Timing probes of the CBCA V sweeps' arm gathers (full resolution, interleaved same-process A/B,
# tools/ab_inproc.py): p1 = no gathers, p2 = every gather re-reads row 0 (probes give wrong maps);
# ax1..3 = gather cache-policy bits (parity checked first).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/ab2; mkdir -p $O
for v in ax1 ax2 ax3; do
  SM_HIP_LIB=$PWD/tools/variants/libsm_hip_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "parity or large" > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --kernels cbca base p1 p2 ax1 ax2 ax3 base > $O/ab_fullres.txt 2>&1 && tail -7 $O/ab_fullres.txt

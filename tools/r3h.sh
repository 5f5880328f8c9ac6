#!/bin/bash
# Round-3 GPU pass h: GF (ximgproc) column sweeps with a register ring (default) — aggregator
# parity and Teddy A/B against the tiled form (gfold); NORM_SCAN T = 12 at 1080p and Teddy;
# kernel-trace stats of the split prep (prepsplit) and the three-kernel prep (base) at full
# resolution, and the split prep's HBM traffic (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
O=gpurun_out/${1:-r3h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_agg.py -x -q --timeout 120 --timeout-method thread > $O/pytest_agg.log 2>&1 \
  || { tail -40 $O/pytest_agg.log; exit 1; }
tail -1 $O/pytest_agg.log
timeout -k 10 300 python tools/ab_inproc.py --workload teddy --agg GF --rounds 8 --steps 10 --copies 2 --kernels gf,step \
  base gfold > $O/teddy_gf.txt 2>&1 && tail -3 $O/teddy_gf.txt \
 && timeout -k 10 400 python tools/ab_inproc.py --workload hd --rounds 5 --steps 3 --copies 2 --kernels cbca_v,step \
  base ns12:fuse_norm_scan=1 > $O/hd_ns.txt 2>&1 && tail -3 $O/hd_ns.txt \
 && timeout -k 10 300 python tools/ab_inproc.py --workload teddy --rounds 8 --steps 10 --copies 2 --kernels cbca_v,step \
  base ns12:fuse_norm_scan=1 > $O/teddy_ns.txt 2>&1 && tail -3 $O/teddy_ns.txt \
 && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_base -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_base.log 2>&1 \
 && SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_prepsplit.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_split -o kt -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/kt_split.log 2>&1 \
 && SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_prepsplit.so timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_fetch.log 2>&1 \
 && SM_HIP_LIB=$PWD/tools/abvar/libsm_hip_prepsplit.so timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $O/pmc_write.log 2>&1 \
 && grep -h "k_prep\|k_pack" $O/kt_base/*stats* $O/kt_split/*stats* | cut -c1-160

#!/bin/bash
# Round-3 GPU pass m: GPU suite on the packed ring-slot pairs + v_mad_u32_u16 ring addresses
# (default library, with the NS set-2 reuse), then same-process A/B against the previous sweeps
# (old), reuse only, and packed slots without the mad addressing (nomad).
set -o pipefail
O=gpurun_out/${1:-r3m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
A="timeout -k 10 400 python tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,step base old reuse nomad > $O/fr.txt 2>&1 && tail -5 $O/fr.txt \
 && $A --workload teddy --rounds 8 --steps 10 --copies 2 --kernels cbca,step base old nomad > $O/teddy.txt 2>&1 && tail -4 $O/teddy.txt \
 && $A --workload fullres --rounds 4 --steps 3 --copies 2 --kernels cbca,sgm,step base base:sub_batch=1,num_streams=2 > $O/fr_streams.txt 2>&1 && tail -3 $O/fr_streams.txt

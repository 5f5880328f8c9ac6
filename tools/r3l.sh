#!/bin/bash
# Round-3 GPU pass l: GPU suite on the NS set-2 reuse + tile-level dividend check (default
# library), then same-process A/B against the previous sweeps (old), reuse only, check only.
set -o pipefail
O=gpurun_out/${1:-r3l}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
A="timeout -k 10 400 python tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 2 --kernels cbca,step base old reuse safe > $O/fr.txt 2>&1 && tail -5 $O/fr.txt \
 && $A --workload teddy --rounds 8 --steps 10 --copies 2 --kernels cbca,step base old > $O/teddy.txt 2>&1 && tail -3 $O/teddy.txt

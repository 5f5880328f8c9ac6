#!/bin/bash
# Round-4 GPU pass g: where the checkpointed SGM differs from the plain sweeps (diagnostic).
set -o pipefail
O=gpurun_out/${1:-r4g}
mkdir -p $O
timeout -k 10 300 python -u tools/ck_diag.py > $O/ck_diag.txt 2>&1; cat $O/ck_diag.txt | head -80

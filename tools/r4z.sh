#!/bin/bash
# Round-4 GPU pass z: the D = 256 checkpointed SGM passes with deeper register rings as the default
# (pass A four tiles, pass B of the first pair three segments): the whole GPU suite, then A/B against
# the previous depths (prev) in the default schedule at full resolution and 1080p x8, then the
# default bench line.
set -o pipefail
O=gpurun_out/${1:-r4z}
mkdir -p $O
PT="python -u -m pytest -v -p no:cacheprovider --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -m gpu tests > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20
[ $rc -eq 0 ] || exit 1
A="timeout -k 10 600 python -u tools/ab_inproc.py"
$A --workload fullres --rounds 5 --steps 3 --copies 3 --kernels sgm_ck,step prev base > $O/ab_fr.txt 2>&1 && grep -E "maps|step=" $O/ab_fr.txt | tail -12 \
 && $A --workload hd --rounds 4 --steps 2 --copies 2 --kernels sgm_ck,step base prev > $O/ab_hd.txt 2>&1 && grep -E "maps|step=" $O/ab_hd.txt | tail -8 \
 && timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err && cut -c1-250 $O/bench.json \
 && echo "r4z done"

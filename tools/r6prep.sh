set -o pipefail
# prep tile heights: k_prep_h 4 -> 8 rows, k_prep_v 64 -> 128 rows (fewer halo re-reads)
O=gpurun_out/r6prep2; mkdir -p $O
timeout -k 10 500 python -u tools/ab_inproc.py --workload fullres --rounds 5 --steps 3 --copies 2 --kernels prep base:num_streams=1,placement_trials=0 h8v128:num_streams=1,placement_trials=0 > $O/ab_fullres.txt 2>&1 || exit $?
grep -A3 "medians" $O/ab_fullres.txt
export SM_HIP_LIB=$GRAFT_REPO_ROOT/tools/abvar/libsm_hip_h8v128.so
bash tools/gpu_round.sh r6prep2/h8v128 pmc || exit $?
python3 -c "import json; d=json.load(open('$O/h8v128/pmc_fullres_b2.json')); print(d['kernels']['prep'])"

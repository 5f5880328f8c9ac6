# Product multi-GPU path on one box: the end-to-end DistributedBatchRunner bench at N = 1 (hd,
# configs[4] shape, 8 pairs), and 2-rank rehearsals of the resident and end-to-end paths with both
# ranks on the box's one GPU (gloo for the collectives: RCCL needs one GPU per rank).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/multi; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_batch.py tests/test_distributed.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_batch.log 2>&1 && tail -1 $O/pytest_batch.log \
 && timeout -k 10 400 python bench.py --e2e --workload hd --steps 3 --warmup 1 > $O/e2e_hd_n1.json 2> $O/e2e_hd_n1.err && cat $O/e2e_hd_n1.json \
 && SM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --workload teddy --steps 10 --warmup 2 --no-cpu-baseline > $O/resident_teddy_n2_gloo.json 2> $O/resident_teddy_n2_gloo.err && cat $O/resident_teddy_n2_gloo.json \
 && SM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --e2e --workload teddy --steps 5 --warmup 1 > $O/e2e_teddy_n2_gloo.json 2> $O/e2e_teddy_n2_gloo.err && cat $O/e2e_teddy_n2_gloo.json

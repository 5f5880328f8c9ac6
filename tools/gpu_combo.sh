bash tools/gpu_multi_rehearsal.sh && bash tools/ab_sgm.sh

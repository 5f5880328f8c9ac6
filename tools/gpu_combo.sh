# One GPU call: the dot2 A/B (tools/ab_dot2.sh: GPU suite + timing), then the full round on the tree.
bash tools/ab_dot2.sh && bash tools/round_gpu.sh r2n

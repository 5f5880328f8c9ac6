"""Print a bench.py JSON line as a short per-kernel table (tools/gpu_step.sh)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms/step", d["ms_per_step"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["kernels"].items():
    print("  %-20s %8.4f ms  %7.1f GB/s  frac %.3f" % (k, v["avg_ms"], v["GB_s"], v["hbm_frac"]))

#!/bin/bash
# Round-4 GPU passes v + w in one call (the pool is short of boxes): pass-A ring depth (apf3/apf4)
# and the H sweeps' tile / prefetch depths (hspf2, hst16, hnpf3, hnt8).
bash tools/r4v.sh && bash tools/r4w.sh

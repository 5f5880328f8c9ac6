"""Host side of aggregation NL (csrc/sm_nl_tree.cpp) against the oracle's tree, on the CPU.

tests/cpp/nl_tree_check.cpp is compiled with g++ together with sm_nl_tree.cpp and the oracle's
C restatement (oracle/sm_oracle_agg.c, oracle/sm_oracle.c: test infrastructure) and run: the
breadth-first tree walked from Kruskal's neighbour lists equals smo_nl_tree node for node, every
list is in increasing (weight, edge index) order (the order the GPU's Boruvka lists are built
in, sm_nl_mst.hip), the records / weight sums fused into the walk equal nl_pack_records and
smo_nl_filter of ones, and lists that are not a spanning tree are rejected.  The GPU lists
themselves are pinned end to end by tests/test_gpu_agg.py (NL volumes bit-exact vs the oracle).
"""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_nl_tree_host_vs_oracle(tmp_path):
    exe = str(tmp_path / "nl_tree_check")
    src = [os.path.join(ROOT, "tests", "cpp", "nl_tree_check.cpp"),
           os.path.join(ROOT, "mystereomatching_amd", "csrc", "sm_nl_tree.cpp")]
    csrc = [os.path.join(ROOT, "oracle", "sm_oracle_agg.c"), os.path.join(ROOT, "oracle", "sm_oracle.c")]
    objs = []
    for c in csrc:
        o = str(tmp_path / (os.path.basename(c) + ".o"))
        r = subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-c", c, "-o", o,
                            f"-I{os.path.join(ROOT, 'oracle')}"], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr[-3000:]
        objs.append(o)
    r = subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-Wall", "-Werror",
                        f"-I{os.path.join(ROOT, 'mystereomatching_amd', 'csrc')}", f"-I{os.path.join(ROOT, 'oracle')}",
                        *src, *objs, "-o", exe, "-lm"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert r.stdout.startswith("ok "), r.stdout

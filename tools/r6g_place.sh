set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r6g; mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 $R/tools/place_probe.py --copies 6 --rounds 3 --out $O/p0.json > $O/p0.txt 2>&1 || exit $?
tail -6 $O/p0.txt
P="timeout -s KILL 300 rocprofv3 --output-format csv"
$P --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_SERIALIZATION_STALL_sum -d $O/c1 -o c1 -- python3 $R/tools/place_probe.py --copies 6 --rounds 2 --out $O/p1.json > $O/p1.txt 2>&1 || exit $?
$P --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum -d $O/c2 -o c2 -- python3 $R/tools/place_probe.py --copies 6 --rounds 2 --out $O/p2.json > $O/p2.txt 2>&1 || exit $?
$P --pmc GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum -d $O/c3 -o c3 -- python3 $R/tools/place_probe.py --copies 6 --rounds 2 --out $O/p3.json > $O/p3.txt 2>&1 || exit $?
cd $R
for k in 1 2 3; do python3 tools/place_counters.py $O/p$k.json $O/counters$k.json $(find $O/c$k -name "*counter_collection.csv") > $O/counters$k.txt 2>&1 || exit $?; done
grep -A7 "^cbca_h_scan" $O/counters1.txt $O/counters2.txt $O/counters3.txt

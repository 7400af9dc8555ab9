# round-3: A/B of the adaptive slice quantum against the spill-free build (NS = the main build):
# Q8a: 8 steps while more than one suspended path per slot waits, Q8b: while more than 1/4 per slot,
# Q6c: 6 steps while more than 1/2, Q12b: 12 steps while more than 1/4; then their HBM traffic
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 400 python scripts/ab_track.py NS=$L/libhc_trifocal.so Q8a=$L/libhc_trifocal_xQ8a.so Q8b=$L/libhc_trifocal_xQ8b.so Q6c=$L/libhc_trifocal_xQ6c.so Q12b=$L/libhc_trifocal_xQ12b.so --rounds 3 > gpurun_out/r3g_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3g_ab.jsonl; [ $rc -eq 0 ] || exit $rc
for v in q8a q8b q12b; do V=$(echo $v | sed 's/q/Q/'); HC_TRIFOCAL_LIB=$L/libhc_trifocal_x$V.so bash scripts/pmc_traffic.sh r3g_$v || exit 1; done
for t in r3g_q8a r3g_q8b r3g_q12b; do python -c "import json; d=json.load(open('gpurun_out/${t}_pmc_summary.json')); print('$t', d['avg_ns'], d['derived'].get('hbm_bytes_per_launch'))"; done

# round-3: A/B of the spill-free stage loop (NS = the main build) against T3 and of the adaptive
# slice quantum (Q8a: 8 steps while more than one path per slot waits, Q8b: while more than 1/4,
# Q6c: 6 steps while more than 1/2), then the HBM traffic of NS, Q8a and Q8b
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 400 python scripts/ab_track.py T3=$L/libhc_trifocal_xT3.so NS=$L/libhc_trifocal.so Q8a=$L/libhc_trifocal_xQ8a.so Q8b=$L/libhc_trifocal_xQ8b.so Q6c=$L/libhc_trifocal_xQ6c.so --rounds 3 > gpurun_out/r3f_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3f_ab.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_traffic.sh r3f_ns || exit 1
HC_TRIFOCAL_LIB=$L/libhc_trifocal_xQ8a.so bash scripts/pmc_traffic.sh r3f_q8a || exit 1
HC_TRIFOCAL_LIB=$L/libhc_trifocal_xQ8b.so bash scripts/pmc_traffic.sh r3f_q8b || exit 1
for t in r3f_ns r3f_q8a r3f_q8b; do python -c "import json; d=json.load(open('gpurun_out/${t}_pmc_summary.json')); print('$t', d['avg_ns'], d['derived'].get('hbm_bytes_per_launch'))"; done

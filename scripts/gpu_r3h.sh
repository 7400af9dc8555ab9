# round-3: adaptive slice quantum, longer quanta while more than one suspended path per slot waits
# (Q8a: 8 steps, Q16a: 16, QIa: no suspension then) against the main build (NS); HBM traffic of Q16a, QIa
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 400 python scripts/ab_track.py NS=$L/libhc_trifocal.so Q8a=$L/libhc_trifocal_xQ8a.so Q16a=$L/libhc_trifocal_xQ16a.so QIa=$L/libhc_trifocal_xQIa.so --rounds 3 > gpurun_out/r3h_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3h_ab.jsonl; [ $rc -eq 0 ] || exit $rc
for v in Q16a QIa; do HC_TRIFOCAL_LIB=$L/libhc_trifocal_x$v.so bash scripts/pmc_traffic.sh r3h_$v || exit 1; done
for t in r3h_Q16a r3h_QIa; do python -c "import json; d=json.load(open('gpurun_out/${t}_pmc_summary.json')); print('$t', d['avg_ns'], d['derived'].get('hbm_bytes_per_launch'))"; done

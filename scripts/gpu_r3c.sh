# round-3 check: GPU tests on the new build, then the A/B of the LU / time-slicing variants and their HBM traffic
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
[ -n "$SKIP_TESTS" ] || timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3c_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3c_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc   # 1 = a failed assertion: the A/B still runs
timeout -k 10 700 python scripts/ab_track.py old=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xold.so S3=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xS3.so R3=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal.so R4=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xR4.so R5=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xR5.so R6=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xR6.so G1=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xG1.so G2=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xG2.so --rounds 3 > gpurun_out/r3c_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3c_ab.jsonl; [ $rc -eq 0 ] || exit $rc
bash scripts/pmc_traffic.sh r3c_r3 || exit 1
HC_TRIFOCAL_LIB=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xR5.so bash scripts/pmc_traffic.sh r3c_r5 || exit 1
HC_TRIFOCAL_LIB=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xold.so bash scripts/pmc_traffic.sh r3c_old || exit 1
for t in r3c_r3 r3c_r5 r3c_old; do python -c "import json; d=json.load(open('gpurun_out/${t}_pmc_summary.json')); print('$t', d['avg_ns'], d['derived'].get('hbm_bytes_per_launch'))"; done

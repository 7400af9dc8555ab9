# round-3: GPU tests on the candidate build (sparse LU with dense re-solve from the kept entry block),
# A/B against the earlier builds, HBM traffic per build, full PMC profile of the candidate
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r3d_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r3d_pytest.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python scripts/ab_track.py old=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xold.so S3=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xS3.so R3=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xR3.so T3=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal.so T5=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xT5.so --rounds 3 > gpurun_out/r3d_ab.jsonl 2>&1; rc=$?; cat gpurun_out/r3d_ab.jsonl; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_LIB=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xS3.so bash scripts/pmc_traffic.sh r3d_s3 || exit 1
HC_TRIFOCAL_LIB=trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_xT5.so bash scripts/pmc_traffic.sh r3d_t5 || exit 1
bash scripts/profile.sh r3d_t3 || exit 1
python scripts/pmc_summary.py r3d_t3 gpurun_out/r3d_t3_pmc_summary.json > /dev/null
for t in r3d_s3 r3d_t5 r3d_t3; do python -c "import json; d=json.load(open('gpurun_out/${t}_pmc_summary.json')); print('$t', d['avg_ns'], d['derived'].get('hbm_fetch_bytes_corrected'), d['derived'].get('hbm_write_bytes'), d['dispatch'].get('Scratch_Size'))"; done

# round 5 validation of build v10.2 in one call: GPU tests, LU-work count,
# default bench line, kernel trace + PMC passes, dataset spread; then the
# abort-priority A/B (time to the first pose, scripts/gpu_r5pd.sh)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5ab}
bash scripts/gpu_r5v.sh $T || exit $?
bash scripts/gpu_r5w.sh $T || exit $?
bash scripts/gpu_r5pd.sh

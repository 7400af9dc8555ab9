# usage: bash scripts/gpu_ab_only.sh TAG ROUNDS NAME=lib ...  -- interleaved A/B timing only (scripts/ab_track.py)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; R=$2; shift 2
timeout -k 10 900 python scripts/ab_track.py "$@" --rounds $R > gpurun_out/${T}_ab.jsonl 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/${T}_ab.jsonl; exit $rc

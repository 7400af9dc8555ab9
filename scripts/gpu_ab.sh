# usage: bash scripts/gpu_ab.sh TAG NAME=lib/libhc_trifocal_NAME.so ...  -- GPU parity of the product
# library, then interleaved A/B timing of the named builds (scripts/ab_track.py, 3 rounds)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python scripts/ab_track.py "$@" --rounds 3 > gpurun_out/${T}_ab.jsonl 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/${T}_ab.jsonl; [ $rc -eq 0 ] || exit $rc

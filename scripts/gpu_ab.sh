# usage: bash scripts/gpu_ab.sh TAG A=lib/libA.so B=lib/libB.so [...]   (paths relative to the package dir)
# interleaved A/B of tracker builds (scripts/ab_track.py), then the parity tests of
# test_gpu_parity.py on the last build (it is loaded through HC_TRIFOCAL_LIB)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=$1; shift
P=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd
args=""; last=""
for kv in "$@"; do args="$args ${kv%%=*}=$P/${kv#*=}"; last=$P/${kv#*=}; done
HC_TRIFOCAL_LIB=$last timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread -k "not cli" > gpurun_out/${T}_parity.log 2>&1; rc=$?; tail -3 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/ab_track.py $args --rounds 3 > gpurun_out/${T}_ab.jsonl; rc=$?; cat gpurun_out/${T}_ab.jsonl; exit $rc

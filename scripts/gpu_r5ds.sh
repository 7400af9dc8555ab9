# round 5: dataset spread of the shipped build incl. the shards of ranks 1..7
# of an 8-GPU config-2 run (scripts/datasets.py)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
T=${1:-r5ds}
L=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 600 python -u scripts/datasets.py $L/libhc_trifocal_luwork.so > gpurun_out/${T}_datasets.jsonl; rc=$?; cat gpurun_out/${T}_datasets.jsonl; exit $rc

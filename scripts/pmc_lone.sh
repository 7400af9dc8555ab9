# usage: bash scripts/pmc_lone.sh TAG SAMPLES -- SQ counter passes on the tracker at SAMPLES samples
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; N=$2
B="python scripts/track_once.py --samples $N --reps 3"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_IFETCH"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${T}_pmc$i -o run -- $B > gpurun_out/${T}_pmc$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

# usage: bash scripts/profile.sh TAG
# kernel trace + stats, then one PMC pass per counter group (never combined with traces)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
B="python bench.py --steps 30 --warmup 3 --no-cpu-baseline --abort-samples 0 --noisy-trials 0 --streams 1 --pipelined-streams 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
           "SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_IFETCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${T}_pmc$i -o run -- $B > gpurun_out/${T}_pmc$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

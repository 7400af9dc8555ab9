# usage: [HC_TRIFOCAL_LIB=lib.so] bash scripts/pmc_traffic.sh TAG
# kernel trace + the two HBM-traffic PMC passes (FETCH_SIZE, WRITE_SIZE) of the
# tracker's config-2 launch, each pass its own run (never combined with tracing)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --abort-samples 0 --noisy-trials 0 --streams 1 --pipelined-streams 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_trace -o run -- $B > gpurun_out/${T}_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for set in "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${T}_pmc$i -o run -- $B > gpurun_out/${T}_pmc$i.log 2>&1; rc=$?; echo "pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_summary.py $T gpurun_out/${T}_pmc_summary.json > /dev/null; echo "summary rc=$?"

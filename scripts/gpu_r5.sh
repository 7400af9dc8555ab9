cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --abort-samples 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_trace -o run -- $B > gpurun_out/r5_trace.log 2>&1; rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d gpurun_out/r5_pmcA -o run -- $B > gpurun_out/r5_pmcA.log 2>&1; rc=$?; echo "pmcA rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/r5_pmcB -o run -- $B > gpurun_out/r5_pmcB.log 2>&1; rc=$?; echo "pmcB rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r5_pmcC -o run -- $B > gpurun_out/r5_pmcC.log 2>&1; rc=$?; echo "pmcC rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r5_pmcD -o run -- $B > gpurun_out/r5_pmcD.log 2>&1; rc=$?; echo "pmcD rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r5_bench.json
find gpurun_out -name "*stats*.csv" | head; find gpurun_out -name "*counter_collection*.csv" | head

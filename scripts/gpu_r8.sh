cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r8_comp -o run -- python scripts/ubench.py > gpurun_out/r8_comp.log 2>&1; rc=$?; echo "comp rc=$rc"; [ $rc -eq 0 ] || exit $rc
HC_TRIFOCAL_KERNEL=v2 timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r8_comp2 -o run -- python scripts/ubench.py > gpurun_out/r8_comp2.log 2>&1; rc=$?; echo "comp2 rc=$rc"; [ $rc -eq 0 ] || exit $rc

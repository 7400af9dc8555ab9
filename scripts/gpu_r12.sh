cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/r12_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r12_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r12_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r12_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./trifocal_pose_estimation_using_improved_gpuhc_amd/bin/magmaHC-main -p trifocal_2op1p_30x30 -d $GRAFT_REPO_ROOT > gpurun_out/r12_cli.log 2>&1; rc=$?; echo "cli rc=$rc"; tail -12 gpurun_out/r12_cli.log; cat Output_Write_Files/*.txt > gpurun_out/r12_cli_outputs.txt 2>/dev/null; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 ./trifocal_pose_estimation_using_improved_gpuhc_amd/bin/magmaHC-main -p trifocal_2op1p_30x30 -d $GRAFT_REPO_ROOT -n 1000 --abort > gpurun_out/r12_cli_abort.log 2>&1; rc=$?; echo "cli abort rc=$rc"; tail -6 gpurun_out/r12_cli_abort.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./scripts/lds_ubench > gpurun_out/r12_lds.json; rc=$?; echo "lds rc=$rc"; cat gpurun_out/r12_lds.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r12_bench.json 2> gpurun_out/r12_bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/r12_bench.json; [ $rc -eq 0 ] || exit $rc
bash scripts/profile.sh r12

cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2r_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -3 gpurun_out/r2r_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/ab_track.py base=$L/libhc_trifocal_base.so new=$L/libhc_trifocal_new.so bfesq=$L/libhc_trifocal_bfesq.so --rounds 3 > gpurun_out/r2r_ab.jsonl 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/r2r_ab.jsonl; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --abort-samples 0 --noisy-trials 0 > gpurun_out/r2r_bench.json 2> gpurun_out/r2r_bench.err; rc=$?; echo "bench rc=$rc"; python -c "import json; d=json.load(open('gpurun_out/r2r_bench.json')); print(d['value'], d['config']['pipelined_paths_per_s'], d['roofline']['kernel_ms'])"

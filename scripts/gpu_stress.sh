# usage: bash scripts/gpu_stress.sh TAG -- time slicing under concurrency (scripts/slice_stress.py):
# 4 streams from cold, 4 streams warmed first, 8 streams from cold
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1; rc=$?; echo "parity rc=$rc"; tail -2 gpurun_out/${T}_parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/slice_stress.py gpurun_out/${T}_stress4.jsonl 4 4 > /dev/null 2>&1; rc=$?; echo "stress4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/slice_stress.py gpurun_out/${T}_stress4w.jsonl 4 4 --warm-streams > /dev/null 2>&1; rc=$?; echo "stress4w rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/slice_stress.py gpurun_out/${T}_stress8.jsonl 8 3 > /dev/null 2>&1; rc=$?; echo "stress8 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python -c "
import json,sys
for f in sys.argv[1:]:
    for l in open(f):
        d=json.loads(l); print(f.split('/')[-1], d['round'], d['wall_ms'], [(x['status'], x['exact'], x['unfinished']) if x['status'] == 0 else x for x in d['launches']])
" gpurun_out/${T}_stress4.jsonl gpurun_out/${T}_stress4w.jsonl gpurun_out/${T}_stress8.jsonl
L=trifocal_pose_estimation_using_improved_gpuhc_amd/lib
if [ -f $L/libhc_trifocal_oldho.so ]; then
  cp $L/libhc_trifocal.so /tmp/libhc_trifocal_new.so
  timeout -k 10 500 python scripts/ab_track.py wrapring=$L/libhc_trifocal_oldho.so ticketring=/tmp/libhc_trifocal_new.so --rounds 3 > gpurun_out/${T}_ab.jsonl 2>&1; rc=$?; echo "ab rc=$rc"; cat gpurun_out/${T}_ab.jsonl
fi

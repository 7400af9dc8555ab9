# A/B of kernel generation x dequeue order on the config-2 workload (tracking only)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1
for v in v3 v4; do for o in natural ltf; do
  HC_TRIFOCAL_KERNEL=$v HC_TRIFOCAL_ORDER=$o timeout -k 10 200 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --abort-samples 0 --noisy-trials 0 > gpurun_out/${T}_${v}_${o}.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${T}_${v}_${o}.json'));print('$v $o', d['roofline']['kernel_ms'], d['value'], d['solutions'])"
done; done

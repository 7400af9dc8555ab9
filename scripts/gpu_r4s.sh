# N=2 rehearsal of bench.py on the shipped build (two ranks on cuda:0 over gloo)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r4_n2.sh r4s

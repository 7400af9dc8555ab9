# round-end rehearsal of the driver's flow on the shipped build: smoke(), then
# the default bench line
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4n_smoke.log 2>&1; rc=$?; tail -3 gpurun_out/r4n_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r4n_bench.json 2> gpurun_out/r4n_bench.err; rc=$?; cat gpurun_out/r4n_bench.json; exit $rc

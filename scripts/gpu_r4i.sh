# per-phase shader cycles of a stage (HC_DIAG_PHASES build of HEAD's sources):
# lone waves (1 sample) and full occupancy (config 2); then parity of the spec
# variants (spec: every lane computes 1/pivot of its own candidate during the search,
# the pivot lane stores it in the pivot-element slot; spec2: + the rows below the
# pivot from the eligibility mask) and their A/B against HEAD; parity on spec2
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
HC_TRIFOCAL_LIB=$GRAFT_REPO_ROOT/trifocal_pose_estimation_using_improved_gpuhc_amd/lib/libhc_trifocal_phases.so timeout -k 10 300 python scripts/diag_phases.py > gpurun_out/r4i_diag_phases.json; rc=$?; cat gpurun_out/r4i_diag_phases.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh r4i base=lib/libhc_trifocal_r4g.so spec=lib/libhc_trifocal_spec.so spec2=lib/libhc_trifocal_spec2.so

# usage: bash scripts/build_variant.sh NAME [extra hipcc flags...]
# builds lib/libhc_trifocal_NAME.so: the product library with hc_kernels.hip
# compiled with extra flags: the diagnostic builds (-DHC_DIAG_PHASES,
# -DHC_DIAG_TIMES [-DHC_DIAG_UTIL], -DHC_DIAG_LUWORK).  The round-2 A/B switches
# (HC_LU_*, HC_EV_*, HC_HX_GROUPED, HC_AB_*, HC_CGESV4, HC_SLICE_Q, HC_PRIO_*)
# were removed from the product sources in round 3; they live in commit 136b029.
# Round 6's scheduling switches (HC_SLICE_HOLD, HC_PRIO_LAS, HC_PRIO_STEPW,
# HC_PRIO_REM) live in commit 02bc69d.
set -e
cd "$(dirname "$0")/../trifocal_pose_estimation_using_improved_gpuhc_amd/csrc"
N=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -I../../include "$@" \
    -c hc_kernels.hip -o /tmp/hc_kernels_$N.o 2>&1 | grep -v "unused" || true
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/libhc_trifocal_$N.so /tmp/hc_kernels_$N.o \
    ../lib/hc_pose.o ../lib/hc_host.o ../lib/GPU_HC_Solver.o
echo "built lib/libhc_trifocal_$N.so"

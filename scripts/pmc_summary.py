#!/usr/bin/env python3
"""Summarise a `scripts/gpu.sh profile` run: per-launch PMC counters of the tracker
kernel plus derived utilisations, stamped with the build id of the library the
run loaded (the bench line's config.build_id in the trace log), which is how
bench.py finds the profile of its own build.  usage: pmc_summary.py TAG [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
base = os.path.join(ROOT, "gpurun_out")
# the headline tracker instantiation (archived ablation and abort-mode launches
# are other instantiations of k_track and are not mixed in)
KNAME = os.environ.get("HC_PMC_KERNEL", "void hc::k_track<false, 5, true, false, true>(hc::KArgs)")
stats = list(csv.DictReader(open(os.path.join(base, f"{tag}_trace", "run_kernel_stats.csv"))))
trk = [r for r in stats if r["Name"] == KNAME][0]
out = {"tag": tag, "build_id": None, "measured_at": None, "kernel": trk["Name"], "calls": int(trk["Calls"]), "avg_ns": float(trk["AverageNs"]),
       "min_ns": float(trk["MinNs"]), "max_ns": float(trk["MaxNs"]), "counters": {}}
# per-dispatch durations (the trace's first launch of a process runs cold:
# caches, TLB and code are warmed by it, so it is reported apart)
tr = os.path.join(base, f"{tag}_trace", "run_kernel_trace.csv")
if os.path.exists(tr):
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) for r in csv.DictReader(open(tr))
            if r["Kernel_Name"] == KNAME]
    if len(durs) > 1:
        warm = sorted(durs[1:])
        out["first_dispatch_ns"] = durs[0]
        out["warm_dispatches"] = len(warm)
        out["warm_avg_ns"] = sum(warm) / len(warm)
        out["warm_median_ns"] = warm[len(warm) // 2] if len(warm) % 2 else (warm[len(warm) // 2 - 1] + warm[len(warm) // 2]) / 2
meta = None
for d in sorted(glob.glob(os.path.join(base, f"{tag}_pmc*"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"] == KNAME:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
            meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
                                      "Accum_VGPR_Count", "SGPR_Count")}
    for k, v in agg.items():
        out["counters"][k] = v / max(1, len(disp))
out["dispatch"] = meta
c = out["counters"]
der = {}
if "SQ_WAVES" in c:
    waves = c["SQ_WAVES"]
    cyc = c["SQ_WAVE_CYCLES"] * 4 / waves              # quad-cycles -> cycles per wave
    der["waves"] = waves
    der["cycles_per_wave"] = cyc
    der["eff_clock_ghz"] = cyc / out["avg_ns"]
    simds = 256 * 4
    # SQ_ACTIVE_INST_* count quad-cycles (MI355X_MICROARCH.md): VALU-active cycles per SIMD / kernel cycles
    if "SQ_ACTIVE_INST_VALU" in c:
        der["valu_active_frac"] = c["SQ_ACTIVE_INST_VALU"] * 4 / simds / cyc
        der["valu_active_cycles_per_inst"] = c["SQ_ACTIVE_INST_VALU"] * 4 / c["SQ_INSTS_VALU"]
    der["valu_per_wave"] = c["SQ_INSTS_VALU"] / waves
    der["lds_per_wave"] = c["SQ_INSTS_LDS"] / waves
    der["frac_wait_inst_any"] = c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"]
    der["frac_wait_any"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    if "SQ_ACTIVE_INST_ANY" in c:
        der["frac_active_any"] = c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"]
        der["frac_wait_inst_lds"] = c["SQ_WAIT_INST_LDS"] / c["SQ_WAVE_CYCLES"]
        der["salu_per_wave"] = c["SQ_INSTS_SALU"] / waves
    if "SQC_ICACHE_MISSES" in c:
        der["icache_miss_rate"] = c["SQC_ICACHE_MISSES"] / max(1.0, c["SQC_ICACHE_MISSES"] + c["SQC_ICACHE_HITS"])
if "FETCH_SIZE" in c:
    der["hbm_fetch_bytes_corrected"] = c["FETCH_SIZE"] * 1024 * 2      # MI355X_MICROARCH.md: x2 on gfx950
if "WRITE_SIZE" in c:
    der["hbm_write_bytes"] = c["WRITE_SIZE"] * 1024
if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
    der["hbm_bytes_per_launch"] = der["hbm_fetch_bytes_corrected"] + der["hbm_write_bytes"]
# FLOPs of the same bench run (its JSON line in the trace log): FLOP per VALU instruction
try:
    import time
    lines = [l for l in open(os.path.join(base, f"{tag}_trace.log")) if l.startswith("{")]
    bl = json.loads(lines[-1])
    out["build_id"] = bl["config"].get("build_id")
    out["measured_at"] = time.strftime("%Y-%m-%dT%H:%M:%SZ",
                                       time.gmtime(os.path.getmtime(os.path.join(base, f"{tag}_trace.log"))))
    out["bench_ms_per_step"] = bl.get("ms_per_step")
    out["bench_kernel_ms"] = bl["roofline"].get("kernel_ms")
    rl = bl["roofline"]
    if "SQ_INSTS_VALU" in c:
        ex = rl.get("executed_gflop_per_launch")
        de = rl.get("dense_lu_gflop_per_launch", rl.get("algorithmic_gflop_per_launch"))
        if not ex and de and rl.get("rk4_steps") is not None:
            # the bench run predates this build's LU-work profile: the same
            # pricing as bench.py, from the committed profile of the build
            sys.path.insert(0, ROOT)
            import bench
            frac, src = bench.lu_executed_fraction(out["build_id"])
            if frac is not None:
                stages = 4 * rl["rk4_steps"] + rl["corrections"]
                ex = de - stages * bench.LU_UPDATE_DENSE_FLOP * (1.0 - frac) / 1e9
                out["lu_executed_fraction"] = frac
                out["lu_executed_fraction_source"] = src
        if ex:
            der["flop_per_valu_executed"] = ex * 1e9 / c["SQ_INSTS_VALU"]
        if de:
            der["flop_per_valu_dense_lu"] = de * 1e9 / c["SQ_INSTS_VALU"]
except (OSError, ValueError, KeyError, IndexError):
    pass
out["derived"] = der
s = json.dumps(out, indent=1)
print(s)
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(s + "\n")

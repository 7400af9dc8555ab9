#!/usr/bin/env python3
"""Static instruction counts of the tracker kernel per phase of a stage (CPU).

Compiles hc_kernels.hip for gfx950 to assembly with -DHC_DIAG_ISA, whose
HC_ISA_MARK comments split the headline kernel k_track<false, 5, true, false, true>
into the phases of one stage: slot control, parking, the dH/dt | H and dH/dx
evaluations, and, per LU pivot step I, the pivot search, the rare pivot path,
the pivot-pattern readlanes, the pivot-row stores, the read-back + 1/pivot +
relabelling, the multiplier and right-hand side, the column-group updates and
the back-substitution step.  Inside the LU the column-group bodies (a
`s_bitcmp` + `s_cbranch_scc1` skip over a store or an update of one group)
(or a two-column `s_and_b32` + `s_cmp_eq_u32` test) are counted apart from the unconditional instructions, so that
scripts/phase_breakdown.py can weigh them with the dynamic frequencies the
HC_DIAG_LUWORK build measures (live groups, rare steps and evaluation kinds
per wave-stage) and check the sum against the rocprofv3 PMC totals.

    python scripts/isa_phases.py [--asm existing.s] [--out profiles/rXX_isa_phases.json]
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "trifocal_pose_estimation_using_improved_gpuhc_amd", "csrc", "hc_kernels.hip")
KERNEL = "_ZN2hc7k_trackILb0ELi5ELb1ELb0ELb1EEEvNS_5KArgsE"


def classify(mn):
    if mn.startswith("s_cbranch") or mn == "s_branch":
        return "branch"
    if mn == "s_nop":
        return "nop"
    if mn == "s_waitcnt" or mn.startswith("s_waitcnt"):
        return "waitcnt"
    if mn.startswith(("s_load", "s_buffer_load", "s_store", "s_dcache", "s_memtime", "s_memrealtime")):
        return "smem"
    if mn.startswith("s_"):
        return "salu"
    if mn.startswith("ds_"):
        return "lds"
    if mn.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mn.startswith("v_readlane") or mn.startswith("v_readfirstlane"):
        return "valu_readlane"
    if mn.startswith("v_"):
        return "valu"
    return "other"


def compile_asm(path):
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
           "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-DHC_DIAG_ISA", SRC, "-o", path]
    subprocess.run(cmd, check=True, capture_output=True)


# scalar instructions that leave SCC alone (between a group test and its branch)
SCC_KEEP = ("s_mov_b32", "s_mov_b64", "s_waitcnt", "s_setprio", "s_cbranch_execz", "s_cbranch_execnz",
            "s_cbranch_vccz", "s_cbranch_vccnz")


def kernel_lines(asm):
    lines = open(asm).read().splitlines()
    start = next(i for i, ln in enumerate(lines) if ln.startswith(KERNEL + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def analyse(lines):
    """{phase: {"fixed": Counter, "groups": [Counter per group body], "steps": set}}."""
    phases = collections.defaultdict(lambda: {"fixed": collections.Counter(), "groups": [], "steps": set()})
    cur, step = "prologue", None
    skip_to = None          # label that ends the current group body
    body = None
    prev_bitcmp = False
    dense = False
    since_branch = []       # classes counted in lu_search since its last branch
    for ln in lines:
        t = ln.strip()
        m = re.match(r";HCPH (\w+)(?: (\d+))?", t)
        if m:
            if m.group(1) == "lu_rare" and cur.endswith("lu_search") and since_branch:
                # the rare path's first instructions, scheduled above its marker
                # (after the search's last branch, in the block that branch skips)
                for cls in since_branch:
                    phases[cur]["fixed"][cls] -= 1
                    phases[("dense_" if dense else "") + "lu_rare"]["fixed"][cls] += 1
            since_branch = []
            cur, step = m.group(1), (int(m.group(2)) if m.group(2) else None)
            if cur in ("lu_dense", "lu_sparse"):
                dense = cur == "lu_dense"
            elif not cur.startswith("lu_"):
                dense = False
            if dense and cur.startswith("lu_"):
                cur = "dense_" + cur      # the dense re-solve (rare: HC_DIAG_LUWORK counts it)
            continue
        if re.match(r"^\.?LBB\w*:", t) or re.match(r"^\.LBB[\w_]+:", t):
            lab = t.split(":")[0]
            if skip_to is not None and lab == skip_to:
                phases[body[0]]["groups"].append(body[1])
                skip_to, body = None, None
            continue
        if not t or t.startswith((";", ".", "//")):
            continue
        mn = t.split()[0]
        cls = classify(mn)
        key = cur
        ph = phases[key]
        if step is not None:
            ph["steps"].add(step)
        if skip_to is not None:
            body[1][cls] += 1
        else:
            ph["fixed"][cls] += 1
            if key.endswith("lu_search"):
                since_branch = [] if cls == "branch" else since_branch + [cls]
        # the group test: the last SCC write before the s_cbranch_scc1 is a bit
        # test (s_bitcmp0 of one column's bit) or a two-column test (s_and_b32 of
        # the pair's bits + s_cmp_eq_u32 with 0); the scheduler may put VALU or
        # LDS work between the test and its branch
        if mn.startswith("s_bitcmp") or (mn == "s_cmp_eq_u32" and t.rstrip().endswith(", 0")):
            prev_bitcmp = True
            continue
        if prev_bitcmp and mn == "s_cbranch_scc1" and skip_to is None and "lu_" in cur:
            skip_to = t.split()[1]
            body = (cur, collections.Counter())
        if mn == "s_cbranch_scc1" or (mn.startswith("s_") and mn not in SCC_KEEP and not mn.startswith("s_nop")):
            prev_bitcmp = False
    return phases


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm", default=None, help="use this assembly instead of compiling")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    asm = a.asm or "/tmp/hc_isa_phases.s"
    if not a.asm:
        compile_asm(asm)
    ph = analyse(kernel_lines(asm))
    out = {"kernel": KERNEL, "phases": {}}
    for k, v in ph.items():
        g = collections.Counter()
        for c in v["groups"]:
            g.update(c)
        out["phases"][k] = {"instances": len(v["steps"]) or 1, "fixed": dict(v["fixed"]),
                            "group_bodies": len(v["groups"]), "group_body_total": dict(g)}
    s = json.dumps(out, indent=1, sort_keys=True)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    sys.exit(main())

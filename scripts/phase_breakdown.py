#!/usr/bin/env python3
"""Instructions per wave-stage of the tracker kernel, by phase (CPU).

Combines three measurements of one build:
  * the static per-phase instruction counts of scripts/isa_phases.py (the
    HC_DIAG_ISA markers; column-group bodies counted apart);
  * the dynamic frequencies of the HC_DIAG_LUWORK build on config 2
    (scripts/lu_work.py: wave-solves, live column groups and rare pivot steps
    per wave-solve, and which right-hand-side evaluation each wave-stage ran);
  * the rocprofv3 PMC totals of the product kernel (scripts/pmc_summary.py:
    SQ_INSTS_VALU / SALU / LDS / BRANCH per launch).
Each phase's count per wave-stage = its unconditional instructions x how often
it runs + its group bodies x the live fraction; "control" is what the PMC
total leaves over (slot phases, parking, stage update, dequeue, suspension).

    python scripts/phase_breakdown.py ISA.json LU_WORK.json PMC.json [--out X.json]
"""
import argparse
import json

CLASSES = ("valu", "valu_readlane", "salu", "lds", "branch", "nop", "waitcnt", "vmem", "smem")


def group_tests_per_solve(ch=2, nv=30):
    """Column groups the sparse LU tests over a solve (hc_lu.hpp LuChunks<2>)."""
    n = 0
    for i in range(nv - 1):
        single = 1 if ((i + 1) & 1) and (i + 1 < nv) else 0
        n += single + (nv - (i + 1 + single) + ch - 1) // ch
    return n


def _group_classes():
    try:
        import sys
        import os
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from trifocal_pose_estimation_using_improved_gpuhc_amd import _abi
        L = _abi.lib()
        if not hasattr(L, "hc_lu_group_class"):
            return []
    except Exception:   # no library here: the classes are given on the command line
        return []
    out = []
    for i in range(29):
        k = 0
        while int(L.hc_lu_group_class(i, k)) >= 0:
            out.append(int(L.hc_lu_group_class(i, k)))
            k += 1
    return out


def always_groups():
    """Column groups the tracker's LU runs without a test (hc_lu.hpp, class 2)."""
    return sum(1 for c in _group_classes() if c == 2)


def dead_groups():
    """Column groups it never runs (class 1)."""
    return sum(1 for c in _group_classes() if c == 1)


def load_last_json(path):
    txt = open(path).read()
    try:
        return json.loads(txt)
    except ValueError:
        return json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("isa")
    ap.add_argument("lu_work")
    ap.add_argument("pmc")
    ap.add_argument("--out")
    ap.add_argument("--always", type=int, default=None, help="untested always-live groups per solve "
                    "(default: from the library's hc_lu_group_class; 0 for builds before v10.1)")
    ap.add_argument("--dead", type=int, default=None, help="untested dead groups per solve (same default)")
    a = ap.parse_args()
    ph = load_last_json(a.isa)["phases"]
    lw = load_last_json(a.lu_work)
    pmc = load_last_json(a.pmc)

    def fixed(name):
        return {c: ph.get(name, {}).get("fixed", {}).get(c, 0) for c in CLASSES}

    def bodies(name):
        p = ph.get(name, {})
        n = max(1, p.get("group_bodies", 0))
        return {c: p.get("group_body_total", {}).get(c, 0) / n for c in CLASSES}, p.get("group_bodies", 0)

    def add(*ds, scale=1.0):
        out = {c: 0.0 for c in CLASSES}
        for d in ds:
            for c in CLASSES:
                out[c] += d.get(c, 0) * scale
        return out

    def sc(d, s):
        return {c: d[c] * s for c in CLASSES}

    stages = lw["wave_stages"]
    solves = lw["wave_solves"] / stages                     # sparse wave-solves per wave-stage
    live = lw["live_groups_per_wave_solve"]
    rare = lw["rare_steps_per_wave_solve"]
    tests = group_tests_per_solve()
    # round 5 (v10.1): the always-live groups run untested (their instructions are
    # in the ISA's fixed counts, and the LU-work count includes them) and the
    # dead ones are gone; only the tested groups' bodies are weighted
    n_always = a.always if a.always is not None else always_groups()
    if n_always:
        tests -= n_always + a.dead if a.dead is not None else n_always + dead_groups()
        live -= n_always
    f_live = live / tests
    kinds = lw["rhs_eval_kinds"]
    kt = sum(kinds.values())
    # the pattern readlanes of the common path sit in the rare path's text
    # (scheduled above the marker): two per pivot step, moved to "pattern"
    rare_fixed = fixed("lu_rare")
    rl_common = min(rare_fixed["valu_readlane"], 2 * 28)
    rare_fixed["valu_readlane"] -= rl_common
    st_body, _ = bodies("lu_store")
    # the update's column-group bodies: under the lu_update marker up to round 4;
    # from round 5 (one exec region per pivot step) they follow the lu_mult marker
    up_body, n_up = bodies("lu_update")
    mu_body, n_mu = bodies("lu_mult")
    up_body = {c: (up_body[c] * n_up + mu_body[c] * n_mu) / max(1, n_up + n_mu) for c in CLASSES}
    rows = {
        "lu_search": sc(fixed("lu_search"), solves),
        "lu_rare_path": sc(rare_fixed, solves * rare / 30.0),
        "lu_pattern_readlanes": sc(add(fixed("lu_pattern"), {"valu_readlane": rl_common}), solves),
        "lu_pivot_row_store": sc(add(fixed("lu_store"), sc(st_body, live)), solves),
        "lu_readback_recip_relabel": sc(fixed("lu_rcp"), solves),
        "lu_multiplier_rhs_fill_and_updates": sc(add(fixed("lu_mult"), fixed("lu_update"), sc(up_body, live)), solves),
        "lu_back_substitution": sc(add(fixed("lu_back"), fixed("lu_back_init")), solves),
        "lu_entry_check": sc(fixed("lu_finite"), solves),
        "eval_rhs": add(fixed("ev_rhs"), sc(fixed("ev_rhs_mixed"), kinds["mixed"] / kt),
                        sc(fixed("ev_rhs_ht"), kinds["dHdt_only"] / kt), sc(fixed("ev_rhs_h"), kinds["H_only"] / kt)),
        "prefix_tables": sc(fixed("ctl_prefix"), lw.get("prefix_rebuilds_per_wave_stage", 0.0)),
        "eval_hx_terms": fixed("ev_hx"),
        "eval_hx_gather": fixed("ev_gather"),
    }
    c = pmc["counters"]
    launch_stages = stages   # the LU-work run is one config-2 launch, like the PMC run
    total = {"valu": c.get("SQ_INSTS_VALU", 0) / launch_stages, "salu": c.get("SQ_INSTS_SALU", 0) / launch_stages,
             "lds": c.get("SQ_INSTS_LDS", 0) / launch_stages, "branch": c.get("SQ_INSTS_BRANCH", 0) / launch_stages}
    acc = {k: 0.0 for k in total}
    table = {}
    for name, d in rows.items():
        v = {"valu": d["valu"] + d["valu_readlane"], "salu": d["salu"], "lds": d["lds"], "branch": d["branch"],
             "readlane": d["valu_readlane"], "nop": d["nop"], "waitcnt": d["waitcnt"]}
        table[name] = {k: round(x, 1) for k, x in v.items()}
        for k in acc:
            acc[k] += v[k]
    table["control_and_other (PMC total - phases)"] = {k: round(total[k] - acc[k], 1) for k in total}
    out = {"per_wave_stage": table, "pmc_total_per_wave_stage": {k: round(x, 1) for k, x in total.items()},
           "inputs": {"isa": a.isa, "lu_work": a.lu_work, "pmc": a.pmc,
                      "build_id": pmc.get("build_id"), "lu_work_build_id": lw.get("build_id")},
           "frequencies": {"wave_stages": stages, "sparse_wave_solves_per_wave_stage": round(solves, 4),
                           "live_groups_per_wave_solve": round(lw["live_groups_per_wave_solve"], 2),
                           "always_live_groups_untested": n_always,
                           "live_tested_groups_per_wave_solve": round(live, 2), "group_tests_per_solve": tests,
                           "live_group_fraction": round(f_live, 4), "rare_steps_per_wave_solve": round(rare, 3),
                           "rhs_eval_kinds": kinds},
           "note": "SQ_INSTS_VALU counts v_readlane as VALU; SALU excludes s_nop / s_waitcnt / branches here and "
                   "may differ from SQ_INSTS_SALU's accounting, so the control row's SALU is approximate"}
    s = json.dumps(out, indent=1)
    if a.out:
        open(a.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Pin experiment: can the CPU-HC restatement reproduce the reference's
committed CPU counts exactly (Output_Write_Files/CPU_Sols_Statistics.txt:1,
11098 converged / 521 real / 6577 infinity, config 2 = srand(0), 100 samples)?

Variables tried (each in its own process):
  ops  = spec  : the oracle as built for the tests (-ffp-contract=off, the
                 arithmetic spec's explicit FMAs);
         plain : libhc_oracle_plain.so, the reference's host operators as
                 plain expressions compiled like the reference CPU build
                 (-O3 -march=native, GCC's default FMA contraction).
  lu   = restated : the oracle's getf2/getrs restatement;
         openblas:<CORE> : OpenBLAS 0.3.23.dev `cgesv_64_` (the version the
                 reference links), kernel set forced with OPENBLAS_CORETYPE.

Test infrastructure only (tests/ may load the oracle); writes one JSON line per variant.
    python tests/cpuhc_pin.py [--samples 100] [--out profiles/r2_cpuhc_pin.json]
"""
import ctypes as C
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPENBLAS = "/opt/conda/lib/python3.9/site-packages/numpy.libs/libopenblas64_p-r0-0cf96a72.3.23.dev.so"
REF = [11098, 521, 6577]


def child(ops, lu, samples):
    sys.path.insert(0, ROOT)
    from oracle import oracle as O
    if ops == "plain":
        O.LIB_PATH = os.path.join(ROOT, "oracle", "build", "libhc_oracle_plain.so")
    lib = O.lib()
    info = {}
    if lu.startswith("openblas"):
        d = os.path.dirname(OPENBLAS)   # its private libgfortran / libquadmath first
        for dep in sorted(os.listdir(d), key=lambda n: not n.startswith("libquadmath")):
            if dep.startswith(("libquadmath", "libgfortran")):
                C.CDLL(os.path.join(d, dep), mode=C.RTLD_GLOBAL)
        ob = C.CDLL(OPENBLAS)
        ob.openblas_get_config64_.restype = C.c_char_p
        ob.openblas_get_corename64_.restype = C.c_char_p
        info = {"openblas_config": ob.openblas_get_config64_().decode(),
                "openblas_core": ob.openblas_get_corename64_().decode()}
        lib.orc_set_external_cgesv(C.cast(ob.cgesv_64_, C.c_void_p))
    prob = os.path.join(ROOT, "data", "problems", "trifocal_2op1p_30x30")
    rans = os.path.join(ROOT, "data", "RANSAC_Data", "trifocal_2op1p_30x30", "Synthetic")
    ss, sp, dhdx, dhdt = O.read_problem(prob)
    loc, tan = O.read_edgels(os.path.join(rans, "Triplet_Edgels", "Triplet_Edgels_000.txt"))
    tgt, dif, _ = O.prepare_target_params(0, [samples], loc, tan, sp)
    t = time.time()
    tr, cc, ic, st, secs = O.cpuhc_track(ss, sp, tgt, dif, dhdx, dhdt)
    counts = [int(v) for v in O.count_solutions(tr, cc, ic)]
    print(json.dumps({"ops": ops, "lu": lu, "samples": samples, "counts": counts,
                      "reference": REF if samples == 100 else None,
                      "exact": counts == REF if samples == 100 else None,
                      "seconds": round(time.time() - t, 1), **info}))


def main():
    samples = int(sys.argv[sys.argv.index("--samples") + 1]) if "--samples" in sys.argv else 100
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "plain"], check=True)
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    variants = [(o, l) for o in ("spec", "plain")
                for l in ("restated", "openblas:Haswell", "openblas:SkylakeX", "openblas:Zen", "openblas:Sandybridge")]
    if only:
        variants = [v for v in variants if f"{v[0]}/{v[1]}" in only]
    lines = []
    for ops, lu in variants:
        env = dict(os.environ, OPENBLAS_NUM_THREADS="1")
        if lu.startswith("openblas:"):
            env["OPENBLAS_CORETYPE"] = lu.split(":")[1]
        p = subprocess.run([sys.executable, __file__, "--child", ops, lu, str(samples)], env=env,
                           capture_output=True, text=True)
        line = p.stdout.strip().splitlines()[-1] if p.returncode == 0 else json.dumps(
            {"ops": ops, "lu": lu, "error": p.stderr[-500:]})
        print(line, flush=True)
        lines.append(line)
    if out:
        with open(out, "w") as f:
            f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    if "--child" in sys.argv:
        i = sys.argv.index("--child")
        child(sys.argv[i + 1], sys.argv[i + 2], int(sys.argv[i + 3]))
    else:
        main()

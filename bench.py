#!/usr/bin/env python3
"""Benchmark: HC paths/s of the MI355X GPU-HC tracker (trifocal_2op1p_30x30).

Workload (BASELINE.json configs[1], per GPU): 100 RANSAC samples x 312 tracks,
Abort_RANSAC=false, synthcurves dataset 000, samples drawn with srand(0) in the
reference's gpu-major order (rank g takes its own contiguous shard of
100*N samples).  One "step" = reset the tracks to the start solutions + one
tracking launch over the rank's samples, inputs already resident in HBM.

Multi-GPU: one process per GPU (torch.distributed, backend nccl == RCCL);
samples are independent so the ranks share nothing on the data path (weak
scaling); RCCL only carries the barrier, the max-over-ranks timing, the
early-stop flag (abort leg) and the 136-byte pose selections (all_gather).

Besides the headline line (config 2) the JSON carries: `pose` (device pose
recovery + maximal support over the config-2 tracks),
`early_abort` (config 3 / 4: time-to-first-good-pose), `noisy_pose` (config 5:
sigma=1px noisy synthcurves, pose success rate vs paths/s), `roofline` and
`cpu_baseline`.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--samples S] [--no-cpu-baseline]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# SURVEY.md §8(d) algorithmic work per unit (flop convention: complex mul 6,
# complex add 2, real x complex 2, complex div 11)
FLOP_PRED_STAGE = 104.3e3    # Hx 12,276 + Ht 12,960 + LU 78,670 + axpys ~360
FLOP_CORR_STAGE = 101.3e3    # Hx 12,276 + H 10,080 + LU 78,670 + update/norms ~300
# The LU's rank-1 updates are 8555 element updates (8 FLOP each = 68,440 FLOP)
# of the 78,670 in the dense algorithm the reference runs; the structurally
# sparse LU executes only the column groups that are non-zero in a pivot row
# of the wave.  `frac_executed_lu` prices the updates as executed, with the
# executed fraction measured by the HC_DIAG_LUWORK build of the same sources
# (scripts/lu_work.py, profiles/*_lu_work.json stamped with the product build id).
LU_UPDATE_DENSE_FLOP = 68440.0


def _profiles_of_build(pattern, bid, pick):
    """(value, file) from the committed profiles matching `pattern` whose
    build_id is `bid` (the loaded library's _abi.build_id()); (None, reason)
    when no profile measured this build.  Newest by the recorded timestamp."""
    import glob
    found = []
    for f in glob.glob(os.path.join(ROOT, "profiles", pattern)):
        try:
            with open(f) as fh:
                txt = fh.read()
        except OSError:
            continue
        try:
            d = json.loads(txt)
        except ValueError:
            try:
                d = json.loads([ln for ln in txt.splitlines() if ln.startswith("{")][-1])
            except (ValueError, IndexError):
                continue
        if d.get("build_id") != bid:
            continue
        v = pick(d)
        if v is not None:
            found.append((d.get("measured_at", ""), v, os.path.relpath(f, ROOT)))
    if not found:
        return None, f"no profiles/{pattern} of build {bid}"
    found.sort()
    return found[-1][1], found[-1][2]


def lu_executed_fraction(bid):
    """Executed fraction of the dense rank-1 update work on config 2, from the
    HC_DIAG_LUWORK profile of this build: (fraction, file) or (None, reason)."""
    return _profiles_of_build("*_lu_work.json", bid,
                              lambda d: None if "scaled" in d.get("config", "") else d.get("executed_fraction"))
FP32_PEAK_TFLOPS = 157.3     # MI355X_MICROARCH.md: FP32 vector peak (64 FLOP/clk/SIMD) == FP32 MFMA peak
HBM_PEAK_GBS = 8000.0
TRACK_KERNEL = "void hc::k_track<false, 5, true, false, true>(hc::KArgs)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--samples", type=int, default=100, help="RANSAC samples per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-small-launch", action="store_true",
                    help="skip the 1- and 8-sample launch timings (profiles: keeps the kernel trace to config 2)")
    ap.add_argument("--cpu-samples", type=int, default=160,
                    help="samples in the bounded CPU baseline run (~15 s on 16 host cores)")
    ap.add_argument("--abort-samples", type=int, default=1000,
                    help="samples per GPU of the early-abort (config 3/4) time-to-first-good-pose run; 0 disables")
    ap.add_argument("--abort-repeats", type=int, default=12,
                    help="runs per abort semantics in the early-abort leg (median, min and max reported)")
    ap.add_argument("--abort-seeds", type=int, default=8,
                    help="early-abort leg: also srand(1..K) draws of the same data (first pose across hypotheses)")
    ap.add_argument("--abort-seed-repeats", type=int, default=3)
    ap.add_argument("--abort-chunk", type=int, default=125,
                    help="samples per launch in the early-abort run (the cross-GPU flag is reduced between launches)")
    ap.add_argument("--noisy-trials", type=int, default=30,
                    help="config 5: RANSAC runs per size on sigma=1px noisy synthcurves (pose success rate); 0 disables")
    ap.add_argument("--noisy-samples", default="100,300,1000",
                    help="config 5: RANSAC samples per run (over all GPUs), comma-separated: the success-rate curve")
    ap.add_argument("--noisy-sigma", type=float, default=1.0)
    ap.add_argument("--streams", type=int, default=1,
                    help="HIP streams the timed steps rotate over: step i runs on stream i %% streams with its own "
                         "track buffers and workspace (1 = strictly serial launches, the reference's timer scope: "
                         "one launch -> sync per RANSAC run, GPU_HC_Solver.cpp:384,446)")
    ap.add_argument("--pipelined-streams", type=int, default=4,
                    help="also time the same steps overlapped on this many streams (one batch's tail overlaps the "
                         "next batch's start); reported as config.pipelined_paths_per_s, 0 disables")
    ap.add_argument("--cpu-samples-4t", type=int, default=40,
                    help="samples of the 4-thread CPU-HC run (the reference's Num_Of_Cores default)")
    ap.add_argument("--cpu-samples-ref", type=int, default=100,
                    help="samples of the reference-build CPU-HC run (plain operators + OpenBLAS 0.3.23 cgesv)")
    return ap.parse_args()


SCHEMA = 5   # bench-line schema: bumped when a field changes meaning (roofline.achieved is dense-priced since 4)


def launch_plan(gpus, environ):
    """How this process runs `--gpus N`: ("single", 1) for N = 1
    without a launcher; ("rank", N) when a launcher (torch.distributed.run) set
    WORLD_SIZE = N; ("spawn", N) for N > 1 without one: bench.py starts the N
    ranks itself (spawn_command) before anything touches the GPU.  A launcher
    whose WORLD_SIZE differs from --gpus is an error, never a silent N = 1 run."""
    if gpus < 1:
        raise SystemExit(f"[bench] --gpus must be >= 1 (got {gpus})")
    ws = environ.get("WORLD_SIZE")
    if ws is None or ws == "":
        return ("single", 1) if gpus == 1 else ("spawn", gpus)
    try:
        world = int(ws)
    except ValueError:
        raise SystemExit(f"[bench] WORLD_SIZE={ws!r} is not an integer")
    if world != gpus:
        raise SystemExit(f"[bench] --gpus {gpus} but the launcher started WORLD_SIZE={world} ranks")
    return ("rank", world) if world > 1 else ("single", 1)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn_command(gpus, argv, port):
    """The child that runs the N ranks: torch.distributed.run on 127.0.0.1, one
    process per GPU (LOCAL_RANK = device), this script with the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def spawn_ranks(gpus, argv):
    """Runs the ranks as a child process (never an exec: this process has not
    touched the GPU, and the ranks are fresh processes) and returns its exit
    code; non-zero when any rank failed to start or run."""
    import subprocess
    env = dict(os.environ, HC_BENCH_SPAWNED="1")
    try:
        # the ranks' stdout through a pipe: rank 0's JSON line to stdout, anything
        # else the ranks or their backend libraries print to stderr, so that
        # stdout holds the one bench line
        p = subprocess.Popen(spawn_command(gpus, argv, free_port()), env=env, stdout=subprocess.PIPE, text=True)
    except OSError as e:
        print(f"[bench] could not start {gpus} ranks: {e}", file=sys.stderr)
        return 1
    for line in p.stdout:
        print(line, end="", file=sys.stdout if line.startswith('{"metric"') else sys.stderr, flush=True)
    return p.wait() or 0


def rank_abort_record(g, runs, shard_paths, chunk_paths):
    """One rank's abort-leg record from its runs' (found itself, paths tracked,
    found byte) triples.  A rank that found nothing itself and tracked fewer
    paths than its shard was stopped by another rank's find; inside a launch
    when the count is not a whole number of chunks (the chunk-boundary
    reduction stops a rank only between chunks, the device flag inside one)."""
    tr = [int(x[1]) for x in runs]
    pstop = [not x[0] and int(x[1]) < shard_paths for x in runs]
    mid = [p and int(x[1]) % chunk_paths != 0 for p, x in zip(pstop, runs)]
    return {"rank": g, "shard_paths": shard_paths,
            "self_found_runs": int(sum(1 for x in runs if x[0])),
            "paths_tracked": {"median": int(np.median(tr)), "min": min(tr), "max": max(tr)},
            "peer_stopped_runs": int(sum(pstop)), "peer_stopped_mid_launch_runs": int(sum(mid))}


def gather_floats(vals, dev, world):
    """Every rank's list of floats (same length on every rank), rank-ordered."""
    if world == 1:
        return [list(vals)]
    import torch
    import torch.distributed as dist
    on = dev if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([float(v) for v in vals], dtype=torch.float64, device=on)
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.cpu().tolist() for p in parts]


def main():
    args = parse()
    mode, world = launch_plan(args.gpus, os.environ)
    if mode == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal of the N>1 path on a one-GPU box (never set by the driver):
    # HC_BENCH_DEVICE pins every rank to one device, HC_BENCH_BACKEND=gloo
    # replaces RCCL (which refuses two ranks on one GPU)
    dev_idx = int(os.environ.get("HC_BENCH_DEVICE", local_rank))
    backend = os.environ.get("HC_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    dist_world = 1
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        dist_world = dist.get_world_size()
        if dist_world != args.gpus:
            raise SystemExit(f"[bench] --gpus {args.gpus} but the process group has {dist_world} ranks")

    from trifocal_pose_estimation_using_improved_gpuhc_amd import (_abi, load_problem, load_ransac_data,
                                                                   prepare_target_params)
    from trifocal_pose_estimation_using_improved_gpuhc_amd.tracker import DeviceTracker

    problem = load_problem()
    data = load_ransac_data(0)
    S = args.samples
    total = S * world
    tgt_all, dif_all, _ = prepare_target_params(problem, data, seed=0, num_samples=total, num_gpus=world)
    # gpu-major shard of this rank (GPU_HC_Solver.cpp:85-88,263-265): equal shards here
    tgt = torch.from_numpy(tgt_all[rank * S:(rank + 1) * S]).to(dev)
    dif = torch.from_numpy(dif_all[rank * S:(rank + 1) * S]).to(dev)

    tr = DeviceTracker(problem, dev)
    res = tr.allocate(S, stats=True)
    stream = torch.cuda.current_stream(dev)

    # step i: batch i on stream i % ns with its own buffers and workspace (independent
    # RANSAC batches; a stream reuses its buffers only after its previous launch)
    NS = max(1, args.streams)
    NP = max(NS, args.pipelined_streams)
    # the serial leg runs on the current stream; the pipelined leg on streams of
    # its own (all non-default: the legacy default stream would order itself
    # against them)
    streams = [stream] + [torch.cuda.Stream(dev) for _ in range(NS - 1)]
    pstreams = [torch.cuda.Stream(dev) for _ in range(args.pipelined_streams)]
    bufs = [res] + [tr.allocate(S, stats=True) for _ in range(NP - 1)]
    wss = [tr.new_workspace(S) for _ in range(NP)]

    def step(i, ns, strs):
        k = i % ns
        with torch.cuda.stream(strs[k]):
            tr.reset_tracks(bufs[k])
        tr.launch(tgt, dif, bufs[k], stream=strs[k], workspace=wss[k])

    def timed(ns, strs):
        """W untimed warmup steps, then K steps bracketed by barrier + sync; max over ranks."""
        for i in range(max(args.warmup, ns)):   # every stream warm (its first launch pays for queue setup)
            step(i, ns, strs)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(i, ns, strs)
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t0          # this rank's own time (before the barrier)
        own.setdefault(ns, el)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        import ctypes
        for k in range(ns):   # a suspended path the time-slicing ring failed to hand over would show here
            st = int(tr.L.hc_trifocal_workspace_status(ctypes.c_void_p(wss[k].data_ptr())))
            if st != 0:
                raise RuntimeError(f"workspace {k}: status {st}")
        for k in range(1, min(ns, args.steps)):   # every batch is the same work: identical results on every stream
            if not (torch.equal(bufs[k].converge, res.converge) and torch.equal(bufs[k].stats, res.stats)
                    and torch.equal(bufs[k].tracks, res.tracks)):
                raise RuntimeError("streams disagree")
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el

    own = {}
    elapsed = timed(NS, streams)
    el_own = own[NS]
    pipe_elapsed = timed(args.pipelined_streams, pstreams) if args.pipelined_streams > 1 else None

    # kernel time of one launch alone (serial, HIP events on the launch stream): the
    # roofline's denominator and the latency of one batch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a_, b_ in ev:
        tr.reset_tracks(res)
        a_.record(stream)
        tr.launch(tgt, dif, res, stream=stream)
        b_.record(stream)
    torch.cuda.synchronize(dev)
    tr.workspace_status()   # raises on a device-side failure (table / time-slicing hand-over)
    launch_ms = np.array([a_.elapsed_time(b_) for a_, b_ in ev])
    # every rank's own kernel time (median of its 5 single launches) and wall time per step
    rank_ms = gather_floats([float(np.median(launch_ms)), el_own * 1e3 / args.steps], dev, world)

    # small launches (1 and 8 samples): the latency-mode tracking kernel the
    # launcher picks when a launch fills at most half of the path slots, against
    # the throughput kernel forced (hc_trifocal_set_small_launch)
    small = {"samples": [] if args.no_small_launch else [1, 8], "latency_kernel_ms": [], "throughput_kernel_ms": []}
    for n in small["samples"]:
        sb = tr.allocate(n)
        for mode, key in ((0, "latency_kernel_ms"), (-1, "throughput_kernel_ms")):
            _abi.lib().hc_trifocal_set_small_launch(mode)
            try:
                sev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(6)]
                for a_, b_ in sev:
                    tr.reset_tracks(sb)
                    a_.record(stream)
                    tr.launch(tgt[:n], dif[:n], sb, stream=stream)
                    b_.record(stream)
                torch.cuda.synchronize(dev)
            finally:
                _abi.lib().hc_trifocal_set_small_launch(0)
            small[key].append(round(float(np.median([a_.elapsed_time(b_) for a_, b_ in sev[1:]])), 4))
        del sb
    tr.workspace_status()

    # the papers' ablation ladder: the same launch through the archived
    # ..._PH (explicit RK, no truncation) and ..._PH_CodeOpt (no truncation) semantics
    ab_buf = tr.allocate(S, stats=True)

    def ablation(**kw):
        aev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(3)]
        for a_, b_ in aev:
            tr.reset_tracks(ab_buf)
            a_.record(stream)
            tr.launch(tgt, dif, ab_buf, stream=stream, truncate=False, **kw)
            b_.record(stream)
        torch.cuda.synchronize(dev)
        tr.workspace_status()
        h = ab_buf.host()
        return (float(np.median([a_.elapsed_time(b_) for a_, b_ in aev])),
                int(4 * h["stats"]["steps"].astype(np.int64).sum() + h["stats"]["corrections"].astype(np.int64).sum()))
    ph_ms, ph_stages = ablation(explicit_rk=True)
    phc_ms, phc_stages = ablation()
    del ab_buf

    # device pose recovery + maximal support over the launch's tracks,
    # timed separately with HIP events on the same stream
    from trifocal_pose_estimation_using_improved_gpuhc_amd import pose as P
    tr.set_ransac_data(data)
    inl = torch.empty((S * 312, 2), dtype=torch.int32, device=dev)
    sel = torch.empty(P.SEL_BYTES, dtype=torch.uint8, device=dev)
    pev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a_, b_ in pev:
        a_.record(stream)
        P.launch_pose_support(res.tracks, res.converge, tr.edgels, tr.K, inl, sel, stream=stream)
        b_.record(stream)
    torch.cuda.synchronize(dev)
    pose_ms = float(np.median([a_.elapsed_time(b_) for a_, b_ in pev]))
    merged = sharding_gather(sel, rank * S * 312)
    pose_res, pose_ok = P.residuals(data, merged)

    host = res.host()
    steps_sum = int(host["stats"]["steps"].astype(np.int64).sum())
    corr_sum = int(host["stats"]["corrections"].astype(np.int64).sum())
    flops = steps_sum * 4 * FLOP_PRED_STAGE + corr_sum * FLOP_CORR_STAGE          # dense-LU convention
    bid = _abi.build_id()
    lu_frac, lu_frac_src = lu_executed_fraction(bid)
    flops_exec = None if lu_frac is None else \
        flops - (steps_sum * 4 + corr_sum) * LU_UPDATE_DENSE_FLOP * (1.0 - lu_frac)   # LU updates as executed
    from trifocal_pose_estimation_using_improved_gpuhc_amd import count_solutions
    counts = count_solutions(host["tracks"], host["converge"], host["infinity"])

    t_max = elapsed                 # already the max over ranks
    ms_per_step = t_max / args.steps * 1e3
    paths = 312 * S * world
    value = paths / (ms_per_step / 1e3)
    pipelined = None if pipe_elapsed is None else paths * args.steps / pipe_elapsed

    # ---- early abort (config 3 at N=1, config 4 at N=8): time-to-first-good-pose.
    # Every rank tracks its gpu-major shard of abort_samples*world samples in
    # chunks; the found flag is max-reduced over ranks (RCCL) after each chunk
    # (sharding.run_abort_chunks), so all ranks stop once any rank has a pose.
    abort_info = None
    if args.abort_samples > 0:
        from trifocal_pose_estimation_using_improved_gpuhc_amd import sharding
        Sa = args.abort_samples
        ta_all, da_all, _ = prepare_target_params(problem, data, seed=0, num_samples=Sa * world, num_gpus=world)
        off, cnt = sharding.shard(Sa * world, world, rank)
        ta = torch.from_numpy(ta_all[off:off + cnt]).to(dev)
        da = torch.from_numpy(da_all[off:off + cnt]).to(dev)
        tr.set_ransac_data(data)
        ra = tr.allocate(cnt, stats=True, abort=True)
        wss = []
        abort_info = {"samples_total": Sa * world, "samples_per_gpu": Sa, "chunk_samples": args.abort_chunk}
        # the cross-process device flag (hcAbortArgs::peer_found): every GPU stops
        # within a path of any GPU's find, not at its next chunk boundary
        peer = sharding.SharedFlag(device=dev) if world > 1 else None
        if peer is not None:
            abort_info["cross_rank_flag_memory"] = peer.memory_kind
            abort_info["cross_rank_stop"] = ("device flag over xGMI (hipIpc) + RCCL all_reduce at chunk boundaries"
                                             if peer.ptr is not None else
                                             f"RCCL all_reduce at chunk boundaries only ({peer.error})")
        n_chunks = len(sharding.chunks(cnt, args.abort_chunk))

        def abort_run(inflight):
            """One config-3 run of this rank's shard: (first-pose seconds, min over
            ranks; wall seconds, max over ranks; paths tracked, summed over ranks;
            this rank's [self found, paths tracked, found byte] of every rank)."""
            tr.reset_tracks(ra)
            torch.cuda.synchronize(dev)
            if peer is not None:
                peer.arm(stream)          # zeroed by its owner, then a barrier
            elif world > 1:
                dist.barrier()
            w0 = time.perf_counter()
            tr.launch_abort_chunked(ta, da, ra, args.abort_chunk, wss, stream=stream, inflight_stop=inflight,
                                    peer_found=peer if peer is not None and peer.ptr is not None else None,
                                    max_count=sharding.max_shard(Sa * world, world))
            torch.cuda.synchronize(dev)
            w = time.perf_counter() - w0
            hz = tr.read_timestamps(wss[0])[2]
            stamps = [tr.read_timestamps(x)[:2] for x in wss[:n_chunks]]
            f = sharding.first_found_seconds(stamps, hz)
            n_tr = int((ra.stats[:, 0] > 0).sum().item())
            # per rank: did it find a pose itself (a found stamp in one of its own
            # launches), how many of its shard's paths it tracked, and the found
            # byte it ended with (its own find, the peer flag or the chunk reduction)
            self_found = any(fs for _, fs in stamps)
            pr = gather_floats([1.0 if self_found else 0.0, float(n_tr), float(bool(ra.found.item()))], dev, world)
            if world > 1:
                v = torch.tensor([f if f >= 0 else 1e30, -w, -float(n_tr)], dtype=torch.float64, device=dev)
                dist.all_reduce(v, op=dist.ReduceOp.MIN)
                f, w = float(v[0].item()), -float(v[1].item())
                f = -1.0 if f >= 1e29 else f
                nt = torch.tensor([n_tr], dtype=torch.int64, device=dev)
                dist.all_reduce(nt)
                n_tr = int(nt.item())
            return f, w, n_tr, pr

        for inflight in (False, True):
            ttfp, wall, tracked = [], [], []
            found_runs, per_rank_runs = [], []
            for _ in range(args.abort_repeats):
                f, w, n_tr, pr = abort_run(inflight)
                per_rank_runs.append(pr)
                found_runs.append(bool(ra.found.item()))
                ttfp.append(f)
                wall.append(w)
                tracked.append(n_tr)
            key = "inflight_stop" if inflight else "reference_semantics"
            ok = [f for f in ttfp if f >= 0]
            spread = lambda v: {"median": round(float(np.median(v)) * 1e3, 3),  # noqa: E731
                                "min": round(float(np.min(v)) * 1e3, 3), "max": round(float(np.max(v)) * 1e3, 3)}
            shards = [sharding.shard(Sa * world, world, g)[1] * 312 for g in range(world)]
            chunk_paths = args.abort_chunk * 312
            ranks = [rank_abort_record(g, [pr[g] for pr in per_rank_runs], shards[g], chunk_paths)
                     for g in range(world)]
            abort_info[key] = {
                "found": all(found_runs),
                "found_runs": int(sum(found_runs)),
                "runs": len(ttfp),
                "time_to_first_good_pose_ms": spread(ok) if ok else None,
                "kernel_exit_wall_ms": spread(wall),
                "paths_tracked": int(np.median(tracked)),
                "per_rank": ranks,
                "peer_stop_observed": any(r_["peer_stopped_runs"] > 0 for r_ in ranks),
                "peer_stop_mid_launch_observed": any(r_["peer_stopped_mid_launch_runs"] > 0 for r_ in ranks)}
        # the first pose over other RANSAC draws of the same data (VERDICT r5:
        # one seed measures one path's latency): srand(1..K), reference semantics,
        # the median of a few runs each and where the first passing sample sits
        seeds = []
        for sd in range(1, args.abort_seeds + 1):
            ts_all, ds_all, _ = prepare_target_params(problem, data, seed=sd, num_samples=Sa * world, num_gpus=world)
            ta.copy_(torch.from_numpy(ts_all[off:off + cnt]))
            da.copy_(torch.from_numpy(ds_all[off:off + cnt]))
            fs = [abort_run(False)[0] for _ in range(args.abort_seed_repeats)]
            bi = ra.batch_index.cpu().numpy()
            hit = np.nonzero(bi >= 0)[0]
            first = float(off + hit[0] // 312) if len(hit) else 1e30
            if world > 1:
                v = torch.tensor([first], dtype=torch.float64, device=dev)
                dist.all_reduce(v, op=dist.ReduceOp.MIN)
                first = float(v.item())
            ok = [f for f in fs if f >= 0]
            seeds.append({"srand": sd, "first_passing_sample": None if first >= 1e29 else int(first),
                          "time_to_first_good_pose_ms": round(float(np.median(ok)) * 1e3, 3) if ok else None})
        if seeds:
            got = [x["time_to_first_good_pose_ms"] for x in seeds if x["time_to_first_good_pose_ms"] is not None]
            abort_info["across_seeds"] = {
                "runs_per_seed": args.abort_seed_repeats, "seeds": seeds,
                "found_seeds": len(got), "median_ms": round(float(np.median(got)), 3) if got else None,
                "quartiles_ms": [round(float(np.percentile(got, 25)), 3), round(float(np.percentile(got, 75)), 3)]
                if got else None,
                "note": "dataset 000, samples srand(1..K) instead of srand(0); reference semantics; the time "
                        "follows where the first passing hypothesis sits in the sample order"}
        if peer is not None:
            peer.close()
        abort_info["note"] = ("device clock (s_memrealtime, rate from hipDeviceAttributeWallClockRate) from the "
                              "first chunk's start, min over ranks; wall = host time to the all-GPU sync, max "
                              "over ranks.  reference_semantics: paths in flight when the pose is found run to "
                              "completion (..._TrunRANSAC.cu:148-152); inflight_stop: they stop at their next "
                              "step boundary (hcAbortArgs::inflight_stop)")

    noisy_info = None
    if args.noisy_trials > 0:
        noisy_info = noisy_pose_leg(args, tr, problem, data, world, rank, dev, stream)

    if rank == 0:
        med_launch_s = float(np.median(launch_ms)) / 1e3
        achieved_tf = flops / med_launch_s / 1e12                  # the reference's (dense) LU
        achieved_exec_tf = None if flops_exec is None else flops_exec / med_launch_s / 1e12
        tb, traffic_src = traffic_bytes(TRACK_KERNEL, bid)
        traffic, traffic_ns = (None, None) if tb is None else tb
        # HBM rate: the profile's bytes over the same profile's kernel time (ADVICE r5:
        # this run's kernel time is contended when a rehearsal pins every rank to one GPU)
        hbm_s = None if traffic is None else ((traffic_ns or float(np.median(launch_ms)) * 1e6) / 1e9)
        alg_bytes = algorithmic_bytes(S)
        k_ms = [r_[0] for r_ in rank_ms]
        line = {
            "metric": "HC paths/sec (312 tracks x RANSAC samples)",
            "value": round(value, 1),
            "unit": "paths/s",
            "n_gpus": world,
            "world_size": dist_world,
            "schema": SCHEMA,
            "distributed": {
                "launcher": ("bench.py (torch.distributed.run child it started)" if os.environ.get("HC_BENCH_SPAWNED")
                             else "external (WORLD_SIZE set)") if world > 1 else "none (one process)",
                "backend": dist.get_backend() if world > 1 else None,
                "world_size_reported_by": "torch.distributed.get_world_size()" if world > 1 else None,
                "devices": ("all ranks on cuda:%d (rehearsal)" % dev_idx) if "HC_BENCH_DEVICE" in os.environ
                           else "cuda:LOCAL_RANK",
                "per_rank_kernel_ms": [round(v, 4) for v in k_ms],
                "kernel_ms_min": round(min(k_ms), 4), "kernel_ms_max": round(max(k_ms), 4),
                "per_rank_step_ms": [round(r_[1], 4) for r_ in rank_ms],
                "note": "kernel ms = median of each rank's 5 single config-2 launches (HIP events); step ms = "
                        "the rank's own timed-loop time per step before the closing barrier; ms_per_step is "
                        "the max over ranks after it"},
            "ms_per_step": round(ms_per_step, 4),
            "steps": args.steps,
            "warmup": args.warmup,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic RANSAC samples from the reference's synthcurves data (Triplet_Edgels_000, srand(0))",
            "config": {"workload": "trifocal_2op1p_30x30 config 2: 100 RANSAC samples x 312 tracks per GPU, "
                                   "Abort_RANSAC=false",
                       "samples_per_gpu": S, "tracks_per_sample": 312, "paths_per_step": paths,
                       "streams": NS,
                       "step": "reset tracks + one tracking launch; steps serialised on one stream, each a "
                               "launch -> sync of one RANSAC batch (the reference's timer scope, "
                               "GPU_HC_Solver.cpp:384,446)" if NS == 1 else
                               f"reset tracks + one tracking launch, steps rotating over {NS} streams",
                       "single_launch_paths_per_s": round(paths / (float(np.median(launch_ms)) / 1e3), 1),
                       "pipelined_paths_per_s": None if pipelined is None else round(pipelined, 1),
                       "small_launch": dict(small, note="ms per tracking launch of 1 / 8 samples (median of 5, HIP "
                                                         "events): the latency-mode kernel the launcher picks at "
                                                         "most half of the path slots, and the throughput kernel "
                                                         "forced"),
                       "pipelined_streams": args.pipelined_streams if pipelined is not None else None,
                       "pipelined_note": "the same K steps with consecutive batches overlapped on "
                                         f"{args.pipelined_streams} streams (own buffers each): a batch's "
                                         "tail runs beside the next batch's start; not the headline",
                       "parallelism": f"samples sharded over {world} GPU(s), no data-path collective",
                       "GPUHC_Max_Steps": tr.settings.max_steps,
                       "GPUHC_Max_Correction_Steps": tr.settings.max_corrections,
                       "kernel": _abi.lib().hc_trifocal_version().decode(),
                       "build_id": bid},
            "roofline": {"bound": "valu_fp32", "achieved": round(achieved_tf, 3), "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved_tf / FP32_PEAK_TFLOPS, 4),
                         "traffic": traffic,
                         "traffic_source": traffic_src,
                         # north_star's "achieved HBM GB/s fraction from rocprof" (VERDICT r4 #2):
                         # the PMC bytes of this build over this run's kernel time
                         "hbm_gbs": None if traffic is None else round(traffic / hbm_s / 1e9, 3),
                         "hbm_frac": None if traffic is None else round(traffic / hbm_s / 1e9 / HBM_PEAK_GBS, 6),
                         "hbm_kernel_ms": None if traffic is None else round(hbm_s * 1e3, 4),
                         "hbm_peak_gbs": HBM_PEAK_GBS,
                         "algorithmic_bytes": alg_bytes,
                         "algorithmic_gbs": round(alg_bytes / (float(np.median(launch_ms)) / 1e3) / 1e9, 3),
                         "traffic_over_algorithmic": None if traffic is None else round(traffic / alg_bytes, 3),
                         "traffic_unit": "HBM bytes per launch of the same kernel (rocprofv3 FETCH_SIZE x2 gfx950 "
                                         "correction + WRITE_SIZE, separate --pmc passes, scripts/gpu.sh profile); "
                                         "algorithmic_bytes: the compulsory bytes of the same launch (bench.algorithmic_bytes, ~0.5 KB/path); "
                                         "hbm_gbs / hbm_frac: traffic / the same profile's average kernel time "
                                         "(hbm_kernel_ms, its rocprofv3 kernel trace), / 8 TB/s",
                         "note": "FP32 VALU-issue/latency bound tracker kernel (no GEMM: 30x30 complex LUs of "
                                 "rank-1 updates); peak = MI355X FP32 vector peak 157.3 TF. achieved = algorithmic "
                                 "FLOPs of the launch's stages (SURVEY 8d: 104.3 kFLOP / predictor stage, 101.3 "
                                 "kFLOP / corrector stage, the LU priced as the reference's dense algorithm) / "
                                 "median single-launch kernel time (HIP events on the launch stream). "
                                 "achieved_executed_lu prices the LU's rank-1 updates over the column groups the "
                                 "structurally sparse LU executes (lu_executed_fraction of the dense 68.4 kFLOP, "
                                 "measured by the HC_DIAG_LUWORK build of this build's sources, "
                                 "lu_executed_fraction_source): the stricter figure.  traffic and the LU fraction "
                                 "come only from profiles stamped with this build_id (null with the reason "
                                 "otherwise).",
                         "achieved_executed_lu": None if achieved_exec_tf is None else round(achieved_exec_tf, 3),
                         "frac_executed_lu": None if achieved_exec_tf is None else
                         round(achieved_exec_tf / FP32_PEAK_TFLOPS, 4),
                         "lu_executed_fraction": None if lu_frac is None else round(lu_frac, 4),
                         "lu_executed_fraction_source": lu_frac_src,
                         "kernel_ms": round(float(np.median(launch_ms)), 4),
                         "executed_gflop_per_launch": None if flops_exec is None else round(flops_exec / 1e9, 3),
                         "dense_lu_gflop_per_launch": round(flops / 1e9, 3),
                         "rk4_steps": steps_sum, "corrections": corr_sum},
            "solutions": {"converged": counts[0], "real": counts[1], "infinity": counts[2]},
            "pose": {"pose_support_ms": round(pose_ms, 4), "candidates": merged["num_candidates"],
                     "path21": merged["path21"], "path31": merged["path31"], "inliers21": merged["inliers21"],
                     "inliers31": merged["inliers31"], "gt_match": pose_ok,
                     "residuals": [round(float(v), 6) for v in pose_res],
                     "note": "device candidate filter + Cayley pose + reprojection inlier scoring of every "
                             "candidate over all triplet edgels + maximal-support selection "
                             "(Evaluations.cpp:298-504), merged over ranks (RCCL all_gather)"},
        }
        tp_ms = float(np.median(launch_ms))
        leg = lambda ms, st: {"kernel_ms": round(ms, 4), "paths_per_s": round(312 * S / (ms / 1e3), 1),  # noqa: E731
                              "stages": st}
        line["ablation"] = {
            "note": "the papers' incremental strategies on MI355X: the same config-2 launch (single launch, HIP "
                    "events) through the archived ..._PH semantics (direct parameter homotopy, explicit RK "
                    "helpers; hc_trifocal_2op1p_30x30_track_ph), ..._PH_CodeOpt (loopy RK; "
                    "hc_trifocal_2op1p_30x30_track_ph_codeopt) and ..._PH_CodeOpt_TrunPaths (depth-sign path "
                    "truncation, ..._TrunPaths.cu:148-155; the headline kernel).  P2C is not built: its "
                    "parameter-to-coefficient generator is not in the reference",
            "ph": leg(ph_ms, ph_stages),
            "ph_codeopt": leg(phc_ms, phc_stages),
            "ph_codeopt_trunpaths": leg(tp_ms, steps_sum * 4 + corr_sum),
            "trunpaths_speedup_over_ph_codeopt": round(phc_ms / tp_ms, 3)}
        if noisy_info is not None:
            line["noisy_pose"] = noisy_info
        if abort_info is not None:
            line["early_abort"] = abort_info
        if not args.no_cpu_baseline and world == 1:   # the CPU baseline is timed at N = 1 only
            line["cpu_baseline"] = cpu_baseline(problem, data, args.cpu_samples, args.cpu_samples_4t,
                                                args.cpu_samples_ref, value)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def sharding_gather(sel, path_offset):
    from trifocal_pose_estimation_using_improved_gpuhc_amd import sharding
    return sharding.gather_pose_selection(sel, path_offset)


def wilson95(k, n):
    """Wilson 95 % score interval of a binomial proportion k / n."""
    if n == 0:
        return None
    z = 1.959964
    p = k / n
    c = (p + z * z / (2 * n)) / (1 + z * z / n)
    h = z * np.sqrt(p * (1 - p) / n + z * z / (4 * n * n)) / (1 + z * z / n)
    return [round(float(c - h), 4), round(float(c + h), 4)]


def noisy_pose_leg(args, tr, problem, data, world, rank, dev, stream):
    """BASELINE.json config 5 (path pruning is always on in the tracker) as a
    curve: for each RANSAC size in --noisy-samples (samples per run over all
    ranks), `--noisy-trials` runs on sigma-px noisy synthcurves, one noise seed
    and one sample draw (srand(trial)) per run; each run = track + device pose
    support, selection merged over ranks; success = the selected pose matches
    GT within the reference's 0.1 rad / 0.1 tolerances (Evaluations.cpp:523-543).
    Reported per size: success rate with its Wilson 95 % interval, paths/s of
    the track + pose phase, ms per run."""
    import torch
    import torch.distributed as dist

    from trifocal_pose_estimation_using_improved_gpuhc_amd import pose as P
    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params, sharding, synthcurves
    sizes = [int(v) for v in str(args.noisy_samples).split(",") if v.strip()]
    noisy = [synthcurves.noisy(data, args.noisy_sigma, synthcurves.DEFAULT_SEED + t) for t in range(args.noisy_trials)]
    curve = []
    for total in sizes:
        off, cnt = sharding.shard(total, world, rank)
        S = max(1, sharding.max_shard(total, world))
        res = tr.allocate(S, stats=False)
        inl = torch.empty((S * 312, 2), dtype=torch.int32, device=dev)
        sel = torch.empty(P.SEL_BYTES, dtype=torch.uint8, device=dev)
        ok_list, okc_list, times, cands = [], [], [], []
        for t in range(args.noisy_trials):
            nd = noisy[t]
            ta, da, _ = prepare_target_params(problem, nd, seed=t, num_samples=total, num_gpus=world)
            tg = torch.from_numpy(ta[off:off + cnt]).to(dev)
            df = torch.from_numpy(da[off:off + cnt]).to(dev)
            tr.set_ransac_data(nd)
            tr.reset_tracks(res)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            if cnt > 0:
                tr.launch(tg, df, res, stream=stream, num_samples=cnt)
                P.launch_pose_support(res.tracks[:cnt * 312], res.converge[:cnt * 312], tr.edgels, tr.K,
                                      inl[:cnt * 312], sel, stream=stream)
            torch.cuda.synchronize(dev)
            if world > 1:
                dist.barrier()
            times.append(time.perf_counter() - t0)
            m = sharding.gather_pose_selection(sel, off * 312)
            out, ok = P.residuals(nd, m)
            ok_list.append(ok)
            okc_list.append(P.success_clamped(nd, m, out))
            cands.append(m["num_candidates"])
        tt = float(np.sum(times))
        if world > 1:
            v = torch.tensor([tt], dtype=torch.float64, device=dev)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            tt = float(v.item())
        k = int(np.sum(ok_list))
        curve.append({"samples_per_run": total, "trials": args.noisy_trials, "successes": k,
                      "success_rate": round(k / args.noisy_trials, 4),
                      "success_rate_95ci": wilson95(k, args.noisy_trials),
                      "successes_acos_clamped": int(np.sum(okc_list)),
                      "paths_per_s": round(312 * total * args.noisy_trials / tt, 1),
                      "ms_per_run": round(tt / args.noisy_trials * 1e3, 3),
                      "median_candidates": int(np.median(cands))})
        del res, inl
    tr.set_ransac_data(data)
    head = next((c for c in curve if c["samples_per_run"] == 100 * world), curve[0])
    return {"workload": "config 5: path pruning (depth-sign truncation, always on) + sigma=%g px noisy "
                        "synthcurves (Triplet_Edgels_000, noise seed 20250215+trial, samples srand(trial)), "
                        "track + device pose support per RANSAC run, at several RANSAC sizes" % args.noisy_sigma,
            "sigma_px": args.noisy_sigma, "trials": args.noisy_trials,
            "samples_per_run": head["samples_per_run"], "success_rate": head["success_rate"],
            "paths_per_s": head["paths_per_s"], "ms_per_run": head["ms_per_run"],
            "median_candidates": head["median_candidates"], "curve": curve}


def algorithmic_bytes(samples):
    """Compulsory HBM bytes of one config-2 launch over `samples` samples (SURVEY
    §8(d)): per path the 31-entry start / track row read (248 B), the
    30 solved entries written back (240 B), converge + infinity (2 B) and the
    stats record (16 B); per sample the target and diff parameters (2 x 34 c64);
    per launch the unified index table (38 880 int32) and the start parameters."""
    return 312 * samples * (31 * 8 + 30 * 8 + 2 + 16) + samples * 2 * 34 * 8 + 38880 * 4 + 34 * 8


def traffic_bytes(kernel, bid):
    """HBM bytes per launch of `kernel` and that profile's own average kernel
    time (ns, its rocprofv3 kernel trace) from the PMC summary of this build
    (PMC counters cannot be collected inside the timed run): ((bytes, ns), file)
    or (None, reason)."""
    return _profiles_of_build("*_pmc_summary.json", bid,
                              lambda d: (d["derived"]["hbm_bytes_per_launch"], d.get("avg_ns"))
                              if d.get("kernel") == kernel and d.get("derived", {}).get("hbm_bytes_per_launch")
                              else None)


def cpu_info():
    """Host CPU model, logical CPUs and physical cores (/proc/cpuinfo)."""
    model, phys = None, set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if ":" not in line:
                    if cur:
                        phys.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, v = (x.strip() for x in line.split(":", 1))
                cur[k] = v
                if k == "model name" and model is None:
                    model = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    return model, os.cpu_count(), len(phys) or None


def reference_build_cpuhc(threads, n):
    """The CPU-HC restatement built the way the reference's CPU build is (plain host
    operators, GCC contraction) and solving through OpenBLAS 0.3.23 `cgesv` with its
    Haswell kernels -- the configuration that reproduces CPU_Sols_Statistics.txt
    exactly (tests/test_oracle_kat.py) -- timed on `threads` threads over config-2
    samples 0..n-1.  Runs tests/cpuhc_pin.py's child in its own process (the
    OpenBLAS kernel set is chosen when the library loads); None if the image lacks
    that OpenBLAS."""
    import subprocess
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OPENBLAS_CORETYPE="Haswell", OMP_NUM_THREADS=str(threads))
    try:
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "plain"], check=True, capture_output=True)
        p = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "cpuhc_pin.py"), "--child", "plain",
                            "openblas:Haswell", str(n)], env=env, capture_output=True, text=True, timeout=300)
        r = json.loads(p.stdout.strip().splitlines()[-1])
    except (OSError, ValueError, IndexError, subprocess.SubprocessError):
        return None
    if "counts" not in r:
        return None
    return {"value": round(312 * n / r["seconds"], 1), "cores": threads, "samples": n, "seconds": r["seconds"],
            "openblas": r.get("openblas_config"),
            "note": "CPU-HC as the reference builds it: plain MAGMA-order operators with GCC FMA contraction "
                    "(CMakeLists.txt:36,57) + OpenBLAS 0.3.23 cgesv (Haswell kernels), the configuration that "
                    "reproduces Output_Write_Files/CPU_Sols_Statistics.txt exactly"}


def cpu_baseline(problem, data, n_samples, n_samples_4t, n_samples_ref, gpu_value):
    """CPU baselines on this host's cores, bounded samples of the config-2 workload:
      value        the oracle's CPU-HC restatement (CPUHC_Generic_Solver_Eval_by_Indx
                   semantics: no path pruning, LAPACK-style cgesv, OpenMP dynamic
                   over paths) on the threads this job may use (OMP_NUM_THREADS,
                   16 per GPU on the GPU box; capped by the host's cores);
      threads4     the same on 4 threads (the reference's Num_Of_Cores default,
                   gpuhc_settings.yaml:34);
      pruned       the oracle's GPU-semantics tracker (depth-sign pruning, the work
                   the GPU does) on the same threads: the apples-to-apples ratio."""
    from oracle import oracle as O
    from trifocal_pose_estimation_using_improved_gpuhc_amd import prepare_target_params
    model, logical, physical = cpu_info()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or 16
    threads = max(1, min(share, physical or logical or 1))
    tgt, dif, _ = prepare_target_params(problem, data, seed=0, num_samples=max(n_samples, n_samples_4t))

    def run(n, th):
        _, _, _, _, secs = O.cpuhc_track(problem.start_sols, problem.start_params, tgt[:n], dif[:n],
                                         problem.dHdx_index, problem.dHdt_index, O.settings(threads=th))
        return 312 * n / secs, secs
    v, secs = run(n_samples, threads)
    v4, secs4 = run(n_samples_4t, 4)
    ref = reference_build_cpuhc(threads, n_samples_ref)
    t0 = time.perf_counter()
    O.gpuhc_track(problem.start_sols, problem.start_params, tgt[:n_samples], dif[:n_samples], problem.unified_index,
                  O.settings(threads=threads))
    secs_p = time.perf_counter() - t0
    vp = 312 * n_samples / secs_p
    return {"value": round(v, 1), "unit": "paths/s", "cores": threads, "kind": "port",
            "sample": f"CPU-HC restatement (oracle/hc_oracle.c orc_cpuhc_track, no path pruning, LAPACK-style "
                      f"cgesv) on config-2 samples 0..{n_samples - 1} ({312 * n_samples} paths), {secs:.1f} s "
                      f"wall on {threads} threads",
            "cpu_model": model, "host_logical_cpus": logical, "host_physical_cores": physical,
            "threads_note": "threads = this job's CPU share (OMP_NUM_THREADS; the GPU box allots 16 per GPU), "
                            "capped by the physical cores.  No all-physical-cores leg: the box's 128 cores are "
                            "shared with other jobs and this job may use 16 threads, so a 128-thread run would "
                            "exceed its CPU share (the per-thread rate scales the 16-thread value)",
            "threads4": {"value": round(v4, 1), "cores": 4, "samples": n_samples_4t, "seconds": round(secs4, 2),
                         "note": "Num_Of_Cores default of gpuhc_settings.yaml:34"},
            "pruned_gpu_semantics": {"value": round(vp, 1), "cores": threads, "samples": n_samples,
                                     "seconds": round(secs_p, 2),
                                     "note": "oracle orc_gpuhc_track: the GPU kernel's semantics (depth-sign "
                                             "pruning) on the same threads"},
            "reference_build": ref,
            "gpu_over_cpu": round(gpu_value / v, 1),
            "gpu_over_cpu_reference_build": round(gpu_value / ref["value"], 1) if ref and ref.get("value") else None,
            "gpu_over_cpu_pruned": round(gpu_value / vp, 1),
            "gpu_over_cpu_4threads": round(gpu_value / v4, 1)}


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Offline model of one config-2 launch's schedule (development tool, CPU).

Paths carry their measured costs (golden N=100 run: steps, corrections);
10240 path slots (1280 workgroups x 4 waves x 2 halves) take work from the
queue; a stage takes tau = max(LONE, FULL * busy / slots) microseconds (lone
wave latency vs. the throughput-bound rate at full load).
Policies: the built-in per-track order, clairvoyant LPT, and round-robin
time slicing with a quantum of Q steps (paths that are not finished after Q
steps are suspended to a FIFO and resumed after the new paths).

    python scripts/sched_sim.py
"""
import collections
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LONE, FULL, SLOTS, DT = 23.6, 40.0, 10240, 20.0   # us, us, slots, us per tick


def load():
    g = np.load(os.path.join(ROOT, "tests", "golden", "gpuhc_N100_seed0.npz"))
    steps = g["steps"].astype(np.int64)
    cost = 4 * steps + g["corrections"].astype(np.int64)
    order = []
    with open(os.path.join(ROOT, "trifocal_pose_estimation_using_improved_gpuhc_amd", "csrc", "hc_track_order.inc")) as f:
        for line in f:
            if not line.startswith("//"):
                order += [int(v) for v in line.replace(",", " ").split()]
    return steps, cost, np.array(order)


def simulate(queue, steps, cost, quantum=None, resume_first=False):
    """queue: path ids in dequeue order.  Returns (makespan ms, utilisation)."""
    per_step = cost / np.maximum(steps, 1)
    done_steps = np.zeros(cost.size)
    q = collections.deque(int(p) for p in queue)
    rq = collections.deque()
    slot_p = np.full(SLOTS, -1)
    slot_left = np.zeros(SLOTS)      # stages left in the slot's current piece
    t, busy_int = 0.0, 0.0

    def piece(p):
        rem_steps = steps[p] - done_steps[p]
        if quantum is None or rem_steps <= quantum:
            n = rem_steps
        else:
            n = quantum
        done_steps[p] += n
        return n * per_step[p], rem_steps > n

    suspended = np.zeros(cost.size, bool)
    while True:
        free = np.flatnonzero(slot_p < 0)
        for s in free:
            src = (rq or q) if resume_first else (q or rq)
            if not src:
                break
            p = src.popleft()
            slot_p[s] = p
            slot_left[s], suspended[p] = piece(p)
        act = slot_p >= 0
        n = int(act.sum())
        if n == 0 and not q and not rq:
            break
        tau = max(LONE, FULL * n / SLOTS)
        slot_left[act] -= DT / tau
        fin = act & (slot_left <= 0)
        for s in np.flatnonzero(fin):
            p = slot_p[s]
            if suspended[p]:
                rq.append(p)
            slot_p[s] = -1
        busy_int += n * DT
        t += DT
    return t / 1e3, busy_int / (t * SLOTS)


def main():
    steps, cost, track_order = load()
    n = cost.size
    S = n // 312
    builtin = np.array([s * 312 + k for k in track_order for s in range(S)])
    lpt = np.argsort(-cost, kind="stable")
    print("builtin", simulate(builtin, steps, cost))
    print("lpt", simulate(lpt, steps, cost))
    print("natural", simulate(np.arange(n), steps, cost))
    for Q in (5, 10, 20, 40):
        print(f"rr Q={Q}", simulate(builtin, steps, cost, quantum=Q))


if __name__ == "__main__":
    main()

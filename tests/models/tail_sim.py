"""Launch-tail simulation for C3: persistent waves of 64 lanes
take tickets of consecutive units (pixel-major samples) from one queue; a lane
runs a unit for ~1.36 iterations per traced ray (the steady state's
iterations per ray) and refills from its wave's window. The tail is the time
from the queue running dry to the last lane's end. Unit lengths: the traced
rays of real samples from the C oracle (tests/models/tail_model.c: 4000 random
pixels x 100 samples, the trapped-path exit applied); the pixel order is the
reference's, reversed, or longest-first by an estimate from other samples.

    /tmp/tail_model 4000 100 /tmp/tail_L.bin && python tests/models/tail_sim.py /tmp/tail_L.bin
"""
import heapq
import sys

import numpy as np

path = sys.argv[1]
NP, NS = 4000, 100
raw = np.fromfile(path, dtype=np.int32)
L = raw[:NP * NS].reshape(NP, NS)
ij = raw[NP * NS:].reshape(NP, 2)
est = L[:, :NS // 2].mean(axis=1)          # per-pixel estimate from samples 0..49
units_L = L[:, NS // 2:]                    # simulated units: samples 50..99
ITER_PER_RAY = 1.36
LANES_PER_WAVE = 64


def simulate(order, waves, ticket_phases=((256, 0.75), (64, 1.0))):
    """order: pixel indices; returns (end, first_dry, tail) in iterations."""
    u = units_L[order].reshape(-1) * ITER_PER_RAY + 1.0  # +1: the refill iteration
    n = len(u)
    nxt = 0  # next unit of the queue
    # per wave: its window [a, b)
    win = [[0, 0] for _ in range(waves)]
    dry = [None] * waves
    lanes = []  # (time free, wave)
    for w in range(waves):
        for _ in range(LANES_PER_WAVE):
            lanes.append((0.0, w))
    heapq.heapify(lanes)
    end = 0.0
    while lanes:
        t, w = heapq.heappop(lanes)
        a, b = win[w]
        if a >= b:  # the window is empty: take a ticket
            if nxt >= n:
                if dry[w] is None:
                    dry[w] = t
                end = max(end, t)
                continue
            size = next(sz for sz, frac in ticket_phases if nxt < frac * n)
            a, b = nxt, min(n, nxt + size)
            nxt = b
        win[w] = [a + 1, b]
        heapq.heappush(lanes, (t + u[a], w))
    first_dry = min(d for d in dry if d is not None)
    return end, first_dry


ref = np.lexsort((ij[:, 0], -ij[:, 1]))   # top row first, left to right (unit order)
orders = {"reference": ref, "reversed": ref[::-1], "longest_first": np.argsort(-est, kind="stable")}
waves = int(round(units_L.size / 244 / LANES_PER_WAVE))  # C3: ~244 units per lane per frame
for name, o in orders.items():
    end, dry = simulate(o, waves)
    print({"order": name, "waves": waves, "end_iter": round(end, 1), "first_dry_iter": round(dry, 1),
           "tail_iter": round(end - dry, 1), "tail_frac": round((end - dry) / end, 4)})

#!/usr/bin/env python3
"""Face items the kernels' wall walks evaluate (oracle statistics hook, FLOP build): per collide
substep each body has the faces the face cull keeps over the walls of its lane's broadphase
mask.  A lane walks the items of the bodies it holds -- four-lane kernel: torso, Aux k+1, leg
k; eight-lane: A_k torso + Aux, B_k Aux + leg; sixteen-lane: one body, the torso on four lanes
and each Aux on two -- so the per-lane walk runs as many iterations as a wave's busiest lane
and the cooperative walk (pob_mesh.h mesh_wave_walk, four items a round) about total / 4.
Prints, over a random-action rollout with autoresets, per layout: items per lane, the wave's
busiest lane, the wave total and the rounds of the cooperative walk (also their maximum over a
step, summed over its collide substeps: what a wave pays).

    python scripts/wall_walk_stats.py [env] [B] [steps]
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import orc  # noqa: E402
import pob_np as P  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "ant_heavenhell"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 60
NSUB = 5
e = orc.OracleEnv(name, count_flops=True)
L = e._L
L.orc_items_record.argtypes = [C.POINTER(C.c_int), C.c_int]
s = e.reset(P.split(P.prngkey(0), B + 1)[1:], first=True)
rng = np.random.default_rng(0)
buf = np.zeros((B, NSUB, 9), np.int32)
L.orc_items_record(buf.ctypes.data_as(C.POINTER(C.c_int)), NSUB)
L.orc_flops_set_mode(orc.FLOPS_EXECUTED)
LAYOUTS = {  # lanes per env: the bodies each lane walks
    "four-lane": [[0, 1, 2], [0, 3, 4], [0, 5, 6], [0, 7, 8]],
    "eight-lane": [[0, 1], [0, 3], [0, 5], [0, 7], [1, 2], [3, 4], [5, 6], [7, 8]],
    "sixteen-lane": [[0], [0], [0], [0], [1], [3], [5], [7], [1], [3], [5], [7], [2], [4], [6], [8]],
}
rec = []
try:
    for t in range(steps):
        buf[:] = 0
        s = e.step(s, rng.uniform(-1, 1, (B, 8)).astype(np.float32), flags=orc.F_EPISODE | orc.F_AUTORESET,
                   nthreads=1, inplace=True)
        rec.append(buf.copy())
finally:
    L.orc_items_record(None, 0)
    L.orc_flops_set_mode(orc.FLOPS_REF_PAIRS)
rec = np.stack(rec)  # (steps, B, NSUB, 9)
print(f"{name} B={B} steps={steps}")
for lay, lanes in LAYOUTS.items():
    per_lane = np.stack([rec[..., l].sum(-1) for l in lanes], -1)  # (steps, B, NSUB, lanes/env)
    epw = 64 // len(lanes)
    W = per_lane.reshape(steps, B // epw, epw, NSUB, len(lanes)).transpose(0, 1, 3, 2, 4).reshape(steps, B // epw, NSUB, 64)
    wmax, wtot = W.max(-1), W.sum(-1)
    rounds = np.maximum(np.ceil(wtot / 4), wmax * 0)  # round 4's cooperative walk: four items a round
    # round 5's walk (pob_mesh.h mesh_wave_walk): eight groups a round, a lane's first and
    # second items; "rank-major": eight groups from any lane's next items
    def _rounds(w, cap):
        w = w.copy()
        n = np.zeros(w.shape[:-1])
        while (w > 0).any():
            live = (w > 0).any(-1)
            take = np.zeros_like(w)
            left = np.full(w.shape[:-1], 8)
            for r in range(cap):
                has = (w - take) > 0
                cum = np.cumsum(has, -1)
                sel = has & (cum <= left[..., None])
                take += sel
                left = left - sel.sum(-1)
            w -= take
            n += live
        return n
    r8 = _rounds(W, 2)
    rrm = _rounds(W, 8)
    per_step_lane = wmax.sum(-1)  # per-lane walk iterations per step per wave
    per_step_coop = rounds.sum(-1)
    print(f"  {lay:13s} items/lane {per_lane.mean():.3f}; per wave-substep busiest lane {wmax.mean():.2f} "
          f"(max {wmax.max()}), total {wtot.mean():.2f} (p99 {np.percentile(wtot, 99):.0f}, max {wtot.max()}), "
          f"coop rounds {rounds.mean():.2f}; per step and wave: lane-walk iterations mean {per_step_lane.mean():.1f} "
          f"max {per_step_lane.max()}, coop rounds mean {per_step_coop.mean():.1f} max {per_step_coop.max()}")
    print(f"  {'':13s} 8 groups, 2 items per lane and round: rounds per step and wave mean {r8.sum(-1).mean():.2f} "
          f"max {r8.sum(-1).max():.0f}; rank-major: mean {rrm.sum(-1).mean():.2f} max {rrm.sum(-1).max():.0f}")

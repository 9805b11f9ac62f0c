#!/usr/bin/env python3
"""Face items the four-lane kernel's wall walk evaluates (oracle statistics hook, FLOP build):
per collide substep each lane walks the faces the face cull keeps of its three bodies over the
walls of its broadphase mask, one face per iteration, so a wave (16 envs x 4 lanes) runs as
many walk iterations as its busiest lane.  Prints, over a random-action rollout with
autoresets, the distribution of items per lane, the wave maximum (iterations of the per-lane
walk) and the wave total / 64 (iterations of a walk whose items were spread over the wave).

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
buf = np.zeros((B, NSUB, 4), np.int32)
L.orc_items_record(buf.ctypes.data_as(C.POINTER(C.c_int)), NSUB)
L.orc_flops_set_mode(orc.FLOPS_EXECUTED)
lane, wmax, wtot = [], [], []
try:
    for t in range(steps):
        buf[:] = 0
        s = e.step(s, rng.uniform(-1, 1, (B, 8)).astype(np.float32), flags=orc.F_EPISODE | orc.F_AUTORESET,
                   nthreads=1, inplace=True)
        lane.append(buf.copy().ravel())
        w = buf.reshape(B // 16, 16, NSUB, 4).transpose(0, 2, 1, 3).reshape(B // 16, NSUB, 64)
        wmax.append(w.max(-1).ravel())
        wtot.append(w.sum(-1).ravel())
finally:
    L.orc_items_record(None, 0)
    L.orc_flops_set_mode(orc.FLOPS_REF_PAIRS)
lane, wmax, wtot = np.concatenate(lane), np.concatenate(wmax), np.concatenate(wtot)
print(f"{name} B={B} steps={steps}: lanes x collide substeps = {lane.size}")
print("items per lane: mean %.3f, P(>0) %.3f, histogram %s" % (lane.mean(), (lane > 0).mean(),
      np.bincount(np.minimum(lane, 12), minlength=13).tolist()))
print("per wave-substep: busiest lane's items (per-lane walk iterations) mean %.2f p50 %d p90 %d max %d" % (
      wmax.mean(), np.median(wmax), np.percentile(wmax, 90), wmax.max()))
print("                  total items mean %.1f p90 %d max %d; spread over 64 lanes: ceil(total/64) mean %.2f" % (
      wtot.mean(), np.percentile(wtot, 90), wtot.max(), np.ceil(wtot / 64).mean()))

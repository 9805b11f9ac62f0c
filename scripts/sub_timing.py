"""Per-phase substep durations of the sixteen-lane kernel (timing experiment, not a test).

Needs a library built with -DPOB_EXP_TIMING -DPOB_EXP_TIMING_SUB (POB_LIB=...): stamps 5..12 of
each wave's row hold the shader-clock durations of the step's substep phases summed over its
ten substeps (sixteen lanes: accel + kinetic, joint projection, the position update, the face
walk alone, contact detection with the position responses, its broadphase + face cull, velocity
projection, velocity-level contacts).  argv: B (<= 16 384: the sixteen-lane kernel up to 4 096, the eight-lane one above), env name."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "po-brax_amd"))
from po_brax_amd import _lib, envs, jumpy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
NAME = sys.argv[2] if len(sys.argv) > 2 else "ant_heavenhell"
key = jumpy.random_prngkey(0)
act = torch.empty((B, 8), device="cuda")
env = envs.create(NAME, batch_size=B, episode_length=1000)
s = env.reset(jumpy.random_split(key, B + 1)[1:].contiguous())
for _ in range(20):
    jumpy.random_actions_(key, B, 0, act)
    s = env.step_(s, act)
torch.cuda.synchronize()
LPE = 16 if B <= (8192 if NAME in ("ant_heavenhell", "ant_tag") else 4096) else 8  # the default switch on 256 CUs
W = (B * LPE + 63) // 64
NTS = 16  # POB_TS_N of a POB_EXP_TIMING_SUB build
buf = np.zeros((W, NTS + 4), np.uint64)
f = _lib.lib.pob_debug_timing
f.argtypes = [C.c_void_p, C.c_int]
assert f(buf.ctypes.data, W) == 0
t = buf[:, 2:2 + NTS].astype(np.int64)
tot = t[:, NTS - 1] - t[:, 0]
print(f"{NAME} B={B} waves={W}: wave ticks p50 {np.median(tot):.0f} max {tot.max()}")
phys = t[:, 2] - t[:, 1]
print(f"physics (stamp 1->2) p50 {np.median(phys):.0f}")
names = (("accel+kinetic", "joint", "position update", "(of detect: the face walk)", "contact detect + position",
          "(of detect: broadphase + face cull)", "velocity projection", "velocity contacts") if LPE == 16 else
         ("accel+kinetic", "joint", "position update", "contact vel (ground+wall)", "contact detect",
          "contact position (ground+wall)", "velocity projection", "-"))
for i, n in zip(range(5, 13), names):
    print(f"{n:26s} p50 {np.median(t[:, i]):8.0f}  p90 {np.percentile(t[:, i], 90):8.0f}  max {t[:, i].max():8.0f}")

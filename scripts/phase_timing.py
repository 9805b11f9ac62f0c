"""Per-wave phase timings of the step kernel (timing experiment, not a test).

Needs a library built with -DPOB_EXP_TIMING (POB_LIB=...); prints the distribution of the
per-wave phase durations (s_memtime ticks) of the last of a few steps (argv: B, env name).
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "po-brax_amd"))
from po_brax_amd import _lib, envs, jumpy  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
NAME = sys.argv[2] if len(sys.argv) > 2 else "ant_heavenhell"
# "gym": time the gym path's masked reset kernel instead; "masked": a masked reset (RESET_OWN)
# of a few done envs (argv[4]: how many, default 8), as a gym step with done envs runs it
GYM = len(sys.argv) > 3 and sys.argv[3] in ("gym", "masked")
MASKED = len(sys.argv) > 3 and sys.argv[3] == "masked"
key = jumpy.random_prngkey(0)
act = torch.empty((B, 8), device="cuda")
if MASKED:
    env = envs.create(NAME, batch_size=B, episode_length=1000)
    s = env.reset(jumpy.random_split(key, B + 1)[1:].contiguous())
    nd = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    done = torch.zeros(B, device="cuda")
    done[torch.randperm(B, generator=torch.Generator().manual_seed(0))[:nd].cuda()] = 1.0
    for _ in range(3):
        s.aux["done"].copy_(done)
        env.unwrapped._reset_where_done(s, _lib.RESET_OWN)
elif GYM:
    gym = envs.create_gym_env(NAME, batch_size=B, seed=0, episode_length=1000)
    gym.reset()
    for _ in range(int(os.environ.get("PT_STEPS", "30"))):  # (the last step's reset waves are recorded)
        jumpy.random_actions_(key, B, 0, act)
        gym.step(act)
else:
    env = envs.create(NAME, batch_size=B, episode_length=1000)
    s = env.reset(jumpy.random_split(key, B + 1)[1:].contiguous())
    for _ in range(5):
        jumpy.random_actions_(key, B, 0, act)
        s = env.step_(s, act)
torch.cuda.synchronize()
LPE = 4 if GYM else (16 if B <= 4096 else (8 if B <= 16384 else 4))  # lanes per env (default switch points on 256 CUs)

W = (B * LPE + 63) // 64
NTS = 10  # POB_TS_N
buf = np.zeros((W, NTS + 4), np.uint64)
f = _lib.lib.pob_debug_timing
f.argtypes = [C.c_void_p, C.c_int]
assert f(buf.ctypes.data, W) == 0
hw, xcc, t = buf[:, 0].astype(np.int64), buf[:, 1].astype(np.int64), buf[:, 2:2 + NTS].astype(np.int64)
rt = buf[:, 2 + NTS:].astype(np.int64)  # device-wide 100 MHz clock: wave start, end
# waves that recorded (a masked reset's idle waves exit first; its rows carry stamp 8)
rec = (t[:, 8] != 0) if GYM else (t != 0).any(axis=1)
hw, xcc, t, rt = hw[rec], xcc[rec], t[rec], rt[rec]
print(f"recorded waves {rec.sum()} of {W}")
cols = [i for i in range(NTS) if (t[:, i] != 0).all()]  # the stamps this build records
t = t[:, cols]
d = np.diff(t, axis=1)
print(f"{NAME} B={B} waves={W} stamps={cols}")
for i in range(d.shape[1]):
    n = f"{cols[i]}->{cols[i + 1]}"
    print(f"{n:6s} ticks p0 {np.percentile(d[:, i], 0):9.0f} p50 {np.percentile(d[:, i], 50):9.0f} "
          f"p90 {np.percentile(d[:, i], 90):9.0f} max {d[:, i].max():9.0f}")
print("stamp - stamp0 p50: " + " ".join(f"{c}:{np.median(t[:, i] - t[:, 0]):.0f}" for i, c in enumerate(cols)))
tot = t[:, -1] - t[:, 0]
print(f"total p0 {tot.min()} p50 {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} max {tot.max()}")
# device-wide clock (10 ns ticks): when waves start and end relative to the first start
r0 = rt[:, 0] - rt[:, 0].min()
r1 = rt[:, 1] - rt[:, 0].min()
pct = lambda a: " ".join(f"p{q} {np.percentile(a, q) / 100:.1f}" for q in (0, 10, 50, 90, 100))
print(f"wave start us: {pct(r0)}")
print(f"wave end   us: {pct(r1)}")
print(f"wave life  us: {pct(r1 - r0)}")
if os.environ.get("PT_DUMP"):  # raw per-wave rows for offline analysis (hw id, xcc, stamps, clock)
    np.savez(os.environ["PT_DUMP"], hw=hw, xcc=xcc, t=t, rt=rt, cols=np.array(cols))

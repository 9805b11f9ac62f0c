"""Debug helper: find the envs whose GPU step differs from the oracle at HH B=65536 (the
bench-size parity case) and save their pre-step state + action for CPU analysis."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "po-brax_amd"))
import orc  # noqa: E402
from test_gpu_parity import _keys, _state_np  # noqa: E402
from test_gpu_headline_parity import _actions  # noqa: E402
from po_brax_amd import envs  # noqa: E402

name, B = (sys.argv[1] if len(sys.argv) > 1 else "ant_heavenhell"), int(sys.argv[2]) if len(sys.argv) > 2 else 65536
env = envs.create(name, batch_size=B, episode_length=3)
keys = _keys(B, 0)
s = env.reset(torch.from_numpy(keys).cuda())
o = orc.OracleEnv(name)
bad_all = []
out = {}
for t, act in enumerate(_actions(1, B, 4)):
    pre = _state_np(s)
    so = o.step(pre, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=3, nthreads=16)
    s = env.step_(s, torch.from_numpy(act).cuda())
    g = _state_np(s)
    bad = np.zeros(B, bool)
    for k in ("pos", "rot", "vel", "ang", "obs"):
        bad |= (g[k] != so[k]).reshape(B, -1).any(1)
    idx = np.nonzero(bad)[0]
    print(f"step {t}: {len(idx)} envs differ: {idx[:20]}")
    if len(idx):
        for k in ("pos", "rot", "vel", "ang", "obs", "steps", "done", "rng", "m0", "m1", "m2", "truncation", "reward"):
            out[f"t{t}_pre_{k}"] = pre[k][idx]
            out[f"t{t}_gpu_{k}"] = g[k][idx]
            out[f"t{t}_orc_{k}"] = so[k][idx]
        out[f"t{t}_act"] = act[idx]
        out[f"t{t}_idx"] = idx
        break
os.makedirs(os.path.join(ROOT, "gpurun_out", "dbg"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "dbg", f"mismatch_{name}_{B}.npz"), **out)

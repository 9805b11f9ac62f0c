"""Time pob_reset (full) and pob_reset_where_done (masked) per kind at a batch size."""
import json, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "po-brax_amd"))
import torch
from po_brax_amd import envs, jumpy, _lib
B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
out = {}
for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
    env = envs.create(name, batch_size=B, episode_length=1000)
    keys = jumpy.random_split(jumpy.random_prngkey(0), B + 1)[1:].contiguous()
    s = env.reset(keys)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ts = []
    for r in range(5):
        ev[0].record(); env.reset(keys); ev[1].record(); torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]))
    # masked: 1 % and 100 % of the envs done (RESET_OWN, keys = info rng)
    u = env.unwrapped
    res = {"full_ms": min(ts)}
    for frac in (0.01, 1.0):
        done = (torch.rand(B, device="cuda") < frac).float()
        tm = []
        for r in range(5):
            s.aux["done"].copy_(done)
            ev[0].record(); u._reset_where_done(s, _lib.RESET_OWN); ev[1].record(); torch.cuda.synchronize()
            tm.append(ev[0].elapsed_time(ev[1]))
        res[f"masked_{frac}_ms"] = min(tm)
    out[name] = res
print(json.dumps({"B": B, **out}))

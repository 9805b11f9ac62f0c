import sys, os
sys.path[:0] = ["po-brax_amd", "oracle", "tests"]
import numpy as np, torch
import orc, pob_np as P
from po_brax_amd import envs
B = 10923
keys = P.split(P.prngkey(0), B + 1)[1:]
e = envs.create("ant_heavenhell", batch_size=B, qp_dtype=torch.float16)
s = e.reset(torch.from_numpy(keys).cuda())
o = orc.OracleEnv("ant_heavenhell").reset(keys, first=True, nthreads=16)
for f in ("pos", "rot", "vel", "ang"):
    g = getattr(s.qp, f).cpu().numpy().view(np.uint16)
    r32 = o[f]
    r = r32.astype(np.float16).view(np.uint16)
    bad = np.argwhere(g != r)
    print(f, len(bad))
    for idx in bad[:12]:
        idx = tuple(idx)
        print(idx, repr(float(r32[idx])), hex(r32[idx:idx[0]+1].view(np.uint32)[0] if False else np.float32(r32[idx]).view(np.uint32)), g[idx], r[idx])

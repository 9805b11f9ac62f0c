"""Debug helper: the out-of-range-input parity case (tests/test_gpu_headline_parity.py
test_out_of_range_inputs_take_exact_fallbacks) on one kernel / guard policy: print every env
and element where the GPU step differs from the oracle (NaN-aware)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("tests", "oracle", "po-brax_amd"):
    sys.path.insert(0, os.path.join(ROOT, p))
lanes, B, gacc = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
if gacc != "none":
    os.environ["POB_HEX_GACC" if lanes == 16 else "POB_OCT_GACC"] = gacc
if lanes <= 8:
    os.environ["POB_HEXA_MAX_B"] = "0"
if lanes == 4:
    os.environ["POB_OCTET_MAX_B"] = "0"
import orc  # noqa: E402
from test_gpu_parity import _keys, _state_np  # noqa: E402
from test_gpu_headline_parity import _actions  # noqa: E402
from po_brax_amd import envs  # noqa: E402

for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
    env = envs.create(name, batch_size=B, episode_length=1000)
    s = env.reset(torch.from_numpy(_keys(B, 40 + lanes)).cuda())
    with torch.no_grad():
        s.qp.vel[1, 0, 0] = 1e25
        s.qp.rot[2, 1] = 0.0
        s.qp.ang[3, 2, 1] = 1e30
    o = orc.OracleEnv(name)
    for t, act in enumerate(_actions(lanes + 2, B, 2)):
        pre = _state_np(s)
        so = o.step(pre, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=1000, nthreads=16)
        s = env.step(s, torch.from_numpy(act).cuda())
        g = _state_np(s)
        for k in ("pos", "rot", "vel", "ang", "obs"):
            a, b = g[k].reshape(B, -1), so[k].reshape(B, -1)
            diff = ~((a == b) | (np.isnan(a) & np.isnan(b)))
            for e in np.nonzero(diff.any(1))[0][:6]:
                cols = np.nonzero(diff[e])[0]
                print(f"{name} step {t} {k} env {e}: {len(cols)} elements differ, first cols {cols[:8]}: "
                      f"gpu {a[e, cols[:4]]} oracle {b[e, cols[:4]]}")

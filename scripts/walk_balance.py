#!/usr/bin/env python3
"""Walk-round statistics behind DESIGN.md §8 (round 6): from the oracle's per-body face items
(statistics hook, as scripts/wall_walk_stats.py) over a random-action rollout, the sixteen-lane
kernel's walk rounds per step -- per wave (4 envs, 8 items a round) against cooperation over a
block of 2 or 4 waves, two interleaved rounds per lane ("double rounds" at a relative cost D),
and an env-to-wave permutation balanced by the previous step's item counts.  What matters is
the slowest wave per step (the kernel waits for it).

    python scripts/walk_balance.py [env] [B] [steps]     (e.g. ant_heavenhell 4096 20)
"""
import ctypes as C, os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import orc, pob_np as P
name = sys.argv[1] if len(sys.argv) > 1 else "ant_heavenhell"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
NSUB = 5
e = orc.OracleEnv(name, count_flops=True)
L = e._L
L.orc_items_record.argtypes = [C.POINTER(C.c_int), C.c_int]
s = e.reset(P.split(P.prngkey(0), B + 1)[1:], first=True)
rng = np.random.default_rng(0)
buf = np.zeros((B, NSUB, 9), np.int32)
L.orc_items_record(buf.ctypes.data_as(C.POINTER(C.c_int)), NSUB)
L.orc_flops_set_mode(orc.FLOPS_EXECUTED)
rec = []
try:
    for t in range(steps):
        buf[:] = 0
        s = e.step(s, rng.uniform(-1, 1, (B, 8)).astype(np.float32), flags=orc.F_EPISODE | orc.F_AUTORESET, nthreads=8, inplace=True)
        rec.append(buf.copy())
finally:
    L.orc_items_record(None, 0); L.orc_flops_set_mode(orc.FLOPS_REF_PAIRS)
rec = np.stack(rec)  # (steps, B, NSUB, 9) items per body
items = rec.sum(-1)  # per env per substep
def rounds(env_items, epg, groups):
    # env_items (steps, B, NSUB); envs per cooperating unit epg, items per round `groups`
    S, Bn, N = env_items.shape
    u = env_items.reshape(S, Bn // epg, epg, N).sum(2)  # (steps, units, NSUB)
    r = np.ceil(u / groups).sum(-1)  # rounds per step per unit
    return r
for label, epg, groups in (("wave of 4 envs, 8 groups (hex now)", 4, 8),
                           ("block of 4 waves = 16 envs, 32 groups", 16, 32),
                           ("block of 2 waves = 8 envs, 16 groups", 8, 16)):
    r = rounds(items, epg, groups)
    print(f"{label:42s} rounds/step: mean {r.mean():.2f}  max over units per step (mean over steps) {r.max(1).mean():.2f}  max {r.max():.0f}")
# double rounds: a substep with k items costs ceil(k/8) rounds now; with two chains per lane,
# ceil(k/16) double rounds of cost D (relative to a single round) + a single round if the rest <= 8
def cost(u, D):
    full = np.floor(u / 16); rest = u - 16 * full
    return full * D + np.where(rest > 8, D, np.where(rest > 0, 1.0, 0.0))
u = items.reshape(items.shape[0], -1, 4, items.shape[2]).sum(2)  # per wave (4 envs)
for D in (1.3, 1.5, 1.7):
    c = cost(u, D).sum(-1)
    print(f"double-round cost {D}: slowest wave per step mean {c.max(1).mean():.2f} (single: {np.ceil(u/8).sum(-1).max(1).mean():.2f}), mean {c.mean():.2f}")
# env -> wave permutation from the previous step's per-env item totals: heavy envs dealt
# round-robin over the waves (sorted descending, snake order), light ones fill
S, Bn, NS = items.shape
W = Bn // 4
def rounds_for(perm, it):
    u = it[perm].reshape(W, 4, NS).sum(1)
    return np.ceil(u / 8).sum(-1)
base, bal = [], []
for t in range(1, S):
    prev = items[t - 1].sum(-1)
    order = np.argsort(-prev, kind="stable")
    # snake deal: rank r -> wave (r mod W) going forward, then backward
    waves = np.empty(Bn, int)
    r = np.arange(Bn); blk = r // W; pos = r % W
    waves[order] = np.where(blk % 2 == 0, pos, W - 1 - pos)
    perm = np.argsort(waves, kind="stable")  # envs grouped by wave
    bal.append(rounds_for(perm, items[t]).max())
    base.append(rounds_for(np.arange(Bn), items[t]).max())
print(f"slowest wave rounds per step: identity {np.mean(base):.2f}, balanced by previous step {np.mean(bal):.2f}")

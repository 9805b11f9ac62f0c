"""CPU, world_size 2 (gloo): index sharding of envs reproduces the single-process batch.

Each rank takes its slice of split(key, B+1)[1:] (po_brax_amd.sharding.shard_range), runs
the CPU oracle's reset + steps on it with its slice of the global action batch, and the
all-gathered shards must equal the unsharded run bit for bit -- the property the GPU
bench relies on.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

B, T = 48, 3


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(rank, world, port, name, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "po-brax_amd"), os.path.join(root, "oracle")]
    import orc
    import pob_np as P
    from po_brax_amd.sharding import shard_range
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(B, world, rank)
    key = P.prngkey(0)
    keys = P.split(key, B + 1)[1 + lo:1 + hi]
    e = orc.OracleEnv(name)
    s = e.reset(keys, first=True)
    for t in range(T):
        key, k = P.split(key)
        act = P.uniform(k, (B, 8), -1, 1)[lo:hi]
        s = e.step(s, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=2)
    obs = torch.from_numpy(s["obs"])
    parts = [torch.empty_like(obs) for _ in range(world)]
    dist.all_gather(parts, obs)
    if rank == 0:
        q.put(torch.cat(parts).numpy())
    dist.destroy_process_group()


def _single(name):
    import orc
    import pob_np as P
    key = P.prngkey(0)
    e = orc.OracleEnv(name)
    s = e.reset(P.split(key, B + 1)[1:], first=True)
    for t in range(T):
        key, k = P.split(key)
        s = e.step(s, P.uniform(k, (B, 8), -1, 1), flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=2)
    return s["obs"]


def test_sharded_equals_single_world2():
    ctx = mp.get_context("spawn")
    for name in ("ant_heavenhell", "ant_tag"):
        q = ctx.Queue()
        port = _free_port()
        procs = [ctx.Process(target=_run, args=(r, 2, port, name, q)) for r in range(2)]
        for p in procs:
            p.start()
        got = q.get(timeout=120)
        for p in procs:
            p.join(timeout=120)
            assert p.exitcode == 0
        np.testing.assert_array_equal(got, _single(name))


def test_shard_range_covers():
    from po_brax_amd.sharding import shard_range
    for total in (1, 7, 64, 65536, 262144):
        for world in (1, 2, 3, 8):
            rs = [shard_range(total, world, r) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))

"""Multi-rank check of the sharded product path with the HIP kernels (run under torchrun).

Each rank runs its shard of a global batch -- brax chain (shard_keys + sharded actions) and
gym chain (create_gym_env(shard=...): global gym-key rows + any-done all-reduce) -- then the
observation shards are all-gathered and rank 0 compares them with the same global batch
stepped by one process on its own device.  Exit code 0 = bit-identical.

    torchrun --nproc-per-node 2 scripts/multirank_check.py --backend gloo   # 2 ranks, 1 GPU
    torchrun --nproc-per-node 8 scripts/multirank_check.py                  # RCCL, 8 GPUs
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "po-brax_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="nccl")
    ap.add_argument("--total", type=int, default=1001)
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--env", default="ant_tag")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    ndev = torch.cuda.device_count()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % ndev)
    torch.cuda.set_device(dev)
    kw = dict(device_id=dev) if args.backend == "nccl" else {}
    dist.init_process_group(args.backend, rank=rank, world_size=world, **kw)
    from po_brax_amd import envs, jumpy
    from po_brax_amd.sharding import ObsGatherer, Shard, gather_obs_ragged, shard_keys
    total, T, name = args.total, args.steps, args.env
    sh = Shard.current(total)
    key = jumpy.random_prngkey(0, device=dev)

    def actions(B, lo):
        ak = jumpy.random_prngkey(7, device=dev)
        out = []
        for _ in range(T):
            a = torch.empty((B, 8), device=dev)
            jumpy.random_actions_(ak, total, lo, a)
            out.append(a)
        return out

    # brax chain, sharded
    env = envs.create(name, batch_size=sh.size, episode_length=5, device=dev)
    s = env.reset(shard_keys(key, total, world, rank))
    for a in actions(sh.size, sh.lo):
        env.step_(s, a)
    brax_obs = gather_obs_ragged(s.obs, total)
    # gym chain, sharded (any-done all-reduce every step)
    g = envs.create_gym_env(name, batch_size=total, seed=3, episode_length=5, device=dev, shard=sh)
    g.reset()
    for a in actions(sh.size, sh.lo):
        g.step(a)
    gym_obs = gather_obs_ragged(g._state.obs, total)
    gym_key = g._key.clone()
    # the overlapped obs gather (ObsGatherer: staging copy on the compute stream, all-gather on
    # a side stream, read one step later): every step's gathered batch
    e2 = envs.create(name, batch_size=sh.size, episode_length=5, device=dev)
    s2 = e2.reset(shard_keys(key, total, world, rank))
    gat = ObsGatherer(total, s2.obs.shape[-1], device=dev if args.backend == "nccl" else "cpu")
    per_step, prev = [], None
    for a in actions(sh.size, sh.lo):
        e2.step_(s2, a)
        p = gat.submit(s2.obs if gat.cuda else s2.obs.cpu())
        if prev is not None:
            per_step.append(gat.result(prev).to(dev, copy=True))
        prev = p
    per_step.append(gat.result(prev).to(dev, copy=True))
    torch.cuda.synchronize(dev)
    ok = True
    if rank == 0:
        e1 = envs.create(name, batch_size=total, episode_length=5, device=dev)
        s1 = e1.reset(shard_keys(key, total, 1, 0))
        ref_steps = []
        for a in actions(total, 0):
            e1.step_(s1, a)
            ref_steps.append(s1.obs.clone())
        g1 = envs.create_gym_env(name, batch_size=total, seed=3, episode_length=5, device=dev)
        g1.reset()
        for a in actions(total, 0):
            g1.step(a)
        gat_ok = len(per_step) == len(ref_steps) and all(torch.equal(x, y) for x, y in zip(per_step, ref_steps))
        ok = (torch.equal(brax_obs, s1.obs) and torch.equal(gym_obs, g1._state.obs) and torch.equal(gym_key, g1._key)
              and gat_ok)
        print(f"multirank {name} world={world} backend={args.backend}: brax {torch.equal(brax_obs, s1.obs)} "
              f"gym {torch.equal(gym_obs, g1._state.obs)} key {torch.equal(gym_key, g1._key)} gather {gat_ok}",
              flush=True)
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
    dist.all_reduce(flag)
    dist.destroy_process_group()
    return int(flag.item())


if __name__ == "__main__":
    sys.exit(main())

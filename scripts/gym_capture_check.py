"""Capture of the sharded gym step's RCCL any-done all-reduce in a hipGraph (run under
torch.distributed.run; one rank on the one-GPU box, or the node's ranks).

A sharded gym vector env (``create_gym_env(shard=Shard.current(total))``) steps eagerly and,
from the same reset, through ``rollout.GymGraphRollout`` (T steps captured once, replayed
twice); rank 0 prints whether obs, reward, done and the gym key agree bit for bit.  Exit
code 0 = equal on every rank.

    torchrun --nproc-per-node 1 scripts/gym_capture_check.py --backend nccl
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
    ap.add_argument("--total", type=int, default=4097)
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--env", default="ant_heavenhell")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist.init_process_group(args.backend, rank=rank, world_size=world,
                            **(dict(device_id=dev) if args.backend == "nccl" else {}))
    from po_brax_amd import envs, jumpy
    from po_brax_amd.rollout import GymGraphRollout
    from po_brax_amd.sharding import Shard
    total, T = args.total, args.steps
    sh = Shard.current(total)
    acts = torch.empty((T, sh.size, 8), device=dev)
    ak = jumpy.random_prngkey(5, device=dev)
    for t in range(T):
        jumpy.random_actions_(ak, total, sh.lo, acts[t])

    def make():  # episode_length 3: every env ends an episode inside the T steps
        g = envs.create_gym_env(args.env, batch_size=total, seed=3, episode_length=3, device=dev, shard=sh)
        g.reset()
        return g

    ga = make()
    for _ in range(2):
        for t in range(T):
            ga.step(acts[t])
    gb = make()
    roll = GymGraphRollout(gb, acts)
    roll.replay()
    roll.replay()
    torch.cuda.synchronize(dev)
    a, b = ga._state, gb._state
    same = {"obs": torch.equal(a.obs, b.obs), "reward": torch.equal(a.reward, b.reward),
            "done": torch.equal(a.done, b.done), "key": torch.equal(ga._key, gb._key)}
    ok = all(same.values())
    print(f"gym capture {args.env} world={world} rank={rank} backend={args.backend}: "
          + " ".join(f"{k} {v}" for k, v in same.items()), flush=True)
    flag = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
    dist.all_reduce(flag)
    dist.destroy_process_group()
    return int(flag.item())


if __name__ == "__main__":
    sys.exit(main())

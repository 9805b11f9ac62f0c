#!/usr/bin/env python3
"""A whole episode of the headline workload, timed in windows (verdict r5 item 5).

bench.py times 20-30 steps right after reset; HH ants spawn against the T-maze's bottom wall with
legs through it, so those steps are the wall-heaviest phase of a 1 000-step episode.  This runs
the bench's exact workload -- ``create(env, batch_size=B, episode_length=1000)``, reset keys
``split(PRNGKey(0), B + 1)[1:]``, the bench's threefry action stream -- for a whole episode
(+ the autoreset step), replaying hipGraphs of ``--chunk`` captured steps back to back (the
actions of a chunk are generated on the device before its replay, outside the timed spans), and
reports per window: ms/step (HIP events around the replay), the envs done at the window's last
step, and the algorithmic FLOPs per env-step of the window (the instrumented CPU restatement
stepping the first ``--flop-envs`` envs through the same keys and actions, bench.py's basis).

    python scripts/episode_bench.py [--env ant_heavenhell] [--B 65536] [--steps 1000] [--chunk 100]

Prints one JSON object (windows + summary).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "po-brax_amd"))
VALU_PEAK_TF = 157.3


def flops_per_step(name: str, total: int, n: int, steps: int, episode_length: int, budget_s: float):
    """the executed FLOPs per env-step of each step (first n envs; oracle, test infrastructure)"""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import orc
    keys = orc.split(np.array([0, 0], np.uint32), total + 1)
    e = orc.OracleEnv(name, count_flops=True)
    s = e.reset(np.ascontiguousarray(keys[1:1 + n]), first=True)
    act_key = keys[0].copy()
    e._L.orc_flops_set_mode(orc.FLOPS_EXECUTED)
    e._L.orc_flops_read_and_reset()
    per, t0 = [], time.time()
    try:
        for t in range(steps):
            kk = orc.split(act_key, 2)
            act_key, k = kk[0].copy(), kk[1].copy()
            a = np.ascontiguousarray(orc.uniform(k, total * 8).reshape(total, 8)[:n])
            e.step(s, a, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=episode_length, nthreads=1,
                   inplace=True)
            per.append(e._L.orc_flops_read_and_reset() / float(n))
            if time.time() - t0 > budget_s:
                break
    finally:
        e._L.orc_flops_set_mode(orc.FLOPS_REF_PAIRS)
    return per


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="ant_heavenhell")
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=1001, help="1 000 episode steps + the autoreset step")
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--episode-length", type=int, default=1000)
    ap.add_argument("--flop-envs", type=int, default=128)
    ap.add_argument("--flop-budget-s", type=float, default=120.0)
    args = ap.parse_args()
    from po_brax_amd import envs, jumpy
    from po_brax_amd.rollout import GraphRollout
    dev = torch.device("cuda:0")
    B, C = args.B, args.chunk
    env = envs.create(args.env, batch_size=B, episode_length=args.episode_length, device=dev)
    key = jumpy.random_prngkey(0, device=dev)
    state = env.reset(jumpy.random_split(key, B + 1)[1:].contiguous())
    act_key = jumpy.random_split(key, B + 1)[0].contiguous()
    acts = torch.empty((C, B, 8), dtype=torch.float32, device=dev)
    # one eager step on a throwaway copy is not needed: capture with warmup=False (the env has
    # been reset, nothing is lazily initialised); the graph is captured once and replayed
    roll = GraphRollout(env, state, acts)
    windows = []
    done_now = state.aux["done"]
    steps_left = args.steps
    t_all = 0.0
    while steps_left > 0:
        n = min(C, steps_left)
        for t in range(C):  # the chunk's actions (a short last chunk uses the first n)
            jumpy.random_actions_(act_key, B, 0, acts[t])
        if n < C:  # a shorter last window: eager steps (the graph holds C)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for t in range(n):
                env.step_(roll.state, acts[t])
            e1.record()
        else:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            roll.replay()
            e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        t_all += ms
        first = args.steps - steps_left
        windows.append({"steps": [first, first + n], "ms_per_step": round(ms / n, 5),
                        "env_steps_per_s": round(B * n / (ms * 1e-3), 1),
                        "graph": n == C, "done_at_last_step": int((done_now != 0).sum())})
        steps_left -= n
    # the bench's 20-step line for comparison: the first window's first steps are in window 0
    per = flops_per_step(args.env, B, args.flop_envs, args.steps, args.episode_length, args.flop_budget_s)
    for w in windows:
        a, b = w["steps"]
        seg = per[a:b]
        if seg:
            f = float(np.mean(seg))
            w["flops_per_env_step"] = round(f, 1)
            w["flop_steps_counted"] = len(seg)
            w["tflops"] = round(f * w["env_steps_per_s"] / 1e12, 3)
            w["valu_frac"] = round(w["tflops"] / VALU_PEAK_TF, 4)
    ms_all = t_all / args.steps
    out = {"env": args.env, "B": B, "episode_length": args.episode_length, "steps": args.steps, "chunk": C,
           "ms_per_step_episode": round(ms_all, 5), "env_steps_per_s_episode": round(B / (ms_all * 1e-3), 1),
           "flop_envs": args.flop_envs, "flop_steps_counted": len(per),
           "flops_per_env_step_episode": round(float(np.mean(per)), 1) if per else None,
           "windows": windows,
           "note": "HIP events around each window's graph replay (actions generated on the device before it); "
                   "FLOPs: the instrumented CPU restatement on the first flop_envs envs, same keys and actions"}
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main())

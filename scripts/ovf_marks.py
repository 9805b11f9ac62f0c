"""How many waves of the four-lane kernel's fast launch overflow their contact pool and are
re-stepped by the fix-up launch (pob_state.ovf_mark, one byte per 16-env wave at its first
env), per step of the bench's workload (reset keys split(PRNGKey(0), B + 1)[1:], the bench's
threefry action stream).  Diagnostic, not a test.

    python scripts/ovf_marks.py [--env ant_heavenhell] [--B 65536] [--steps 60]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "po-brax_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="ant_heavenhell")
    ap.add_argument("--B", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=60)
    args = ap.parse_args()
    from po_brax_amd import envs, jumpy
    dev = torch.device("cuda:0")
    B = args.B
    env = envs.create(args.env, batch_size=B, episode_length=1000, device=dev)
    key = jumpy.random_prngkey(0, device=dev)
    s = env.reset(jumpy.random_split(key, B + 1)[1:].contiguous())
    act_key = jumpy.random_split(key, B + 1)[0].contiguous()
    act = torch.empty((B, 8), device=dev)
    per = []
    for t in range(args.steps):
        jumpy.random_actions_(act_key, B, 0, act)
        s = env.step_(s, act)
        m = s.aux["ovf_mark"][::16]
        per.append(int((m != 0).sum()))
    print(json.dumps({"env": args.env, "B": B, "waves": (B + 15) // 16, "marked_per_step": per}))


if __name__ == "__main__":
    main()

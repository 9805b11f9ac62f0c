#!/usr/bin/env python3
"""bench.py -- env-steps/s of the fused MI355X rollout step (BASELINE.json metric).

Workload (BASELINE.json configs / SURVEY.md §8(d)): AntHeavenHell, batch 65 536 per GPU,
brax chain ``create('ant_heavenhell', batch_size=B)`` = AutoReset(Vmap(Episode(ActionRepeat
(env)))) with episode_length 1000, i.e. ONE fused HIP kernel per env-step (PBD physics,
POMDP logic, obs, episode counter, autoreset).  Synthetic inputs as the survey prescribes:
``key = PRNGKey(0)``, reset keys ``split(key, B_total + 1)[1:]`` (sharded by index), per step
``key, k = split(key)``, ``action = uniform(k, (B_total, 8), -1, 1)`` -- all generated on the
device by the threefry kernels BEFORE the timed region (inputs resident in HBM).

Multi-GPU: one process per GPU (torchrun), each rank owns B envs (weak scaling, no
collective on the data path); barrier + synchronize bracket the K timed steps and the
max over ranks is reported.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "po-brax_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# algorithmic HBM bytes per env-step of k_step, fp32, in-place state:
#   reads : qp of the 9 dynamic bodies (117 f) + task bodies' xy + action (8) + prev done,
#           steps, truncation, 3 metrics, rng (2)
#   writes: qp (117 f) + task bodies + obs (D) + reward, done, steps, truncation,
#           3 metrics, rng (2)
_TASK_READ = {"ant_heavenhell": 6, "ant_gather": 48, "ant_tag": 2, "ant": 0}
_TASK_WRITE = {"ant_heavenhell": 0, "ant_gather": 48, "ant_tag": 3, "ant": 0}
_OBS = {"ant_heavenhell": 114, "ant_gather": 211, "ant_tag": 103, "ant": 87}
MIXED = ("ant_heavenhell", "ant_gather", "ant_tag")  # --env mixed (BASELINE.json config 5)


def bytes_per_env_step(name: str, qp_bytes: int = 4) -> int:
    """qp elements (dynamic bodies + task bodies' positions) at qp_bytes, the rest float32."""
    qp = (117 + _TASK_READ[name]) + (117 + _TASK_WRITE[name])
    rest = (8 + 1 + 1 + 1 + 3 + 2) + (_OBS[name] + 1 + 1 + 1 + 1 + 3 + 2)
    return qp_bytes * qp + 4 * rest


def mixed_sizes(B: int):
    base, rem = divmod(B, len(MIXED))
    return [base + (1 if i < rem else 0) for i in range(len(MIXED))]


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--env", default="ant_heavenhell", choices=sorted(_OBS) + ["mixed"],
                    help="'mixed' = HH + GA + TAG batches (B split 3 ways) in one launch per step")
    ap.add_argument("--qp-dtype", default="f32", choices=["f32", "f16"],
                    help="qp storage (f16 = binary16 qp, float32 arithmetic)")
    ap.add_argument("--batch", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--episode-length", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gather-obs", action="store_true",
                    help="also time an RCCL all-gather of the final obs batch (N>1)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from po_brax_amd import envs, jumpy
    from po_brax_amd.sharding import shard_keys, shard_range

    B = args.batch
    total = B * world
    lo, hi = shard_range(total, world, rank)
    qp_dtype = torch.float16 if args.qp_dtype == "f16" else torch.float32
    key = jumpy.random_prngkey(0, device=dev)
    if args.env == "mixed":
        # rank r owns global envs [lo, hi); within it the kinds follow one another
        env = envs.create_mixed(MIXED, episode_length=args.episode_length, device=dev, qp_dtype=qp_dtype)
        sizes = mixed_sizes(B)
        keys = shard_keys(key, total, world, rank)
        env.batch_sizes = sizes
        state = [e.reset(keys[o:o + b].contiguous()) for e, o, b in zip(env.envs, env.offsets(), sizes)]
    else:
        env = envs.create(args.env, batch_size=B, episode_length=args.episode_length, device=dev,
                          qp_dtype=qp_dtype)
        state = env.reset(shard_keys(key, total, world, rank))
    act_key = jumpy.random_split(key, total + 1)[0].contiguous()  # VmapGymWrapper: key <- keys[0]

    T = args.warmup + args.steps
    pre = T * B * 8 * 4 <= (6 << 30)
    if pre:
        acts = torch.empty((T, B, 8), dtype=torch.float32, device=dev)
        for t in range(T):
            jumpy.random_actions_(act_key, total, lo, acts[t])
    else:
        acts = torch.empty((1, B, 8), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()

    def act_at(t):
        if pre:
            return acts[t]
        jumpy.random_actions_(act_key, total, lo, acts[0])
        return acts[0]

    for t in range(args.warmup):
        env.step_(state, act_at(t))
    torch.cuda.synchronize()

    # timed region: K steps, per-step events bracket the one fused kernel of each step
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    for k in range(args.steps):
        env.step_(state, act_at(args.warmup + k))
        evs[k + 1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    gpu_ms = evs[0].elapsed_time(evs[-1])
    per = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    elapsed = torch.tensor([wall, gpu_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    wall, gpu_ms = float(elapsed[0]), float(elapsed[1])
    ms_per_step = 1e3 * wall / args.steps
    value = total * args.steps / wall
    obs_last = torch.cat([s.obs.reshape(-1) for s in state]) if args.env == "mixed" else state.obs
    finite = bool(torch.isfinite(obs_last).all())

    gather_ms = None
    if args.gather_obs and world > 1:
        from po_brax_amd.sharding import gather_obs
        gather_obs(obs_last)
        torch.cuda.synchronize()
        dist.barrier()
        g0 = time.perf_counter()
        for _ in range(5):
            gather_obs(obs_last)
        torch.cuda.synchronize()
        gather_ms = 1e3 * (time.perf_counter() - g0) / 5

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    # roofline of the dominant kernel (k_step): algorithmic bytes and FLOPs per launch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    kern_ms = sum(per) / len(per)
    qb = 2 if args.qp_dtype == "f16" else 4
    kinds = list(zip(MIXED, mixed_sizes(B))) if args.env == "mixed" else [(args.env, B)]
    bpe = sum(bytes_per_env_step(n, qb) * b for n, b in kinds) / B
    try:
        import orc  # test-infrastructure oracle: FLOP count of the restated algorithm only
        fpe = sum(orc.flops_per_env_step(n, B=64, steps=10) * b for n, b in kinds) / B
    except Exception as ex:  # pragma: no cover
        print(f"flop count unavailable: {ex}", file=sys.stderr)
        fpe = float("nan")
    hbm_gbs = bpe * B / (kern_ms * 1e-3) / 1e9
    tflops = fpe * B / (kern_ms * 1e-3) / 1e12
    roofline = {
        "bound": "valu", "achieved": round(tflops, 3), "peak": 157.3, "unit": "TFLOP/s",
        "frac": round(tflops / 157.3, 5), "traffic": None,
        "kernel": "k_step_mixed" if args.env == "mixed" else f"k_step_quad<{args.env}>",
        "kernel_ms": round(kern_ms, 4),
        "flops_per_env_step": round(fpe, 1), "bytes_per_env_step": round(bpe, 1),
        "hbm": {"achieved": round(hbm_gbs, 2), "peak": 8000.0, "unit": "GB/s",
                "frac": round(hbm_gbs / 8000.0, 6)},
    }

    tr = committed_traffic(args.env, B, args.qp_dtype)
    if tr is not None:
        roofline["traffic"] = tr["traffic_bytes"]
        roofline["traffic_source"] = (f"profiles/{tr['source']}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + "
                                      f"WRITE_SIZE per launch of the same kernel and config")

    cpu = None
    if not args.no_cpu_baseline and world == 1:
        cpu = cpu_baseline("ant_heavenhell" if args.env == "mixed" else args.env, args.cpu_seconds)

    line = {
        "metric": f"env-steps/sec {args.env} batch {B}/GPU",
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.env} B={B}/GPU, create(batch_size=B, episode_length="
                               f"{args.episode_length}) autoreset chain, PBD 10 substeps, random "
                               "uniform(-1,1) actions (threefry)"
                               + (f", kinds {dict(kinds)} in one launch" if args.env == "mixed" else ""),
                   "env": args.env, "global_batch": total, "episode_length": args.episode_length,
                   "qp_storage": args.qp_dtype, "parallelism": f"env-shard x{world}"},
        "gpu_event_ms_per_step": round(gpu_ms / args.steps, 4),
        "roofline": roofline, "cpu_baseline": cpu, "obs_finite": finite,
    }
    if gather_ms is not None:
        line["obs_allgather_ms"] = round(gather_ms, 3)
    print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def committed_traffic(env: str, B: int, qp: str):
    """HBM bytes per launch from the newest committed PMC profile of this exact config
    (profiles/*_traffic.json, written by profiles/summarize.py); None if there is none."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            t = json.load(open(p))
        except (OSError, ValueError):
            continue
        if t.get("env") == env and t.get("batch") == B and t.get("qp_storage", "f32") == qp and \
                "k_step" in (t.get("kernel") or ""):
            best = t
    return best


def cpu_baseline(name: str, seconds: float) -> dict:
    """The C oracle (kind "port": CPU restatement, same algorithm) on the host cores."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import orc
    import pob_np as P
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))
    Bc = 4096
    e = orc.OracleEnv(name)
    s = e.reset(P.split(P.prngkey(0), Bc + 1)[1:], first=True, nthreads=cores)
    rng = np.random.default_rng(0)
    acts = rng.uniform(-1, 1, (4, Bc, 8)).astype(np.float32)
    e.step(s, acts[0], flags=3, nthreads=cores, inplace=True)  # warm the thread pool
    n, t0 = 0, time.perf_counter()
    while True:
        e.step(s, acts[n % 4], flags=3, nthreads=cores, inplace=True)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": round(Bc * n / dt, 1), "unit": "env-steps/s", "cores": cores, "kind": "port",
            "sample": f"{name} B={Bc}, {n} steps ({dt:.1f} s) of the same fused step with OpenMP "
                      f"over envs, gcc -O2 (oracle/pob_oracle.c)",
            "cpu": platform.processor() or platform.machine()}


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""bench.py -- env-steps/s of the fused MI355X rollout step (BASELINE.json metric).

Workload (BASELINE.json configs / SURVEY.md §8(d)): AntHeavenHell, batch 65 536 (the
metric's "batch 65536 @1/2/4/8 GPU": the global batch split over the N ranks), brax chain ``create('ant_heavenhell', batch_size=B)`` = AutoReset(Vmap(Episode(ActionRepeat
(env)))) with episode_length 1000, i.e. ONE fused HIP kernel per env-step (PBD physics,
POMDP logic, obs, episode counter, autoreset; the four-lane kernel as a fast launch plus a
fix-up launch that steps only the rare waves whose wall-contact store overflowed).  Synthetic inputs as the survey prescribes:
``key = PRNGKey(0)``, reset keys ``split(key, B_total + 1)[1:]`` (sharded by index), per step
``key, k = split(key)``, ``action = uniform(k, (B_total, 8), -1, 1)`` -- all generated on the
device by the threefry kernels BEFORE the timed region (inputs resident in HBM).

Modes (other BASELINE configs):
  --global-batch G       G envs split over the ranks (strong scaling; the default, G = 65 536):
                         config 4 is ``--env ant_tag --gather-obs`` and config 5
                         ``--env mixed --qp-dtype f16 --global-batch 262144``
  --batch B              B envs PER GPU instead (weak scaling, opt-in; labelled "weak")
  --gather-obs           RCCL all-gather of the observation batch of every timed step, on a
                         side stream overlapped with the next step (sharding.ObsGatherer)
  --gym                  the create_gym_env path (AutoresetVmapGymWrapper: step kernel,
                         cross-rank any-done all-reduce, masked gym reset kernel); on one
                         GPU the K gym steps are replayed from a hipGraph too

Multi-GPU: one process per GPU (torchrun); barrier + synchronize bracket the K timed steps
and the max over ranks is reported.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
# (POB_PKG_ROOT: another checkout's package directory, for interleaved A/B runs of two builds)
sys.path.insert(0, os.environ.get("POB_PKG_ROOT", os.path.join(ROOT, "po-brax_amd")))

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
# --obs-mask: po_env_mask(env, **kw) (standard_observability_masks.py) of the po-envs; stock
# Ant: the reference's own POSITION / VELOCITY sets (po_brax/standard_observability_masks.py)
OBS_MASKS = {"none": None, "no-cfrc": dict(cfrc=False), "position": dict(velocity=False, cfrc=False, task=False),
             "position+task": dict(velocity=False, cfrc=False)}
HEADLINE_METRIC = "env-steps/sec AntHeavenHell batch 65536 @1/2/4/8 GPU; % HBM roofline"  # BASELINE.json
VALU_PEAK_TF = 157.3   # FP32 vector peak, MI355X_MICROARCH.md (chip-level parameters)
HBM_PEAK_GBS = 8000.0  # HBM3E spec peak
SIMDS = 1024           # 256 CUs x 4 SIMDs
CLK_MAX_GHZ = 2.4      # max shader clock; a wave64 VALU instruction holds its SIMD 2 cycles
FLOP_ENVS = 1024       # envs of the bench workload the FLOP count replays (single-threaded oracle)
FLOP_BUDGET_S = 40.0   # its time budget (the count covers the steps done within it)


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
    ap.add_argument("--global-batch", type=int, default=65536,
                    help="total envs split over the ranks (strong scaling, the default)")
    ap.add_argument("--batch", type=int, default=0,
                    help="envs PER GPU (weak scaling, opt-in); overrides --global-batch")
    ap.add_argument("--episode-length", type=int, default=1000)
    ap.add_argument("--gym", action="store_true", help="create_gym_env path (gym-side autoreset)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="CPU-baseline budget per leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--flop-envs", type=int, default=FLOP_ENVS,
                    help="envs of this run's workload the FLOP count replays (0: the quick B = 64 / 10-step count)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (default: OMP_NUM_THREADS, the pool's per-GPU share)")
    ap.add_argument("--gather-obs", action="store_true",
                    help="RCCL all-gather of every timed step's obs batch, overlapped with the next step (N>1)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="torch.distributed backend for N>1 ('nccl' = RCCL; 'gloo' lets several ranks share "
                         "one GPU for a functional rehearsal, not a measurement)")
    ap.add_argument("--policy-mlp", type=int, default=0, metavar="H",
                    help="time the RL unroll instead: a 2-layer tanh MLP (hidden H) policy and the step, "
                         "captured together per step (rollout.PolicyRollout); not the headline workload")
    ap.add_argument("--groups", type=int, default=1,
                    help="graph rollout: env groups stepped on their own streams (rollout.GraphRollout)")
    ap.add_argument("--no-graph", action="store_true",
                    help="launch every step from Python instead of replaying the K steps from a "
                         "hipGraph (po_brax_amd.rollout); --gather-obs and the gloo-sharded gym path are eager")
    ap.add_argument("--obs-mask", default="none", choices=sorted(OBS_MASKS),
                    help="observation mask fused into the step kernel (create(..., obs_mask=idx), C ABI v7): "
                         "the step also stores obs[:, idx] (BASELINE config 2: '--global-batch 4096 "
                         "--obs-mask no-cfrc')")
    ap.add_argument("--dry-run", action="store_true",
                    help="launch rehearsal without a GPU: parse the arguments, join the process group (gloo), "
                         "gather the rank table and print the rank-0 line with no measurement")
    ap.add_argument("--legacy-spring", action="store_true",
                    help="brax <= 0.0.12 spring/impulse dynamics (the physics notebooks/ant_tag.ipynb:449 "
                         "pins) instead of PBD")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `python bench.py --gpus N` without torchrun: start the N ranks here, before anything
        # touches the GPU in this process (children by subprocess, never exec)
        return launch_ranks(args.gpus)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    if args.dry_run:
        return dry_run(args, world, rank)
    dev = torch.device("cuda", local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = dict(device_id=dev) if args.dist_backend == "nccl" else {}
        dist.init_process_group(args.dist_backend, rank=rank, world_size=world, **kw)
    if args.gym and args.env == "mixed":
        ap.error("--gym runs one env kind")
    if args.legacy_spring and args.env == "mixed":
        ap.error("--legacy-spring runs one env kind")
    if args.obs_mask != "none" and args.env == "mixed":
        ap.error("--obs-mask runs one env kind")
    mask = obs_mask_of(args.env, args.obs_mask)
    ranks = rank_devices(dev, world)  # every rank's device, gathered over the process group
    ekw = {"legacy_spring": True} if args.legacy_spring else {}
    if mask is not None:
        ekw["obs_mask"] = mask

    from po_brax_amd import envs, jumpy
    from po_brax_amd.sharding import ObsGatherer, Shard, shard_keys

    strong = args.batch <= 0
    total = args.global_batch if strong else args.batch * world
    shard = Shard(total, world, rank)
    lo, B = shard.lo, shard.size
    qp_dtype = torch.float16 if args.qp_dtype == "f16" else torch.float32
    key = jumpy.random_prngkey(0, device=dev)
    gym = None
    if args.gym:
        gym = envs.create_gym_env(args.env, batch_size=total, seed=0, episode_length=args.episode_length,
                                  device=dev, qp_dtype=qp_dtype, shard=shard if world > 1 else None, **ekw)
        gym.reset()
        state = None
    elif args.env == "mixed":
        # rank r owns global envs [lo, hi); within it the kinds follow one another
        env = envs.create_mixed(MIXED, episode_length=args.episode_length, device=dev, qp_dtype=qp_dtype)
        sizes = mixed_sizes(B)
        keys = shard_keys(key, total, world, rank)
        env.batch_sizes = sizes
        state = [e.reset(keys[o:o + b].contiguous()) for e, o, b in zip(env.envs, env.offsets(), sizes)]
    else:
        env = envs.create(args.env, batch_size=B, episode_length=args.episode_length, device=dev,
                          qp_dtype=qp_dtype, **ekw)
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

    def obs_of():
        if gym is not None:
            return gym._state.obs
        return torch.cat([s.obs.reshape(-1) for s in state]) if args.env == "mixed" else state.obs

    do_gather = args.gather_obs and world > 1 and args.env != "mixed"
    gatherer = ObsGatherer(total, obs_of().shape[-1], device=dev) if do_gather else None
    gather_ev = []  # (start, end) events of each timed step's all-gather (side stream)

    def one_step(t):
        if gym is not None:
            gym.step(act_at(t))
        else:
            env.step_(state, act_at(t))
        if gatherer is not None:  # step t's obs gathered on the side stream during step t + 1
            gatherer.submit(obs_of())

    for t in range(args.warmup):
        one_step(t)
    torch.cuda.synchronize()

    # the gym path's K steps replay from a graph too; sharded, its per-step any-done all-reduce
    # is captured with them over RCCL (rollout.GymGraphRollout), gloo steps eagerly
    use_graph = not args.no_graph and not do_gather and pre and \
        (gym is None or world == 1 or args.dist_backend == "nccl") and (gym is None or args.steps % 2 == 0)
    roll = None
    if args.policy_mlp:
        if gym is not None or args.env == "mixed" or do_gather:
            ap.error("--policy-mlp runs the create() chain of one env kind")
        from po_brax_amd.rollout import PolicyRollout
        gen = torch.Generator(device=dev).manual_seed(0)
        D, H = state.obs.shape[1], args.policy_mlp
        W1 = torch.randn((D, H), generator=gen, device=dev) * D ** -0.5
        W2 = torch.randn((H, 8), generator=gen, device=dev) * H ** -0.5

        def policy(obs):
            return torch.tanh(torch.tanh(obs @ W1) @ W2)

        roll = PolicyRollout(env, state, policy, args.steps)
    elif use_graph:  # capture the K timed steps (capture does not run them)
        from po_brax_amd.rollout import GraphRollout, GymGraphRollout
        if gym is not None:
            roll = GymGraphRollout(gym, acts[args.warmup:args.warmup + args.steps])
        else:
            roll = GraphRollout(env, state, acts[args.warmup:args.warmup + args.steps],
                                groups=args.groups if args.env != "mixed" else 1)

    # timed region: K steps.  Eager: events bracket each step's kernels on torch's current
    # stream, which the kernels use (with --gather-obs the all-gathers run on their own
    # stream, overlapped).  Graph: one replay of the K captured steps; the per-kernel time
    # then comes from an eager pass of K more steps after the timed region.
    ev_a = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_b = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    g0, g1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    if roll is not None:
        g0.record()
        roll.replay()
        g1.record()
    else:
        for k in range(args.steps):
            ev_a[k].record()
            one_step(args.warmup + k)
            ev_b[k].record()
            if gatherer is not None:
                p = (gatherer.k - 1) % gatherer.depth
                gather_ev.append((gatherer._t0[p], gatherer._done[p]))
        if gatherer is not None:  # the last gather belongs to the timed steps too
            gatherer.result((gatherer.k - 1) % gatherer.depth)
    torch.cuda.synchronize()
    gather_ms = [a.elapsed_time(b) for a, b in gather_ev] if gatherer is not None else []
    if world > 1:
        dist.barrier()
    wall = time.perf_counter() - t0
    if roll is not None and gym is None and not args.policy_mlp:  # untimed: per-step kernel durations
        for k in range(args.steps):
            ev_a[k].record()
            one_step(args.warmup + k)
            ev_b[k].record()
        torch.cuda.synchronize()
    per = ([ev_a[k].elapsed_time(ev_b[k]) for k in range(args.steps)]
           if roll is None or (gym is None and not args.policy_mlp) else [])
    eager_ms = sum(per) / len(per) if per else float("nan")
    # the dominant kernel's time per launch: from the graph replay (back-to-back launches, no
    # host gaps) when there is one -- an eager step's event pair also holds the host's launch
    # time whenever the kernel is shorter than it (small batches)
    kern_ms = g0.elapsed_time(g1) / args.steps if roll is not None else eager_ms
    gather_ms = (sum(gather_ms) / len(gather_ms)) if do_gather else None
    overlap = gather_overlap(ev_a, ev_b, gather_ev) if do_gather and roll is None else None
    # every rank's numbers, gathered (the line reports the MAX and the per-rank table)
    table = gather_rank_stats([wall, kern_ms, gather_ms or 0.0, eager_ms,
                               _num((overlap or {}).get("overlap_frac")), float(B)],
                              world, dev if args.dist_backend == "nccl" else torch.device("cpu"))
    wall, kern_ms_max = max(r[0] for r in table), max(r[1] for r in table)
    gather_max = max(r[2] for r in table)
    ms_per_step = 1e3 * wall / args.steps
    value = total * args.steps / wall
    finite = bool(torch.isfinite(obs_of()).all())

    if rank != 0:
        if world > 1:
            dist.barrier()
            dist.destroy_process_group()
        return 0

    # roofline of the dominant kernel (k_step) on this rank: algorithmic FLOPs per launch
    # (the path is FP32-VALU bound, not HBM or MFMA) and bytes per launch
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    qb = 2 if args.qp_dtype == "f16" else 4
    kinds = list(zip(MIXED, mixed_sizes(B))) if args.env == "mixed" else [(args.env, B)]
    bpe = sum(bytes_per_env_step(n, qb) * b for n, b in kinds) / B + 4 * (0 if mask is None else len(mask))
    fw = None
    try:
        import orc  # test-infrastructure oracle: FLOP count of the restated algorithm only
        okw = {"legacy_spring": 1} if args.legacy_spring else {}
        f_ref = sum(orc.flops_per_env_step(n, B=64, steps=10, mode=orc.FLOPS_REF_PAIRS, **okw) * b
                    for n, b in kinds) / B
        # the executed count on this run's own workload: the first envs of each kind's range of
        # this rank, reset from the bench's keys and stepped with its action stream through the
        # warm-up and the timed steps (verdict r4: not a B = 64 / 10-step extrapolation)
        offs = [lo + sum(b for _, b in kinds[:i]) for i in range(len(kinds))]
        if args.flop_envs <= 0:
            raise RuntimeError("--flop-envs 0")
        fws = [orc.flops_bench_workload(n, total, first=o, n=min(b, max(1, args.flop_envs // len(kinds))), warmup=args.warmup,
                                        steps=args.steps, episode_length=args.episode_length,
                                        time_budget_s=FLOP_BUDGET_S / len(kinds), **okw)
               for (n, b), o in zip(kinds, offs)]
        f_exe = sum(f["mean"] * b for f, (_, b) in zip(fws, kinds)) / B
        fw = {"envs_counted": sum(f["envs"] for f in fws), "timed_steps_counted": min(f["timed_steps_counted"] for f in fws),
              "per_step_min": round(sum(f["min"] * b for f, (_, b) in zip(fws, kinds)) / B, 1),
              "per_step_median": round(sum(f["median"] * b for f, (_, b) in zip(fws, kinds)) / B, 1),
              "per_step_max": round(sum(f["max"] * b for f, (_, b) in zip(fws, kinds)) / B, 1)}
    except Exception as ex:  # pragma: no cover
        if str(ex) != "--flop-envs 0":
            print(f"flop count unavailable: {ex}", file=sys.stderr)
        try:
            f_exe = sum(orc.flops_per_env_step(n, B=64, steps=10, mode=orc.FLOPS_EXECUTED, **okw) * b
                        for n, b in kinds) / B
        except Exception:
            f_ref = f_exe = float("nan")
    ks = kern_ms * 1e-3
    hbm_gbs = bpe * B / ks / 1e9
    tflops = f_exe * B / ks / 1e12
    kname = "k_step_mixed" if args.env == "mixed" else (
        f"k_step_legacy<{args.env}>" if args.legacy_spring else f"{step_kernel(B, args.env)}<{args.env}>")
    if split_launch(args.env, B, args.legacy_spring):
        kname += " fast launch + fix-up launch (kernel_ms: both; traffic / valu: the fast launch)"
    roofline = {
        "bound": "valu", "achieved": round(tflops, 3), "peak": VALU_PEAK_TF, "unit": "TFLOP/s",
        "frac": round(tflops / VALU_PEAK_TF, 5), "traffic": None,
        "kernel": kname + (" + gym any-done + k_reset(where done)" if gym is not None else "")
                  + (" + policy MLP GEMMs (per-step replay time, not the step kernel alone)" if args.policy_mlp else ""),
        "kernel_ms": round(kern_ms, 4), "units_per_launch": B,
        "kernel_ms_source": "hipGraph replay of the K timed steps / K" if roll is not None
                            else "HIP events around each eager step",
        "eager_event_ms": round(eager_ms, 4),
        "flops_per_env_step": round(f_exe, 1),
        "flops_basis": "instrumented CPU restatement (oracle/pob_oracle.c, ORC_COUNT_FLOPS): the float operations "
                       "(FMA = 2) of the branches the algorithm executes on the pairs the kernel evaluates -- its "
                       "broadphase and face cull only skip work that cannot produce a contact -- counted on this "
                       "run's own workload (the first envs of each kind's range: same reset keys, same action "
                       "stream, warm-up included; mean over the timed steps)",
        "flops_basis_version": "r5-workload (r4: the same executed count, extrapolated from B = 64 / 10 steps; r1-r3: "
                               "the all-pairs count)",
        "flops_workload": fw,
        "flops_reference_per_env_step": round(f_ref, 1),
        "flops_reference_basis": "the same count with every capsule x wall x triangle pair evaluated, as brax's "
                                 "unculled capsule x TriangulatedBox pairs do (64 envs, 10 random-action steps from "
                                 "reset); the kernel does "
                                 f"{f_ref / f_exe if f_exe == f_exe and f_exe else float('nan'):.1f}x less work",
        "bytes_per_env_step": round(bpe, 1),
        "hbm": {"achieved": round(hbm_gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hbm_gbs / HBM_PEAK_GBS, 6)},
    }
    build = build_identity()
    prof, stale = committed_profile(args.env, B, args.qp_dtype, args.legacy_spring, build["lib_sha256"],
                                    args.obs_mask)
    if stale is not None and gym is None:  # a profile of this config, but of another build of libpob.so
        roofline["traffic_stale_profile"] = (f"profiles/{stale['source']} profiled a different libpob.so "
                                             f"({(stale.get('build') or {}).get('lib_sha256', 'unrecorded')[:12]}); "
                                             "its counters are not reported for this build")
    if prof is not None and gym is None:
        if prof.get("traffic_bytes"):
            roofline["traffic"] = prof["traffic_bytes"]
            roofline["traffic_source"] = (f"profiles/{prof['source']}: rocprofv3 --pmc FETCH_SIZE (x2, gfx950) + "
                                          f"WRITE_SIZE per launch of the same kernel and config")
        if prof.get("valu_insts"):
            vi = prof["valu_insts"]
            roofline["valu_insts_per_launch"] = vi
            # a wave64 VALU instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md)
            roofline["valu_issue_frac"] = round(2.0 * vi / (SIMDS * ks * CLK_MAX_GHZ * 1e9), 4)
            if prof.get("grbm_gui_active"):
                cyc = prof["grbm_gui_active"] / 8.0  # GRBM sums the 8 XCDs
                roofline["valu_issue_frac_profiled_clock"] = round(2.0 * vi / (SIMDS * cyc), 4)
            roofline["valu_source"] = (f"profiles/{prof['source']}: SQ_INSTS_VALU per launch x 2 cycles / "
                                       f"({SIMDS} SIMDs x live kernel time x {CLK_MAX_GHZ} GHz); "
                                       "profiled_clock: / (SIMDs x GRBM_GUI_ACTIVE/8) of the profiled launch")

    cpu = None
    if not args.no_cpu_baseline and world == 1 and gym is None:
        cpu = cpu_baseline("ant_heavenhell" if args.env == "mixed" else args.env, B, args.cpu_seconds,
                           args.cpu_threads, legacy=args.legacy_spring)

    par = f"env-shard x{world}" + (" (strong: global batch split)" if strong else " (weak: batch per GPU)")
    line = {
        "metric": HEADLINE_METRIC if (args.env == "ant_heavenhell" and strong and total == 65536 and gym is None
                                      and not args.policy_mlp and not args.legacy_spring)
                  else f"env-steps/sec {args.env} " + ("legacy_spring " if args.legacy_spring else "")
                  + (f"global batch {total}" if strong else f"batch {args.batch}/GPU")
                  + (f" with a {args.policy_mlp}-hidden MLP policy in the loop" if args.policy_mlp else "")
                  + (f" + obs mask ({args.obs_mask})" if mask is not None else ""),
        "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
        "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
        "config": {"workload": f"{args.env} B={B}/GPU (global {total}), "
                               + ("create_gym_env (AutoresetVmapGymWrapper, gym-side autoreset)"
                                  if gym is not None else "create(batch_size=B) autoreset chain")
                               + f", episode_length {args.episode_length}, "
                               + ("legacy spring/impulse (brax <= 0.0.12)" if args.legacy_spring else "PBD")
                               + " 10 substeps, random "
                               "uniform(-1,1) actions (threefry)"
                               + (f", kinds {dict(kinds)} in one launch" if args.env == "mixed" else "")
                               + (", RCCL obs all-gather per step" if do_gather else "")
                               + (f", obs mask '{args.obs_mask}' ({len(mask)} of {_OBS[args.env]} columns) "
                                  "stored by the step kernel" if mask is not None else "")
                               + (f", MLP policy (D x {args.policy_mlp} x 8, tanh) per step in the same graph"
                                  if args.policy_mlp else ""),
                   "env": args.env, "global_batch": total, "batch_per_gpu": B,
                   "episode_length": args.episode_length, "qp_storage": args.qp_dtype, "parallelism": par,
                   "dynamics": "legacy_spring" if args.legacy_spring else "pbd",
                   "obs_mask": args.obs_mask, "obs_mask_columns": 0 if mask is None else len(mask),
                   "path": "gym" if gym is not None else "brax",
                   "launch": "hipGraph replay of the K steps" if roll is not None else "eager per step"},
        "gpu_event_ms_per_step": round(kern_ms_max, 4),
        "roofline": roofline, "cpu_baseline": cpu, "obs_finite": finite,
        # what ran: the process group's size and each rank's device (so a reader can tell N ranks
        # on N devices from N ranks sharing one)
        "world_size": world, "dist_backend": args.dist_backend if world > 1 else None,
        "rank_devices": ranks, "distinct_devices": len({r["device"] for r in ranks}),
        "per_rank": per_rank_rows(table, ranks, do_gather),
        "build": build,
    }
    if do_gather:
        # device time of one step's all-gather (side stream, max over ranks) and how much of
        # it ran under the next step's kernel (rank 0's events; the table has every rank's)
        line["obs_allgather_ms"] = round(gather_max, 4)
        line["obs_allgather_bytes"] = total * obs_of().shape[-1] * 4
        line["obs_allgather_overlap"] = overlap
        line["obs_allgather_exposed_ms_per_step"] = round(max(0.0, ms_per_step - kern_ms_max), 4)
    print(json.dumps(line))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def gather_rank_stats(vals, world: int, device) -> list:
    """every rank's list of floats (all_gather over the process group), rank order"""
    t = torch.tensor(vals, dtype=torch.float64, device=device)
    if world == 1:
        return [t.tolist()]
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    return [p.tolist() for p in parts]


def per_rank_rows(table, ranks, gather: bool) -> list:
    """the rank-0 line's per-rank table: device, envs, wall and kernel time (and the gather's)"""
    rows = []
    for r, (v, d) in enumerate(zip(table, ranks)):
        row = {"rank": r, "device": d.get("device"), "envs": int(v[5]), "kernel_ms": _r4(v[1]),
               "eager_event_ms": _r4(v[3]), "wall_s": _r4(v[0])}
        if gather:
            row["obs_allgather_ms"] = _r4(v[2])
            row["obs_allgather_overlap_frac"] = _r4(v[4])
        rows.append(row)
    return rows


def _num(x) -> float:
    return float("nan") if x is None else float(x)


def _r4(x):
    return None if x is None or x != x else round(float(x), 4)


def gather_overlap(ev_a, ev_b, gather_ev) -> dict:
    """How much of each step's all-gather (side stream, events gather_ev[k]) ran while step
    k + 1's kernel did ([ev_a[k + 1], ev_b[k + 1]] on the compute stream): the events' times
    relative to ev_a[0].  The last step's gather has no next step and is left out."""
    ref = ev_a[0]
    tot = ov = 0.0
    for k in range(len(gather_ev) - 1):
        g0, g1 = ref.elapsed_time(gather_ev[k][0]), ref.elapsed_time(gather_ev[k][1])
        s0, s1 = ref.elapsed_time(ev_a[k + 1]), ref.elapsed_time(ev_b[k + 1])
        tot += g1 - g0
        ov += max(0.0, min(g1, s1) - max(g0, s0))
    n = max(1, len(gather_ev) - 1)
    return {"gathers": len(gather_ev) - 1, "mean_ms": round(tot / n, 4), "overlapped_ms": round(ov / n, 4),
            "overlap_frac": round(ov / tot, 4) if tot > 0 else None,
            "basis": "HIP events: side-stream all-gather of step k vs step k + 1's compute-stream span"}


def dry_run(args, world: int, rank: int) -> int:
    """--dry-run: the multi-rank plumbing of a real run (argument parser, process group, rank
    table gather, shard sizes, the rank-0 line) with no device work -- what the CPU tests
    run through launch_ranks."""
    from po_brax_amd.sharding import Shard
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)
    strong = args.batch <= 0
    total = args.global_batch if strong else args.batch * world
    shard = Shard(total, world, rank)
    me = {"rank": rank, "device": f"cpu:{rank}", "pid": os.getpid()}
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    table = gather_rank_stats([float("nan"), float("nan"), 0.0, float("nan"), float("nan"), float(shard.size)],
                              world, torch.device("cpu"))
    if rank == 0:
        print(json.dumps({"dry_run": True, "env": args.env, "world_size": world, "global_batch": total,
                          "scaling": "strong" if strong else "weak", "steps": args.steps, "warmup": args.warmup,
                          "obs_mask": args.obs_mask, "gather_obs": args.gather_obs,
                          "rank_devices": ranks, "per_rank": per_rank_rows(table, ranks, args.gather_obs)}))
        sys.stdout.flush()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


def launch_ranks(n: int, argv=None, script: str = None) -> int:
    """Run this command as ``n`` ranks on this node (what torchrun would do): child processes
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, sharing this
    process's stdout (rank 0 prints the JSON line).  Returns non-zero if any rank fails; the
    other ranks are then terminated (they would wait at a barrier).  SIGTERM / Ctrl-C of this
    process terminates every rank too (then killed after 30 s) and returns 143 / 130."""
    import signal
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]

    class _Term(Exception):
        pass

    def _on_term(signum, frame):
        raise _Term()

    try:
        old = signal.signal(signal.SIGTERM, _on_term)
    except ValueError:  # not the main thread: no handler (the caller owns signals)
        old = None
    procs, live, rc = [], [], 0
    try:
        for r in range(n):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__),
                                           *(sys.argv[1:] if argv is None else argv)], env=env))
            live.append(procs[-1])
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 1
                    print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the others", file=sys.stderr)
                    _stop(live)
                    live = []
                    break
            if live:
                time.sleep(0.2)
    except (_Term, KeyboardInterrupt) as ex:
        rc = 143 if isinstance(ex, _Term) else 130
        print(f"bench.py: {'SIGTERM' if rc == 143 else 'interrupted'}; stopping {len(live)} rank(s)", file=sys.stderr)
    finally:
        _stop(live)
        if old is not None:
            signal.signal(signal.SIGTERM, old)
    return rc


def _stop(procs) -> None:
    """terminate, then kill after 30 s, the given child processes (exact PIDs we started)"""
    import subprocess
    for q in procs:
        if q.poll() is None:
            q.terminate()
    for q in procs:
        try:
            q.wait(timeout=30)
        except subprocess.TimeoutExpired:
            q.kill()
            q.wait()


def rank_devices(dev, world: int) -> list:
    """[{rank, device, pci}] of every rank (all_gather_object over the process group)."""
    me = {"rank": int(os.environ.get("RANK", "0")), "device": f"cuda:{dev.index}"}
    try:
        pr = torch.cuda.get_device_properties(dev)
        me["pci"] = f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
        me["device"] = me["pci"]
    except Exception:  # pragma: no cover (older torch: no PCI ids)
        pass
    if world == 1:
        return [me]
    out = [None] * world
    dist.all_gather_object(out, me)
    return out


def step_kernel(B: int, env: str = "ant_heavenhell") -> str:
    """The step kernel pob_step launches for a batch of B envs (pob_kernels.hip pob_step:
    sixteen lanes per env up to POB_HEXA_MAX_B (per kind: HH and TAG 32, else 16 x the CU
    count), eight up to POB_OCTET_MAX_B (16 384), four above)."""
    n_cu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    hex_default = {"ant_heavenhell": 32, "ant_tag": 32}.get(env, 16) * n_cu
    if B <= int(os.environ.get("POB_HEXA_MAX_B", str(hex_default))):
        return "k_step_hex"
    if B <= int(os.environ.get("POB_OCTET_MAX_B", "16384")):
        return "k_step_oct"
    return "k_step_quad"


def split_launch(env: str, B: int, legacy: bool) -> bool:
    """Does pob_step launch the four-lane kernel as a fast launch + a fix-up launch here
    (pob_kernels.hip quad_split_launch: HH, GA, TAG on the four-lane kernel and, since round 6,
    the mixed launch; GA at <= 3 waves per SIMD stays one launch; POB_QUAD_SPLIT overrides)?"""
    f = os.environ.get("POB_QUAD_SPLIT")
    if env == "mixed" and not legacy:
        return int(f) != 0 if f else True
    if legacy or env == "ant" or step_kernel(B, env) != "k_step_quad":
        return False
    n_cu = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
    if env == "ant_gather" and 4 * B <= 3 * 64 * 4 * n_cu:
        return False
    return int(f) != 0 if f else True


def committed_profile(env: str, B: int, qp: str, legacy: bool = False, lib_sha256: str = None,
                      obs_mask: str = "none"):
    """(profile, stale): the counters per launch of the newest committed PMC profile of this
    exact config (profiles/*_traffic.json, written by profiles/summarize.py) whose profiled
    run loaded the same libpob.so (the bench line's build.lib_sha256), and the newest profile
    of the config from any other build (None when there is a current one)."""
    cur, stale = None, None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json"))):
        try:
            t = json.load(open(p))
        except (OSError, ValueError):
            continue
        if t.get("env") == env and t.get("batch") == B and t.get("qp_storage", "f32") == qp and \
                "k_step" in (t.get("kernel") or "") and bool(t.get("legacy_spring", False)) == bool(legacy) and \
                (t.get("obs_mask") or "none") == obs_mask:
            k = (t.get("generated", 0.0), p)  # newest by the summary's timestamp, then name
            same = lib_sha256 is not None and (t.get("build") or {}).get("lib_sha256") == lib_sha256
            if same and (cur is None or k > cur[0]):
                cur = (k, t)
            elif not same and (stale is None or k > stale[0]):
                stale = (k, t)
    return (cur[1] if cur else None), (stale[1] if stale and not cur else None)


def build_identity() -> dict:
    """The loaded libpob.so (path, sha256) and the sha256 of the sources it is built from."""
    import hashlib
    from po_brax_amd import _lib
    h = hashlib.sha256()
    with open(_lib.LIB_PATH, "rb") as f:
        h.update(f.read())
    src = hashlib.sha256()
    csrc = os.path.join(ROOT, "po-brax_amd", "csrc")
    for fn in sorted(os.listdir(csrc)) if os.path.isdir(csrc) else []:
        if fn.endswith((".hip", ".h", ".cpp")):
            src.update(fn.encode())
            with open(os.path.join(csrc, fn), "rb") as f:
                src.update(f.read())
    return {"lib": os.path.relpath(_lib.LIB_PATH, ROOT) if _lib.LIB_PATH.startswith(ROOT) else _lib.LIB_PATH,
            "lib_sha256": h.hexdigest(), "csrc_sha256": src.hexdigest(), "abi": _lib.ABI_VERSION}


def obs_mask_of(env: str, name: str):
    """The --obs-mask column indices (None for 'none')."""
    kw = OBS_MASKS[name]
    if kw is None:
        return None
    from po_brax_amd import standard_observability_masks as M
    if env == "ant":
        parts = [M.POSITION["ant"]] + ([] if kw.get("velocity") is False else [M.VELOCITY["ant"]])
        import numpy as np
        return np.concatenate(parts)
    return M.po_env_mask(env, **kw)


def cpu_baseline(name: str, B: int, seconds: float, threads: int = 0, legacy: bool = False) -> dict:
    """The C restatement (kind "port": same algorithm, oracle/pob_oracle.c) compiled
    -O3 -march=native on this host, timed on the same workload (this GPU's batch B): on the
    process's CPU share and on one thread (OpenMP over envs, static schedule; time-boxed).

    The share is ``OMP_NUM_THREADS`` (the GPU pool sets 16 per GPU and asks jobs to size their
    thread pools to it: ``sched_getaffinity`` there lists the whole shared host, 256 cores,
    most of them other tenants'), or every affinity core when it is unset; ``threads`` (bench
    ``--cpu-threads``, e.g. all cores of a dedicated host) overrides it.  The reported
    ``value`` is the multi-threaded leg.  No all-cores leg runs on the GPU pool: its hosts are
    shared, each GPU's job gets a 16-thread CPU share and the pool's rules ask jobs to size
    their thread pools to it (the line says so in ``all_cores``); ``--cpu-threads N`` times N
    threads on a dedicated host."""
    import numpy as np
    import orc
    import pob_np as P
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        aff = os.cpu_count() or 1
    share = max(1, min(aff, int(os.environ.get("OMP_NUM_THREADS") or aff)))
    nt_multi = max(1, min(aff, threads)) if threads > 0 else share
    e = orc.OracleEnv(name, native=True, **({"legacy_spring": 1} if legacy else {}))
    s = e.reset(P.split(P.prngkey(0), B + 1)[1:], first=True, nthreads=nt_multi)
    acts = np.random.default_rng(0).uniform(-1, 1, (2, B, 8)).astype(np.float32)
    out = {}
    for leg, nt in (("multi", nt_multi), ("single", 1)):
        e.step(s, acts[0], flags=3, nthreads=nt, inplace=True)  # warm caches / the thread pool
        n, t0 = 0, time.perf_counter()
        while True:
            e.step(s, acts[n % 2], flags=3, nthreads=nt, inplace=True)
            n += 1
            if time.perf_counter() - t0 >= seconds:
                break
        dt = time.perf_counter() - t0
        out[leg] = (B * n / dt, n, dt, nt)
    v, n, dt, _ = out["multi"]
    v1 = out["single"][0]
    return {"value": round(v, 1), "unit": "env-steps/s", "cores": nt_multi, "kind": "port",
            "single_thread_value": round(v1, 1),
            "all_cores": (f"measured: {nt_multi} threads = every affinity core" if nt_multi >= aff else
                          f"not run: this host's {aff} affinity cores are shared by the GPU pool's jobs, which "
                          f"give each GPU's job a {share}-thread CPU share (OMP_NUM_THREADS) and require thread "
                          "pools sized to it; an all-core leg would time other tenants' load. "
                          "`bench.py --cpu-threads N` times N threads on a dedicated host"),
            "sample": f"{name} B={B} (the GPU workload's batch)" + (", legacy spring dynamics" if legacy else "")
                      + ", the same fused step (oracle/pob_oracle.c, "
                      "gcc -O3 -march=native, OpenMP over envs): "
                      + "; ".join(f"{o[1]} steps in {o[2]:.1f} s on {o[3]} thread(s)" for o in out.values()),
            "threads_basis": ("--cpu-threads" if threads > 0 else
                              "OMP_NUM_THREADS (the pool's per-GPU CPU share)" if share < aff else "all affinity cores"),
            "cpu": orc.cpu_model(), "nproc": os.cpu_count(), "affinity_cores": aff}


if __name__ == "__main__":
    sys.exit(main())

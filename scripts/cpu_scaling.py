"""Thread scaling of the CPU restatement on this host (bench.py's cpu_baseline leg at 1, 2, 4,
... threads up to every affinity core): the evidence behind the line's all_cores_linear_bound.
Run it on a host you have to yourself; on the GPU pool it stops at OMP_NUM_THREADS (the per-GPU
share the pool's shared hosts give a job, bench.py cpu_baseline).

    python scripts/cpu_scaling.py [--env ant_heavenhell] [--B 16384] [--steps 4]
Prints one JSON object."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="ant_heavenhell")
    ap.add_argument("--B", type=int, default=16384)
    ap.add_argument("--steps", type=int, default=4, help="steps after the reset, the same in every leg")
    args = ap.parse_args()
    import numpy as np
    import orc
    import pob_np as P
    aff = len(os.sched_getaffinity(0))
    # at most OMP_NUM_THREADS when it is set (the GPU pool's per-GPU share: 16)
    top = max(1, min(aff, int(os.environ.get("OMP_NUM_THREADS") or aff)))
    threads = sorted({1, *[t for t in (2, 4, 8, 16, 32, 64, 128, 256) if t <= top], top})
    e = orc.OracleEnv(args.env, native=True)
    keys = P.split(P.prngkey(0), args.B + 1)[1:]
    acts = np.random.default_rng(0).uniform(-1, 1, (args.steps, args.B, 8)).astype(np.float32)
    rows = []
    for nt in threads:  # every leg: the same reset, the same steps (the same work)
        s = e.reset(keys, first=True, nthreads=top)
        t0 = time.perf_counter()
        for t in range(args.steps):
            e.step(s, acts[t], flags=3, nthreads=nt, inplace=True)
        dt = time.perf_counter() - t0
        rows.append({"threads": nt, "env_steps_per_s": round(args.B * args.steps / dt, 1), "seconds": round(dt, 2)})
    one = rows[0]["env_steps_per_s"]
    for r in rows:
        r["vs_linear"] = round(r["env_steps_per_s"] / (one * r["threads"]), 3)
    print(json.dumps({"env": args.env, "B": args.B, "cpu": orc.cpu_model(), "affinity_cores": aff, "max_threads": top,
                      "kind": "port (oracle/pob_oracle.c, gcc -O3 -march=native, OpenMP over envs)",
                      "note": "every leg steps the same envs from the same reset through the same actions",
                      "rows": rows}))


if __name__ == "__main__":
    main()

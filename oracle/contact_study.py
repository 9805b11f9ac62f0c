"""Ant x Arena contact model study -- TEST INFRASTRUCTURE (oracle only, CPU).

Compares the brax v1 capsule x TriangulatedBox restatement (wall_contact = 0, the reference's
algorithm) with the round-1..3 model (wall_contact = 1: the deepest sphere-box contact over
the capsule's end points, one per capsule) on the workloads' own states:

  stats       contact statistics of the mesh model over random-action rollouts (contacts per
              capsule per collide substep, faces surviving the face cull, segment points inside
              a box, degenerate zero-distance contacts)
  one-step    the two models stepped once from the SAME state (mesh-model rollout states at
              several times, the HH spawn states, and wall-stress states: ants teleported onto
              the arena walls): share of envs whose qp changes, size of the change
  trajectory  both models run from the same reset: share of envs apart after T steps
  cull        the face cull's exactness: the mesh model with and without it, bit-identical

    python oracle/contact_study.py [--B 1024] [--T 300] > profiles/r4_contact_study.txt
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import orc  # noqa: E402
import pob_np as P  # noqa: E402

FLAGS = orc.F_EPISODE | orc.F_AUTORESET
KINDS = ("ant_heavenhell", "ant_tag", "ant_gather")
QP = ("pos", "rot", "vel", "ang")


def _acts(seed, B, T):
    rng = np.random.default_rng(seed)
    return [rng.uniform(-1, 1, (B, 8)).astype(np.float32) for _ in range(T)]


def _copy(s):
    return {k: v.copy() for k, v in s.items()}


def _diff(a, b):
    """per env: max |a - b| over the 9 ant bodies' pos (m) and over every qp field"""
    dp = np.abs(a["pos"][:, :9] - b["pos"][:, :9]).reshape(len(a["pos"]), -1).max(1)
    dq = np.zeros_like(dp)
    for f in QP:
        dq = np.maximum(dq, np.abs(a[f][:, :9] - b[f][:, :9]).reshape(len(a[f]), -1).max(1))
    return dp, dq


def _report_one_step(tag, dp, dq):
    moved = dq > 0
    n = len(dp)
    line = f"  {tag:<34} envs differing: {moved.sum():5d}/{n} ({100 * moved.mean():5.1f} %)"
    if moved.any():
        line += (f"  |dpos| max {dp.max():.3e}  median(differing) {np.median(dp[moved]):.3e}"
                 f"  any-qp max {dq.max():.3e}")
    print(line)


def stats(name, B, T, seed=0):
    L = orc.lib()
    e = orc.OracleEnv(name, wall_contact=0)
    s = e.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True)
    L.orc_contact_stats_enable(1)
    buf = (C.c_longlong * 16)()
    L.orc_contact_stats(buf)
    t0 = time.time()
    for a in _acts(seed + 1, B, T):
        e.step(s, a, flags=FLAGS, episode_length=1000, inplace=True)
    L.orc_contact_stats(buf)
    L.orc_contact_stats_enable(0)
    st = list(buf)
    caps = sum(st[8:16])
    print(f"[stats] {name} B={B} T={T} ({time.time() - t0:.1f} s, single thread)")
    print(f"  detections {st[7]}, capsule-detections {caps}, capsule x wall pairs evaluated {st[0]}, "
          f"faces past the face cull {st[1]} ({st[1] / max(1, st[0]):.3f} per pair)")
    print(f"  triangle contacts {st[2]} ({st[2] / max(1, caps):.4f} per capsule-detection); capsule-detections with "
          f">= 1 wall contact {st[3]} ({100 * st[3] / max(1, caps):.2f} %); most contacts of one capsule {st[4]}")
    print(f"  contacts per capsule-detection histogram (0..6, >=7): {st[8:16]}")
    print(f"  contacts whose segment point is inside the box: {st[5]}; zero-distance (segment touching "
          f"the triangle) contacts: {st[6]}")


def one_step(name, B, T, seed=0):
    em, es = orc.OracleEnv(name, wall_contact=0), orc.OracleEnv(name, wall_contact=1)
    s = em.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True, nthreads=8)
    ss = es.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True, nthreads=8)
    dp, dq = _diff(s, ss)
    print(f"[one-step] {name} B={B}: the two models stepped once from the same state")
    _report_one_step("reset (sys.info only: obs cfrc)", np.abs(s["obs"] - ss["obs"]).max(1),
                     np.abs(s["obs"] - ss["obs"]).max(1))
    acts = _acts(seed + 2, B, T)
    probe = sorted({0, 1, 10, 50, 100, T - 1})
    for t, a in enumerate(acts):
        if t in probe:
            a1 = em.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8)
            a2 = es.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8)
            _report_one_step(f"step {t} of a mesh-model rollout", *_diff(a1, a2))
        em.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8, inplace=True)


def wall_stress(name, B, seed=3):
    """ants teleported so that the torso lands uniformly in the arena's bounding box (many touch
    or straddle a wall), then one step of each model from the same state"""
    em, es = orc.OracleEnv(name, wall_contact=0), orc.OracleEnv(name, wall_contact=1)
    s = em.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True, nthreads=8)
    rng = np.random.default_rng(seed)
    box = {"ant_heavenhell": ((-7.25, -1.0), (7.25, 9.0)), "ant_tag": ((-6.0, -6.0), (6.0, 6.0)),
           "ant_gather": ((-7.5, -7.5), (7.5, 7.5))}[name]
    xy = rng.uniform(box[0], box[1], (B, 2)).astype(np.float32)
    sh = xy - s["pos"][:, 0, :2]
    s["pos"][:, :10, :2] += sh[:, None, :]
    a = _acts(seed + 4, B, 1)[0]
    a1 = em.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8)
    a2 = es.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8)
    print(f"[wall-stress] {name} B={B}: torso teleported uniformly over the arena's bounding box")
    _report_one_step("one step from the teleported state", *_diff(a1, a2))


def trajectory(name, B, T, seed=0):
    em, es = orc.OracleEnv(name, wall_contact=0), orc.OracleEnv(name, wall_contact=1)
    k = P.split(P.prngkey(seed), B + 1)[1:]
    s1, s2 = em.reset(k, first=True, nthreads=8), es.reset(k, first=True, nthreads=8)
    for a in _acts(seed + 5, B, T):
        em.step(s1, a, flags=orc.F_EPISODE, episode_length=10 ** 6, nthreads=8, inplace=True)
        es.step(s2, a, flags=orc.F_EPISODE, episode_length=10 ** 6, nthreads=8, inplace=True)
    d = np.linalg.norm(s1["pos"][:, 0] - s2["pos"][:, 0], axis=1)
    print(f"[trajectory] {name} B={B}: both models {T} steps from the same reset, no autoreset: torso apart by "
          f"> 1e-4 m in {100 * (d > 1e-4).mean():.1f} %, > 1e-2 m in {100 * (d > 1e-2).mean():.1f} %, "
          f"> 0.1 m in {100 * (d > 0.1).mean():.1f} % of envs; median {np.median(d):.3e} m")


def cull_exact(name, B, T, seed=7):
    L = orc.lib()
    e = orc.OracleEnv(name, wall_contact=0)
    k = P.split(P.prngkey(seed), B + 1)[1:]
    outs = []
    for cull in (1, 0):
        L.orc_set_face_cull(cull)
        s = e.reset(k, first=True, nthreads=8)
        for a in _acts(seed + 1, B, T):
            e.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8, inplace=True)
        outs.append(s)
    L.orc_set_face_cull(1)
    same = all(np.array_equal(outs[0][f], outs[1][f]) for f in QP + ("obs",))
    print(f"[cull] {name} B={B} T={T}: face cull on vs off bit-identical: {same}")
    return same


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--T", type=int, default=300)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    print(f"# Ant x Arena contact study (oracle/contact_study.py, B={a.B}, T={a.T}; {orc.cpu_model()})")
    for name in KINDS:
        if a.only and name != a.only:
            continue
        stats(name, min(a.B, 512), a.T)
        one_step(name, a.B, a.T)
        wall_stress(name, a.B)
        trajectory(name, a.B, 100)
        cull_exact(name, min(a.B, 256), 60)
        print()


if __name__ == "__main__":
    main()

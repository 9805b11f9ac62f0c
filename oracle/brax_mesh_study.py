"""brax capsule_mesh spelling study -- TEST INFRASTRUCTURE (oracle only, CPU).

The restatement's capsule x TriangulatedBox contacts (oracle/pob_oracle.c capsule_wall_mesh)
can be evaluated in the exact geometric form or in brax v1's own spelling [ext, recalled], one
deviation at a time (orc_set_mesh_variant bits, DESIGN.md §3 "deviation table"):

  1 eps-normal   normal = (S - P) / (1e-6 + dist); a touching / piercing segment (S == P)
                 gives the zero normal instead of the face's outward normal
  (safe-norm     capsule_mesh's jp.safe_norm(penetration_vec, axis=1) zeroes the distance only
                 when ALL twelve triangles' S - P are within 1e-8 of zero: never for a box, so
                 the plain norm is brax's value; not a variant)
  4 pos-tri      the contact sits at the triangle point P, not at the capsule surface S - r n
  8 form         brax's closest-point forms (segment-segment with unit directions, mid-point
                 parameters and (denom + 1e-6); segment-plane with (n.(b - a) + 1e-6);
                 barycentric closest triangle point; ties averaged)

For each variant v: one env-step from the SAME state with the variant and with the exact
form (v = 0), on the HH spawn states (ants spawn against the T-maze's bottom wall, legs
through it), on mesh-model rollout states, and on wall-stress states (torso teleported over
the arena); reported: the share of envs whose qp moves by more than the north-star tolerance
(|a - b| > 1e-5 max(1, |b|) on any qp component of the 9 ant bodies), and the largest moves.
The noise floor is the same measure for a 1-ulp change of the input positions (what any
reassociation of the float arithmetic, e.g. XLA's, does to one step).  A contact-level table
compares the forms' contacts (normal, penetration, segment parameter) on random capsule-wall
configurations.

    python oracle/brax_mesh_study.py [--B 1024] > profiles/r5_brax_mesh_study.txt
"""
from __future__ import annotations

import argparse
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import orc  # noqa: E402
import pob_np as P  # noqa: E402

FLAGS = orc.F_EPISODE | orc.F_AUTORESET
QP = ("pos", "rot", "vel", "ang")
VARIANTS = ((1, "eps-normal"), (4, "pos-tri"), (8, "form"), (1 | 4, "eps-normal+pos-tri"),
            (13, "all three (brax spelling)"))
BASE = 0  # the form each variant is measured against (--unpinned: the adopted spelling, 13)
# the choices nothing pins (round 6, verdict r5 item 4; oracle/pob_oracle.c MV_DIAG ..): each on
# top of the adopted spelling, measured against it
UNPINNED = ((13 | 16, "other diagonal (V1-V3)"), (13 | 32, "winding reversed (n inward)"),
            (13 | 64, "edges as loop p2->p0"), (13 | 128, "world frame"),
            (13 | 16 | 32 | 64 | 128, "all four"))
TOL = 1e-5


def _acts(seed, B, T):
    rng = np.random.default_rng(seed)
    return [rng.uniform(-1, 1, (B, 8)).astype(np.float32) for _ in range(T)]


def _moved(a, b):
    """per env: any qp component of the ant bodies outside TOL (relative to max(1, |b|)); and
    the largest |a - b| per field (mx['far']: share of envs whose positions move > 1 mm)"""
    bad = np.zeros(len(a["pos"]), bool)
    mx = {"far": float((np.abs(a["pos"][:, :9] - b["pos"][:, :9]).reshape(len(bad), -1).max(1) > 1e-3).mean())}
    for f in QP:
        d = np.abs(a[f][:, :9].astype(np.float64) - b[f][:, :9])
        rel = d / np.maximum(1.0, np.abs(b[f][:, :9]))
        bad |= (rel > TOL).reshape(len(d), -1).any(1)
        mx[f] = float(d.max())
    return bad, mx


def _line(tag, bad, mx):
    return (f"    {tag:<26} envs beyond 1e-5: {bad.sum():5d}/{len(bad)} ({100 * bad.mean():5.1f} %), pos > 1 mm: "
            f"{100 * mx['far']:5.1f} %   max |d| "
            f"pos {mx['pos']:.2e} m  rot {mx['rot']:.2e}  vel {mx['vel']:.2e} m/s  ang {mx['ang']:.2e} rad/s")


def _step(e, s, a, variant):
    L = orc.lib()
    prev = L.orc_get_mesh_variant()
    L.orc_set_mesh_variant(variant)
    try:
        return e.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8)
    finally:
        L.orc_set_mesh_variant(prev)


def _ulp(s):
    t = {k: v.copy() for k, v in s.items()}
    t["pos"][:, :9] = np.nextafter(t["pos"][:, :9], np.float32(np.inf))
    return t


def _study_states(e, s, a, title):
    print(f"  [{title}]")
    base = _step(e, s, a, BASE)
    print(_line("noise floor (1-ulp pos)", *_moved(_step(e, _ulp(s), a, BASE), base)))
    for v, name in VARIANTS:
        print(_line(f"{v:2d} {name}", *_moved(_step(e, s, a, v), base)))


def one_step(name, B, seed=0):
    e = orc.OracleEnv(name)
    s = e.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True, nthreads=8)
    acts = _acts(seed + 2, B, 101)
    rollout_form = "brax spelling" if orc.lib().orc_get_mesh_variant() == 13 else "exact form"
    print(f"[one step] {name} B={B}")
    for t, a in enumerate(acts):
        if t in (0, 10, 100):
            _study_states(e, s, a, "spawn states (reset)" if t == 0 else f"step {t} of a rollout ({rollout_form})")
        e.step(s, a, flags=FLAGS, episode_length=1000, nthreads=8, inplace=True)


def wall_stress(name, B, seed=3):
    e = orc.OracleEnv(name)
    s = e.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True, nthreads=8)
    rng = np.random.default_rng(seed)
    box = {"ant_heavenhell": ((-7.25, -1.0), (7.25, 9.0)), "ant_tag": ((-6.0, -6.0), (6.0, 6.0)),
           "ant_gather": ((-7.5, -7.5), (7.5, 7.5))}[name]
    xy = rng.uniform(box[0], box[1], (B, 2)).astype(np.float32)
    sh = xy - s["pos"][:, 0, :2]
    s["pos"][:, :10, :2] += sh[:, None, :]
    print(f"[wall stress] {name} B={B}: torso teleported uniformly over the arena's bounding box")
    _study_states(e, s, _acts(seed + 4, B, 1)[0], "teleported states")


def contact_table(n=20000, seed=11):
    """the forms' contacts on random capsules near one HH wall (halfsize 2.5 x .5 x .5, rotated
    180 degrees like wall 5): matched by (face, triangle) order where both forms agree on the
    contact set"""
    L = orc.lib()
    prev = L.orc_get_mesh_variant()
    rng = np.random.default_rng(seed)
    wall = np.array([0.0, -0.5, 0.5, -1.0, 0.0, 2.5, 0.5, 0.5], np.float32)
    rows = {v: [] for v, _ in VARIANTS}
    nset = {v: 0 for v, _ in VARIANTS}
    npierce = 0
    for _ in range(n):
        c = np.array([rng.uniform(-3, 3), rng.uniform(-1.3, 0.3), rng.uniform(-0.1, 1.1)], np.float32)
        d = rng.normal(size=3)
        d = (d / np.linalg.norm(d) * 0.2828).astype(np.float32)
        a, b, r = c + d, c - d, 0.08
        L.orc_set_mesh_variant(BASE)
        c0 = orc.mesh_contacts(wall, a, b, True, r)[:, :5]
        if len(c0) == 0:
            continue
        if (c0[:, 4] >= r).any():
            npierce += 1
        for v, _ in VARIANTS:
            L.orc_set_mesh_variant(v)
            cv = orc.mesh_contacts(wall, a, b, True, r)[:, :5]
            if len(cv) != len(c0):
                nset[v] += 1
                continue
            rows[v].append(np.abs(cv - c0))
    L.orc_set_mesh_variant(prev)
    print(f"[contacts] {n} random leg capsules (r = 0.08, half-length 0.283) near an HH wall; "
          f"{npierce} configurations with a touching / piercing triangle")
    for v, name in VARIANTS:
        if rows[v]:
            m = np.concatenate(rows[v])
            print(f"    {v:2d} {name:<26} contact sets differ in {nset[v]} configs; over matched contacts max |d tau| "
                  f"{m[:, 0].max():.2e}  max |d n| {m[:, 1:4].max():.2e}  max |d pen| {m[:, 4].max():.2e}  "
                  f"median |d n| {np.median(m[:, 1:4].max(1)):.2e}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=1024)
    ap.add_argument("--rollout-variant", type=int, default=None,
                    help="the spelling the rollouts run in (default: the oracle's)")
    ap.add_argument("--unpinned", action="store_true",
                    help="the unpinned choices (triangulation, winding, edge loop, frame) against the adopted spelling")
    a = ap.parse_args()
    global VARIANTS, BASE
    if a.unpinned:
        VARIANTS, BASE = UNPINNED, 13
    if a.rollout_variant is not None:
        orc.lib().orc_set_mesh_variant(a.rollout_variant)
    t0 = time.time()
    print(f"# brax capsule_mesh spelling study (oracle/brax_mesh_study.py, B={a.B}; {orc.cpu_model()})")
    print(f"# one env-step from the same state, variant vs {'the adopted spelling (13)' if BASE else 'the exact form'}; "
          f"'beyond 1e-5': any qp component of the "
          f"9 ant bodies with |a - b| > 1e-5 max(1, |b|)")
    contact_table()
    for name in ("ant_heavenhell", "ant_tag", "ant_gather"):
        one_step(name, a.B)
        wall_stress(name, a.B)
    print(f"# {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()

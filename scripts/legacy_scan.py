"""Exploration: brax <= 0.0.12 legacy (spring / impulse) physics variants against frame 1
of the notebook trajectory (tests/golden/ant_tag_notebook_trajectory.json).  float64.
Prints the max body-position error at frames 1..3 for every variant combination."""
import itertools
import json
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pob_np as P  # noqa: E402

d = json.load(open(os.path.join(ROOT, "tests", "golden", "ant_tag_notebook_trajectory.json")))
POS = np.array(d["pos"])[:, :9]
ROT = np.array(d["rot"])[:, :9]


def rot(v, q):
    s = q[..., :1]; u = q[..., 1:]
    return 2 * np.sum(u * v, -1, keepdims=True) * u + (s * s - np.sum(u * u, -1, keepdims=True)) * v + 2 * s * np.cross(u, v)


def qmul(u, v):
    w1, x1, y1, z1 = np.moveaxis(u, -1, 0); w2, x2, y2, z2 = np.moveaxis(v, -1, 0)
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], -1)


MASS = np.array([b[1] for b in P.ANT_BODIES])
J = P.ANT_JOINTS
PAR = np.array([j[0] for j in J]); CHI = np.array([j[1] for j in J])
OFFP = np.array([P.f32(j[2]) for j in J]); OFFC = np.array([P.f32(j[3]) for j in J])
EQ = [P.euler_to_quat(P.f32(j[4])) for j in J]
AX = np.array([P.rotate(np.array([1., 0, 0]), q) for q in EQ])
REF = np.array([P.rotate(np.array([0, 0, 1.]), q) for q in EQ])
LIM = np.array([j[5] for j in J], float) * np.pi / 180
GB = [0, 2, 4, 6, 8]
GE = np.array([P.capsule_ends(i)[0][0] for i in GB])
GR = np.array([P.capsule_ends(i)[1] for i in GB])


def step(x, q, v, w, act, V):
    h = 0.05 / 10
    k, c, ad, kl = 18000.0, 80.0, 20.0, 18000.0
    erp = 0.1 * 10 / 0.05
    g = np.array([0, 0, -9.8])
    for _ in range(10):
        if V["order"] == "kin_first":
            x, q = kinetic(x, q, v, w, h)
        dv, dw = joints(x, q, v, w, act, V, k, c, ad, kl)
        v = v + (dv + g) * h
        w = np.exp(-0.05 * h) * w + dw * h
        dvc, dwc = contacts(x, q, v, w, V, erp)
        v = v + dvc; w = w + dwc
        if V["order"] == "kin_last":
            x, q = kinetic(x, q, v, w, h)
    return x, q, v, w


def kinetic(x, q, v, w, h):
    x = x + v * h
    wq = np.concatenate([np.zeros((len(w), 1)), w], -1)
    q = q + 0.5 * h * qmul(wq, q)
    return x, q / np.linalg.norm(q, axis=-1, keepdims=True)


def joints(x, q, v, w, act, V, k, c, ad, kl):
    p, ch = PAR, CHI
    rp, rc = rot(OFFP, q[p]), rot(OFFC, q[ch])
    posp, posc = x[p] + rp, x[ch] + rc
    velp, velc = v[p] + np.cross(w[p], rp), v[ch] + np.cross(w[ch], rc)
    imp = k * (posp - posc) + c * (velp - velc)
    dv = np.zeros((9, 3)); dw = np.zeros((9, 3))
    ap, ac = rot(AX, q[p]), rot(AX, q[ch])
    fp, fc = rot(REF, q[p]), rot(REF, q[ch])
    psi = np.arctan2(np.sum(np.cross(fp, fc) * ap, -1), np.sum(fp * fc, -1))
    dang = np.where(psi < LIM[:, 0], LIM[:, 0] - psi, 0.0)
    dang = np.where(psi > LIM[:, 1], LIM[:, 1] - psi, dang)
    tq = k * np.cross(ap, ac) - kl * ap * dang[:, None] - ad * (w[p] - w[ch])
    ta = ap * (act * 350.0)[:, None]
    for j in range(8):
        dv[p[j]] += -imp[j] / MASS[p[j]]; dv[ch[j]] += imp[j] / MASS[ch[j]]
        dw[p[j]] += np.cross(rp[j], -imp[j]) + tq[j] - ta[j]
        dw[ch[j]] += np.cross(rc[j], imp[j]) - tq[j] + ta[j]
    return dv, dw


def contacts(x, q, v, w, V, erp):
    dv = np.zeros((9, 3)); dw = np.zeros((9, 3))
    n = np.array([0, 0, 1.0])
    for b, e, r in zip(GB, GE, GR):
        ctr = x[b] + P.rotate(e, q[b])
        surf = ctr - n * r
        pen = r - ctr[2]
        vel = v[b] + np.cross(w[b], (surf if V["vel_at"] == "surface" else ctr) - x[b])
        rel = (surf if V["lever"] == "surface" else ctr) - x[b]
        nv = vel @ n
        ang = n @ np.cross(np.cross(rel, n), rel)
        m = MASS[b]
        imp = (-nv + erp * pen) / (1 / m + ang)
        vd = vel - nv * n
        nd = np.linalg.norm(vd)
        impd = min(nd / (1 / m + ang), 1.0 * imp)
        dird = vd / (1e-6 + nd)
        apn = 1.0 if (pen > 0 and nv < 0 and imp > 0) else 0.0
        apd = apn * (1.0 if nd > 0.01 else 0.0)
        Pn = imp * n * apn; Pd = -impd * dird * apd
        dv[b] += (Pn + Pd) / m
        dw[b] += np.cross(rel, Pn + Pd)
    return dv, dw


def actions(T):
    rng = P.np_prngkey(0)
    out = []
    for _ in range(T):
        rng, rng1 = P.np_split(rng, 2)
        out.append(P.f32(P.np_uniform(rng1, (8,), -1, 1)))
    return out


def run(V, T=3):
    x, q = POS[0].copy(), ROT[0].copy()
    v = np.zeros((9, 3)); w = np.zeros((9, 3))
    errs = []
    for t, a in enumerate(actions(T)):
        x, q, v, w = step(x, q, v, w, a, V)
        errs.append(np.abs(x - POS[t + 1]).max())
    return errs


if __name__ == "__main__":
    for order, vel_at, lever in itertools.product(["kin_first", "kin_last"], ["surface", "center"], ["surface", "center"]):
        V = dict(order=order, vel_at=vel_at, lever=lever)
        print(V, " ".join(f"{e:.2e}" for e in run(V)))


def detail(V):
    x, q = POS[0].copy(), ROT[0].copy()
    v = np.zeros((9, 3)); w = np.zeros((9, 3))
    a = actions(1)[0]
    x1, q1, v1, w1 = step(x, q, v, w, a, V)
    np.set_printoptions(precision=5, suppress=True, linewidth=150)
    print("act", a)
    print("dx model - frame1 (x1e3):\n", (x1 - POS[1]) * 1e3)
    print("model displacement (x1e3):\n", (x1 - POS[0]) * 1e3)
    print("frame displacement (x1e3):\n", (POS[1] - POS[0]) * 1e3)
    qd = np.sum(q1 * ROT[1], -1)
    print("rot err (1-|dot|):", 1 - np.abs(qd))

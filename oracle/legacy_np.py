"""NumPy (float64) restatement of brax v1 *legacy-spring* physics -- TEST INFRASTRUCTURE ONLY.

Pinned against the only physics artefact the reference holds: the 21-frame trajectory of
``notebooks/ant_tag.ipynb:449`` (cell ``ant_tag.ipynb:470-477``: un-jitted numpy-path reset,
then 20 jitted ``AntTagEnv.step`` calls; the embedded Config carries ``stiffness: 18000``,
``springDamping: 80``, ``baumgarteErp: 0.1`` and no ``dynamicsMode``, i.e. brax <= 0.0.12).
All 20 frames are reproduced to <= 1e-5 m / 1e-5 in the quaternions
(tests/test_oracle_golden.py::test_legacy_matches_notebook_frames), which pins:

* the reset's joint velocities: ``qvel = uniform(split(rng, 5)[2], (8,), -.1, .1)`` (the cell's
  ``rng2``) and brax ``System.default_qp``'s velocity semantics [ext]: a child body gets the
  angular velocity ``rotate(axis_j * qvel_j, parent.rot)`` of its own joint only (no
  accumulation down the tree) and zero linear velocity;
* the legacy substep [ext, brax System.step]: kinetic (x += v h; q += h/2 [0,w] q, normalise)
  -> joints + actuators as accelerations (v += (dv + g) h; w = e^{-0.05 h} w + dw h) ->
  one-way ground contacts as velocity impulses (Baumgarte, capped Coulomb drag);
* revolute joints: anchor spring ``k (p_p - p_c) + c (v_p - v_c)``, axis alignment
  ``k ap x ac``, limit spring ``-k ap dang`` outside ``angle_limit``, damping
  ``-20 (w_p - w_c)``;
* torque actuators: ``ap * act * 350``, and NO actuator torque while the joint is outside its
  angle limits (the frames 2..20 fit at 1e-6 m only with this gate; without it frame 2 is off by
  2.4 mm);
* capsule-plane contacts at the capsule's end sphere; the drag uses the normal's effective
  mass and is capped by friction * normal impulse, applied only when penetrating, approaching
  and the impulse is positive, and the tangential speed exceeds 0.01.
"""
from __future__ import annotations

import numpy as np

import pob_np as P

N_DYN = 9
J = P.ANT_JOINTS
PAR = np.array([j[0] for j in J])
CHI = np.array([j[1] for j in J])
OFFP = np.array([P.f32(j[2]) for j in J])
OFFC = np.array([P.f32(j[3]) for j in J])
_EQ = [P.euler_to_quat(P.f32(j[4])) for j in J]
AXIS = np.array([P.rotate(np.array([1.0, 0, 0]), q) for q in _EQ])   # hinge axis (joint frame x)
REF = np.array([P.rotate(np.array([0, 0, 1.0]), q) for q in _EQ])    # angle reference (joint frame z)
LIM = np.array([j[5] for j in J], float) * np.pi / 180
MASS = np.array([b[1] for b in P.ANT_BODIES])
GROUND_BODIES = (0, 2, 4, 6, 8)   # Torso and the four lower legs (collide_include x Ground)


def rot(v, q):
    """rotate batched vectors v (...,3) by wxyz quaternions q (...,4)."""
    s = q[..., :1]
    u = q[..., 1:]
    return 2 * np.sum(u * v, -1, keepdims=True) * u + (s * s - np.sum(u * u, -1, keepdims=True)) * v \
        + 2 * s * np.cross(u, v)


def qmul(u, v):
    w1, x1, y1, z1 = np.moveaxis(u, -1, 0)
    w2, x2, y2, z2 = np.moveaxis(v, -1, 0)
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], -1)


def joint_velocities(rot_bodies, qvel):
    """System.default_qp joint velocities [ext]: child ang = rotate(axis * qvel, parent rot)."""
    vel = np.zeros((N_DYN, 3))
    ang = np.zeros((N_DYN, 3))
    for j in range(len(J)):
        ang[CHI[j]] = P.rotate(AXIS[j], rot_bodies[PAR[j]]) * qvel[j]
    return vel, ang


def joint_angles(q):
    ap = rot(AXIS, q[PAR])
    fp, fc = rot(REF, q[PAR]), rot(REF, q[CHI])
    return np.arctan2(np.sum(np.cross(fp, fc) * ap, -1), np.sum(fp * fc, -1))


class LegacyAnt:
    """The Ant's 9 dynamic bodies on the ground plane (no wall contacts)."""

    def __init__(self, stiffness=18000.0, spring_damping=80.0, angular_damping=20.0, strength=350.0,
                 dt=0.05, substeps=10, baumgarte_erp=0.1, friction=1.0, elasticity=0.0, ang_damp=-0.05,
                 gravity=-9.8, gate_actuators=True):
        self.gate = gate_actuators  # False only for the tests' negative control
        self.k, self.c, self.ad, self.strength = stiffness, spring_damping, angular_damping, strength
        self.h = dt / substeps
        self.substeps = substeps
        self.erp = baumgarte_erp * substeps / dt
        self.mu, self.e = friction, elasticity
        self.ang_damp = ang_damp
        self.g = np.array([0.0, 0.0, gravity])
        self.ge = np.array([P.capsule_ends(i)[0][0] for i in GROUND_BODIES])
        self.gr = np.array([P.capsule_ends(i)[1] for i in GROUND_BODIES])

    def joints(self, x, q, v, w, act):
        p, c = PAR, CHI
        rp, rc = rot(OFFP, q[p]), rot(OFFC, q[c])
        imp = self.k * ((x[p] + rp) - (x[c] + rc)) + self.c * ((v[p] + np.cross(w[p], rp)) - (v[c] + np.cross(w[c], rc)))
        ap, ac = rot(AXIS, q[p]), rot(AXIS, q[c])
        psi = joint_angles(q)
        dang = np.where(psi < LIM[:, 0], LIM[:, 0] - psi, 0.0)
        dang = np.where(psi > LIM[:, 1], LIM[:, 1] - psi, dang)
        tq = self.k * np.cross(ap, ac) - self.k * ap * dang[:, None] - self.ad * (w[p] - w[c])
        ta = ap * (np.where((dang != 0.0) & self.gate, 0.0, act) * self.strength)[:, None]
        dv = np.zeros((N_DYN, 3))
        dw = np.zeros((N_DYN, 3))
        for j in range(len(J)):
            dv[p[j]] -= imp[j] / MASS[p[j]]
            dv[c[j]] += imp[j] / MASS[c[j]]
            dw[p[j]] += np.cross(rp[j], -imp[j]) + tq[j] - ta[j]
            dw[c[j]] += np.cross(rc[j], imp[j]) - tq[j] + ta[j]
        return dv, dw

    def contacts(self, x, q, v, w):
        dv = np.zeros((N_DYN, 3))
        dw = np.zeros((N_DYN, 3))
        n = np.array([0.0, 0.0, 1.0])
        for b, e, r in zip(GROUND_BODIES, self.ge, self.gr):
            ctr = x[b] + P.rotate(e, q[b])
            rel = ctr - n * r - x[b]
            pen = r - ctr[2]
            cvel = v[b] + np.cross(w[b], rel)
            nv = cvel @ n
            ang = n @ np.cross(np.cross(rel, n), rel)
            m = MASS[b]
            impulse = (-(1.0 + self.e) * nv + self.erp * pen) / (1.0 / m + ang)
            vd = cvel - nv * n
            nd = np.linalg.norm(vd)
            imp_d = min(nd / (1.0 / m + ang), self.mu * impulse)
            apply_n = 1.0 if (pen > 0 and nv < 0 and impulse > 0) else 0.0
            apply_d = apply_n * (1.0 if nd > 0.01 else 0.0)
            Pt = impulse * n * apply_n - imp_d * vd / (1e-6 + nd) * apply_d
            dv[b] += Pt / m
            dw[b] += np.cross(rel, Pt)
        return dv, dw

    def step(self, x, q, v, w, act):
        """One control step; returns (x, q, v, w, Info.contact vel, ang)."""
        cv, cw = np.zeros_like(v), np.zeros_like(w)
        h = self.h
        for _ in range(self.substeps):
            x = x + v * h
            q = q + 0.5 * h * qmul(np.concatenate([np.zeros((len(w), 1)), w], -1), q)
            q = q / np.linalg.norm(q, axis=-1, keepdims=True)
            dv, dw = self.joints(x, q, v, w, act)
            v = v + (dv + self.g) * h
            w = np.exp(self.ang_damp * h) * w + dw * h
            dvc, dwc = self.contacts(x, q, v, w)
            v, w = v + dvc, w + dwc
            cv, cw = cv + dvc, cw + dwc
        return x, q, v, w, cv, cw


def notebook_rollout(frame0_pos, frame0_rot, T=20):
    """Replay ``ant_tag.ipynb:470-477`` from its recorded frame 0: qvel from the reset key's
    ``split(rng, 5)[2]``, actions ``uniform(split(rng)[1], (8,), -1, 1)`` per step (numpy path,
    float64 -> float32).  Returns the 9 ant bodies' (pos, rot) for frames 1..T."""
    key = P.np_prngkey(0)
    qvel = P.np_uniform(P.np_split(key, 5)[2], (8,), -0.1, 0.1)
    x, q = np.array(frame0_pos, float), np.array(frame0_rot, float)
    v, w = joint_velocities(q, qvel)
    ant = LegacyAnt()
    out = []
    rng = key
    for _ in range(T):
        rng, rng1 = P.np_split(rng, 2)
        act = P.f32(P.np_uniform(rng1, (8,), -1, 1))
        x, q, v, w, _, _ = ant.step(x, q, v, w, act)
        out.append((x.copy(), q.copy()))
    return out

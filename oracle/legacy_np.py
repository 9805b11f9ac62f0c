"""NumPy (float64) restatement of brax v1 *legacy* (spring / impulse) physics -- TEST
INFRASTRUCTURE ONLY.

Purpose: pin the physics against the only physics artefact the reference holds, the
21-frame trajectory of ``notebooks/ant_tag.ipynb:449`` (brax <= 0.0.12 legacy dynamics:
the embedded config carries ``stiffness: 18000``, ``springDamping: 80``,
``baumgarteErp: 0.1`` and no ``dynamicsMode``).  brax itself is not vendored (SURVEY.md
§8(c)); this is the recalled brax v1 System.step [ext]:

    per substep:  kinetic (x += v dt; q += dt/2 [0,w] q, normalise)
                  joints (springs: anchor stiffness + damping, axis alignment, angle limits,
                          angular damping) + torque actuators  -> potential (v, w += a dt)
                  colliders (one-way impulses, Baumgarte, friction) -> v, w += dv
    Info.contact = sum of the collider velocity updates
"""
from __future__ import annotations

import numpy as np

import pob_np as P

N_DYN = 9


def _rot(v, q):
    """rotate batched vectors v (...,3) by quaternions q (...,4)."""
    s = q[..., :1]
    u = q[..., 1:]
    t = np.sum(u * v, -1, keepdims=True)
    c = s * s - np.sum(u * u, -1, keepdims=True)
    return 2 * t * u + c * v + 2 * s * np.cross(u, v)


def _qmul(u, v):
    w1, x1, y1, z1 = np.moveaxis(u, -1, 0)
    w2, x2, y2, z2 = np.moveaxis(v, -1, 0)
    return np.stack([w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
                     w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
                     w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2,
                     w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2], -1)


class LegacyAnt:
    """Ant (9 dynamic bodies) on the ground plane; walls far away (no wall contacts)."""

    def __init__(self, stiffness=18000., spring_damping=80., angular_damping=20., limit_strength=None,
                 strength=350., dt=0.05, substeps=10, baumgarte_erp=0.1, friction=1.0, elasticity=0.0,
                 ang_damp=-0.05, gravity=-9.8, variant=None):
        self.v = dict(variant or {})
        self.k = stiffness
        self.c = spring_damping
        self.ad = angular_damping
        self.kl = stiffness if limit_strength is None else limit_strength
        self.strength = strength
        self.h = dt / substeps
        self.substeps = substeps
        self.erp = baumgarte_erp * substeps / dt
        self.mu = friction
        self.e = elasticity
        self.ang_damp = ang_damp
        self.g = np.array([0, 0, gravity])
        self.mass = np.array([b[1] for b in P.ANT_BODIES])
        J = P.ANT_JOINTS
        self.par = np.array([j[0] for j in J])
        self.chi = np.array([j[1] for j in J])
        self.offp = np.array([P.f32(j[2]) for j in J])
        self.offc = np.array([P.f32(j[3]) for j in J])
        q = [P.euler_to_quat(P.f32(j[4])) for j in J]
        self.axis = np.array([P.rotate(np.array([1., 0, 0]), qq) for qq in q])
        self.ref = np.array([P.rotate(np.array([0, 0, 1.]), qq) for qq in q])
        self.lim = np.array([j[5] for j in J], float) * np.pi / 180
        # ground contacts: torso (sphere) + 4 feet (end -1)
        self.gb, self.ge, self.gr = [], [], []
        for i in (0, 2, 4, 6, 8):
            ends, r = P.capsule_ends(i)
            self.gb.append(i)
            self.ge.append(ends[0])
            self.gr.append(r)
        self.gb = np.array(self.gb)
        self.ge = np.array(self.ge)
        self.gr = np.array(self.gr)

    def angle_vel(self, x, q, v, w):
        qp, qc = q[self.par], q[self.chi]
        ap = _rot(self.axis, qp)
        fp, fc = _rot(self.ref, qp), _rot(self.ref, qc)
        psi = np.arctan2(np.sum(np.cross(fp, fc) * ap, -1), np.sum(fp * fc, -1))
        dpsi = np.sum((w[self.chi] - w[self.par]) * ap, -1)
        return psi, dpsi

    def joints(self, x, q, v, w, act):
        V = self.v
        nb = x.shape[0]
        dv = np.zeros((nb, 3))
        dw = np.zeros((nb, 3))
        p, c = self.par, self.chi
        rp, rc = _rot(self.offp, q[p]), _rot(self.offc, q[c])
        pos_p, pos_c = x[p] + rp, x[c] + rc
        vel_p = v[p] + (0 if V.get("lin_only") else np.cross(w[p], rp))
        vel_c = v[c] + (0 if V.get("lin_only") else np.cross(w[c], rc))
        imp = (pos_p - pos_c) * self.k + self.c * (vel_p - vel_c)
        dvp = -imp / self.mass[p][:, None]
        dvc = imp / self.mass[c][:, None]
        dap = np.cross(rp, -imp)
        dac = np.cross(rc, imp)
        ap = _rot(self.axis, q[p])
        ac = _rot(self.axis, q[c])
        torque = self.k * np.cross(ap, ac) * V.get("align_sign", 1.0)
        psi, _ = self.angle_vel(x, q, v, w)
        lo, hi = self.lim[:, 0], self.lim[:, 1]
        dang = np.where(psi < lo, lo - psi, 0.0)
        dang = np.where(psi > hi, hi - psi, dang)
        torque = torque - self.kl * (ac if V.get("limit_child") else ap) * dang[:, None] * V.get("limit_sign", 1.0)
        torque = torque - self.ad * (w[p] - w[c])
        dap = dap + torque
        dac = dac - torque
        # torque actuators: act * strength about the parent's axis
        ta = (ac if V.get("act_child") else ap) * (act * self.strength)[:, None] * V.get("act_sign", 1.0)
        dap_a = -ta
        dac_a = ta
        for j in range(len(p)):
            dv[p[j]] += dvp[j]; dv[c[j]] += dvc[j]
            dw[p[j]] += dap[j] + dap_a[j]; dw[c[j]] += dac[j] + dac_a[j]
        return dv, dw

    def contacts(self, x, q, v, w):
        nb = x.shape[0]
        dv = np.zeros((nb, 3))
        dw = np.zeros((nb, 3))
        n = np.array([0, 0, 1.0])
        for b, e, r in zip(self.gb, self.ge, self.gr):
            pe = x[b] + P.rotate(e, q[b])
            pos = pe - n * r
            pen = r - pe[2]
            rel = pos - x[b]
            cvel = v[b] + np.cross(w[b], rel)
            nv = np.dot(n, cvel)
            t1 = np.cross(rel, n)
            ang = np.dot(n, np.cross(t1, rel))
            m = self.mass[b]
            impulse = (-(1 + self.e) * nv + self.erp * pen) / (1 / m + ang)
            vd = cvel - nv * n
            nd = np.linalg.norm(vd)
            imp_d = nd / (1 / m + ang)
            imp_d = min(imp_d, self.mu * impulse)
            dird = vd / (1e-6 + nd)
            if self.v.get("no_nv_cond"):
                apply_n = 1.0 if (pen > 0 and impulse > 0) else 0.0
            else:
                apply_n = 1.0 if (pen > 0 and nv < 0 and impulse > 0) else 0.0
            apply_d = apply_n * (1.0 if nd > self.v.get("drag_thresh", 0.01) else 0.0)
            if self.v.get("no_friction"):
                apply_d = 0.0
            Pn = impulse * n * apply_n
            Pd = -imp_d * dird * apply_d
            dv[b] += (Pn + Pd) / m
            dw[b] += np.cross(rel, Pn) + np.cross(rel, Pd)
        return dv, dw

    def step(self, x, q, v, w, act):
        x, q, v, w = x.copy(), q.copy(), v.copy(), w.copy()
        cv = np.zeros_like(v)
        cw = np.zeros_like(w)
        h = self.h
        V = self.v
        for _ in range(self.substeps):
            if V.get("kinetic_last"):
                dv, dw = self.joints(x, q, v, w, act)
                v = v + (dv + self.g) * h
                w = np.exp(self.ang_damp * h) * w + dw * h
                dvc, dwc = self.contacts(x, q, v, w)
                v = v + dvc; w = w + dwc; cv += dvc; cw += dwc
                x = x + v * h
                dq = _qmul(np.concatenate([np.zeros((len(w), 1)), w], -1), q)
                q = q + 0.5 * h * dq
                q = q / np.linalg.norm(q, axis=-1, keepdims=True)
                continue
            # kinetic
            x = x + v * h
            wq = np.concatenate([np.zeros((len(w), 1)), w], -1)
            dq = _qmul(q, wq) if V.get("qdot_right") else _qmul(wq, q)
            q = q + 0.5 * h * dq
            q = q / np.linalg.norm(q, axis=-1, keepdims=True)
            # potential: joints + actuators
            dv, dw = self.joints(x, q, v, w, act)
            v = np.exp(0.0 * h) * v + (dv + self.g) * h
            w = np.exp(self.ang_damp * h) * w + dw * h
            # collisions
            dvc, dwc = self.contacts(x, q, v, w)
            v = v + dvc
            w = w + dwc
            cv += dvc
            cw += dwc
        return x, q, v, w, cv, cw

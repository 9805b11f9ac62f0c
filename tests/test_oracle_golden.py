"""CPU tests: pin the oracle (numpy + C restatement) against the reference's golden data.

* threefry: public jax KATs split(PRNGKey(0)), split(PRNGKey(42));
* kinematics: frame 0 of the trajectory embedded in notebooks/ant_tag.ipynb:449
  (tests/golden/ant_tag_notebook_trajectory.json) -- the un-jitted numpy-path reset of the
  notebook cell ant_tag.ipynb:470-477;
* construction tables: wall boxes of draw_t_maze / draw_arena (envs/utils.py:6-119), the
  AntGather object grid (ant_gather.py:85-91);
* reset invariants of the three envs (ant_*.py reset / sample_init_qp);
* legacy-spring physics: frames 1..20 of the same trajectory (the cell's 20 jitted steps) by
  the float64 restatement oracle/legacy_np.py, which also pins brax default_qp's joint-velocity
  semantics and the torque actuators' limit gate.
The PBD physics step itself stays parity-unpinned against brax (no artefact records it).
"""
import json
import os

import numpy as np
import pytest

import orc
import pob_np as P

HERE = os.path.dirname(os.path.abspath(__file__))
KAT = json.load(open(os.path.join(HERE, "golden", "threefry_kat.json")))
TRAJ = json.load(open(os.path.join(HERE, "golden", "ant_tag_notebook_trajectory.json")))


def test_threefry_public_kats_numpy():
    assert P.split(P.prngkey(0)).tolist() == KAT["public"]["split_PRNGKey0"]
    assert P.split(P.prngkey(42)).tolist() == KAT["public"]["split_PRNGKey42"]


def test_threefry_public_kats_c_oracle():
    assert orc.split(P.prngkey(0), 2).tolist() == KAT["public"]["split_PRNGKey0"]
    assert orc.split(P.prngkey(42), 2).tolist() == KAT["public"]["split_PRNGKey42"]


def test_threefry_restated_vectors_c_vs_numpy():
    r = KAT["restated"]
    assert orc.split(P.prngkey(0), 5).tolist() == r["split_PRNGKey0_5"]
    assert orc.split(P.prngkey(7), 65).tolist() == r["split_PRNGKey7_65"]
    lib = orc.lib()
    import ctypes as C
    for key, n, lo, hi, name in ((0, 8, -0.1, 0.1, "uniform_PRNGKey0_8"), (3, 7, -1.0, 1.0, "uniform_PRNGKey3_7")):
        k = P.prngkey(key)
        out = np.zeros(n, np.float32)
        l, h = np.array([lo], np.float32), np.array([hi], np.float32)
        lib.orc_uniform(k.ctypes.data_as(orc._UP), n, orc._p(l), orc._p(h), 1, orc._p(out))
        np.testing.assert_array_equal(out, np.array(r[name], np.float32))
    k = P.prngkey(0)
    assert lib.orc_randint(k.ctypes.data_as(orc._UP), 0, 4) == r["randint4_PRNGKey0"]
    idx = np.zeros(16, np.int32)
    lib.orc_choice_idx(k.ctypes.data_as(orc._UP), 156, 16, idx.ctypes.data_as(C.POINTER(C.c_int)))
    assert idx.tolist() == r["choice_idx_PRNGKey0_156_16"]


def _notebook_frame0_qpos():
    key = P.np_prngkey(0)
    ks = P.np_split(key, 2)
    ant_xy = P.np_uniform(ks[1], (2,), -4.5, 4.5)
    qpos = P.default_angle() + P.np_uniform(ks[1], (8,), -.1, .1)
    return ant_xy, qpos


def test_notebook_frame0_numpy_fk():
    """notebooks/ant_tag.ipynb:449 frame 0 = default_qp(numpy-path qpos) + ant_xy."""
    ant_xy, qpos = _notebook_frame0_qpos()
    pos, rot, _, _ = P.default_qp(qpos)
    pos[:, :2] += ant_xy
    np.testing.assert_allclose(pos, np.array(TRAJ["pos"][0])[:9], atol=1e-12, rtol=0)
    np.testing.assert_allclose(rot, np.array(TRAJ["rot"][0])[:9], atol=1e-12, rtol=0)


def test_notebook_frame0_c_oracle_fk_f32():
    """The float32 C restatement of default_qp reproduces frame 0 to float32 accuracy."""
    ant_xy, qpos = _notebook_frame0_qpos()
    e = orc.OracleEnv("ant_tag")
    pos, rot, _, _ = e.default_qp(qpos.astype(np.float32), np.zeros(8, np.float32))
    pos = pos.astype(np.float64)
    pos[:9, :2] += ant_xy
    np.testing.assert_allclose(pos[:9], np.array(TRAJ["pos"][0])[:9], atol=3e-6, rtol=0)
    np.testing.assert_allclose(rot[:9], np.array(TRAJ["rot"][0])[:9], atol=3e-6, rtol=0)


def _traj_frames():
    return np.array(TRAJ["pos"])[:, :9], np.array(TRAJ["rot"])[:, :9]


def _qerr(q, ref):
    s = np.sign(np.sum(q * ref, -1))[:, None]  # q and -q are the same rotation
    return np.abs(q * s - ref).max()


def test_legacy_matches_notebook_frames():
    """notebooks/ant_tag.ipynb:470-477 frames 1..20 (legacy-spring brax, jitted float32) by the
    float64 restatement: <= 1e-6 m at frame 1, <= 2e-5 over all 20 frames (float32 drift)."""
    import legacy_np as LG
    pos, rot = _traj_frames()
    out = LG.notebook_rollout(pos[0], rot[0], 20)
    for t, (x, q) in enumerate(out, start=1):
        tol = 2e-6 if t == 1 else 2e-5
        assert np.abs(x - pos[t]).max() <= tol, (t, np.abs(x - pos[t]).max())
        assert _qerr(q, rot[t]) <= tol, (t, _qerr(q, rot[t]))


def test_legacy_pins_have_teeth():
    """Negative controls: the alternatives the fixture rejects (each off by >= 0.5 mm)."""
    import legacy_np as LG
    pos, rot = _traj_frames()
    key = P.np_prngkey(0)
    acts = []
    rng = key
    for _ in range(2):
        rng, r1 = P.np_split(rng, 2)
        acts.append(P.f32(P.np_uniform(r1, (8,), -1, 1)))
    qvel = P.np_uniform(P.np_split(key, 5)[2], (8,), -0.1, 0.1)
    ant = LG.LegacyAnt()
    # (a) joint velocities accumulated down the tree, with the bodies' linear velocities
    v_acc, w_acc = np.zeros((9, 3)), np.zeros((9, 3))
    for j in range(8):
        p, c = LG.PAR[j], LG.CHI[j]
        w_acc[c] = w_acc[p] + P.rotate(LG.AXIS[j], rot[0][p]) * qvel[j]
        anchor = pos[0][p] + P.rotate(LG.OFFP[j], rot[0][p])
        v_acc[c] = v_acc[p] + np.cross(w_acc[p], anchor - pos[0][p]) + np.cross(w_acc[c], pos[0][c] - anchor)
    assert np.abs(ant.step(pos[0], rot[0], v_acc, w_acc, acts[0])[0] - pos[1]).max() > 5e-4
    # the pinned form (= pob_np.default_qp's velocities)
    v0, w0 = LG.joint_velocities(rot[0], qvel)
    _, _, v_np, w_np = P.default_qp(LG.joint_angles(rot[0]), qvel)
    np.testing.assert_allclose(w_np, w0, atol=1e-12)
    assert not v_np.any()
    x, q, v, w, _, _ = ant.step(pos[0], rot[0], v0, w0, acts[0])
    assert np.abs(x - pos[1]).max() <= 2e-6
    assert np.abs(ant.step(x, q, v, w, acts[1])[0] - pos[2]).max() <= 2e-6
    # (b) torque actuators not gated at the joint limits: frame 2 off by mm
    ungated = LG.LegacyAnt(gate_actuators=False)
    assert np.abs(ungated.step(x, q, v, w, acts[1])[0] - pos[2]).max() > 5e-4


def notebook_legacy_state(env, pos0, rot0):
    """TAG state (B = 1) at the notebook's frame 0: the 9 ant rows from the recorded frame,
    joint velocities from the reset key's split(rng, 5)[2] (oracle/legacy_np.py)."""
    import legacy_np as LG
    s = env.empty(1)
    s["rot"][0, :, 0] = 1.0
    s["pos"][0, :9] = pos0
    s["rot"][0, :9] = rot0
    qvel = P.np_uniform(P.np_split(P.np_prngkey(0), 5)[2], (8,), -0.1, 0.1)
    _, w = LG.joint_velocities(np.asarray(rot0, float), qvel)
    s["ang"][0, :9] = w
    s["pos"][0, 10] = (3.0, 3.0, 0.5)   # the target, out of the way (it never collides)
    s["pos"][0, 11] = (0.0, 0.0, 0.5)   # the arena body
    return s


def notebook_actions(T):
    rng = P.np_prngkey(0)
    out = []
    for _ in range(T):
        rng, r1 = P.np_split(rng, 2)
        out.append(P.np_uniform(r1, (8,), -1, 1).astype(np.float32))
    return out


def test_c_oracle_legacy_matches_notebook_frames():
    """The float32 C restatement in legacy-spring mode (orc legacy_spring=1) reproduces the
    notebook's 20 frames.  AntTag with cage 5.5 puts the box walls' inner faces at +-6.5 like
    the notebook's capsule walls (no wall contact either way)."""
    pos, rot = _traj_frames()
    e = orc.OracleEnv("ant_tag", legacy_spring=1, tag_cage_xy=(5.5, 5.5))
    s = notebook_legacy_state(e, pos[0].astype(np.float32), rot[0].astype(np.float32))
    worst = 0.0
    for t, a in enumerate(notebook_actions(20), start=1):
        s = e.step(s, a[None], flags=0)
        dx = np.abs(s["pos"][0, :9] - pos[t]).max()
        dq = _qerr(s["rot"][0, :9].astype(np.float64), rot[t])
        worst = max(worst, dx, dq)
        assert dx <= 2e-5 and dq <= 2e-5, (t, dx, dq)
    assert worst > 0.0


def test_notebook_config_matches_restated_ant():
    cfg = TRAJ["config"]
    bodies = {b["name"]: b for b in cfg["bodies"]}
    for name, mass, r, length, end, rot in P.ANT_BODIES:
        b = bodies[name]
        assert b["mass"] == mass
        cap = b["colliders"][0]["capsule"]
        assert np.float32(cap["radius"]) == np.float32(r) and np.float32(cap["length"]) == np.float32(length)
        assert cap.get("end", 0) == end
    for j, (p, c, offp, offc, erot, lim) in zip(cfg["joints"], P.ANT_JOINTS):
        assert [j["parentOffset"][k] for k in "xyz"] == pytest.approx(offp)
        assert [j["childOffset"][k] for k in "xyz"] == pytest.approx(offc)
        assert [j["rotation"].get(k, 0.0) for k in "xyz"] == pytest.approx(erot)
        assert (j["angleLimit"][0]["min"], j["angleLimit"][0]["max"]) == lim
    assert cfg["dt"] == pytest.approx(0.05) and cfg["substeps"] == 10
    assert cfg["gravity"]["z"] == pytest.approx(-9.8)
    assert all(a["strength"] == 350.0 for a in cfg["actuators"])


def test_gather_grid_156():
    g = []
    for y in range(-6, 7):
        for x in range(-6, 7):
            if np.hypot(x, y) > 2:
                g.append((x, y))
    assert len(g) == 156 and g[0] == (-6, -6) and g[-1] == (6, 6)


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_oracle_reset_invariants(name):
    B = 128
    keys = P.split(P.prngkey(0), B + 1)[1:]
    e = orc.OracleEnv(name)
    s = e.reset(keys)
    assert s["obs"].shape == (B, {"ant_heavenhell": 114, "ant_gather": 211, "ant_tag": 103}[name])
    assert np.isfinite(s["obs"]).all()
    # obs joint angles (angle_vel, a3) recover the sampled joint angles qpos
    da = P.default_angle()
    for b in range(4):
        ks = P.split(keys[b], 5 if name != "ant_gather" else 4)
        noise = P.uniform(ks[1], (8,), -0.1, 0.1)
        qpos = (da.astype(np.float32) + noise).astype(np.float32)
        np.testing.assert_allclose(s["obs"][b, 7:15], qpos, atol=2e-5)
        qvel = P.uniform(ks[2], (8,), -0.1, 0.1)
        np.testing.assert_allclose(s["obs"][b, 21:29], qvel, atol=2e-5)
    # the ant rests on the ground: lowest collider point at z = 0
    assert (s["pos"][:, 0, 2] > 0.25).all()
    if name == "ant_heavenhell":
        tgt, hell = s["pos"][:, 11], s["pos"][:, 12]
        assert set(np.unique(tgt[:, 0])) <= {-5.25, 5.25}
        np.testing.assert_array_equal(tgt[:, 0], -hell[:, 0])
        np.testing.assert_array_equal(s["pos"][:, 10], np.tile([0, 7, 1], (B, 1)))
        # rng3 reuse: the goal swap is the stable argsort of bits(split(rng3)[1], 2)
        for b in range(8):
            r3 = P.split(keys[b], 5)[3]
            first = P.permutation_indices(r3, 2)[0]
            assert tgt[b, 0] == (-5.25 if first == 0 else 5.25)
        np.testing.assert_array_equal(s["rng"], np.stack([P.split(k, 5)[0] for k in keys]))
    elif name == "ant_gather":
        objs = s["pos"][:, 11:27]
        assert (objs[:, :8, 2] == 1).all() and (objs[:, 8:, 2] == 0).all()
        for b in range(B):
            xy = {tuple(v) for v in objs[b, :, :2]}
            assert len(xy) == 16 and all(np.hypot(*v) > 2 for v in xy)
        for b in range(4):
            r3 = P.split(keys[b], 4)[3]
            idx = P.permutation_indices(r3, 156)[:16]
            grid = np.array([(x, y) for y in range(-6, 7) for x in range(-6, 7) if np.hypot(x, y) > 2])
            np.testing.assert_array_equal(objs[b, :, :2], grid[idx])
        np.testing.assert_array_equal(s["rng"], keys)  # ant_gather.py:106 keeps the input key
    else:
        d = np.hypot(*(s["pos"][:, 10, :2] - s["pos"][:, 0, :2]).T)
        assert (s["pos"][:, 10, 2] == 0.5).all()
        axy = np.stack([P.uniform(P.split(k, 5)[3], (2,), -4.5, 4.5) for k in keys])
        np.testing.assert_allclose(s["pos"][:, 9, :2], axy)  # Ground shifted by ant_xy (quirk 6)
        tgt = s["pos"][:, 10, :2]
        assert (np.hypot(*(tgt - axy).T) > 5).all()
        assert (np.abs(tgt) <= 4.5).all()
        del d


def test_oracle_wall_tables_hh():
    """draw_t_maze(6.25, 8, 2, .5) -> SURVEY App. A wall table (via contacts: the ant
    spawned against the bottom wall is pushed out; the maze is closed)."""
    e = orc.OracleEnv("ant_heavenhell")
    B = 64
    keys = P.split(P.prngkey(1), B + 1)[1:]
    s = e.reset(keys)
    for _ in range(50):
        s = e.step(s, np.zeros((B, 8), np.float32), nthreads=4)
    x, y = s["pos"][:, 0, 0], s["pos"][:, 0, 1]
    assert (y > -0.05).all() and (np.abs(x) < 2.0).all()  # inside the corridor, above the wall


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_oracle_rollout_stable(name):
    B = 64
    e = orc.OracleEnv(name)
    s = e.reset(P.split(P.prngkey(3), B + 1)[1:], first=True)
    rng = np.random.default_rng(0)
    for _ in range(60):
        s = e.step(s, rng.uniform(-1, 1, (B, 8)).astype(np.float32), flags=orc.F_EPISODE | orc.F_AUTORESET,
                   episode_length=1000, nthreads=4, inplace=True)
    assert np.isfinite(s["obs"]).all() and np.isfinite(s["pos"]).all()
    q = np.linalg.norm(s["rot"][:, :9], axis=-1)
    np.testing.assert_allclose(q, 1.0, atol=1e-5)

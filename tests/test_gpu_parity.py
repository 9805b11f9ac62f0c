"""GPU parity: the HIP kernels (through libpob.so's C ABI) vs the CPU oracle.

Bar (BASELINE.json north star): bit-exact on integer / key / done / goal / pickup fields,
within 1e-5 relative on float qp state.  The engine and the oracle follow the same op
order with IEEE float32 arithmetic (both built with -ffp-contract=off, fixed-polynomial
transcendentals), so the float fields are asserted BIT-EXACT too (EXACT below); the
1e-5 tolerance is checked first so a failure reports its magnitude.
"""
import json
import os

import numpy as np
import pytest
import torch

import orc
import pob_np as P

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
NAMES = ["ant_heavenhell", "ant_gather", "ant_tag", "ant"]
RTOL, ATOL = 1e-5, 1e-6
EXACT = True  # measured: every float field of every step matches the oracle bit for bit


def _np(t):
    t = t.detach().cpu()
    if t.dtype == torch.bool:
        t = t.to(torch.float32)
    return t.numpy()


def close(a, b, what, rtol=RTOL, atol=ATOL):
    a = _np(a) if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    np.testing.assert_allclose(a.astype(np.float64), b.astype(np.float64), rtol=rtol, atol=atol, err_msg=what)
    exact = bool(np.array_equal(a.astype(np.float32), b.astype(np.float32)))
    if EXACT:
        np.testing.assert_array_equal(a.astype(np.float32), b.astype(np.float32), err_msg=f"{what} (bit-exact)")
    return exact


def _envs():
    from po_brax_amd import envs
    return envs


def _keys(B, seed=0):
    return P.split(P.prngkey(seed), B + 1)[1:]


def _state_np(s):
    """GPU State -> oracle state dict (reference layout)."""
    d = dict(pos=_np(s.qp.pos), rot=_np(s.qp.rot), vel=_np(s.qp.vel), ang=_np(s.qp.ang), obs=_np(s.obs),
             reward=_np(s.reward), done=_np(s.aux["done"]), rng=_np(s.aux["rng"]).astype(np.uint32))
    for k in range(3):
        d[f"m{k}"] = _np(s.aux[f"m{k}"])
    if "steps" in s.info:
        d["steps"] = _np(s.info["steps"])
        d["truncation"] = _np(s.aux["truncation"])
    else:
        d["steps"] = np.zeros_like(d["reward"]); d["truncation"] = np.zeros_like(d["reward"])
    if "first_qp" in s.info:
        fq = s.info["first_qp"]
        d.update(first_pos=_np(fq.pos), first_rot=_np(fq.rot), first_vel=_np(fq.vel), first_ang=_np(fq.ang),
                 first_obs=_np(s.info["first_obs"]))
    return {k: np.ascontiguousarray(v) for k, v in d.items()}


def compare_states(g, o, what, exact_report=None):
    gs = _state_np(g)
    exact = True
    for k in ("pos", "rot", "vel", "ang", "obs", "reward", "m0", "m1", "m2", "steps", "truncation"):
        exact &= close(gs[k], o[k], f"{what}: {k}")
    np.testing.assert_array_equal(gs["done"], o["done"], err_msg=f"{what}: done")
    np.testing.assert_array_equal(gs["rng"], o["rng"], err_msg=f"{what}: rng")
    if exact_report is not None:
        exact_report.append((what, exact))
    return exact


# ------------------------------------------------------------------------ RNG kernels
def test_threefry_kernels_match_kats():
    from po_brax_amd import jumpy
    kat = json.load(open(os.path.join(HERE, "golden", "threefry_kat.json")))
    assert _np(jumpy.random_split(jumpy.random_prngkey(0))).tolist() == kat["public"]["split_PRNGKey0"]
    assert _np(jumpy.random_split(jumpy.random_prngkey(42))).tolist() == kat["public"]["split_PRNGKey42"]
    assert _np(jumpy.random_split(jumpy.random_prngkey(7), 65)).tolist() == kat["restated"]["split_PRNGKey7_65"]
    u = jumpy.random_uniform(jumpy.random_prngkey(0), (8,), -0.1, 0.1)
    np.testing.assert_array_equal(_np(u), np.array(kat["restated"]["uniform_PRNGKey0_8"], np.float32))
    u = jumpy.random_uniform(jumpy.random_prngkey(3), (7,), -1.0, 1.0)
    np.testing.assert_array_equal(_np(u), np.array(kat["restated"]["uniform_PRNGKey3_7"], np.float32))


def test_sharded_actions_and_keys():
    from po_brax_amd import jumpy
    from po_brax_amd.sharding import shard_keys, shard_range
    total, world = 1000, 3
    key = jumpy.random_prngkey(5)
    full = P.split(P.prngkey(5), total + 1)[1:]
    for r in range(world):
        lo, hi = shard_range(total, world, r)
        np.testing.assert_array_equal(_np(shard_keys(key, total, world, r)), full[lo:hi])
    k = jumpy.random_prngkey(11)
    kn = P.prngkey(11)
    for step in range(3):
        kn, sub = P.split(kn)
        ref = P.uniform(sub, (total, 8), -1, 1)
        for r in range(world):
            lo, hi = shard_range(total, world, r)
            kk = k.clone()
            act = torch.empty((hi - lo, 8), dtype=torch.float32, device="cuda")
            jumpy.random_actions_(kk, total, lo, act)
            np.testing.assert_array_equal(_np(act), ref[lo:hi])
        jumpy.random_actions_(k, total, 0, torch.empty((total, 8), device="cuda"))
        np.testing.assert_array_equal(_np(k), kn)


# -------------------------------------------------------------------------- kinematics
def test_default_qp_reproduces_notebook_frame0():
    traj = json.load(open(os.path.join(HERE, "golden", "ant_tag_notebook_trajectory.json")))
    ks = P.np_split(P.np_prngkey(0), 2)
    ant_xy = P.np_uniform(ks[1], (2,), -4.5, 4.5)
    qpos = (P.default_angle() + P.np_uniform(ks[1], (8,), -.1, .1)).astype(np.float32)
    env = _envs().AntTagEnv()
    qp = env.sys.default_qp(torch.from_numpy(qpos), torch.zeros(8))
    pos = _np(qp.pos).astype(np.float64)
    pos[:9, :2] += ant_xy
    np.testing.assert_allclose(pos[:9], np.array(traj["pos"][0])[:9], atol=3e-6, rtol=0)
    np.testing.assert_allclose(_np(qp.rot)[:9], np.array(traj["rot"][0])[:9], atol=3e-6, rtol=0)
    o = orc.OracleEnv("ant_tag")
    opos, orot, ovel, oang = o.default_qp(qpos, np.zeros(8, np.float32))
    np.testing.assert_array_equal(_np(qp.pos), opos)
    np.testing.assert_array_equal(_np(qp.rot), orot)


# ------------------------------------------------------------------------------ reset
@pytest.mark.parametrize("name", NAMES)
def test_reset_parity(name):
    B = 512
    keys = _keys(B)
    env = _envs().create(name, batch_size=B)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name).reset(keys, first=True)
    compare_states(s, o, f"{name} reset")
    fq = s.info["first_qp"]
    np.testing.assert_array_equal(_np(fq.pos), _np(s.qp.pos))


# ------------------------------------------------------------------------------- step
@pytest.mark.parametrize("name", NAMES)
def test_step_parity_per_step(name):
    """30 steps; every step the oracle restarts from the GPU's state (one-step parity)."""
    B, T = 256, 30
    envs = _envs()
    env = envs.create(name, batch_size=B, episode_length=20)
    s = env.reset(torch.from_numpy(_keys(B, 1)).cuda())
    o = orc.OracleEnv(name)
    rng = np.random.default_rng(0)
    report = []
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=20)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} step {t}", report)
    n_exact = sum(e for _, e in report)
    print(f"{name}: {n_exact}/{len(report)} steps bit-exact on every float field")


@pytest.mark.parametrize("name", NAMES)
def test_trajectory_parity_free_running(name):
    """Both engines run 25 steps independently from the same reset (stronger than per-step:
    any float divergence would compound through the contact dynamics)."""
    B, T = 128, 25
    env = _envs().create(name, batch_size=B, episode_length=1000)
    keys = _keys(B, 2)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    so = o.reset(keys, first=True)
    rng = np.random.default_rng(4)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        s = env.step_(s, torch.from_numpy(act).cuda())
        so = o.step(so, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=1000, inplace=True)
    compare_states(s, so, f"{name} free-running t={T}")


def test_functional_and_inplace_agree():
    B = 128
    env = _envs().create("ant_heavenhell", batch_size=B)
    keys = torch.from_numpy(_keys(B)).cuda()
    s1 = env.reset(keys)
    s2 = env.reset(keys)
    act = torch.rand((B, 8), device="cuda") * 2 - 1
    a = env.step(s1, act)
    pos_before = s1.qp.pos.clone()
    b = env.step_(s2, act)
    assert torch.equal(a.qp.pos, b.qp.pos) and torch.equal(a.obs, b.obs)
    assert torch.equal(s1.qp.pos, pos_before)  # functional step leaves its input intact


# ------------------------------------------------------------------------- autoreset
@pytest.mark.parametrize("name", NAMES)
def test_gym_autoreset_parity(name):
    """AutoresetVmapGymWrapper (wrappers.py:240-262) with the device-side any(done)."""
    B, T = 96, 25
    envs = _envs()
    g = envs.create_gym_env(name, batch_size=B, seed=3, episode_length=7)
    obs = g.reset()
    o = orc.OracleEnv(name)
    key = P.prngkey(3)
    ks = P.split(key, B + 1)
    so, gkey = o.reset(ks[1:]), ks[0].copy()
    np.testing.assert_array_equal(_np(obs), so["obs"])
    rng = np.random.default_rng(1)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        obs, rew, done, info = g.step(torch.from_numpy(act).cuda())
        so = o.step(so, act, flags=orc.F_EPISODE, episode_length=7, inplace=True)
        np.testing.assert_array_equal(_np(done), so["done"], err_msg=f"t={t}")
        o.gym_autoreset(so, gkey)
        close(obs, so["obs"], f"{name} gym obs t={t}")
        close(g._state.qp.pos, so["pos"], f"{name} gym pos t={t}")
        np.testing.assert_array_equal(_np(g._key), gkey, err_msg=f"gym key t={t}")
        np.testing.assert_array_equal(_np(g._state.info["steps"]), so["steps"])


def test_randomized_autoreset_naive():
    """RandomizedAutoResetWrapperNaive (wrappers.py:30-52): reset(info.rng) where done."""
    B = 64
    envs = _envs()
    name = "ant_tag"
    env = envs.wrappers.RandomizedAutoResetWrapperNaive(envs.create(name, batch_size=B, auto_reset=False,
                                                                    episode_length=5))
    s = env.reset(torch.from_numpy(_keys(B)).cuda())
    o = orc.OracleEnv(name)
    rng = np.random.default_rng(2)
    for t in range(8):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        prev = _state_np(s)
        if t > 0:
            prev["steps"] = np.where(prev["done"] != 0, 0, prev["steps"]).astype(np.float32)
        so = o.step(prev, act, flags=orc.F_EPISODE, episode_length=5)
        s = env.step(s, torch.from_numpy(act).cuda())
        # reset the done envs from their (post-step) info['rng']
        done = so["done"] != 0
        if done.any():
            fresh = o.reset(so["rng"][done])
            for k in ("pos", "rot", "vel", "ang", "obs"):
                so[k][done] = fresh[k]
        close(s.qp.pos, so["pos"], f"naive pos t={t}")
        close(s.obs, so["obs"], f"naive obs t={t}")


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("mode", ["own", "gym"])
def test_sparse_masked_reset_rows(name, mode):
    """Masked resets with a handful of done envs per wave (the gym step's usual case: rows
    written straight from the quad's registers) next to a wave whose 16 envs are all done
    (rows staged in LDS), B = 1 000 (ragged last wave).  Done rows equal the oracle's reset
    -- from the env's own info['rng'] (RandomizedAutoResetWrapperNaive, wrappers.py:30-52)
    or from split(gym_key, B + 1)[1 + b] (AutoresetVmapGymWrapper, wrappers.py:245-262) --
    and every other row, and every field the mode does not own, is untouched."""
    from po_brax_amd import _lib
    B = 1000
    envs = _envs()
    env = envs.create(name, batch_size=B, auto_reset=False, episode_length=1000)
    s = env.reset(torch.from_numpy(_keys(B, 21)).cuda())
    rng = np.random.default_rng(5)
    for _ in range(2):
        s = env.step_(s, torch.from_numpy(rng.uniform(-1, 1, (B, 8)).astype(np.float32)).cuda())
    done = np.zeros(B, np.float32)
    done[[3, 17, 18, 200, 515, 777, 998, 999]] = 1.0   # one or two per wave (direct rows)
    done[320:336] = 1.0                                  # a whole wave (staged rows)
    done[480:483] = 1.0                                  # three in one wave (direct rows)
    s.aux["done"].copy_(torch.from_numpy(done).cuda())
    before = _state_np(s)
    o = orc.OracleEnv(name)
    d = done != 0
    if mode == "own":
        env.unwrapped._reset_where_done(s, _lib.RESET_OWN)
        fresh = o.reset(before["rng"][d])
    else:
        gk = P.prngkey(9)
        gin = torch.from_numpy(gk.astype(np.uint32)).cuda()
        gout = torch.zeros(2, dtype=torch.uint32, device="cuda")
        words = torch.zeros(8, dtype=torch.uint32, device="cuda")
        words[0] = 1  # the step's any-done word: set
        s.aux["any_done"], s.aux["any_done_clear"] = words[0:4], words[4:8]
        env.unwrapped._reset_where_done(s, _lib.RESET_GYM, gin, gout, total=B, first=0)
        ks = P.split(gk, B + 1)
        fresh = o.reset(ks[1:][d])
        np.testing.assert_array_equal(_np(gout), ks[0], err_msg="advanced gym key")
        assert int(words[4]) == 0
    after = _state_np(s)
    for k in ("pos", "rot", "vel", "ang", "obs"):
        exp = before[k].copy()
        exp[d] = fresh[k]
        close(after[k], exp, f"{name} {mode} sparse masked reset {k}")
    exp_steps = np.where(d, 0.0, before["steps"]) if mode == "gym" else before["steps"]
    np.testing.assert_array_equal(after["steps"], exp_steps)
    for k in ("reward", "done", "m0", "m1", "m2", "truncation"):
        np.testing.assert_array_equal(after[k], before[k], err_msg=k)
    np.testing.assert_array_equal(after["rng"], before["rng"])


# ---------------------------------------------------------------------- misc surface
def test_obs_mask_gather():
    from po_brax_amd import standard_observability_masks as M
    obs = torch.randn((1000, 87), device="cuda")
    for idx in (M.POSITION["ant"], M.VELOCITY["ant"], M.CFRC["ant"]):
        got = M.apply_mask(obs, idx)
        assert torch.equal(got, obs[:, torch.as_tensor(idx, device="cuda")])
    o2 = torch.randn((64, 114), device="cuda")
    idx = M.po_env_mask("ant_heavenhell", cfrc=False)
    assert torch.equal(M.apply_mask(o2, idx), o2[:, torch.as_tensor(idx, device="cuda")])


def test_registry_errors():
    envs = _envs()
    with pytest.raises(KeyError):
        envs.create("no_such_env")
    with pytest.raises(ValueError):
        envs.create_gym_env("ant_heavenhell", batch_size=-1)
    with pytest.raises(NotImplementedError):
        envs.create("humanoid")


def test_unbatched_env_api():
    """Un-vmapped brax usage: reset(key (2,)) -> unbatched shapes; step works on them."""
    envs = _envs()
    env = envs.AntHeavenHellEnv()
    s = env.reset(torch.tensor([0, 0], dtype=torch.uint32))
    assert s.qp.pos.shape == (14, 3) and s.obs.shape == (114,) and s.reward.shape == ()
    s2 = env.step(s, torch.zeros(8))
    assert s2.obs.shape == (114,) and "hits" in s2.metrics
    o = orc.OracleEnv("ant_heavenhell")
    so = o.reset(np.zeros((1, 2), np.uint32))
    np.testing.assert_array_equal(_np(s.obs), so["obs"][0])


def test_large_batch_properties():
    """HH at the headline batch (65 536): finite, unit quaternions, done/reward logic."""
    B, T = 65536, 20
    env = _envs().create("ant_heavenhell", batch_size=B, episode_length=1000)
    from po_brax_amd import jumpy
    key = jumpy.random_prngkey(0)
    keys = jumpy.random_split(key, B + 1)[1:].contiguous()
    s = env.reset(keys)
    act = torch.empty((B, 8), device="cuda")
    for _ in range(T):
        jumpy.random_actions_(key, B, 0, act)
        s = env.step_(s, act)
    torch.cuda.synchronize()
    assert torch.isfinite(s.obs).all() and torch.isfinite(s.qp.pos).all()
    qn = s.qp.rot[:, :9].norm(dim=-1)
    assert torch.allclose(qn, torch.ones_like(qn), atol=1e-5)
    r, d = s.reward, s.done
    assert bool(((r != 0) <= (d != 0)).all())  # every non-zero reward ends the episode (HH)
    assert set(torch.unique(r).tolist()) <= {-2.0, -1.0, 0.0, 1.0}


# ------------------------------------------------------------------- wall contacts
def _walls(name):
    """(centre xy, z-rotation deg, half-extent xy) of the arena walls, from the brax config
    export (checked against SURVEY.md Appendix A in tests/test_export.py)."""
    import ctypes as C
    from po_brax_amd import _lib
    from po_brax_amd.io.config import brax_config_of
    p = _lib.pob_params()
    assert _lib.lib.pob_default_params(C.byref(p)) == 0
    arena = [b for b in brax_config_of(name, p)["bodies"] if b["name"] == "Arena"][0]
    return [((c["position"]["x"], c["position"]["y"]), c["rotation"]["z"],
             (c["box"]["halfsize"]["x"], c["box"]["halfsize"]["y"])) for c in arena["colliders"]]


def _near_wall(xy, walls, reach):
    """bool per point: within `reach` of some wall box (xy only)."""
    hit = np.zeros(len(xy), bool)
    for (cx, cy), rz, (hx, hy) in walls:
        a = np.deg2rad(rz)
        d = xy - np.array([cx, cy])
        lx = d[:, 0] * np.cos(a) + d[:, 1] * np.sin(a)
        ly = -d[:, 0] * np.sin(a) + d[:, 1] * np.cos(a)
        ex = np.maximum(np.abs(lx) - hx, 0)
        ey = np.maximum(np.abs(ly) - hy, 0)
        hit |= np.hypot(ex, ey) < reach
    return hit


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_step_parity_against_walls(name):
    """Ants teleported onto random points of the arena's bounding box (many start touching
    or inside a wall): every capsule x triangle branch (end points, edges, the segment crossing a
    face, several faces / walls per capsule,
    several walls per wave) runs; one-step parity for 8 steps."""
    B, T = 512, 8
    env = _envs().create(name, batch_size=B, episode_length=1000)
    s = env.reset(torch.from_numpy(_keys(B, 5)).cuda())
    walls = _walls(name)
    ext = np.array([[abs(c[0]) + max(h), abs(c[1]) + max(h)] for c, _, h in walls]).max(0)
    lo = np.array([-ext[0], min(c[1] - max(h) for c, _, h in walls)])
    hi = np.array([ext[0], max(c[1] + max(h) for c, _, h in walls)])
    rng = np.random.default_rng(7)
    cand = rng.uniform(lo, hi, (64 * B, 2))
    close_ = cand[_near_wall(cand, walls, 1.0)]
    xy = np.concatenate([close_[: 3 * B // 4], cand[: B - 3 * B // 4]]).astype(np.float32)
    xy = xy[rng.permutation(B)]
    torso = _np(s.qp.pos)[:, 0, :2]
    off = torch.from_numpy(xy - torso).cuda()
    s.qp.pos[:, :9, :2] += off[:, None, :]  # the 9 ant bodies
    near = _near_wall(xy.astype(np.float64), walls, 1.0)
    assert near.sum() >= 3 * B // 4, near.sum()
    o = orc.OracleEnv(name)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=1000)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} wall step {t}")


# ---------------------------------------------------------------------- ragged batches
@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("B", [1, 5, 17, 63])
def test_ragged_batch_parity(name, B):
    """Batches that leave a partial wave (16 envs / wave): the tail wave's staged loads and
    stores and its idle lanes must not touch other rows.  Short episodes so autoreset runs."""
    T = 12
    env = _envs().create(name, batch_size=B, episode_length=5)
    s = env.reset(torch.from_numpy(_keys(B, 11)).cuda())
    o = orc.OracleEnv(name)
    rng = np.random.default_rng(B)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=5)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} B={B} step {t}")


def test_batch_size_zero_follows_reference():
    """envs/__init__.py:64 (`if batch_size:`): create(batch_size=0) is the unbatched env;
    create_gym_env rejects batch_size <= 0 with ValueError (:115-117)."""
    envs = _envs()
    s = envs.create("ant_heavenhell", batch_size=0).reset(torch.tensor([0, 0], dtype=torch.uint32))
    assert s.obs.shape == (114,)
    with pytest.raises(ValueError):
        envs.create_gym_env("ant_heavenhell", batch_size=0)

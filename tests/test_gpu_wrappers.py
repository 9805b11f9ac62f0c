"""GPU parity of the wrapper semantics of po_brax/envs/wrappers.py that the fused kernels
fold in, each against the CPU oracle (bit-exact) or a NumPy restatement of the reference
code path:

* ActionRepeatWrapper(action_repeat=2)             wrappers.py:16-24
* RandomizedAutoResetWrapperCached                 wrappers.py:83-123
* AutoresetGymWrapper (unbatched gym env)          wrappers.py:232-237
* EvalGymWrapper queues r_q / dr_q / l_q + get_stats wrappers.py:175-229
* sharded AutoresetVmapGymWrapper (two shards of one batch on one GPU, any-done combined
  across the shards as the RCCL all-reduce does)    wrappers.py:240-262, sharding.py
* State edits between steps (state.replace(done=...)) are honoured by the engine
"""
import math

import numpy as np
import pytest
import torch

import orc
import pob_np as P
from test_gpu_parity import _keys, _np, _state_np, compare_states

pytestmark = pytest.mark.gpu
FLAGS = orc.F_EPISODE | orc.F_AUTORESET


def _envs():
    from po_brax_amd import envs
    return envs


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_tag", "ant_gather"])
def test_action_repeat_2(name):
    """create(..., action_repeat=2): dt 0.1, 20 substeps (wrappers.py:21-23)."""
    envs = _envs()
    B = 256
    env = envs.create(name, batch_size=B, action_repeat=2, episode_length=6)
    assert abs(env.sys.config.dt - 0.1) < 1e-12 and env.sys.config.substeps == 20
    keys = _keys(B, 4)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name, action_repeat=2)
    compare_states(s, o.reset(keys, first=True), f"{name} ar=2 reset")
    rng = np.random.default_rng(3)
    for t in range(8):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=FLAGS, episode_length=6)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} ar=2 step {t}")
    # and it differs from action_repeat=1 (the substeps really doubled)
    e1 = envs.create(name, batch_size=B, episode_length=6)
    s1 = e1.step(e1.reset(torch.from_numpy(keys).cuda()), torch.zeros((B, 8), device="cuda"))
    s2 = env.step(env.reset(torch.from_numpy(keys).cuda()), torch.zeros((B, 8), device="cuda"))
    assert not torch.equal(s1.qp.pos, s2.qp.pos)


def test_randomized_autoreset_cached():
    """Every n-th step: (rng, rng1) = split(info.rng); first_qp/first_obs <- reset(rng1);
    info.rng <- rng; then the AutoReset-style step against first_qp/first_obs."""
    envs = _envs()
    name, B, n, L = "ant_tag", 128, 3, 4
    env = envs.wrappers.RandomizedAutoResetWrapperCached(
        envs.create(name, batch_size=B, auto_reset=False, episode_length=L), n_steps_between_updates=n)
    keys = _keys(B, 6)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    so = o.reset(keys, first=True)
    compare_states(s, so, "cached reset")
    rng = np.random.default_rng(5)
    steps = 0
    for t in range(10):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        steps += 1
        if steps % n == 0:
            ks = np.stack([P.split(k, 2) for k in so["rng"]])  # (B, 2, 2)
            fresh = o.reset(np.ascontiguousarray(ks[:, 1]))
            for f in ("pos", "rot", "vel", "ang", "obs"):
                so["first_" + f] = fresh[f].copy()
            so["rng"] = np.ascontiguousarray(ks[:, 0])
        so = o.step(so, act, flags=FLAGS, episode_length=L)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"cached step {t}")
        np.testing.assert_array_equal(_np(s.info["first_obs"]), so["first_obs"], err_msg=f"first_obs {t}")


def test_autoreset_gym_wrapper_unbatched():
    """create_gym_env(batch_size=None): unbatched GymWrapper; on done, key1, key2 =
    split(key); reset(key2); key <- key1 (brax GymWrapper._reset) -- obs is the new obs."""
    envs = _envs()
    name, L = "ant_heavenhell", 3
    g = envs.create_gym_env(name, batch_size=None, seed=5, episode_length=L)
    obs = g.reset()
    o = orc.OracleEnv(name)
    k = P.split(P.prngkey(5), 2)
    so, key = o.reset(k[1:2]), k[0].copy()
    np.testing.assert_array_equal(_np(obs), so["obs"][0])
    rng = np.random.default_rng(2)
    resets = 0
    for t in range(8):
        act = rng.uniform(-1, 1, (8,)).astype(np.float32)
        obs, rew, done, info = g.step(torch.from_numpy(act).cuda())
        so = o.step(so, act[None], flags=orc.F_EPISODE, episode_length=L)
        assert float(done) == float(so["done"][0]), t
        assert float(rew) == float(so["reward"][0]), t
        if so["done"][0]:
            resets += 1
            k = P.split(key, 2)
            so, key = o.reset(k[1:2]), k[0].copy()
        np.testing.assert_array_equal(_np(obs), so["obs"][0], err_msg=f"t={t}")
        np.testing.assert_array_equal(_np(g._key), key, err_msg=f"key t={t}")
    assert resets >= 2


def test_eval_gym_wrapper_queues():
    """EvalGymWrapper over a batched gym env: the per-episode queues equal the reference's
    r_q / dr_q / l_q (NaN-seeded, appended in env order of d.nonzero()) and get_stats is
    their nanmean."""
    envs = _envs()
    B, T, L, disc = 64, 23, 5, 0.9
    g = envs.create_gym_env("ant_tag", batch_size=B, seed=1, episode_length=L, eval_metrics=True, discount=disc)
    g.reset()
    # NumPy restatement of wrappers.py:191-229 (float32 buffers, int lengths)
    ret = np.zeros(B, np.float32)
    dret = np.zeros(B, np.float32)
    ln = np.zeros(B, np.int32)
    cd = np.ones(B, np.float32)
    r_q, dr_q, l_q = [math.nan], [math.nan], [math.nan]
    gen = torch.Generator(device="cuda").manual_seed(0)
    for t in range(T):
        act = torch.rand((B, 8), generator=gen, device="cuda") * 2 - 1
        o, r, d, info = g.step(act)
        r, d = _np(r).astype(np.float32), _np(d) != 0
        ret += r
        ln += 1
        dret += r * cd
        cd *= np.float32(disc)
        if d.any():
            idx = d.nonzero()
            r_q.extend(ret[idx]); dr_q.extend(dret[idx]); l_q.extend(ln[idx])
            ret[idx] = 0; dret[idx] = 0; ln[idx] = 0; cd[idx] = 1
    assert len(r_q) > B  # several episodes finished
    np.testing.assert_array_equal(np.array(g.r_q[1:], np.float32), np.array(r_q[1:], np.float32))
    np.testing.assert_array_equal(np.array(g.dr_q[1:], np.float32), np.array(dr_q[1:], np.float32))
    np.testing.assert_array_equal(np.array(g.l_q[1:]), np.array(l_q[1:]))
    assert math.isnan(g.r_q[0])
    st = g.get_stats()
    np.testing.assert_allclose(st["charts/mean_episodic_return"], np.nanmean(np.array(r_q, np.float64)), rtol=1e-6)
    np.testing.assert_allclose(st["charts/mean_discounted_episodic_return"],
                               np.nanmean(np.array(dr_q, np.float64)), rtol=1e-6)
    np.testing.assert_allclose(st["charts/mean_episodic_length"], np.nanmean(np.array(l_q, np.float64)), rtol=1e-6)


def test_eval_gym_wrapper_queue_growth():
    """The device queue grows past its initial capacity (host reads the count rarely)."""
    envs = _envs()
    B = 32
    g = envs.create_gym_env("ant_heavenhell", batch_size=B, seed=2, episode_length=1, eval_metrics=True)
    g._cap0 = 40  # tiny buffer (grown to 64 B = 2 048 at reset): every step finishes all B episodes
    g.reset()
    assert g._lq.shape[0] - 1 == 64 * B
    for _ in range(80):
        g.step(torch.zeros((B, 8), device="cuda"))
    assert g._lq.shape[0] - 1 > 64 * B  # grew
    assert len(g.l_q) == 1 + 80 * B and all(x == 1 for x in g.l_q[1:])


@pytest.mark.parametrize("name", ["ant_tag", "ant_heavenhell"])
def test_sharded_gym_two_shards_one_gpu(name):
    """Two shards (49 + 48 of 97 envs) stepped separately, their any-done words combined
    (what sharding.all_reduce_any_done does over RCCL), then each shard's masked reset with
    its rows of split(gym_key, 98): together they equal the unsharded gym env bit for bit."""
    envs = _envs()
    from po_brax_amd.sharding import Shard
    total, L = 97, 4
    single = envs.create_gym_env(name, batch_size=total, seed=3, episode_length=L)
    parts = [envs.create_gym_env(name, batch_size=total, seed=3, episode_length=L, shard=Shard(total, 2, r))
             for r in range(2)]
    o1 = single.reset()
    op = [p.reset() for p in parts]
    assert torch.equal(o1, torch.cat(op))
    gen = torch.Generator(device="cuda").manual_seed(4)
    n_any = 0
    for t in range(14):
        act = torch.rand((total, 8), generator=gen, device="cuda") * 2 - 1
        o1, r1, d1, _ = single.step(act)
        for p in parts:
            sh = p._shard
            p._step_local(act[sh.lo:sh.hi].contiguous())
        anyd = torch.maximum(parts[0]._any[:1].view(torch.int32), parts[1]._any[:1].view(torch.int32))
        n_any += int(anyd.item())
        for p in parts:
            p._any[:1].view(torch.int32).copy_(anyd)
        outs = [p._autoreset() for p in parts]
        assert torch.equal(o1, torch.cat([x[0] for x in outs])), t
        assert torch.equal(r1, torch.cat([x[1] for x in outs])), t
        for p in parts:
            assert torch.equal(p._key, single._key), t
    assert n_any >= 3


def test_state_replace_done_is_honoured():
    """brax-style edit between steps: state.replace(done=ones) makes the AutoResetWrapper
    step zero the step counters (the reference's where(done, 0, steps)) for every env."""
    envs = _envs()
    name, B = "ant_tag", 64
    env = envs.create(name, batch_size=B, episode_length=50)
    keys = _keys(B, 2)
    s = env.reset(torch.from_numpy(keys).cuda())
    act = np.random.default_rng(0).uniform(-1, 1, (3, B, 8)).astype(np.float32)
    for t in range(2):
        s = env.step(s, torch.from_numpy(act[t]).cuda())
    s = s.replace(done=torch.ones_like(s.done))
    ref = _state_np(s)
    ref["done"] = np.ones(B, np.float32)
    so = orc.OracleEnv(name).step(ref, act[2], flags=FLAGS, episode_length=50)
    s2 = env.step(s, torch.from_numpy(act[2]).cuda())
    compare_states(s2, so, "after replace(done=1)")
    assert bool((s2.info["steps"] == 1).all())


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_inplace_fast_path(name):
    """step_ on a State the engine returned from an in-place step reuses its cached C state
    (envs/env.py fast path) and returns the same object: equal to functional steps bit for
    bit over an autoreset episode, and a brax-style edit (state.replace(done=...)) between
    in-place steps still reaches the kernel (the oracle step from the edited state)."""
    envs = _envs()
    B, L = 96, 4
    keys = torch.from_numpy(_keys(B, 8)).cuda()
    e1, e2 = (envs.create(name, batch_size=B, episode_length=L) for _ in range(2))
    s1, s2 = e1.reset(keys), e2.reset(keys)
    act = np.random.default_rng(3).uniform(-1, 1, (9, B, 8)).astype(np.float32)
    for t in range(8):
        a = torch.from_numpy(act[t]).cuda()
        s1 = e1.step(s1, a)
        prev = s2
        s2 = e2.step_(s2, a)
        if t >= 2:
            assert s2 is prev  # the fast path returns the stepped State itself
        assert "_fast" in s2.aux
    for f in ("pos", "rot", "vel", "ang"):
        assert torch.equal(getattr(s1.qp, f), getattr(s2.qp, f)), f
    assert torch.equal(s1.obs, s2.obs) and torch.equal(s1.reward, s2.reward) and torch.equal(s1.done, s2.done)
    for k in s1.metrics:
        assert torch.equal(s1.metrics[k], s2.metrics[k]), k
    # an edit between in-place steps takes the full path and is honoured
    s3 = s2.replace(done=torch.ones_like(s2.done))
    ref = _state_np(s3)
    ref["done"] = np.ones(B, np.float32)
    so = orc.OracleEnv(name).step(ref, act[8], flags=FLAGS, episode_length=L)
    s4 = e2.step_(s3, torch.from_numpy(act[8]).cuda())
    compare_states(s4, so, f"{name}: in-place after replace(done=1)")


@pytest.mark.parametrize("name", ["ant_tag", "ant_gather"])
def test_inplace_fast_path_sees_info_entry_edits(name):
    """The reference's wrappers edit info entries in place (``state.info['first_qp'] = s.qp``,
    ``info.update(steps=...)``, wrappers.py:105-111): the dict keeps its identity, so the
    in-place fast path must compare the entries themselves.  Reassigning info['steps'] (to
    steps one short of the time limit) and info['first_obs'] (to a new tensor) between step_
    calls reaches the kernel: the step reads and writes the NEW tensors, equal to the oracle
    step from the edited state."""
    envs = _envs()
    B, L = 64, 50
    env = envs.create(name, batch_size=B, episode_length=L)
    keys = _keys(B, 5)
    s = env.reset(torch.from_numpy(keys).cuda())
    act = np.random.default_rng(6).uniform(-1, 1, (4, B, 8)).astype(np.float32)
    for t in range(3):
        s = env.step_(s, torch.from_numpy(act[t]).cuda())
    assert "_fast" in s.aux
    old_steps, old_first_obs = s.info["steps"], s.info["first_obs"]
    old_steps_val = old_steps.clone()
    new_steps = torch.full_like(old_steps, float(L - 1))
    new_first_obs = torch.linspace(-1, 1, old_first_obs.numel(), device="cuda").reshape(old_first_obs.shape)
    s.info["steps"] = new_steps
    s.info.update(first_obs=new_first_obs)
    ref = _state_np(s)
    so = orc.OracleEnv(name).step(ref, act[3], flags=FLAGS, episode_length=L)
    s2 = env.step_(s, torch.from_numpy(act[3]).cuda())
    compare_states(s2, so, f"{name}: in-place after info edits")
    assert s2.info["steps"] is new_steps and s2.info["first_obs"] is new_first_obs
    assert bool((s2.aux["done"] == 1).all())  # every env hit the time limit -> autoreset from new_first_obs
    assert torch.equal(s2.obs, new_first_obs)
    assert torch.equal(old_steps, old_steps_val)  # the old buffer was not stepped


def _eval_np(em, metrics, reward, done, steps):
    """brax <= 0.0.12 EvalWrapper.step [ext], restated in NumPy (parity-unpinned: no reference
    artefact holds EvalWrapper output)."""
    m = dict(metrics, reward=reward)
    d = done.astype(np.float32)
    cur = {k: em["cur"][k] + m[k].astype(np.float32) for k in em["cur"]}
    return {"steps": em["steps"] + np.sum(steps * d, dtype=np.float64),
            "n": em["n"] + np.sum(d, dtype=np.float64),
            "comp": {k: em["comp"][k] + np.sum(cur[k] * d, dtype=np.float64) for k in cur},
            "cur": {k: cur[k] * (1 - d) for k in cur}}


@pytest.mark.parametrize("name", ["ant_tag", "ant_gather"])
def test_eval_wrapper_metrics(name):
    """create(..., eval_metrics=True) (po_brax/envs/__init__.py:69-70, brax EvalWrapper [ext]):
    the per-env current-episode metrics and the completed-episode totals after every step equal
    a NumPy restatement of brax EvalWrapper driven by the ORACLE's step outputs (env fields
    compared bit-exact first), over episodes of 3 steps so that several complete."""
    envs = _envs()
    B, L, T = 128, 3, 7
    env = envs.create(name, batch_size=B, episode_length=L, eval_metrics=True)
    u = env.unwrapped
    keys = _keys(B, 12)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    so = o.reset(keys, first=True)
    names = list(s.info["eval_metrics"]["current_episode_metrics"])
    assert set(names) == set(u.reset_metrics) | {"reward"}
    em = {"cur": {k: np.zeros(B, np.float32) for k in names}, "comp": {k: 0.0 for k in names},
          "n": 0.0, "steps": 0.0}
    rng = np.random.default_rng(2)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(so, act, flags=FLAGS, episode_length=L)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} eval step {t}")
        om = {n: so[f"m{u.slot_names.index(n)}"] for n in u.step_metrics}
        em = _eval_np(em, om, so["reward"], so["done"], so["steps"])
        g = s.info["eval_metrics"]
        for k in names:
            np.testing.assert_array_equal(_np(g["current_episode_metrics"][k]), em["cur"][k], err_msg=f"{t} cur {k}")
            np.testing.assert_allclose(float(g["completed_episodes_metrics"][k]), em["comp"][k], rtol=1e-5,
                                       atol=1e-4, err_msg=f"{t} comp {k}")
        assert float(g["completed_episodes"]) == em["n"], t
        np.testing.assert_allclose(float(g["completed_episodes_steps"]), em["steps"], rtol=1e-6)
    assert em["n"] >= B  # at least one full round of episodes completed


def test_eval_wrapper_heavenhell_metric_mismatch_raises():
    """AntHeavenHell's step adds metrics['hits'] (ant_heavenhell.py:122) that its reset lacks:
    brax EvalWrapper's tree_multimap over the two dicts fails there, and so does this one."""
    envs = _envs()
    env = envs.create("ant_heavenhell", batch_size=8, eval_metrics=True)
    s = env.reset(torch.from_numpy(_keys(8, 1)).cuda())
    with pytest.raises(ValueError, match="tree_multimap"):
        env.step(s, torch.zeros((8, 8), device="cuda"))

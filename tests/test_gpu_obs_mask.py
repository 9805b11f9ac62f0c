"""GPU: the observation mask fused into the step (C ABI v7, ``create(..., obs_mask=idx)``).

BASELINE.json config 2 is "AntHeavenHell batch=4096 (physics + obs-mask kernel)": the step
kernel itself stores ``obs[:, idx]`` (``state.info['obs_masked']``) from the observation rows it
assembles -- no second launch.  Checked against the CPU oracle's state (``obs[:, idx]`` of the
oracle's observation, bit-exact) at HH 4 096 x 114 (the sixteen-lane kernel), and against the
kernel's own obs on the eight-lane (TAG 8 192, GA 16 384), four-lane (HH 16 385: ragged last
wave) and mixed launches, through reset, autoreset and the gym path.
Reference: po_brax/standard_observability_masks.py:5-67 (index sets applied as obs[:, idx]).
"""
import os

import numpy as np
import pytest
import torch

import orc
import pob_np as P
from test_gpu_parity import _keys, _state_np, compare_states

pytestmark = pytest.mark.gpu
FLAGS = orc.F_EPISODE | orc.F_AUTORESET
NT = max(1, min(16, len(os.sched_getaffinity(0))))


def _envs():
    from po_brax_amd import envs
    return envs


def _mask(name):
    from po_brax_amd import standard_observability_masks as M
    return M.po_env_mask(name, cfrc=False)  # positions, velocities, task entries: no contact forces


def _check(s, idx, what):
    got = s.info["obs_masked"]
    exp = s.obs[:, torch.as_tensor(idx, device=s.obs.device)]
    assert got.shape == exp.shape, what
    assert torch.equal(got, exp), what


def test_obs_mask_config2_hh4096_vs_oracle():
    """Config 2: HH B = 4 096 x 114, the masked columns equal the oracle state's obs[:, idx]."""
    name, B, L = "ant_heavenhell", 4096, 3
    idx = _mask(name)
    env = _envs().create(name, batch_size=B, episode_length=L, obs_mask=idx)
    assert env.masked_observation_size == len(idx) == 30
    keys = _keys(B)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    so = o.reset(keys, first=True, nthreads=NT)
    np.testing.assert_array_equal(s.info["obs_masked"].cpu().numpy(), so["obs"][:, idx])
    rng = np.random.default_rng(1)
    for t in range(4):  # step 3 autoresets every env (first_obs rows)
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=FLAGS, episode_length=L, nthreads=NT)
        s = env.step_(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"masked step {t}")
        np.testing.assert_array_equal(s.info["obs_masked"].cpu().numpy(), so["obs"][:, idx], err_msg=f"step {t}")


@pytest.mark.parametrize("name,B", [("ant_tag", 8192), ("ant_gather", 16384), ("ant_heavenhell", 16385),
                                    ("ant", 4096)])
def test_obs_mask_every_kernel(name, B):
    from po_brax_amd import standard_observability_masks as M
    idx = M.POSITION["ant"] if name == "ant" else _mask(name)[::-1].copy()  # any order, repeats allowed
    env = _envs().create(name, batch_size=B, episode_length=2, obs_mask=np.concatenate([idx, idx[:3]]))
    s = env.reset(torch.from_numpy(_keys(B)).cuda())
    idx2 = np.concatenate([idx, idx[:3]])
    _check(s, idx2, f"{name} reset")
    rng = np.random.default_rng(2)
    for t in range(3):
        s = env.step(s, torch.from_numpy(rng.uniform(-1, 1, (B, 8)).astype(np.float32)).cuda())
        _check(s, idx2, f"{name} step {t}")


def test_obs_mask_mixed_and_gym():
    envs = _envs()
    idx = {n: _mask(n) for n in ("ant_heavenhell", "ant_gather", "ant_tag")}
    g = envs.create_gym_env("ant_heavenhell", batch_size=2048, seed=0, episode_length=5,
                            obs_mask=idx["ant_heavenhell"])
    g.reset()
    rng = np.random.default_rng(3)
    for t in range(7):  # gym autoresets at step 5 (the masked reset path re-gathers)
        g.step(torch.from_numpy(rng.uniform(-1, 1, (2048, 8)).astype(np.float32)).cuda())
        _check(g._state, idx["ant_heavenhell"], f"gym step {t}")


def test_obs_mask_errors():
    envs = _envs()
    with pytest.raises(ValueError):
        envs.create("ant_heavenhell", batch_size=8, obs_mask=[0, 114])
    with pytest.raises(TypeError):
        envs.create("ant_heavenhell", batch_size=8, obs_mask=[0.5])
    with pytest.raises(ValueError):  # (not wrapped into range by the int32 cast)
        envs.create("ant_heavenhell", batch_size=8, obs_mask=np.array([2 ** 32 + 3], np.int64))
    env = envs.create("ant_heavenhell", batch_size=8)
    assert env.masked_observation_size == 0 and env.obs_mask is None


def test_obs_mask_mixed_launch():
    """The mixed launch (config 5's one kernel for HH + GA + TAG): every segment stores its own
    kind's masked columns (each env's table holds its mask; indices valid for all three)."""
    from po_brax_amd import jumpy
    envs = _envs()
    idx = np.array([0, 1, 2, 14, 15, 28, 29, 60, 102], np.int64)
    names = ["ant_heavenhell", "ant_gather", "ant_tag"]
    mix = envs.create_mixed(names, episode_length=3, qp_dtype=torch.float16, obs_mask=idx)
    sizes = [700, 500, 301]
    key = jumpy.random_prngkey(4)
    ms = mix.reset(key, sizes)
    act = torch.empty((sum(sizes), 8), device="cuda")
    for t in range(4):
        jumpy.random_actions_(key, sum(sizes), 0, act)
        ms = mix.step_(ms, [a.contiguous() for a in mix.split_actions(act)])
        for n, s in zip(names, ms):
            _check(s, idx, f"mixed {n} step {t}")


@pytest.mark.parametrize("qp_dtype", [torch.float32, torch.float16])
def test_obs_mask_written_by_masked_reset(qp_dtype):
    """ABI v8: the masked reset writes the masked columns of the rows it resets (no
    second gather launch after it) -- rows written straight from registers (one to three done
    envs per wave, float32 storage) and rows staged in LDS (a whole wave; binary16 storage
    always) -- and leaves every other row's masked columns as the step wrote them."""
    from po_brax_amd import _lib
    name, B = "ant_heavenhell", 1000
    idx = _mask(name)
    env = _envs().create(name, batch_size=B, auto_reset=False, episode_length=1000, obs_mask=idx,
                         qp_dtype=qp_dtype)
    s = env.reset(torch.from_numpy(_keys(B, 23)).cuda())
    _check(s, idx, "reset")
    rng = np.random.default_rng(6)
    for _ in range(2):
        s = env.step_(s, torch.from_numpy(rng.uniform(-1, 1, (B, 8)).astype(np.float32)).cuda())
    done = np.zeros(B, np.float32)
    done[[3, 17, 18, 200, 515, 777, 998, 999]] = 1.0
    done[320:336] = 1.0
    done[480:483] = 1.0
    s.aux["done"].copy_(torch.from_numpy(done).cuda())
    before = s.info["obs_masked"].clone()
    env.unwrapped._reset_where_done(s, _lib.RESET_OWN)
    torch.cuda.synchronize()
    _check(s, idx, "masked reset")
    keep = torch.from_numpy(done == 0).cuda()
    assert torch.equal(s.info["obs_masked"][keep], before[keep])
    assert not torch.equal(s.info["obs_masked"][~keep], before[~keep])

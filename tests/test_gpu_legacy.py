"""GPU: the legacy-spring dynamics mode (``legacy_spring=True``; brax <= 0.0.12, the physics of
the reference's only recorded trajectory, notebooks/ant_tag.ipynb:449).

* the HIP kernel k_step_legacy vs the C oracle in legacy mode, bit-exact, for every env kind,
  reset (sys.info = the colliders' impulses) and per-step / free-running steps, on both block
  shapes (64-thread blocks for B <= 4096, 256-thread above);
* the HIP kernel vs the notebook's 20 recorded frames (<= 2e-5 m / 2e-5 in the quaternions;
  the float64 restatement oracle/legacy_np.py and the float32 C oracle reach 9e-6 / 6e-6).
"""
import json
import os

import numpy as np
import pytest
import torch

import orc
import pob_np as P
from test_gpu_parity import NAMES, _keys, _np, _state_np, compare_states

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _envs():
    from po_brax_amd import envs
    return envs


@pytest.mark.parametrize("name", NAMES)
def test_legacy_reset_and_step_parity(name):
    B, T = 200, 12
    env = _envs().create(name, batch_size=B, episode_length=9, legacy_spring=True)
    keys = _keys(B, 5)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name, legacy_spring=1)
    compare_states(s, o.reset(keys, first=True), f"{name} legacy reset")
    rng = np.random.default_rng(7)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = o.step(_state_np(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=9)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} legacy step {t}")


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 4097), ("ant_tag", 1000), ("ant_gather", 300)])
def test_legacy_free_running(name, B):
    """Both engines run 15 steps independently (B = 4097: the 256-thread block shape)."""
    T = 15
    env = _envs().create(name, batch_size=B, episode_length=1000, legacy_spring=True)
    keys = _keys(B, 9)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name, legacy_spring=1)
    so = o.reset(keys, first=True, nthreads=8)
    rng = np.random.default_rng(11)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        s = env.step_(s, torch.from_numpy(act).cuda())
        so = o.step(so, act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=1000, inplace=True, nthreads=8)
    compare_states(s, so, f"{name} legacy free-running B={B}")


def test_legacy_kernel_matches_notebook_frames():
    """notebooks/ant_tag.ipynb:470-477: the notebook's frame 0 (with the reset's joint
    velocities from split(rng, 5)[2]) stepped 20 times with the cell's actions reproduces
    frames 1..20.  AntTag with cage 5.5 puts the box walls' inner faces at +-6.5, where the
    notebook's capsule walls were (no wall contact either way)."""
    import legacy_np as LG
    traj = json.load(open(os.path.join(HERE, "golden", "ant_tag_notebook_trajectory.json")))
    pos = np.array(traj["pos"])[:, :9]
    rot = np.array(traj["rot"])[:, :9]
    env = _envs().AntTagEnv(legacy_spring=True, cage_xy=(5.5, 5.5))
    s = env.reset(torch.from_numpy(_keys(1, 0)).cuda())
    qvel = P.np_uniform(P.np_split(P.np_prngkey(0), 5)[2], (8,), -0.1, 0.1)
    _, w0 = LG.joint_velocities(rot[0], qvel)
    s.qp.pos[0, :9] = torch.from_numpy(pos[0].astype(np.float32)).cuda()
    s.qp.rot[0, :9] = torch.from_numpy(rot[0].astype(np.float32)).cuda()
    s.qp.vel[0, :9] = 0.0
    s.qp.ang[0, :9] = torch.from_numpy(w0.astype(np.float32)).cuda()
    rng = P.np_prngkey(0)
    for t in range(1, 21):
        rng, r1 = P.np_split(rng, 2)
        act = P.np_uniform(r1, (8,), -1, 1).astype(np.float32)
        s = env.step(s, torch.from_numpy(act[None]).cuda())
        x = _np(s.qp.pos)[0, :9].astype(np.float64)
        q = _np(s.qp.rot)[0, :9].astype(np.float64)
        sg = np.sign(np.sum(q * rot[t], -1))[:, None]
        assert np.abs(x - pos[t]).max() <= 2e-5, (t, np.abs(x - pos[t]).max())
        assert np.abs(q * sg - rot[t]).max() <= 2e-5, (t, np.abs(q * sg - rot[t]).max())


def test_legacy_rejected_by_mixed_step():
    envs = _envs()
    from po_brax_amd import jumpy
    m = envs.create_mixed(["ant_heavenhell", "ant_tag"], legacy_spring=True)
    s = m.reset(jumpy.random_prngkey(0), [8, 8])
    with pytest.raises(ValueError):
        m.step(s, torch.zeros((16, 8), device="cuda"))


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 65536), ("ant_tag", 65536), ("ant_gather", 16384)])
def test_legacy_per_step_parity_bench_sizes(name, B):
    """Legacy dynamics at the BASELINE.json batch sizes (configs 1/4 HH / TAG 65 536, config 3
    GA 16 384): reset parity, then per-step parity with the oracle restarted from the GPU's
    state each step, bit-exact on every field; episode length 3 makes step 3 autoreset every
    env (the first_qp / first_obs rows run)."""
    from test_gpu_headline_parity import NT, _actions
    T, L = 4, 3
    env = _envs().create(name, batch_size=B, episode_length=L, legacy_spring=True)
    keys = _keys(B, 23)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name, legacy_spring=1)
    compare_states(s, o.reset(keys, first=True, nthreads=NT), f"{name} legacy B={B} reset")
    n_done = 0
    for t, act in enumerate(_actions(29, B, T)):
        so = o.step(_state_np(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=L, nthreads=NT)
        s = env.step_(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} legacy B={B} step {t}")
        n_done += int(so["done"].sum())
    assert n_done >= B

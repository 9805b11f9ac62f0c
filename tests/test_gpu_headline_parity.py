"""GPU parity at the BASELINE.json batch sizes, on the launch paths the bench takes.

``pob_step`` runs the sixteen-lanes-per-env kernel (``k_step_hex``) while its waves fit one
up to a per-kind batch (HH and TAG 32, GA and the stock ant 16 x the CU count: 8 192 /
4 096 on MI355X; ``POB_HEXA_MAX_B`` overrides), the
eight-lane kernel (``k_step_oct``) for B <= 16 384 and the four-lane kernel (``k_step_quad``)
above -- with one-wave (64-thread) blocks when the smaller-batch kernels are disabled
(``POB_HEXA_MAX_B=0``, ``POB_OCTET_MAX_B=0``) and B <= 4 096, 256-thread blocks otherwise; the
mixed launch is always the four-lane kernel in 256-thread blocks.  The small-batch parity
tests (test_gpu_parity.py, B <= 512) take the sixteen-lane path, so this file checks, against
the CPU oracle (OpenMP over envs):

* the headline config: AntHeavenHell B = 65 536 (config 1 of the bench),
* AntTag B = 65 536 (config 4's total batch on one GPU), AntGather B = 16 384 (config 3),
* AntHeavenHell B = 4 096 (config 2, the last one-wave-block batch) and B = 4 097 (the
  first 256-thread-block batch, ragged: its last wave holds one env),
* the mixed launch with binary16 qp storage, HH + GA + TAG over B = 32 768 (config 5's
  per-GPU batch),
* a wall-stress case on the 256-thread path (ants teleported onto the arena walls).

Each is reset parity plus per-step parity (the oracle restarts from the GPU's state each
step), bit-exact on every field.  Episode length 3 makes step 3 autoreset every env.

Parity unpinned: these tests pin the kernels to the oracle, not to brax.  The PBD
solver and the wall contacts (the oracle's default MV_BRAX spelling of capsule x
TriangulatedBox, recalled; its unpinned choices measured in DESIGN.md §3) have no reference
artefact, so agreement here is kernel == restatement, bit for bit.
"""
import os

import numpy as np
import pytest
import torch

import orc
import pob_np as P
from test_gpu_parity import _keys, _near_wall, _state_np, _walls, compare_states
from test_gpu_variants import _assert_fp16_step, _state_np32

pytestmark = pytest.mark.gpu
FLAGS = orc.F_EPISODE | orc.F_AUTORESET
NT = max(1, min(16, len(os.sched_getaffinity(0))))  # the box's CPU share is 16


def _envs():
    from po_brax_amd import envs
    return envs


def _actions(seed, B, T):
    rng = np.random.default_rng(seed)
    return [rng.uniform(-1, 1, (B, 8)).astype(np.float32) for _ in range(T)]


def _per_step(name, B, T=4, L=3, seed=0):
    env = _envs().create(name, batch_size=B, episode_length=L)
    keys = _keys(B, seed)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    compare_states(s, o.reset(keys, first=True, nthreads=NT), f"{name} B={B} reset")
    n_done = 0
    for t, act in enumerate(_actions(seed + 1, B, T)):
        so = o.step(_state_np(s), act, flags=FLAGS, episode_length=L, nthreads=NT)
        s = env.step_(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} B={B} step {t}")
        n_done += int(so["done"].sum())
    assert n_done >= B  # step L autoresets every env: the first_qp / first_obs rows ran


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 65536), ("ant_tag", 65536), ("ant_gather", 16384),
                                    ("ant_heavenhell", 16385), ("ant_heavenhell", 4096), ("ant_heavenhell", 4097),
                                    ("ant_gather", 4097), ("ant_tag", 4097), ("ant", 4097),
                                    ("ant_gather", 16385), ("ant_gather", 49153)])
def test_per_step_parity_bench_sizes(name, B):
    """(AntGather on the four-lane kernel: B <= 3 waves per SIMD takes the three-wave build
    k_step_quad_ga3, B = 49 153 the four-wave one on a 256-CU device.)"""
    _per_step(name, B)


@pytest.mark.parametrize("B", [64, 4097])
def test_per_step_parity_four_lane_small(monkeypatch, B):
    """The four-lane kernel at small batches (sixteen- and eight-lane kernels disabled):
    one-wave blocks (B = 64) and 256-thread blocks with a one-env tail wave (B = 4 097)."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "0")
    monkeypatch.setenv("POB_OCTET_MAX_B", "0")
    for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
        _per_step(name, B, seed=B)


@pytest.mark.parametrize("B", [61, 4097])
def test_per_step_parity_eight_lane_small(monkeypatch, B):
    """The eight-lane kernel at small batches (sixteen-lane kernel disabled), ragged tails."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "0")
    for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
        _per_step(name, B, seed=B + 1)


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 8192), ("ant_tag", 8192), ("ant_gather", 8191), ("ant", 8190)])
def test_per_step_parity_sixteen_lane(monkeypatch, name, B):
    """The sixteen-lane kernel at two waves per SIMD (config 4's per-GPU TAG batch: the default
    launch for HH and TAG there; POB_HEXA_MAX_B selects it for GA and the stock ant)."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "8192")
    _per_step(name, B, seed=5)


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 8192), ("ant_tag", 8192), ("ant_gather", 8191)])
def test_per_step_parity_eight_lane_8192(monkeypatch, name, B):
    """The eight-lane kernel at config 4's per-GPU batch (the default launch there for GA;
    HH and TAG with the sixteen-lane kernel disabled)."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "0")
    _per_step(name, B, seed=6)


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag", "ant"])
@pytest.mark.parametrize("B", [4096, 8192, 16400])  # sixteen-lane; sixteen (HH, TAG) or eight; four
def test_free_running_300_steps(name, B):
    """GPU and oracle each run 300 steps from the same reset with no restart (episode length
    100: three autoresets per env on the way), every kernel's default batch range: any float
    divergence would compound through the contact dynamics, so bit-equality at the end is a
    strong statement about every step on the way."""
    T, L = 300, 100
    env = _envs().create(name, batch_size=B, episode_length=L)
    keys = _keys(B, 77)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name)
    so = o.reset(keys, first=True, nthreads=NT)
    rng = np.random.default_rng(B)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        s = env.step_(s, torch.from_numpy(act).cuda())
        so = o.step(so, act, flags=FLAGS, episode_length=L, nthreads=NT, inplace=True)
    compare_states(s, so, f"{name} B={B} free-running t={T}")


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 65536), ("ant_gather", 16384), ("ant_tag", 65536)])
def test_gym_parity_full_size(name, B):
    """The gym path (create_gym_env -> AutoresetVmapGymWrapper, wrappers.py:240-262) at the
    bench's sizes: every step's obs, done, qp, episode counter and gym key equal the oracle's
    (episode length 4: every env resets at step 4 through the gym key's split rows)."""
    import pob_np as P
    from test_gpu_parity import close, _np
    envs = _envs()
    L, T = 4, 6
    g = envs.create_gym_env(name, batch_size=B, seed=3, episode_length=L)
    obs = g.reset()
    o = orc.OracleEnv(name)
    ks = P.split(P.prngkey(3), B + 1)
    so, gkey = o.reset(ks[1:], nthreads=NT), ks[0].copy()
    np.testing.assert_array_equal(_np(obs), so["obs"])
    rng = np.random.default_rng(B)
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        obs, rew, done, info = g.step(torch.from_numpy(act).cuda())
        so = o.step(so, act, flags=orc.F_EPISODE, episode_length=L, inplace=True, nthreads=NT)
        np.testing.assert_array_equal(_np(done), so["done"], err_msg=f"t={t}")
        o.gym_autoreset(so, gkey, nthreads=NT)
        close(obs, so["obs"], f"{name} B={B} gym obs t={t}")
        close(rew, so["reward"], f"{name} B={B} gym reward t={t}")
        close(g._state.qp.pos, so["pos"], f"{name} B={B} gym pos t={t}")
        close(g._state.qp.rot, so["rot"], f"{name} B={B} gym rot t={t}")
        np.testing.assert_array_equal(_np(g._key), gkey, err_msg=f"gym key t={t}")
        np.testing.assert_array_equal(_np(g._state.info["steps"]), so["steps"])


def _prefix_identical(Ba, Bb, env_a=None, env_b=None):
    envs = _envs()
    for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
        for qp_dtype in (torch.float32, torch.float16):
            keys = torch.from_numpy(_keys(Bb, 3)).cuda()
            ea = envs.create(name, batch_size=Ba, episode_length=5, qp_dtype=qp_dtype)
            eb = envs.create(name, batch_size=Bb, episode_length=5, qp_dtype=qp_dtype)
            sa, sb = ea.reset(keys[:Ba].contiguous()), eb.reset(keys)
            for act in _actions(7, Bb, 8):
                a = torch.from_numpy(act).cuda()
                sa = ea.step_(sa, a[:Ba].contiguous())
                sb = eb.step_(sb, a)
            for f in ("pos", "rot", "vel", "ang"):
                assert torch.equal(getattr(sa.qp, f), getattr(sb.qp, f)[:Ba]), (name, qp_dtype, f)
            assert torch.equal(sa.obs, sb.obs[:Ba]), (name, qp_dtype)
            assert torch.equal(sa.reward, sb.reward[:Ba]), (name, qp_dtype)
            assert torch.equal(sa.aux["done"], sb.aux["done"][:Ba]), (name, qp_dtype)


def test_octet_quad_switch_prefix_identical():
    """The first 16 384 envs of a B = 16 385 run (four-lane kernel) equal a B = 16 384 run
    (eight-lane kernel) bit for bit, fp32 and fp16 storage, for every kind."""
    _prefix_identical(16384, 16385)


def test_hexa_octet_switch_prefix_identical(monkeypatch):
    """At a switch of 16 x the CU count (the default for AntGather and the stock ant; HH and TAG
    switch later, pob_kernels.hip hexa_max_batch): the first n envs of a B = n + 1 run
    (eight-lane kernel) equal a B = n run (sixteen-lane kernel) bit for bit, fp32 and fp16
    storage, for every kind."""
    n = 16 * torch.cuda.get_device_properties(0).multi_processor_count
    monkeypatch.setenv("POB_HEXA_MAX_B", str(n))
    _prefix_identical(n, n + 1)


def test_hexa_default_switch_prefix_identical():
    """At the per-kind default switches (HH and TAG 32 x CUs): B = n + 1 (the eight-lane kernel;
    HH with its contact pool) against B = n (the sixteen-lane kernel at two waves per SIMD)."""
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    envs = _envs()
    for name, n in (("ant_heavenhell", 32 * n_cu), ("ant_tag", 32 * n_cu)):
        keys = torch.from_numpy(_keys(n + 1, 3)).cuda()
        ea = envs.create(name, batch_size=n, episode_length=5)
        eb = envs.create(name, batch_size=n + 1, episode_length=5)
        sa, sb = ea.reset(keys[:n].contiguous()), eb.reset(keys)
        for act in _actions(7, n + 1, 6):
            a = torch.from_numpy(act).cuda()
            sa = ea.step_(sa, a[:n].contiguous())
            sb = eb.step_(sb, a)
        for f in ("pos", "rot", "vel", "ang"):
            assert torch.equal(getattr(sa.qp, f), getattr(sb.qp, f)[:n]), (name, f)
        assert torch.equal(sa.obs, sb.obs[:n]), name


def test_hexa_octet_switch_prefix_identical_8192(monkeypatch):
    """The same across an overridden switch (POB_HEXA_MAX_B = 8 192: the sixteen-lane kernel
    at two waves per SIMD against the eight-lane kernel at B = 8 193)."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "8192")
    _prefix_identical(8192, 8193)


def test_quad_block_switch_prefix_identical(monkeypatch):
    """Four-lane kernel only: B = 4 097 (256-thread blocks) vs B = 4 096 (one-wave blocks)."""
    monkeypatch.setenv("POB_HEXA_MAX_B", "0")
    monkeypatch.setenv("POB_OCTET_MAX_B", "0")
    _prefix_identical(4096, 4097)


def test_mixed_fp16_config5_parity():
    """BASELINE config 5 per GPU: HH + GA + TAG mixed, B = 32 768, binary16 qp storage, one
    launch per step.  Each kind's segment against the oracle: the float32 step of the
    decoded fp16 state, rounded to fp16, equals the GPU's fp16 qp bit for bit."""
    envs = _envs()
    from po_brax_amd import jumpy
    names = ["ant_heavenhell", "ant_gather", "ant_tag"]
    B = 32768
    sizes = [B // 3 + (1 if i < B % 3 else 0) for i in range(3)]
    L = 3
    mix = envs.create_mixed(names, episode_length=L, qp_dtype=torch.float16)
    key = jumpy.random_prngkey(0)
    ms = mix.reset(key, sizes)
    oes = [orc.OracleEnv(n) for n in names]
    keys = P.split(P.prngkey(0), B + 1)[1:]
    for n, s, o, off, b in zip(names, ms, oes, mix.offsets(), sizes):
        ro = o.reset(keys[off:off + b], first=True, nthreads=NT)
        for f in ("pos", "rot", "vel", "ang"):
            np.testing.assert_array_equal(getattr(s.qp, f).cpu().numpy().view(np.uint16),
                                          ro[f].astype(np.float16).view(np.uint16), err_msg=f"{n} reset {f}")
        np.testing.assert_array_equal(s.obs.cpu().numpy(), ro["obs"], err_msg=f"{n} reset obs")
    for t, act in enumerate(_actions(11, B, 4)):
        acts = mix.split_actions(torch.from_numpy(act).cuda())
        sos = [o.step(_state_np32(s), a.cpu().numpy(), flags=FLAGS, episode_length=L, nthreads=NT)
               for o, s, a in zip(oes, ms, acts)]
        ms = mix.step_(ms, [a.contiguous() for a in acts])
        for n, s, so in zip(names, ms, sos):
            _assert_fp16_step(s, so, f"mixed fp16 {n} step {t}")


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_tag"])
@pytest.mark.parametrize("kernel", ["default", "four_lane"])
def test_wall_stress_256_thread_blocks(monkeypatch, name, kernel):
    """test_gpu_parity.test_step_parity_against_walls at B = 8 192: ants teleported onto the
    walls, on the default launch (the sixteen-lane kernel for HH and TAG, eight lanes for GA)
    and on the four-lane kernel in 256-thread blocks (four waves sharing the block's LDS wall
    rows; many walls' contacts per wave: the contact pools' overflow paths).  Parity unpinned
    against brax (kernel == restatement; module docstring)."""
    if kernel == "four_lane":
        monkeypatch.setenv("POB_HEXA_MAX_B", "0")
        monkeypatch.setenv("POB_OCTET_MAX_B", "0")
    B, T = 8192, 4
    env = _envs().create(name, batch_size=B, episode_length=1000)
    s = env.reset(torch.from_numpy(_keys(B, 5)).cuda())
    walls = _walls(name)
    ext = np.array([[abs(c[0]) + max(h), abs(c[1]) + max(h)] for c, _, h in walls]).max(0)
    lo = np.array([-ext[0], min(c[1] - max(h) for c, _, h in walls)])
    hi = np.array([ext[0], max(c[1] + max(h) for c, _, h in walls)])
    rng = np.random.default_rng(9)
    cand = rng.uniform(lo, hi, (16 * B, 2))
    near = cand[_near_wall(cand, walls, 1.0)]
    assert len(near) >= 3 * B // 4
    xy = np.concatenate([near[: 3 * B // 4], cand[: B - 3 * B // 4]]).astype(np.float32)[rng.permutation(B)]
    off = torch.from_numpy(xy - s.qp.pos[:, 0, :2].cpu().numpy()).cuda()
    s.qp.pos[:, :9, :2] += off[:, None, :]
    o = orc.OracleEnv(name)
    for t, act in enumerate(_actions(13, B, T)):
        so = o.step(_state_np(s), act, flags=FLAGS, episode_length=1000, nthreads=NT)
        s = env.step(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} wall B={B} step {t}")


@pytest.mark.parametrize("lanes,B,gacc", [(16, 70, "1"), (16, 70, "0"), (8, 70, "1"), (8, 9000, "0"), (4, 70, None)])
def test_out_of_range_inputs_take_exact_fallbacks(monkeypatch, lanes, B, gacc):
    """The kernels' fast reciprocal / square root / quaternion normalisation fall back to
    the IEEE forms behind wave-uniform guards (pob_math.h pob_rcp, qnormalize).  States that
    take the fallbacks -- a torso at 1e25 m/s (joint anchors drift beyond 2^96), a zero
    quaternion (normalisation fallback), a 1e30 rad/s spin -- must still match the oracle
    bit for bit (NaN / inf included), in the lanes that hold them and in their neighbours,
    on the sixteen-, eight- and four-lane kernels.  The sixteen- and eight-lane kernels run
    both guard policies (pob_math.h GuardAcc: no branches, the wave reruns its substeps under
    the branch guards when a lane saw an operand out of range; GuardBranch)."""
    if gacc is not None:
        monkeypatch.setenv("POB_HEX_GACC" if lanes == 16 else "POB_OCT_GACC", gacc)
    if lanes <= 8:
        monkeypatch.setenv("POB_HEXA_MAX_B", "0")
    if lanes == 4:
        monkeypatch.setenv("POB_OCTET_MAX_B", "0")
    for name in ("ant_heavenhell", "ant_gather", "ant_tag", "ant"):
        env = _envs().create(name, batch_size=B, episode_length=1000)
        keys = _keys(B, 40 + lanes)
        s = env.reset(torch.from_numpy(keys).cuda())
        with torch.no_grad():
            s.qp.vel[1, 0, 0] = 1e25
            s.qp.rot[2, 1] = 0.0
            s.qp.ang[3, 2, 1] = 1e30
        o = orc.OracleEnv(name)
        for t, act in enumerate(_actions(lanes + 2, B, 2)):
            so = o.step(_state_np(s), act, flags=FLAGS, episode_length=1000, nthreads=NT)
            s = env.step(s, torch.from_numpy(act).cuda())
            compare_states(s, so, f"{name} B={B} lanes={lanes} step {t}")


def test_config4_tag_shard_equals_slice_of_full_batch():
    """BASELINE config 4 at full size: AntTag, global batch 65 536 over 8 ranks.  Rank 5's
    shard (8 192 envs: the eight-lane kernel) stepped from its own rows of the global reset
    keys and actions equals rows [40 960, 49 152) of the whole batch stepped on one GPU (the
    four-lane kernel), bit for bit -- the index-sharding property bench.py's strong-scaling
    runs rely on, across the kernel switch."""
    from po_brax_amd import envs, jumpy
    from po_brax_amd.sharding import shard_keys, shard_range
    total, world, rank, T = 65536, 8, 5, 8
    lo, hi = shard_range(total, world, rank)
    key = jumpy.random_prngkey(0)
    full = envs.create("ant_tag", batch_size=total, episode_length=4)
    part = envs.create("ant_tag", batch_size=hi - lo, episode_length=4)
    sf = full.reset(shard_keys(key, total, 1, 0))
    sp = part.reset(shard_keys(key, total, world, rank))
    k1, k2 = key.clone(), key.clone()
    af = torch.empty((total, 8), device="cuda")
    ap = torch.empty((hi - lo, 8), device="cuda")
    for t in range(T):
        jumpy.random_actions_(k1, total, 0, af)
        jumpy.random_actions_(k2, total, lo, ap)
        sf = full.step_(sf, af)
        sp = part.step_(sp, ap)
    torch.cuda.synchronize()
    for f in ("pos", "rot", "vel", "ang"):
        assert torch.equal(getattr(sf.qp, f)[lo:hi], getattr(sp.qp, f)), f
    assert torch.equal(sf.obs[lo:hi], sp.obs) and torch.equal(sf.done[lo:hi], sp.done)
    assert torch.equal(sf.info["rng"][lo:hi], sp.info["rng"])
    assert bool(sf.done.all())  # step 8 of 4-step episodes: the time limit (after one autoreset)


def test_config5_mixed_fp16_full_global_batch_properties():
    """BASELINE config 5 at its full global batch on one GPU: HH + GA + TAG mixed in one
    launch per step, 262 144 envs, binary16 qp storage, autoreset: every output finite, the
    dynamic bodies' quaternions unit within binary16 rounding, the reference's dtypes (TAG
    bool done, GA int32 counts), rewards from each task's set, and episodes ending at the
    run's last step (every env reaches the time limit)."""
    from po_brax_amd import envs, jumpy
    total, T = 262144, 5
    names = ["ant_heavenhell", "ant_gather", "ant_tag"]
    sizes = [total // 3 + (1 if i < total % 3 else 0) for i in range(3)]
    m = envs.create_mixed(names, episode_length=5, qp_dtype=torch.float16)
    key = jumpy.random_prngkey(3)
    s = m.reset(key, sizes)
    act = torch.empty((total, 8), device="cuda")
    for t in range(T):
        jumpy.random_actions_(key, total, 0, act)
        s = m.step_(s, act)
    torch.cuda.synchronize()
    rsets = {"ant_heavenhell": {-2.0, -1.0, 0.0, 1.0}, "ant_gather": {-10.0, -1.0, 0.0, 1.0},
             "ant_tag": {-1.0, 0.0, 1.0}}
    for name, st in zip(names, s):
        assert st.qp.pos.dtype == torch.float16
        assert torch.isfinite(st.obs).all() and torch.isfinite(st.qp.pos.float()).all(), name
        qn = st.qp.rot[:, :9].float().norm(dim=-1)
        assert torch.allclose(qn, torch.ones_like(qn), atol=2e-3), name
        assert set(torch.unique(st.reward).tolist()) <= rsets[name], name
        assert bool((st.info["steps"] <= 5).all()), name
    assert s[2].done.dtype == torch.bool and s[1].metrics["apples"].dtype == torch.int32
    assert all(bool((st.aux["done"] != 0).all()) for st in s)  # step 5 of 5: the time limit


@pytest.mark.parametrize("name,B", [("ant_heavenhell", 16400), ("ant_tag", 16400), ("ant_gather", 65536)])
def test_fixup_launch_parity(monkeypatch, name, B):
    """The four-lane kernel's split launch (pob_kernels.hip MODE 1 / 2): every wave forced
    through the fix-up launch (POB_QUAD_FORCE_FIXUP=1: the fast launch marks every wave and
    stores nothing, the fix-up launch steps the marked waves with the in-kernel re-walks) is
    bit-exact against the oracle; the one-launch form (POB_QUAD_SPLIT=0) too."""
    monkeypatch.setenv("POB_QUAD_FORCE_FIXUP", "1")
    _per_step(name, B, T=4, seed=21)
    monkeypatch.delenv("POB_QUAD_FORCE_FIXUP")
    monkeypatch.setenv("POB_QUAD_SPLIT", "0")
    _per_step(name, B, T=4, seed=22)


def test_fixup_launch_mixed_forced(monkeypatch):
    """The mixed launch as one launch, split, and split with every wave forced through the
    fix-up launch: bit for bit the same states."""
    from po_brax_amd import jumpy
    envs = _envs()
    names = ["ant_heavenhell", "ant_gather", "ant_tag"]
    sizes = [6000, 5000, 4001]
    outs = []
    for split, force in (("0", "0"), ("1", "0"), ("1", "1")):  # one launch; split; split, all fixed up
        monkeypatch.setenv("POB_QUAD_SPLIT", split)
        monkeypatch.setenv("POB_QUAD_FORCE_FIXUP", force)
        mix = envs.create_mixed(names, episode_length=3, qp_dtype=torch.float16)
        key = jumpy.random_prngkey(9)
        ms = mix.reset(key, sizes)
        act = torch.empty((sum(sizes), 8), device="cuda")
        for t in range(4):
            jumpy.random_actions_(key, sum(sizes), 0, act)
            ms = mix.step_(ms, [a.contiguous() for a in mix.split_actions(act)])
        outs.append([(s.qp.pos.clone(), s.obs.clone(), s.reward.clone()) for s in ms])
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            for x, y in zip(a, b):
                assert torch.equal(x, y)


def test_split_launch_marks_are_out_of_band():
    """round 5 marked a wave for the fix-up launch with a signalling NaN in its first
    obs element, so an AUTORESET copy of a first_obs row holding that bit pattern would have sent
    an already stepped wave (in-place step) through the fix-up launch a second time.  The marks
    live in pob_state.ovf_mark now (ABI v8): the same pattern planted in the first first_obs row
    of every 16-env wave changes nothing -- per-step parity against the oracle through the
    autoresets that copy it into obs."""
    name, B, L = "ant_heavenhell", 16400, 2  # B > 16 384: the four-lane kernel's split launch
    env = _envs().create(name, batch_size=B, episode_length=L)
    keys = _keys(B, 31)
    s = env.reset(torch.from_numpy(keys).cuda())
    s.info["first_obs"].view(torch.int32)[::16, 0] = 0x7FA5A5A5
    o = orc.OracleEnv(name)
    planted = 0
    for t, act in enumerate(_actions(32, B, 4)):
        so = o.step(_state_np(s), act, flags=FLAGS, episode_length=L, nthreads=NT)
        s = env.step_(s, torch.from_numpy(act).cuda())
        compare_states(s, so, f"{name} B={B} step {t}")
        planted += int((s.obs.view(torch.int32)[::16, 0] == 0x7FA5A5A5).sum())
    assert planted >= 2 * (B // 16)  # steps 1 and 3 autoreset every env: the pattern is in obs


def test_step_without_mark_array_takes_one_launch():
    """A C caller that leaves pob_state.ovf_mark NULL gets the one-launch form of the four-lane
    kernel: the same bits as the split launch the engine's own states take."""
    import ctypes as C
    from po_brax_amd import _lib
    name, B, L = "ant_heavenhell", 16400, 3
    env = _envs().create(name, batch_size=B, episode_length=L)
    u = env.unwrapped
    keys = _keys(B, 41)
    a = env.reset(torch.from_numpy(keys).cuda())
    b = env.reset(torch.from_numpy(keys).cuda())
    flags = _lib.F_EPISODE | _lib.F_AUTORESET
    for t, act in enumerate(_actions(42, B, 3)):
        act = torch.from_numpy(act).cuda()
        a = env.step_(a, act)
        bufs = u._bufs_of(b)
        cs = u._cstate(bufs)
        cs.ovf_mark = None
        _lib.check(_lib.lib.pob_step(u._handle, B, C.byref(cs), C.c_void_p(act.data_ptr()), C.byref(cs), flags, L,
                                     C.c_void_p(_lib.stream_handle(u.device))))
        torch.cuda.synchronize()
        for x, y in ((a.qp.pos, b.qp.pos), (a.qp.rot, b.qp.rot), (a.qp.vel, b.qp.vel), (a.obs, b.obs),
                     (a.reward, b.reward), (a.aux["done"], b.aux["done"])):
            assert torch.equal(x.view(torch.int32), y.view(torch.int32)), f"step {t}"

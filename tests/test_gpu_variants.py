"""GPU parity of the engine variants: binary16 qp storage, the mixed-kind launch and the
stock brax ant's env surface.

* fp16 storage (BASELINE.json config 5): the kernels decode binary16 qp, compute in float32
  and round the new qp to binary16 (round-to-nearest-even).  Parity bar: starting from the
  GPU's own fp16 state, the oracle's float32 step on the decoded state, rounded to fp16
  with numpy, equals the GPU's fp16 qp BIT FOR BIT, and every float32 field (obs, reward,
  metrics) is bit-exact.  (There is no fp16 reference; the drift of an fp16-stored rollout
  against an fp32 one is a property of the storage format, reported by
  test_fp16_rollout_drift with its own tolerance.)
* mixed launch: one pob_step_mixed over HH + GA + TAG (+ ant) batches equals the per-kind
  pob_step launches bit for bit, in float32 and in fp16 storage.
"""
import numpy as np
import pytest
import torch

import orc
import pob_np as P

pytestmark = pytest.mark.gpu
NAMES = ["ant_heavenhell", "ant_gather", "ant_tag", "ant"]
QP = ("pos", "rot", "vel", "ang")


def _np(t):
    t = t.detach().cpu()
    if t.dtype == torch.bool:
        t = t.to(torch.float32)
    return t.numpy()


def _keys(B, seed=0):
    return P.split(P.prngkey(seed), B + 1)[1:]


def _state_np32(s):
    """GPU State (any qp dtype) -> float32 oracle state dict (fp16 decoded exactly)."""
    d = dict(pos=_np(s.qp.pos), rot=_np(s.qp.rot), vel=_np(s.qp.vel), ang=_np(s.qp.ang), obs=_np(s.obs),
             reward=_np(s.reward), done=_np(s.aux["done"]), rng=_np(s.aux["rng"]).astype(np.uint32),
             steps=_np(s.info["steps"]), truncation=_np(s.aux["truncation"]))
    for k in range(3):
        d[f"m{k}"] = _np(s.aux[f"m{k}"])
    fq = s.info["first_qp"]
    d.update(first_pos=_np(fq.pos), first_rot=_np(fq.rot), first_vel=_np(fq.vel), first_ang=_np(fq.ang),
             first_obs=_np(s.info["first_obs"]))
    return {k: np.ascontiguousarray(v.astype(np.float32) if v.dtype == np.float16 else v) for k, v in d.items()}


def _assert_fp16_step(g, o, what):
    for k in QP:
        gv = _np(getattr(g.qp, k))
        assert gv.dtype == np.float16, (what, k, gv.dtype)
        np.testing.assert_array_equal(gv.view(np.uint16), o[k].astype(np.float16).view(np.uint16),
                                      err_msg=f"{what}: {k} (fp16 bits)")
    for k in ("obs", "reward", "m0", "m1", "m2", "steps", "truncation", "done"):
        gv = _np(g.aux[k]) if k in ("done", "m0", "m1", "m2", "truncation") else (
            _np(g.info["steps"]) if k == "steps" else _np(getattr(g, k)))
        np.testing.assert_array_equal(gv.astype(np.float32), o[k], err_msg=f"{what}: {k}")
    np.testing.assert_array_equal(_np(g.aux["rng"]).astype(np.uint32), o["rng"], err_msg=f"{what}: rng")


@pytest.mark.parametrize("name", NAMES)
def test_fp16_storage_reset_and_step_parity(name):
    from po_brax_amd import envs
    B, T, L = 256, 25, 12
    env = envs.create(name, batch_size=B, episode_length=L, qp_dtype=torch.float16)
    keys = _keys(B, 3)
    s = env.reset(torch.from_numpy(keys).cuda())
    o = orc.OracleEnv(name).reset(keys, first=True)
    for k in QP:
        np.testing.assert_array_equal(_np(getattr(s.qp, k)).view(np.uint16), o[k].astype(np.float16).view(np.uint16),
                                      err_msg=f"reset {k}")
        np.testing.assert_array_equal(_np(getattr(s.info["first_qp"], k)).view(np.uint16),
                                      o[k].astype(np.float16).view(np.uint16), err_msg=f"reset first_{k}")
    np.testing.assert_array_equal(_np(s.obs), o["obs"])
    oe = orc.OracleEnv(name)
    rng = np.random.default_rng(5)
    n_done = 0
    for t in range(T):
        act = rng.uniform(-1, 1, (B, 8)).astype(np.float32)
        so = oe.step(_state_np32(s), act, flags=orc.F_EPISODE | orc.F_AUTORESET, episode_length=L)
        s = env.step(s, torch.from_numpy(act).cuda())
        _assert_fp16_step(s, so, f"{name} fp16 step {t}")
        n_done += int(so["done"].sum())
    assert n_done > 0  # the episode limit L forces autoresets from the fp16 first_qp


def test_fp16_rollout_drift():
    """fp16-stored vs fp32-stored rollout from the same fp16-representable start: the
    per-step rounding of the stored qp (relative 2^-11) is the only difference; report its
    effect after 10 steps (tolerance documented in DESIGN.md)."""
    from po_brax_amd import envs
    B = 1024
    e32 = envs.create("ant_tag", batch_size=B, episode_length=1000, auto_reset=False)
    e16 = envs.create("ant_tag", batch_size=B, episode_length=1000, auto_reset=False, qp_dtype=torch.float16)
    k = torch.from_numpy(_keys(B, 9)).cuda()
    s32, s16 = e32.reset(k), e16.reset(k)
    for f in QP:  # same start: the fp16 state, widened
        getattr(s32.qp, f).copy_(getattr(s16.qp, f).float())
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(10):
        a = torch.rand((B, 8), generator=g, device="cuda") * 2 - 1
        s32, s16 = e32.step(s32, a), e16.step(s16, a)
    alive = (s32.aux["done"] == 0) & (s16.aux["done"] == 0)
    d = (s32.qp.pos[:, :9] - s16.qp.pos[:, :9].float()).abs()[alive]
    med, p99, mx = d.median().item(), d.quantile(0.99).item(), d.max().item()
    print(f"fp16 storage, |pos drift| after 10 steps: median {med:.2e} p99 {p99:.2e} max {mx:.2e} m")
    # binary16 spacing is 2^-8 m at |x| in [4, 8): the rounding alone moves a body by up to
    # 2e-3 m per step, and contacts amplify it in a few envs -- the tolerance is statistical
    assert torch.isfinite(d).all() and med < 1e-2 and p99 < 0.1


@pytest.mark.parametrize("qp_dtype", [torch.float32, torch.float16])
def test_mixed_launch_equals_per_kind(qp_dtype):
    from po_brax_amd import envs
    names = ["ant_heavenhell", "ant_gather", "ant_tag", "ant"]
    sizes = [100, 64, 130, 37]  # ragged: segments end mid-block
    mix = envs.create_mixed(names, episode_length=9, qp_dtype=qp_dtype)
    single = [envs.create(n, batch_size=b, episode_length=9, qp_dtype=qp_dtype) for n, b in zip(names, sizes)]
    from po_brax_amd import jumpy
    key = jumpy.random_prngkey(21)
    ms = mix.reset(key, sizes)
    keys = jumpy.random_split(key, sum(sizes) + 1)[1:]
    ss = [e.reset(keys[o:o + b].contiguous()) for e, o, b in zip(single, mix.offsets(), sizes)]
    ak = jumpy.random_prngkey(4)
    act = torch.empty((sum(sizes), 8), device="cuda")
    for t in range(15):
        jumpy.random_actions_(ak, sum(sizes), 0, act)
        ms = mix.step(ms, act)
        ss = [e.step(s, a.contiguous()) for e, s, a in zip(single, ss, mix.split_actions(act))]
        for n, a, b in zip(names, ms, ss):
            for f in QP:
                assert torch.equal(getattr(a.qp, f), getattr(b.qp, f)), (t, n, f)
            for f in ("obs", "reward"):
                assert torch.equal(getattr(a, f), getattr(b, f)), (t, n, f)
            assert torch.equal(a.done, b.done), (t, n)
            assert torch.equal(a.aux["rng"], b.aux["rng"]), (t, n)
            for m in a.metrics:
                assert torch.equal(a.metrics[m], b.metrics[m]), (t, n, m)


def test_mixed_inplace_and_validation():
    from po_brax_amd import envs
    mix = envs.create_mixed(["ant_heavenhell", "ant_tag"])
    ms = mix.reset(torch.tensor([0, 3], dtype=torch.uint32), [64, 64])
    act = torch.zeros((128, 8), device="cuda")
    out = mix.step_(ms, act)
    assert out[0].qp.pos.data_ptr() == ms[0].qp.pos.data_ptr()
    with pytest.raises(ValueError):
        envs.MixedEnv([envs.create("ant_tag", batch_size=1), envs.create("ant_tag", batch_size=1,
                                                                         qp_dtype=torch.float16)])
    with pytest.raises(TypeError):
        envs.MixedEnv([envs.create("ant_tag", batch_size=1, eval_metrics=True)])


def test_stock_ant_env_surface():
    from po_brax_amd import envs, standard_observability_masks as M
    env = envs.create("ant", batch_size=8)
    assert env.observation_size == 87 and env.action_size == 8
    s = env.reset(torch.from_numpy(_keys(8)).cuda())
    assert "rng" not in s.info
    assert list(s.metrics) == ["reward_ctrl_cost", "reward_contact_cost", "reward_forward", "reward_survive"]
    s = env.step(s, torch.zeros((8, 8), device="cuda"))
    assert torch.all(s.metrics["reward_survive"] == 1)
    # the 'ant' masks index this observation
    pos = M.apply_mask(s.obs, M.POSITION["ant"])
    vel = M.apply_mask(s.obs, M.VELOCITY["ant"])
    cfrc = M.apply_mask(s.obs, M.CFRC["ant"])
    assert pos.shape == (8, 13) and vel.shape == (8, 14) and cfrc.shape == (8, 60)
    assert torch.equal(pos[:, 0], s.qp.pos[:, 0, 2])       # torso z
    assert torch.equal(vel[:, :3], s.qp.vel[:, 0])          # torso velocity


@pytest.mark.parametrize("B", [70, 9000, 16400])  # sixteen- / eight- / four-lane kernels, ragged tails
@pytest.mark.parametrize("qp_dtype", [torch.float32, torch.float16])
@pytest.mark.parametrize("name", NAMES)
def test_staged_load_equals_per_lane_load(name, qp_dtype, B, monkeypatch):
    """The opt-in LDS-staged state load (POB_STAGE=1) and the default per-lane loads give the
    same step bit for bit (autoreset chain, three steps, every output field)."""
    from po_brax_amd import envs
    env = envs.create(name, batch_size=B, episode_length=2, qp_dtype=qp_dtype)
    s0 = env.reset(torch.from_numpy(_keys(B, 21)).cuda())
    gen = torch.Generator(device="cuda").manual_seed(5)
    acts = [torch.rand((B, 8), device="cuda", generator=gen) * 2 - 1 for _ in range(3)]
    outs = []
    for stage in ("0", "1"):
        monkeypatch.setenv("POB_STAGE", stage)
        s = s0
        for a in acts:
            s = env.step(s, a)
        torch.cuda.synchronize()
        outs.append(s)
    a, b = outs
    for f in QP:
        assert torch.equal(getattr(a.qp, f), getattr(b.qp, f)), f
    assert torch.equal(a.obs, b.obs) and torch.equal(a.reward, b.reward) and torch.equal(a.done, b.done)
    for k in a.aux:
        if isinstance(a.aux[k], torch.Tensor) and k != "ovf_mark":  # (the split launch's scratch)
            assert torch.equal(a.aux[k], b.aux[k]), k


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather"])
def test_unaligned_state_uses_fallback_loads(name, monkeypatch):
    """qp tensors that are not 16-B aligned take the per-lane load path (no vector loads)
    even with the staged load enabled; results must equal the aligned (staged) path bit for
    bit."""
    monkeypatch.setenv("POB_STAGE", "1")
    from po_brax_amd import envs
    B = 70  # ragged: the last wave holds 6 envs
    env = envs.create(name, batch_size=B, episode_length=50)
    s = env.reset(torch.from_numpy(_keys(B, 13)).cuda())

    def shifted(t):  # same values, storage offset by one element -> 4-B aligned only
        buf = torch.empty(t.numel() + 1, dtype=t.dtype, device=t.device)
        v = buf[1:].view(t.shape)
        v.copy_(t)
        return v

    qp2 = type(s.qp)(shifted(s.qp.pos), shifted(s.qp.rot), shifted(s.qp.vel), shifted(s.qp.ang))
    assert qp2.pos.data_ptr() % 16 != 0
    s2 = s.replace(qp=qp2)
    act = torch.rand((B, 8), device="cuda") * 2 - 1
    a = env.step(s, act)
    b2 = env.step(s2, act)
    for f in QP:
        assert torch.equal(getattr(a.qp, f), getattr(b2.qp, f)), f
    assert torch.equal(a.obs, b2.obs) and torch.equal(a.reward, b2.reward)


@pytest.mark.parametrize("inplace", [False, True])
def test_typed_step_outputs(inplace):
    """The reference's dtypes come from the step kernel's typed outputs (C ABI v5), not
    conversion kernels: AntTag done bool + truncation int32, AntGather apples / bombs int32;
    each equals the conversion of the engine's float32 buffer, in single-kind and mixed
    launches, functional and in-place."""
    from po_brax_amd import envs
    B = 300
    keys = torch.from_numpy(_keys(3 * B, 31)).cuda()
    gen = torch.Generator(device="cuda").manual_seed(9)
    kinds = ["ant_tag", "ant_gather", "ant_heavenhell"]

    def check(name, s):
        a = s.aux
        if name == "ant_tag":
            assert s.done.dtype == torch.bool and torch.equal(s.done, a["done"] != 0)
            assert s.info["truncation"].dtype == torch.int32
            assert torch.equal(s.info["truncation"], a["truncation"].to(torch.int32))
        elif name == "ant_gather":
            for k, slot in (("apples", "m0"), ("bombs", "m1")):
                assert s.metrics[k].dtype == torch.int32 and torch.equal(s.metrics[k], a[slot].to(torch.int32)), k
        else:
            assert s.done.dtype == torch.float32

    mixed = envs.create_mixed(kinds, episode_length=3)
    ms = mixed.reset(torch.tensor([0, 31], dtype=torch.uint32), [B, B, B])
    for i, name in enumerate(kinds):
        env = envs.create(name, batch_size=B, episode_length=3)
        s = env.reset(keys[i * B:(i + 1) * B].contiguous())
        for _ in range(4):  # step 3 autoresets every env (done / truncation flip)
            act = torch.rand((B, 8), device="cuda", generator=gen) * 2 - 1
            s = env.step_(s, act) if inplace else env.step(s, act)
            check(name, s)
    for _ in range(4):
        acts = [torch.rand((B, 8), device="cuda", generator=gen) * 2 - 1 for _ in kinds]
        ms = mixed.step_(ms, acts) if inplace else mixed.step(ms, acts)
        for name, s in zip(kinds, ms):
            check(name, s)

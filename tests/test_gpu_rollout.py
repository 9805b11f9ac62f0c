"""GPU: a rollout replayed from a hipGraph (po_brax_amd.rollout) equals the same steps
launched one by one, bit for bit -- single-kind chains and the mixed fp16 launch."""
import pytest
import torch

from test_gpu_parity import _keys

pytestmark = pytest.mark.gpu


def _acts(T, B, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    return torch.rand((T, B, 8), generator=g, device="cuda") * 2 - 1


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_graph_rollout_equals_eager(name):
    from po_brax_amd import envs
    from po_brax_amd.rollout import GraphRollout
    B, T = 1000, 12
    keys = torch.from_numpy(_keys(B, 1)).cuda()
    e1, e2 = (envs.create(name, batch_size=B, episode_length=5) for _ in range(2))
    s1, s2 = e1.reset(keys), e2.reset(keys)
    acts = _acts(T, B, 0)
    for t in range(T):
        e1.step_(s1, acts[t])
    roll = GraphRollout(e2, s2, acts)
    roll.replay()
    torch.cuda.synchronize()
    for f in ("pos", "rot", "vel", "ang"):
        assert torch.equal(getattr(s1.qp, f), getattr(s2.qp, f)), f
    assert torch.equal(s1.obs, s2.obs) and torch.equal(s1.reward, s2.reward)
    assert torch.equal(s1.aux["done"], s2.aux["done"]) and torch.equal(s1.info["steps"], s2.info["steps"])
    # a second replay continues from the stepped state (new env-steps, same actions)
    for t in range(T):
        e1.step_(s1, acts[t])
    roll.replay()
    torch.cuda.synchronize()
    assert torch.equal(s1.qp.pos, s2.qp.pos) and torch.equal(s1.obs, s2.obs)


def test_graph_rollout_mixed_fp16():
    from po_brax_amd import envs, jumpy
    from po_brax_amd.rollout import GraphRollout
    names = ["ant_heavenhell", "ant_gather", "ant_tag"]
    sizes = [300, 200, 301]
    m1, m2 = (envs.create_mixed(names, episode_length=6, qp_dtype=torch.float16) for _ in range(2))
    key = jumpy.random_prngkey(2)
    s1, s2 = m1.reset(key, sizes), m2.reset(key, sizes)
    acts = _acts(9, sum(sizes), 3)
    for t in range(9):
        m1.step_(s1, acts[t])
    GraphRollout(m2, s2, acts).replay()
    torch.cuda.synchronize()
    for a, b in zip(s1, s2):
        assert torch.equal(a.qp.pos, b.qp.pos) and torch.equal(a.qp.rot, b.qp.rot) and torch.equal(a.obs, b.obs)


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_grouped_graph_rollout_equals_eager(name):
    """GraphRollout(groups=3): the batch's env groups stepped on their own streams (ragged
    split) equal the same steps launched one by one, bit for bit, including the typed
    public outputs of the whole batch's State."""
    from po_brax_amd import envs
    from po_brax_amd.rollout import GraphRollout
    B, T = 1001, 9
    keys = torch.from_numpy(_keys(B, 4)).cuda()
    e1, e2 = (envs.create(name, batch_size=B, episode_length=4) for _ in range(2))
    s1, s2 = e1.reset(keys), e2.reset(keys)
    acts = _acts(T, B, 7)
    for t in range(T):
        s1 = e1.step_(s1, acts[t])
    roll = GraphRollout(e2, s2, acts, groups=3)
    s2 = roll.replay()
    torch.cuda.synchronize()
    for f in ("pos", "rot", "vel", "ang"):
        assert torch.equal(getattr(s1.qp, f), getattr(s2.qp, f)), f
    assert torch.equal(s1.obs, s2.obs) and torch.equal(s1.reward, s2.reward)
    assert s1.done.dtype == s2.done.dtype and torch.equal(s1.done, s2.done)
    assert torch.equal(s1.info["steps"], s2.info["steps"])
    assert torch.equal(s1.info["truncation"], s2.info["truncation"])
    for k in s1.metrics:
        assert s1.metrics[k].dtype == s2.metrics[k].dtype and torch.equal(s1.metrics[k], s2.metrics[k]), k


def test_capture_survives_gc_of_dead_envs():
    """Regression for the driver's round-2 GPU suite failure (hipErrorStreamCaptureInvalidated
    in a GraphRollout capture): a cyclic-GC pass inside a global-mode capture finalises dead
    envs, and pob_env_destroy used to hipFree their tables there.  Now (1) an env has no
    env <-> System cycle, so dropping it frees it at once, and (2) pob_env_destroy never calls
    the HIP runtime (the frees are deferred to the next pob_env_create).  Both are checked:
    an env kept alive only by an explicit cycle is collected INSIDE a capture, and the captured
    steps replay equal to eager ones."""
    import gc
    import weakref
    from po_brax_amd import envs
    e = envs.create("ant_heavenhell", batch_size=8)
    ref = weakref.ref(e.unwrapped)
    del e
    assert ref() is None  # freed by reference counting: no cycle left behind
    dead = envs.create("ant_gather", batch_size=8).unwrapped
    dead._cycle = dead  # only the cyclic GC can free it
    dref = weakref.ref(dead)
    del dead
    B = 256
    keys = torch.from_numpy(_keys(B, 9)).cuda()
    e1, e2 = (envs.create("ant_tag", batch_size=B, episode_length=5) for _ in range(2))
    s1, s2 = e1.reset(keys), e2.reset(keys)
    acts = _acts(3, B, 11)
    s1 = e1.step_(s1, acts[0])
    s2 = e2.step_(s2, acts[0])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s2 = e2.step_(s2, acts[1])
        gc.collect()  # finalises the dead env (pob_env_destroy) in the middle of the capture
        s2 = e2.step_(s2, acts[2])
    assert dref() is None
    g.replay()
    for t in (1, 2):
        s1 = e1.step_(s1, acts[t])
    torch.cuda.synchronize()
    for f in ("pos", "rot", "vel", "ang"):
        assert torch.equal(getattr(s1.qp, f), getattr(s2.qp, f)), f
    assert torch.equal(s1.obs, s2.obs) and torch.equal(s1.done, s2.done)
    # the deferred tables are released by the next create or by pob_release_deferred (outside
    # any capture)
    from po_brax_amd import _lib
    doomed = envs.create("ant_tag", batch_size=8).unwrapped
    del doomed
    assert _lib.release_deferred() >= 1
    assert _lib.release_deferred() == 0


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_gather", "ant_tag"])
def test_gym_graph_rollout_equals_eager(name):
    """create_gym_env steps replayed from a hipGraph (rollout.GymGraphRollout: step kernel +
    device any-done + masked gym reset, wrappers.py:245-262) equal gym.step called eagerly,
    bit for bit, over episodes short enough that several gym resets (and key advances) happen
    inside the captured steps; a second replay continues from the first."""
    from po_brax_amd import envs
    from po_brax_amd.rollout import GymGraphRollout
    B, T = 300, 6
    g1, g2 = (envs.create_gym_env(name, batch_size=B, seed=5, episode_length=3) for _ in range(2))
    o1, o2 = g1.reset(), g2.reset()
    assert torch.equal(o1, o2)
    acts = _acts(T, B, 13)
    roll = GymGraphRollout(g2, acts)
    for rep in range(2):
        for t in range(T):
            o1, r1, d1, m1 = g1.step(acts[t])
        o2, r2, d2, m2 = roll.replay()
        torch.cuda.synchronize()
        assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(d1, d2), rep
        for f in ("pos", "rot", "vel", "ang"):
            assert torch.equal(getattr(g1._state.qp, f), getattr(g2._state.qp, f)), (rep, f)
        assert torch.equal(g1._key, g2._key), rep
        for k in m1:
            assert torch.equal(m1[k], m2[k]), (rep, k)


def test_gym_graph_rollout_refuses_host_bookkeeping_and_stale_buffers():
    """An eval_metrics gym (EvalGymWrapper: host-side queue count and growth, forwarded
    attributes) is refused at construction instead of being captured with a queue that replay
    never advances; replaying after gym.reset() (new state and key buffers) raises instead of
    silently stepping the captured, stale buffers."""
    from po_brax_amd import envs
    from po_brax_amd.rollout import GymGraphRollout
    B = 64
    acts = _acts(2, B, 17)
    ev = envs.create_gym_env("ant_tag", batch_size=B, seed=1, episode_length=3, eval_metrics=True)
    ev.reset()
    with pytest.raises(NotImplementedError, match="EvalGymWrapper"):
        GymGraphRollout(ev, acts)
    g = envs.create_gym_env("ant_tag", batch_size=B, seed=1, episode_length=3)
    g.reset()
    roll = GymGraphRollout(g, acts)
    roll.replay()
    g.reset()
    with pytest.raises(RuntimeError, match="rebuild"):
        roll.replay()
    torch.cuda.synchronize()


@pytest.mark.parametrize("name", ["ant_heavenhell", "ant_tag"])
def test_policy_rollout_equals_eager(name):
    """rollout.PolicyRollout: an MLP policy (hipBLASLt GEMMs + tanh) and the fused step
    captured together per step, replayed from one graph, equal the same loop run eagerly --
    observations, actions, rewards, dones and the final state, bit for bit, over episodes
    short enough to autoreset inside the unroll; a second replay continues from the first."""
    from po_brax_amd import envs
    from po_brax_amd.rollout import PolicyRollout
    B, T = 512, 7
    keys = torch.from_numpy(_keys(B, 21)).cuda()
    e1, e2 = (envs.create(name, batch_size=B, episode_length=4) for _ in range(2))
    s1, s2 = e1.reset(keys), e2.reset(keys)
    g = torch.Generator(device="cuda").manual_seed(5)
    D = e1.observation_size
    W1 = torch.randn((D, 64), generator=g, device="cuda") * 0.1
    W2 = torch.randn((64, 8), generator=g, device="cuda") * 0.3

    def policy(obs):
        return torch.tanh(torch.tanh(obs @ W1) @ W2)

    roll = PolicyRollout(e2, s2, policy, T)
    for rep in range(2):
        obs_l, act_l, rew_l, done_l = [], [], [], []
        for t in range(T):
            obs_l.append(s1.obs.clone())
            a = policy(s1.obs)
            act_l.append(a)
            s1 = e1.step_(s1, a)
            rew_l.append(s1.reward.clone())
            done_l.append(s1.aux["done"].clone())
        s2 = roll.replay()
        torch.cuda.synchronize()
        assert torch.equal(torch.stack(obs_l), roll.obs), rep
        assert torch.equal(torch.stack(act_l), roll.actions), rep
        assert torch.equal(torch.stack(rew_l), roll.reward) and torch.equal(torch.stack(done_l), roll.done), rep
        for f in ("pos", "rot", "vel", "ang"):
            assert torch.equal(getattr(s1.qp, f), getattr(s2.qp, f)), (rep, f)
    assert float(roll.done.sum()) > 0  # autoresets happened inside the unroll

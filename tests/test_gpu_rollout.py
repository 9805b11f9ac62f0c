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

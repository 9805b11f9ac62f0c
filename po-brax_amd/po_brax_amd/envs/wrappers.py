"""Wrappers of ``po_brax/envs/wrappers.py`` and the brax wrappers it builds on.

The wrapper objects do not run anything themselves: they fold into flags of the one fused
step kernel (``pob_step``) and into the masked reset kernel (``pob_reset_where_done``), so a
wrapped step is still ONE device launch (two for the autoresetting gym/randomized
wrappers) and never synchronises the host:

==========================================  =============================================
reference                                    here
==========================================  =============================================
ActionRepeatWrapper  wrappers.py:16-24       rebuilds the engine with dt, substeps x ar
brax EpisodeWrapper [ext]                     POB_F_EPISODE (steps, truncation, time limit)
brax VmapWrapper [ext] / VectorWrapper :13    pass-through (batching is native)
brax AutoResetWrapper [ext] / alias :27       POB_F_AUTORESET (first_qp / first_obs)
RandomizedAutoResetWrapperNaive :30-52        POB_F_ZERO_STEPS_ON_DONE + reset(info.rng)
RandomizedAutoResetWrapperOnTerminal :55-80   same outputs as Naive (cond only skips work)
RandomizedAutoResetWrapperCached :83-123      host step counter refreshes first_qp/obs
VmapGymWrapper :126-172                       gym VectorEnv API over device tensors
AutoresetVmapGymWrapper :240-262              device-side any(done) + gym-key reset
AutoresetGymWrapper :232-237                  single env, full reset on done
EvalGymWrapper :175-229                       device-side episode statistics
brax EvalWrapper [ext]                        device-side episode metrics
==========================================  =============================================
"""
from __future__ import annotations

import math
from typing import Optional

import numpy as np
import torch

from .. import _lib
from .. import jumpy as jp
from .env import Env, State, Wrapper, QP, F_EPISODE, F_AUTORESET, F_ZERO


class ActionRepeatWrapper(Wrapper):
    """Just change action duration (wrappers.py:16-24): dt and substeps x action_repeat."""

    def __init__(self, env: Env, action_repeat: int):
        super().__init__(env)
        if hasattr(self.unwrapped, "_set_action_repeat"):
            self.unwrapped._set_action_repeat(action_repeat)
        self.action_repeat = action_repeat


class EpisodeWrapper(Wrapper):
    """brax EpisodeWrapper: info['steps'] += 1, done at episode_length, info['truncation']."""

    def __init__(self, env: Env, episode_length: int, action_repeat: int = 1):
        super().__init__(env)
        if action_repeat != 1:
            raise NotImplementedError("EpisodeWrapper(action_repeat != 1): use ActionRepeatWrapper "
                                      "(po_brax.envs.create passes 1, __init__.py:62)")
        if episode_length <= 0:
            raise ValueError("episode_length must be positive")
        self.episode_length = int(episode_length)
        self.action_repeat = action_repeat

    def _chain_reset(self, rng, episode, first):
        return self.env._chain_reset(rng, True, first)

    def _chain_step(self, state, action, flags, episode_length, inplace):
        if flags & F_EPISODE:
            raise NotImplementedError("nested EpisodeWrapper")
        return self.env._chain_step(state, action, flags | F_EPISODE, self.episode_length, inplace)


class VmapWrapper(Wrapper):
    """brax VmapWrapper: batching is native to the engine -- a pass-through."""


VectorWrapper = VmapWrapper  # wrappers.py:13


class AutoResetWrapper(Wrapper):
    """brax AutoResetWrapper: reset done envs to info['first_qp'] / info['first_obs']."""

    def _chain_reset(self, rng, episode, first):
        return self.env._chain_reset(rng, episode, True)

    def _chain_step(self, state, action, flags, episode_length, inplace):
        if flags & F_EPISODE:
            raise NotImplementedError("EpisodeWrapper outside AutoResetWrapper is not supported")
        return self.env._chain_step(state, action, flags | F_AUTORESET, episode_length, inplace)


class RandomizedAutoResetWrapperNaive(Wrapper):
    """wrappers.py:30-52: re-sample ``reset(state.info['rng'])`` for envs that are done."""

    def _chain_step(self, state, action, flags, episode_length, inplace):
        if flags & F_EPISODE:
            raise NotImplementedError("EpisodeWrapper outside the autoreset wrapper is not supported")
        s = self.env._chain_step(state, action, flags | F_ZERO, episode_length, inplace)
        self.unwrapped._reset_where_done(s, _lib.RESET_OWN)
        return s


class RandomizedAutoResetWrapperOnTerminal(RandomizedAutoResetWrapperNaive):
    """wrappers.py:55-80: identical outputs (the cond only skips work when nothing is done;
    the masked reset kernel skips every env that is not done anyway)."""


class RandomizedAutoResetWrapperCached(Wrapper):
    """wrappers.py:83-123: first_qp / first_obs refreshed from reset(split(rng)[1]) every
    ``n_steps_between_updates`` calls of ``step`` (a host-side counter, as in the reference)."""

    def __init__(self, env: Env, n_steps_between_updates: int = 200):
        super().__init__(env)
        self.n_steps_between_updates = n_steps_between_updates
        self.steps = 0

    def _chain_reset(self, rng, episode, first):
        return self.env._chain_reset(rng, episode, True)

    def _chain_step(self, state, action, flags, episode_length, inplace):
        if flags & F_EPISODE:
            raise NotImplementedError("EpisodeWrapper outside the autoreset wrapper is not supported")
        self.steps += 1
        if self.steps % self.n_steps_between_updates == 0:
            rng = state.info["rng"]
            ks = jp.random_split_batch(rng, 2)  # (B, 2, 2)
            fresh = self.env._chain_reset(ks[:, 1].contiguous(), False, False)
            fq = state.info["first_qp"]
            for dst, src in ((fq.pos, fresh.qp.pos), (fq.rot, fresh.qp.rot), (fq.vel, fresh.qp.vel),
                             (fq.ang, fresh.qp.ang), (state.info["first_obs"], fresh.obs)):
                dst.copy_(src)
            rng.copy_(ks[:, 0])
        return self.env._chain_step(state, action, flags | F_AUTORESET, episode_length, inplace)


class EvalWrapper(Wrapper):
    """brax EvalWrapper [ext] (``create(..., eval_metrics=True)``, __init__.py:69-70): per-env
    running episode metrics and completed-episode totals, restated from brax <= 0.0.12:

        nstate.metrics['reward'] = nstate.reward
        completed_episodes_steps += sum(nstate.info['steps'] * nstate.done)
        current = tree_multimap(+, current, nstate.metrics)
        completed_episodes += sum(nstate.done)
        completed_metrics = tree_multimap(a + sum(b * done), completed_metrics, current)
        current = current * (1 - nstate.done)

    The step's metric keys must equal the reset's, as jax's ``tree_multimap`` requires:
    AntHeavenHell adds ``hits`` on step (ant_heavenhell.py:122), so there the reference raises
    and so does this wrapper (ValueError).  Device tensors, no host sync; sums are float32."""

    def _chain_reset(self, rng, episode, first):
        s = self.env._chain_reset(rng, episode, first)
        s.metrics["reward"] = s.reward
        cur = {k: torch.zeros_like(v, dtype=torch.float32) for k, v in s.metrics.items()}
        s.info["eval_metrics"] = {
            "current_episode_metrics": cur,
            "completed_episodes_metrics": {k: torch.zeros((), device=v.device) for k, v in cur.items()},
            "completed_episodes": torch.zeros((), device=s.reward.device),
            "completed_episodes_steps": torch.zeros((), device=s.reward.device),
        }
        return s

    def _chain_step(self, state, action, flags, episode_length, inplace):
        em = state.info.pop("eval_metrics")
        ns = self.env._chain_step(state, action, flags, episode_length, inplace)
        state.info["eval_metrics"] = em
        ns.metrics["reward"] = ns.reward
        done = ns.aux["done"] if "done" in ns.aux else ns.done.to(torch.float32)
        if set(ns.metrics) != set(em["current_episode_metrics"]):
            raise ValueError(f"EvalWrapper: step metrics {sorted(ns.metrics)} do not match the reset's "
                             f"{sorted(em['current_episode_metrics'])} (jax tree_multimap structure mismatch)")
        cur = {k: em["current_episode_metrics"][k] + ns.metrics[k].to(torch.float32)
               for k in em["current_episode_metrics"]}
        comp = {k: em["completed_episodes_metrics"][k] + (cur[k] * done).sum() for k in cur}
        steps = ns.info.get("steps")
        nem = {
            "current_episode_metrics": {k: v * (1.0 - done) for k, v in cur.items()},
            "completed_episodes_metrics": comp,
            "completed_episodes": em["completed_episodes"] + done.sum(),
            "completed_episodes_steps": em["completed_episodes_steps"]
            + ((steps * done).sum() if steps is not None else 0.0),
        }
        ns.info["eval_metrics"] = nem
        return ns


# --------------------------------------------------------------------------- gym side
class Box:
    """Minimal gym.spaces.Box (gym is not a dependency of the engine)."""

    def __init__(self, low, high, shape=None, dtype="float32", device="cpu"):
        self.low, self.high = np.asarray(low, dtype=dtype), np.asarray(high, dtype=dtype)
        self.shape = tuple(shape if shape is not None else self.low.shape)
        self.dtype = np.dtype(dtype)
        self._device = device
        self._gen = torch.Generator(device="cpu").manual_seed(0)

    def sample(self) -> torch.Tensor:
        lo, hi = torch.as_tensor(self.low), torch.as_tensor(self.high)
        u = torch.rand(self.shape, generator=self._gen, dtype=torch.float32)
        lo = torch.where(torch.isfinite(lo), lo, torch.full_like(lo, -1.0))
        hi = torch.where(torch.isfinite(hi), hi, torch.full_like(hi, 1.0))
        return (lo + u * (hi - lo)).to(self._device)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class VmapGymWrapper:
    """wrappers.py:126-172: gym VectorEnv API for a batched env (device tensors in/out).

    ``shard`` (engine extension, po_brax_amd.sharding.Shard): this process runs rows
    [shard.lo, shard.hi) of a global batch of ``batch_size`` envs; reset keys are that
    slice of ``split(key, batch_size + 1)[1:]`` and the gym key follows the global chain, so
    the ranks together reproduce the single-process run bit for bit."""

    def __init__(self, env: Env, batch_size: int, seed: int = 0, backend: Optional[str] = None,
                 shard=None):
        self._env = env
        self.metadata = {"render.modes": ["human", "rgb_array"],
                         "video.frames_per_second": 1 / self._env.sys.config.dt}
        if shard is not None and shard.total != int(batch_size):
            raise ValueError(f"shard.total {shard.total} != batch_size {batch_size}")
        self._shard = shard
        self.total_envs = int(batch_size)
        self.num_envs = shard.size if shard is not None else int(batch_size)
        self.backend = backend
        self.device = env.unwrapped.device
        self._state = None
        self.seed(seed)
        D, A = self._env.observation_size, self._env.action_size
        self.single_observation_space = Box(-np.inf * np.ones(D), np.inf * np.ones(D), device=self.device)
        self.observation_space = Box(-np.inf * np.ones((self.num_envs, D)), np.inf * np.ones((self.num_envs, D)),
                                     device=self.device)
        self.single_action_space = Box(-np.ones(A), np.ones(A), device=self.device)
        self.action_space = Box(-np.ones((self.num_envs, A)), np.ones((self.num_envs, A)), device=self.device)

    def seed(self, seed: int = 0):
        self._key = jp.random_prngkey(seed, device=self.device)

    def _reset(self, key):
        if self._shard is None:
            keys = jp.random_split(key, self.num_envs + 1)
            state = self._env._chain_reset(keys[1:].contiguous(), False, False)
            return state, state.obs, keys[0].contiguous()
        num, first, count = self._shard.gym_key_rows()
        keys = jp.random_split_rows(key, num, first, count)
        state = self._env._chain_reset(keys, False, False)
        return state, state.obs, jp.random_split_rows(key, num, 0, 1)[0].contiguous()

    def reset(self):
        self._state, obs, self._key = self._reset(self._key)
        return obs

    def step(self, action):
        self._state = self._env._chain_step(self._state, action, 0, 0, True)
        s = self._state
        return s.obs, s.reward, s.done, s.metrics

    def render(self, mode="human"):
        raise NotImplementedError("rendering is out of scope for the accelerated path")

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self._env, name)


class AutoresetVmapGymWrapper(VmapGymWrapper):
    """wrappers.py:240-262, with the ``if done.any()`` decided on the device: the step
    kernel ORs into an any-done word, the masked reset kernel re-samples the done envs from
    ``split(gym_key, B+1)[1:]`` and advances the gym key only when something was done.
    Sharded (``shard``), the any-done word is all-reduced (MAX) over the ranks first and the
    keys are this rank's rows of ``split(gym_key, B_total + 1)`` (sharding.py)."""

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        # two any-done words (16 B apart), used by alternate steps: step k's kernel ORs into
        # word k % 2 and its masked reset reads that word and zeroes the other one for step
        # k + 1 (pob_state.any_done_clear), so no fill kernel runs per step
        self._words = torch.zeros(8, dtype=torch.uint32, device=self.device)
        self._parity = 0
        self._any = self._words[0:4]
        self._key2 = torch.empty(2, dtype=torch.uint32, device=self.device)

    def step(self, action):
        from ..sharding import all_reduce_any_done
        self._step_local(action)
        sh = self._shard
        if sh is not None:  # (a no-op without a process group)
            all_reduce_any_done(self._any, sh.group)
        return self._autoreset()

    # the two halves of step (the cross-rank any-done reduction goes between them)
    def _step_local(self, action):
        s = self._state
        p = self._parity
        self._any = self._words[4 * p:4 * p + 4]  # zero: initial, or cleared by the last reset
        nxt = self._words[4 * (1 - p):4 * (1 - p) + 4]
        s.aux["any_done"], s.aux["any_done_clear"] = self._any, nxt
        self._state = s = self._env._chain_step(s, action, 0, 0, True)
        s.aux["any_done"], s.aux["any_done_clear"] = self._any, nxt
        return s

    def _autoreset(self):
        s, sh = self._state, self._shard
        self._env.unwrapped._reset_where_done(s, _lib.RESET_GYM, self._key, self._key2,
                                              total=self.total_envs, first=sh.lo if sh is not None else 0)
        self._key, self._key2 = self._key2, self._key
        self._parity ^= 1
        return s.obs, s.reward, s.done, s.metrics


class AutoresetGymWrapper:
    """wrappers.py:232-237 (brax GymWrapper for one env): full reset when done."""

    def __init__(self, env: Env, seed: int = 0, backend: Optional[str] = None):
        self._env = env
        self.device = env.unwrapped.device
        self.metadata = {"render.modes": ["human", "rgb_array"],
                         "video.frames_per_second": 1 / env.sys.config.dt}
        self.backend = backend
        self._state = None
        D, A = env.observation_size, env.action_size
        self.observation_space = Box(-np.inf * np.ones(D), np.inf * np.ones(D), device=self.device)
        self.action_space = Box(-np.ones(A), np.ones(A), device=self.device)
        self.seed(seed)

    def seed(self, seed: int = 0):
        self._key = jp.random_prngkey(seed, device=self.device)

    def _reset(self, key):
        k = jp.random_split(key, 2)
        state = self._env._chain_reset(k[1].contiguous(), False, False)
        return state, state.obs, k[0].contiguous()

    def reset(self):
        self._state, obs, self._key = self._reset(self._key)
        return obs

    def step(self, action):
        self._state = self._env._chain_step(self._state, action, 0, 0, False)
        s = self._state
        obs, reward, done, info = s.obs, s.reward, s.done, s.metrics
        if bool(done):  # host sync, as the reference's `if done:`
            self._state, obs, self._key = self._reset(self._key)
        return obs, reward, done, info

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return getattr(self._env, name)


class EvalGymWrapper:
    """wrappers.py:175-229: episode return / discounted return / length statistics.

    The reference appends every finished episode's return, discounted return and length to
    the queues ``r_q``, ``dr_q``, ``l_q`` (each seeded with NaN) after a host-side
    ``if d.any(): d.nonzero()`` per step, and ``get_stats`` is the nanmean of each queue.
    Here the queues are device buffers filled without a host sync: the finished episodes'
    values are scattered in env order (the order of ``d.nonzero()``) to
    ``count + cumsum(d) - 1``, the other envs to a discard slot past the end.  The host reads
    the device count only when the buffer might overflow (at most ``num_envs`` entries per
    step): the capacity starts at 64 steps' worth and grows whenever fewer than 16 steps of
    room remain after a read, so reads stay at most one per 16 steps.  Returns are float32 like the
    reference's ``zeros_like(obs[..., -1])`` buffers; lengths are int32."""

    def __init__(self, env, discount: float = 1.0, capacity: int = 1 << 16):
        self.env = env
        self._discount = float(discount)
        self.num_envs = getattr(env, "num_envs", 1)
        self._cap0 = int(capacity)

    def __getattr__(self, name):
        if name.startswith("__") or name in ("env", "num_envs"):
            raise AttributeError(name)
        return getattr(self.env, name)

    def reset(self, **kwargs):
        o = self.env.reset(**kwargs)
        like = torch.atleast_1d(o[..., -1])
        dev = like.device
        n = like.shape[0]
        self.episode_returns = torch.zeros_like(like, dtype=torch.float32)
        self.discounted_episode_returns = torch.zeros_like(like, dtype=torch.float32)
        self.episode_lengths = torch.zeros_like(like, dtype=torch.int32)
        self.current_discount = torch.ones_like(like, dtype=torch.float32)
        cap = max(self._cap0, 64 * n)  # room for 64 steps in which every env finishes
        self._q = torch.zeros((3, cap + 1), dtype=torch.float32, device=dev)  # + discard slot
        self._lq = torch.zeros(cap + 1, dtype=torch.int32, device=dev)
        self._count = torch.zeros((), dtype=torch.int64, device=dev)
        self._known, self._since = 0, 0  # host lower bound of the count, steps since read
        return o

    def _ensure_room(self, n: int) -> None:
        cap = self._lq.shape[0] - 1
        if self._known + (self._since + 1) * n <= cap:
            return
        self._known, self._since = int(self._count), 0  # host sync (rare)
        if self._known + 16 * n > cap:  # grow early: >= 16 steps of room after every sync
            new = max(2 * cap, self._known + 64 * n)
            q = torch.zeros((3, new + 1), dtype=self._q.dtype, device=self._q.device)
            lq = torch.zeros(new + 1, dtype=self._lq.dtype, device=self._lq.device)
            q[:, :self._known] = self._q[:, :self._known]
            lq[:self._known] = self._lq[:self._known]
            self._q, self._lq = q, lq

    def step(self, action):
        o, r, d, info = self.env.step(action)
        r = torch.atleast_1d(r).to(torch.float32)
        db = torch.atleast_1d(d) != 0
        n = db.shape[0]
        self.episode_returns += r
        self.episode_lengths += 1
        self.discounted_episode_returns += r * self.current_discount
        self.current_discount *= self._discount
        self._ensure_room(n)
        cap = self._lq.shape[0] - 1
        slot = torch.where(db, self._count + torch.cumsum(db, 0, dtype=torch.int64) - 1,
                           torch.full_like(self._count, cap).expand(n))
        self._q[0].scatter_(0, slot, self.episode_returns)
        self._q[1].scatter_(0, slot, self.discounted_episode_returns)
        self._lq.scatter_(0, slot, self.episode_lengths)
        self._count += db.sum()
        self._since += 1
        keep = ~db
        self.episode_returns *= keep
        self.discounted_episode_returns *= keep
        self.episode_lengths *= keep
        self.current_discount = torch.where(db, torch.ones_like(self.current_discount), self.current_discount)
        return o, r, d, info

    def _queues(self):
        c = int(self._count)
        return self._q[0, :c].cpu().numpy(), self._q[1, :c].cpu().numpy(), self._lq[:c].cpu().numpy()

    @property
    def r_q(self):
        return [math.nan] + list(self._queues()[0])

    @property
    def dr_q(self):
        return [math.nan] + list(self._queues()[1])

    @property
    def l_q(self):
        return [math.nan] + list(self._queues()[2])

    def get_stats(self):
        r, dr, ln = self._queues()
        mean = lambda v: np.float32(np.mean(v.astype(np.float64))) if len(v) else np.float32(np.nan)  # noqa: E731
        return {"charts/mean_episodic_return": np.array(mean(r)),
                "charts/mean_discounted_episodic_return": np.array(mean(dr)),
                "charts/mean_episodic_length": np.array(mean(ln))}

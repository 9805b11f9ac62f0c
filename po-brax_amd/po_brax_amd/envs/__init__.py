"""Env registry and factories -- the drop-in surface of ``po_brax.envs`` (__init__.py:29-121).

The three partially observable Ant tasks and the stock brax ``ant`` (whose 87-dim
observation the masks of standard_observability_masks.py index) run on the MI355X engine;
the other stock brax envs the reference re-exports (``fetch``, ``humanoid`` ...) are out of
this path's scope and raise ``NotImplementedError`` when created.  ``create_mixed`` (an
engine extension) steps several env batches with one kernel launch.
"""
from __future__ import annotations

import functools
from typing import Callable, Optional

from .env import Env, State, QP, Wrapper, System
from .ant_heavenhell import AntHeavenHellEnv
from .ant_gather import AntGatherEnv
from .ant_tag import AntTagEnv
from .ant import AntEnv
from .mixed import MixedEnv
from . import wrappers
from .wrappers import (VmapGymWrapper, AutoresetVmapGymWrapper, AutoresetGymWrapper, EvalGymWrapper,
                       ActionRepeatWrapper, EpisodeWrapper, VmapWrapper, VectorWrapper, AutoResetWrapper,
                       EvalWrapper, RandomizedAutoResetWrapperNaive, RandomizedAutoResetWrapperOnTerminal,
                       RandomizedAutoResetWrapperCached)

HAI_ACTION_REPEAT = 6  # __init__.py:28 (unused by the reference too)


def _stock(name):
    def make(**kwargs):
        raise NotImplementedError(
            f"stock brax env '{name}' is not part of the accelerated po-brax path "
            "(only ant_heavenhell, ant_gather and ant_tag run on the MI355X engine)")
    return make


_envs = {
    'ant': AntEnv,
    'ant_tag': AntTagEnv,
    'ant_heavenhell': AntHeavenHellEnv,
    'ant_gather': AntGatherEnv,
    **{n: _stock(n) for n in ('fast', 'fetch', 'grasp', 'halfcheetah', 'hopper', 'humanoid',
                              'humanoidstandup', 'inverted_pendulum', 'inverted_double_pendulum',
                              'reacher', 'reacherangle', 'ur5e', 'walker2d')},
}


def create(env_name: str,
           episode_length: int = 1000,
           action_repeat: int = 1,
           auto_reset: bool = True,
           batch_size: Optional[int] = None,
           eval_metrics: bool = False,
           **kwargs) -> Env:
    """Creates an Env (po_brax/envs/__init__.py:50-72)."""
    env = _envs[env_name](**kwargs)
    if action_repeat is not None:
        env = wrappers.ActionRepeatWrapper(env, action_repeat=action_repeat)
    if episode_length is not None:
        env = wrappers.EpisodeWrapper(env, episode_length, 1)
    if batch_size:
        env = wrappers.VmapWrapper(env)
    if auto_reset:
        env = wrappers.AutoResetWrapper(env)
    if eval_metrics:
        env = wrappers.EvalWrapper(env)
    return env


def create_mixed(env_names, episode_length: int = 1000, action_repeat: int = 1,
                 auto_reset: bool = True, **kwargs) -> MixedEnv:
    """MixedEnv of ``create(name, batch_size=1, ...)`` chains (one per name); batch sizes are
    given to ``MixedEnv.reset``.  ``kwargs`` (e.g. ``qp_dtype``, ``device``) go to every env."""
    return MixedEnv([create(n, episode_length=episode_length, action_repeat=action_repeat,
                            auto_reset=auto_reset, batch_size=1, **kwargs) for n in env_names])


def create_fn(env_name: str, **kwargs) -> Callable[..., Env]:
    """Returns a function that when called, creates an Env (:75-77)."""
    return functools.partial(create, env_name, **kwargs)


def create_gym_env(env_name: str,
                   batch_size: Optional[int] = None,
                   seed: int = 0,
                   backend: Optional[str] = None,
                   **kwargs):
    """Creates a gym Env / VectorEnv with gym-side autoreset (:98-121).

    Engine extension: ``shard=po_brax_amd.sharding.Shard(batch_size, world, rank, group)``
    runs this process's slice of the batch (one process per GPU) with the reference's
    global key chain and a cross-rank any-done (sharding.py)."""
    kwargs['auto_reset'] = False
    eval_metrics = kwargs.pop('eval_metrics', False)
    discount = kwargs.pop('discount', 1.)
    shard = kwargs.pop('shard', None)
    environment = create(env_name=env_name, batch_size=batch_size, **kwargs)
    if batch_size is None:
        if shard is not None:
            raise ValueError('`shard` needs a batched env (batch_size)')
        e = AutoresetGymWrapper(environment, seed=seed, backend=backend)
    else:
        if batch_size <= 0:
            raise ValueError('`batch_size` should either be None or a positive integer.')
        e = AutoresetVmapGymWrapper(environment, batch_size, seed=seed, backend=backend, shard=shard)
    if eval_metrics:
        e = EvalGymWrapper(e, discount=discount)
    return e

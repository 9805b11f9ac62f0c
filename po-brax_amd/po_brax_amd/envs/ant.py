"""Stock brax Ant (``po_brax.envs._envs['ant']``, po_brax/envs/__init__.py:30).

The reference re-exports brax's own ``Ant`` (brax <= 0.0.12 ``envs/ant.py`` [ext]); the
observability masks of ``po_brax/standard_observability_masks.py:7,26,62`` index its
87-dim observation.  It shares the ant, the physics kernel and the contact model with
the po-envs: bodies 0-8 ant + 9 Ground, no arena.

  reset  ``rng, rng1, rng2 = split(rng, 3)``; qpos = default_angle + U(rng1, +-0.1),
         qvel = U(rng2, +-0.1); ``default_qp``; obs from ``sys.info``; reward = done = 0
  step   forward = (x_torso' - x_torso) / dt; ctrl = .5 sum(a^2);
         contact = .5e-3 sum(clip(contact.vel, -1, 1)^2); survive = 1;
         reward = forward - ctrl - contact + survive; done = z_torso < .2 or > 1
  obs    qp.pos[0, 2:] (1) | rot[0] (4) | joint angles (8) | vel[0] (3) | ang[0] (3) |
         joint vels (8) | clip(contact.vel) (10x3) | clip(contact.ang) (10x3) = 87

The brax State of this env carries no ``info['rng']`` (it lives in ``state.aux``).
"""
from __future__ import annotations

import torch

from .ant_heavenhell import ANT_BODIES, _common_params
from .env import PoBraxEnv


class AntEnv(PoBraxEnv):
    """Trains an ant to run in the +x direction (brax.envs.ant.Ant)."""

    kind = "ant"
    body_names = ANT_BODIES
    slot_names = ("reward_ctrl_cost", "reward_contact_cost", "reward_forward")
    reset_metrics = ("reward_ctrl_cost", "reward_contact_cost", "reward_forward")
    step_metrics = ("reward_ctrl_cost", "reward_contact_cost", "reward_forward")
    info_rng = False

    def __init__(self, **kwargs):
        super().__init__(**kwargs)

    def _set_params(self, p: dict) -> None:
        _common_params(self._params, p)

    def _metric_dtypes(self, metrics, after_step):
        # reward_survive is a constant (1 after a step, 0 after reset): one cached tensor per
        # batch shape, so that a step launches no fill kernel
        ref = metrics["reward_forward"]
        key = (after_step, tuple(ref.shape), ref.device)
        cache = self.__dict__.setdefault("_survive", {})
        if key not in cache:
            cache[key] = torch.ones_like(ref) if after_step else torch.zeros_like(ref)
        return {**metrics, "reward_survive": cache[key]}

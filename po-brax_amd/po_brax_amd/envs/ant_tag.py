"""AntTag: tag a scripted, randomly evading (frozen, non-colliding) target.

Mirrors ``po_brax/envs/ant_tag.py`` (constructor :38-61, reset :63-105 incl. the
rejection-sampled spawn, step :107-127, adversary :129-146, obs :148-181) on the fused
HIP kernels.  Body order: 0-8 ant, 9 Ground, 10 Target, 11 Arena.  ``done`` is bool
after a step (``logical_or(dead, tag)``, ant_tag.py:127) and float32 after reset.
"""
from __future__ import annotations

from typing import Sequence

import torch

from .ant_heavenhell import ANT_BODIES, _common_params
from .env import PoBraxEnv


class AntTagEnv(PoBraxEnv):
    """
    Args:
        tag_radius: radius within which the target is tagged (ends the episode)
        visible_radius: radius within which the target is visible
        target_step: length of the target's evasive steps
        min_spawn_distance: minimum spawn distance of the target from the ant
        cage_xy: arena half extents
        dying_cost: reward on death
    """

    kind = "ant_tag"
    body_names = ANT_BODIES + ("Target", "Arena")
    slot_names = ("hits",)
    reset_metrics = ("hits",)
    step_metrics = ("hits",)
    done_dtype = torch.bool

    def __init__(self,
                 tag_radius: float = 1.5,
                 visible_radius: float = 3.,
                 target_step: float = 0.5,
                 min_spawn_distance: float = 5.,
                 cage_xy: Sequence[float] = (4.5, 4.5),
                 dying_cost: float = -1.,
                 **kwargs):
        super().__init__(tag_radius=tag_radius, visible_radius=visible_radius,
                         target_step=target_step, min_spawn_distance=min_spawn_distance,
                         cage_xy=cage_xy, dying_cost=dying_cost, **kwargs)

    def _set_params(self, p: dict) -> None:
        P = self._params
        P.tag_tag_radius = float(p.pop("tag_radius"))
        P.tag_visible_radius = float(p.pop("visible_radius"))
        P.tag_target_step = float(p.pop("target_step"))
        P.tag_min_spawn_distance = float(p.pop("min_spawn_distance"))
        cage = p.pop("cage_xy")
        P.tag_cage_xy[0], P.tag_cage_xy[1] = float(cage[0]), float(cage[1])
        P.tag_dying_cost = float(p.pop("dying_cost"))
        _common_params(P, p)

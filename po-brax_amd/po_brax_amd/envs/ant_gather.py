"""AntGather: collect apples (+1), avoid bombs (-1); a 2 x n_bins range sensor.

Mirrors ``po_brax/envs/ant_gather.py`` (constructor :59-91, reset :93-123, step :125-150,
readings :152-181, obs :183-213) on the fused HIP kernels.  Body order: 0-8 ant,
9 Ground, 10 Arena, 11.. Target_1..n_apples, then Bomb_1..n_bombs.  Caught objects move
to the waiting area (last grid point + 2 * sensor_range); there is no in-episode
respawn (objects are re-drawn only by a reset).
"""
from __future__ import annotations

import math
from typing import Sequence

import torch

from .ant_heavenhell import ANT_BODIES, _common_params
from .env import PoBraxEnv


class AntGatherEnv(PoBraxEnv):
    """
    Args:
        n_apples / n_bombs: number of apples (+1) and bombs (-1)
        cage_xy: arena half extents
        robot_object_spacing: objects spawn on integer grid points farther than this from 0
        catch_range: distance at which an object is caught
        n_bins, sensor_range, sensor_span: range sensor
        dying_cost: reward on death
    """

    kind = "ant_gather"
    slot_names = ("apples", "bombs", "objects")
    int_metrics = (0, 1)  # ant_gather.py:147-148: in_range.sum() -> int32 after step
    reset_metrics = ("apples", "bombs", "objects")
    step_metrics = ("apples", "bombs", "objects")

    def __init__(self,
                 n_apples: int = 8,
                 n_bombs: int = 8,
                 cage_xy: Sequence[float] = (6, 6),
                 robot_object_spacing: float = 2.,
                 catch_range: float = 1.,
                 n_bins: int = 10,
                 sensor_range: float = 6.,
                 sensor_span: float = math.pi,
                 dying_cost: float = -10.,
                 **kwargs):
        self.n_apples, self.n_bombs = int(n_apples), int(n_bombs)
        self.n_objects = self.n_apples + self.n_bombs
        self.n_bins = int(n_bins)
        super().__init__(n_apples=n_apples, n_bombs=n_bombs, cage_xy=cage_xy,
                         robot_object_spacing=robot_object_spacing, catch_range=catch_range,
                         n_bins=n_bins, sensor_range=sensor_range, sensor_span=sensor_span,
                         dying_cost=dying_cost, **kwargs)
        self.object_indices = torch.arange(11, 11 + self.n_objects)

    def _set_params(self, p: dict) -> None:
        P = self._params
        P.ga_n_apples, P.ga_n_bombs = int(p.pop("n_apples")), int(p.pop("n_bombs"))
        cage = p.pop("cage_xy")
        P.ga_cage_xy[0], P.ga_cage_xy[1] = float(cage[0]), float(cage[1])
        P.ga_robot_object_spacing = float(p.pop("robot_object_spacing"))
        P.ga_catch_range = float(p.pop("catch_range"))
        P.ga_n_bins = int(p.pop("n_bins"))
        P.ga_sensor_range = float(p.pop("sensor_range"))
        P.ga_sensor_span = float(p.pop("sensor_span"))
        P.ga_dying_cost = float(p.pop("dying_cost"))
        _common_params(P, p)

    def _body_names(self):
        return (list(ANT_BODIES) + ["Arena"] + [f"Target_{i + 1}" for i in range(self.n_apples)]
                + [f"Bomb_{i + 1}" for i in range(self.n_bombs)])



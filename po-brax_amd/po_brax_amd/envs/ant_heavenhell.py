"""AntHeavenHell: T-maze POMDP -- a priest within ``visible_radius`` reveals the heaven side.

Mirrors ``po_brax/envs/ant_heavenhell.py`` (constructor :51-73, reset :75-103,
step :106-123, obs :125-158); the computation runs in the fused HIP kernels of libpob.so
(``k_reset<HEAVENHELL>``, ``k_step<HEAVENHELL>``).  Body order (``sys.body.index``):
0-8 ant, 9 Ground, 10 Priest, 11 Target (heaven), 12 Hell, 13 Arena.  obs (114,) =
torso pos/rot, 8 joint angles, torso vel/ang, 8 joint velocities, clip(contact.vel)
(14x3), clip(contact.ang) (14x3), heaven direction.
"""
from __future__ import annotations

from typing import Sequence

from .env import PoBraxEnv

ANT_BODIES = ("$ Torso", "Aux 1", "$ Body 4", "Aux 2", "$ Body 7", "Aux 3", "$ Body 10",
              "Aux 4", "$ Body 13", "Ground")


class AntHeavenHellEnv(PoBraxEnv):
    """AntHeavenHell. Basically TMaze with partial observability.

    Args:
        heaven_hell: xy positions of heaven, hell (swapped at random on reset)
        priest_position: xy of the priest (top of the T)
        visible_radius: radius within which the ant sees the priest (and reaches heaven/hell)
        dying_cost: reward on death (torso z < 0.2 or > 1.0)
    """

    kind = "ant_heavenhell"
    body_names = ANT_BODIES + ("Priest", "Target", "Hell", "Arena")
    slot_names = ("heavens", "hells", "hits")
    reset_metrics = ("heavens", "hells")
    step_metrics = ("heavens", "hells", "hits")  # ant_heavenhell.py:122 adds 'hits'

    def __init__(self,
                 heaven_hell: Sequence[Sequence[float]] = ((-5.25, 7.), (5.25, 7.)),
                 priest_position: Sequence[float] = (0, 7.),
                 visible_radius: float = 2.,
                 dying_cost: float = -2.,
                 **kwargs):
        super().__init__(heaven_hell=heaven_hell, priest_position=priest_position,
                         visible_radius=visible_radius, dying_cost=dying_cost, **kwargs)

    def _set_params(self, p: dict) -> None:
        hh, pr = p.pop("heaven_hell"), p.pop("priest_position")
        if len(hh) != 2 or any(len(x) != 2 for x in hh) or len(pr) != 2:
            raise ValueError("heaven_hell must be ((x, y), (x, y)) and priest_position (x, y)")
        for i in range(2):
            for j in range(2):
                self._params.hh_heaven_hell[i][j] = float(hh[i][j])
        self._params.hh_priest[0], self._params.hh_priest[1] = float(pr[0]), float(pr[1])
        self._params.hh_visible_radius = float(p.pop("visible_radius"))
        self._params.hh_dying_cost = float(p.pop("dying_cost"))
        _common_params(self._params, p)
        self.visible_radius = self._params.hh_visible_radius
        self.dying_cost = self._params.hh_dying_cost


def _common_params(params, p: dict) -> None:
    """Engine-level knobs shared by the envs: PBD joint solver scales, and ``legacy_spring``
    (as brax's ``Ant(legacy_spring=True)`` [ext]: the brax <= 0.0.12 spring dynamics the
    notebook trajectory notebooks/ant_tag.ipynb:449 was made with)."""
    if "legacy_spring" in p:
        params.legacy_spring = 1 if p.pop("legacy_spring") else 0
    if "solver_scale_pos" in p:
        params.solver_scale_pos = float(p.pop("solver_scale_pos"))
    if "solver_scale_ang" in p:
        params.solver_scale_ang = float(p.pop("solver_scale_ang"))
    # the reference envs swallow unknown **kwargs (ant_*.py __init__ signatures)

"""The brax ``Config`` of an engine env as a JSON dict (``MessageToDict`` layout).

Built from the same constants the kernels' tables come from: brax's ant
(``brax.envs.ant._SYSTEM_CONFIG`` as serialised in ``notebooks/ant_tag.ipynb:449``) and the
po-env extensions -- ``extend_ant_cfg`` of ``ant_heavenhell.py:13-39``,
``ant_gather.py:17-39``, ``ant_tag.py:13-25`` with the walls of ``envs/utils.py:6-119``
(``add_box_wall_to_body``, ``draw_arena``, ``draw_t_maze``).  The engine runs brax's PBD
mode, so the emitted config carries ``dynamicsMode: "pbd"`` and omits the legacy spring
fields (``stiffness``, ``springDamping``, ``baumgarteErp``).  Scalars are rounded to
float32 as the proto fields store them.  Body order = ``sys.body.index``.
"""
from __future__ import annotations

import math
from typing import Dict, List

import numpy as np


def f32(x: float) -> float:
    """A float32 proto field as MessageToDict prints it (shortest float32 repr)."""
    return float(str(np.float32(x)))


def _v(x=0.0, y=0.0, z=0.0) -> Dict[str, float]:
    return {"x": f32(x), "y": f32(y), "z": f32(z)}


_MATERIAL = {"friction": 1.0, "elasticity": 0.0}
_FREE = {"position": _v(), "rotation": _v(), "all": False}
_FROZEN = {"position": _v(1, 1, 1), "rotation": _v(1, 1, 1), "all": True}

# name, mass, capsule (radius, length, end), collider rotation (degrees, xyz) or None
ANT_BODIES = (
    ("$ Torso", 10.0, (0.25, 0.5, 1), None),
    ("Aux 1", 1.0, (0.08, 0.44284272, 0), (90.0, -45.0, 0.0)),
    ("$ Body 4", 1.0, (0.08, 0.7256854, -1), (90.0, -45.0, 0.0)),
    ("Aux 2", 1.0, (0.08, 0.44284272, 0), (90.0, 45.0, 0.0)),
    ("$ Body 7", 1.0, (0.08, 0.7256854, -1), (90.0, 45.0, 0.0)),
    ("Aux 3", 1.0, (0.08, 0.44284272, 0), (-90.0, 45.0, 0.0)),
    ("$ Body 10", 1.0, (0.08, 0.7256854, -1), (-90.0, 45.0, 0.0)),
    ("Aux 4", 1.0, (0.08, 0.44284272, 0), (-90.0, -45.0, 0.0)),
    ("$ Body 13", 1.0, (0.08, 0.7256854, -1), (-90.0, -45.0, 0.0)),
)
# parent, child, parent_offset, child_offset, rotation (degrees), angle limit (degrees)
ANT_JOINTS = (
    ("$ Torso", "Aux 1", (0.2, 0.2), (-0.1, -0.1), ("y", -90.0), (-30.0, 30.0)),
    ("Aux 1", "$ Body 4", (0.1, 0.1), (-0.2, -0.2), ("z", 135.0), (30.0, 70.0)),
    ("$ Torso", "Aux 2", (-0.2, 0.2), (0.1, -0.1), ("y", -90.0), (-30.0, 30.0)),
    ("Aux 2", "$ Body 7", (-0.1, 0.1), (0.2, -0.2), ("z", 45.0), (-70.0, -30.0)),
    ("$ Torso", "Aux 3", (-0.2, -0.2), (0.1, 0.1), ("y", -90.0), (-30.0, 30.0)),
    ("Aux 3", "$ Body 10", (-0.1, -0.1), (0.2, 0.2), ("z", 135.0), (-70.0, -30.0)),
    ("$ Torso", "Aux 4", (0.2, -0.2), (-0.1, 0.1), ("y", -90.0), (-30.0, 30.0)),
    ("Aux 4", "$ Body 13", (0.1, -0.1), (-0.2, 0.2), ("z", 45.0), (30.0, 70.0)),
)
GROUND_COLLIDERS = ("$ Torso", "$ Body 4", "$ Body 7", "$ Body 10", "$ Body 13")


def _ant_body(name, mass, cap, rot) -> dict:
    c = {}
    if rot is not None:
        c["rotation"] = _v(*rot)
    c["capsule"] = {"radius": f32(cap[0]), "length": f32(cap[1]), "end": cap[2]}
    c["material"] = dict(_MATERIAL)
    return {"name": name, "colliders": [c], "inertia": _v(1, 1, 1), "mass": f32(mass), "frozen": dict(_FREE)}


def _joint(parent, child, po, co, rot, lim) -> dict:
    r = {rot[0]: f32(rot[1])}
    r.update({k: 0.0 for k in "xyz" if k != rot[0]})
    return {"name": f"{parent}_{child}", "parent": parent, "child": child,
            "parentOffset": _v(*po), "childOffset": _v(*co), "rotation": r,
            "angularDamping": 20.0, "angleLimit": [{"min": f32(lim[0]), "max": f32(lim[1])}]}


def _frozen_body(name: str, colliders: List[dict]) -> dict:
    return {"name": name, "colliders": colliders, "inertia": _v(1, 1, 1), "mass": 1.0, "frozen": dict(_FROZEN)}


def _sphere(radius: float) -> dict:
    return {"sphere": {"radius": f32(radius)}, "material": dict(_MATERIAL)}


def _box_wall(fx, fy, tx, ty, half_height, width) -> dict:
    """envs/utils.py:6-28 add_box_wall_to_body."""
    vx, vy = tx - fx, ty - fy
    length = math.hypot(vx, vy)
    zr = math.degrees(math.acos(vx / length))
    return {"position": _v((fx + tx) / 2, (fy + ty) / 2, 0.0), "rotation": _v(0, 0, zr),
            "box": {"halfsize": _v(length / 2, width, half_height)}, "material": dict(_MATERIAL)}


def _arena(points, half_height, width) -> dict:
    n = len(points)
    return _frozen_body("Arena", [_box_wall(*points[i], *points[(i + 1) % n], half_height, width) for i in range(n)])


def _draw_arena(cage_x, cage_y, h=0.5):
    """envs/utils.py:60-83 (use_boxes: wall half-width r/2)."""
    r = h / 2
    x, y = cage_x, cage_y
    return _arena([(x + r, y + r), (x + r, -y - r), (-x - r, -y - r), (-x - r, y + r)], h, r)


def _draw_t_maze(t_x, t_y, hw=2.0, r=0.5):
    """envs/utils.py:87-119."""
    return _arena([(-t_x - r, t_y + r), (t_x + r, t_y + r), (t_x + r, t_y - hw - r), (hw + r, t_y - hw - r),
                   (hw + r, -r), (-hw - r, -r), (-hw - r, t_y - hw - r), (-t_x - r, t_y - hw - r)], r, r)


def brax_config(env) -> dict:
    """brax Config dict of an engine env (``env`` may be wrapped)."""
    e = env.unwrapped
    return brax_config_of(e.kind, e._params, e._action_repeat)


def brax_config_of(kind: str, p, action_repeat: int = 1) -> dict:
    """brax Config dict for env ``kind`` with constructor parameters ``p`` (pob_params)."""
    bodies = [_ant_body(*b) for b in ANT_BODIES]
    bodies.append({"name": "Ground", "colliders": [{"plane": {}, "material": dict(_MATERIAL)}],
                   "inertia": _v(1, 1, 1), "mass": 1.0, "frozen": dict(_FROZEN)})
    defaults: List[dict] = []
    arena = False
    if kind == "ant_heavenhell":
        hhp = [tuple(p.hh_heaven_hell[0]), tuple(p.hh_heaven_hell[1]), tuple(p.hh_priest)]
        bodies += [_frozen_body(n, [_sphere(0.5)]) for n in ("Priest", "Target", "Hell")]
        defaults.append({"qps": [{"name": "Priest", "pos": _v(hhp[2][0], hhp[2][1], 1.0)}], "angles": []})
        t_x = max(h[0] for h in hhp) + 1.0
        t_y = max(h[1] for h in hhp) + 1.0
        bodies.append(_draw_t_maze(t_x, t_y))
        arena = True
    elif kind == "ant_gather":
        bodies.append(_draw_arena(p.ga_cage_xy[0] + 1.0, p.ga_cage_xy[1] + 1.0))
        bodies += [_frozen_body(f"Target_{i + 1}", [_sphere(0.25)]) for i in range(p.ga_n_apples)]
        bodies += [_frozen_body(f"Bomb_{i + 1}", [_sphere(0.25)]) for i in range(p.ga_n_bombs)]
        arena = True
    elif kind == "ant_tag":
        bodies.append(_frozen_body("Target", [_sphere(0.5)]))
        bodies.append(_draw_arena(p.tag_cage_xy[0] + 1.0, p.tag_cage_xy[1] + 1.0))
        arena = True
    if arena:
        defaults.append({"qps": [{"name": "Arena", "pos": _v(0, 0, 0.5)}], "angles": []})
    collide = [{"first": b, "second": "Ground"} for b in GROUND_COLLIDERS]
    if arena:
        collide += [{"first": b[0], "second": "Arena"} for b in ANT_BODIES]
    ar = int(action_repeat)
    return {
        "bodies": bodies,
        "joints": [_joint(*j) for j in ANT_JOINTS],
        "actuators": [{"name": f"{j[0]}_{j[1]}", "joint": f"{j[0]}_{j[1]}", "strength": 350.0, "torque": {}}
                      for j in ANT_JOINTS],
        "friction": 1.0, "gravity": {"z": f32(-9.8), "x": 0.0, "y": 0.0}, "angularDamping": f32(-0.05),
        "collideInclude": collide, "dt": f32(0.05 * ar), "substeps": 10 * ar, "frozen": {"all": False},
        "defaults": defaults, "forces": [], "elasticity": 0.0, "velocityDamping": 0.0, "colliderCutoff": 0,
        "meshGeometries": [], "dynamicsMode": "pbd",
    }

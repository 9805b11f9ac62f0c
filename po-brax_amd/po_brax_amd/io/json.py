"""``brax.io.json`` for engine envs: ``{"config": <Config dict>, "pos": [T][N][3],
"rot": [T][N][4]}`` -- the payload format of ``notebooks/ant_tag.ipynb:449``."""
from __future__ import annotations

import json as _json
from typing import Sequence

import torch

from .config import brax_config


def frames(qps: Sequence, env_index: int = 0):
    """Per-frame (pos, rot) lists of ONE env from a sequence of QPs (batched or not; any
    qp storage dtype).  Frames are gathered with one device->host copy."""
    pos = torch.stack([q.pos if q.pos.ndim == 2 else q.pos[env_index] for q in qps]).float().cpu()
    rot = torch.stack([q.rot if q.rot.ndim == 2 else q.rot[env_index] for q in qps]).float().cpu()
    return pos.tolist(), rot.tolist()


def to_dict(env, qps: Sequence, env_index: int = 0) -> dict:
    pos, rot = frames(qps, env_index)
    return {"config": brax_config(env), "pos": pos, "rot": rot}


def dumps(env, qps: Sequence, env_index: int = 0) -> str:
    """JSON text of a trajectory (``brax.io.json.dumps(sys, qps)``)."""
    return _json.dumps(to_dict(env, qps, env_index))

"""Observation index masks for partially observable variants of brax envs.

Same index sets as ``po_brax/standard_observability_masks.py:5-67`` (POSITION, VELOCITY,
TARGET_POS, OBJECT_POS, HEADINGS, CFRC), stored as half-open ranges and materialised as
int64 index tensors.  ``apply_mask(obs, idx)`` is the column gather ``obs[:, idx]`` run by
the ``k_obs_gather`` HIP kernel (pob_obs_gather).  The ``'ant'`` sets index the 87-dim stock
brax Ant observation; for the po-envs' own observations use ``po_env_mask(...)``.
"""
from __future__ import annotations

from typing import Dict, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._lib import lib, check

Ranges = Sequence[Tuple[int, int]]

_POSITION: Dict[str, Ranges] = {
    'acrobot': [(0, 2)], 'ant': [(0, 13)], 'fetch': [(0, 6), (10, 49)], 'grasp': [(8, 56)],
    'halfcheetah': [(0, 11)], 'hopper': [(0, 8)], 'humanoid': [(0, 22), (45, 144)],
    'humanoidstandup': [(0, 22), (45, 144)], 'inverted_pendulum': [(0, 6)],
    'inverted_double_pendulum': [(0, 5)], 'reacher': [(4, 6)], 'reacherangle': [(4, 6)],
    'ur5e': [(0, 6), (10, 34)], 'walker2d': [(0, 11)],
}
_VELOCITY: Dict[str, Ranges] = {
    'acrobot': [(2, 4)], 'ant': [(13, 27)], 'fetch': [(49, 88)], 'grasp': [(56, 104), (107, 110)],
    'halfcheetah': [(11, 23)], 'hopper': [(8, 14)], 'humanoid': [(22, 45), (144, 210)],
    'humanoidstandup': [(22, 45), (144, 210)], 'inverted_pendulum': [(6, 10)],
    'inverted_double_pendulum': [(5, 25)], 'reacher': [(6, 8)], 'reacherangle': [(6, 8)],
    'ur5e': [(34, 58)], 'walker2d': [(11, 20)],
}
_TARGET_POS: Dict[str, Ranges] = {
    'fetch': [(6, 10)], 'grasp': [(4, 8)], 'reacher': [(0, 4), (8, 11)],
    'reacherangle': [(0, 4), (8, 11)], 'ur5e': [(6, 10)],
}
_OBJECT_POS: Dict[str, Ranges] = {'grasp': [(0, 4)]}
_HEADINGS: Dict[str, Ranges] = {'grasp': [(104, 107), (110, 116)]}
_CFRC: Dict[str, Ranges] = {
    'ant': [(27, 87)], 'fetch': [(88, 101)], 'grasp': [(116, 132)], 'humanoid': [(210, 299)],
    'humanoidstandup': [(210, 299)], 'ur5e': [(58, 66)],
}


def _idx(ranges: Ranges) -> np.ndarray:
    return np.concatenate([np.arange(a, b) for a, b in ranges]).astype(np.int64)


POSITION = {k: _idx(v) for k, v in _POSITION.items()}
VELOCITY = {k: _idx(v) for k, v in _VELOCITY.items()}
TARGET_POS = {k: _idx(v) for k, v in _TARGET_POS.items()}
OBJECT_POS = {k: _idx(v) for k, v in _OBJECT_POS.items()}
HEADINGS = {k: _idx(v) for k, v in _HEADINGS.items()}
CFRC = {k: _idx(v) for k, v in _CFRC.items()}

# po-env observation layouts (ant_*.py _get_obs): 29 ant entries, then 2 x 3N contact
# entries, then the task entries.
_PO_LAYOUT = {'ant_heavenhell': (14, 1), 'ant_gather': (27, 20), 'ant_tag': (12, 2)}


def po_env_mask(env_name: str, position=True, velocity=True, cfrc=True, task=True,
                n_bodies: int = None, n_task: int = None) -> np.ndarray:
    """Column indices of a po-env observation (HH 114, GA 211, TAG 103 by default)."""
    N, T = _PO_LAYOUT[env_name]
    N = n_bodies or N
    T = n_task if n_task is not None else T
    parts = []
    if position:
        parts.append(np.arange(0, 15))
    if velocity:
        parts.append(np.arange(15, 29))
    if cfrc:
        parts.append(np.arange(29, 29 + 6 * N))
    if task:
        parts.append(np.arange(29 + 6 * N, 29 + 6 * N + T))
    return np.concatenate(parts).astype(np.int64) if parts else np.zeros(0, np.int64)


def apply_mask(obs: torch.Tensor, idx, out: torch.Tensor = None) -> torch.Tensor:
    """``obs[..., idx]`` on the device (HIP column gather); obs (B, D) float32 contiguous."""
    squeeze = obs.ndim == 1
    o = obs.reshape(-1, obs.shape[-1]).contiguous()
    if o.dtype != torch.float32:
        raise TypeError("obs must be float32")
    B, D = o.shape
    if isinstance(idx, torch.Tensor):
        idx = idx.cpu().numpy()
    ia = np.asarray(idx, dtype=np.int64).ravel()
    if ia.size and (ia.min() < 0 or ia.max() >= D):
        raise IndexError(f"mask index out of range for obs dim {D}")
    ii = torch.from_numpy(ia.astype(np.int32)).to(o.device).contiguous()
    K = ii.numel()
    if out is None:
        out = torch.empty((B, K), dtype=torch.float32, device=o.device)
    if B and K:
        check(lib.pob_obs_gather(o.data_ptr(), B, D, ii.data_ptr(), K, out.data_ptr(),
                                 _lib.stream_handle(o.device)))
    return out[0] if squeeze else out

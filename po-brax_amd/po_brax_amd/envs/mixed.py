"""Several env batches of different kinds stepped by ONE kernel launch.

BASELINE.json config 5 ("all three variants mixed + autoreset") runs AntHeavenHell,
AntGather and AntTag batches side by side.  Each keeps its own brax chain (``create(...)``
with its own State pytree and semantics); ``MixedEnv.step`` folds the per-env launches
into one ``pob_step_mixed`` call, whose grid is the concatenation of the envs' block
ranges, so small per-kind batches still fill the GPU together.

Key derivation treats the mix as ONE batch of ``B_total = sum(B_k)`` envs laid out
kind after kind: reset keys ``split(key, B_total + 1)[1:]`` and actions
``uniform(k, (B_total, 8))`` are sliced per kind (the same global-index rule as the
multi-GPU sharding), so a mixed rollout equals the per-kind rollouts it is made of.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence

import torch

from .. import _lib
from .._lib import lib, check
from . import env as _env_mod
from .env import Env, PoBraxEnv, State, Wrapper
from .wrappers import ActionRepeatWrapper, AutoResetWrapper, EpisodeWrapper, VectorWrapper, VmapWrapper

# wrappers that only fold into kernel flags (anything that post-processes a step's output
# on the stream would read it before the fused launch)
_FOLDING = (ActionRepeatWrapper, EpisodeWrapper, VmapWrapper, VectorWrapper, AutoResetWrapper)


class MixedEnv:
    """A list of env chains stepped together.  ``reset(key, batch_sizes)`` /
    ``step(states, actions)`` take and return one State / action batch per env."""

    def __init__(self, envs: Sequence[Env]):
        envs = list(envs)
        if not 1 <= len(envs) <= _lib.MIX_MAX:
            raise ValueError(f"MixedEnv takes 1..{_lib.MIX_MAX} envs")
        for e in envs:
            w = e
            while isinstance(w, Wrapper):
                if not isinstance(w, _FOLDING):
                    raise TypeError(f"{type(w).__name__} cannot be fused into a mixed step")
                w = w.env
            if not isinstance(w, PoBraxEnv):
                raise TypeError("MixedEnv needs engine envs (po_brax_amd.envs.create)")
        base = [e.unwrapped for e in envs]
        if len({(u.device, u.qp_dtype) for u in base}) != 1:
            raise ValueError("mixed envs must share device and qp_dtype")
        self.envs = envs
        self.device = base[0].device
        self.batch_sizes: List[int] = []

    @property
    def total_batch(self) -> int:
        return sum(self.batch_sizes)

    def offsets(self) -> List[int]:
        out, o = [], 0
        for b in self.batch_sizes:
            out.append(o)
            o += b
        return out

    def reset(self, key, batch_sizes: Sequence[int]) -> List[State]:
        from .. import jumpy
        if len(batch_sizes) != len(self.envs) or any(int(b) <= 0 for b in batch_sizes):
            raise ValueError("one positive batch size per env")
        self.batch_sizes = [int(b) for b in batch_sizes]
        key = jumpy._dev_key(key)
        keys = jumpy.random_split(key, self.total_batch + 1)[1:]
        return [e.reset(keys[o:o + b].contiguous()) for e, o, b in zip(self.envs, self.offsets(), self.batch_sizes)]

    def split_actions(self, act: torch.Tensor) -> List[torch.Tensor]:
        """(B_total, 8) -> per-env row blocks (views)."""
        return [act[o:o + b] for o, b in zip(self.offsets(), self.batch_sizes)]

    def step(self, states: Sequence[State], actions) -> List[State]:
        return self._step(states, actions, False)

    def step_(self, states: Sequence[State], actions) -> List[State]:
        """In-place variant (each state's buffers are overwritten)."""
        return self._step(states, actions, True)

    def _step(self, states, actions, inplace: bool) -> List[State]:
        if isinstance(actions, torch.Tensor):
            actions = self.split_actions(actions)
        if len(states) != len(self.envs) or len(actions) != len(self.envs):
            raise ValueError("one state and one action batch per env")
        _env_mod._CAPTURE = []
        try:
            outs = [e._chain_step(s, a, 0, 0, inplace) for e, s, a in zip(self.envs, states, actions)]
            rec = _env_mod._CAPTURE
        finally:
            _env_mod._CAPTURE = None
        if len(rec) != len(self.envs):
            raise RuntimeError("mixed step: unexpected launch count")
        flags, L = rec[0]["flags"], rec[0]["episode_length"]
        if any(r["flags"] != flags or r["episode_length"] != L for r in rec):
            raise ValueError("mixed envs must share the wrapper chain (flags / episode_length)")
        n = len(rec)
        handles = (C.c_void_p * n)(*[r["env"]._handle.value for r in rec])
        bs = (C.c_int * n)(*[r["B"] for r in rec])
        ins = (_lib.pob_state * n)(*[r["ci"] for r in rec])
        outs_c = (_lib.pob_state * n)(*[r["co"] for r in rec])
        acts = (C.c_void_p * n)(*[r["act"].data_ptr() for r in rec])
        check(lib.pob_step_mixed(n, handles, bs, ins, acts, outs_c, flags, L,
                                 _lib.stream_handle(self.device)))
        # the folding wrappers return the engine's result untouched (None while capturing)
        assert all(o is None for o in outs)
        return [r["env"]._state_of(r["bout"], True, r["squeeze"]) for r in rec]

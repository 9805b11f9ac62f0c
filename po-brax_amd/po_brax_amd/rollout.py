"""Multi-step rollouts replayed from a HIP graph.

``env.step_`` issues one fused kernel per env-step from Python (ctypes argument marshalling,
a launch per step).  For a fixed-shape loop -- the same State buffers stepped in place with
actions taken from a device array -- the launches can be captured once into a hipGraph
(``torch.cuda.CUDAGraph``: the kernels go to torch's current stream, which is the capture
stream inside ``torch.cuda.graph``) and replayed with one call, so consecutive step kernels
run back to back with no host work in between.  This is the MI355X replacement for the
reference's ``jax.jit`` / ``lax.scan`` of the step function over time: everything executed
is the same kernels on the same data, nothing is skipped.

    roll = GraphRollout(env, state, actions)   # actions: (T, B, 8) device tensor
    roll.replay()                              # T env-steps, in place on ``state``

``state`` must be stepped in place (its buffers are the graph's buffers); refill
``actions`` between replays to feed new actions (``roll.actions`` is the captured array).
Works for ``create(...)`` chains and ``MixedEnv`` (one launch per step either way); the gym
wrappers keep their eager path.
"""
from __future__ import annotations

from typing import Sequence

import torch


class GraphRollout:
    def __init__(self, env, state, actions: torch.Tensor, warmup: bool = False):
        """Capture ``actions.shape[0]`` in-place steps of ``env`` on ``state``.

        Capture does not execute the kernels; ``warmup=True`` first runs one eager step on a
        side stream (needed only when the env has never been stepped in this process, so
        that lazily initialised state is set up outside the capture)."""
        if actions.dim() != 3:
            raise ValueError("actions must be (T, B, A)")
        self.env, self.state, self.actions = env, state, actions
        self.steps = int(actions.shape[0])
        dev = actions.device
        if warmup:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self._step(0)
            torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for t in range(self.steps):
                self._step(t)

    def _step(self, t: int):
        # (a MixedEnv splits the (B_total, A) rows into its per-kind blocks itself)
        self.env.step_(self.state, self.actions[t])

    def replay(self):
        """Run the captured steps (stream-ordered on torch's current stream)."""
        self.graph.replay()
        return self.state


def graph_rollout(env, state, actions: Sequence[torch.Tensor] | torch.Tensor) -> GraphRollout:
    """Convenience: capture a rollout of ``actions`` (T, B, A) and return it (not run)."""
    if not isinstance(actions, torch.Tensor):
        actions = torch.stack(list(actions))
    return GraphRollout(env, state, actions)

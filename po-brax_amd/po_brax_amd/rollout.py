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

import contextlib
import gc
from typing import Sequence

import torch


def _release_deferred():
    """Outside a capture: free the tables of envs destroyed (possibly by a GC pass inside the
    capture) since the last env creation (include/pob.h pob_release_deferred)."""
    from . import _lib
    _lib.release_deferred()


@contextlib.contextmanager
def no_gc():
    """Keep the cyclic garbage collector off for the span of a hipGraph capture: a collection
    there runs arbitrary finalisers, and any HIP runtime call one makes that is illegal during
    a global-mode capture (hipFree, a synchronisation) invalidates the capture.  (The engine's
    own handles are already safe -- no env <-> System cycle, and pob_env_destroy defers its
    frees -- this guards the caller's objects too.)"""
    was = gc.isenabled()
    gc.disable()
    try:
        yield
    finally:
        if was:
            gc.enable()


def _slice_state(state, lo: int, hi: int, B: int):
    """The State of envs [lo, hi): every per-env tensor (first dim B, batch-major, so the
    slice is a contiguous view) sliced, the same object -> the same view (the engine tells
    its public tensors from caller replacements by identity, envs/env.py _bufs_of)."""
    from .envs.env import QP, State
    memo = {}

    def sl(x):
        if isinstance(x, torch.Tensor):
            if x.dim() >= 1 and x.shape[0] == B:
                if id(x) not in memo:
                    memo[id(x)] = x[lo:hi]
                return memo[id(x)]
            return x
        if isinstance(x, QP):
            return QP(sl(x.pos), sl(x.rot), sl(x.vel), sl(x.ang))
        if isinstance(x, dict):
            return {k: sl(v) for k, v in x.items()}
        return x

    return State(sl(state.qp), sl(state.obs), sl(state.reward), sl(state.done), sl(state.metrics),
                 sl(state.info), sl(state.aux))


class GraphRollout:
    def __init__(self, env, state, actions: torch.Tensor, warmup: bool = False, groups: int = 1):
        """Capture ``actions.shape[0]`` in-place steps of ``env`` on ``state``.

        Capture does not execute the kernels; ``warmup=True`` first runs one eager step on a
        side stream (needed only when the env has never been stepped in this process, so
        that lazily initialised state is set up outside the capture).

        ``groups = G > 1`` (single-kind envs): the batch is split into G contiguous env groups
        whose step chains are captured on G streams -- the groups are independent, so group
        g's step t + 1 may start while group g' still finishes step t, filling the SIMDs a
        launch's last waves leave idle.  Every env still takes exactly the same steps with
        the same kernels and actions (results bit-identical to ``groups = 1``)."""
        if actions.dim() != 3:
            raise ValueError("actions must be (T, B, A)")
        self.env, self.state, self.actions = env, state, actions
        self.steps = int(actions.shape[0])
        dev = actions.device
        B = int(actions.shape[1])
        groups = max(1, min(int(groups), B))
        if groups > 1 and isinstance(state, (list, tuple)):
            raise ValueError("groups > 1 needs a single-kind env")
        if warmup:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                self.state = self.env.step_(self.state, self.actions[0])
            torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        if groups == 1:
            with no_gc(), torch.cuda.graph(self.graph):
                for t in range(self.steps):
                    # follow the returned State: its public typed outputs (TAG done, GA
                    # counts) are the buffers the captured kernels write
                    self.state = self.env.step_(self.state, self.actions[t])
            _release_deferred()
            return
        bounds = [(B * g // groups, B * (g + 1) // groups) for g in range(groups)]
        # the typed step outputs (TAG bool done, GA int32 counts) live in the whole batch's
        # buffers, so that the groups write slices of them
        u = env.unwrapped
        u._typed_outputs(self.state.aux, B, "steps" in self.state.info)
        parts = [_slice_state(self.state, lo, hi, B) for lo, hi in bounds]
        streams = [None] + [torch.cuda.Stream(dev) for _ in range(groups - 1)]
        with no_gc(), torch.cuda.graph(self.graph):
            cap = torch.cuda.current_stream(dev)
            for st in streams[1:]:
                st.wait_stream(cap)  # fork from the capture stream
            for t in range(self.steps):
                for g, (lo, hi) in enumerate(bounds):
                    with torch.cuda.stream(streams[g] or cap):
                        parts[g] = self.env.step_(parts[g], self.actions[t, lo:hi])
            for st in streams[1:]:
                cap.wait_stream(st)  # join
        self.parts = parts
        _release_deferred()
        # the whole batch's State after a step (public fields in the reference's dtypes)
        self.state = u._state_of(u._bufs_of(self.state), True, False)

    def replay(self):
        """Run the captured steps (stream-ordered on torch's current stream)."""
        self.graph.replay()
        return self.state


def graph_rollout(env, state, actions: Sequence[torch.Tensor] | torch.Tensor) -> GraphRollout:
    """Convenience: capture a rollout of ``actions`` (T, B, A) and return it (not run)."""
    if not isinstance(actions, torch.Tensor):
        actions = torch.stack(list(actions))
    return GraphRollout(env, state, actions)


class GymGraphRollout:
    """``T`` steps of a gym vector env (``create_gym_env``: ``AutoresetVmapGymWrapper``,
    wrappers.py:240-262) captured into one hipGraph: per step the fused step kernel (which
    also ORs the device any-done word) and the masked gym reset kernel (which reads that word,
    re-samples the done envs from ``split(gym_key, B + 1)`` and advances the key only if
    something was done).  The decision ``if done.any()`` lives on the device, so the whole
    loop is capture-safe; nothing is skipped -- the same kernels run on the same buffers as
    ``gym.step`` called T times.

    The wrapper's host-side bookkeeping (the alternating any-done words and gym-key buffers)
    is advanced by the capture itself, so ``T`` must be even: after T steps it is back where
    it started, and every replay continues from the device state the last one left.
    ``actions`` (T, B, A) is read at replay time (refill it between replays).  Sharded
    (``create_gym_env(shard=...)``) under an RCCL process group, each step's 4-byte any-done
    all-reduce is captured with the kernels (RCCL collectives are stream-ordered and
    capturable: bit-equal to the eager steps through a one-rank communicator,
    ``scripts/gym_capture_check.py``, profiles/r7w); a gloo group's host-side collective
    cannot be captured, so that case is refused."""

    def __init__(self, gym, actions: torch.Tensor):
        from .envs.wrappers import AutoresetVmapGymWrapper, EvalGymWrapper
        if actions.dim() != 3 or actions.shape[0] % 2:
            raise ValueError("actions must be (T, B, A) with T even")
        # Only the bare device-side gym is capture-safe.  A wrapper with host-side per-step
        # bookkeeping (EvalGymWrapper's queue count / growth; it forwards _shard / _state to the
        # inner gym) would not advance on replay -- its queue would overrun its fixed capacity --
        # and may sync the host inside the capture, so it is refused by type.
        if isinstance(gym, EvalGymWrapper):
            raise NotImplementedError("GymGraphRollout cannot capture an EvalGymWrapper (host-side episode "
                                      "queues); capture the inner gym and step the eval wrapper eagerly")
        if not isinstance(gym, AutoresetVmapGymWrapper):
            raise NotImplementedError(f"GymGraphRollout captures create_gym_env's AutoresetVmapGymWrapper, "
                                      f"not {type(gym).__name__}")
        sh = getattr(gym, "_shard", None)
        if sh is not None:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_backend(sh.group) != "nccl":
                raise NotImplementedError("a sharded gym step captures its any-done all-reduce over RCCL "
                                          "(backend nccl) only; over gloo it steps eagerly")
        if gym._state is None:
            raise ValueError("reset() the gym before capturing its steps")
        self.gym, self.actions = gym, actions
        self.steps = int(actions.shape[0])
        dev = actions.device
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with no_gc(), torch.cuda.graph(self.graph):
            for t in range(self.steps):
                gym.step(self.actions[t])
        # the buffers the captured kernels read and write (T even: the key pair is back in order)
        self._captured = (gym._state, gym._key, gym._key2)
        _release_deferred()

    def replay(self):
        """Run the captured gym steps; returns (obs, reward, done, metrics) of the last."""
        st, k, k2 = self._captured
        g = self.gym
        if g._state is not st or g._key is not k or g._key2 is not k2:
            raise RuntimeError("the gym was reset or stepped outside the captured graph since capture; "
                               "rebuild the GymGraphRollout")
        self.graph.replay()
        return st.obs, st.reward, st.done, st.metrics


class PolicyRollout:
    """``T`` env-steps with the policy in the loop, replayed from ONE hipGraph: per step
    ``action = policy(obs)`` (any torch ops -- an MLP on hipBLASLt, sampling with a device
    generator -- static shapes, no host sync) then the fused step kernel, and the trajectory
    written to device buffers.  This is the MI355X counterpart of the reference's training-side
    ``jax.lax.scan`` over (policy, ``env.step``): one replay runs the whole unroll with no
    per-step host work.

        roll = PolicyRollout(env, state, policy, steps=T)
        roll.replay()        # T steps, in place on ``state``
        roll.obs[t]          # (B, D) observation the policy acted on at step t
        roll.actions[t], roll.reward[t], roll.done[t]   # its action, then the step's reward / done

    ``done`` is float32 (the engine's done; AntTag's public bool done is ``done != 0``).  The
    capture is preceded by ``warmup`` eager policy calls on a side stream (library handles and
    workspaces must exist before a capture); they do not step the env."""

    def __init__(self, env, state, policy, steps: int, warmup: int = 2):
        if steps <= 0:
            raise ValueError("steps must be positive")
        self.env, self.state, self.policy, self.steps = env, state, policy, int(steps)
        obs = state.obs
        dev = obs.device
        B, D = int(obs.shape[0]), int(obs.shape[1])
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(max(1, int(warmup))):
                a = policy(obs)
        torch.cuda.current_stream(dev).wait_stream(side)
        if not (isinstance(a, torch.Tensor) and a.shape == (B, env.action_size) and a.is_cuda):
            raise ValueError(f"policy must map obs (B, D) to a (B, {env.action_size}) device tensor")
        T = self.steps
        self.obs = torch.empty((T, B, D), dtype=obs.dtype, device=dev)
        self.actions = torch.empty((T, B, env.action_size), dtype=torch.float32, device=dev)
        self.reward = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.done = torch.empty((T, B), dtype=torch.float32, device=dev)
        torch.cuda.synchronize(dev)
        self.graph = torch.cuda.CUDAGraph()
        with no_gc(), torch.cuda.graph(self.graph):
            for t in range(T):
                self.obs[t].copy_(self.state.obs)
                self.actions[t].copy_(policy(self.state.obs))
                self.state = env.step_(self.state, self.actions[t])
                self.reward[t].copy_(self.state.reward)
                self.done[t].copy_(self.state.aux["done"] if "done" in self.state.aux else self.state.done)

    def replay(self):
        """Run the captured unroll (stream-ordered on torch's current stream)."""
        self.graph.replay()
        return self.state

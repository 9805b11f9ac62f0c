"""brax.jumpy RNG entry points on the device (jax.random threefry2x32 semantics).

``random_prngkey`` / ``random_split`` / ``random_uniform`` follow the jitted branch of
brax.jumpy [ext] as used throughout the reference (``more_jp.py:57-77``,
``wrappers.py:160-164``, ``ant_*.py`` reset), i.e. jax.random with the pre-partitionable
threefry scheme.  Keys are ``torch.uint32`` tensors of shape ``(..., 2)``.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import lib, check


def random_prngkey(seed: int, device=None) -> torch.Tensor:
    """jax.random.PRNGKey(seed) with jax's default 32-bit mode (x64 off).  jax converts a
    Python int seed through ``np.int64`` first ("avoid overflow error in X32 mode ... supports
    the common use-case of instantiating with Python hashes") and then to int32, which keeps
    the low 32 bits; the key is [seed >> 32 of the 32-bit value (a LOGICAL shift, = 0),
    seed & 0xFFFFFFFF], so PRNGKey(-1) = [0, 4294967295] and PRNGKey(2**40 + 5) = [0, 5].
    Seeds outside int64 raise OverflowError (as np.int64 does).  [ext] jax's random.PRNGKey;
    no reference fixture pins seeds outside int32 -- parity unpinned there."""
    seed = int(seed)
    if not -(1 << 63) <= seed < (1 << 63):
        raise OverflowError(f"seed {seed} does not fit in int64 (jax PRNGKey converts through np.int64)")
    k = torch.tensor([0, seed & 0xFFFFFFFF], dtype=torch.uint32)
    return k.to(device if device is not None else "cuda")


def _dev_key(key) -> torch.Tensor:
    key = torch.as_tensor(key)
    if key.dtype != torch.uint32:
        raise TypeError("keys must be torch.uint32")
    if key.device.type != "cuda":
        key = key.to("cuda")
    return key.contiguous()


def random_split(key: torch.Tensor, num: int = 2) -> torch.Tensor:
    """jax.random.split(key, num) -> (num, 2)."""
    key = _dev_key(key)
    out = torch.empty((num, 2), dtype=torch.uint32, device=key.device)
    check(lib.pob_random_split(key.data_ptr(), num, 0, num, out.data_ptr(), _lib.stream_handle(key.device)))
    return out


def random_split_rows(key: torch.Tensor, num: int, first: int, count: int) -> torch.Tensor:
    """Rows [first, first + count) of jax.random.split(key, num) -> (count, 2) (a shard's
    slice of a global split, computed without the other rows)."""
    key = _dev_key(key)
    out = torch.empty((count, 2), dtype=torch.uint32, device=key.device)
    check(lib.pob_random_split(key.data_ptr(), int(num), int(first), int(count), out.data_ptr(),
                               _lib.stream_handle(key.device)))
    return out


def random_split_batch(keys: torch.Tensor, num: int = 2) -> torch.Tensor:
    """vmap(split)(keys): (B, 2) -> (B, num, 2)."""
    return _split_many(_dev_key(keys).reshape(-1, 2), num)


def _split_many(keys, num):
    keys = keys.contiguous()
    out = torch.empty((keys.shape[0], num, 2), dtype=torch.uint32, device=keys.device)
    check(lib.pob_random_split_batch(keys.data_ptr(), keys.shape[0], num, out.data_ptr(),
                                     _lib.stream_handle(keys.device)))
    return out


def random_uniform(key: torch.Tensor, shape=(), low: float = 0.0, high: float = 1.0) -> torch.Tensor:
    """jax.random.uniform(key, shape, minval=low, maxval=high) in float32."""
    key = _dev_key(key)
    shape = tuple(shape) if not isinstance(shape, int) else (shape,)
    n = 1
    for s in shape:
        n *= int(s)
    out = torch.empty(shape, dtype=torch.float32, device=key.device)
    if n:
        check(lib.pob_random_uniform(key.data_ptr(), n, 0, n, float(low), float(high), out.data_ptr(),
                                     _lib.stream_handle(key.device)))
    return out


def random_actions_(key_io: torch.Tensor, total: int, first: int, act: torch.Tensor) -> torch.Tensor:
    """Bench/rollout helper: ``key, k = split(key)``; ``act = uniform(k, (total, A), -1, 1)``
    rows ``[first, first + B)`` written into ``act`` (B, A); ``key_io`` advanced in place."""
    B, A = act.shape
    check(lib.pob_random_actions(key_io.data_ptr(), int(total), int(first), B, A, act.data_ptr(),
                                 _lib.stream_handle(act.device)))
    return act

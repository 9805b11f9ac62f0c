"""ctypes binding of libpob.so (the C ABI declared in include/pob.h).

The product path is HIP-only: importing this module loads the in-tree ``libpob.so``
built by ``__graft_entry__.build()`` and raises ImportError if it is missing -- there is
no CPU fallback.  The per-step entry points (pob_step, pob_reset, pob_reset_where_done_shard)
are called through the pybind11 module ``_pob`` (``pob`` below); the rest through ctypes.  ``torch`` is imported first so that libpob.so binds to the HIP runtime
torch already loaded (same SONAME, libamdhip64.so.7).
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (load torch's HIP runtime before libpob.so)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("POB_LIB", os.path.join(HERE, "libpob.so"))

POB_OK, POB_EINVAL, POB_EHIP, POB_ENOMEM = 0, -1, -2, -3
F_EPISODE, F_AUTORESET, F_ZERO_STEPS_ON_DONE = 1, 2, 4
RESET_GYM, RESET_OWN = 0, 1
KINDS = {"ant_heavenhell": 0, "ant_gather": 1, "ant_tag": 2, "ant": 3}
QP_F32, QP_F16 = 0, 1
MIX_MAX = 4
ABI_VERSION = 8


class pob_params(C.Structure):
    _fields_ = [
        ("hh_heaven_hell", (C.c_float * 2) * 2), ("hh_priest", C.c_float * 2),
        ("hh_visible_radius", C.c_float), ("hh_dying_cost", C.c_float),
        ("ga_n_apples", C.c_int), ("ga_n_bombs", C.c_int), ("ga_cage_xy", C.c_float * 2),
        ("ga_robot_object_spacing", C.c_float), ("ga_catch_range", C.c_float),
        ("ga_n_bins", C.c_int), ("ga_sensor_range", C.c_float), ("ga_sensor_span", C.c_float),
        ("ga_dying_cost", C.c_float),
        ("tag_tag_radius", C.c_float), ("tag_visible_radius", C.c_float),
        ("tag_target_step", C.c_float), ("tag_min_spawn_distance", C.c_float),
        ("tag_cage_xy", C.c_float * 2), ("tag_dying_cost", C.c_float),
        ("action_repeat", C.c_int), ("solver_scale_pos", C.c_float), ("solver_scale_ang", C.c_float),
        ("qp_storage", C.c_int), ("legacy_spring", C.c_int),
    ]


_VP = C.c_void_p


class pob_state(C.Structure):
    _fields_ = [(n, _VP) for n in (
        "pos", "rot", "vel", "ang", "obs", "reward", "done", "steps", "truncation",
        "m0", "m1", "m2", "rng", "first_pos", "first_rot", "first_vel", "first_ang",
        "first_obs", "any_done", "done_u8", "trunc_i32", "m0_i32", "m1_i32", "any_done_clear", "obs_masked",
        "ovf_mark")]


# Every symbol include/pob.h declares (checked by tests/test_lib_symbols.py).
EXPORTS = (
    "pob_abi_version", "pob_last_error", "pob_default_params", "pob_env_create",
    "pob_env_destroy", "pob_release_deferred", "pob_env_dims", "pob_env_default_angle", "pob_reset", "pob_step",
    "pob_step_mixed", "pob_reset_where_done", "pob_reset_where_done_shard", "pob_default_qp",
    "pob_random_split", "pob_random_split_batch", "pob_random_uniform", "pob_random_actions", "pob_obs_gather",
    "pob_env_set_obs_mask",
)


class PobError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libpob.so not found at {LIB_PATH}: build it with `python -c 'import "
            "__graft_entry__ as g; g.build()'` (the HIP path has no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    lib.pob_abi_version.restype = C.c_int
    lib.pob_last_error.restype = C.c_char_p
    lib.pob_default_params.argtypes = [C.POINTER(pob_params)]
    lib.pob_env_create.argtypes = [C.c_int, C.POINTER(pob_params), C.POINTER(_VP)]
    lib.pob_env_destroy.argtypes = [_VP]
    lib.pob_env_destroy.restype = None
    lib.pob_release_deferred.argtypes = []
    lib.pob_env_dims.argtypes = [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
    lib.pob_env_default_angle.argtypes = [_VP, C.POINTER(C.c_float)]
    lib.pob_reset.argtypes = [_VP, C.c_int, _VP, C.POINTER(pob_state), _VP]
    lib.pob_step.argtypes = [_VP, C.c_int, C.POINTER(pob_state), _VP, C.POINTER(pob_state),
                             C.c_uint32, C.c_int, _VP]
    lib.pob_step_mixed.argtypes = [C.c_int, C.POINTER(_VP), C.POINTER(C.c_int), C.POINTER(pob_state),
                                   C.POINTER(_VP), C.POINTER(pob_state), C.c_uint32, C.c_int, _VP]
    lib.pob_reset_where_done.argtypes = [_VP, C.c_int, C.c_int, _VP, _VP, C.POINTER(pob_state), _VP]
    lib.pob_reset_where_done_shard.argtypes = [_VP, C.c_int, C.c_int, C.c_int, C.c_int, _VP, _VP,
                                               C.POINTER(pob_state), _VP]
    lib.pob_default_qp.argtypes = [_VP, C.c_int, _VP, _VP, _VP, _VP, _VP, _VP, _VP]
    lib.pob_random_split.argtypes = [_VP, C.c_int, C.c_int, C.c_int, _VP, _VP]
    lib.pob_random_split_batch.argtypes = [_VP, C.c_int, C.c_int, _VP, _VP]
    lib.pob_random_uniform.argtypes = [_VP, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, _VP, _VP]
    lib.pob_random_actions.argtypes = [_VP, C.c_int, C.c_int, C.c_int, C.c_int, _VP, _VP]
    lib.pob_obs_gather.argtypes = [_VP, C.c_int, C.c_int, _VP, C.c_int, _VP, _VP]
    lib.pob_env_set_obs_mask.argtypes = [_VP, C.POINTER(C.c_int32), C.c_int]
    if lib.pob_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH}: ABI version {lib.pob_abi_version()} != {ABI_VERSION}; rebuild it")
    for name in EXPORTS:
        if name not in ("pob_abi_version", "pob_last_error", "pob_env_destroy"):
            getattr(lib, name).restype = C.c_int
    return lib


lib = _load()


def _load_pyext():
    """The pybind11 binding of the per-step entry points (csrc/pob_py.cpp), bound to the
    functions of the libpob.so loaded above (so a POB_LIB build is used by both bindings)."""
    try:
        from . import _pob
    except ImportError as e:
        raise ImportError(f"po_brax_amd._pob (pybind11 binding) is not built: {e}; build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'`") from e
    addr = lambda f: C.cast(f, C.c_void_p).value  # noqa: E731
    _pob.bind(addr(lib.pob_step), addr(lib.pob_reset), addr(lib.pob_reset_where_done_shard),
              addr(lib.pob_last_error))
    return _pob


pob = _load_pyext()


def check(rc: int) -> None:
    """Map a status code to the reference's exception types."""
    if rc == POB_OK:
        return
    msg = (lib.pob_last_error() or b"").decode()
    if rc == POB_EINVAL:
        raise ValueError(msg)
    raise PobError(f"libpob status {rc}: {msg}")


def release_deferred() -> int:
    """Free the device tables of destroyed envs now (pob_release_deferred; otherwise they wait
    for the next env creation).  Calls hipFree: never inside a hipGraph capture."""
    return int(lib.pob_release_deferred())


def stream_handle(device=None) -> int:
    """hipStream_t of torch's current stream (kernels are stream-ordered with torch)."""
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()

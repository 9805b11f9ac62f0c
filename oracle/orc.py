"""ctypes binding of the C oracle (oracle/pob_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
Arrays are numpy, laid out exactly like the product's tensors (batch-major).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libpob_oracle.so")
KINDS = {"ant_heavenhell": 0, "ant_gather": 1, "ant_tag": 2, "ant": 3}
F_EPISODE, F_AUTORESET = 1, 2


FLOPS_LIB_PATH = os.path.join(HERE, "build", "libpob_oracle_flops.so")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def native_lib_path() -> str:
    """-O3 -march=native build for the CPU baseline, keyed by the host CPU model (built on
    the machine that runs it: a -march=native binary may not run on another CPU)."""
    import hashlib
    tag = hashlib.sha1(cpu_model().encode()).hexdigest()[:10]
    return os.path.join(HERE, "build", f"libpob_oracle_native_{tag}.so")


def build(force: bool = False, count_flops: bool = False, native: bool = False) -> str:
    """Compile the oracle with gcc (-ffp-contract=off keeps IEEE op order).  The
    ``count_flops`` variant defines ORC_COUNT_FLOPS (algorithmic FLOP counter); the
    ``native`` variant (-O3 -march=native) is the timed CPU baseline.
    Every variant computes the same bits: explicit fmaf, no contraction, no fast-math."""
    src = os.path.join(HERE, "pob_oracle.c")
    path = native_lib_path() if native else (FLOPS_LIB_PATH if count_flops else LIB_PATH)
    if force or not os.path.exists(path) or os.path.getmtime(path) < max(
            os.path.getmtime(src), os.path.getmtime(os.path.join(HERE, "pob_oracle.h"))):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        extra = ["-DORC_COUNT_FLOPS"] if count_flops else []
        opt = ["-O3", "-march=native"] if native else ["-O2", "-mfma"]
        tmp = f"{path}.{os.getpid()}.tmp"
        subprocess.check_call([
            "gcc", *opt, "-std=c99", "-D_GNU_SOURCE", "-ffp-contract=off", "-fno-fast-math",
            "-fopenmp", "-fPIC", "-shared", *extra, "-o", tmp, src, "-lm"])
        os.replace(tmp, path)
    return path


class Params(C.Structure):
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
        ("legacy_spring", C.c_int), ("wall_contact", C.c_int),
    ]


_FP = C.POINTER(C.c_float)
_UP = C.POINTER(C.c_uint32)


class State(C.Structure):
    _fields_ = [("pos", _FP), ("rot", _FP), ("vel", _FP), ("ang", _FP), ("obs", _FP),
                ("reward", _FP), ("done", _FP), ("steps", _FP), ("truncation", _FP),
                ("m0", _FP), ("m1", _FP), ("m2", _FP), ("rng", _UP),
                ("first_pos", _FP), ("first_rot", _FP), ("first_vel", _FP), ("first_ang", _FP),
                ("first_obs", _FP)]


_lib = None
_flib = None
_nlib = None


def _declare(_lib):
    if True:
        _lib.orc_env_create.restype = C.c_void_p
        _lib.orc_env_create.argtypes = [C.c_int, C.POINTER(Params)]
        _lib.orc_env_destroy.argtypes = [C.c_void_p]
        _lib.orc_env_dims.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        _lib.orc_default_params.argtypes = [C.POINTER(Params)]
        _lib.orc_reset.argtypes = [C.c_void_p, C.c_int, _UP, C.POINTER(State), C.c_int]
        _lib.orc_step.argtypes = [C.c_void_p, C.c_int, C.POINTER(State), _FP, C.POINTER(State),
                                  C.c_int, C.c_int, C.c_int]
        _lib.orc_gym_autoreset.argtypes = [C.c_void_p, C.c_int, _UP, C.POINTER(State), C.c_int]
        _lib.orc_default_qp.argtypes = [C.c_void_p, _FP, _FP, _FP, _FP, _FP, _FP]
        _lib.orc_contact_info.argtypes = [C.c_void_p, _FP, _FP, _FP, _FP, _FP, _FP]
        _lib.orc_split.argtypes = [_UP, C.c_int, _UP]
        _lib.orc_uniform.argtypes = [_UP, C.c_int, _FP, _FP, C.c_int, _FP]
        _lib.orc_randint.argtypes = [_UP, C.c_int, C.c_int]
        _lib.orc_choice_idx.argtypes = [_UP, C.c_int, C.c_int, C.POINTER(C.c_int)]
        _lib.orc_flops_read_and_reset.restype = C.c_longlong
        _lib.orc_flops_set_mode.argtypes = [C.c_int]
        _lib.orc_math_check.argtypes = [C.c_int, C.c_int, _FP, _FP, _FP]
        _lib.orc_contact_stats.argtypes = [C.POINTER(C.c_longlong)]
        _lib.orc_set_face_cull.argtypes = [C.c_int]
        _lib.orc_set_mesh_variant.argtypes = [C.c_int]
        _lib.orc_get_mesh_variant.restype = C.c_int
        _lib.orc_contact_stats_enable.argtypes = [C.c_int]
        _lib.orc_mesh_contacts.argtypes = [_FP, _FP, _FP, C.c_int, C.c_float, _FP]
    return _lib


def lib():
    global _lib
    if _lib is None:
        _lib = _declare(C.CDLL(build()))
    return _lib


def flops_lib():
    global _flib
    if _flib is None:
        _flib = _declare(C.CDLL(build(count_flops=True)))
    return _flib


def native_lib():
    global _nlib
    if _nlib is None:
        _nlib = _declare(C.CDLL(build(native=True)))
    return _nlib


def _p(a, t=_FP):
    return a.ctypes.data_as(t) if a is not None else None


def default_params(**kw) -> Params:
    p = Params()
    lib().orc_default_params(C.byref(p))
    for k, v in kw.items():
        if k == "hh_heaven_hell":
            for i in range(2):
                for j in range(2):
                    p.hh_heaven_hell[i][j] = v[i][j]
        elif isinstance(getattr(p, k), C.Array):
            for i, x in enumerate(v):
                getattr(p, k)[i] = x
        else:
            setattr(p, k, v)
    return p


class OracleEnv:
    """One env kind; state dicts of numpy arrays in the reference layout."""

    def __init__(self, name: str, count_flops: bool = False, native: bool = False, **params):
        self.name = name
        self._L = flops_lib() if count_flops else (native_lib() if native else lib())
        self.params = default_params(**params)
        self.h = self._L.orc_env_create(KINDS[name], C.byref(self.params))
        n, d, a = C.c_int(), C.c_int(), C.c_int()
        self._L.orc_env_dims(self.h, C.byref(n), C.byref(d), C.byref(a))
        self.N, self.D, self.A = n.value, d.value, a.value

    def __del__(self):
        try:
            self._L.orc_env_destroy(self.h)
        except Exception:
            pass

    def empty(self, B: int, first: bool = False):
        N, D = self.N, self.D
        s = dict(pos=np.zeros((B, N, 3), np.float32), rot=np.zeros((B, N, 4), np.float32),
                 vel=np.zeros((B, N, 3), np.float32), ang=np.zeros((B, N, 3), np.float32),
                 obs=np.zeros((B, D), np.float32), reward=np.zeros(B, np.float32),
                 done=np.zeros(B, np.float32), steps=np.zeros(B, np.float32),
                 truncation=np.zeros(B, np.float32), m0=np.zeros(B, np.float32),
                 m1=np.zeros(B, np.float32), m2=np.zeros(B, np.float32),
                 rng=np.zeros((B, 2), np.uint32))
        if first:
            s.update(first_pos=np.zeros((B, N, 3), np.float32), first_rot=np.zeros((B, N, 4), np.float32),
                     first_vel=np.zeros((B, N, 3), np.float32), first_ang=np.zeros((B, N, 3), np.float32),
                     first_obs=np.zeros((B, D), np.float32))
        return s

    @staticmethod
    def _cstate(s) -> State:
        st = State()
        for name, _t in State._fields_:
            a = s.get(name)
            if a is not None:
                assert a.flags.c_contiguous
                setattr(st, name, _p(a, _UP if name == "rng" else _FP))
        return st

    def reset(self, keys: np.ndarray, first: bool = False, nthreads: int = 1):
        keys = np.ascontiguousarray(keys, np.uint32)
        s = self.empty(keys.shape[0], first)
        cs = self._cstate(s)
        self._L.orc_reset(self.h, keys.shape[0], _p(keys, _UP), C.byref(cs), nthreads)
        return s

    def step(self, s, act: np.ndarray, flags: int = 0, episode_length: int = 1000,
             nthreads: int = 1, inplace: bool = False):
        act = np.ascontiguousarray(act, np.float32)
        B = act.shape[0]
        out = s if inplace else {k: v.copy() for k, v in s.items()}
        ci, co = self._cstate(s), self._cstate(out)
        self._L.orc_step(self.h, B, C.byref(ci), _p(act), C.byref(co), flags, episode_length, nthreads)
        return out

    def gym_autoreset(self, s, gym_key: np.ndarray, nthreads: int = 1):
        cs = self._cstate(s)
        self._L.orc_gym_autoreset(self.h, s["done"].shape[0], _p(gym_key, _UP), C.byref(cs), nthreads)
        return s

    def default_qp(self, qpos, qvel):
        N = self.N
        qpos = np.ascontiguousarray(qpos, np.float32); qvel = np.ascontiguousarray(qvel, np.float32)
        out = [np.zeros((N, 3), np.float32), np.zeros((N, 4), np.float32),
               np.zeros((N, 3), np.float32), np.zeros((N, 3), np.float32)]
        self._L.orc_default_qp(self.h, _p(qpos), _p(qvel), *[_p(o) for o in out])
        return out


def split(key, n):
    key = np.ascontiguousarray(key, np.uint32)
    out = np.zeros((n, 2), np.uint32)
    lib().orc_split(_p(key, _UP), n, _p(out, _UP))
    return out


FLOPS_REF_PAIRS, FLOPS_EXECUTED = 0, 1


def flops_per_env_step(name: str, B: int = 64, steps: int = 10, flags: int = F_EPISODE | F_AUTORESET,
                       seed: int = 0, mode: int = FLOPS_REF_PAIRS, **params) -> float:
    """Algorithmic FLOPs of one fused env-step (physics + POMDP + obs), counted by the
    instrumented restatement on a random-action rollout (single-threaded).

    mode FLOPS_REF_PAIRS: every capsule x wall x end pair is evaluated (the reference's
    algorithm); FLOPS_EXECUTED: only the pairs the HIP kernel evaluates after its exact
    culls (same results).  Executed branches only in both (an inactive contact is free)."""
    import pob_np as P
    e = OracleEnv(name, count_flops=True, **params)
    s = e.reset(P.split(P.prngkey(seed), B + 1)[1:], first=True)
    rng = np.random.default_rng(seed)
    e._L.orc_flops_set_mode(mode)
    e._L.orc_flops_read_and_reset()
    try:
        for _ in range(steps):
            s = e.step(s, rng.uniform(-1, 1, (B, 8)).astype(np.float32), flags=flags, nthreads=1, inplace=True)
        return e._L.orc_flops_read_and_reset() / float(B * steps)
    finally:
        e._L.orc_flops_set_mode(FLOPS_REF_PAIRS)


def uniform(key, n: int, lo: float = -1.0, hi: float = 1.0) -> np.ndarray:
    """jax.random.uniform(key, (n,), lo, hi) in float32 (the C restatement of pob_np.uniform)."""
    key = np.ascontiguousarray(key, np.uint32)
    lo_a, hi_a = np.array([lo], np.float32), np.array([hi], np.float32)
    out = np.zeros(n, np.float32)
    lib().orc_uniform(_p(key, _UP), n, _p(lo_a), _p(hi_a), 1, _p(out))
    return out


def flops_bench_workload(name: str, total: int, first: int = 0, n: int = 1024, warmup: int = 20, steps: int = 200,
                         flags: int = F_EPISODE | F_AUTORESET, episode_length: int = 1000, mode: int = FLOPS_EXECUTED,
                         seed: int = 0, time_budget_s: float = 60.0, **params) -> dict:
    """Algorithmic FLOPs per env-step on bench.py's own workload: the global envs
    [first, first + n) of a batch of ``total`` reset from ``split(PRNGKey(seed), total + 1)[1:]``,
    stepped with the bench's action stream (``key = split(PRNGKey(seed), total + 1)[0]``; per
    step ``key, k = split(key)``, ``uniform(k, (total, 8), -1, 1)`` rows [first, first + n)),
    warm-up steps included so that the timed steps see the bench's states.  Per-step means
    (FLOPs / env) of the timed steps and their spread; single-threaded instrumented build.
    Stops after ``time_budget_s`` (the count then covers the steps done)."""
    import time
    keys = split(np.array([0, seed & 0xFFFFFFFF], np.uint32), total + 1)
    e = OracleEnv(name, count_flops=True, **params)
    s = e.reset(np.ascontiguousarray(keys[1 + first:1 + first + n]), first=True)
    act_key = keys[0].copy()
    e._L.orc_flops_set_mode(mode)
    e._L.orc_flops_read_and_reset()
    per, t0 = [], time.time()
    try:
        for t in range(warmup + steps):
            kk = split(act_key, 2)
            act_key, k = kk[0].copy(), kk[1].copy()
            a = np.ascontiguousarray(uniform(k, total * 8).reshape(total, 8)[first:first + n])
            e.step(s, a, flags=flags, episode_length=episode_length, nthreads=1, inplace=True)
            per.append(e._L.orc_flops_read_and_reset() / float(n))
            if time.time() - t0 > time_budget_s:
                break
    finally:
        e._L.orc_flops_set_mode(FLOPS_REF_PAIRS)
    timed = np.array(per[warmup:] if len(per) > warmup else per, np.float64)
    return {"mean": float(timed.mean()), "min": float(timed.min()), "median": float(np.median(timed)),
            "max": float(timed.max()), "warmup_mean": float(np.mean(per[:warmup])) if warmup and per else None,
            "steps_counted": len(per), "timed_steps_counted": len(timed), "envs": n, "first": first, "total": total}


def mesh_contacts(wall, a, b, seg: bool, r: float) -> np.ndarray:
    """The oracle's capsule x TriangulatedBox contacts of one capsule (world end points a, b;
    seg False: the sphere at a) against one wall box (cx, cy, cz, cos, sin, hx, hy, hz):
    rows (tau, nx, ny, nz, pen, cd) in (face, triangle) order; cd: the contact position is the
    segment point moved by -cd n (the triangle point)."""
    w = np.ascontiguousarray(wall, np.float32)
    pa = np.ascontiguousarray(a, np.float32)
    pb = np.ascontiguousarray(b, np.float32)
    out = np.zeros((12, 6), np.float32)
    n = lib().orc_mesh_contacts(_p(w), _p(pa), _p(pb), int(bool(seg)), float(r), _p(out))
    return out[:n].copy()


def math_check(op: int, a: np.ndarray, b: np.ndarray = None) -> np.ndarray:
    """The spec's atan2f (op 0: atan2f(a, b)) or substep quaternion normalisation (op 1:
    rows of a (n, 4)) as the oracle computes them."""
    a = np.ascontiguousarray(a, np.float32)
    n = a.shape[0]
    b = np.ascontiguousarray(b if b is not None else np.zeros(n), np.float32)
    out = np.zeros_like(a)
    lib().orc_math_check(op, n, _p(a), _p(b), _p(out))
    return out

"""NumPy restatement of the reference's RNG and kinematics -- TEST INFRASTRUCTURE ONLY.

This module is part of the oracle (see oracle/README.md): only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it, and
only as a checker.  The product path (``po-brax_amd/``) never imports it.

What it restates (the reference's arithmetic lives in un-vendored brax v1 / jax, see
SURVEY.md §8(c); ``[ext]`` = recalled public semantics):

* ``threefry2x32``/``split``/``random_bits``/``uniform``/``randint``/``choice`` --
  jax.random (pre-``jax_threefry_partitionable``) as called through brax.jumpy under
  jit: ``more_jp.py:57-77``, ``ant_heavenhell.py:88-99``, ``ant_gather.py:110-118``,
  ``ant_tag.py:63-105,129-146``.  Pinned by the public KATs split(PRNGKey(0)) and
  split(PRNGKey(42)) (tests/golden/threefry_kat.json).
* the numpy path of brax.jumpy (``random_prngkey``/``random_split``/``random_uniform``
  un-jitted: PCG64 ``default_rng``) used by the notebook that produced the golden
  trajectory (``notebooks/ant_tag.ipynb:470-477``).
* ``euler_to_quat``/``rotate``/``quat_mul`` and ``System.default_angle``/``default_qp``
  forward kinematics (a4 in SURVEY.md §8(a)), pinned by frame 0 of
  ``notebooks/ant_tag.ipynb:449``.
"""
from __future__ import annotations

import numpy as np

U32 = np.uint32
_ROT = ((13, 15, 26, 6), (17, 29, 16, 24))


# --------------------------------------------------------------------------- threefry
def _rotl(x, r):
    return ((x << U32(r)) | (x >> U32(32 - r))).astype(U32)


def threefry2x32(key, x0, x1):
    """jax ``threefry2x32_p`` on uint32 arrays (20 rounds)."""
    k0, k1 = U32(key[0]), U32(key[1])
    ks = (k0, k1, U32(k0 ^ k1 ^ U32(0x1BD11BDA)))
    with np.errstate(over="ignore"):
        a = (np.asarray(x0, U32) + ks[0]).astype(U32)
        b = (np.asarray(x1, U32) + ks[1]).astype(U32)
        for i in range(5):
            for r in _ROT[i % 2]:
                a = (a + b).astype(U32)
                b = _rotl(b, r)
                b = (a ^ b).astype(U32)
            a = (a + ks[(i + 1) % 3]).astype(U32)
            b = (b + ks[(i + 2) % 3] + U32(i + 1)).astype(U32)
    return a, b


def threefry_2x32(key, count):
    """jax.random ``threefry_2x32(keypair, count)``: pad odd, split halves, concat."""
    count = np.asarray(count, U32).ravel()
    odd = count.size % 2
    if odd:
        count = np.concatenate([count, np.zeros(1, U32)])
    h = count.size // 2
    y0, y1 = threefry2x32(key, count[:h], count[h:])
    out = np.concatenate([y0, y1])
    return out[:-1] if odd else out


def split(key, num=2):
    return threefry_2x32(key, np.arange(2 * num, dtype=U32)).reshape(num, 2)


def random_bits(key, n):
    return threefry_2x32(key, np.arange(n, dtype=U32))


def uniform(key, shape, lo, hi):
    """jax.random.uniform in float32: ``max(lo, f*(hi-lo)+lo)``, f in [0,1)."""
    n = int(np.prod(shape)) if shape else 1
    bits = random_bits(key, n)
    f = ((bits >> U32(9)) | U32(0x3F800000)).view(np.float32) - np.float32(1.0)
    lo = np.asarray(lo, np.float32)
    hi = np.asarray(hi, np.float32)
    out = f.reshape(shape) * (hi - lo) + lo
    return np.maximum(lo, out).astype(np.float32)


def randint(key, lo, hi):
    """jax.random.randint for a scalar; the (2^16 mod span)^2 multiplier is 0 for span 4."""
    span = U32(hi - lo)
    _k1, k2 = split(key)
    hi_bits = random_bits(_k1, 1)[0]
    lo_bits = random_bits(k2, 1)[0]
    mult = U32((U32(2 ** 16) % span) * (U32(2 ** 16) % span) % span)
    with np.errstate(over="ignore"):
        off = (U32(hi_bits % span) * mult + U32(lo_bits % span)) % span
    return int(lo + int(off))


def permutation_indices(key, n):
    """jax ``_shuffle(key, arange(n))`` -- ceil(3 ln n / ln(2^32-1)) stable key sorts."""
    rounds = int(np.ceil(3 * np.log(max(1, n)) / np.log(np.iinfo(np.uint32).max)))
    x = np.arange(n)
    for _ in range(rounds):
        key, sub = split(key)
        sk = random_bits(sub, n)
        x = x[np.argsort(sk, kind="stable")]
    return x


def choice_noreplace(key, a, k):
    return np.asarray(a)[permutation_indices(key, len(a))[:k]]


def prngkey(seed):
    """jax.random.PRNGKey(seed), x64 off: the seed goes through np.int64, then int32 (low 32
    bits); high word = logical shift by 32 = 0.  Outside int64: OverflowError."""
    seed = int(seed)
    if not -(1 << 63) <= seed < (1 << 63):
        raise OverflowError(seed)
    return np.array([0, seed & 0xFFFFFFFF], U32)


# ------------------------------------------------------------ brax.jumpy numpy path
def np_prngkey(seed):
    return np.random.default_rng(seed).integers(0, 2 ** 32, dtype="uint32", size=2)


def np_split(key, num=2):
    return np.random.default_rng(key).integers(0, 2 ** 32, dtype="uint32", size=(num, 2))


def np_uniform(key, shape, lo, hi):
    return np.random.default_rng(key).uniform(size=shape, low=lo, high=hi)


# --------------------------------------------------------------------- brax.math
def euler_to_quat(v):
    """Tait-Bryan intrinsic x-y'-z'' from degrees (brax.math.euler_to_quat [ext])."""
    v = np.asarray(v, np.float64)
    c1, c2, c3 = np.cos(v * np.pi / 360)
    s1, s2, s3 = np.sin(v * np.pi / 360)
    return np.array([c1 * c2 * c3 - s1 * s2 * s3,
                     s1 * c2 * c3 + c1 * s2 * s3,
                     c1 * s2 * c3 - s1 * c2 * s3,
                     c1 * c2 * s3 + s1 * s2 * c3])


def quat_mul(u, v):
    return np.array([
        u[0] * v[0] - u[1] * v[1] - u[2] * v[2] - u[3] * v[3],
        u[0] * v[1] + u[1] * v[0] + u[2] * v[3] - u[3] * v[2],
        u[0] * v[2] - u[1] * v[3] + u[2] * v[0] + u[3] * v[1],
        u[0] * v[3] + u[1] * v[2] - u[2] * v[1] + u[3] * v[0]])


def rotate(vec, q):
    s, u = q[0], q[1:]
    r = 2 * (np.dot(u, vec) * u) + (s * s - np.dot(u, u)) * vec
    return r + 2 * s * np.cross(u, vec)


def quat_rot_axis(axis, angle):
    s, c = np.sin(angle / 2), np.cos(angle / 2)
    return np.array([c, axis[0] * s, axis[1] * s, axis[2] * s])


# ------------------------------------------------------------------ the brax Ant
# (bodies / joints as carried by the system JSON in notebooks/ant_tag.ipynb:449)
ANT_BODIES = [  # name, mass, capsule radius, length, end, collider euler (deg)
    ("$ Torso", 10.0, 0.25, 0.5, 1, (0, 0, 0)),
    ("Aux 1", 1.0, 0.08, 0.44284272, 0, (90, -45, 0)),
    ("$ Body 4", 1.0, 0.08, 0.7256854, -1, (90, -45, 0)),
    ("Aux 2", 1.0, 0.08, 0.44284272, 0, (90, 45, 0)),
    ("$ Body 7", 1.0, 0.08, 0.7256854, -1, (90, 45, 0)),
    ("Aux 3", 1.0, 0.08, 0.44284272, 0, (-90, 45, 0)),
    ("$ Body 10", 1.0, 0.08, 0.7256854, -1, (-90, 45, 0)),
    ("Aux 4", 1.0, 0.08, 0.44284272, 0, (-90, -45, 0)),
    ("$ Body 13", 1.0, 0.08, 0.7256854, -1, (-90, -45, 0)),
]
ANT_JOINTS = [  # parent, child, parent_offset, child_offset, euler rotation, (min,max) deg
    (0, 1, (0.2, 0.2, 0), (-0.1, -0.1, 0), (0, -90, 0), (-30, 30)),
    (1, 2, (0.1, 0.1, 0), (-0.2, -0.2, 0), (0, 0, 135), (30, 70)),
    (0, 3, (-0.2, 0.2, 0), (0.1, -0.1, 0), (0, -90, 0), (-30, 30)),
    (3, 4, (-0.1, 0.1, 0), (0.2, -0.2, 0), (0, 0, 45), (-70, -30)),
    (0, 5, (-0.2, -0.2, 0), (0.1, 0.1, 0), (0, -90, 0), (-30, 30)),
    (5, 6, (-0.1, -0.1, 0), (0.2, 0.2, 0), (0, 0, 135), (-70, -30)),
    (0, 7, (0.2, -0.2, 0), (-0.1, 0.1, 0), (0, -90, 0), (-30, 30)),
    (7, 8, (0.1, -0.1, 0), (-0.2, 0.2, 0), (0, 0, 45), (30, 70)),
]


def f32(x):
    """Config floats live in a float32 protobuf; brax reads them back as python floats."""
    return np.asarray(np.asarray(x, np.float32), np.float64)


def default_angle():
    return np.array([(f32(lo) + f32(hi)) * np.pi / 360 for *_, (lo, hi) in ANT_JOINTS])


def capsule_ends(i):
    """Capsule end points in body frame (end=0: both, +-1: that end), radius."""
    _, _, r, length, end, rot = ANT_BODIES[i]
    r, length = f32(r), f32(length)
    axis = rotate(np.array([0.0, 0.0, 1.0]), euler_to_quat(f32(rot)))
    seg = length / 2 - r
    if end == 0:
        return [axis * seg, -axis * seg], r
    return [axis * seg * end], r


def default_qp(qpos, qvel=None):
    """Forward kinematics of the ant tree + min-z lift (System.default_qp, a4)."""
    qvel = np.zeros(8) if qvel is None else np.asarray(qvel, np.float64)
    pos = np.zeros((9, 3)); rot = np.zeros((9, 4)); rot[0, 0] = 1.0
    vel = np.zeros((9, 3)); ang = np.zeros((9, 3))
    for j, (p, c, offp, offc, erot, _lim) in enumerate(ANT_JOINTS):
        axis = rotate(np.array([1.0, 0.0, 0.0]), euler_to_quat(f32(erot)))
        local = quat_rot_axis(axis, qpos[j])
        rot[c] = quat_mul(rot[p], local)
        anchor = pos[p] + rotate(f32(offp), rot[p])
        pos[c] = anchor - rotate(f32(offc), rot[c])
        # brax default_qp [ext]: own joint's axis * qvel rotated by the parent, no linear
        # velocity (pinned by the notebook trajectory: oracle/legacy_np.py)
        ang[c] = rotate(axis, rot[p]) * qvel[j]
    zmin = np.inf
    for i in range(9):
        ends, r = capsule_ends(i)
        for e in ends:
            zmin = min(zmin, (pos[i] + rotate(e, rot[i]))[2] - r)
    pos[:, 2] -= zmin
    return pos, rot, vel, ang

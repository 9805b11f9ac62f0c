"""CPU: libpob.so loads and exports every entry point include/pob.h declares (no compute)."""
import ctypes
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pob.h")
LIB = os.path.join(ROOT, "po-brax_amd", "po_brax_amd", "libpob.so")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pob_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert "pob_step" in names and "pob_reset" in names and len(names) >= 15


def test_lib_exports_every_declared_symbol():
    import __graft_entry__ as g
    g.build_lib()
    import torch  # noqa: F401  (same HIP runtime load order as the product)
    lib = ctypes.CDLL(LIB)
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.check_output(["nm", "-D", "--defined-only", LIB]).decode()
    exported = set(re.findall(r" T (pob_\w+)", out))
    assert set(_declared()) <= exported
    from po_brax_amd import _lib
    assert lib.pob_abi_version() == _lib.ABI_VERSION == 8


def test_python_binding_covers_header():
    from po_brax_amd import _lib
    assert set(_lib.EXPORTS) == set(_declared())


def test_default_params_without_gpu():
    from po_brax_amd import _lib
    p = _lib.pob_params()
    assert _lib.lib.pob_default_params(ctypes.byref(p)) == 0
    assert p.ga_n_apples == 8 and p.ga_n_bins == 10 and abs(p.hh_visible_radius - 2.0) < 1e-7
    assert abs(p.solver_scale_pos - 0.6) < 1e-7 and abs(p.solver_scale_ang - 0.2) < 1e-7


def test_errors_are_reported_without_gpu():
    from po_brax_amd import _lib
    import pytest
    with pytest.raises(ValueError):
        _lib.check(_lib.lib.pob_reset(None, 4, None, None, None))
    assert b"env is NULL" in _lib.lib.pob_last_error()


def _struct_fields(name):
    """Field names of `typedef struct name {...} name;` in include/pob.h, in order."""
    src = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, flags=re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = decl.strip()
        if decl:
            fields += [re.sub(r"[\s*]|\[.*\]", "", d.split()[-1] if i == 0 else d) for i, d in enumerate(decl.split(","))]
    return fields


def test_ctypes_state_layout_matches_header():
    """The ctypes mirror of pob_state lists the header's fields in the header's order (every
    field is a pointer, so equal order means equal layout)."""
    from po_brax_amd import _lib
    assert [n for n, _ in _lib.pob_state._fields_] == _struct_fields("pob_state")


def test_pybind_module_binds_the_loaded_library():
    """po_brax_amd._pob (pybind11, csrc/pob_py.cpp) is built, bound to the entry points of the
    libpob.so the ctypes layer loaded, and maps C status codes to ValueError / RuntimeError
    (no GPU needed: a NULL env is rejected before any HIP call)."""
    import __graft_entry__ as g
    g.build_pyext()
    import pytest
    from po_brax_amd import _lib
    assert _lib.pob.ENTRY_POINTS == ("pob_step", "pob_reset", "pob_reset_where_done_shard")
    assert set(_lib.pob.ENTRY_POINTS) <= set(_declared())
    with pytest.raises(ValueError, match="env is NULL"):
        _lib.pob.step(0, 4, 0, 0, 0, 0, 0, 0)
    with pytest.raises(ValueError, match="env is NULL"):
        _lib.pob.reset(0, 4, 0, 0, 0)
    with pytest.raises(ValueError, match="env is NULL"):
        _lib.pob.reset_where_done_shard(0, 4, 4, 0, 0, 0, 0, 0, 0)

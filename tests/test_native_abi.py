"""CPU checks of the C ABI library (no GPU compute): it loads, exports every entry point declared in
include/vap_hip.h, the ctypes table matches, and host-only entry points behave."""
import ctypes
import os
import re

import pytest

import vap_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "vap_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(vap_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_header_symbols():
    from voiceactivityprojection_amd import _native as N

    lib = N.lib()
    decl = header_functions()
    assert len(decl) >= 20
    for name in decl:
        assert hasattr(lib, name), f"{name} declared in include/vap_hip.h but not exported"
    assert sorted(N.EXPORTED) == decl, "ctypes signature table out of sync with include/vap_hip.h"
    assert b"gfx950" in lib.vap_build_info()


def test_library_is_gfx950_code_object():
    from voiceactivityprojection_amd import _native as N

    blob = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


@pytest.mark.parametrize("n", [320000, 37392, 320319, 960000, 160000, 32320, 40960])
def test_frame_lengths_match_oracle(n):
    from voiceactivityprojection_amd import _native as N

    assert N.frame_lengths(n) == O.frame_lengths(n)


def test_errors_are_loud():
    from voiceactivityprojection_amd import _native as N

    lib = N.lib()
    with pytest.raises(ValueError):
        N.check(lib.vap_frame_lengths(0, (ctypes.c_int64 * 6)()))
    bad = N.VapDims(128, 4, 1, 3, 1, 4, 0)
    h = ctypes.c_void_p()
    with pytest.raises(NotImplementedError):
        N.check(lib.vap_create(ctypes.byref(bad), ctypes.byref(h)))
    bad = N.VapDims(256, 8, 1, 3, 1, 4, 0)  # head_dim 32 not specialised
    with pytest.raises(NotImplementedError):
        N.check(lib.vap_create(ctypes.byref(bad), ctypes.byref(h)))


def test_no_cpu_fallback_in_product_path():
    """The engine raises on CPU tensors instead of computing on the CPU."""
    import torch
    from vap.model import VapGPT

    m = VapGPT()
    with pytest.raises(RuntimeError, match="HIP"):
        m(torch.zeros(1, 2, 40960))
    with pytest.raises(AssertionError):
        m(torch.zeros(1, 1, 40960))
    with pytest.raises(RuntimeError, match="HIP"):
        m.objective.get_labels(torch.zeros(1, 200, 2))


def _header_struct_fields(name):
    src = open(os.path.join(REPO, "include", "vap_hip.h")).read()
    body = re.search(r"typedef struct %s \{(.*?)\}" % name, src, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    return re.findall(r"\bint\s+([a-z_0-9]+)\s*;", body)


def test_integration_stub_binds_the_library(monkeypatch):
    """INTEGRATION.md §3's ctypes stub (what a maintainer would add to the reference) is executed
    against the built library, so it cannot drift from include/vap_hip.h: its VapDims must be the
    header's struct vap_dims, and vap_create / vap_num_params / vap_param_info / vap_frame_lengths
    through it must give the reference's state-dict schema and frame counts."""
    from voiceactivityprojection_amd import _native as N
    from voiceactivityprojection_amd.weights import synthetic_state_dict

    md = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", md, flags=re.S)
    stub = next(b for b in blocks if "vap/native.py" in b)
    monkeypatch.setenv("VAP_HIP_LIB", N.LIB_PATH)
    ns = {}
    exec(compile(stub, "INTEGRATION.md:stub", "exec"), ns)
    VapDims, lib, ok = ns["VapDims"], ns["_lib"], ns["_ok"]
    assert [f for f, _ in VapDims._fields_] == _header_struct_fields("vap_dims")
    assert ctypes.sizeof(VapDims) == ctypes.sizeof(N.VapDims)
    lens = (ctypes.c_int64 * 6)()
    ok(lib.vap_frame_lengths(320000, lens))
    assert list(lens) == O.frame_lengths(320000)
    for lstm in (1, 2):
        h = ctypes.c_void_p()
        ok(lib.vap_create(ctypes.byref(VapDims(256, 4, 1, 3, lstm, 4, 1, 0, 0)), ctypes.byref(h)))
        n = ctypes.c_int()
        ok(lib.vap_num_params(h, ctypes.byref(n)))
        keys = []
        for i in range(n.value):
            k, numel = ctypes.c_char_p(), ctypes.c_int64()
            ok(lib.vap_param_info(h, i, ctypes.byref(k), ctypes.byref(numel)))
            keys.append((k.value.decode(), numel.value))
        lib.vap_destroy(h)
        sd = synthetic_state_dict(seed=0, lstm_layers=lstm)
        assert sorted(keys) == sorted((k, v.size) for k, v in sd.items())


def test_product_package_does_not_import_oracle():
    for root, _, files in os.walk(os.path.join(REPO, "voiceactivityprojection_amd")):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(root, f)).read()
                assert "vap_oracle" not in txt and "oracle/" not in txt, f"{f} references the oracle"

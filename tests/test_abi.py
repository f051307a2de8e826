"""CPU: the C-ABI library loads and exports every symbol include/yalm_hip.h
declares (no compute calls: there is no GPU here)."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "yalm_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(yalm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    syms = declared_symbols()
    for s in ("yalm_upload", "yalm_free", "yalm_decoder_create", "yalm_forward", "yalm_block", "yalm_matmul",
              "yalm_mha", "yalm_ffn", "yalm_generate_greedy"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from yalm_amd import runtime

    out = subprocess.run(["nm", "-D", "--defined-only", runtime.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT (yalm_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert hasattr(runtime.lib, s)
    assert sorted(runtime.EXPORTED) == declared_symbols()


def test_library_is_gfx950_code_object():
    from yalm_amd import runtime

    data = open(runtime.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data


def test_runtime_raises_without_library(tmp_path, monkeypatch):
    """No silent fallback: a missing .so is an ImportError."""
    import importlib.util
    import shutil

    pkg = tmp_path / "yalm_amd"
    shutil.copytree(os.path.join(ROOT, "yalm_amd"), pkg, ignore=shutil.ignore_patterns("*.so", "csrc", "host"))
    spec = importlib.util.spec_from_file_location("yalm_amd_copy.runtime", pkg / "runtime.py",
                                                  submodule_search_locations=None)
    import sys
    import types

    parent = types.ModuleType("yalm_amd_copy")
    parent.__path__ = [str(pkg)]
    monkeypatch.setitem(sys.modules, "yalm_amd_copy", parent)
    mod = importlib.util.module_from_spec(spec)
    try:
        spec.loader.exec_module(mod)
    except ImportError as e:
        assert "no cpu fallback" in str(e).lower()
    else:
        raise AssertionError("runtime imported without libyalm_hip.so")

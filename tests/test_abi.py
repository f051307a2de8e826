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


def test_attn_wo_plan_host_arithmetic():
    """yalm_attn_wo_plan (pure host arithmetic, no device): Mistral-7B at 512 co-resident
    slots (2 per CU x 256) fuses with the key splits that fit beside the mergers and the
    Wo workgroups; a dim-8192 model (512 Wo workgroups) leaves fewer than 2
    splits, so it keeps the separate launches instead of running every context in head
    mode; the per-rank configs of Mistral TP2/4/8 (Wo rows of 4, 2, 1 KiB) fuse; shapes
    outside the fused contract (head_dim 64, Wo rows of 512 B) never fuse."""
    from yalm_amd import models as M
    from yalm_amd import runtime

    ok, S, grid = runtime.attn_wo_plan(M.MISTRAL_7B, 512)
    assert ok and S == 25 and grid == 8 * (S + 3) + 32 + 256
    big = M.MISTRAL_7B.with_(dim=8192)
    assert runtime.attn_wo_plan(big, 512)[0] is False
    # short windows (all contexts in head mode) may fuse with S = 1
    ok, S, _ = runtime.attn_wo_plan(big.with_(max_seq_len=256), 512)
    assert ok and S == 1
    assert runtime.attn_wo_plan(M.MISTRAL_7B.with_(head_dim=64, n_heads=64, n_kv_heads=16), 512)[0] is False
    for tp in (2, 4, 8):
        local = M.MISTRAL_7B.with_(n_heads=32 // tp, n_kv_heads=8 // tp, hidden_dim=14336 // tp,
                                   vocab_size=32000 // tp)
        ok, S, grid = runtime.attn_wo_plan(local, 512)
        assert ok and 2 <= S <= 32 and grid <= 512, (tp, S, grid)
    assert runtime.attn_wo_plan(M.MISTRAL_7B.with_(n_heads=2, n_kv_heads=2), 512)[0] is False
    assert runtime.attn_wo_plan(M.MISTRAL_7B.with_(n_heads=4, n_kv_heads=1, weight_dtype=M.F8E5M2), 512)[0] is False


def test_prefill_forms_spec_validation():
    """yalm_set_prefill_forms: explicit forms, no environment; a bad key / width is an
    argument error (no device is touched for the NULL-decoder test-hook forms)."""
    import pytest
    from yalm_amd import runtime

    runtime.set_gemm_forms("qkv:256,wo:192,8p:0,persist:0,skinny:0,qkv1:0,skl:0")
    runtime.set_gemm_forms("")
    for bad in ("bogus:1", "qkv:100", "qkv", "8p=0"):
        with pytest.raises(runtime.YalmError):
            runtime.set_gemm_forms(bad)
    runtime.set_gemm_forms("")

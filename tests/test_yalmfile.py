""".yalm format + converter parity against fixtures produced by the
REFERENCE converter (/root/reference/convert.py, run once here by
tests/golden/make_golden.py; the outputs are committed data)."""
import json
import os
import struct

import numpy as np
import pytest

from golden import make_golden
from yalm_amd import convert, models as M, yalmfile


def _header(path):
    d = open(path, "rb").read()
    n = struct.unpack("<Q", d[:8])[0]
    h = json.loads(d[8:8 + n])
    md = h.pop("__metadata__")
    return md, h, [k for k in h], d[8 + n:]


@pytest.mark.parametrize("dt,tie", [("fp32", False), ("fp16", False), ("fp8", False), ("fp16", True)])
def test_converter_matches_reference_convert_py(tmp_path, golden_dir, dt, tie):
    """Our numpy converter vs reference convert.py output on the same HF dir:
    identical metadata, tensor layout (order, dtype, shape, offsets) and data
    bytes. (convert.py itself is not byte-reproducible: safetensors writes
    __metadata__ from a hash map, so only its key order may differ.)"""
    hf = tmp_path / "hf"
    make_golden.write_hf_dir(str(hf), tie=tie)
    out = tmp_path / "out.yalm"
    convert.convert(str(hf), str(out), dt)
    ref = os.path.join(golden_dir, f"tiny_{dt}{'_tied' if tie else ''}.yalm")
    md1, h1, k1, b1 = _header(ref)
    md2, h2, k2, b2 = _header(str(out))
    assert md1 == md2
    assert k1 == k2
    assert h1 == h2
    assert b1 == b2


def test_read_reference_fixture(golden_dir):
    yd = yalmfile.read_yalm(os.path.join(golden_dir, "tiny_fp16.yalm"))
    cfg = M.config_from_metadata(yd.metadata)
    assert (cfg.dim, cfg.hidden_dim, cfg.n_layers, cfg.n_heads, cfg.n_kv_heads, cfg.vocab_size) == (
        64, 128, 2, 4, 2, 384)
    assert cfg.act == M.SILU and cfg.weight_dtype == M.F16 and cfg.max_seq_len == 64
    shapes = M.tensor_shapes(cfg)
    for name, (shape, is_norm) in shapes.items():
        t = yd.tensors[name]
        assert t.shape == shape
        assert t.dtype == ("F32" if is_norm else "F16")
    tok = yd.tensors["tokenizer.tokens"].data.tobytes().split(b"\0")[:-1]
    assert len(tok) == 384 and tok[1] == b"<s>" and tok[3] == b"<0x00>"
    yd.close()


def test_roundtrip(tmp_path):
    cfg = M.TINY.with_(weight_dtype=M.F8E5M2)
    t = M.synth_host_tensors(cfg, seed=2)
    dts = {k: ("F32" if v.dtype == np.float32 else "F8_E5M2") for k, v in t.items()}
    p = tmp_path / "m.yalm"
    yalmfile.write_yalm(str(p), t, cfg.metadata(), dts)
    yd = yalmfile.read_yalm(str(p))
    assert M.config_from_metadata(yd.metadata).weight_dtype == M.F8E5M2
    for k, v in t.items():
        np.testing.assert_array_equal(yd.tensors[k].data.reshape(v.shape), v)
    yd.close()


def test_max_seq_len_cap_and_context():
    """model.cpp:31-36: min(meta, 4096), overridden by -T context."""
    md = M.MISTRAL_7B.with_(max_seq_len=32768).metadata()
    assert M.config_from_metadata(md).max_seq_len == 4096
    assert M.config_from_metadata(md, context=512).max_seq_len == 512


def test_e5m2_conversion_matches_torch():
    torch = pytest.importorskip("torch")
    rng = np.random.default_rng(0)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s for s in (1e-6, 1e-3, 1, 1e3, 1e5)])
    x = np.concatenate([x, np.array([0.0, -0.0, 65536.0, 57344.0, 61440.0, np.inf, -np.inf], np.float32)])
    ref = torch.from_numpy(x).to(torch.float8_e5m2).view(torch.uint8).numpy()
    np.testing.assert_array_equal(convert.f32_to_e5m2(x), ref)


def test_bad_files(tmp_path):
    p = tmp_path / "bad.yalm"
    p.write_bytes(b"\x00" * 4)
    with pytest.raises(yalmfile.YalmFormatError):
        yalmfile.read_yalm(str(p))
    hdr = json.dumps({"a": {"dtype": "F32", "shape": [4], "data_offsets": [0, 8]}}).encode()
    p.write_bytes(struct.pack("<Q", len(hdr)) + hdr + b"\0" * 16)
    with pytest.raises(yalmfile.YalmFormatError):
        yalmfile.read_yalm(str(p))  # bad size (codec.cpp:108-111)

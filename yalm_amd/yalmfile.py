""".yalm file reader/writer (pure Python + numpy).

A .yalm file is a safetensors file (reference codec.cpp:116-175): an 8-byte
little-endian header length, a JSON header holding ``__metadata__`` (all
values strings, convert.py:59-81) and per-tensor ``dtype``/``shape``/
``data_offsets``, then the packed tensor bytes. Reading memory-maps the file
and returns zero-copy numpy views (the reference mmaps too, codec.cpp:130).
"""

from __future__ import annotations

import json
import mmap
import struct
from dataclasses import dataclass, field

import numpy as np

# safetensors dtype strings accepted by the reference (codec.cpp:58-80)
DTYPE_SIZE = {"F32": 4, "F16": 2, "BF16": 2, "F8_E5M2": 1, "F8_E4M3": 1, "I32": 4, "I16": 2, "I8": 1, "U8": 1}
# numpy storage types (fp8 and bf16 are kept as raw unsigned bits)
NP_STORAGE = {
    "F32": np.float32,
    "F16": np.float16,
    "BF16": np.uint16,
    "F8_E5M2": np.uint8,
    "F8_E4M3": np.uint8,
    "I32": np.int32,
    "I16": np.int16,
    "I8": np.int8,
    "U8": np.uint8,
}


# safetensors' serialisation order: dtype descending in its Dtype enum order,
# then name (so a .yalm we write has the same tensor layout as convert.py's).
DTYPE_RANK = {"U8": 4, "I8": 5, "F8_E5M2": 6, "F8_E4M3": 7, "I16": 9, "F16": 11, "BF16": 12, "I32": 13, "F32": 15}


class YalmFormatError(ValueError):
    pass


@dataclass
class Tensor:
    name: str
    dtype: str
    shape: tuple
    data: np.ndarray  # flat view of the raw storage

    @property
    def nbytes(self) -> int:
        return self.data.nbytes


@dataclass
class YalmData:
    metadata: dict = field(default_factory=dict)
    tensors: dict = field(default_factory=dict)
    _mm: object = None

    def close(self):
        self.tensors = {}
        if self._mm is not None:
            try:
                self._mm.close()
            except BufferError:
                pass  # live numpy views keep the mapping; it closes with them
            self._mm = None


def read_yalm(path: str) -> YalmData:
    """YALMData::from_file (codec.cpp:116-175) + Tensor::from_json (codec.cpp:58-114)."""
    with open(path, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    size = len(mm)
    if size < 8:
        raise YalmFormatError("file too small")
    (json_size,) = struct.unpack("<Q", mm[:8])
    if json_size == 0 or json_size > size - 8:
        raise YalmFormatError("bad header length")
    header = json.loads(bytes(mm[8 : 8 + json_size]).decode("utf-8"))
    base = 8 + json_size
    bytes_size = size - base
    buf = np.frombuffer(mm, dtype=np.uint8)
    out = YalmData(_mm=mm)
    for key, val in header.items():
        if key == "__metadata__":
            out.metadata = dict(val)
            continue
        dt = val.get("dtype", "")
        if dt not in DTYPE_SIZE:
            raise YalmFormatError(f"bad dtype for {key}: {dt!r}")
        shape = tuple(int(s) for s in val["shape"])
        if len(shape) > 4:
            raise YalmFormatError(f"{key}: shape exceeds 4 dimensions")
        offs = val["data_offsets"]
        if len(offs) != 2:
            raise YalmFormatError(f"{key}: bad data_offsets")
        start, end = int(offs[0]), int(offs[1])
        if start < 0 or end <= start or end > bytes_size:
            raise YalmFormatError(f"{key}: bad offsets")
        numel = int(np.prod(shape)) if shape else 1
        if numel * DTYPE_SIZE[dt] != end - start:
            raise YalmFormatError(f"{key}: bad size")
        raw = buf[base + start : base + end]
        out.tensors[key] = Tensor(key, dt, shape, raw.view(NP_STORAGE[dt]))
    return out


def _np_dtype_code(arr: np.ndarray, dtype: str | None) -> str:
    if dtype is not None:
        return dtype
    if arr.dtype == np.float32:
        return "F32"
    if arr.dtype == np.float16:
        return "F16"
    if arr.dtype == np.uint8:
        return "U8"
    if arr.dtype == np.int32:
        return "I32"
    raise YalmFormatError(f"cannot infer safetensors dtype for {arr.dtype}")


def write_yalm(path: str, tensors: dict, metadata: dict, dtypes: dict | None = None) -> None:
    """Write a .yalm (safetensors layout). ``tensors`` maps name -> ndarray;
    ``dtypes`` optionally overrides the dtype string (e.g. "F8_E5M2" for raw
    uint8 E5M2 bytes). Tensors are laid out in safetensors' order (DTYPE_RANK,
    then name) and the header is padded to 8 bytes, as safetensors does."""
    dtypes = dtypes or {}
    items = []
    for name, arr in tensors.items():
        arr = np.ascontiguousarray(arr)
        items.append((name, _np_dtype_code(arr, dtypes.get(name)), arr))
    items.sort(key=lambda t: (-DTYPE_RANK[t[1]], t[0]))
    header = {"__metadata__": {k: str(v) for k, v in metadata.items()}}
    off = 0
    for name, dt, arr in items:
        header[name] = {"dtype": dt, "shape": list(arr.shape), "data_offsets": [off, off + arr.nbytes]}
        off += arr.nbytes
    hb = json.dumps(header, separators=(",", ":")).encode("utf-8")
    hb += b" " * ((8 - len(hb) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for _, _, arr in items:
            f.write(arr.tobytes())

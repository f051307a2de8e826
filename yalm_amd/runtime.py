"""ctypes binding of libyalm_hip.so (C ABI: include/yalm_hip.h).

Python mirror of the reference's device-facing API: ``DeviceModel`` is
``Model::cuda()`` (model.cpp:380-394, weights uploaded once, tied embedding
not duplicated), ``Decoder`` is ``InferenceState::cuda()`` + ``Model::forward``
(model.cpp:323-345, 396-407). Every call goes through the HIP library; there
is no CPU path here (the CPU oracle lives in oracle/, test-only).
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import models as M

HERE = os.path.dirname(os.path.abspath(__file__))
# YALM_LIB: another build of the same ABI (A/B timing of two revisions, tools/build_ab_lib.sh)
LIB_PATH = os.environ.get("YALM_LIB") or os.path.join(HERE, "libyalm_hip.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} is missing: build it with `make -C {os.path.dirname(HERE)}` "
        "(or __graft_entry__.build()). There is no CPU fallback."
    )

lib = ctypes.CDLL(LIB_PATH)

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_float = ctypes.c_float
c_size_t = ctypes.c_size_t


class Config(ctypes.Structure):
    """yalm_config (model.h:41-68)."""

    _fields_ = [
        ("dim", c_int),
        ("hidden_dim", c_int),
        ("head_dim", c_int),
        ("n_layers", c_int),
        ("n_heads", c_int),
        ("n_kv_heads", c_int),
        ("vocab_size", c_int),
        ("max_seq_len", c_int),
        ("rope_theta", c_float),
        ("rotary_dim", c_int),
        ("norm_eps", c_float),
        ("act", c_int),
        ("qkv_clip", c_float),
        ("weight_dtype", c_int),
    ]

    @classmethod
    def from_model(cls, c: M.ModelConfig) -> "Config":
        return cls(
            c.dim, c.hidden_dim, c.head_dim, c.n_layers, c.n_heads, c.n_kv_heads, c.vocab_size, c.max_seq_len,
            c.rope_theta, c.rotary_dim, c.norm_eps, c.act, c.qkv_clip, c.weight_dtype,
        )


class BlockWeights(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("rms_att", "rms_ffn", "wq", "wk", "wv", "wo", "w1", "w2", "w3",
                                        "key_cache", "value_cache")]


class ModelWeights(ctypes.Structure):
    _fields_ = [("token_embedding", c_void_p), ("rms_final", c_void_p), ("wcls", c_void_p),
                ("blocks", ctypes.POINTER(BlockWeights))]


def _sig(name, restype, argtypes):
    if os.environ.get("YALM_LIB") and not hasattr(lib, name):
        return None  # an older build under A/B timing may lack newer entry points
    f = getattr(lib, name)
    f.restype = restype
    f.argtypes = argtypes
    return f


_sig("yalm_last_error", ctypes.c_char_p, [])
_sig("yalm_set_device", c_int, [c_int])
_sig("yalm_upload", c_void_p, [c_void_p, c_size_t])
_sig("yalm_alloc", c_void_p, [c_size_t])
_sig("yalm_download", c_int, [c_void_p, c_void_p, c_size_t])
_sig("yalm_register_host", c_int, [c_void_p, c_size_t])
_sig("yalm_unregister_host", c_int, [c_void_p])
_sig("yalm_free", c_int, [c_void_p])
_sig("yalm_stream_create", c_int, [ctypes.POINTER(c_void_p)])
_sig("yalm_stream_destroy", c_int, [c_void_p])
_sig("yalm_stream_sync", c_int, [c_void_p])
_sig("yalm_synth", c_int, [c_void_p, c_size_t, c_int, ctypes.c_uint64, c_float, c_float, c_void_p])
_sig("yalm_decoder_create", c_int, [ctypes.POINTER(Config), ctypes.POINTER(ModelWeights), c_void_p,
                                     ctypes.POINTER(c_void_p)])
_sig("yalm_decoder_destroy", c_int, [c_void_p])
_sig("yalm_forward", c_int, [c_void_p, c_int, c_int, c_int, c_void_p])
_sig("yalm_generate_greedy", c_int, [c_void_p, c_int, c_int, c_int, c_void_p])
_sig("yalm_enqueue_greedy", c_int, [c_void_p, c_int])
_sig("yalm_device_step", c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
_sig("yalm_device_tokens", c_int, [c_void_p, c_void_p, c_int, ctypes.POINTER(c_int)])
_sig("yalm_block", c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int])
_sig("yalm_get_x", c_int, [c_void_p, c_void_p])
_sig("yalm_set_x", c_int, [c_void_p, c_void_p])
_sig("yalm_get_logits", c_int, [c_void_p, c_void_p])
_sig("yalm_time_kernel", c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_float)])
_sig("yalm_kernel_name", ctypes.c_char_p, [c_void_p, c_int])
_sig("yalm_set_gemv_config", c_int, [c_void_p, c_int, c_int, c_int, c_int])
_sig("yalm_stream_envelope", c_int, [ctypes.c_size_t, c_int, ctypes.POINTER(c_float)])
_sig("yalm_decoder_attn_wo", c_int, [c_void_p])
_sig("yalm_attn_wo_trace", c_int, [c_void_p, c_void_p, ctypes.c_size_t, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
_sig("yalm_matmul", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int])
_sig("yalm_mha", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int])
_sig("yalm_argmax", c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_int)])
_sig("yalm_ffn", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int])
_sig("yalm_prefill", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p])
_sig("yalm_tp_unique_id", c_int, [c_void_p])
_sig("yalm_decoder_create_tp", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p])
_sig("yalm_tp_ipc_alloc", c_int, [c_void_p, c_int, c_void_p, ctypes.POINTER(c_void_p), c_void_p])
_sig("yalm_stream_create_cu_part", c_int, [c_int, c_int, ctypes.POINTER(c_void_p)])
_sig("yalm_decoder_set_launch", c_int, [c_void_p, c_int])
_sig("yalm_decoder_create_tp_ipc", c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p])
_sig("yalm_copy_2d", c_int, [c_void_p, ctypes.c_size_t, c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t])
_sig("yalm_prefill_time", c_int, [c_void_p, c_int, c_int, ctypes.POINTER(c_float)])
_sig("yalm_prefill_info", c_int, [c_void_p, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
_sig("yalm_set_prefill_precision", c_int, [c_void_p, c_int])
_sig("yalm_gemm_f16", c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int])
_sig("yalm_attn_prefill", c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int])
_sig("yalm_set_prefill_forms", c_int, [c_void_p, ctypes.c_char_p])
_sig("yalm_graph_kernels", c_int, [c_void_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])
_sig("yalm_attn_wo_plan", c_int, [c_void_p, c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)])

EXPORTED = [
    "yalm_last_error", "yalm_set_device", "yalm_upload", "yalm_alloc", "yalm_download", "yalm_register_host",
    "yalm_unregister_host", "yalm_free", "yalm_stream_create", "yalm_stream_destroy", "yalm_stream_sync",
    "yalm_synth", "yalm_decoder_create", "yalm_decoder_destroy", "yalm_forward", "yalm_generate_greedy",
    "yalm_enqueue_greedy", "yalm_device_step", "yalm_device_tokens", "yalm_block", "yalm_get_x", "yalm_set_x", "yalm_get_logits",
    "yalm_time_kernel", "yalm_kernel_name", "yalm_set_gemv_config", "yalm_matmul", "yalm_mha", "yalm_ffn",
    "yalm_prefill", "yalm_prefill_time", "yalm_gemm_f16", "yalm_attn_prefill", "yalm_tp_unique_id",
    "yalm_decoder_create_tp", "yalm_copy_2d", "yalm_tp_ipc_alloc", "yalm_decoder_create_tp_ipc",
    "yalm_decoder_attn_wo", "yalm_attn_wo_trace", "yalm_stream_envelope",
    "yalm_argmax", "yalm_set_prefill_forms", "yalm_attn_wo_plan", "yalm_graph_kernels",
    "yalm_stream_create_cu_part", "yalm_decoder_set_launch", "yalm_prefill_info", "yalm_set_prefill_precision",
]
PREFILL_FAST, PREFILL_SPLIT = 0, 1  # yalm_set_prefill_precision

HYDRATE_KV_CACHE, OUTPUT_LOGITS = 0, 1
# yalm_decoder_set_launch flags (include/yalm_hip.h)
LAUNCH_EAGER, LAUNCH_SYNC, LAUNCH_SEPARATE_ATTN_WO = 1, 2, 4
TP_HANDLE_BYTES = 128  # YALM_TP_HANDLE_BYTES: IPC handle + GPU UUID + CU mask


class YalmError(RuntimeError):
    pass


def check(rc: int) -> None:
    if rc != 0:
        raise YalmError(f"yalm error {rc}: {lib.yalm_last_error().decode()}")


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


# ------------------------------------------------------------- kernel-level test API
def matmul(x: np.ndarray, w: np.ndarray, dtype: int) -> np.ndarray:
    """matmul_cuda (infer.cu:937-957): W (d, n) @ x (n,)."""
    d, n = w.shape
    x = np.ascontiguousarray(x, dtype=np.float32)
    w = np.ascontiguousarray(w)
    out = np.zeros(d, np.float32)
    check(lib.yalm_matmul(_ptr(out), _ptr(x), _ptr(w), n, d, dtype))
    return out


def mha(kb, vb, q, head_dim, kv_len, max_seq_len, n_heads, n_kv_heads, att_init=None):
    """mha_cuda (infer.cu:890-935): returns (xout, att)."""
    kb = np.ascontiguousarray(kb, dtype=np.float16).view(np.uint16)
    vb = np.ascontiguousarray(vb, dtype=np.float16).view(np.uint16)
    q = np.ascontiguousarray(q, dtype=np.float32)
    xout = np.zeros(n_heads * head_dim, np.float32)
    att = np.zeros(n_heads * max_seq_len, np.float32) if att_init is None else np.array(att_init, np.float32)
    check(lib.yalm_mha(_ptr(xout), _ptr(att), _ptr(kb), _ptr(vb), _ptr(q), head_dim, kv_len, max_seq_len, n_heads,
                       n_kv_heads))
    return xout, att


def argmax(logits: np.ndarray, n_shards: int = 1) -> int:
    """Device argmax (sampler.cpp:27-38 semantics) of host logits; n_shards > 1:
    the tensor-parallel per-shard pairs + pick."""
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    out = c_int()
    check(lib.yalm_argmax(_ptr(lg), lg.size, n_shards, ctypes.byref(out)))
    return out.value


def ffn(x, w1, w2, w3, act: int, dtype: int) -> np.ndarray:
    """ffn_cuda (infer.cu:959-1007)."""
    hidden_dim, dim = w1.shape
    x = np.ascontiguousarray(x, dtype=np.float32)
    w1, w2, w3 = (np.ascontiguousarray(a) for a in (w1, w2, w3))
    out = np.zeros(dim, np.float32)
    check(lib.yalm_ffn(_ptr(out), _ptr(x), _ptr(w1), _ptr(w2), _ptr(w3), hidden_dim, dim, act, dtype))
    return out


def stream_envelope(nbytes: int, iters: int = 16) -> float:
    """ms of one pure HBM read pass over nbytes (yalm_stream_envelope)."""
    ms = c_float()
    check(lib.yalm_stream_envelope(nbytes, iters, ctypes.byref(ms)))
    return ms.value


class Stream:
    """A decoder stream; cu_part = (part, n_parts): restricted to CU block `part` of
    n_parts (yalm_stream_create_cu_part), so n_parts rank processes on one GPU run on
    disjoint CUs -- the one-GPU rehearsal of tensor parallelism."""

    def __init__(self, cu_part=None):
        self.h = c_void_p()
        if cu_part is None:
            check(lib.yalm_stream_create(ctypes.byref(self.h)))
        else:
            check(lib.yalm_stream_create_cu_part(cu_part[0], cu_part[1], ctypes.byref(self.h)))

    def close(self):
        if self.h:
            check(lib.yalm_stream_destroy(self.h))
            self.h = None


def tp_unique_id() -> bytes:
    """RCCL unique id for yalm_decoder_create_tp (rank 0 makes it, all ranks use it)."""
    buf = ctypes.create_string_buffer(128)
    check(lib.yalm_tp_unique_id(buf))
    return buf.raw


def gemm_f16(a: np.ndarray, w: np.ndarray) -> np.ndarray:
    """MFMA GEMM of the prefill path: a (M, K) f16 @ w (N, K)^T f16 -> (M, N) f32."""
    a = np.ascontiguousarray(a, dtype=np.float16)
    w = np.ascontiguousarray(w, dtype=np.float16)
    (M, K), N = a.shape, w.shape[0]
    c = np.zeros((M, N), np.float32)
    check(lib.yalm_gemm_f16(_ptr(c), _ptr(a), _ptr(w), M, N, K))
    return c


def set_gemm_forms(spec: str = "") -> None:
    """The prefill GEMM forms of the gemm_f16 test hook (yalm_set_prefill_forms(NULL, spec))."""
    check(lib.yalm_set_prefill_forms(None, spec.encode() if spec else None))


def attn_wo_plan(cfg: M.ModelConfig, slots: int):
    """(fused?, key splits, grid) of the fused attention + Wo launch for cfg at `slots`
    co-resident workgroups (yalm_attn_wo_plan: host arithmetic, no device)."""
    c = Config.from_model(cfg)
    s, g = c_int(), c_int()
    ok = lib.yalm_attn_wo_plan(ctypes.byref(c), slots, ctypes.byref(s), ctypes.byref(g))
    return bool(ok), s.value, g.value


def attn_prefill(q, kc, vc, T, pos0, n_heads, n_kv_heads, head_dim) -> np.ndarray:
    """Causal GQA prefill attention: q (T, n_heads*D) f16, kc/vc (pos0+T, n_kv*D) f16 -> (T, n_heads*D) f16."""
    q = np.ascontiguousarray(q, dtype=np.float16)
    kc = np.ascontiguousarray(kc, dtype=np.float16)
    vc = np.ascontiguousarray(vc, dtype=np.float16)
    o = np.zeros((T, n_heads * head_dim), np.float16)
    check(lib.yalm_attn_prefill(_ptr(o), _ptr(q), _ptr(kc), _ptr(vc), T, pos0, n_heads, n_kv_heads, head_dim))
    return o


# ------------------------------------------------------------- model + decoder
class DeviceModel:
    """Model::cuda(): all weights resident in HBM (one allocation per tensor;
    a tied classifier aliases the embedding instead of a second upload, unlike
    model.cpp:388/393)."""

    def __init__(self, cfg: M.ModelConfig):
        self.cfg = cfg
        self.ptrs: dict = {}
        self._owned: list = []
        self.tp = (0, 1)

    def _alloc(self, nbytes: int) -> int:
        p = lib.yalm_alloc(nbytes)
        if not p:
            raise YalmError(lib.yalm_last_error().decode())
        self._owned.append(p)
        return p

    @classmethod
    def from_arrays(cls, cfg: M.ModelConfig, tensors: dict, tp=(0, 1)) -> "DeviceModel":
        """Upload host tensors (numpy; names as in .yalm). tp = (rank, size):
        upload only this rank's shards (models.tp_shard)."""
        rank, size = tp
        M.tp_check(cfg, size)
        self = cls(cfg)
        self.tp = tp
        items = dict(tensors)
        if size > 1 and cfg.tied:
            items["tp.wcls"] = tensors["model.embed.weight"]
        for name in list(M.tensor_shapes(cfg)) + (["tp.wcls"] if size > 1 and cfg.tied else []):
            a = np.ascontiguousarray(M.shard_array(cfg, name, items[name], rank, size))
            p = lib.yalm_upload(a.ctypes.data, a.nbytes)
            if not p:
                raise YalmError(lib.yalm_last_error().decode())
            self._owned.append(p)
            self.ptrs[name] = p
        return self

    @classmethod
    def from_yalm(cls, path: str, context: int = 0) -> "DeviceModel":
        from .yalmfile import read_yalm

        yd = read_yalm(path)
        tied = "model.output.weight" not in yd.tensors
        cfg = M.config_from_metadata(yd.metadata, context, tied)
        arrays = {k: t.data for k, t in yd.tensors.items()}
        try:
            return cls.from_arrays(cfg, arrays)
        finally:
            arrays.clear()
            yd.close()

    @classmethod
    def synthetic(cls, cfg: M.ModelConfig, seed: int = 1, tp=(0, 1), peak: float = 1.0,
                  real: "M.Realistic" = None) -> "DeviceModel":
        """Random-weight model of cfg's shape generated directly in HBM with the
        deterministic hash shared with the oracle (no PCIe upload). tp = (rank,
        size): keep only this rank's shards — each sharded tensor is generated
        whole in a scratch buffer and its slice copied out (yalm_copy_2d), so
        every rank holds exactly the slices of the same full model. real: the
        realistic model (models.Realistic): each patched tensor is downloaded, patched
        by models.realistic_patch and uploaded again (single GPU only)."""
        rank, size = tp
        M.tp_check(cfg, size)
        if real is not None and size > 1:
            raise ValueError("the realistic synthetic model is built for one GPU (tp size 1)")
        self = cls(cfg)
        self.tp = tp
        names = list(M.tensor_shapes(cfg).items())
        if size > 1 and cfg.tied:
            names.append(("tp.wcls", ((cfg.vocab_size, cfg.dim), False)))
        for name, (shape, is_norm) in names:
            n = int(np.prod(shape))
            dt = M.F32 if is_norm else cfg.weight_dtype
            eb = M.DTYPE_BYTES[dt]
            src_name = "model.embed.weight" if name == "tp.wcls" else name
            scale, offset = M.synth_params(src_name, is_norm, peak, real, cfg.tied)
            sh = M.tp_shard(cfg, name, rank, size)
            if sh is None:
                p = self._alloc(n * eb)
                check(lib.yalm_synth(p, n, dt, M.synth_seed(seed, src_name), scale, offset, None))
            else:
                full = lib.yalm_alloc(n * eb)
                if not full:
                    raise YalmError(lib.yalm_last_error().decode())
                try:
                    check(lib.yalm_synth(full, n, dt, M.synth_seed(seed, src_name), scale, offset, None))
                    kind, start, cnt = sh
                    rows, cols = shape
                    if kind == "rows":
                        p = self._alloc(cnt * cols * eb)
                        check(lib.yalm_copy_2d(p, cols * eb, full + start * cols * eb, cols * eb, cols * eb, cnt))
                    else:
                        p = self._alloc(rows * cnt * eb)
                        check(lib.yalm_copy_2d(p, cnt * eb, full + start * eb, cols * eb, cnt * eb, rows))
                finally:
                    check(lib.yalm_stream_sync(None))
                    lib.yalm_free(full)
            self.ptrs[name] = p
        check(lib.yalm_stream_sync(None))
        if real is not None:
            shapes = M.tensor_shapes(cfg)
            for name in M.realistic_names(cfg):
                shape, is_norm = shapes[name]
                dt = M.F32 if is_norm else cfg.weight_dtype
                a = np.empty(shape, {M.F32: np.float32, M.F16: np.float16, M.F8E5M2: np.uint8}[dt])
                check(lib.yalm_download(a.ctypes.data, self.ptrs[name], a.nbytes))
                M.realistic_patch(cfg, name, a, real)
                p = lib.yalm_upload(a.ctypes.data, a.nbytes)
                if not p:
                    raise YalmError(lib.yalm_last_error().decode())
                old = self.ptrs[name]
                self._owned[self._owned.index(old)] = p
                lib.yalm_free(old)
                self.ptrs[name] = p
        return self

    def weights_struct(self):
        cfg = self.cfg
        blocks = (BlockWeights * cfg.n_layers)()
        for l in range(cfg.n_layers):
            n = M.layer_names(l)
            for k, name in n.items():
                setattr(blocks[l], k, self.ptrs[name])
        emb = self.ptrs["model.embed.weight"]
        wcls = self.ptrs.get("model.output.weight", self.ptrs.get("tp.wcls", emb))
        mw = ModelWeights(emb, self.ptrs["model.norm.weight"], wcls, blocks)
        return mw, blocks

    def close(self):
        for p in self._owned:
            lib.yalm_free(p)
        self._owned = []
        self.ptrs = {}


class Decoder:
    """InferenceState on the device + Model::forward (graph-replayed)."""

    def __init__(self, model: DeviceModel, tp_id: bytes = None, tp_gather=None, kv_caches=None,
                 cu_part=None, launch: int = 0):
        """Tensor parallel over model.tp = (rank, size), one of:
        tp_id: the RCCL unique id (tp_unique_id() on rank 0, shared with the
        other ranks); tp_gather: a function mapping this rank's 128-byte rank
        record (IPC handle, GPU UUID, CU mask) to the list of every rank's record
        (e.g. via torch.distributed.all_gather_object) for the IPC exchange transport.
        Neither: a single-GPU decoder. kv_caches: optional per-layer (key, value)
        device pointers ([max_seq_len][kv_dim] f16 each, caller-owned), as
        Block::cuda() hands its own caches over (model.cpp:185-211); default: the
        decoder allocates zeroed caches. cu_part = (part, n_parts): decode on a
        stream restricted to that CU block (Stream). launch: yalm_decoder_set_launch
        flags (LAUNCH_*)."""
        self.model = model
        self.cfg = model.cfg
        self._c = Config.from_model(self.cfg)
        mw, self._blocks = model.weights_struct()
        if kv_caches is not None:
            for l, (kp, vp) in enumerate(kv_caches):
                self._blocks[l].key_cache = kp
                self._blocks[l].value_cache = vp
        self._mw = mw
        self.h = None
        self.stream = Stream(cu_part) if cu_part is not None else None
        sh = self.stream.h if self.stream else None
        h = c_void_p()
        if tp_gather is not None:
            rank, size = getattr(model, "tp", (0, 1))
            buf = c_void_p()
            handle = ctypes.create_string_buffer(TP_HANDLE_BYTES)
            check(lib.yalm_tp_ipc_alloc(ctypes.byref(self._c), size, sh, ctypes.byref(buf), handle))
            handles = tp_gather(handle.raw)
            assert len(handles) == size and all(len(x) == TP_HANDLE_BYTES for x in handles)
            hb = ctypes.create_string_buffer(b"".join(handles), TP_HANDLE_BYTES * size)
            check(lib.yalm_decoder_create_tp_ipc(ctypes.byref(self._c), ctypes.byref(mw), rank, size, buf, hb, sh,
                                                 ctypes.byref(h)))
        elif tp_id is None:
            check(lib.yalm_decoder_create(ctypes.byref(self._c), ctypes.byref(mw), sh, ctypes.byref(h)))
        else:
            rank, size = getattr(model, "tp", (0, 1))
            idb = ctypes.create_string_buffer(bytes(tp_id), 128)
            check(lib.yalm_decoder_create_tp(ctypes.byref(self._c), ctypes.byref(mw), rank, size, idb, sh,
                                             ctypes.byref(h)))
        self.h = h
        if launch:
            self.set_launch(launch)

    def set_launch(self, flags: int) -> None:
        """yalm_decoder_set_launch: LAUNCH_EAGER | LAUNCH_SYNC | LAUNCH_SEPARATE_ATTN_WO (0 = default)."""
        check(lib.yalm_decoder_set_launch(self.h, flags))

    def forward(self, token: int, pos: int, mode: int = OUTPUT_LOGITS):
        if mode == OUTPUT_LOGITS:
            out = np.empty(self.cfg.vocab_size, np.float32)
            check(lib.yalm_forward(self.h, token, pos, mode, out.ctypes.data))
            return out
        check(lib.yalm_forward(self.h, token, pos, mode, None))
        return None

    def prefill(self, tokens, pos0: int = 0, logprobs: bool = True):
        """Batched MFMA prefill of positions pos0.. (fills the KV cache); returns
        log p(tokens[i+1] | ..tokens[i]) per position (last entry 0) or None."""
        tok = np.ascontiguousarray(tokens, dtype=np.int32)
        out = np.zeros(len(tok), np.float32) if logprobs else None
        check(lib.yalm_prefill(self.h, _ptr(tok), len(tok), pos0, _ptr(out) if logprobs else None))
        return out

    def set_prefill_precision(self, mode: int) -> None:
        """PREFILL_FAST (f16 activation operands) or PREFILL_SPLIT (every operand [hi | lo])."""
        check(lib.yalm_set_prefill_precision(self.h, mode))

    def prefill_info(self):
        """(passes, scaled layers) of the last prefill: the f16 range guard's re-runs."""
        p, n = c_int(), c_int()
        check(lib.yalm_prefill_info(self.h, ctypes.byref(p), ctypes.byref(n)))
        return p.value, n.value

    def set_prefill_forms(self, spec: str = "") -> None:
        """Select another exact prefill GEMM form (yalm_set_prefill_forms), "" = defaults."""
        check(lib.yalm_set_prefill_forms(self.h, spec.encode() if spec else None))

    def prefill_time(self, n: int, iters: int = 3) -> float:
        ms = c_float()
        check(lib.yalm_prefill_time(self.h, n, iters, ctypes.byref(ms)))
        return ms.value

    def generate_greedy(self, token: int, pos: int, n: int) -> list:
        out = np.zeros(max(n, 1), np.int32)
        check(lib.yalm_generate_greedy(self.h, token, pos, n, out.ctypes.data))
        return out[:n].tolist()

    def enqueue_greedy(self, n: int) -> None:
        check(lib.yalm_enqueue_greedy(self.h, n))

    def device_step(self):
        t, p = c_int(), c_int()
        check(lib.yalm_device_step(self.h, ctypes.byref(t), ctypes.byref(p)))
        return t.value, p.value

    def device_tokens(self, cap: int = 1 << 16) -> list:
        """Greedy tokens produced on the device since the last generate_greedy."""
        out = np.zeros(max(cap, 1), np.int32)
        n = c_int()
        check(lib.yalm_device_tokens(self.h, out.ctypes.data, cap, ctypes.byref(n)))
        return out[:min(n.value, cap)].tolist()

    def block(self, layer, pos, kv_sink, kv_pos, kv_len):
        check(lib.yalm_block(self.h, layer, pos, kv_sink, kv_pos, kv_len))

    def get_x(self) -> np.ndarray:
        out = np.empty(self.cfg.dim, np.float32)
        check(lib.yalm_get_x(self.h, out.ctypes.data))
        return out

    def set_x(self, x: np.ndarray) -> None:
        x = np.ascontiguousarray(x, dtype=np.float32)
        check(lib.yalm_set_x(self.h, x.ctypes.data))

    def get_logits(self) -> np.ndarray:
        out = np.empty(self.cfg.vocab_size, np.float32)
        check(lib.yalm_get_logits(self.h, out.ctypes.data))
        return out

    def time_kernel(self, kernel_id: int, iters: int) -> float:
        ms = c_float()
        check(lib.yalm_time_kernel(self.h, kernel_id, iters, ctypes.byref(ms)))
        return ms.value

    def set_gemv_config(self, kind: int, threads: int = 0, unroll: int = 0, gpw: int = 0) -> None:
        check(lib.yalm_set_gemv_config(self.h, kind, threads, unroll, gpw))

    @property
    def attn_wo(self) -> bool:
        """True when the launch path runs attention + Wo as one launch (attn_wo.h)."""
        return bool(lib.yalm_decoder_attn_wo(self.h))

    def attn_wo_trace(self):
        """((workgroups, 16) uint64 stamps, attention workgroups) of the last fused
        attention + Wo launch (decoder created with YALM_ATTN_WO_TRACE=1)."""
        buf = np.zeros(16 * 8192, np.uint64)
        nb, na = c_int(), c_int()
        check(lib.yalm_attn_wo_trace(self.h, buf.ctypes.data, buf.size, ctypes.byref(nb), ctypes.byref(na)))
        return buf[: 16 * nb.value].reshape(nb.value, 16), na.value

    def graph_kernels(self, mode: int = 2) -> int:
        """Kernel launches per forward of graph `mode` (2 = the device greedy step)."""
        k, n = c_int(), c_int()
        check(lib.yalm_graph_kernels(self.h, mode, ctypes.byref(k), ctypes.byref(n)))
        return k.value

    def kernel_name(self, kernel_id: int) -> str:
        return lib.yalm_kernel_name(self.h, kernel_id).decode()

    def close(self):
        if self.h:
            check(lib.yalm_decoder_destroy(self.h))
            self.h = None
        if getattr(self, "stream", None) is not None:
            self.stream.close()
            self.stream = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

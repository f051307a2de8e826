"""CPU, world_size 2 over gloo: the tensor-parallel split (models.tp_shard /
shard_array, the same slicing the GPU path uploads or synthesises per rank)
restated in float64 numpy with torch.distributed all-reduce / all-gather must
reproduce the unsharded forward's logits. This pins the sharding math of
yalm_decoder_create_tp (include/yalm_hip.h) without GPUs; the GPU kernels'
TP path is covered at world size 1 by test_gpu_tp.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from yalm_amd import models as M
import ref_numpy as R

CFGS = {
    "tiny-untied": M.TINY,
    "tiny-tied": M.TINY.with_(tied=True),
}
TOKENS = [1, 17, 300, 5, 5, 99, 2, 250, 31, 8]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_cfg(c, size):
    return c.with_(n_heads=c.n_heads // size, n_kv_heads=c.n_kv_heads // size, hidden_dim=c.hidden_dim // size,
                   vocab_size=c.vocab_size // size)


def _worker(rank, size, port, name, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        cfg = CFGS[name]
        full = M.synth_host_tensors(cfg, seed=4)
        t = dict(full)
        if cfg.tied:
            t["tp.wcls"] = full["model.embed.weight"]
        shards = {k: np.ascontiguousarray(M.shard_array(cfg, k, v, rank, size)) for k, v in t.items()}

        def allreduce(v):
            tt = torch.from_numpy(np.ascontiguousarray(v))
            dist.all_reduce(tt)
            return tt.numpy()

        def allgather(v):
            parts = [torch.empty(len(v), dtype=torch.float64) for _ in range(size)]
            dist.all_gather(parts, torch.from_numpy(np.ascontiguousarray(v)))
            return torch.cat(parts).numpy()

        m = R.RefModel(_local_cfg(cfg, size), shards, allreduce, allgather)
        logits = [m.forward(tok, pos) for pos, tok in enumerate(TOKENS)]
        if rank == 0:
            ref = R.RefModel(cfg, full)
            want = [ref.forward(tok, pos) for pos, tok in enumerate(TOKENS)]
            err = max(float(np.max(np.abs(a - b)) / np.max(np.abs(b))) for a, b in zip(logits, want))
            q.put(err)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name", list(CFGS))
def test_tp2_sharded_forward_matches_unsharded(name):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    err = q.get(timeout=5)
    assert err < 1e-10, err


def test_tp_shard_covers_every_tensor_once():
    """Concatenating the shards of every rank gives back each full tensor."""
    cfg = M.MISTRAL_7B
    for size in (2, 4, 8):
        M.tp_check(cfg, size)
        for name, (shape, _) in M.tensor_shapes(cfg).items():
            sh = [M.tp_shard(cfg, name, r, size) for r in range(size)]
            if sh[0] is None:
                assert all(s is None for s in sh)
                continue
            kind = sh[0][0]
            axis = 0 if kind == "rows" else 1
            assert sum(s[2] for s in sh) == shape[axis]
            assert [s[1] for s in sh] == [r * sh[0][2] for r in range(size)]

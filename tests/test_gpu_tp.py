"""GPU: the tensor-parallel decoder path (yalm_decoder_create_tp: RCCL
communicator, Wo / W2 partials into xs + ncclAllReduce captured in the graph,
sharded-vocabulary logits all-gather and (value, index) argmax pick) at world
size 1 in one process, against the plain decoder on the same weights: the
arithmetic is identical (x + W v either way), so logits and greedy tokens must
match bit for bit. The split itself (world size 2) is pinned on the CPU by
test_tp_cpu.py; N > 1 on GPUs runs under bench.py --tp."""
import numpy as np
import pytest

from yalm_amd import models as M

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg", [M.SMALL, M.TINY.with_(tied=True), M.SMALL.with_(weight_dtype=M.F8E5M2)])
def test_tp1_matches_single_gpu_decoder(cfg):
    from yalm_amd import runtime as R

    dm = R.DeviceModel.synthetic(cfg, seed=9)
    ref = R.Decoder(dm)
    tp = R.Decoder(dm, tp_id=R.tp_unique_id())
    prompt = [3, 77, 12, 5, 200, 9]
    for pos, t in enumerate(prompt[:-1]):
        a = ref.forward(t, pos)
        b = tp.forward(t, pos)
        np.testing.assert_array_equal(a, b)
    ga = ref.generate_greedy(prompt[-1], len(prompt) - 1, 24)
    gb = tp.generate_greedy(prompt[-1], len(prompt) - 1, 24)
    assert ga == gb
    tp.close()
    ref.close()
    dm.close()


def test_tp_shard_synthesis_matches_full_model():
    """DeviceModel.synthetic(tp=(r, 2)) slices == the full tensors' slices."""
    from yalm_amd import runtime as R

    cfg = M.TINY
    full = M.synth_host_tensors(cfg, seed=2)
    for r in range(2):
        dm = R.DeviceModel.synthetic(cfg, seed=2, tp=(r, 2))
        for name in ("model.layers.1.attn.wq.weight", "model.layers.0.attn.wo.weight", "model.layers.1.mlp.w2.weight",
                     "model.output.weight", "model.norm.weight"):
            want = np.ascontiguousarray(M.shard_array(cfg, name, full[name], r, 2))
            got = np.empty_like(want)
            R.check(R.lib.yalm_download(got.ctypes.data, dm.ptrs[name], got.nbytes))
            np.testing.assert_array_equal(got, want)
        dm.close()


def test_tp1_ipc_matches_single_gpu_decoder():
    """The IPC exchange transport at world size 1: bit-exact vs the plain decoder."""
    from yalm_amd import runtime as R

    cfg = M.SMALL
    dm = R.DeviceModel.synthetic(cfg, seed=9)
    ref = R.Decoder(dm)
    tp = R.Decoder(dm, tp_gather=lambda h: [h])
    prompt = [3, 77, 12, 5, 200, 9]
    for pos, t in enumerate(prompt[:-1]):
        np.testing.assert_array_equal(ref.forward(t, pos), tp.forward(t, pos))
    assert ref.generate_greedy(prompt[-1], len(prompt) - 1, 24) == tp.generate_greedy(prompt[-1], len(prompt) - 1, 24)
    tp.close()
    ref.close()
    dm.close()


def _tp_cfg(size):
    return M.SMALL.with_(n_kv_heads=4) if size == 4 else M.SMALL


def _tp_ipc_worker(rank, size, port, q):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from yalm_amd import runtime as R

        cfg = _tp_cfg(size)
        dm = R.DeviceModel.synthetic(cfg, seed=9, tp=(rank, size))

        def gather(h):
            out = [None] * size
            dist.all_gather_object(out, h)
            return out

        dec = R.Decoder(dm, tp_gather=gather)
        prompt = [3, 77, 12, 5, 200, 9]
        logits = [dec.forward(t, pos) for pos, t in enumerate(prompt[:-1])]
        toks = dec.generate_greedy(prompt[-1], len(prompt) - 1, 24)
        # a second sequence through the same decoder: the exchange sequence numbers keep counting
        toks2 = dec.generate_greedy(11, 0, 8)
        q.put((rank, [l.copy() for l in logits], toks, toks2))
        dec.close()
        dm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size", [2, 4])
def test_tp_ipc_multi_rank_on_one_gpu(size):
    """TP over `size` processes sharing this GPU through the IPC exchange: every
    rank sees the same logits and greedy tokens, equal to the single-GPU
    decoder's within fp32 reassociation (x + sum of rank partials vs one
    GEMV over the full row)."""
    import socket

    import torch.multiprocessing as mp

    from yalm_amd import runtime as R

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_ipc_worker, args=(r, size, port, q)) for r in range(size)]
    for p in procs:
        p.start()
    import queue
    import time

    res, t0 = [], time.time()
    while len(res) < size:  # fail fast when a rank dies instead of waiting out the queue
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
            assert time.time() - t0 < 300, "timeout"
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    for r in res[1:]:
        for a, b in zip(res[0][1], r[1]):
            np.testing.assert_array_equal(a, b)
        assert r[2] == res[0][2] and r[3] == res[0][3]

    cfg = _tp_cfg(size)
    dm = R.DeviceModel.synthetic(cfg, seed=9)
    ref = R.Decoder(dm)
    prompt = [3, 77, 12, 5, 200, 9]
    for (pos, t), got in zip(enumerate(prompt[:-1]), res[0][1]):
        want = ref.forward(t, pos)
        assert np.max(np.abs(got - want)) / np.max(np.abs(want)) < 1e-4
    assert res[0][2] == ref.generate_greedy(prompt[-1], len(prompt) - 1, 24)
    assert res[0][3] == ref.generate_greedy(11, 0, 8)
    ref.close()
    dm.close()

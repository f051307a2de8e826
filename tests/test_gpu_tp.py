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


# head_dim 128: the fused attention + Wo launch runs on every rank (round 5); per rank at
# TP2 / TP4 the Wo rows are 2 KiB / 1 KiB (attn_wo.h KB 2 / 1), the TP1 rows 4 KiB
FUSED = M.ModelConfig(dim=1024, hidden_dim=2048, head_dim=128, n_layers=3, n_heads=16, n_kv_heads=4,
                      vocab_size=1536, max_seq_len=1040, rope_theta=10000.0, act=M.SILU, weight_dtype=M.F16)


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
@pytest.mark.parametrize("dtype", [M.F16, M.F8E5M2], ids=["f16", "fp8"])
def test_tp1_fused_attn_wo_matches_single_gpu(transport, dtype):
    """TP1 through either transport runs the fused attention + Wo launch (its Wo partial into
    xs for RCCL, pushed to the exchange for IPC) and the exchange-consuming GEMVs: bit-exact
    vs the plain decoder (x + Wo v either way; a one-rank sum is the value itself)."""
    from yalm_amd import runtime as R

    cfg = FUSED.with_(weight_dtype=dtype, max_seq_len=200)
    dm = R.DeviceModel.synthetic(cfg, seed=9)
    ref = R.Decoder(dm)
    tp = R.Decoder(dm, tp_id=R.tp_unique_id()) if transport == "rccl" else R.Decoder(dm, tp_gather=lambda h: [h])
    try:
        assert ref.attn_wo and tp.attn_wo
        prompt = [3, 77, 12, 5, 200, 9]
        for pos, t in enumerate(prompt[:-1]):
            np.testing.assert_array_equal(ref.forward(t, pos), tp.forward(t, pos))
        assert ref.generate_greedy(prompt[-1], 5, 220) == tp.generate_greedy(prompt[-1], 5, 220)  # past the window
        if transport == "ipc":  # no exchange launches: the same kernel count as one GPU
            assert tp.graph_kernels(2) == ref.graph_kernels(2)
    finally:
        tp.close()
        ref.close()
        dm.close()


HYDR = 1030


def _tok(pos):
    return (pos * 7 + 3) % FUSED.vocab_size


def _tp_fused_worker(rank, size, port, q, cu_mask=False):
    import os

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        from yalm_amd import runtime as R

        dm = R.DeviceModel.synthetic(FUSED, seed=13, tp=(rank, size))

        def gather(h):
            out = [None] * size
            dist.all_gather_object(out, h)
            return out

        dec = R.Decoder(dm, tp_gather=gather, cu_part=(rank, size) if cu_mask else None)
        kernels = dec.graph_kernels(2)
        fused = dec.attn_wo
        for pos in range(HYDR):  # HYDRATE graph: the last layer's W2 exchange has no consumer
            dec.forward(_tok(pos), pos, R.HYDRATE_KV_CACHE)
        logits = [dec.forward(_tok(pos), pos) for pos in range(HYDR, HYDR + 16)]  # 17 key chunks, ring + sinks
        toks = dec.generate_greedy(5, HYDR + 16, 16)
        # Block::block under tensor parallelism: x in, one layer, the exchanged sum collected
        x0 = np.linspace(-1.0, 1.0, FUSED.dim).astype(np.float32)
        dec.set_x(x0)
        dec.block(1, 7, 0, 7, 8)
        xb = dec.get_x()
        q.put((rank, kernels, fused, [lg.copy() for lg in logits], toks, xb))
        dec.close()
        dm.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cu_mask", [False, True], ids=["shared-cus", "cu-masked"])
@pytest.mark.parametrize("size", [2, 4])
def test_tp_ipc_fused_launch_lean_multi_rank(size, cu_mask):
    """IPC tensor parallelism over `size` processes on this GPU with the launch-lean path:
    the fused attention + Wo launch on every rank (Wo rows of 2 / 1 KiB), the Wo and W2
    partials pushed to the exchange and summed inside the next GEMV, the argmax exchange
    inside the argmax launch; every rank identical. shared-cus: the ranks share every CU of
    this GPU, so each consumer is preceded by a 1-wave gate launch (no exchange kernel sums
    anything); cu-masked: each rank decodes on its own CU block (yalm_stream_create_cu_part),
    the gate-free production sequence with the consumers' in-GEMV wait on a real peer
    (ADVICE r5). After 1030 hydrated positions, logits at
    kv 1031 .. 1040 (17 key chunks) and past max_seq_len (ring + sinks) within 1e-4 of the
    single-GPU decoder's, 16 greedy tokens identical to it; yalm_block's x under TP within
    1e-5 of the single decoder's."""
    import queue
    import socket
    import time

    import torch.multiprocessing as mp

    from yalm_amd import runtime as R

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_tp_fused_worker, args=(r, size, port, q, cu_mask)) for r in range(size)]
    for p in procs:
        p.start()
    res, t0 = [], time.time()
    while len(res) < size:
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
        for a, b in zip(res[0][3], r[3]):
            np.testing.assert_array_equal(a, b)
        assert r[4] == res[0][4]
        np.testing.assert_array_equal(r[5], res[0][5])
    dm = R.DeviceModel.synthetic(FUSED, seed=13)
    ref = R.Decoder(dm)
    try:
        assert all(r[2] for r in res), "the fused attention + Wo launch must run on every rank"
        # ranks sharing this GPU's CUs get a 1-wave gate launch before each of the 2 L consumers
        # (yalm_hip.hip tpx_consume); one GPU per rank, or disjoint CU masks, has none
        gates = 0 if cu_mask else 2 * FUSED.n_layers
        assert all(r[1] == ref.graph_kernels(2) + gates for r in res), ([r[1] for r in res], ref.graph_kernels(2))
        for pos in range(HYDR):
            ref.forward(_tok(pos), pos, R.HYDRATE_KV_CACHE)
        for pos, got in zip(range(HYDR, HYDR + 16), res[0][3]):
            want = ref.forward(_tok(pos), pos)
            assert np.max(np.abs(got - want)) / np.max(np.abs(want)) < 1e-4, pos
        assert res[0][4] == ref.generate_greedy(5, HYDR + 16, 16)
        x0 = np.linspace(-1.0, 1.0, FUSED.dim).astype(np.float32)
        ref.set_x(x0)
        ref.block(1, 7, 0, 7, 8)
        xr = ref.get_x()
        assert np.max(np.abs(res[0][5] - xr)) / np.max(np.abs(xr)) < 1e-5
    finally:
        ref.close()
        dm.close()


def _missing_peer_worker(rank, port, q):
    import os
    import time

    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=2)
    try:
        from yalm_amd import runtime as R

        dm = R.DeviceModel.synthetic(FUSED, seed=13, tp=(rank, 2))

        def gather(h):
            out = [None] * 2
            dist.all_gather_object(out, h)
            return out

        dec = R.Decoder(dm, tp_gather=gather)
        if rank == 0:  # rank 1 never runs a forward: every exchange of rank 0 waits for it
            t0 = time.time()
            err = ""
            try:
                dec.forward(5, 0)
            except R.YalmError as e:
                err = str(e)
            q.put((time.time() - t0, err))
        dist.barrier()  # rank 1 keeps its exchange buffer mapped until rank 0 is done
        dec.close()
        dm.close()
    finally:
        dist.destroy_process_group()


def test_tp_ipc_missing_peer_fails_fast():
    """A rank whose peer never runs the forward: the first exchange wait gives up at its 2 s
    deadline, every later wait of the same forward (2 L + 1 exchanges) gives up at once
    (tp_exchange.h tpx_give_up), and the call reports it -- a broken transport costs one
    timeout, not 2 s per exchange (bench.py then still reports the other transport)."""
    import queue
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_missing_peer_worker, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        dt, err = q.get(timeout=240)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert "IPC exchange gave up" in err, err
    assert 1.5 < dt < 2 * 2.0 + 2.0, dt  # one 2-s deadline (plus setup), not one per exchange

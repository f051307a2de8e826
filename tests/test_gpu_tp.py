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

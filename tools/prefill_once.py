"""One Llama-3.2-3B 4096-position prefill pass (yalm_prefill_time, 2 iterations after a
warm-up) in the given form, for rocprofv3 kernel stats. usage: prefill_once.py fast|split"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime as R  # noqa: E402

form = sys.argv[1] if len(sys.argv) > 1 else "fast"
cfg = M.LLAMA_32_3B.with_(max_seq_len=4096)
dm = R.DeviceModel.synthetic(cfg, seed=5)
dec = R.Decoder(dm)
if form == "split":
    dec.set_prefill_precision(R.PREFILL_SPLIT)
print(f"{form}: {dec.prefill_time(4096, 2):.3f} ms per pass")
dec.close()
dm.close()

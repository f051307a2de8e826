"""Attention-kernel latency vs kv_len on the Mistral-7B attention shape
(32 q / 8 kv heads x 128), timed back-to-back with HIP events
(yalm_time_kernel id 1), plus the per-token cost of a trivial GEMV of the
same launch class for reference."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402

cfg = M.MISTRAL_7B.with_(n_layers=2, vocab_size=512, hidden_dim=1024)
dm = runtime.DeviceModel.synthetic(cfg)
dec = runtime.Decoder(dm)
pos = 0
for target in [1, 32, 64, 65, 128, 256, 512, 1024, 2048, 4096]:
    while pos < target:
        dec.forward(1, pos, runtime.HYDRATE_KV_CACHE if pos + 1 < target else runtime.OUTPUT_LOGITS)
        pos += 1
    t = dec.time_kernel(1, 200)
    print(f"kv_len={target:5d}  attention {t * 1e3:7.2f} us/launch", flush=True)
dec.close()
dm.close()

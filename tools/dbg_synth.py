import sys, numpy as np
sys.path.insert(0, '.')
from yalm_amd import runtime, models as M
for dt, scale, off in ((M.F32, 0.2, 1.0), (M.F16, 0.035, 0.0), (M.F8E5M2, 0.035, 0.0)):
    n = 100003
    nb = n * M.DTYPE_BYTES[dt]
    p = runtime.lib.yalm_alloc(nb)
    seed = M.synth_seed(9, f"t{dt}")
    runtime.check(runtime.lib.yalm_synth(p, n, dt, seed, scale, off, None))
    runtime.check(runtime.lib.yalm_stream_sync(None))
    host = np.empty(nb, np.uint8)
    runtime.check(runtime.lib.yalm_download(host.ctypes.data, p, nb))
    ref = M.synth_array(n, dt, seed, scale, off)
    st = {M.F32: np.float32, M.F16: np.float16, M.F8E5M2: np.uint8}[dt]
    h = host.view(st); r = ref.view(st)
    bad = np.nonzero(h.view(np.uint8 if dt == M.F8E5M2 else (np.uint16 if dt == M.F16 else np.uint32)) != r.view(np.uint8 if dt == M.F8E5M2 else (np.uint16 if dt == M.F16 else np.uint32)))[0]
    print(dt, len(bad), bad[:10], h[bad[:10]], r[bad[:10]])
    if dt == M.F8E5M2 and len(bad):
        f16 = M.synth_array(n, M.F16, seed, scale, 0.0)
        print(" f16 bits", f16[bad[:10]].view(np.uint16), [hex(x) for x in f16[bad[:10]].view(np.uint16)])

"""Timeline of the fused attention + Wo launch (attn_wo.h) on a Mistral-7B-shaped
synthetic model: the last layer's launch of the last token, from the
per-workgroup s_memrealtime stamps (100 MHz) of yalm_attn_wo_trace.

usage: python tools/attn_wo_trace.py [--model mistral-7b] [--ctx 150] [--dtype fp16|fp8]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["YALM_ATTN_WO_TRACE"] = "1"

from yalm_amd import models as M  # noqa: E402
from yalm_amd import runtime  # noqa: E402


def q(v):
    return f"min {v.min():6.2f} med {np.median(v):6.2f} max {v.max():6.2f}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--ctx", type=int, default=150)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp8"])
    ap.add_argument("--time", type=int, default=0, help="also time the fused launch (yalm_time_kernel 8), iterations")
    args = ap.parse_args()
    runtime.check(runtime.lib.yalm_set_device(0))
    cfg = M.PRESETS[args.model].with_(weight_dtype=M.F16 if args.dtype == "fp16" else M.F8E5M2)
    dm = runtime.DeviceModel.synthetic(cfg, seed=1)
    dec = runtime.Decoder(dm)
    assert dec.attn_wo, "decoder does not run the fused attention + Wo launch"
    toks = [(7 * pos + 1) % cfg.vocab_size for pos in range(args.ctx)]
    if args.ctx > 64 and args.dtype == "fp16":  # long contexts: hydrate by the batched prefill
        dec.prefill(toks, 0, logprobs=False)
    else:
        for pos, t in enumerate(toks):
            dec.forward(t, pos, runtime.HYDRATE_KV_CACHE)
    dec.forward(5, args.ctx)
    tr, na = dec.attn_wo_trace()
    if args.time:
        print(f"yalm_time_kernel(8) at kv_len {args.ctx + 1}: {dec.time_kernel(8, args.time) * 1e3:.2f} us")
    tr = tr.astype(np.int64)
    clk = tr[:, 8:]
    tr = tr[:, :8]
    t0 = tr[:, 0].min()
    us = (tr - t0) / 100.0
    att, wo = us[:na], us[na:]
    writers = att[tr[:na, 1] > 0]
    print(f"[{args.model} kv_len {args.ctx + 1}] grid {len(tr)} = {na} attention + {len(tr) - na} Wo workgroups; "
          f"launch span {us[:, 3].max():.2f} us")
    print(f"attention start  {q(att[:, 0])}")
    print(f"attention end    {q(att[:, 3])}")
    # attention units stamp [2] (first loads landed); mergers leave it 0 and stamp [5] / [7]
    # (gather issued / every partial seen); a phase a workgroup never reached reads 0
    act_m = tr[:na, 2] > 0
    mer_m = (tr[:na, 2] == 0) & (tr[:na, 7] > 0)
    active = att[act_m]
    print(f"active attention units: {len(active)}")
    print(f"  loads landed   {q(active[:, 2])}")
    print(f"  last scores    {q(active[:, 4])}")
    print(f"  last softmax   {q(active[:, 5])}")
    print(f"  P.V combined   {q(active[:, 6])}")
    print(f"  outputs issued {q(active[:, 7])}")
    a_tr, a_clk = tr[:na][act_m], clk[:na][act_m]

    def phase(rows, rclk, k0, k1, name):
        dt = (rows[:, k1] - rows[:, k0]) / 100.0
        dc = rclk[:, k1] - rclk[:, k0]
        print(f"  {name:18s} med {np.median(dt):6.2f} max {dt.max():6.2f} us  {np.median(dc):8.0f} shader clocks"
              f"  ({np.median(dc) / np.maximum(np.median(dt), 1e-3) / 1e3:5.2f} GHz)")

    for k0, k1, name in ((2, 4, "loads->last scores"), (4, 5, "scores->softmax"),
                         (5, 6, "softmax->P.V"), (6, 7, "P.V->issued")):
        phase(a_tr, a_clk, k0, k1, name)
    if mer_m.any():
        m_tr, m_clk = tr[:na][mer_m], clk[:na][mer_m]
        mergers = att[mer_m]
        print(f"mergers: {len(mergers)}")
        print(f"  gather issued  {q(mergers[:, 5])}")
        print(f"  all partials   {q(mergers[:, 7])}")
        print(f"  head signalled {q(mergers[:, 1])}")
        # the hop: the last partial of this merger's head issued -> seen -> head out
        phase(m_tr, m_clk, 5, 7, "spin (issued->seen)")
        phase(m_tr, m_clk, 7, 1, "fold->signalled")
        last_part = active[:, 7].max()
        print(f"  last partial issued {last_part:6.2f} us; last partial seen {mergers[:, 7].max():6.2f} us; "
              f"last head {mergers[:, 1].max():6.2f} us")
    print(f"head signalled   {q(writers[:, 1])}  ({len(writers)} writers)")
    # where each workgroup ran (slot 8: HW_ID | XCC_ID << 32): CU = (XCC, SE, SH, CU id)
    hw = clk[:, 0].astype(np.uint64)
    hwid, xcc = (hw & 0xFFFFFFFF).astype(np.int64), (hw >> np.uint64(32)).astype(np.int64) & 0xF
    cu_key = xcc * 4096 + ((hwid >> 13) & 0x7) * 256 + ((hwid >> 12) & 1) * 16 + ((hwid >> 8) & 0xF)
    wo_keys = cu_key[na:]
    wo_per_cu = {}
    for k_ in wo_keys:
        wo_per_cu[k_] = wo_per_cu.get(k_, 0) + 1
    heads_cu = cu_key[:na][tr[:na, 1] > 0]
    share = [wo_per_cu.get(k_, 0) for k_ in heads_cu]
    print(f"placement: {len(set(cu_key.tolist()))} distinct CUs; Wo workgroups on {len(wo_per_cu)} CUs "
          f"(per CU: {sorted(set(wo_per_cu.values()))}); head writers' CUs host "
          f"{np.bincount(share).tolist() if share else []} Wo workgroups (count of writers with 0, 1, 2, ..)")
    # which Wo workgroup shares each head writer's CU (workgroup index b of the writer, j of the Wo)
    wo_of_cu = {k_: j for j, k_ in enumerate(wo_keys.tolist())}
    pairs = [(int(b), wo_of_cu.get(int(cu_key[b]), -1)) for b in np.nonzero(tr[:na, 1] > 0)[0]]
    print(f"  head writer b -> co-resident Wo j: {pairs[:12]}{' ...' if len(pairs) > 12 else ''}; "
          f"j == b for {sum(1 for b, j in pairs if j == b)} of {len(pairs)}")
    wo_ex = wo[:, 3]
    on_head_cu = np.array([k_ in set(heads_cu.tolist()) for k_ in wo_keys])
    if on_head_cu.any():
        print(f"  Wo end on head CUs {q(wo_ex[on_head_cu])}; elsewhere {q(wo_ex[~on_head_cu])}")
        print(f"  Wo poll passed on head CUs {q(wo[on_head_cu, 2])}; elsewhere {q(wo[~on_head_cu, 2])}")
    print(f"Wo start         {q(wo[:, 0])}")
    print(f"Wo slice landed  {q(wo[:, 1])}")
    print(f"Wo poll passed   {q(wo[:, 2])}")
    print(f"Wo end           {q(wo[:, 3])}")
    w_tr, w_clk = tr[na:], clk[na:]
    dt = (w_tr[:, 3] - w_tr[:, 2]) / 100.0
    dc = w_clk[:, 3] - w_clk[:, 2]
    print(f"  Wo poll->end     {np.median(dt):6.2f} us  {np.median(dc):8.0f} shader clocks")
    dec.close()
    dm.close()


if __name__ == "__main__":
    main()

"""CPU: the address range of the short-prompt (T <= 64) skinny GEMMs, bounded on the host
(the r4y illegal-address question of the LDS-DMA skinny form).

The index arithmetic of yalm_amd/csrc/prefill_skinny.h is restated here for every GEMM
the prefill launches at T = 1..64 (prefill.hip enqueue_prefill, the `small` path) at the
production shapes: sk_stage_a's A-row reads (rows clamped to T - 1, columns inside the
K chunk) and skinny_gemm_lds_kernel's weight-row DMA sources (rows of the workgroup's
64-row block, columns inside the chunk, the clamped tail stages), against the sizes of
the buffers they read (PrefillBufs, the weight tensors). The K split sk_pick_ks is
restated too, with its invariants (KC a multiple of the 128-column DMA stage, the A chunk
within 32 KB of LDS, no chunk straddling the B wrap of the k | v GEMM).
"""
import pytest

from yalm_amd import models as M

SK_ROWS, SK_U = 64, 8
SK_KSTEP = 32 * SK_U
SKL_KS = 128
SK_AMAX = 8
SK_MAX_T = 64


def sk_pick_ks(kn, TP):
    """prefill.hip sk_pick_ks: kn = [(N, K, mult)]."""
    best, kmin, wg1 = -1, 1 << 30, 0
    for N, K, mult in kn:
        kmin = min(kmin, K // mult)
        wg1 += N // SK_ROWS * mult
    for ks in range(1, kmin // SK_KSTEP + 1):
        ok = True
        for N, K, mult in kn:
            s = ks * mult
            ok = ok and K % s == 0 and (K // s) % SK_KSTEP == 0 and TP * (K // s) * 2 <= 32768
        if not ok:
            continue
        best = ks
        if wg1 * ks >= 512:
            break
    return best


def a_max_elem(T, lda, K, KS):
    """Largest f16 element index (exclusive end of a 16-byte read) sk_stage_a touches in A."""
    MT = (T + 15) // 16
    TP = 16 * MT
    KC = K // KS
    cpr, nch = KC // 8, TP * KC // 8
    assert nch <= 256 * SK_AMAX, "the A chunk must fit one round of loads"
    hi = 0
    for ks in range(KS):
        k0 = ks * KC
        i = nch - 1  # the largest chunk index (later u clamp to it)
        for i in range(max(0, nch - 2 * cpr), nch):  # the last rows' chunks: the largest addresses
            r, c = divmod(i, cpr)
            hi = max(hi, min(r, T - 1) * lda + k0 + 8 * c + 8)
    return hi


def b_max(N_rows_block_end, kb, K, KS):
    """(largest B row + 1, largest B column + 1) the DMA sources reach: rows of the last
    64-row block, columns of the clamped last 128-column stage of the last chunk."""
    KC = K // KS
    assert KC % SKL_KS == 0
    nst = KC // SKL_KS
    col_hi = 0
    for ks in range(KS):
        k0 = ks * KC
        assert not (k0 < kb < k0 + KC), "a K chunk straddles the B wrap"
        kw0 = k0 if k0 < kb else k0 - kb
        col_hi = max(col_hi, kw0 + (nst - 1) * SKL_KS + 8 * 15 + 8)
    return N_rows_block_end, col_hi


CFGS = {"mistral-7b": M.MISTRAL_7B, "llama-3.2-3b": M.LLAMA_32_3B,
        "gqa-d128": M.ModelConfig(dim=512, hidden_dim=1024, head_dim=128, n_layers=3, n_heads=4, n_kv_heads=2,
                                  vocab_size=1024, max_seq_len=320, rope_theta=1e6),
        "d768": M.ModelConfig(dim=768, hidden_dim=1536, head_dim=128, n_layers=2, n_heads=6, n_kv_heads=2,
                              vocab_size=1920, max_seq_len=320, rope_theta=1e6)}


@pytest.mark.parametrize("name", list(CFGS))
def test_skinny_gemm_reads_stay_inside_their_buffers(name):
    c = CFGS[name]
    cap = c.max_seq_len
    q_dim, kv_dim = c.q_dim, c.kv_dim
    # PrefillBufs allocations in f16 elements (prefill.hip ensure_bufs)
    xn_elems = cap * c.dim * 2
    o_elems = cap * q_dim * 2
    h_elems = cap * c.hidden_dim * 2
    for T in range(1, SK_MAX_T + 1):
        TP = 16 * ((T + 15) // 16)
        ks_qkv = sk_pick_ks([(q_dim, c.dim, 1), (2 * kv_dim, 2 * c.dim, 2)], TP)
        ks_wo = sk_pick_ks([(c.dim, q_dim, 1)], TP)
        ks_glu = sk_pick_ks([(2 * c.hidden_dim, c.dim, 1)], TP)
        ks_w2 = sk_pick_ks([(c.dim, c.hidden_dim, 1)], TP)
        assert min(ks_qkv, ks_wo, ks_glu, ks_w2) > 0, (T, ks_qkv, ks_wo, ks_glu, ks_w2)
        # (A buffer, lda, K, kb, KS, B rows, B row width = kb)
        gemms = [
            ("q", xn_elems, 2 * c.dim, c.dim, c.dim, ks_qkv, q_dim),
            ("k|v", xn_elems, 2 * c.dim, 2 * c.dim, c.dim, 2 * ks_qkv, 2 * kv_dim),
            ("wo", o_elems, q_dim, q_dim, q_dim, ks_wo, c.dim),
            ("glu", xn_elems, c.dim, c.dim, c.dim, ks_glu, 2 * c.hidden_dim),
            ("w2", h_elems, c.hidden_dim, c.hidden_dim, c.hidden_dim, ks_w2, c.dim),
        ]
        for g, a_elems, lda, K, kb, KS, nrows in gemms:
            hi = a_max_elem(T, lda, K, KS)
            assert hi <= a_elems, (name, T, g, hi, a_elems)
            assert hi <= T * lda, (name, T, g, "A read past row T - 1")
            assert (T * lda if T > 0 else 0) <= a_elems
            assert nrows % SK_ROWS == 0, (name, g, nrows)
            rows_end, col_hi = b_max(nrows, kb, K, KS)
            assert col_hi <= kb, (name, T, g, col_hi, kb)
            assert (K // KS) * TP * 2 <= 32768, (name, T, g)

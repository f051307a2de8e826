"""GPU: exact-index parity of the device greedy sampler (argmax_kernel and the
tensor-parallel argmax_pick_kernel, misc_kernels.h) with the oracle's
sample_argmax (reference sampler.cpp:27-38: strict '>' scan from -FLT_MAX, so
the FIRST maximum wins, NaNs never win, and a row where nothing exceeds
-FLT_MAX returns 0). Index work: the bar is bit-exact.

The kernel runs 1024 threads; thread t, batch k (8 float4 loads in flight)
covers elements base + (k * 1024 + t) * 4 .. + 3, base stepping by 32768; the
n % 4 tail is a separate loop. The planted ties below sit inside one float4,
across waves (where the wave order and the index order disagree), across
batches of one thread, across base iterations, in the tail, and across
tensor-parallel shards."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu

FMAX = np.float32(3.4028234663852886e38)


def rt():
    from yalm_amd import runtime

    return runtime


def oracle_argmax(lg):
    lg = np.ascontiguousarray(lg, np.float32)
    return int(O.olib.orc_sample_argmax(O.P(lg), lg.size))


def planted(n, idxs, val=5.0, seed=0, base=None):
    rng = np.random.default_rng(seed)
    lg = rng.standard_normal(n).astype(np.float32) if base is None else np.full(n, base, np.float32)
    for i in idxs:
        lg[i] = val
    return lg


def thread_k(t, k, base=0):
    return base + (k * 1024 + t) * 4


CASES = {
    "same-float4": planted(32000, [17, 19]),
    "float4-lanes-0-3": planted(32000, [4 * 77 + 3, 4 * 77]),
    "across-waves-index-order": planted(32000, [thread_k(900, 0), thread_k(2, 1)]),
    "across-waves-3": planted(32000, [thread_k(1023, 0), thread_k(64, 1), thread_k(0, 2)]),
    "across-batches": planted(32000, [thread_k(5, 0) + 1, thread_k(5, 7) + 1]),
    "across-base-iters": planted(128256, [40000, 100]),
    "across-base-iters-2": planted(128256, [127999, 40000, 98304]),
    "tail-ties-earlier": planted(32003, [31999, 32001]),
    "tail-only-max": planted(32003, [32002]),
    "tail-tie-in-tail": planted(32003, [32001, 32002]),
    "last-element": planted(32000, [31999]),
    "first-element": planted(32000, [0, 31999]),
    "all-nan": np.full(4099, np.nan, np.float32),
    "all-neg-inf": np.full(32000, -np.inf, np.float32),
    "all-neg-fltmax": np.full(32000, -FMAX, np.float32),
    "neg-fltmax-and-inf": planted(32000, [7], val=-FMAX, base=-np.inf),
    "nan-then-values": planted(32000, [0, 1, 2], val=np.nan),
    "pos-inf-ties": planted(32000, [500, 900], val=np.inf),
    "nan-around-max": planted(32000, [10, 12], val=np.nan),
    "small-n": planted(5, [3, 4]),
    "n-1": np.array([-1.0], np.float32),
}


@pytest.mark.parametrize("name", sorted(CASES))
def test_argmax_planted_ties(name):
    lg = CASES[name]
    assert rt().argmax(lg) == oracle_argmax(lg)


@pytest.mark.parametrize("seed", range(8))
@pytest.mark.parametrize("n", [32000, 32003, 128256])
def test_argmax_quantised_many_ties(seed, n):
    """Logits on a coarse grid: the maximum appears many times at random places."""
    rng = np.random.default_rng(seed)
    lg = np.round(rng.standard_normal(n) * 1.5).astype(np.float32)
    assert rt().argmax(lg) == oracle_argmax(lg)


@pytest.mark.parametrize("shards", [2, 4, 8])
@pytest.mark.parametrize("case", ["cross-shard", "in-shard", "all-neg-inf", "neg-inf-shard", "nan-shard", "random"])
def test_argmax_tensor_parallel_pick(shards, case):
    """Per-shard pairs + pick (the TP greedy path) == the unsharded first max."""
    n = 32000
    ns = n // shards
    if case == "cross-shard":
        lg = planted(n, [3 * ns // 4 + ns * (shards - 1), ns + 5])  # tie: a later shard and shard 1
    elif case == "in-shard":
        lg = planted(n, [ns - 1, ns - 2, 2 * ns - 1 if shards > 1 else 0])
    elif case == "all-neg-inf":
        lg = np.full(n, -np.inf, np.float32)
    elif case == "neg-inf-shard":  # shard 0 has nothing above -FLT_MAX; a later shard holds -5
        lg = np.full(n, -np.inf, np.float32)
        lg[ns * (shards - 1) + 3] = -5.0
    elif case == "nan-shard":
        lg = planted(n, [], seed=3)
        lg[:ns] = np.nan
    else:
        rng = np.random.default_rng(shards)
        lg = np.round(rng.standard_normal(n) * 1.5).astype(np.float32)
    assert rt().argmax(lg, shards) == oracle_argmax(lg)


def test_oracle_argmax_semantics():
    """The oracle itself on the same cases, restated in Python (sampler.cpp:27-38)."""
    def ref(lg):
        best, m = 0, -FMAX
        for i, v in enumerate(lg.tolist()):
            if v > m:
                best, m = i, v
        return best

    for name in ("same-float4", "tail-ties-earlier", "all-nan", "all-neg-fltmax", "pos-inf-ties", "small-n"):
        assert oracle_argmax(CASES[name]) == ref(CASES[name]), name

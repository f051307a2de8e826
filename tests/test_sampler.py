"""CPU: the host samplers (yalm_amd/host/sampler.cpp, the -t / perplexity
consumers of the logits) against the oracle's restatement of the reference
sampler (sampler.cpp:6-65). Temperature sampling draws std::rand() after
srand(seed) (main.cpp:50 seeds with the wall clock; a fixed seed makes it
reproducible), so with the same seed and the same logits the draw sequence
must be identical. sample_prob: within 1e-6 relative (the reference build's
-ffast-math may vectorise its float sum; ours sums in order). The empirical
distribution of the draws must follow softmax(logits / T)."""
import os
import subprocess

import numpy as np
import pytest

import oracle_py as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST = os.path.join(ROOT, "yalm_amd", "host")

O.olib.orc_srand.argtypes = [O.ci]
O.olib.orc_srand.restype = None
O.olib.orc_sample.argtypes = [O.vp, O.ci, O.cf]
O.olib.orc_sample.restype = O.ci


@pytest.fixture(scope="module")
def sample_dump():
    subprocess.run(["make", "-C", HOST, "-j4", "sample_dump"], check=True, capture_output=True)
    return os.path.join(HOST, "sample_dump")


def host_run(binary, logits, seed, temp, count, idx, tmp_path):
    f = tmp_path / "logits.f32"
    np.ascontiguousarray(logits, np.float32).tofile(f)
    out = subprocess.run([binary, str(f), str(seed), repr(float(temp)), str(count)] + [str(i) for i in idx],
                         capture_output=True, check=True, text=True).stdout.split("\n")
    return int(out[0]), [int(t) for t in out[1].split()], [float.fromhex(x) for x in out[2:2 + len(idx)]]


def oracle_run(logits, seed, temp, count, idx):
    lg = np.ascontiguousarray(logits, np.float32)
    O.olib.orc_srand(seed)
    draws = [int(O.olib.orc_sample(O.P(lg), lg.size, temp)) for _ in range(count)]
    probs = [float(O.olib.orc_sample_prob(O.P(lg), lg.size, i)) for i in idx]
    return int(O.olib.orc_sample_argmax(O.P(lg), lg.size)), draws, probs


@pytest.mark.parametrize("seed", [0, 1, 42])
@pytest.mark.parametrize("temp", [0.0, 0.7, 1.0, 1.5])
def test_temperature_sampling_matches_oracle(sample_dump, tmp_path, seed, temp):
    rng = np.random.default_rng(seed + 100)
    logits = (rng.standard_normal(32000) * 3).astype(np.float32)
    idx = [0, int(np.argmax(logits)), 31999, 12345]
    a_h, d_h, p_h = host_run(sample_dump, logits, seed, temp, 300, idx, tmp_path)
    a_o, d_o, p_o = oracle_run(logits, seed, temp, 300, idx)
    assert a_h == a_o
    assert d_h == d_o
    np.testing.assert_allclose(p_h, p_o, rtol=1e-6)


def test_sampling_distribution(sample_dump, tmp_path):
    """20000 draws at T = 0.8 over 8 logits: every frequency within 5 sigma of
    softmax(logits / T) (both implementations)."""
    logits = np.array([1.0, 0.5, -0.3, 2.0, 0.0, -1.5, 1.2, 0.9], np.float32)
    p = np.exp(logits / 0.8 - np.max(logits / 0.8))
    p /= p.sum()
    n = 20000
    _, d_h, _ = host_run(sample_dump, logits, 7, 0.8, n, [], tmp_path)
    _, d_o, _ = oracle_run(logits, 7, 0.8, n, [])
    for d in (d_h, d_o):
        freq = np.bincount(d, minlength=8) / n
        assert np.all(np.abs(freq - p) <= 5 * np.sqrt(p * (1 - p) / n)), (freq, p)

"""The associative-memory oracle (oracle/nk_assoc_oracle.c, test infrastructure)
pinned before it checks the device: BLAKE3 against published digests (the
blake3 crate is a dependency of the reference that is not vendored under
/root/reference, so its algorithm is restated), and the Willshaw network
against an independent numpy restatement of src/associative.rs:29-61."""
import numpy as np
import pytest

from oracle import cbind


# BLAKE3 digests of the empty input, b"abc" and the official test-vector
# input of length 8 (bytes i % 251) — published values
@pytest.mark.parametrize("data,hexd", [
    (b"", "af1349b9f5f9a1a6a0404dea36dcc9499bcb25c9adc112b7cc9a93cae41f3262"),
    (b"abc", "6437b3ac38465133ffb63b75273a8db548c558465d79db03fd359c6cd5bd9d85"),
    (bytes(range(8)), "2351207d04fc16ade43ccab08600939c7c1fa70a5c0aaca76063d04c3228eaeb"),
])
def test_blake3_published_digests(data, hexd):
    assert cbind.blake3(data).hex() == hexd


def _np_recall(W, noisy, steps):
    s = (np.frombuffer(noisy, np.uint8) > 0).astype(np.int32)
    for _ in range(steps):
        t = ((W.astype(np.int32) @ s) > 0).astype(np.int32)
        if np.array_equal(t, s):
            break
        s = t
    return (s * 255).astype(np.uint8).tobytes()


@pytest.mark.parametrize("n,dens", [(8, 0.3), (50, 0.1), (200, 0.03)])
def test_willshaw_oracle_matches_numpy(n, dens):
    rng = np.random.default_rng(n)
    o = cbind.OracleWillshaw(n)
    W = np.zeros((n, n), np.uint8)
    for _ in range(12):
        p = ((rng.random(n) < dens) * 255).astype(np.uint8)
        o.store(p.tobytes())
        on = p > 0
        W[np.ix_(on, on)] = 1
    assert o.stored_count == 12
    for steps in (0, 1, 3, 10):
        q = ((rng.random(n) < dens) * rng.integers(1, 256, n)).astype(np.uint8).tobytes()
        assert o.recall(q, steps) == _np_recall(W, q, steps)
    with pytest.raises(ValueError):
        o.store(b"\x01" * (n + 1))


def test_kmer_pattern_rule():
    """pattern bits = digest byte i % 32 mod pattern_size, i < pattern_size / 100
    (src/associative.rs:84-96); pattern_size 2^k (k <= 10) else 1024 (:73)."""
    for k, n in ((3, 8), (10, 1024), (11, 1024), (31, 1024)):
        a = cbind.OracleAssoc(k)
        assert a.pattern_size == n
        for kmer in (0, 1, 0xDEADBEEF, 2**64 - 1):
            d = cbind.blake3(int(kmer).to_bytes(8, "little"))
            want = np.zeros(n, np.uint8)
            for i in range(n // 100):
                want[d[i % 32] % n] = 255
            assert a.kmer_pattern(kmer) == want.tobytes()

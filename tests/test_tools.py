"""Build-time generators (CPU): the committed bitsliced XOR programs are exactly what
tools/gen_xor_networks.py produces, and the parity rows they were derived from are
the oracle's encode matrix ([upstream klauspost matrix.go buildMatrix])."""
import importlib.util
import os

import numpy as np

from oracle import rs_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GEN = os.path.join(ROOT, "tools", "gen_xor_networks.py")
INC = os.path.join(ROOT, "replication_erasurecoding_object_store_amd", "csrc", "rs_xor_networks.inc")


def _gen():
    spec = importlib.util.spec_from_file_location("gen_xor_networks", GEN)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_xor_networks_regenerate_identically(tmp_path):
    mod = _gen()
    mod.OUT = str(tmp_path / "rs_xor_networks.inc")
    mod.main()
    with open(mod.OUT) as a, open(INC) as b:
        assert a.read() == b.read(), "rs_xor_networks.inc is stale: rerun tools/gen_xor_networks.py"


def test_xor_network_rows_are_the_oracle_encode_matrix():
    mod = _gen()
    for k, m in mod.SHAPES:
        rows = np.array(mod.parity_rows(k, m), dtype=np.uint8)
        assert np.array_equal(rows, np.asarray(rs_oracle.build_matrix(k, m), dtype=np.uint8)[k:]), (k, m)


def _planes(col: np.ndarray):
    """32 bytes -> 8 plane words, plane j bit b = bit j of byte b."""
    return [sum(((int(col[b]) >> j) & 1) << b for b in range(32)) for j in range(8)]


def test_xor_programs_compute_the_encode():
    """The generated XOR programs (per input, as emitted; and shared over groups of 4
    inputs, the rejected form) evaluated on random bitsliced columns give the
    oracle's parity bytes."""
    mod = _gen()
    rng = np.random.default_rng(5)
    for k, m in mod.SHAPES:
        data = rng.integers(0, 256, (k, 32), dtype=np.uint8)
        shards = [bytearray(data[c].tobytes()) for c in range(k)] + [bytearray(32) for _ in range(m)]
        rs_oracle.encode(k, m, shards)
        want = [_planes(np.frombuffer(bytes(shards[k + r]), np.uint8)) for r in range(m)]
        for group in (1, 4):
            y = mod.evaluate(k, m, [_planes(data[c]) for c in range(k)], group)
            got = [y[r * 8:(r + 1) * 8] for r in range(m)]
            assert got == want, (k, m)


def test_pair_programs_compute_the_encode():
    """The 1 KiB-task pair programs (encode_bs16_kernel): the shapes they are emitted
    for satisfy C[r ^ 1][c] = C[r][c ^ 1], and ya ^ swap(yb) over 16-byte columns (one
    input of each pair per half-word) gives the oracle's parity bytes of both rows of
    every packed row."""
    mod = _gen()
    rng = np.random.default_rng(6)
    for k, m in mod.PAIR_SHAPES:
        assert mod.pair_symmetric(k, m), (k, m)
        data = rng.integers(0, 256, (k, 16), dtype=np.uint8)
        shards = [bytearray(data[c].tobytes()) for c in range(k)] + [bytearray(16) for _ in range(m)]
        rs_oracle.encode(k, m, shards)
        planes = [[sum(((int(data[c][b]) >> j) & 1) << b for b in range(16)) for j in range(8)] for c in range(k)]
        y = mod.evaluate_pairs(k, m, planes)
        for r in range(m):
            want = _planes(np.concatenate([np.frombuffer(bytes(shards[k + r]), np.uint8), np.zeros(16, np.uint8)]))
            got = [(v >> (16 * (r & 1))) & 0xFFFF for v in y[(r // 2) * 8:(r // 2) * 8 + 8]]
            assert got == want, (k, m, r)
    assert not mod.pair_symmetric(6, 3) and not mod.pair_symmetric(4, 3)

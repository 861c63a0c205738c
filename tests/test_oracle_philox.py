"""The in-kernel noise's specification (oracle/philox.py): Philox4x32-10 vs
Random123's published known-answer vectors, and the Box-Muller transform's
moments."""
import numpy as np

from oracle import philox


def test_philox4x32_10_known_answers():
    # Random123 kat_vectors (philox4x32, 10 rounds): counter, key -> output
    kat = [
        ([0, 0, 0, 0], [0, 0], [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]),
        ([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2, [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]),
        ([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0],
         [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]),
    ]
    for ctr, key, want in kat:
        got = philox.philox4x32_10(np.array(ctr, np.uint32), np.array(key, np.uint32))
        assert [int(x) for x in got] == want


def test_normal_moments_and_independence():
    z = philox.noise_ncdhw(12345, [7, 7], 2, 8, 16, 16, 16)
    assert z.dtype == np.float32 and np.isfinite(z).all()
    flat = z.reshape(-1).astype(np.float64)
    assert abs(flat.mean()) < 0.01 and abs(flat.std() - 1.0) < 0.01
    # 4th moment of N(0, 1) = 3; tails present but bounded (u1 >= 2^-24 -> |z| <= 5.77)
    assert abs((flat ** 4).mean() - 3.0) < 0.1 and np.abs(flat).max() < 5.8
    # channels and batches are different streams
    c = np.corrcoef(z.reshape(16, -1))
    assert np.abs(c - np.eye(16)).max() < 0.05
    # another timestep or seed: another draw; the same: the same bits
    assert not np.array_equal(z, philox.noise_ncdhw(12345, [6, 6], 2, 8, 16, 16, 16))
    assert not np.array_equal(z, philox.noise_ncdhw(12346, [7, 7], 2, 8, 16, 16, 16))
    assert np.array_equal(z, philox.noise_ncdhw(12345, [7, 7], 2, 8, 16, 16, 16))

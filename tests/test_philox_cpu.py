"""The noise-stream restatement (oracle/philox_ref.py) against the published Philox4x32-10
known-answer vectors (Random123 kat_vectors) -- it is the checker of the Langevin kernel's
in-kernel noise (tests/test_gpu_parity.py) and of the sharded sampler (test_distributed_cpu)."""
import numpy as np

from oracle import philox_ref

KAT = [  # counter words, key words -> output words
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def test_philox_known_answers():
    for c, k, want in KAT:
        got = philox_ref.philox4x32_10_words(*[np.array([w], np.uint64) for w in c], *k)[0]
        assert tuple(int(v) for v in got) == want


def test_counter_form_and_normal_stream():
    w = philox_ref.philox4x32_10(np.array([0, 1 << 32], np.uint64), 0)
    assert tuple(int(v) for v in w[0]) == KAT[0][2]
    v = philox_ref.normal(1234, 0, 1 << 16)
    assert abs(v.mean()) < 0.02 and abs(v.std() - 1) < 0.02
    # a shard starting at counter k draws the tail of the stream starting at 0
    np.testing.assert_array_equal(philox_ref.normal(1234, 8, 64), v[32:96])

"""Multi-batch codec (src/vsr/multi_batch.zig) through the exported C functions."""
import ctypes

import numpy as np
import pytest

from tigerbeetle_amd import native


def encode(lib, counts, element_size):
    payload = sum(counts) * element_size
    trailer = lib.tb_multi_batch_trailer_total_size(element_size, len(counts))
    buf = ctypes.create_string_buffer(bytes(range(256)) * ((payload + trailer + 255) // 256 + 1))
    c = (ctypes.c_uint16 * len(counts))(*counts)
    size = lib.tb_multi_batch_encode_trailer(buf, payload, element_size, c, len(counts))
    assert size == payload + trailer
    return buf.raw[:size]


def decode(lib, body, element_size):
    counts = (ctypes.c_uint16 * 65534)()
    payload = ctypes.c_uint32(0)
    nb = lib.tb_multi_batch_decode(body, len(body), element_size, counts, 65534,
                                   ctypes.byref(payload))
    return nb, list(counts[:max(nb, 0)]), payload.value


@pytest.mark.parametrize("element_size", [16, 128])
def test_round_trip(element_size):
    lib = native.load()
    rng = np.random.default_rng(1)
    for _ in range(50):
        nb = int(rng.integers(1, 80))
        counts = [int(x) for x in rng.integers(0, 20, size=nb)]
        body = encode(lib, counts, element_size)
        assert len(body) % element_size == 0
        got_nb, got, payload = decode(lib, body, element_size)
        assert got_nb == nb and got == counts and payload == sum(counts) * element_size


def test_trailer_layout_matches_the_reference_example():
    # multi_batch.zig:24-39: 4 batches of 128-byte events (8, 1, 0, 4 events) -> 128-byte trailer,
    # items written from the end: [padding..., 4, 0, 1, 8, postamble 4].
    lib = native.load()
    body = encode(lib, [8, 1, 0, 4], 128)
    assert len(body) == 13 * 128 + 128
    trailer = np.frombuffer(body[-128:], dtype=np.uint16)
    assert list(trailer[-5:]) == [4, 0, 1, 8, 4]
    assert all(trailer[:-5] == 0xFFFF)


def test_invalid_bodies_are_rejected():
    lib = native.load()
    body = bytearray(encode(lib, [2, 3], 128))
    assert decode(lib, bytes(body), 128)[0] == 2
    bad = bytearray(body)
    bad[-2:] = b"\x00\x00"  # zero batches
    assert decode(lib, bytes(bad), 128)[0] == -1
    bad = bytearray(body)
    bad[-128] = 0  # padding byte not 0xFF
    assert decode(lib, bytes(bad), 128)[0] == -1
    assert decode(lib, bytes(body[:-128]), 128)[0] == -1
    assert decode(lib, bytes(body) + bytes(128), 128)[0] == -1

"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports every
symbol include/lz4mi.h declares, its host xxh32 matches the reference, and the
GPU entry points fail loudly (no silent CPU fallback) when no gfx950 device is
present."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as O
from conftest import ROOT, cases_of

lz4mi = pytest.importorskip("lz4mi")


def _declared():
    with open(os.path.join(ROOT, "include", "lz4mi.h")) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(lz4mi_[a-z0-9_]+)\s*\(", text))
    names.discard("lz4mi_compress_bound")                 # static inline in the header
    return names


def test_library_exports_every_declared_symbol():
    L = lz4mi.lib()
    declared = _declared()
    assert declared == set(lz4mi.EXPORTS)
    for name in declared:
        assert hasattr(L, name), name
        assert ctypes.cast(getattr(L, name), ctypes.c_void_p).value


def test_status_messages_are_the_reference_strings():
    assert lz4mi.status_message(-1) == "LZ4: Output Buffer Too Small"
    assert lz4mi.status_message(-2) == "LZ4: Malformed Input"
    assert lz4mi.status_message(-3) == "LZ4: Invalid Offset 0"
    assert lz4mi.status_message(-4) == "LZ4: Dictionary Offset Out of Bounds"
    assert lz4mi.status_message(-5) == "LZ4: Invalid Magic Number"
    assert lz4mi.status_message(-7) == "LZ4: Content Checksum Error"


def test_host_xxh32_matches_reference(manifest):
    (c,) = cases_of(manifest, "xxh32")
    base = O.generate(c["input"]["gen"], c["input"]["seed"], c["input"]["n"])
    for n, h0, h1 in c["rows"]:
        assert "%08x" % lz4mi.xxh32(base[:n], 0) == h0
        assert "%08x" % lz4mi.xxh32(base[:n], 12345) == h1
        assert lz4mi.xxh32(base[:n], 0, standard=True) == O.xxh32_std(base[:n])
    assert lz4mi.xxh32(b"") == 0x02CC5D05 and lz4mi.xxh32(b"Hello World") == 0xB1FD16EE


def _has_gpu():
    try:
        return lz4mi.device_count() > 0 and lz4mi.lib().lz4mi_init(0) == 0
    except Exception:
        return False


def test_gpu_entry_points_fail_loudly_without_device():
    if _has_gpu():
        pytest.skip("a GPU is present")
    with pytest.raises(lz4mi.Lz4miError) as ei:
        lz4mi.compress_block(np.zeros(100, dtype=np.uint8))
    assert ei.value.status == lz4mi.ERR_NO_DEVICE
    with pytest.raises(lz4mi.Lz4miError):
        lz4mi.decompress_blocks([np.array([0x10, 1], dtype=np.uint8)], [1])

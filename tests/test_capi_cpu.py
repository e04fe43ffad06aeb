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


def test_one_device_per_process_status():
    """a second device is refused with its own status, not a generic argument
    error (the library's stream and scratch live on the first device it was bound to)."""
    assert lz4mi.ERR_DEVICE_BOUND == -103
    assert lz4mi.status_message(-103) == "lz4mi: library already bound to another device (one device per process)"


def test_host_encoder_rejects_positions_past_int32():
    """start + len past 2^31 would overflow the encoder's int32 positions
    (the table holds position + 1); the host entry points refuse it before reading src."""
    import ctypes
    L = lz4mi.lib()
    src = (ctypes.c_uint8 * 64)()
    table = (ctypes.c_int32 * 16384)()
    out = (ctypes.c_uint8 * 64)()
    big = 1 << 32
    r = L.lz4mi_host_compress_block(src, big, (1 << 31) - 10, 20, table, out, 64, 0)
    assert r == lz4mi.ERR_ARG
    offs = (ctypes.c_uint64 * 2)()
    clen = (ctypes.c_uint32 * 2)()
    r = L.lz4mi_host_compress_chain(src, big, (1 << 31) - 10, 20, 4 << 20, table, out, offs, clen)
    assert r == lz4mi.ERR_ARG


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


def source_hash():
    """The Makefile's SRC_HASH: sha256 of SRC then HDR, in Makefile order, first 16 hex digits."""
    import hashlib
    pkg = os.path.join(ROOT, "divortio-lz4_amd")
    with open(os.path.join(pkg, "Makefile")) as f:
        mk = f.read()
    files = []
    for var in ("SRC", "HDR"):
        files += re.search(r"^%s := (.*)$" % var, mk, flags=re.M).group(1).split()
    h = hashlib.sha256()
    for name in files:
        with open(os.path.join(pkg, name), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def test_loaded_library_was_built_from_this_tree():
    """Build provenance: the library's compiled-in source hash equals the hash of the
    sources beside it (a stale liblz4mi.so fails here, on CPU and on the GPU box)."""
    assert lz4mi.build_id() == source_hash()
    assert lz4mi.build_id() in lz4mi.lib().lz4mi_version().decode()


def test_streaming_xxh32_matches_reference_class(manifest):
    """lz4mi_xxh32_reset/update/digest vs class XXHash32 (xxhash32Stateful.js) on the golden chunkings."""
    (g,) = cases_of(manifest, "xxh32_stateful")
    base = O.generate(g["input"]["gen"], g["input"]["seed"], g["input"]["n"])
    for n, chunk, seed, h in g["rows"]:
        st = lz4mi.XXHash32(seed)
        for p in range(0, n, chunk):
            st.update(base[p:min(n, p + chunk)])
        assert "%08x" % st.digest() == h, (n, chunk)
        assert st.digest() == lz4mi.xxh32(base[:n], seed)          # digest() leaves the state unchanged
    seed, n, h = g["empty_updates"]
    st = lz4mi.XXHash32(seed)
    for part in (base[:0], base[:5], base[:0], base[5:n]):
        st.update(part)
    assert "%08x" % st.digest() == h
    (c,) = cases_of(manifest, "xxh32")
    st = lz4mi.XXHash32(0)
    for p in range(0, 1000, 37):
        st.update(base[:0])
    gen = O.generate(c["input"]["gen"], c["input"]["seed"], 1000)
    st = lz4mi.XXHash32(0)
    for p in range(0, 1000, 37):
        st.update(gen[p:p + 37])
    assert "%08x" % st.digest() == c["stateful_1000"]


def test_streaming_xxh32_length_modes():
    """The class wraps totalLen at 2^32 and tests it signed (:37,:113); LEN64 keeps the full
    length. Both agree below 2 GiB, and with the spec convergence flag match the spec digest."""
    data = O.generate("random", 5, 5000)
    for std in (False, True):
        a = lz4mi.XXHash32(3, standard=std).update(data).digest()
        b = lz4mi.XXHash32(3, standard=std, len64=True).update(data).digest()
        assert a == b == lz4mi.xxh32(data, 3, standard=std)
    assert lz4mi.XXHash32(0, standard=True).update(data).digest() == O.xxh32_std(data)

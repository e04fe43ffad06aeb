"""TEST INFRASTRUCTURE ONLY — ctypes loader for the CPU oracle (lz4_oracle.c).

The oracle restates the reference algorithms (see lz4_oracle.c header for the
file:line citations) and is pinned by tests/golden/ fixtures generated from the
reference JavaScript. Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product path never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liblz4oracle.so")
_lib = None

GEN_RANDOM, GEN_REPETITIVE, GEN_TILES216, GEN_COPY, GEN_RUNS, GEN_TEXT = range(6)
GENERATORS = {"random": GEN_RANDOM, "repetitive": GEN_REPETITIVE, "tiles216": GEN_TILES216,
              "copy": GEN_COPY, "runs": GEN_RUNS, "text": GEN_TEXT}

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i32p = ctypes.POINTER(ctypes.c_int32)
_i64p = ctypes.POINTER(ctypes.c_int64)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(
                os.path.join(_HERE, "lz4_oracle.c")):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_xxh32.restype = ctypes.c_uint32
        L.orc_xxh32.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_xxh32_std.restype = ctypes.c_uint32
        L.orc_xxh32_std.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_xxh32_stateful.restype = ctypes.c_uint32
        L.orc_xxh32_stateful.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_compress_block_ex.restype = ctypes.c_int32
        L.orc_compress_block_ex.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32, _i32p]
        L.orc_compress_block.restype = ctypes.c_int32
        L.orc_compress_block.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
        L.orc_decompress_block.restype = ctypes.c_int32
        L.orc_decompress_block.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64,
                                           ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32, _i64p]
        L.orc_frame_bound.restype = ctypes.c_int64
        L.orc_frame_bound.argtypes = [ctypes.c_int64]
        L.orc_compress_frame_ex.restype = ctypes.c_int64
        L.orc_compress_frame_ex.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                            ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64]
        L.orc_compress_frame.restype = ctypes.c_int64
        L.orc_compress_frame.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                         ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                         ctypes.c_void_p, ctypes.c_int64]
        L.orc_decompress_frame.restype = ctypes.c_int32
        L.orc_decompress_frame.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                           ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                           _i64p, _i32p]
        L.orc_generate.restype = None
        L.orc_generate.argtypes = [ctypes.c_int32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_int64]
        L.orc_blocks_mt.restype = ctypes.c_int32
        L.orc_blocks_mt.argtypes = [ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data if a is not None and a.size else None


def _u8(x):
    if x is None:
        return None
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    return np.ascontiguousarray(x, dtype=np.uint8)


def xxh32(data, seed=0):
    a = _u8(data)
    return lib().orc_xxh32(_ptr(a), a.size, seed & 0xFFFFFFFF)


def xxh32_std(data, seed=0):
    """Spec XXH32 (differs from the reference's variant for len >= 16)."""
    a = _u8(data)
    return lib().orc_xxh32_std(_ptr(a), a.size, seed & 0xFFFFFFFF)


def xxh32_stateful(chunks, seed=0):
    """class XXHash32 (xxhash32Stateful.js) fed the given chunks in order."""
    arrs = [_u8(c) for c in chunks]
    data = np.concatenate(arrs) if arrs else np.zeros(0, dtype=np.uint8)
    lens = np.array([a.size for a in arrs], dtype=np.uint64)
    return lib().orc_xxh32_stateful(_ptr(data), lens.ctypes.data if lens.size else None, lens.size,
                                    seed & 0xFFFFFFFF)


def generate(kind, seed, n):
    """Seeded synthetic input (SURVEY.md §8d generators)."""
    k = GENERATORS[kind] if isinstance(kind, str) else kind
    out = np.empty(n, dtype=np.uint8)
    lib().orc_generate(k, seed & 0xFFFFFFFF, _ptr(out), n)
    return out


def compress_bound(n):
    return n + n // 255 + 16


def compress_block(src, start=0, length=None, table=None, out=None, out_off=0):
    """blockCompress.js:31 restated. Returns (bytes_written, out, table)."""
    s = _u8(src)
    if length is None:
        length = s.size - start
    if table is None:
        table = np.zeros(16384, dtype=np.int32)
    if out is None:
        out = np.zeros(out_off + compress_bound(length), dtype=np.uint8)
    n = lib().orc_compress_block(_ptr(s), s.size, _ptr(out), out.size, start, length,
                                 table.ctypes.data, out_off)
    return n, out, table


def compress_raw(src, out, start, length, table, out_off):
    """compressBlock with the reference's exception: returns (status, written); status
    -8 (RangeError of output.set, blockCompress.js:100/198) leaves `out`/`table` as
    the reference leaves them when it throws."""
    s = _u8(src)
    st = ctypes.c_int32(0)
    n = lib().orc_compress_block_ex(_ptr(s), s.size, _ptr(out), out.size, start, length, table.ctypes.data,
                                    out_off, ctypes.byref(st))
    return st.value, n


def compress_block_bytes(src):
    n, out, _ = compress_block(src)
    return out[:n].copy()


def decompress_block(comp, out_size, in_off=0, in_size=None, out=None, out_off=0, dictionary=None,
                     js_compat=False, in_total=None):
    """blockDecompress.js:30 restated. Returns (status, written, out)."""
    c = _u8(comp)
    if in_size is None:
        in_size = c.size - in_off
    if in_total is None:
        in_total = c.size
    if out is None:
        out = np.zeros(out_off + out_size, dtype=np.uint8)
    d = _u8(dictionary)
    w = ctypes.c_int64(0)
    st = lib().orc_decompress_block(_ptr(c), in_total, in_off, in_size, _ptr(out), out.size, out_off,
                                    _ptr(d), 0 if d is None else d.size, 1 if js_compat else 0,
                                    ctypes.byref(w))
    return st, w.value, out


def compress_frame(data, dictionary=None, max_block_size=4194304, block_independence=False,
                   content_checksum=False, add_content_size=True, block_checksum=False):
    a = _u8(data)
    d = _u8(dictionary)
    cap = lib().orc_frame_bound(a.size) + 64 + (4 * (a.size // 65536 + 2) if block_checksum else 0)
    out = np.zeros(cap, dtype=np.uint8)
    n = lib().orc_compress_frame_ex(_ptr(a), a.size, _ptr(d), 0 if d is None else d.size, max_block_size,
                                    int(bool(block_independence)), int(bool(content_checksum)),
                                    int(bool(add_content_size)), int(bool(block_checksum)), _ptr(out), cap)
    return out[:n].copy()


def decompress_frame(frame, dictionary=None, verify_checksum=True, js_compat=False, out_cap=None):
    """Returns (status, bytes). out_cap defaults to a generous bound."""
    f = _u8(frame)
    d = _u8(dictionary)
    if out_cap is None:
        out_cap = max(64, f.size * 256 + (1 << 20))
    out = np.zeros(out_cap, dtype=np.uint8)
    olen = ctypes.c_int64(0)
    ver = ctypes.c_int32(0)
    st = lib().orc_decompress_frame(_ptr(f), f.size, _ptr(d), 0 if d is None else d.size,
                                    int(bool(verify_checksum)), int(bool(js_compat)), _ptr(out), out_cap,
                                    ctypes.byref(olen), ctypes.byref(ver))
    return st, out[:olen.value].copy()


def blocks_mt(mode, inp, in_off, in_len, out, out_off, out_cap, nthreads):
    """Multi-threaded CPU pass over independent blocks (mode 0 decompress, 1 compress,
    2 decompress with the reference decoder's bytes, js_compat)."""
    n = len(in_len)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    lib().orc_blocks_mt(mode, _ptr(inp), in_off.ctypes.data, in_len.ctypes.data, _ptr(out),
                        out_off.ctypes.data, out_cap.ctypes.data, out_len.ctypes.data, status.ctypes.data,
                        n, nthreads)
    return out_len, status


def census(kind, seed0, nblocks, bs, nthreads, js_compat=True, chunk=256):
    """Per block b (seed seed0 + b): xxh32 of the generated bytes, the compressed length and its xxh32
    (the oracle encoder, fresh table), and the decode's status, length and xxh32 (the reference decoder's
    bytes with js_compat, each block in an array of its own). Host threads, `chunk` blocks at a time."""
    from concurrent.futures import ThreadPoolExecutor
    res = {k: [] for k in ("src_xxh", "comp_len", "comp_xxh", "dec_status", "dec_len", "dec_xxh")}
    cap = compress_bound(bs)
    with ThreadPoolExecutor(nthreads) as ex:     # the C calls drop the GIL
        for b0 in range(0, nblocks, chunk):
            k = min(chunk, nblocks - b0)
            host = np.concatenate(list(ex.map(lambda b: generate(kind, seed0 + b, bs), range(b0, b0 + k))))
            res["src_xxh"] += list(ex.map(lambda j: xxh32(host[j * bs:(j + 1) * bs]), range(k)))
            in_off = np.arange(k, dtype=np.uint64) * bs
            in_len = np.full(k, bs, dtype=np.uint32)
            comp = np.zeros(k * cap, dtype=np.uint8)
            c_off = np.arange(k, dtype=np.uint64) * cap
            c_cap = np.full(k, cap, dtype=np.uint32)
            clen, _ = blocks_mt(1, host, in_off, in_len, comp, c_off, c_cap, nthreads)
            res["comp_len"] += [int(x) for x in clen]
            res["comp_xxh"] += list(ex.map(lambda j: xxh32(comp[j * cap:j * cap + int(clen[j])]), range(k)))
            host[:] = 0
            dlen, dst = blocks_mt(2 if js_compat else 0, comp, c_off, clen, host, in_off, in_len, nthreads)
            res["dec_status"] += [int(x) for x in dst]
            res["dec_len"] += [int(x) for x in dlen]
            res["dec_xxh"] += list(ex.map(lambda j: xxh32(host[j * bs:j * bs + int(dlen[j])]), range(k)))
    return res


def digest_of_digests(hashes):
    """XXH32 over the u32 digests, little-endian, in order (tests/golden 'bench_batch_js_decode')."""
    return xxh32(np.array([h & 0xFFFFFFFF for h in hashes], dtype="<u4").view(np.uint8))

"""Python binding of liblz4mi.so (include/lz4mi.h) — the MI355X LZ4 block codec.

Used by bench.py, __graft_entry__ and the tests. Every compute entry point goes
through the HIP C-ABI; there is no CPU fallback: if the library or a gfx950
device is missing, calls raise Lz4miError.

Mirrors the reference's raw-block and frame functions
(src/block/blockCompress.js:31, src/block/blockDecompress.js:30,
src/xxhash32/xxhash32.js:21) with the same argument meaning and error strings.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_DIR, "liblz4mi.so")

OK = 0
ERR_OUTPUT_TOO_SMALL, ERR_MALFORMED, ERR_OFFSET0, ERR_DICT_OOB = -1, -2, -3, -4
ERR_MAGIC, ERR_VERSION, ERR_CHECKSUM, ERR_RANGE, ERR_CROSS_BLOCK = -5, -6, -7, -8, -9
ERR_BLOCK_CHECKSUM = -10
ERR_HIP, ERR_ARG, ERR_NO_DEVICE, ERR_DEVICE_BOUND = -100, -101, -102, -103

DEVICE_PTRS = 0x1
JS_COMPAT = 0x2
JS_EXACT = 0x8
XXH_STANDARD = 0x4
XXH_LEN64 = 0x10
BLOCK_CHECKSUM = 0x20
FRAME_WORDS = 0x40

GEN_RANDOM, GEN_REPETITIVE, GEN_TILES216 = 0, 1, 2
GENERATORS = {"random": GEN_RANDOM, "repetitive": GEN_REPETITIVE, "tiles216": GEN_TILES216}
# decode batches of at most this many blocks take the small-batch path (the library's default,
# csrc/lz4mi_capi.cpp small_blocks(); LZ4MI_SMALL_BLOCKS changes it, read once per process)
SMALL_BLOCKS = int(os.environ.get("LZ4MI_SMALL_BLOCKS", "192"))

# every symbol include/lz4mi.h declares (checked by tests/test_capi_cpu.py)
EXPORTS = ("lz4mi_status_message", "lz4mi_init", "lz4mi_device_count", "lz4mi_version",
           "lz4mi_decompress_blocks", "lz4mi_compress_blocks", "lz4mi_compress_block_table",
           "lz4mi_xxh32", "lz4mi_xxh32_blocks", "lz4mi_frame_pack", "lz4mi_generate_blocks",
           "lz4mi_build_id", "lz4mi_xxh32_reset", "lz4mi_xxh32_update", "lz4mi_xxh32_digest",
           "lz4mi_frame_decompress", "lz4mi_frame_index", "lz4mi_compress_chain",
           "lz4mi_host_compress_block", "lz4mi_host_compress_chain", "lz4mi_host_decompress_block")


class Lz4miError(RuntimeError):
    def __init__(self, status, message=None):
        self.status = status
        super().__init__(message or status_message(status))


_lib = None
_vp = ctypes.c_void_p


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Lz4miError(ERR_NO_DEVICE, "liblz4mi.so not built (run __graft_entry__.build())")
        # PyTorch wheels bundle their own libamdhip64 under a different file name;
        # load torch first so one HIP runtime serves both (a second runtime
        # instance in the process cannot see the GPU).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.lz4mi_status_message.restype = ctypes.c_char_p
        L.lz4mi_status_message.argtypes = [ctypes.c_int32]
        L.lz4mi_version.restype = ctypes.c_char_p
        L.lz4mi_build_id.restype = ctypes.c_char_p
        L.lz4mi_xxh32_reset.restype = None
        L.lz4mi_xxh32_reset.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32]
        L.lz4mi_xxh32_update.restype = None
        L.lz4mi_xxh32_update.argtypes = [_vp, _vp, ctypes.c_size_t]
        L.lz4mi_xxh32_digest.restype = ctypes.c_uint32
        L.lz4mi_xxh32_digest.argtypes = [_vp]
        L.lz4mi_init.restype = ctypes.c_int32
        L.lz4mi_init.argtypes = [ctypes.c_int32]
        L.lz4mi_device_count.restype = ctypes.c_int32
        L.lz4mi_decompress_blocks.restype = ctypes.c_int32
        L.lz4mi_decompress_blocks.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, _vp, _vp,
                                              ctypes.c_uint32, ctypes.c_uint32, _vp]
        L.lz4mi_compress_blocks.restype = ctypes.c_int32
        L.lz4mi_compress_blocks.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp]
        L.lz4mi_compress_block_table.restype = ctypes.c_int64
        L.lz4mi_compress_block_table.argtypes = [_vp, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, _vp, _vp,
                                                 ctypes.c_uint64, ctypes.c_int32, ctypes.c_uint32, _vp]
        L.lz4mi_xxh32.restype = ctypes.c_uint32
        L.lz4mi_xxh32.argtypes = [_vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32]
        L.lz4mi_xxh32_blocks.restype = ctypes.c_int32
        L.lz4mi_xxh32_blocks.argtypes = [_vp, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp]
        L.lz4mi_frame_pack.restype = ctypes.c_int32
        L.lz4mi_frame_pack.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_uint32, ctypes.c_uint32, _vp]
        L.lz4mi_frame_decompress.restype = ctypes.c_int32
        L.lz4mi_frame_decompress.argtypes = [_vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp]
        L.lz4mi_compress_chain.restype = ctypes.c_int32
        L.lz4mi_compress_chain.argtypes = [_vp, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, _vp,
                                           _vp, _vp, _vp, ctypes.c_uint32, _vp]
        L.lz4mi_host_compress_block.restype = ctypes.c_int64
        L.lz4mi_host_compress_block.argtypes = [_vp, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, _vp, _vp,
                                                ctypes.c_uint64, ctypes.c_int32]
        L.lz4mi_host_compress_chain.restype = ctypes.c_int32
        L.lz4mi_host_compress_chain.argtypes = [_vp, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                                _vp, _vp, _vp, _vp]
        L.lz4mi_host_decompress_block.restype = ctypes.c_int64
        L.lz4mi_host_decompress_block.argtypes = [_vp, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int64, _vp,
                                                  ctypes.c_uint64, ctypes.c_int64, _vp, ctypes.c_uint32, ctypes.c_uint32]
        L.lz4mi_frame_index.restype = ctypes.c_int32
        L.lz4mi_frame_index.argtypes = [_vp, ctypes.c_uint64, _vp, _vp, ctypes.c_uint32, _vp, ctypes.c_uint32, _vp]
        L.lz4mi_generate_blocks.restype = ctypes.c_int32
        L.lz4mi_generate_blocks.argtypes = [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, _vp]
        _lib = L
    return _lib


def status_message(status):
    return lib().lz4mi_status_message(int(status)).decode()


def _check(st):
    if st != OK:
        raise Lz4miError(st)


def init(device=-1):
    _check(lib().lz4mi_init(device))


def device_count():
    return lib().lz4mi_device_count()


def build_id():
    """Hash of the sources liblz4mi.so was compiled from (see Makefile SRC_HASH)."""
    return lib().lz4mi_build_id().decode()


def _p(a):
    return a.ctypes.data if a is not None and a.size else None


def _u8(x):
    if x is None:
        return None
    if isinstance(x, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(x), dtype=np.uint8)
    return np.ascontiguousarray(x, dtype=np.uint8)


def compress_bound(n):
    return n + n // 255 + 16


# ---------------------------------------------------------------- host API
def xxh32(data, seed=0, standard=False):
    """xxHash32 (reference variant by default; host CPU, one serial chain)."""
    a = _u8(data)
    return lib().lz4mi_xxh32(_p(a), a.size, seed & 0xFFFFFFFF, XXH_STANDARD if standard else 0)


class XXHash32:
    """Streaming XXH32 (class XXHash32, src/xxhash32/xxhash32Stateful.js:13-152) over the
    library's host implementation: update(chunk) any number of times, digest() any time.
    len64=True keeps the 64-bit length (the reference wraps it at 2 GiB, :37)."""

    def __init__(self, seed=0, standard=False, len64=False):
        self._st = np.zeros(7, dtype=np.uint64)       # lz4mi_xxh32_state
        lib().lz4mi_xxh32_reset(self._st.ctypes.data, seed & 0xFFFFFFFF,
                                (XXH_STANDARD if standard else 0) | (XXH_LEN64 if len64 else 0))

    def update(self, data):
        a = _u8(data)
        lib().lz4mi_xxh32_update(self._st.ctypes.data, _p(a), a.size)
        return self

    def digest(self):
        return lib().lz4mi_xxh32_digest(self._st.ctypes.data)


def compress_blocks(blocks):
    """Independent raw blocks -> list of compressed byte arrays (GPU)."""
    arrs = [_u8(b) for b in blocks]
    n = len(arrs)
    if n == 0:
        return []
    in_len = np.array([a.size for a in arrs], dtype=np.uint32)
    in_off = np.zeros(n, dtype=np.uint64)
    in_off[1:] = np.cumsum(in_len[:-1].astype(np.uint64))
    src = np.concatenate(arrs) if in_len.sum() else np.zeros(1, dtype=np.uint8)
    bounds = np.array([compress_bound(int(x)) for x in in_len], dtype=np.uint64)
    out_off = np.zeros(n, dtype=np.uint64)
    out_off[1:] = np.cumsum(bounds[:-1])
    out = np.zeros(int(bounds.sum()), dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    _check(lib().lz4mi_compress_blocks(_p(src), _p(in_off), _p(in_len), _p(out), _p(out_off), _p(out_len), n, 0,
                                       None))
    return [out[int(o):int(o) + int(l)].copy() for o, l in zip(out_off, out_len)]


def compress_block(data):
    return compress_blocks([data])[0]


def compress_raw(src, output, src_start, src_len, hash_table, output_offset):
    """compressBlock(src, output, srcStart, srcLen, hashTable, outputOffset) with
    the reference's full semantics (table in/out, absolute positions)."""
    s = _u8(src)
    assert hash_table.dtype == np.int32 and hash_table.size == 16384 and hash_table.flags.c_contiguous
    assert output.dtype == np.uint8 and output.flags.c_contiguous
    r = lib().lz4mi_compress_block_table(_p(s), s.size, src_start, src_len, hash_table.ctypes.data,
                                         _p(output), output.size, output_offset or 0, 0, None)
    if r < 0:
        raise Lz4miError(int(r))
    return 0 if output_offset is None else int(r)   # (dIndex - undefined) | 0 (blockCompress.js:232)


def compress_chain(src, start, length, block_size, hash_table, host=False):
    """Dependent blocks in order with one carried table (lz4mi_compress_chain, or with `host`
    the host encoder lz4mi_host_compress_chain): returns the list of compressed blocks, each
    what compressBlock(src, scratch, start_b, n_b, table, 0) writes; hash_table (int32[16384])
    is updated in place."""
    s = _u8(src)
    assert hash_table.dtype == np.int32 and hash_table.size == 16384 and hash_table.flags.c_contiguous
    nb = -(-length // block_size) if length > 0 else 0
    if nb == 0:
        return []
    ns = [min(block_size, length - b * block_size) for b in range(nb)]
    bounds = np.array([compress_bound(n) for n in ns], dtype=np.uint64)
    out_off = np.zeros(nb, dtype=np.uint64)
    out_off[1:] = np.cumsum(bounds[:-1])
    out = np.zeros(int(bounds.sum()), dtype=np.uint8)
    comp_len = np.zeros(nb, dtype=np.uint32)
    if host:
        _check(lib().lz4mi_host_compress_chain(_p(s), s.size, start, length, block_size, hash_table.ctypes.data,
                                               _p(out), _p(out_off), _p(comp_len)))
    else:
        _check(lib().lz4mi_compress_chain(_p(s), s.size, start, length, block_size, hash_table.ctypes.data,
                                          _p(out), _p(out_off), _p(comp_len), 0, None))
    return [out[int(o):int(o) + int(n)].copy() for o, n in zip(out_off, comp_len)]


def host_decompress_raw(inp, input_offset, input_size, output, output_offset=0, dictionary=None, spec=False):
    """decompressBlock on the host decoder (lz4mi_host_decompress_block): writes into `output`
    (numpy uint8, the whole output array) and returns bytes written; raises with the reference's
    message. Reference bytes (F1 included) unless `spec`."""
    a = _u8(inp)
    d = None if dictionary is None else _u8(dictionary)
    assert output.dtype == np.uint8 and output.flags.c_contiguous
    r = lib().lz4mi_host_decompress_block(_p(a), a.size, input_offset, input_size, _p(output), output.size,
                                          output_offset, None if d is None else _p(d), 0 if d is None else d.size,
                                          0 if spec else JS_EXACT)
    if r < 0:
        raise Lz4miError(int(r))
    return int(r)


def host_compress_raw(src, output, src_start, src_len, hash_table, output_offset):
    """compressRaw on the host encoder (lz4mi_host_compress_block): the same contract as
    compress_raw, no device involved."""
    s = _u8(src)
    assert hash_table.dtype == np.int32 and hash_table.size == 16384 and hash_table.flags.c_contiguous
    assert output.dtype == np.uint8 and output.flags.c_contiguous
    r = lib().lz4mi_host_compress_block(_p(s), s.size, src_start, src_len, hash_table.ctypes.data, _p(output),
                                        output.size, output_offset or 0)
    if r < 0:
        raise Lz4miError(int(r))
    return 0 if output_offset is None else int(r)


def _dec_flags(js_compat, js_exact):
    return JS_COMPAT if js_compat else (JS_EXACT if js_exact else 0)


def decompress_blocks(blocks, out_sizes, js_compat=False, dictionary=None, js_exact=False):
    """Independent compressed blocks -> (statuses, outputs) (GPU).
    js_compat: the serial reference-exact kernel; js_exact: the parallel spec
    kernel plus a serial re-decode of the blocks the reference's F1 rewrite changes."""
    arrs = [_u8(b) for b in blocks]
    n = len(arrs)
    in_len = np.array([a.size for a in arrs], dtype=np.uint32)
    in_off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        in_off[1:] = np.cumsum(in_len[:-1].astype(np.uint64))
    src = np.concatenate(arrs) if n and in_len.sum() else np.zeros(1, dtype=np.uint8)
    out_cap = np.array(out_sizes, dtype=np.uint32)
    out_off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        out_off[1:] = np.cumsum(out_cap[:-1].astype(np.uint64))
    out = np.zeros(max(1, int(out_cap.sum())), dtype=np.uint8)
    out_len = np.zeros(n, dtype=np.uint32)
    status = np.zeros(n, dtype=np.int32)
    d = _u8(dictionary)
    _check(lib().lz4mi_decompress_blocks(_p(src), _p(in_off), _p(in_len), _p(out), _p(out_off), _p(out_cap),
                                         _p(d), 0 if d is None else d.size, _p(out_len), _p(status), n,
                                         _dec_flags(js_compat, js_exact), None))
    outs = [out[int(o):int(o) + min(int(l), int(c))].copy() for o, l, c in zip(out_off, out_len, out_cap)]
    return status, outs, out_len


def decompress_raw(inp, input_offset, input_size, output, output_offset=0, dictionary=None, js_compat=False,
                   js_exact=False):
    """decompressBlock(input, inputOffset, inputSize, output, outputOffset, dictionary):
    writes into `output` (numpy uint8) and returns bytes written; raises with the
    reference's message on error."""
    a = _u8(inp)
    seg = a[input_offset:input_offset + input_size]
    in_off = np.zeros(1, dtype=np.uint64)
    in_len = np.array([seg.size], dtype=np.uint32)
    out_off = np.array([output_offset], dtype=np.uint64)
    out_cap = np.array([max(0, output.size - output_offset)], dtype=np.uint32)
    out_len = np.zeros(1, dtype=np.uint32)
    status = np.zeros(1, dtype=np.int32)
    d = _u8(dictionary)
    seg = np.ascontiguousarray(seg) if seg.size else np.zeros(1, dtype=np.uint8)
    _check(lib().lz4mi_decompress_blocks(_p(seg), _p(in_off), _p(in_len), _p(output), _p(out_off), _p(out_cap),
                                         _p(d), 0 if d is None else d.size, _p(out_len), _p(status), 1,
                                         _dec_flags(js_compat, js_exact), None))
    if status[0] != OK:
        raise Lz4miError(int(status[0]))
    return int(out_len[0])


def xxh32_blocks(blocks, seed=0, standard=False):
    arrs = [_u8(b) for b in blocks]
    n = len(arrs)
    ln = np.array([a.size for a in arrs], dtype=np.uint32)
    off = np.zeros(n, dtype=np.uint64)
    if n > 1:
        off[1:] = np.cumsum(ln[:-1].astype(np.uint64))
    src = np.concatenate(arrs) if n and ln.sum() else np.zeros(1, dtype=np.uint8)
    h = np.zeros(n, dtype=np.uint32)
    _check(lib().lz4mi_xxh32_blocks(_p(src), _p(off), _p(ln), seed & 0xFFFFFFFF, _p(h), n,
                                    XXH_STANDARD if standard else 0, None))
    return h


# -------------------------------------------------------------- device API
# Raw device pointers (ints, e.g. torch tensor .data_ptr()) and a hipStream_t
# handle (int, e.g. torch.cuda.current_stream().cuda_stream). Async.
def decompress_blocks_dev(in_ptr, in_off_ptr, in_len_ptr, out_ptr, out_off_ptr, out_cap_ptr, out_len_ptr,
                          status_ptr, nblocks, stream=0, js_compat=False, dict_ptr=None, dict_len=0,
                          frame_words=False, js_exact=False):
    """Batch decode on device pointers. frame_words: in_len holds frame size words (bit 31 =
    stored block, copied in the same launch; include/lz4mi.h LZ4MI_FRAME_WORDS). js_exact: the
    reference decoder's bytes (LZ4MI_JS_EXACT, the JS layer's default)."""
    _check(lib().lz4mi_decompress_blocks(in_ptr, in_off_ptr, in_len_ptr, out_ptr, out_off_ptr, out_cap_ptr,
                                         dict_ptr, dict_len, out_len_ptr, status_ptr, nblocks,
                                         DEVICE_PTRS | _dec_flags(js_compat, js_exact) |
                                         (FRAME_WORDS if frame_words else 0), stream or None))


def compress_blocks_dev(in_ptr, in_off_ptr, in_len_ptr, out_ptr, out_off_ptr, out_len_ptr, nblocks, stream=0):
    _check(lib().lz4mi_compress_blocks(in_ptr, in_off_ptr, in_len_ptr, out_ptr, out_off_ptr, out_len_ptr, nblocks,
                                       DEVICE_PTRS, stream or None))


def xxh32_blocks_dev(in_ptr, off_ptr, len_ptr, hashes_ptr, nblocks, seed=0, stream=0, standard=False):
    _check(lib().lz4mi_xxh32_blocks(in_ptr, off_ptr, len_ptr, seed & 0xFFFFFFFF, hashes_ptr, nblocks,
                                    DEVICE_PTRS | (XXH_STANDARD if standard else 0), stream or None))


def frame_decompress_dev(frame_ptr, frame_len, out_ptr, out_cap, stream=0, js_exact=False):
    """Decode a device-resident LZ4 frame into out (device pointers): returns the info dict
    (include/lz4mi.h lz4mi_frame_decompress); raises if the frame needs the host path."""
    info = np.zeros(8, dtype=np.int64)
    _check(lib().lz4mi_frame_decompress(frame_ptr, frame_len, out_ptr, out_cap, info.ctypes.data,
                                        DEVICE_PTRS | (JS_EXACT if js_exact else 0), stream or None))
    keys = ("status", "flg", "content_size", "written", "stored_blocks", "checksum_pos", "block_max", "overflow")
    return dict(zip(keys, (int(x) for x in info)))


def generate_blocks_dev(out_ptr, kind, seed0, block_size, nblocks, stream=0):
    k = GENERATORS[kind] if isinstance(kind, str) else kind
    _check(lib().lz4mi_generate_blocks(out_ptr, k, seed0, block_size, nblocks, stream or None))


def frame_pack_dev(raw_ptr, raw_off_ptr, raw_len_ptr, comp_ptr, comp_off_ptr, comp_len_ptr, frame_ptr, rec_off_ptr,
                   nblocks, stream=0, block_checksum=False):
    """Device-side frame block records (size word + compressed or stored payload [+ XXH32 of
    the payload with block_checksum]) at rec_off."""
    _check(lib().lz4mi_frame_pack(raw_ptr, raw_off_ptr, raw_len_ptr, comp_ptr, comp_off_ptr, comp_len_ptr, frame_ptr,
                                  rec_off_ptr, nblocks, DEVICE_PTRS | (BLOCK_CHECKSUM if block_checksum else 0),
                                  stream or None))


def frame_index_dev(frame_ptr, frame_len, pay_off_ptr, size_word_ptr, cap_blocks, info_ptr, stream=0):
    """Block index of a device-resident frame (include/lz4mi.h lz4mi_frame_index): device
    pointers, asynchronous on `stream`."""
    _check(lib().lz4mi_frame_index(frame_ptr, frame_len, pay_off_ptr, size_word_ptr, cap_blocks, info_ptr,
                                   DEVICE_PTRS, stream or None))

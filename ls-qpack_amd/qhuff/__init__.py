"""Python plumbing over libqhuff.so (include/qhuff.h).

The product is the C-ABI library (HIP kernels for gfx950 + host C); this
module only binds it with ctypes so tests and bench.py can drive it with
torch device tensors.  There is no CPU fallback: if libqhuff.so is missing or
no gfx950 device is usable, Codec() raises.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)                 # .../ls-qpack_amd
LIB_PATH = os.environ.get("QHUFF_LIB") or os.path.join(PKG_ROOT, "libqhuff.so")
HEADER = os.path.join(os.path.dirname(PKG_ROOT), "include", "qhuff.h")
HEADERS = (HEADER, os.path.join(os.path.dirname(PKG_ROOT), "include",
                                "qhuff_lsqpack.h"))

OK = 0
EINVAL, ENOMEM, ENODEV, ERANGE, EDEVICE = -22, -12, -19, -34, -5
ENC_PAYLOAD, ENC_LITERAL3, ENC_LITERAL5, ENC_LITERAL7 = 0, 3, 5, 7
DEC_OK, DEC_ERROR = 0, 1
HUFF_DEC_OK, HUFF_DEC_END_SRC, HUFF_DEC_END_DST, HUFF_DEC_ERROR = 0, 1, 2, 3

# every function include/qhuff.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "qhuff_open", "qhuff_close", "qhuff_encode_bound", "qhuff_decode_bound",
    "qhuff_encode_batch", "qhuff_decode_batch", "qhuff_encode_batch_host",
    "qhuff_decode_batch_host", "qhuff_enc_enc_str", "qhuff_enc_str_size",
    "qhuff_huff_decode", "qhuff_huff_decode_ex", "qhuff_abi_version",
    "qhuff_last_error", "qhuff_shard_cuts",
    "qhuff_synth_batch", "qhuff_device_error", "qhuff_profile_read",
    "qhuff_xxh32_headers", "qhuff_xxh32_batch",
    "qhuff_scan_field_section", "qhuff_scan_encoder_stream",
    "qhuff_literals_bound", "qhuff_decode_literals_host",
    "qhuff_decode_literals_ex", "qhuff_batch_hint", "qhuff_batch_needs_full",
    "qhuff_frame_literal", "qhuff_xxh32_headers_host",
    "qhuff_svc_open", "qhuff_svc_close", "qhuff_svc_encode",
    "qhuff_svc_decode", "qhuff_svc_stats",
    "qhuff_timing_enable", "qhuff_timing_read", "qhuff_kernel_variant",
    "qhuff_dec_int", "qhuff_encode_batch_host_multi",
    "qhuff_decode_batch_host_multi", "qhuff_encode_batch_multi",
    "qhuff_decode_batch_multi", "qhuff_host_register", "qhuff_host_unregister",
    # include/qhuff_lsqpack.h
    "qhuff_lsqpack_enc_enc_str", "qhuff_lsqpack_huff_decode",
    "qhuff_lsqpack_set_decode_full", "qhuff_lsqpack_set_device",
    "qhuff_lsqpack_set_context",
)
EPROTO, ETRUNC = -71, -61
TIMING_SLOTS = 256                        # QHUFF_TIMING_SLOTS
KIND_ENCODE, KIND_DECODE, KIND_HASH = 0, 1, 2
LIT_NAME, LIT_VALUE = 1, 2
MAX_STRLEN = 65535                        # QHUFF_MAX_STRLEN (LSXPACK_MAX_STRLEN)

XXH_SEED = 39378473                       # LSQPACK_XXH_SEED, lsqpack.c:623


class QhuffError(RuntimeError):
    pass


class Literal(C.Structure):
    """struct qhuff_literal (include/qhuff.h)"""
    _fields_ = [("pos", C.c_uint32), ("len", C.c_uint32),
                ("huffman", C.c_uint8), ("prefix_bits", C.c_uint8),
                ("kind", C.c_uint8), ("hdr_len", C.c_uint8),
                ("instr", C.c_uint32)]


class Shard(C.Structure):
    """struct qhuff_shard (include/qhuff.h): one device-resident shard"""
    _fields_ = [("in_", C.c_void_p), ("in_off", C.c_void_p),
                ("n", C.c_uint32), ("out", C.c_void_p),
                ("out_off", C.c_void_p), ("status", C.c_void_p),
                ("stream", C.c_void_p)]


class DecodeRetval(C.Structure):
    """struct qhuff_decode_retval (= struct huff_decode_retval,
    lsqpack.c:3420-3431)"""
    _fields_ = [("status", C.c_int), ("n_dst", C.c_uint), ("n_src", C.c_uint)]


class DecodeState(C.Structure):
    """struct qhuff_huff_decode_state (= struct lsqpack_huff_decode_state,
    lsqpack.h:747-757)"""
    _fields_ = [("resume", C.c_int), ("state", C.c_uint8), ("eos", C.c_uint8)]


DECODE_FULL_FN = C.CFUNCTYPE(DecodeRetval, C.c_void_p, C.c_int, C.c_void_p,
                             C.c_int, C.POINTER(DecodeState), C.c_int)


_lib = None


def lib():
    """Load libqhuff.so (built by `make -C ls-qpack_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise QhuffError("libqhuff.so not built: run make -C %s" % PKG_ROOT)
        # One HIP runtime per process: PyTorch ships its own libamdhip64
        # (NEEDED as "libamdhip64.so", soname libamdhip64.so.7).  Loaded
        # first, it satisfies libqhuff's libamdhip64.so.7 dependency; loaded
        # after libqhuff it would be a second runtime (the GPU appears twice,
        # occupancy queries and torch.cuda break).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = C.CDLL(LIB_PATH)
        vp, u32p = C.c_void_p, C.c_void_p
        L.qhuff_open.restype = C.c_int
        L.qhuff_open.argtypes = [C.c_int, C.POINTER(C.c_void_p)]
        L.qhuff_close.restype = None
        L.qhuff_close.argtypes = [vp]
        L.qhuff_encode_bound.restype = C.c_uint64
        L.qhuff_encode_bound.argtypes = [C.c_uint64, C.c_uint32, C.c_uint]
        L.qhuff_decode_bound.restype = C.c_uint64
        L.qhuff_decode_bound.argtypes = [C.c_uint64, C.c_uint32]
        L.qhuff_encode_batch.restype = C.c_int
        L.qhuff_encode_batch.argtypes = [vp, vp, u32p, C.c_uint32, C.c_uint,
                                         vp, u32p, vp]
        L.qhuff_decode_batch.restype = C.c_int
        L.qhuff_decode_batch.argtypes = [vp, vp, u32p, C.c_uint32, vp, u32p,
                                         vp, vp]
        L.qhuff_encode_batch_host.restype = C.c_int
        L.qhuff_encode_batch_host.argtypes = [vp, vp, u32p, C.c_uint32,
                                              C.c_uint, vp, u32p]
        L.qhuff_decode_batch_host.restype = C.c_int
        L.qhuff_decode_batch_host.argtypes = [vp, vp, u32p, C.c_uint32, vp,
                                              u32p, vp]
        L.qhuff_enc_enc_str.restype = C.c_int
        L.qhuff_enc_enc_str.argtypes = [vp, C.c_uint, vp, C.c_size_t,
                                        C.c_char_p, C.c_uint]
        L.qhuff_profile_read.restype = C.c_uint64
        L.qhuff_profile_read.argtypes = [vp, vp, C.c_uint64]
        L.qhuff_enc_str_size.restype = C.c_uint
        L.qhuff_enc_str_size.argtypes = [vp, C.c_char_p, C.c_uint]
        L.qhuff_huff_decode_ex.restype = DecodeRetval
        L.qhuff_huff_decode_ex.argtypes = [vp, vp, C.c_int, vp, C.c_int,
                                           C.POINTER(DecodeState), C.c_int]
        L.qhuff_huff_decode.restype = DecodeRetval
        L.qhuff_huff_decode.argtypes = [vp, vp, C.c_int, vp, C.c_int]
        L.qhuff_abi_version.restype = C.c_int
        L.qhuff_abi_version.argtypes = []
        L.qhuff_lsqpack_enc_enc_str.restype = C.c_int
        L.qhuff_lsqpack_enc_enc_str.argtypes = [C.c_uint, vp, C.c_size_t,
                                                C.c_char_p, C.c_uint]
        L.qhuff_lsqpack_huff_decode.restype = DecodeRetval
        L.qhuff_lsqpack_huff_decode.argtypes = [vp, C.c_int, vp, C.c_int,
                                                C.POINTER(DecodeState),
                                                C.c_int]
        L.qhuff_lsqpack_set_decode_full.restype = None
        L.qhuff_lsqpack_set_decode_full.argtypes = [C.c_void_p]
        L.qhuff_lsqpack_set_context.restype = C.c_int
        L.qhuff_lsqpack_set_context.argtypes = [C.c_void_p]
        L.qhuff_lsqpack_set_device.restype = C.c_int
        L.qhuff_lsqpack_set_device.argtypes = [C.c_int]
        L.qhuff_last_error.restype = C.c_char_p
        L.qhuff_last_error.argtypes = [vp]
        L.qhuff_shard_cuts.restype = C.c_int
        L.qhuff_shard_cuts.argtypes = [u32p, C.c_uint32, C.c_uint32, u32p]
        L.qhuff_device_error.restype = C.c_int
        L.qhuff_device_error.argtypes = [vp]
        L.qhuff_synth_batch.restype = C.c_uint64
        L.qhuff_synth_batch.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32,
                                        C.c_uint32, C.c_char_p, C.c_uint32,
                                        vp, u32p]
        L.qhuff_xxh32_headers.restype = C.c_int
        L.qhuff_xxh32_headers.argtypes = [vp, vp, u32p, C.c_uint32,
                                          C.c_uint32, u32p, u32p, vp]
        L.qhuff_xxh32_batch.restype = C.c_int
        L.qhuff_xxh32_batch.argtypes = [vp, vp, u32p, C.c_uint32, C.c_uint32,
                                        u32p, vp]
        L.qhuff_scan_field_section.restype = C.c_int
        L.qhuff_scan_field_section.argtypes = [C.c_char_p, C.c_size_t,
                                               C.c_uint32, vp, C.c_uint32,
                                               C.POINTER(C.c_uint32)]
        L.qhuff_scan_encoder_stream.restype = C.c_int
        L.qhuff_scan_encoder_stream.argtypes = [
            C.c_char_p, C.c_size_t, C.c_uint32, vp, C.c_uint32,
            C.POINTER(C.c_uint32), C.POINTER(C.c_size_t)]
        L.qhuff_literals_bound.restype = C.c_uint64
        L.qhuff_literals_bound.argtypes = [vp, C.c_uint32]
        L.qhuff_decode_literals_host.restype = C.c_int
        L.qhuff_decode_literals_host.argtypes = [vp, vp, vp, C.c_uint32, vp,
                                                 u32p, vp]
        L.qhuff_decode_literals_ex.restype = C.c_int
        L.qhuff_decode_literals_ex.argtypes = [vp, vp, vp, C.c_uint32,
                                               C.c_uint32, vp, u32p, vp]
        L.qhuff_xxh32_headers_host.restype = C.c_int
        L.qhuff_xxh32_headers_host.argtypes = [vp, vp, u32p, C.c_uint32,
                                               C.c_uint32, u32p, u32p]
        L.qhuff_svc_open.restype = C.c_int
        L.qhuff_svc_open.argtypes = [vp, C.c_uint, C.c_uint,
                                     C.POINTER(C.c_void_p)]
        L.qhuff_svc_close.restype = None
        L.qhuff_svc_close.argtypes = [vp]
        L.qhuff_svc_encode.restype = C.c_int
        L.qhuff_svc_encode.argtypes = [vp, vp, u32p, C.c_uint32, C.c_uint, vp,
                                       u32p]
        L.qhuff_svc_decode.restype = C.c_int
        L.qhuff_svc_decode.argtypes = [vp, vp, u32p, C.c_uint32, vp, u32p, vp]
        L.qhuff_svc_stats.restype = C.c_int
        L.qhuff_svc_stats.argtypes = [vp, C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64),
                                      C.POINTER(C.c_uint64)]
        L.qhuff_timing_enable.restype = C.c_int
        L.qhuff_timing_enable.argtypes = [vp, C.c_int]
        L.qhuff_kernel_variant.restype = C.c_int
        L.qhuff_kernel_variant.argtypes = [vp, C.c_int]
        L.qhuff_batch_hint.restype = C.c_int
        L.qhuff_batch_hint.argtypes = [vp, C.c_int, C.c_int]
        L.qhuff_batch_needs_full.restype = C.c_int
        L.qhuff_batch_needs_full.argtypes = [u32p, C.c_uint32]
        L.qhuff_timing_read.restype = C.c_int
        L.qhuff_timing_read.argtypes = [vp, u32p, C.POINTER(C.c_double),
                                        C.c_uint32]
        L.qhuff_frame_literal.restype = C.c_int
        L.qhuff_frame_literal.argtypes = [C.c_uint, vp, C.c_size_t,
                                          C.c_char_p, C.c_uint, C.c_char_p,
                                          C.c_uint]
        L.qhuff_dec_int.restype = C.c_int
        L.qhuff_dec_int.argtypes = [C.c_char_p, C.c_size_t, C.c_uint,
                                    C.POINTER(C.c_uint64),
                                    C.POINTER(C.c_size_t)]
        L.qhuff_encode_batch_host_multi.restype = C.c_int
        L.qhuff_encode_batch_host_multi.argtypes = [vp, C.c_uint32, vp, u32p,
                                                    C.c_uint32, C.c_uint, vp,
                                                    u32p]
        L.qhuff_decode_batch_host_multi.restype = C.c_int
        L.qhuff_decode_batch_host_multi.argtypes = [vp, C.c_uint32, vp, u32p,
                                                    C.c_uint32, vp, u32p, vp]
        L.qhuff_encode_batch_multi.restype = C.c_int
        L.qhuff_encode_batch_multi.argtypes = [vp, C.c_uint32, vp, C.c_uint,
                                               vp, C.c_int]
        L.qhuff_decode_batch_multi.restype = C.c_int
        L.qhuff_decode_batch_multi.argtypes = [vp, C.c_uint32, vp, vp,
                                               C.c_int]
        L.qhuff_host_register.restype = C.c_int
        L.qhuff_host_register.argtypes = [vp, C.c_size_t]
        L.qhuff_host_unregister.restype = C.c_int
        L.qhuff_host_unregister.argtypes = [vp]
        _lib = L
    return _lib


# ---- host-only helpers (no device needed) ---------------------------------

def encode_bound(in_bytes, n, mode=ENC_PAYLOAD):
    return int(lib().qhuff_encode_bound(in_bytes, n, mode))


def decode_bound(in_bytes, n):
    return int(lib().qhuff_decode_bound(in_bytes, n))


def _np_ptr(a):
    return a.ctypes.data_as(C.c_void_p)


def shard_cuts(in_off, g):
    """Byte-balanced contiguous partition into g shards -> g+1 string
    indices (include/qhuff.h qhuff_shard_cuts)."""
    import numpy as np
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    cuts = np.zeros(g + 1, dtype=np.uint32)
    rc = lib().qhuff_shard_cuts(_np_ptr(in_off), len(in_off) - 1, g,
                                _np_ptr(cuts))
    if rc:
        raise QhuffError("qhuff_shard_cuts: %d" % rc)
    return cuts


def batch_needs_full(in_off):
    """qhuff_batch_needs_full: 1 if host offsets describe a batch the full
    kernel is for (a string > 128 bytes or a tile past the 3 KB stage)."""
    import numpy as np
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    return int(lib().qhuff_batch_needs_full(_np_ptr(in_off), len(in_off) - 1))


def _scan(fn, buf, pos_base, *extra):
    cap = 64
    while True:
        lits = (Literal * cap)()
        n = C.c_uint32()
        rc = fn(buf, len(buf), pos_base, lits, cap, C.byref(n), *extra)
        if rc == ERANGE:
            cap = max(2 * cap, n.value)
            continue
        return rc, list(lits[:n.value])


def scan_field_section(buf, pos_base=0):
    """Literals of one encoded field section -> (rc, [Literal])."""
    return _scan(lib().qhuff_scan_field_section, bytes(buf), pos_base)


def scan_encoder_stream(buf, pos_base=0):
    """Literals of the complete encoder-stream instructions in buf ->
    (rc, [Literal], consumed bytes)."""
    consumed = C.c_size_t()
    rc, lits = _scan(lib().qhuff_scan_encoder_stream, bytes(buf), pos_base,
                     C.byref(consumed))
    return rc, lits, consumed.value


def dec_int(buf, prefix_bits):
    """qhuff_dec_int (the scanners' lsqpack_dec_int, complete buffer) ->
    (rc, value, consumed)."""
    v, used = C.c_uint64(), C.c_size_t()
    rc = lib().qhuff_dec_int(bytes(buf), len(buf), prefix_bits, C.byref(v),
                             C.byref(used))
    return rc, (v.value if rc == OK else None), (used.value if rc == OK else 0)


def frame_literal(prefix_bits, s, huff, first_byte=0, dst_len=1 << 16):
    """lsqpack_enc_enc_str framing of s given its precomputed Huffman
    payload (include/qhuff.h qhuff_frame_literal) -> bytes or -1."""
    buf = C.create_string_buffer(max(dst_len, 1))
    buf[0] = first_byte
    r = lib().qhuff_frame_literal(prefix_bits, buf, dst_len, s, len(s), huff,
                                  len(huff))
    return r if r < 0 else buf.raw[:r]


TOKEN_ALPHABET = b"abcdefghijklmnopqrstuvwxyz0123456789-_./:;=, "
BASE64_ALPHABET = (b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
                   b"0123456789+/")


def synth_batch(n, seed=0, min_len=8, max_len=64, alphabet=TOKEN_ALPHABET):
    """Synthetic header strings: returns (data uint8,
    in_off uint32[n+1]) numpy arrays."""
    import numpy as np
    data = np.zeros(max(n * max_len, 1), dtype=np.uint8)
    off = np.zeros(n + 1, dtype=np.uint32)
    tot = lib().qhuff_synth_batch(seed, n, min_len, max_len, alphabet,
                                  len(alphabet), _np_ptr(data), _np_ptr(off))
    return data[:tot].copy(), off


# ---- exact-signature shims (include/qhuff_lsqpack.h) -------------------------

def lsqpack_enc_enc_str(prefix_bits, s, first_byte=0, dst_len=1 << 16):
    """qhuff_lsqpack_enc_enc_str -> bytes or -1 (thread's default context)."""
    buf = C.create_string_buffer(max(dst_len, 1))
    buf[0] = first_byte
    r = lib().qhuff_lsqpack_enc_enc_str(prefix_bits, buf, dst_len, s, len(s))
    return r if r < 0 else buf.raw[:r]


def lsqpack_huff_decode(src, dst_len, state=None, final=1):
    """qhuff_lsqpack_huff_decode -> (status, dst[:n_dst], n_dst, n_src,
    state)."""
    s = C.create_string_buffer(bytes(src), len(src) + 1)
    d = C.create_string_buffer(max(dst_len, 1))
    st = state if state is not None else DecodeState(0, 0, 0)
    rv = lib().qhuff_lsqpack_huff_decode(s, len(src), d, dst_len, C.byref(st),
                                         final)
    return rv.status, d.raw[:rv.n_dst], rv.n_dst, rv.n_src, st


def lsqpack_set_decode_full(fn):
    """Register the streaming decoder (a DECODE_FULL_FN or None); returns
    the ctypes callback object, which the caller must keep alive."""
    cb = fn if fn is None or isinstance(fn, DECODE_FULL_FN) else DECODE_FULL_FN(fn)
    lib().qhuff_lsqpack_set_decode_full(
        C.cast(cb, C.c_void_p) if cb is not None else None)
    return cb


# ---- one batch over several contexts (qhuff_*_batch_*multi) ---------------

def _ctx_array(codecs):
    arr = (C.c_void_p * len(codecs))(*[c._ctx.value for c in codecs])
    return arr


def host_register(arr):
    """qhuff_host_register over a contiguous numpy array: the host-memory
    calls then move it by DMA directly (no staging copy) -> rc."""
    assert arr.flags["C_CONTIGUOUS"]
    return int(lib().qhuff_host_register(_np_ptr(arr), arr.nbytes))


def host_unregister(arr):
    return int(lib().qhuff_host_unregister(_np_ptr(arr)))


class registered:
    """with registered(a, b, ...): the arrays are registered for direct DMA
    inside the block (raises QhuffError if a registration fails)."""

    def __init__(self, *arrays):
        self.arrays = arrays
        self.done = []

    def __enter__(self):
        for a in self.arrays:
            rc = host_register(a)
            if rc:
                self.__exit__()
                raise QhuffError("qhuff_host_register: %d %s"
                                 % (rc, lib().qhuff_last_error(None).decode()))
            self.done.append(a)
        return self

    def __exit__(self, *exc):
        while self.done:
            host_unregister(self.done.pop())
        return False


def encode_host_multi(codecs, data, in_off, mode=ENC_PAYLOAD):
    """qhuff_encode_batch_host_multi: host batch sharded over the contexts
    -> (out bytes, global out_off)."""
    import numpy as np
    data = np.ascontiguousarray(data, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    n = len(in_off) - 1
    out = np.zeros(encode_bound(int(in_off[-1] - in_off[0]), n, mode),
                   dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    rc = lib().qhuff_encode_batch_host_multi(
        _ctx_array(codecs), len(codecs), _np_ptr(data), _np_ptr(in_off), n,
        mode, _np_ptr(out), _np_ptr(out_off))
    if rc:
        raise QhuffError("qhuff_encode_batch_host_multi: %d" % rc)
    return out[:out_off[-1]], out_off


def decode_host_multi(codecs, data, in_off):
    """qhuff_decode_batch_host_multi -> (out bytes, out_off, status)."""
    import numpy as np
    data = np.ascontiguousarray(data, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    n = len(in_off) - 1
    out = np.zeros(decode_bound(int(in_off[-1] - in_off[0]), n),
                   dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    rc = lib().qhuff_decode_batch_host_multi(
        _ctx_array(codecs), len(codecs), _np_ptr(data), _np_ptr(in_off), n,
        _np_ptr(out), _np_ptr(out_off), _np_ptr(status))
    if rc:
        raise QhuffError("qhuff_decode_batch_host_multi: %d" % rc)
    return out[:out_off[-1]], out_off, status[:n]


def batch_multi(codecs, shards, encode, mode=ENC_PAYLOAD, rebase=True):
    """qhuff_encode_batch_multi / qhuff_decode_batch_multi over
    device-resident shards: shards[k] = dict(in_, in_off, n, out, out_off,
    status, stream) of torch tensors / ints (stream: a torch stream or
    None) -> base list (g + 1 entries)."""
    g = len(codecs)
    arr = (Shard * g)()
    for k, s in enumerate(shards):
        st = s.get("stream")
        arr[k] = Shard(s["in_"].data_ptr(), s["in_off"].data_ptr(), s["n"],
                       s["out"].data_ptr(), s["out_off"].data_ptr(),
                       s["status"].data_ptr() if s.get("status") is not None
                       else None,
                       st.cuda_stream if st is not None else None)
    base = (C.c_uint64 * (g + 1))()
    if encode:
        rc = lib().qhuff_encode_batch_multi(_ctx_array(codecs), g, arr, mode,
                                            base, int(rebase))
    else:
        rc = lib().qhuff_decode_batch_multi(_ctx_array(codecs), g, arr, base,
                                            int(rebase))
    if rc:
        raise QhuffError("qhuff_%s_batch_multi: %d"
                         % ("encode" if encode else "decode", rc))
    return list(base)


# ---- device codec ----------------------------------------------------------

class Codec:
    """One qhuff_ctx on one GPU.  Tensor arguments are torch CUDA(HIP)
    tensors; offsets are int32 tensors reinterpreted as uint32."""

    def __init__(self, device=0):
        self._ctx = C.c_void_p()
        rc = lib().qhuff_open(device, C.byref(self._ctx))
        if rc != OK:
            raise QhuffError("qhuff_open(device=%d) failed: %d (%s)" % (
                device, rc, lib().qhuff_last_error(None).decode()))
        self.device = device

    def close(self):
        if self._ctx:
            svc = getattr(self, "_service", None)
            if svc is not None:
                svc._svc = C.c_void_p()      # qhuff_close frees it
            lib().qhuff_close(self._ctx)
            self._ctx = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def profile_read(self):
        """Phase stamps of the last launch (QHUFF_PROFILE build), as a
        numpy uint64 array, or None in a normal build."""
        import numpy as np
        n = lib().qhuff_profile_read(self._ctx, None, 0)
        if not n:
            return None
        a = np.zeros(n, dtype=np.uint64)
        lib().qhuff_profile_read(self._ctx, a.ctypes.data, n)
        return a

    def device_error(self):
        """Synchronise and return (then clear) the sticky device error word
        (0 = none, 1 = a look-back wait gave up)."""
        return int(lib().qhuff_device_error(self._ctx))

    def timing(self, on=True, every=1):
        """qhuff_timing_enable: time every later launch of this context (or
        every `every`-th of each kind) by its dispatch's own start / stop
        timestamps."""
        self._check(lib().qhuff_timing_enable(
            self._ctx, max(1, int(every)) if on else 0), "qhuff_timing_enable")

    def kernel_variant(self, kind):
        """qhuff_kernel_variant: 1 if the last launch of kind (KIND_ENCODE /
        KIND_DECODE) ran the full kernel, 0 for the lean one."""
        r = lib().qhuff_kernel_variant(self._ctx, kind)
        if r < 0:
            self._check(r, "qhuff_kernel_variant")
        return r

    def batch_hint(self, kind, hint):
        """qhuff_batch_hint: the next launch of kind runs the full (1) or
        lean (0) kernel, or no hint (-1: the full kernel)."""
        self._check(lib().qhuff_batch_hint(self._ctx, kind, hint),
                    "qhuff_batch_hint")

    def timing_read(self, max_launches=TIMING_SLOTS):
        """qhuff_timing_read -> list of (kind, microseconds) of the launches
        timed since timing() or the last read, oldest first (KIND_*)."""
        kinds = (C.c_uint32 * max_launches)()
        us = (C.c_double * max_launches)()
        n = lib().qhuff_timing_read(self._ctx, kinds, us, max_launches)
        if n < 0:
            self._check(n, "qhuff_timing_read")
        return [(int(kinds[i]), float(us[i])) for i in range(n)]

    def _check(self, rc, what):
        if rc != OK:
            err = lib().qhuff_last_error(self._ctx)
            raise QhuffError("%s failed: %d (%s)" % (what, rc,
                             err.decode() if err else ""))

    @staticmethod
    def _stream(stream):
        if stream is None:
            import torch
            stream = torch.cuda.current_stream()
        return C.c_void_p(stream.cuda_stream)

    # device-resident batch calls ------------------------------------------
    def encode_into(self, data, in_off, n, mode, out, out_off, stream=None):
        rc = lib().qhuff_encode_batch(self._ctx, data.data_ptr(),
                                      in_off.data_ptr(), n, mode,
                                      out.data_ptr(), out_off.data_ptr(),
                                      self._stream(stream))
        self._check(rc, "qhuff_encode_batch")

    def decode_into(self, data, in_off, n, out, out_off, status, stream=None):
        rc = lib().qhuff_decode_batch(self._ctx, data.data_ptr(),
                                      in_off.data_ptr(), n, out.data_ptr(),
                                      out_off.data_ptr(), status.data_ptr(),
                                      self._stream(stream))
        self._check(rc, "qhuff_decode_batch")

    def encode(self, data, in_off, mode=ENC_PAYLOAD, stream=None):
        """data: uint8 cuda tensor, in_off: int32 cuda tensor [n+1].
        Returns (out uint8 [bound], out_off int32 [n+1])."""
        import torch
        n = in_off.numel() - 1
        in_bytes = int(data.numel())
        out = torch.empty(encode_bound(in_bytes, n, mode), dtype=torch.uint8,
                          device=data.device)
        out_off = torch.empty(n + 1, dtype=torch.int32, device=data.device)
        self.encode_into(data, in_off, n, mode, out, out_off, stream)
        return out, out_off

    def decode(self, data, in_off, stream=None):
        import torch
        n = in_off.numel() - 1
        out = torch.empty(decode_bound(int(data.numel()), n),
                          dtype=torch.uint8, device=data.device)
        out_off = torch.empty(n + 1, dtype=torch.int32, device=data.device)
        status = torch.empty(max(n, 1), dtype=torch.uint8, device=data.device)
        self.decode_into(data, in_off, n, out, out_off, status, stream)
        return out, out_off, status[:n]

    # header hashing (XXH32, lsqpack.c:1681-1685) ---------------------------
    def xxh32_headers_into(self, data, off, n, seed, name_hash, nameval_hash,
                           stream=None):
        rc = lib().qhuff_xxh32_headers(self._ctx, data.data_ptr(),
                                       off.data_ptr(), n, seed,
                                       name_hash.data_ptr(),
                                       nameval_hash.data_ptr(),
                                       self._stream(stream))
        self._check(rc, "qhuff_xxh32_headers")

    def xxh32_headers(self, data, off, seed=XXH_SEED, stream=None):
        """off: int32 cuda tensor [2n+1] (name, value, name, value ...).
        Returns (name_hash, nameval_hash) int32 tensors [n] (uint32 bits)."""
        import torch
        n = (off.numel() - 1) // 2
        h1 = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        h2 = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        self.xxh32_headers_into(data, off, n, seed & 0xffffffff, h1, h2,
                                stream)
        return h1[:n], h2[:n]

    def xxh32_headers_host(self, data, off, seed=XXH_SEED):
        """Host numpy buffers -> (name_hash, nameval_hash) uint32[n]."""
        import numpy as np
        data = np.ascontiguousarray(data, dtype=np.uint8)
        off = np.ascontiguousarray(off, dtype=np.uint32)
        n = (len(off) - 1) // 2
        h1 = np.zeros(max(n, 1), dtype=np.uint32)
        h2 = np.zeros(max(n, 1), dtype=np.uint32)
        rc = lib().qhuff_xxh32_headers_host(self._ctx, _np_ptr(data),
                                            _np_ptr(off), n, seed & 0xffffffff,
                                            _np_ptr(h1), _np_ptr(h2))
        self._check(rc, "qhuff_xxh32_headers_host")
        return h1[:n], h2[:n]

    def xxh32(self, data, in_off, seed=XXH_SEED, stream=None):
        """hash[i] = XXH32(string i, seed); int32 tensor [n]."""
        import torch
        n = in_off.numel() - 1
        h = torch.empty(max(n, 1), dtype=torch.int32, device=data.device)
        rc = lib().qhuff_xxh32_batch(self._ctx, data.data_ptr(),
                                     in_off.data_ptr(), n, seed & 0xffffffff,
                                     h.data_ptr(), self._stream(stream))
        self._check(rc, "qhuff_xxh32_batch")
        return h[:n]

    # host-memory batch calls (numpy) ----------------------------------------
    def encode_host(self, data, in_off, mode=ENC_PAYLOAD, out=None,
                    out_off=None):
        """Host buffers in and out (PCIe-inclusive path).  out / out_off may
        be given (reused, already faulted-in buffers of the bound size)."""
        import numpy as np
        data = np.ascontiguousarray(data, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
        n = len(in_off) - 1
        if out is None:
            out = np.zeros(encode_bound(int(in_off[-1] - in_off[0]), n, mode),
                           dtype=np.uint8)
        if out_off is None:
            out_off = np.zeros(n + 1, dtype=np.uint32)
        rc = lib().qhuff_encode_batch_host(self._ctx, _np_ptr(data),
                                           _np_ptr(in_off), n, mode,
                                           _np_ptr(out), _np_ptr(out_off))
        self._check(rc, "qhuff_encode_batch_host")
        return out[:out_off[-1]], out_off

    def decode_host(self, data, in_off, out=None, out_off=None, status=None):
        import numpy as np
        data = np.ascontiguousarray(data, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
        n = len(in_off) - 1
        if out is None:
            out = np.zeros(decode_bound(int(in_off[-1] - in_off[0]), n),
                           dtype=np.uint8)
        if out_off is None:
            out_off = np.zeros(n + 1, dtype=np.uint32)
        if status is None:
            status = np.zeros(max(n, 1), dtype=np.uint8)
        rc = lib().qhuff_decode_batch_host(self._ctx, _np_ptr(data),
                                           _np_ptr(in_off), n, _np_ptr(out),
                                           _np_ptr(out_off), _np_ptr(status))
        self._check(rc, "qhuff_decode_batch_host")
        return out[:out_off[-1]], out_off, status[:n]

    def decode_literals_host(self, buf, lits, max_len=None):
        """Decode pre-parsed literals of host buffer buf in one GPU batch ->
        (list of bytes, status uint8 ndarray).  max_len (e.g. MAX_STRLEN for
        field-section literals) calls qhuff_decode_literals_ex: a literal
        longer than it once decoded is an ERROR."""
        import numpy as np
        n = len(lits)
        arr = (Literal * max(n, 1))(*lits)
        src = np.frombuffer(bytes(buf) + b"\0", dtype=np.uint8)
        cap = int(lib().qhuff_literals_bound(arr, n))
        out = np.zeros(cap, dtype=np.uint8)
        out_off = np.zeros(n + 1, dtype=np.uint32)
        status = np.zeros(max(n, 1), dtype=np.uint8)
        if max_len is None:
            rc = lib().qhuff_decode_literals_host(
                self._ctx, _np_ptr(src), arr, n, _np_ptr(out), _np_ptr(out_off),
                _np_ptr(status))
        else:
            rc = lib().qhuff_decode_literals_ex(
                self._ctx, _np_ptr(src), arr, n, max_len, _np_ptr(out),
                _np_ptr(out_off), _np_ptr(status))
        self._check(rc, "qhuff_decode_literals_host")
        return ([out[out_off[i]:out_off[i + 1]].tobytes() for i in range(n)],
                status[:n])

    def service(self, slots=0, idle_us=0):
        """Attach the low-latency service (qhuff_svc_open) -> Service."""
        self._service = Service(self, slots, idle_us)
        return self._service

    # per-string mirrors of the reference entry points ----------------------
    def enc_enc_str(self, prefix_bits, s, first_byte=0, dst_len=1 << 20):
        buf = C.create_string_buffer(max(dst_len, 1))
        buf[0] = first_byte
        r = lib().qhuff_enc_enc_str(self._ctx, prefix_bits, buf, dst_len, s,
                                    len(s))
        return r if r < 0 else buf.raw[:r]

    def enc_str_size(self, s):
        return int(lib().qhuff_enc_str_size(self._ctx, s, len(s)))

    def huff_decode(self, src, dst_len=None, state=None, final=1):
        """qhuff_huff_decode_ex (lsqpack_huff_decode's arguments on this
        context) -> (status, dst bytes [:n_dst], n_src)."""
        if dst_len is None:
            dst_len = len(src) * 8 // 5 + 1
        s = C.create_string_buffer(bytes(src), len(src) + 1)
        d = C.create_string_buffer(max(dst_len, 1))
        st = state if state is not None else DecodeState(0, 0, 0)
        rv = lib().qhuff_huff_decode_ex(self._ctx, s, len(src), d, dst_len,
                                        C.byref(st), final)
        return rv.status, d.raw[:rv.n_dst], rv.n_src


class Service:
    """The resident low-latency service on a Codec's context (qhuff_svc_*):
    small host-memory batches without a kernel launch per call.  While it is
    open, the context's own host-path calls that fit a slot use it too."""

    def __init__(self, codec, slots=0, idle_us=0):
        self.codec = codec                   # keeps the context alive
        self._svc = C.c_void_p()
        rc = lib().qhuff_svc_open(codec._ctx, slots, idle_us,
                                  C.byref(self._svc))
        if rc != OK:
            err = lib().qhuff_last_error(codec._ctx)
            raise QhuffError("qhuff_svc_open failed: %d (%s)" % (
                rc, err.decode() if err else ""))

    def close(self):
        if self._svc:
            lib().qhuff_svc_close(self._svc)
            self._svc = C.c_void_p()
        if getattr(self.codec, "_service", None) is self:
            self.codec._service = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def _check(self, rc, what):
        if rc != OK:
            err = lib().qhuff_last_error(self.codec._ctx)
            raise QhuffError("%s failed: %d (%s)" % (what, rc,
                             err.decode() if err else ""))

    def stats(self):
        """(calls served by the kernel, kernel launches, calls sent to the
        host path)"""
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        self._check(lib().qhuff_svc_stats(self._svc, C.byref(a), C.byref(b),
                                          C.byref(c)), "qhuff_svc_stats")
        return a.value, b.value, c.value

    def encode(self, data, in_off, mode=ENC_PAYLOAD, out=None, out_off=None):
        import numpy as np
        data = np.ascontiguousarray(data, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
        n = len(in_off) - 1
        if out is None:
            out = np.zeros(encode_bound(int(in_off[-1] - in_off[0]), n, mode),
                           dtype=np.uint8)
        if out_off is None:
            out_off = np.zeros(n + 1, dtype=np.uint32)
        self._check(lib().qhuff_svc_encode(self._svc, _np_ptr(data),
                                           _np_ptr(in_off), n, mode,
                                           _np_ptr(out), _np_ptr(out_off)),
                    "qhuff_svc_encode")
        return out[:out_off[-1]], out_off

    def decode(self, data, in_off, out=None, out_off=None, status=None):
        import numpy as np
        data = np.ascontiguousarray(data, dtype=np.uint8)
        in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
        n = len(in_off) - 1
        if out is None:
            out = np.zeros(decode_bound(int(in_off[-1] - in_off[0]), n),
                           dtype=np.uint8)
        if out_off is None:
            out_off = np.zeros(n + 1, dtype=np.uint32)
        if status is None:
            status = np.zeros(max(n, 1), dtype=np.uint8)
        self._check(lib().qhuff_svc_decode(self._svc, _np_ptr(data),
                                           _np_ptr(in_off), n, _np_ptr(out),
                                           _np_ptr(out_off), _np_ptr(status)),
                    "qhuff_svc_decode")
        return out[:out_off[-1]], out_off, status[:n]

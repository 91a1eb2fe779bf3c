"""ctypes view of the CPU oracle (oracle/qhuff_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "libqhuff_oracle.so")

OK, END_SRC, END_DST, ERROR = 0, 1, 2, 3


class RetVal(C.Structure):
    _fields_ = [("status", C.c_int), ("n_dst", C.c_uint), ("n_src", C.c_uint)]


class DecState(C.Structure):
    _fields_ = [("resume", C.c_int), ("state", C.c_uint8), ("eos", C.c_uint8)]


def build():
    srcs = [os.path.join(ORACLE_DIR, f)
            for f in ("qhuff_oracle.c", "xxh32_oracle.c")]
    if (not os.path.exists(ORACLE_SO) or os.path.getmtime(ORACLE_SO)
            < max(os.path.getmtime(s) for s in srcs)):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return ORACLE_SO


_lib = None


def lib():
    global _lib
    if _lib is None:
        # QHUFF_ORACLE_LIB: another build of the same oracle (the
        # sanitizer run, tests/test_sanitize.py)
        L = C.CDLL(os.environ.get("QHUFF_ORACLE_LIB") or build())
        u8p = C.POINTER(C.c_uint8)
        L.oq_enc_str_size.restype = C.c_uint
        L.oq_enc_str_size.argtypes = [C.c_char_p, C.c_uint]
        L.oq_huffman_enc.restype = C.c_void_p
        L.oq_huffman_enc.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p]
        L.oq_enc_enc_str.restype = C.c_int
        L.oq_enc_enc_str.argtypes = [C.c_uint, C.c_void_p, C.c_size_t,
                                     C.c_char_p, C.c_uint]
        for fn in (L.oq_huff_decode, L.oq_huff_decode_full):
            fn.restype = RetVal
            fn.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_int,
                           C.POINTER(DecState), C.c_int]
        L.oq_encode_sizes.restype = C.c_ulonglong
        L.oq_encode_sizes.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_uint, C.c_void_p]
        L.oq_encode_batch.restype = None
        L.oq_encode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_uint, C.c_void_p, C.c_void_p]
        L.oq_decode_batch.restype = C.c_int
        L.oq_decode_batch.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                      C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_int]
        L.oq_bench_pass.restype = C.c_double
        L.oq_bench_pass.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                    C.c_int, C.c_int, C.c_uint,
                                    C.POINTER(C.c_ulonglong)]
        L.oq_code_of.restype = None
        L.oq_code_of.argtypes = [C.c_uint, C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint)]
        L.oq_xxh32.restype = C.c_uint32
        L.oq_xxh32.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32]
        L.oq_xxh32_headers.restype = None
        L.oq_xxh32_headers.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32,
                                       C.c_uint32, C.c_void_p, C.c_void_p]
        _lib = L
    return _lib


XXH_SEED = 39378473                       # LSQPACK_XXH_SEED, lsqpack.c:623


def xxh32(s: bytes, seed: int = XXH_SEED) -> int:
    return lib().oq_xxh32(s, len(s), seed & 0xffffffff)


def xxh32_headers(data: np.ndarray, off: np.ndarray, seed: int = XXH_SEED):
    """off[2n+1] (name, value, ...) -> (name_hash, nameval_hash) uint32[n]."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint32)
    n = (len(off) - 1) // 2
    h1 = np.zeros(max(n, 1), dtype=np.uint32)
    h2 = np.zeros(max(n, 1), dtype=np.uint32)
    lib().oq_xxh32_headers(_p(data), _p(off), n, seed & 0xffffffff, _p(h1),
                           _p(h2))
    return h1[:n], h2[:n]


# ---- per-string helpers --------------------------------------------------

def code_of(sym):
    c, b = C.c_uint32(), C.c_uint()
    lib().oq_code_of(sym, C.byref(c), C.byref(b))
    return c.value, b.value


def enc_str_size(s: bytes) -> int:
    return lib().oq_enc_str_size(s, len(s))


def huffman_enc(s: bytes) -> bytes:
    """qenc_huffman_enc output (forced Huffman, no framing)."""
    n = enc_str_size(s)
    buf = C.create_string_buffer(n + 16)
    src = C.create_string_buffer(s, len(s) + 16)
    base = C.addressof(src)
    end = lib().oq_huffman_enc(src, base + len(s), buf)
    assert end - C.addressof(buf) == n
    return buf.raw[:n]


def enc_enc_str(prefix_bits: int, s: bytes, first_byte: int = 0,
                dst_len: int = 1 << 20):
    """lsqpack_enc_enc_str(prefix_bits, dst, dst_len, s, len(s)) with
    dst[0] preset to first_byte.  Returns bytes or -1."""
    buf = C.create_string_buffer(max(dst_len, 1))
    buf[0] = first_byte
    r = lib().oq_enc_enc_str(prefix_bits, buf, dst_len, s, len(s))
    return r if r < 0 else buf.raw[:r]


def huff_decode(src: bytes, full=False, dst_len=None):
    """Complete-string decode (resume 0, final 1).  Returns (status, bytes)."""
    if dst_len is None:
        dst_len = len(src) * 8 // 5 + 1
    s = C.create_string_buffer(src, len(src) + 1)
    d = C.create_string_buffer(max(dst_len, 1))
    st = DecState(0, 0, 0)
    fn = lib().oq_huff_decode_full if full else lib().oq_huff_decode
    rv = fn(s, len(src), d, dst_len, C.byref(st), 1)
    return rv.status, d.raw[:rv.n_dst] if rv.status == OK else b""


def huff_decode_chunked(src: bytes, in_chunk: int, out_chunk: int,
                        out_cap: int = 0x1000):
    """Streaming use of the resumable nibble decoder, the way
    test/test_huff_dec.c:318-371 drives lsqpack_huff_decode_full."""
    out = C.create_string_buffer(out_cap)
    sb = C.create_string_buffer(src, len(src) + 1)
    base_in, base_out = C.addressof(sb), C.addressof(out)
    st = DecState(0, 0, 0)
    in_off = out_off = 0
    n_read = min(len(src), in_chunk)
    n_write = min(out_cap, out_chunk)
    while True:
        rv = lib().oq_huff_decode_full(base_in + in_off, n_read,
                                       base_out + out_off, n_write,
                                       C.byref(st),
                                       int(len(src) == in_off + n_read))
        if rv.status == ERROR:
            return ERROR, b""
        in_off += rv.n_src
        out_off += rv.n_dst
        if rv.status == OK:
            return OK, out.raw[:out_off]
        n_write = min(out_cap - out_off, out_chunk)
        n_read = min(len(src) - in_off, in_chunk)
        if in_off >= len(src) and rv.status == END_SRC:
            return rv.status, out.raw[:out_off]


# ---- batch helpers (numpy) ------------------------------------------------

def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def encode_batch(data: np.ndarray, in_off: np.ndarray, mode: int = 0):
    """Returns (out bytes ndarray, out_off ndarray[n+1])."""
    n = len(in_off) - 1
    data = np.ascontiguousarray(data, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    tot = lib().oq_encode_sizes(_p(data), _p(in_off), n, mode, _p(out_off))
    out = np.zeros(max(int(tot), 1), dtype=np.uint8)
    lib().oq_encode_batch(_p(data), _p(in_off), n, mode, _p(out), _p(out_off))
    return out[:tot], out_off


def decode_batch(data: np.ndarray, in_off: np.ndarray, full=False):
    """Returns (out bytes ndarray, out_off[n+1], status[n])."""
    n = len(in_off) - 1
    data = np.ascontiguousarray(data, dtype=np.uint8)
    in_off = np.ascontiguousarray(in_off, dtype=np.uint32)
    cap = int(in_off[-1]) * 8 // 5 + n + 16
    out = np.zeros(cap, dtype=np.uint8)
    out_off = np.zeros(n + 1, dtype=np.uint32)
    status = np.zeros(max(n, 1), dtype=np.uint8)
    lib().oq_decode_batch(_p(data), _p(in_off), n, _p(out), _p(out_off),
                          _p(status), int(full))
    return out[:out_off[-1]], out_off, status[:n]


def bench_pass(data, in_off, op, nthreads, slot_bytes=128):
    """op 0: enc_enc_str(7,...), 1: huff_decode (fast), 2: _full."""
    sink = C.c_ulonglong()
    return lib().oq_bench_pass(_p(data), _p(in_off), len(in_off) - 1, op,
                               nthreads, slot_bytes, C.byref(sink))


def decoded_prefix(src: bytes):
    """(symbols, eos): the symbols of src decoded before its error -- every
    whole code before the EOS code, or before padding that cannot complete
    one -- and whether the error is the EOS code.  A bit-level greedy decode
    over the oracle's code table (test-side; what the GPU's Keep kernel
    returns for a rejected string)."""
    codes = {}
    for s in range(257):
        c, n = code_of(s)
        codes[(n, c)] = s
    bits = "".join(format(b, "08b") for b in src)
    out, i = [], 0
    while True:
        for L in range(5, 31):
            if i + L > len(bits):
                return bytes(out), False
            sym = codes.get((L, int(bits[i:i + L], 2)))
            if sym is not None:
                break
        if sym == 256:
            return bytes(out), True
        out.append(sym)
        i += L

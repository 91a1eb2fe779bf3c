"""CPU-side checks of the product boundary: libqhuff.so builds for gfx950,
loads, exports every entry point include/qhuff.h declares, and its host-only
helpers behave.  No kernel is launched here (no GPU in the build container)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import _paths  # noqa: F401
from _paths import ROOT
import qhuff


def header_functions():
    names = set()
    for h in qhuff.HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        text = re.sub(r"typedef[^;]*;", "", text)   # function-pointer types
        names |= set(re.findall(r"\b(qhuff_\w+)\s*\(", text))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    lib = qhuff.lib()
    declared = header_functions()
    assert len(declared) >= 14
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(qhuff.EXPORTS) == declared
    out = subprocess.check_output(["nm", "-D", "--defined-only",
                                   qhuff.LIB_PATH]).decode()
    exported = set(re.findall(r" T (qhuff_\w+)", out))
    assert set(declared) <= exported


def test_library_has_gfx950_code_object():
    blob = open(qhuff.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_header_is_plain_c():
    """The boundary headers must compile as C99 with no HIP/torch types."""
    src = "".join('#include "%s"\n' % h for h in qhuff.HEADERS) + \
        "int main(void){return QHUFF_ABI_VERSION != 7;}\n"
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-x", "c",
                        "-fsyntax-only", "-"], input=src, text=True,
                       capture_output=True)
    assert r.returncode == 0, r.stderr


def test_open_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    ctx = C.c_void_p()
    rc = qhuff.lib().qhuff_open(0, C.byref(ctx))
    assert rc == qhuff.ENODEV and not ctx.value
    with pytest.raises(qhuff.QhuffError):
        qhuff.Codec(0)


def test_bounds():
    assert qhuff.decode_bound(5, 1) >= 8
    for n in (1, 10, 1000):
        # 30-bit code per byte
        assert qhuff.encode_bound(64 * n, n, 0) >= (64 * n * 30 + 7) // 8
        assert qhuff.encode_bound(64 * n, n, 7) >= qhuff.encode_bound(64 * n, n, 0)


def xorshift(x):
    x ^= (x << 13) & 0xFFFFFFFFFFFFFFFF
    x ^= x >> 7
    x ^= (x << 17) & 0xFFFFFFFFFFFFFFFF
    return x


def test_synth_batch_matches_generator_spec():
    """xorshift64, seed 0x9E3779B97F4A7C15, len = 8 + r % 57,
    bytes alphabet[r % |alphabet|]."""
    data, off = qhuff.synth_batch(200)
    x = 0x9E3779B97F4A7C15
    a = qhuff.TOKEN_ALPHABET
    pos = 0
    for i in range(200):
        x = xorshift(x)
        ln = 8 + x % 57
        assert off[i] == pos and off[i + 1] - off[i] == ln
        for k in range(ln):
            x = xorshift(x)
            assert data[pos] == a[x % len(a)]
            pos += 1
    assert off[200] == pos == len(data)


def test_shard_cuts_balance():
    data, off = qhuff.synth_batch(10000, seed=3)
    for g in (1, 2, 3, 4, 8):
        cuts = qhuff.shard_cuts(off, g)
        assert cuts[0] == 0 and cuts[-1] == 10000
        assert np.all(np.diff(cuts.astype(np.int64)) >= 0)
        sizes = [int(off[cuts[k + 1]]) - int(off[cuts[k]]) for k in range(g)]
        assert sum(sizes) == len(data)
        assert max(sizes) - min(sizes) <= 2 * 64
    # degenerate: more shards than strings, empty batch
    off3 = np.array([0, 5, 9, 20], dtype=np.uint32)
    cuts = qhuff.shard_cuts(off3, 8)
    assert cuts[0] == 0 and cuts[-1] == 3 and np.all(np.diff(cuts.astype(int)) >= 0)
    cuts = qhuff.shard_cuts(np.array([0], dtype=np.uint32), 4)
    assert list(cuts) == [0, 0, 0, 0, 0]


def test_abi_version_matches_header():
    """the loaded library reports the header's QHUFF_ABI_VERSION (no device
    needed); ABI 2 kept version 1's 5-argument qhuff_huff_decode beside
    qhuff_huff_decode_ex; ABI 3 adds the qhuff_svc_* service
    and keeps every earlier entry point"""
    assert qhuff.lib().qhuff_abi_version() == 7
    src = open(os.path.join(ROOT, "include", "qhuff.h")).read()
    assert "#define QHUFF_ABI_VERSION 7" in src
    assert "qhuff_huff_decode(qhuff_ctx *ctx, const unsigned char *src, " \
           "int src_len,\n                  unsigned char *dst, int dst_len);" \
        in src


def test_service_entry_points_reject_null():
    """qhuff_svc_* with no context / service: QHUFF_EINVAL, no device touched"""
    L = qhuff.lib()
    p = C.c_void_p()
    assert L.qhuff_svc_open(None, 0, 0, C.byref(p)) == qhuff.EINVAL
    assert not p.value
    assert L.qhuff_svc_encode(None, None, None, 0, 0, None, None) == qhuff.EINVAL
    assert L.qhuff_svc_decode(None, None, None, 0, None, None, None) == \
        qhuff.EINVAL
    assert L.qhuff_svc_stats(None, None, None, None) == qhuff.EINVAL
    L.qhuff_svc_close(None)

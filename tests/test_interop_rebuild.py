"""Configs 1 and 5 through the reference's own fixtures.

The reference's interop round trip (bin/interop-encode.c:120-246, driving
lsqpack_enc_encode, lsqpack.c:1983-2119) cannot run here: lsqpack.c needs
huff-tables.h, which the reference mount lacks.  Its committed outputs can:
each tests/golden/data/{netbsd,fb-req,fb-resp}.out.256.100.1 is rebuilt end
to end on the GPU --

  1. every frame is scanned for string literals (qhuff_scan_field_section /
     qhuff_scan_encoder_stream, host framing walk);
  2. ALL literals of the file are decoded in one launch
     (qhuff_decode_literals_host);
  3. the decoded strings are re-encoded by the DEVICE literal modes
     (QHUFF_ENC_LITERAL3/5/7 = lsqpack_enc_enc_str(3/5/7, ...)), one launch
     per prefix width;
  4. each literal's wire bytes are blanked in a copy of the file, and the
     device output is spliced back with the instruction bits above the H bit
     OR-ed into its first byte --

and the result must be the reference's file, byte for byte.
"""
import os

import numpy as np
import pytest

import _paths  # noqa: F401
import qpack_frames as Q

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                    "data")


def scan_file(qhuff, buf):
    """All literals of an interop file, positions relative to the file."""
    lits, pos = [], 0
    for sid, fr in Q.read_interop(buf):
        base = pos + 12
        if sid == 0:
            rc, ls, used = qhuff.scan_encoder_stream(fr, base)
            assert rc == qhuff.OK and used == len(fr)
        else:
            rc, ls = qhuff.scan_field_section(fr, base)
            assert rc == qhuff.OK
        lits += ls
        pos = base + len(fr)
    assert pos == len(buf)
    return lits


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["netbsd", "fb-req", "fb-resp"])
def test_rebuild_interop_stream_with_device_literal_modes(name):
    import torch
    import qhuff
    buf = open(os.path.join(DATA, name + ".out.256.100.1"), "rb").read()
    codec = qhuff.Codec(0)
    lits = scan_file(qhuff, buf)
    assert len(lits) > 50

    strs, status = codec.decode_literals_host(buf, lits)     # one launch
    assert not status.any()

    out = bytearray(buf)
    for lt in lits:                                  # blank every literal
        out[lt.pos - lt.hdr_len:lt.pos + lt.len] = bytes(lt.hdr_len + lt.len)
    spliced = 0
    for p in (3, 5, 7):
        idx = [i for i, lt in enumerate(lits) if lt.prefix_bits == p]
        if not idx:
            continue
        off = np.zeros(len(idx) + 1, dtype=np.uint32)
        np.cumsum([len(strs[i]) for i in idx], out=off[1:])
        data = np.frombuffer(b"".join(strs[i] for i in idx) + b"\0" * 16,
                             dtype=np.uint8).copy()
        enc, eoff = codec.encode(torch.from_numpy(data).cuda(),
                                 torch.from_numpy(off.view(np.int32)).cuda(),
                                 p)                          # device LITERALp
        torch.cuda.synchronize()
        eoff = eoff.cpu().numpy().view(np.uint32)
        enc = enc[:int(eoff[-1])].cpu().numpy().tobytes()
        keep = ~((1 << (p + 1)) - 1) & 0xFF          # instruction bits
        for j, i in enumerate(idx):
            lt = lits[i]
            w = bytearray(enc[eoff[j]:eoff[j + 1]])
            start = lt.pos - lt.hdr_len
            assert len(w) == lt.hdr_len + lt.len, (name, i)
            w[0] |= buf[start] & keep
            out[start:start + len(w)] = w
            spliced += 1
    assert spliced == len(lits)
    assert codec.device_error() == 0
    codec.close()
    assert bytes(out) == buf

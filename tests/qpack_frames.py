"""Minimal QPACK wire reader for the golden reference streams (test-only).

Reads the offline-interop container written by the reference's
bin/interop-encode.c:120-170 (u64 BE stream id, u32 BE length, payload;
stream 0 = encoder stream) and walks RFC 9204 encoder-stream and field-section
instructions far enough to locate every string literal: its prefix width
(3, 5 or 7 bits, the prefixes lsqpack_enc_enc_str is called with at
lsqpack.c:1983-2119), its H (Huffman) bit and its payload bytes.  This lets the
tests pin the Huffman codec against bytes the reference itself produced.
"""
import struct


class Truncated(Exception):
    pass


def read_int(buf, pos, prefix_bits):
    """HPACK prefixed integer (RFC 7541 5.1; lsqpack.c:2372-2441)."""
    if pos >= len(buf):
        raise Truncated()
    mask = (1 << prefix_bits) - 1
    v = buf[pos] & mask
    pos += 1
    if v < mask:
        return v, pos
    m = 0
    while True:
        if pos >= len(buf):
            raise Truncated()
        b = buf[pos]
        pos += 1
        v += (b & 0x7F) << m
        m += 7
        if not b & 0x80:
            return v, pos


def enc_int(first, value, prefix_bits):
    """RFC 7541 5.1 prefixed integer OR-ed into the first byte (what
    lsqpack_enc_int writes, lsqpack.c:784-814) -> bytes."""
    mask = (1 << prefix_bits) - 1
    if value < mask:
        return bytes([first | value])
    out, value = bytearray([first | mask]), value - mask
    while value >= 128:
        out.append(0x80 | (value & 0x7f))
        value >>= 7
    out.append(value)
    return bytes(out)


def read_literal(buf, pos, prefix_bits):
    """A string literal whose H bit sits just above an N-bit length prefix.
    Returns a dict with the literal's framing and payload."""
    start = pos
    h = (buf[pos] >> prefix_bits) & 1
    n, pos = read_int(buf, pos, prefix_bits)
    if pos + n > len(buf):
        raise Truncated()
    return {"prefix_bits": prefix_bits, "huffman": h, "start": start,
            "first_byte": buf[start], "payload": bytes(buf[pos:pos + n]),
            "wire": bytes(buf[start:pos + n]), "end": pos + n}


def read_interop(data):
    """Yield (stream_id, payload) frames; stop at a truncated frame."""
    pos = 0
    while pos + 12 <= len(data):
        sid, ln = struct.unpack(">QI", data[pos:pos + 12])
        if pos + 12 + ln > len(data):
            return
        yield sid, data[pos + 12:pos + 12 + ln]
        pos += 12 + ln


def encoder_stream_instructions(buf):
    """Walk encoder-stream instructions (RFC 9204 4.3).  Yields tuples
    (kind, info) where kind is 'insert_nameref', 'insert_literal', 'dup' or
    'capacity'.  Stops silently at a truncated instruction."""
    pos = 0
    try:
        while pos < len(buf):
            b = buf[pos]
            if b & 0x80:                                   # 1Txxxxxx
                static = bool(b & 0x40)
                idx, pos = read_int(buf, pos, 6)
                val = read_literal(buf, pos, 7)
                pos = val["end"]
                yield "insert_nameref", {"static": static, "index": idx,
                                         "value": val}
            elif b & 0x40:                                 # 01Hxxxxx
                name = read_literal(buf, pos, 5)
                val = read_literal(buf, name["end"], 7)
                pos = val["end"]
                yield "insert_literal", {"name": name, "value": val}
            elif b & 0x20:                                 # 001xxxxx
                cap, pos = read_int(buf, pos, 5)
                yield "capacity", {"capacity": cap}
            else:                                          # 000xxxxx
                idx, pos = read_int(buf, pos, 5)
                yield "dup", {"index": idx}
    except Truncated:
        return


def field_section_literals(buf):
    """Walk one encoded field section (RFC 9204 4.5) and return its string
    literals (names and values)."""
    lits = []
    _, pos = read_int(buf, 0, 8)           # Required Insert Count
    _, pos = read_int(buf, pos, 7)         # S + Delta Base
    while pos < len(buf):
        b = buf[pos]
        if b & 0x80:                                       # indexed
            _, pos = read_int(buf, pos, 6)
        elif b & 0x40:                                     # literal, name ref
            _, pos = read_int(buf, pos, 4)
            v = read_literal(buf, pos, 7)
            lits.append(v)
            pos = v["end"]
        elif b & 0x20:                                     # literal name
            n = read_literal(buf, pos, 3)
            v = read_literal(buf, n["end"], 7)
            lits += [n, v]
            pos = v["end"]
        elif b & 0x10:                                     # indexed post-base
            _, pos = read_int(buf, pos, 4)
        else:                                              # post-base name ref
            _, pos = read_int(buf, pos, 3)
            v = read_literal(buf, pos, 7)
            lits.append(v)
            pos = v["end"]
    return lits


def stream_literals(data):
    """All string literals in an interop file: encoder-stream literals and
    field-section literals, in file order."""
    out = []
    for sid, payload in read_interop(data):
        if sid == 0:
            for kind, info in encoder_stream_instructions(payload):
                if kind == "insert_nameref":
                    out.append(info["value"])
                elif kind == "insert_literal":
                    out += [info["name"], info["value"]]
        else:
            try:
                out += field_section_literals(payload)
            except Truncated:
                pass
    return out


def qif_strings(text):
    """Names and values of a QIF file (tab-separated, blank line between
    header lists, '#' comments)."""
    s = set()
    for line in text.split(b"\n"):
        if not line or line.startswith(b"#"):
            continue
        name, _, value = line.partition(b"\t")
        s.add(name)
        s.add(value)
    return s


def qif_header_lists(text):
    """List of header lists [(name, value), ...] in file order."""
    lists, cur = [], []
    for line in text.split(b"\n"):
        if line.startswith(b"#"):
            continue
        if not line:
            if cur:
                lists.append(cur)
                cur = []
            continue
        name, _, value = line.partition(b"\t")
        cur.append((name, value))
    if cur:
        lists.append(cur)
    return lists


# ---- strict restatement of the reference's framing rules (for the scanner
# tests on adversarial input: the reference's AFL seed corpora) -------------

class ProtoError(Exception):
    """lsqpack_dec_int / _int24 return -2 (lsqpack.c:2423, 2435, 2459)."""


MASK64 = (1 << 64) - 1


def dec_int(buf, pos, prefix_bits):
    """lsqpack_dec_int (lsqpack.c:2372-2436) on a complete buffer -> (value,
    pos); Truncated (-1) when the buffer ends inside the integer (within one
    call fewer than LSQPACK_UINT64_ENC_SZ = 11 bytes are read before that
    can happen, 2413-2420), ProtoError (-2) when the value needs more than
    64 bits (2426-2435)."""
    if pos >= len(buf):
        raise Truncated()
    pmax = (1 << prefix_bits) - 1
    val = buf[pos] & pmax
    pos += 1
    if val < pmax:
        return val, pos
    M = 0
    while True:
        if pos >= len(buf):
            raise Truncated()
        B = buf[pos]
        pos += 1
        val = (val + ((B & 0x7F) << M)) & MASK64
        M += 7
        if not (B & 0x80 and M < 64):
            break
    if M <= 63 or (M == 70 and buf[pos - 1] <= 1 and val >> 63):
        return val, pos
    raise ProtoError()


def dec_int24(buf, pos, prefix_bits):
    """lsqpack_dec_int24 (lsqpack.c:2443-2460): values >= 2^24 fail (-2)."""
    v, pos = dec_int(buf, pos, prefix_bits)
    if v >= 1 << 24:
        raise ProtoError()
    return v, pos


MAX_STRLEN = 65535            # LSXPACK_MAX_STRLEN, lsxpack_header.h:12-13


def _lit(buf, pos, prefix_bits, kind, instr, max_len=0):
    """max_len: the field-section clamp -- a declared length above it fails
    as soon as it is decoded (lsqpack.c:3682-3685, 3769-3772)."""
    if pos >= len(buf):
        raise Truncated()
    h = (buf[pos] >> prefix_bits) & 1
    n, p = dec_int24(buf, pos, prefix_bits)
    if max_len and n > max_len:
        raise ProtoError()
    if p + n > len(buf):
        raise Truncated()
    return (p, n, h, prefix_bits, p - pos, kind, instr), p + n


LIT_NAME, LIT_VALUE = 1, 2


def ref_scan_field_section(buf):
    """Literal spans of one field section under the reference's integer rules
    (RFC 9204 4.5; parse_header_prefix / parse_header_data, lsqpack.c:
    3955-4046, 3567-3915) -> ("ok" | "trunc" | "proto", [(pos, len, huffman,
    prefix_bits, hdr_len, kind, instr)])."""
    lits = []
    try:
        _, pos = dec_int(buf, 0, 8)            # Required Insert Count
        _, pos = dec_int(buf, pos, 7)          # S + Delta Base
        while pos < len(buf):
            b, at = buf[pos], pos
            if b & 0x80:                       # indexed field line
                _, pos = dec_int24(buf, pos, 6)
            elif b & 0x40:                     # literal with name reference
                _, pos = dec_int24(buf, pos, 4)
                lit, pos = _lit(buf, pos, 7, LIT_VALUE, at, MAX_STRLEN)
                lits.append(lit)
            elif b & 0x20:                     # literal with literal name
                n, pos = _lit(buf, pos, 3, LIT_NAME, at, MAX_STRLEN)
                v, pos = _lit(buf, pos, 7, LIT_VALUE, at, MAX_STRLEN)
                lits += [n, v]
            elif b & 0x10:                     # indexed post-base
                _, pos = dec_int24(buf, pos, 4)
            else:                              # post-base name reference
                _, pos = dec_int24(buf, pos, 3)
                lit, pos = _lit(buf, pos, 7, LIT_VALUE, at, MAX_STRLEN)
                lits.append(lit)
    except Truncated:
        return "trunc", []
    except ProtoError:
        return "proto", []
    return "ok", lits


def ref_scan_encoder_stream(buf):
    """Literal spans of the complete encoder-stream instructions in buf
    (RFC 9204 4.3; lsqpack_dec_enc_in, lsqpack.c:4574-4960: name index and
    lengths by dec_int24, capacity by dec_int, duplicate by dec_int24) ->
    ("ok" | "proto", [spans], consumed); a partial last instruction is left
    unconsumed (the reference resumes there)."""
    lits, pos = [], 0
    while pos < len(buf):
        b, at, q = buf[pos], pos, pos
        got = []
        try:
            if b & 0x80:                       # insert with name reference
                _, q = dec_int24(buf, q, 6)
                lit, q = _lit(buf, q, 7, LIT_VALUE, at)
                got.append(lit)
            elif b & 0x40:                     # insert with literal name
                n, q = _lit(buf, q, 5, LIT_NAME, at)
                v, q = _lit(buf, q, 7, LIT_VALUE, at)
                got += [n, v]
            elif b & 0x20:                     # set dynamic table capacity
                _, q = dec_int(buf, q, 5)
            else:                              # duplicate
                _, q = dec_int24(buf, q, 5)
        except Truncated:
            break
        except ProtoError:
            return "proto", [], 0
        lits += got
        pos = q
    return "ok", lits, pos


def fuzz_records(data, strict=True, single=False):
    """Records as bin/fuzz-decode.c:152-202 reads them: u64 BE stream id, u32
    BE size, payload, while more than 12 bytes remain; a size past the end
    is clamped (non-strict) or ends the walk (strict: the reference aborts);
    single: the first record only."""
    out, pos = [], 0
    while pos + 12 < len(data):
        sid, size = struct.unpack(">QI", data[pos:pos + 12])
        pos += 12
        if size > len(data) - pos:
            if strict:
                raise ValueError("truncated preamble at %d" % pos)
            size = len(data) - pos
        out.append((sid, bytes(data[pos:pos + size])))
        pos += size
        if single:
            break
    return out

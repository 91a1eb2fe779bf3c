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

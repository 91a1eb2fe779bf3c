#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ from the reference's OWN
test data (run in the build container, where /root/reference exists).

Nothing here executes reference code: the reference's C test files are read
as TEXT and their initializer data (known-answer vectors) is extracted by a
small C-initializer parser; the reference's committed data files (QIF corpora,
reference-encoded interop streams) are copied byte for byte.

Sources (all under /root/reference):
  test/test_huff_dec.c       tests[] (decode KATs) + bad_padding_tests[]
  test/test_enc_str.c        tests[] (lsqpack_enc_enc_str KATs, prefix 3)
  test/test_read_enc_stream.c tests[] (encoder-stream bytes -> dyn table)
  test/test_qpack.c          header_block_tests[] (headers -> enc/prefix/
                             header-block bytes)
  test/test_header_alloc_clamp.c  the two over-long-length blocks main()
                             builds (LSXPACK_MAX_STRLEN clamp, LQRHS_ERROR)
  test/test_int.c            tests[] (lsqpack_dec_int vectors, fed one byte
                             per call) + test_overlong_integer_full_buffer
  lsqpack.c                  static_table[] (QPACK static table, data)
  fuzz/input/256.100.1/*     interop-encode output, -t 256 -s 100 -a 1
  test/qifs/*.qif            QIF corpora the streams above were encoded from
  fuzz/decode/{a,b,c,d}/*    AFL seed corpora of the decoder (preambles and
                             test cases, copied as data/fuzz/*; names and
                             harness in fuzz_decode.json)

Output: kat_*.json (hex strings + source file:line), and copies of the data
files under tests/golden/data/.  A SHA-256 manifest is written to
MANIFEST.sha256.  Usage: python tests/golden/make_golden.py [REF_ROOT]
"""
import hashlib
import json
import os
import re
import shutil
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"


# --------------------------------------------------------------------------
# A small tokenizer + evaluator for C static initializers.

TOK = re.compile(r'''
    (?P<ws>\s+)
  | (?P<comment>/\*.*?\*/|//[^\n]*|\#[^\n]*)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<chr>'(?:\\.|[^'\\])')
  | (?P<num>0[xX][0-9a-fA-F]+[uUlL]*|0[bB][01]+[uUlL]*|\d+[uUlL]*)
  | (?P<id>[A-Za-z_]\w*)
  | (?P<op>[{}()\[\],.=|+\-*&<>;~!?:/%^])
  | (?P<other>.)
''', re.X | re.S)


def tokenize(text, base_line):
    pos, line, out = 0, base_line, []
    while pos < len(text):
        m = TOK.match(text, pos)
        if not m:
            raise ValueError("cannot tokenize at line %d: %r"
                             % (line, text[pos:pos + 20]))
        kind = m.lastgroup
        val = m.group(kind)
        if kind not in ("ws", "comment", "other"):
            out.append((kind, val, line))
        line += val.count("\n")
        pos = m.end()
    return out


def c_string_bytes(lit):
    """Decode one C string literal body (without quotes) to bytes.  Hex
    escapes are greedy, as in C."""
    s, i, out = lit, 0, bytearray()
    simple = {"n": 10, "t": 9, "r": 13, "0": 0, "\\": 92, '"': 34, "'": 39,
              "a": 7, "b": 8, "f": 12, "v": 11}
    while i < len(s):
        c = s[i]
        if c != "\\":
            out += c.encode("latin-1")
            i += 1
            continue
        i += 1
        c = s[i]
        if c in "xX":
            j = i + 1
            while j < len(s) and s[j] in "0123456789abcdefABCDEF":
                j += 1
            v = int(s[i + 1:j], 16)
            assert v < 256, "hex escape out of range"
            out.append(v)
            i = j
        elif c in "01234567":
            j = i
            while j < len(s) and j < i + 3 and s[j] in "01234567":
                j += 1
            out.append(int(s[i:j], 8))
            i = j
        else:
            out.append(simple[c])
            i += 1
    return bytes(out)


class Parser:
    def __init__(self, toks):
        self.t, self.i = toks, 0

    def peek(self, k=0):
        return self.t[self.i + k] if self.i + k < len(self.t) else (None, None, 0)

    def take(self):
        tok = self.t[self.i]
        self.i += 1
        return tok

    def expect(self, v):
        tok = self.take()
        assert tok[1] == v, "expected %r got %r at line %d" % (v, tok[1], tok[2])

    def init_list(self):
        """Parse '{' items '}' -> list, or dict if designated."""
        self.expect("{")
        items, named = [], {}
        while self.peek()[1] != "}":
            if self.peek()[1] == "." and self.peek(2)[1] == "=":
                self.take()
                name = self.take()[1]
                self.expect("=")
                named[name] = self.value()
            else:
                items.append(self.value())
            if self.peek()[1] == ",":
                self.take()
        self.expect("}")
        return named if named else items

    def value(self):
        if self.peek()[1] == "{":
            return self.init_list()
        return self.expr()

    def expr(self):
        """Collect tokens of one initializer expression and evaluate it."""
        toks, depth = [], 0
        while True:
            k, v, ln = self.peek()
            if v in (",", "}") and depth == 0:
                break
            if v == "(":
                depth += 1
            elif v == ")":
                depth -= 1
            toks.append(self.take())
        return evaluate(toks)


CASTS = re.compile(r"\(\s*(?:const\s+)?(?:unsigned\s+)?(?:char|int|uint8_t)\s*\*?\s*\)")


def evaluate(toks):
    if all(k == "str" for k, _, _ in toks):
        return b"".join(c_string_bytes(v[1:-1]) for _, v, _ in toks)
    # drop pointer casts like (unsigned char *)
    parts, i = [], 0
    while i < len(toks):
        k, v, ln = toks[i]
        if v == "(" and i + 2 < len(toks):
            j = i + 1
            words = []
            while j < len(toks) and toks[j][1] != ")":
                words.append(toks[j][1])
                j += 1
            if words and set(words) <= {"const", "unsigned", "char", "int",
                                         "uint8_t", "*"} and ("*" in words
                                                              or "char" in words):
                i = j + 1
                continue
        parts.append(toks[i])
        i += 1
    if parts and all(k == "str" for k, _, _ in parts):
        return b"".join(c_string_bytes(v[1:-1]) for _, v, _ in parts)
    src = []
    i = 0
    while i < len(parts):
        k, v, ln = parts[i]
        if k == "id" and v == "__LINE__":
            src.append(str(ln))
        elif k == "id" and v == "NULL":
            return None
        elif k == "id" and v == "UINT64_MAX":
            src.append(str((1 << 64) - 1))
        elif k == "id" and v == "sizeof":
            # sizeof("literal") -> len + 1
            assert parts[i + 1][1] == "(" and parts[i + 2][0] == "str"
            src.append(str(len(c_string_bytes(parts[i + 2][1][1:-1])) + 1))
            i += 4
            continue
        elif k == "id":
            src.append("__SYM__%s" % v)
        elif k == "num":
            src.append(str(int(v.rstrip("uUlL"), 0)))
        elif k == "chr":
            src.append(str(c_string_bytes(v[1:-1])[0]))
        else:
            src.append(v)
        i += 1
    expr = " ".join(src)
    if "__SYM__" in expr:
        return {"symbolic": expr.replace("__SYM__", "")}
    return int(eval(expr, {"__builtins__": {}}))


def find_array(path, name):
    """Return (parsed list, first line) of `... name[] = { ... };`."""
    text = open(path, encoding="latin-1").read()
    m = re.search(r"\b%s\s*\[\s*\]\s*=\s*\n?\s*\{" % re.escape(name), text)
    assert m, "%s not found in %s" % (name, path)
    start = text.index("{", m.start())
    line = text.count("\n", 0, start) + 1
    toks = tokenize(text[start:], line)
    p = Parser(toks)
    return p.init_list()


def rel(p):
    return os.path.relpath(p, REF)


def hpack_int(first, value, prefix_bits):
    """RFC 7541 5.1 prefixed integer OR-ed into `first` (the reference's
    lsqpack_enc_int, lsqpack.c:784-814, with room to spare)."""
    mask = (1 << prefix_bits) - 1
    if value < mask:
        return bytes([first | value])
    out, value = bytearray([first | mask]), value - mask
    while value >= 128:
        out.append(0x80 | (value & 0x7f))
        value >>= 7
    out.append(value)
    return bytes(out)


def clamp_cases(path):
    """The blocks test/test_header_alloc_clamp.c builds in main(): each
    `Case N` writes bytes with `*p++ = EXPR;` / `*p = EXPR;`, appends
    `lsqpack_enc_int(p, end, bignum, PREFIX)` and asserts the status of
    decode_block().  Parsed as text: the statements are evaluated with the
    initializer evaluator, the integer encoded by hpack_int."""
    text = open(path, encoding="latin-1").read()
    big = int(re.search(r"const\s+unsigned\s+bignum\s*=\s*(\d+)\s*;",
                        text).group(1))
    cases = []
    starts = [m.start() for m in re.finditer(r"/\*\s*Case\s+\d+", text)]
    for k, s in enumerate(starts):
        e = starts[k + 1] if k + 1 < len(starts) else text.index("printf", s)
        body = text[s:e]
        line = text.count("\n", 0, s) + 1
        title = re.sub(r"\n\s*\*", " ",
                       re.match(r"/\*\s*(.*?)\*/", body, re.S).group(1))
        blk = bytearray()
        stmt = re.compile(r"\*p(\+\+)?\s*=\s*([^;]+);|lsqpack_enc_int\(\s*p\s*,"
                          r"\s*end\s*,\s*(\w+)\s*,\s*(\d+)\s*\)"
                          r"|rhs\s*==\s*(\w+)")
        status, pending = None, None
        for m in stmt.finditer(body):
            if m.group(2) is not None:
                v = evaluate(tokenize(m.group(2), 0))
                if m.group(1):
                    blk.append(v & 0xff)
                else:
                    pending = v & 0xff
            elif m.group(3) is not None:
                assert m.group(3) == "bignum" and pending is not None
                blk += hpack_int(pending, big, int(m.group(4)))
                pending = None
            else:
                status = m.group(5)
        assert status and pending is None
        cases.append({"source": "%s:%d" % (rel(path), line),
                      "what": " ".join(title.split()),
                      "block": bytes(blk).hex(), "declared_len": big,
                      "expect": status})
    return cases


def as_bytes(v, size=None):
    if isinstance(v, (bytes, bytearray)):
        b = bytes(v)
    elif isinstance(v, list):
        b = bytes(x & 0xff for x in v)
    elif v is None:
        b = b""
    else:
        raise TypeError(v)
    if size is not None:
        b = (b + b"\0" * size)[:size]
    return b


# --------------------------------------------------------------------------

def main():
    out = {}
    f = os.path.join(REF, "test/test_huff_dec.c")
    dec = []
    for t in find_array(f, "tests"):
        line, src, src_sz, dst, dst_sz = t
        dec.append({"source": "%s:%d" % (rel(f), line),
                    "huff": as_bytes(src)[:src_sz].hex(),
                    "plain": as_bytes(dst)[:dst_sz].hex()})
    bad = []
    for t in find_array(f, "bad_padding_tests"):
        line, src, src_sz = t
        bad.append({"source": "%s:%d" % (rel(f), line),
                    "huff": as_bytes(src)[:src_sz].hex()})
    out["kat_huff_decode.json"] = {"decode_ok": dec, "decode_error": bad}

    f = os.path.join(REF, "test/test_enc_str.c")
    enc = []
    for t in find_array(f, "tests"):
        line, prefix, s, slen, obuf, ret = t
        enc.append({"source": "%s:%d" % (rel(f), line), "prefix_bits": prefix,
                    "str": as_bytes(s)[:slen].hex(),
                    "out": as_bytes(obuf)[:max(ret, 0)].hex(),
                    "retval": ret})
    out["kat_enc_str.json"] = {"enc_str": enc}

    f = os.path.join(REF, "test/test_read_enc_stream.c")
    es = []
    for t in find_array(f, "tests"):
        line, inp, isz, n_entries, table = t
        ents = [[as_bytes(nm).hex(), as_bytes(vl).hex()]
                for nm, vl in table[:n_entries]]
        es.append({"source": "%s:%d" % (rel(f), line),
                   "enc_stream": as_bytes(inp)[:isz].hex(),
                   "dyn_table": ents})
    out["kat_enc_stream.json"] = {"enc_stream": es}

    f = os.path.join(REF, "test/test_qpack.c")
    hb = []
    for t in find_array(f, "header_block_tests"):
        hdrs = []
        for h in t["qhbt_headers"][:t["qhbt_n_headers"]]:
            hdrs.append([as_bytes(h[0]).hex(), as_bytes(h[1]).hex()])
        hb.append({"source": "%s:%d" % (rel(f), t["qhbt_lineno"]),
                   "table_size": t["qhbt_table_size"],
                   "headers": hdrs,
                   "enc": as_bytes(t.get("qhbt_enc_buf"))[:t["qhbt_enc_sz"]].hex(),
                   "prefix": as_bytes(t.get("qhbt_prefix_buf"))[:t["qhbt_prefix_sz"]].hex(),
                   "header": as_bytes(t.get("qhbt_header_buf"))[:t["qhbt_header_sz"]].hex()})
    out["kat_header_blocks.json"] = {"header_blocks": hb}

    f = os.path.join(REF, "test/test_header_alloc_clamp.c")
    out["kat_header_alloc_clamp.json"] = {
        "max_strlen": 65535, "max_strlen_source": "lsxpack_header.h:12-13",
        "clamp_sites": "lsqpack.c:3682-3685, 3769-3772, 3350-3351",
        "cases": clamp_cases(f)}

    f = os.path.join(REF, "test/test_int.c")
    iv = []
    for t in find_array(f, "tests"):
        e = {"source": "%s:%d" % (rel(f), t["it_lineno"]),
             "prefix_bits": t["it_prefix_bits"],
             "encoded": as_bytes(t["it_encoded"])[:t["it_enc_sz"]].hex(),
             "retval": t["it_dec_retval"]}
        if "it_decoded" in t:
            e["decoded"] = str(t["it_decoded"])     # (u64: JSON-safe)
        iv.append(e)
    text = open(f, encoding="latin-1").read()
    fn = text.index("test_overlong_integer_full_buffer (void)")
    ov = find_array(f, "encoded")
    rv = re.search(r"lsqpack_dec_int\(&src, encoded \+ sizeof\(encoded\), (\d+),"
                   r"[^;]*;\s*assert\(rv == (-?\d+)\)", text[fn:], re.S)
    out["kat_int.json"] = {
        "dec_int": iv,
        "note": "tests[] are fed one byte per lsqpack_dec_int call: every "
                "strict prefix returns -1, the last byte the retval "
                "(test/test_int.c:198-214)",
        "overlong_full_buffer": {
            "source": "%s:%d" % (rel(f), text.count("\n", 0, fn) + 1),
            "prefix_bits": int(rv.group(1)),
            "encoded": as_bytes(ov).hex(), "retval": int(rv.group(2))}}

    f = os.path.join(REF, "lsqpack.c")
    st = []
    for name, val, nlen, vlen in find_array(f, "static_table"):
        st.append([as_bytes(name)[:nlen].decode("latin-1"),
                   as_bytes(val)[:vlen].decode("latin-1")])
    out["qpack_static_table.json"] = {"source": "lsqpack.c:104-209",
                                      "static_table": st}

    for name, obj in out.items():
        with open(os.path.join(HERE, name), "w") as fp:
            json.dump(obj, fp, indent=1, sort_keys=True)
            fp.write("\n")

    data = os.path.join(HERE, "data")
    os.makedirs(data, exist_ok=True)
    copied = []
    for sub in ("fuzz/input/256.100.1", "test/qifs"):
        d = os.path.join(REF, sub)
        for fn in sorted(os.listdir(d)):
            shutil.copyfile(os.path.join(d, fn), os.path.join(data, fn))
            copied.append(os.path.join("data", fn))

    # AFL seed corpora of the decoder (fuzz/decode/{a,b,c,d}): each dir's
    # preamble (if any) and test cases, renamed to safe names; the manifest
    # keeps the original names and the harness each dir is run with
    # (fuzz/decode/*/README, setup.sh; bin/fuzz-decode.c:152-202 framing)
    harness = {
        "a": {"program": "fuzz-decode", "table_size": 256, "risked": 100},
        "b": {"program": "fuzz-decode", "table_size": 4096, "risked": 100},
        "c": {"program": "interop-decode", "table_size": 256, "risked": 100},
        "d": {"program": "fuzz-decode", "table_size": 256, "risked": 100},
    }
    fz = {"source": "fuzz/decode/*", "framing":
          "records of u64 BE stream id, u32 BE size, payload (stream 0 = "
          "encoder stream); fuzz-decode: preamble strict, all records, then "
          "the test case's FIRST record with its size clamped to the file "
          "(bin/fuzz-decode.c:152-202, 331-332); interop-decode: every "
          "record of the test case", "dirs": {}}
    for sub in sorted(harness):
        d = os.path.join(REF, "fuzz/decode", sub)
        dst = os.path.join(data, "fuzz", sub)
        os.makedirs(dst, exist_ok=True)
        ent = dict(harness[sub], preamble=None, cases=[])
        if os.path.exists(os.path.join(d, "preamble")):
            shutil.copyfile(os.path.join(d, "preamble"),
                            os.path.join(dst, "preamble"))
            ent["preamble"] = "data/fuzz/%s/preamble" % sub
            copied.append(os.path.join("data", "fuzz", sub, "preamble"))
        tc = os.path.join(d, "test-cases")
        for k, fn in enumerate(sorted(os.listdir(tc))):
            safe = "case%02d" % k
            shutil.copyfile(os.path.join(tc, fn), os.path.join(dst, safe))
            ent["cases"].append({"file": "data/fuzz/%s/%s" % (sub, safe),
                                 "original": "fuzz/decode/%s/test-cases/%s"
                                             % (sub, fn)})
            copied.append(os.path.join("data", "fuzz", sub, safe))
        fz["dirs"][sub] = ent
    out["fuzz_decode.json"] = fz
    with open(os.path.join(HERE, "fuzz_decode.json"), "w") as fp:
        json.dump(fz, fp, indent=1, sort_keys=True)
        fp.write("\n")

    # fixtures written by the other generator (make_xxh32_golden.py) keep
    # their manifest lines
    others = [fn for fn in ("xxh32.json",)
              if os.path.exists(os.path.join(HERE, fn))]
    man = []
    for fn in sorted(list(out) + copied + others):
        h = hashlib.sha256(open(os.path.join(HERE, fn), "rb").read()).hexdigest()
        man.append("%s  %s" % (h, fn))
    with open(os.path.join(HERE, "MANIFEST.sha256"), "w") as fp:
        fp.write("\n".join(man) + "\n")
    print("wrote", ", ".join(sorted(out)), "and", len(copied), "data files")


if __name__ == "__main__":
    main()

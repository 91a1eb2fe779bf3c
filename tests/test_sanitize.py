"""Host code under AddressSanitizer + UndefinedBehaviorSanitizer, on the CPU
(SURVEY.md 5 "host ASan/UBSan").  GPU code cannot be
sanitized on this pool; the host code that parses untrusted wire bytes
(qhuff_frames.cpp), replays the reference decoder's stopping point
(qhuff_fastwalk.h) and the oracle can.

1. tests/c/san_check (gcc ASan + UBSan, any report aborts): every record of
   the reference's interop streams and AFL seed corpora, a seeded havoc of
   each and random bytes through both scanners; each literal's span, its
   Huffman decode at several dst_len, the fast-walk replay, the streaming
   decoder and the literal re-framing checked against the oracle.
2. The CPU suites of the scanner / oracle / shim / hook tests run again in a
   python whose libqhuff.so and oracle are the host-instrumented builds
   (clang ASan runtime preloaded)."""
import glob
import os
import subprocess
import sys

import pytest

from _paths import ROOT

CDIR = os.path.join(ROOT, "tests", "c")
SAN = os.path.join(CDIR, "_build", "san")
GOLD = os.path.join(ROOT, "tests", "golden", "data")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "-C", CDIR, "san"], capture_output=True,
                       text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    return SAN


def test_san_check_driver(built):
    files = sorted(glob.glob(os.path.join(GOLD, "*.out.256.100.1"))
                   + glob.glob(os.path.join(GOLD, "fuzz", "*", "*")))
    assert len(files) >= 20
    r = subprocess.run([os.path.join(built, "san_check")] + files,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" \
        not in r.stderr
    assert "failures 0" in r.stdout
    n_lits = int(r.stdout.split("literals ")[1].split()[0])
    assert n_lits > 5000


def _asan_runtime():
    rt = glob.glob("/opt/rocm/lib/llvm/lib/clang/*/lib/linux/"
                   "libclang_rt.asan-x86_64.so")
    if not rt:
        pytest.skip("clang ASan runtime not in this image")
    return rt[0]


def test_cpu_suites_under_asan(built):
    env = dict(os.environ)
    env.update({"LD_PRELOAD": _asan_runtime(),
                "ASAN_OPTIONS": "detect_leaks=0:abort_on_error=1",
                "UBSAN_OPTIONS": "print_stacktrace=1",
                "QHUFF_LIB": os.path.join(built, "libqhuff_san.so"),
                "QHUFF_ORACLE_LIB": os.path.join(built,
                                                 "libqhuff_oracle_san.so")})
    suites = ["test_oracle_golden.py", "test_frames.py", "test_fuzz_inputs.py",
              "test_fastwalk.py", "test_enc_hook.py", "test_abi.py",
              "test_exhaustive.py", "test_nghttp2_diff.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p",
                        "no:cacheprovider", "-m", "not gpu"]
                       + [os.path.join(ROOT, "tests", s) for s in suites],
                       env=env, capture_output=True, text=True, timeout=1200,
                       cwd=ROOT)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "runtime error" not in r.stderr
    assert "AddressSanitizer" not in r.stderr

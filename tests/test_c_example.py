"""examples/hook_demo.c: the INTEGRATION.md seams used from plain C99 (only
include/qhuff.h + libqhuff.so).  CPU: it builds with gcc -Werror and links
the library.  GPU: on each reference-encoded interop stream it decodes every
literal in one batch and re-creates every literal's wire bytes exactly."""
import os
import subprocess

import pytest

import _paths  # noqa: F401

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples")
BIN = os.path.join(EX, "hook_demo")
DATA = os.path.join(ROOT, "tests", "golden", "data")


def test_hook_demo_builds_and_links():
    subprocess.check_call(["make", "-s", "-C", EX])
    out = subprocess.check_output(["ldd", BIN]).decode()
    assert "libqhuff.so" in out and "not found" not in out


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["netbsd", "fb-req", "fb-resp"])
def test_hook_demo_round_trips_reference_streams(name):
    r = subprocess.run([BIN, os.path.join(DATA, name + ".out.256.100.1")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "re-framed mismatches 0" in r.stdout

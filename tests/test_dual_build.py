"""The QH_DUAL decode build (128-string tiles, two strings per
lane, 8 waves per workgroup) is an off-by-default option; its parity with
the oracle is kept checked here, in a child process that loads
libqhuff_dual.so (the library is chosen at import time)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DUAL = os.path.join(ROOT, "ls-qpack_amd", "libqhuff_dual.so")


@pytest.mark.gpu
def test_dual_build_decode_parity():
    if not os.path.exists(DUAL):
        pytest.fail("libqhuff_dual.so not built (make -C ls-qpack_amd dual)")
    env = dict(os.environ, QHUFF_LIB=DUAL)
    r = subprocess.run([sys.executable, "-u",
                        os.path.join(ROOT, "tests", "_dual_parity.py")],
                       env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "dual parity ok" in r.stdout

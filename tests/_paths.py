"""sys.path setup shared by tests: the product package lives in ls-qpack_amd/."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ls-qpack_amd")
if PKG not in sys.path:
    sys.path.insert(0, PKG)

"""Decode parity of the QH_DUAL build (128-string tiles, two strings per
lane; `make -C ls-qpack_amd dual`), run in its own process by
tests/test_dual_build.py because the library is chosen at import time
(QHUFF_LIB).  Reuses the decode checks of test_gpu_parity.py against the
oracle: KATs, reference-encoded stream literals, random valid strings of
every alphabet, garbage inputs (status + bytes), multi-unit / slow tiles,
edge batches (empty, n = 1, one huge string), the full 1M-string round
trip and the host path."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import test_gpu_parity as T  # noqa: E402
import qhuff  # noqa: E402


def main():
    lib = os.environ.get("QHUFF_LIB", "")
    assert lib.endswith("libqhuff_dual.so"), lib
    codec = qhuff.Codec(0)
    T.test_decode_kats(codec)
    for corpus in ("netbsd", "fb-req", "fb-resp"):
        T.test_reference_encoded_stream_literals(codec, corpus)
    for alpha in sorted(T.ALPHAS):
        T.test_decode_random_valid(codec, alpha)
    T.test_decode_garbage(codec)
    for lo, hi in ((30, 90), (100, 400), (0, 2000)):
        T.test_multi_unit_tiles(codec, lo, hi)
    T.test_edge_batches(codec)
    T.test_full_size_round_trip(codec)
    T.test_host_path_and_mirrors(codec)
    assert codec.device_error() == 0
    codec.close()
    print("dual parity ok")


if __name__ == "__main__":
    main()

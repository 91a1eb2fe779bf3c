#!/usr/bin/env python3
"""Residency census of both kernels: for grids of k workgroups per CU, how
many were co-resident (diagnostic for the persistent-grid sizing)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ls-qpack_amd"))

import torch
import qhuff


def main():
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    c = qhuff.Codec(0)
    for which, name in ((0, "encode"), (1, "decode")):
        for k in (1, 2, 3, 4):
            g = k * ncu
            print("%s grid %4d (%d/CU): resident %d" % (name, g, k,
                                                     c.residency(which, g)))
    c.close()


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Transformer tuning variant (reference tuning/transformer_tuning.py): the main CLI on a
10% strided subset with --weight_decay and MultiStepLR([10, 15], 0.1).  The reference
script was stale (called model(tokens, mask) against the 4-argument forward); this one
drives the current model."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import transformer_test  # noqa: E402


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--subset_stride" not in argv:
        argv += ["--subset_stride", "10"]
    if "--weight_decay" not in argv:
        argv += ["--weight_decay", "5e-4"]
    if "--scheduler" not in argv:
        argv += ["--scheduler", "multistep"]
    return transformer_test.main(argv)


if __name__ == "__main__":
    main()

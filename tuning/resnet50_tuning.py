#!/usr/bin/env python3
"""ResNet-50 tuning variant (reference tuning/resnet50_tuning.py): the main CLI on a 10%
strided subset of train and test with --weight_decay and --gamma (StepLR(2, gamma) for
NGD, cosine for SGD)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import resnet50_test  # noqa: E402


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if "--subset_stride" not in argv:
        argv += ["--subset_stride", "10"]
    if "--weight_decay" not in argv:
        argv += ["--weight_decay", "5e-4"]
    if "--gamma" not in argv:
        argv += ["--gamma", "0.75"]
    if "--ngd" not in argv and "--optimizer" not in argv:
        argv += ["--optimizer", "sgd", "--scheduler", "cosine"]
    return resnet50_test.main(argv)


if __name__ == "__main__":
    main()

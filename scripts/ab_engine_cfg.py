#!/usr/bin/env python3
"""A/B probe of engine launch-configuration choices without environment switches in the
product: sets module attributes, then runs bench.py's main in-process.

    python scripts/ab_engine_cfg.py [--table conv_tuned.json] -- <bench.py args>
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    rest = []
    if "--" in argv:
        i = argv.index("--")
        argv, rest = argv[:i], argv[i + 1:]
    ap = argparse.ArgumentParser()
    ap.add_argument("--table", default=None, help="conv tile table to use instead of the in-tree one")
    a = ap.parse_args(argv)
    from faster_distributed_training_amd.ops import conv_igemm as ci
    if a.table:
        with open(a.table) as f:
            ci._TUNED = json.load(f)
    sys.argv = ["bench.py"] + rest
    import bench
    bench.main()


if __name__ == "__main__":
    main()

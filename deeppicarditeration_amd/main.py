"""CLI of the reference (`picard train <cfg.yaml> [KEY VAL ...]`, picard/main.py:12-23):

    python -m deeppicarditeration_amd.main train scripts/burgers/base_100d_T1.0_w0.0_0.yaml PICARD.N 2
"""
import argparse
import sys
from pathlib import Path


def train(argv):
    ap = argparse.ArgumentParser(prog="picard train")
    ap.add_argument("configfile")
    ap.add_argument("overrides", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    if not Path(a.configfile).exists():
        raise SystemExit(f"config file {a.configfile} does not exist")
    from .config import load_cfg
    from .runner import PicardRunner
    cfg = load_cfg(a.configfile, [x.lstrip("-") for x in a.overrides])
    PicardRunner(cfg).run()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("train",):
        print(__doc__)
        return 2
    return train(argv[1:]) or 0


if __name__ == "__main__":
    sys.exit(main())

"""CLI of the reference (`picard train <cfg.yaml> [KEY VAL ...]`, picard/main.py:12-23):

    picard train scripts/burgers/base_100d_T1.0_w0.0_0.yaml PICARD.N 2
    python -m deeppicarditeration_amd.main train scripts/burgers/base_100d_T1.0_w0.0_0.yaml PICARD.N 2
    torchrun --nproc-per-node 8 -m deeppicarditeration_amd.main train <cfg.yaml>   (MC-sharded labels)
"""
import argparse
import os
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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        PicardRunner(cfg).run()
        return
    # torchrun --nproc-per-node G -m deeppicarditeration_amd.main train cfg.yaml: one process per GPU,
    # RCCL ("nccl" on ROCm) for the label moments' all-gather and the weight broadcast
    import datetime

    import torch
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    # Only rank 0 fits, checkpoints and evaluates; the other ranks wait in the weight broadcast for
    # that whole time, which at the shipped sizes can exceed the 10-minute default collective
    # timeout, after which the RCCL watchdog would abort them.  DPI_DIST_TIMEOUT_S (default 6 h)
    # bounds a wait instead.
    timeout = datetime.timedelta(seconds=float(os.environ.get("DPI_DIST_TIMEOUT_S", 6 * 3600)))
    dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
    try:
        PicardRunner(cfg, device=f"cuda:{local}", rank=dist.get_rank(), world=dist.get_world_size()).run()
    finally:
        dist.destroy_process_group()


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] not in ("train",):
        print(__doc__)
        return 2
    return train(argv[1:]) or 0


if __name__ == "__main__":
    sys.exit(main())

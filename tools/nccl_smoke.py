"""One-GPU RCCL smoke of the N > 1 bench path's process-group calls: run as
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29511 tools/nccl_smoke.py
it executes, on the "nccl" backend (RCCL), exactly the calls bench.py --gpus N makes:
dist.init_process_group("nccl", device_id=dev), the label moments' all_gather_into_tensor
(async, then work.wait() — a stream wait under RCCL), the device-tensor MAX all-reduce of the
range-guard flag (ShardedLabeler._reduce_flag), the timing all-reduce and barrier, and checks
that the gathered-and-reduced labels equal the single-rank call bit for bit.  Prints one JSON line."""
import json
import os
import sys
import time
from pathlib import Path

import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    t0 = time.perf_counter()
    dist.init_process_group("nccl", device_id=dev)
    t_init = time.perf_counter() - t0
    import deeppicarditeration_amd as dpi
    from deeppicarditeration_amd import _lib as L
    from deeppicarditeration_amd.sharding import ShardedLabeler
    torch.manual_seed(0)
    eq = dpi.Cha(100, 1.0, 5.0, 1.0)
    net = dpi.construct_mlp(101, 1, [128] * 4, ["ELU"] * 4, None)
    M = 4096
    gen = dpi.OnlineDataGenerator(eq, net, 80, 1, device=dev, t_always_uniform=True, n_estimate_terminal=M,
                                  n_estimate_integral=M, n_euler_steps=50, seed=1)
    world, rank = dist.get_world_size(), dist.get_rank()
    lab = ShardedLabeler(gen, rank=rank, world=world, group=dist.group.WORLD)
    tx, pb = gen.sample_t_and_x(16)
    ws = gen.point_baseline(tx)
    m0, m1 = lab.shard(M)
    mom = gen.label_moments(tx, pb, M, m0, m1, L.DPI_BOTH, ws).contiguous()
    flat = torch.empty((world * mom.shape[0],) + tuple(mom.shape[1:]), dtype=mom.dtype, device=dev)
    work = dist.all_gather_into_tensor(flat, mom, group=dist.group.WORLD, async_op=True)
    work.wait()
    y = gen.finalize(gen.moments_reduce(flat.view((world,) + tuple(mom.shape))), M, L.DPI_BOTH, ws)
    y1 = ShardedLabeler(gen).labels(tx, pb)
    flag = lab._reduce_flag(0) if world > 1 else None
    t = torch.tensor([1.0, 2.0], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dev_flag = torch.tensor([0.0], device=dev)
    dist.all_reduce(dev_flag, op=dist.ReduceOp.MAX)  # the range-guard flag's device all-reduce
    dist.barrier()
    torch.cuda.synchronize()
    out = {"backend": dist.get_backend(), "world": world, "init_s": round(t_init, 3),
           "all_gather_into_tensor_bytes": flat.numel() * 4, "labels_bit_identical": bool(torch.equal(y, y1)),
           "max_abs_diff": float((y - y1).abs().max()), "flag": flag, "device_flag": float(dev_flag.item()),
           "timing_all_reduce": t.tolist(), "rccl": torch.cuda.nccl.version() if hasattr(torch.cuda, "nccl") else None}
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()
    assert out["labels_bit_identical"], out


if __name__ == "__main__":
    main()

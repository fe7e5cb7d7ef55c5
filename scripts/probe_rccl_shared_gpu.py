"""Probe: can two RCCL ranks share one GPU on this box? (all_reduce + all_to_all_single + all_gather)"""
import os
import sys
import torch
import torch.distributed as dist


def main():
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    t = torch.full((4,), float(rank + 1), device=dev)
    dist.all_reduce(t)
    s = torch.arange(world * 2, dtype=torch.int64, device=dev) + 100 * rank
    r = torch.empty_like(s)
    dist.all_to_all_single(r, s)
    outs = [torch.empty(3, device=dev) for _ in range(world)]
    dist.all_gather(outs, torch.full((3,), float(rank), device=dev))
    torch.cuda.synchronize()
    print(f"rank {rank}: allreduce {t.tolist()} a2a {r.tolist()} ag {[o[0].item() for o in outs]}", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()

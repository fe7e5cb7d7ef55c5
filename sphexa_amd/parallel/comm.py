"""Communication layer: one process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm) for device
tensors, gloo for the CPU path and CPU multi-process tests.

Replaces the reference's MPI layer (domain/include/cstone/primitives/mpi_wrappers.hpp:40-196, mpi_cuda.cuh:41-91):
  * point-to-point Isend/Probe(ANY_SOURCE)/Recv  -> ``alltoallv``: a count pre-exchange (RCCL cannot probe) followed
    by one grouped all_to_all_single of a packed device buffer (every peer pair on its own xGMI link)
  * MPI_Allreduce(MIN/SUM/MAX) on host scalars    -> ``allreduce`` on device tensors (no host staging)
  * tag/epoch protocol                            -> not needed: collectives are stream ordered and issued in the
                                                     same order on every rank
World size 1 short-circuits every call. With the gloo backend, device tensors are staged through host memory (gloo has
no all-to-all for device tensors): this lets several ranks share one GPU in tests of the multi-rank GPU path.
"""

from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

SUM, MIN, MAX = "sum", "min", "max"
_OPS = {SUM: dist.ReduceOp.SUM, MIN: dist.ReduceOp.MIN, MAX: dist.ReduceOp.MAX}


class Comm:
    def __init__(self, group=None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.size, self.backend = 0, 1, None

    def _staged(self, t: torch.Tensor) -> bool:
        return self.backend == "gloo" and t.is_cuda

    # -------------------------------------------------------------------------------------------- collectives
    def allreduce(self, t: torch.Tensor, op: str = SUM) -> torch.Tensor:
        if self.size > 1:
            if self._staged(t):
                h = t.cpu()
                dist.all_reduce(h, op=_OPS[op], group=self.group)
                t.copy_(h)
            else:
                dist.all_reduce(t, op=_OPS[op], group=self.group)
        return t

    def allreduce_scalar(self, v: float, op: str = SUM, device=None, dtype=torch.float64) -> float:
        if self.size == 1:
            return v
        t = torch.tensor([v], dtype=dtype, device=device or self._dev())
        self.allreduce(t, op)
        return t.item()

    def barrier(self):
        if self.size > 1:
            if self.backend == "nccl":
                dist.barrier(group=self.group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=self.group)

    def _dev(self):
        return torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")

    def exchange_counts(self, send_counts: Sequence[int]) -> List[int]:
        """all-to-all of one integer per peer (replaces MPI_Probe + MPI_Get_count)"""
        if self.size == 1:
            return list(send_counts)
        s = torch.tensor(list(send_counts), dtype=torch.int64, device=self._dev())
        r = torch.empty_like(s)
        dist.all_to_all_single(r, s, group=self.group)
        return [int(v) for v in r.cpu().tolist()]

    def alltoallv(self, send: torch.Tensor, send_counts: Sequence[int], recv_counts: Sequence[int] | None = None,
                  ) -> Tuple[torch.Tensor, List[int]]:
        """variable all-to-all along dim 0. ``send`` rows are grouped by destination rank in rank order."""
        if self.size == 1:
            return send[: send_counts[0]].clone(), list(send_counts)
        if recv_counts is None:
            recv_counts = self.exchange_counts(send_counts)
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        staged = self._staged(send)
        src = send.contiguous().cpu() if staged else send.contiguous()
        recv = torch.empty(shape, dtype=send.dtype, device=src.device)
        dist.all_to_all_single(recv, src, output_split_sizes=list(recv_counts),
                               input_split_sizes=list(send_counts), group=self.group)
        return (recv.to(send.device) if staged else recv), list(recv_counts)

    def allgather_var(self, t: torch.Tensor) -> List[torch.Tensor]:
        """gather tensors of different first-dimension sizes from all ranks"""
        if self.size == 1:
            return [t]
        if self._staged(t):
            return [o.to(t.device) for o in Comm.allgather_var(self, t.cpu())]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        ns = [torch.empty_like(n) for _ in range(self.size)]
        dist.all_gather(ns, n, group=self.group)
        sizes = [int(v.item()) for v in ns]
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        outs = [torch.empty_like(pad) for _ in range(self.size)]
        dist.all_gather(outs, pad, group=self.group)
        return [o[:s] for o, s in zip(outs, sizes)]


def init_distributed(backend: str | None = None) -> Comm:
    """initialise torch.distributed from torchrun-style environment variables if present"""
    if dist.is_available() and not dist.is_initialized() and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return Comm()

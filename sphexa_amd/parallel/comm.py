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

RCCL audit mode (``SPHX_COMM_CHECK=1`` or ``Comm(check=True)``): RCCL refuses two ranks on one GPU, so the RCCL path
cannot run on a 1-GPU box. Instead, every collective issued over gloo is checked against the constraints RCCL puts on
it — contiguous tensors of an RCCL dtype, integer split sizes that sum to the tensor extents, send/receive tensors on
one device — and appended to a per-rank signature log (op, dtype, trailing shape). ``verify_sequence()`` all-gathers a
hash of that log and raises if any two ranks issued a different sequence of collectives (the condition that deadlocks
or corrupts an RCCL communicator).
"""

from __future__ import annotations

import os
import zlib
from typing import List, Sequence, Tuple

import torch
import torch.distributed as dist

from ..utils.phase_prof import timed_comm

SUM, MIN, MAX = "sum", "min", "max"
_OPS = {SUM: dist.ReduceOp.SUM, MIN: dist.ReduceOp.MIN, MAX: dist.ReduceOp.MAX}
# element types RCCL can reduce / move (ncclDataType_t)
RCCL_DTYPES = {torch.uint8, torch.int8, torch.int32, torch.int64, torch.float16, torch.bfloat16, torch.float32,
               torch.float64}


class CommCheckError(RuntimeError):
    pass


def _stage_host(t: torch.Tensor) -> torch.Tensor:
    """gloo staging: device tensor -> host bounce buffer (a copy an RCCL run does not make; scripts/sync_inventory.py
    leaves it out of the synchronization count)"""
    return t.contiguous().cpu()


def _stage_dev(t: torch.Tensor, device) -> torch.Tensor:
    """gloo staging: host bounce buffer -> device"""
    return t.to(device)


class Comm:
    def __init__(self, group=None, check: bool | None = None):
        self.group = group
        if dist.is_available() and dist.is_initialized():
            self.rank = dist.get_rank(group)
            self.size = dist.get_world_size(group)
            self.backend = dist.get_backend(group)
        else:
            self.rank, self.size, self.backend = 0, 1, None
        self.check = os.environ.get("SPHX_COMM_CHECK") == "1" if check is None else check
        self.log: List[str] = []

    def _staged(self, t: torch.Tensor) -> bool:
        return self.backend == "gloo" and t.is_cuda

    # ----------------------------------------------------------------------------------------- RCCL audit
    def _audit(self, op: str, *tensors: torch.Tensor, splits: Sequence[Sequence[int]] = ()):
        if not self.check or self.size == 1:
            return
        dev = tensors[0].device
        for t in tensors:
            if not t.is_contiguous():
                raise CommCheckError(f"{op}: non-contiguous tensor {tuple(t.shape)}")
            if t.dtype not in RCCL_DTYPES:
                raise CommCheckError(f"{op}: dtype {t.dtype} is not an RCCL type")
            if t.device != dev:
                raise CommCheckError(f"{op}: tensors on {dev} and {t.device}")
        for sp, t in zip(splits, tensors):
            if any((not isinstance(v, int)) or v < 0 for v in sp) or len(sp) != self.size:
                raise CommCheckError(f"{op}: bad split sizes {list(sp)[:8]}")
            if sum(sp) != (t.shape[0] if t.dim() else 1):
                raise CommCheckError(f"{op}: splits sum {sum(sp)} != extent {t.shape[0]}")
        t = tensors[0]
        self.log.append(f"{op}:{str(t.dtype)}:{tuple(t.shape[1:])}")

    def verify_sequence(self) -> int:
        """all ranks must have issued the same collectives in the same order; returns the number checked"""
        if self.size == 1:
            return len(self.log)
        sig = zlib.crc32("|".join(self.log).encode()) & 0x7FFFFFFF
        t = torch.tensor([sig, len(self.log)], dtype=torch.int64, device=self._dev())
        outs = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(outs, t, group=self.group)
        vals = [tuple(int(v) for v in o.cpu().tolist()) for o in outs]
        if len(set(vals)) != 1:
            raise CommCheckError(f"ranks issued different collective sequences: {vals}")
        return len(self.log)

    # -------------------------------------------------------------------------------------------- collectives
    def allreduce(self, t: torch.Tensor, op: str = SUM) -> torch.Tensor:
        if self.size > 1:
            self._audit("allreduce_" + op, t)
            with timed_comm("allreduce", t, self._staged(t)):
                if self._staged(t):
                    h = _stage_host(t)
                    dist.all_reduce(h, op=_OPS[op], group=self.group)
                    t.copy_(_stage_dev(h, t.device))
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
            if self.check:
                self.log.append("barrier")
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
        s = torch.tensor([int(v) for v in send_counts], dtype=torch.int64, device=self._dev())
        r = torch.empty_like(s)
        self._audit("exchange_counts", s, r)
        dist.all_to_all_single(r, s, group=self.group)
        return [int(v) for v in r.cpu().tolist()]

    def exchange_counts_dev(self, counts: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """all-to-all of the rows of a (size, k) int64 tensor (row q goes to rank q), on the device: no host copy.
        The caller brings send and receive counts to the host together (one synchronization). ``out``: contiguous
        destination of the received rows (e.g. the second half of one send|recv buffer)"""
        if self.size == 1:
            return counts.clone() if out is None else out.copy_(counts)
        s = counts.contiguous()
        staged = self._staged(s)
        with timed_comm("exchange_counts", s, staged):
            src = _stage_host(s) if staged else s
            r = torch.empty_like(src) if (staged or out is None) else out
            self._audit("exchange_counts", src, r)
            dist.all_to_all_single(r, src, group=self.group)
            if staged:
                r = _stage_dev(r, counts.device)
                if out is not None:
                    out.copy_(r)
                    return out
            return r

    def allgather_fixed(self, t: torch.Tensor) -> List[torch.Tensor]:
        """all-gather of equal-shape tensors (no size exchange, no host copy over RCCL)"""
        if self.size == 1:
            return [t]
        staged = self._staged(t)
        with timed_comm("allgather_fixed", t, staged):
            src = _stage_host(t) if staged else t.contiguous()
            outs = [torch.empty_like(src) for _ in range(self.size)]
            self._audit("allgather", src)
            dist.all_gather(outs, src, group=self.group)
            return [_stage_dev(o, t.device) for o in outs] if staged else outs

    def allgather_stacked(self, t: torch.Tensor) -> torch.Tensor:
        """all-gather of equal-shape tensors into one (size, *shape) tensor: over RCCL straight into the stacked
        buffer (all_gather_into_tensor), over gloo the list form + one stack"""
        if self.size == 1:
            return t.unsqueeze(0)
        if self.backend == "nccl" and t.is_cuda:
            src = t.contiguous()
            out = torch.empty((self.size,) + tuple(src.shape), dtype=src.dtype, device=src.device)
            with timed_comm("allgather_fixed", src):
                self._audit("allgather", src)
                dist.all_gather_into_tensor(out, src, group=self.group)
            return out
        if self._staged(t):
            # gloo with a device tensor: stacked on the host, one copy up (no device concatenation kernel)
            with timed_comm("allgather_fixed", t, True):
                src = _stage_host(t)
                outs = [torch.empty_like(src) for _ in range(self.size)]
                self._audit("allgather", src)
                dist.all_gather(outs, src, group=self.group)
                return _stage_dev(torch.stack(outs), t.device)
        return torch.stack(self.allgather_fixed(t))

    def alltoallv(self, send: torch.Tensor, send_counts: Sequence[int], recv_counts: Sequence[int] | None = None,
                  ) -> Tuple[torch.Tensor, List[int]]:
        """variable all-to-all along dim 0. ``send`` rows are grouped by destination rank in rank order."""
        if self.size == 1:
            return send[: send_counts[0]].clone(), list(send_counts)
        if recv_counts is None:
            recv_counts = self.exchange_counts(send_counts)
        send_counts = [int(v) for v in send_counts]
        recv_counts = [int(v) for v in recv_counts]
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        staged = self._staged(send)
        with timed_comm("alltoallv", send, staged):
            src = _stage_host(send) if staged else send.contiguous()
            recv = torch.empty(shape, dtype=send.dtype, device=src.device)
            self._audit("alltoallv", src, recv, splits=(send_counts, recv_counts))
            dist.all_to_all_single(recv, src, output_split_sizes=list(recv_counts),
                                   input_split_sizes=list(send_counts), group=self.group)
            return (_stage_dev(recv, send.device) if staged else recv), list(recv_counts)

    def alltoallv_start(self, send: torch.Tensor, send_counts: Sequence[int], recv_counts: Sequence[int]
                        ) -> "PendingExchange":
        """``alltoallv`` with known receive counts, issued without waiting: over RCCL the all-to-all runs on the
        communicator's stream while the caller's stream keeps computing; ``PendingExchange.wait()`` makes the
        caller's stream wait for it (no host synchronization). Over gloo, host tensors move asynchronously on gloo's
        worker threads; device tensors are staged through host memory synchronously."""
        if self.size == 1:
            return PendingExchange(send[: int(send_counts[0])].clone(), None, send.device, None)
        send_counts = [int(v) for v in send_counts]
        recv_counts = [int(v) for v in recv_counts]
        shape = (sum(recv_counts),) + tuple(send.shape[1:])
        staged = self._staged(send)
        with timed_comm("alltoallv_start", send, staged):
            src = _stage_host(send) if staged else send.contiguous()
            recv = torch.empty(shape, dtype=send.dtype, device=src.device)
            self._audit("alltoallv", src, recv, splits=(send_counts, recv_counts))
            work = dist.all_to_all_single(recv, src, output_split_sizes=recv_counts, input_split_sizes=send_counts,
                                          group=self.group, async_op=not staged)
            return PendingExchange(recv, work, send.device, src)

    def allgather_var(self, t: torch.Tensor) -> List[torch.Tensor]:
        """gather tensors of different first-dimension sizes from all ranks"""
        if self.size == 1:
            return [t]
        if self._staged(t):
            return [_stage_dev(o, t.device) for o in Comm.allgather_var(self, _stage_host(t))]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
        self._audit("allgather_count", n)
        ns = [torch.empty_like(n) for _ in range(self.size)]
        dist.all_gather(ns, n, group=self.group)
        sizes = [int(v) for v in torch.cat(ns).cpu().tolist()]  # one host copy for all ranks
        mx = max(sizes)
        pad = torch.zeros((mx,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        self._audit("allgather", pad)
        outs = [torch.empty_like(pad) for _ in range(self.size)]
        dist.all_gather(outs, pad, group=self.group)
        return [o[:s] for o, s in zip(outs, sizes)]


class PendingExchange:
    """an all-to-all in flight: ``wait()`` returns the received rows on the sender's device"""

    def __init__(self, recv: torch.Tensor, work, device, keep):
        self.recv, self.work, self.device = recv, work, device
        self._keep = keep  # the packed send buffer stays alive until the exchange has completed

    def wait(self) -> torch.Tensor:
        with timed_comm("alltoallv_wait"):
            if self.work is not None:
                self.work.wait()
                self.work = None
            self._keep = None
            return self.recv if self.recv.device == self.device else _stage_dev(self.recv, self.device)


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

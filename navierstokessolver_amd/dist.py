"""Multi-rank plumbing (one process per GPU, launched by torch.distributed.run).

* nccl_id(): rank 0 makes an ncclUniqueId (RCCL) and broadcasts it over the default
  process group; every rank hands it to ns_create -- the data path then runs on RCCL
  over xGMI inside libnsgpu.so (neighbour send/recv of ghost rows, allreduce of the
  residual / mean / min-max scalars).
* TorchHostTransport: the same exchanges through torch.distributed (gloo) on the host,
  plugged into ns_create as an ns_host_transport.  Used by the 2-process GPU test on a
  single-GPU box (RCCL cannot put two ranks on one device) to exercise the full slab
  decomposition with the real kernels."""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L


def nccl_id(dist) -> bytes:
    import torch
    n = L.lib().ns_nccl_id_size()
    t = torch.zeros(n, dtype=torch.uint8)
    if dist.get_rank() == 0:
        buf = ctypes.create_string_buffer(n)
        L.check(L.lib().ns_nccl_get_id(buf))
        t = torch.frombuffer(bytearray(buf.raw), dtype=torch.uint8).clone()
    dist.broadcast(t, 0)
    return bytes(t.tolist())


class TorchHostTransport:
    """ns_host_transport over torch.distributed point-to-point + all_reduce (gloo)."""

    def __init__(self, dist):
        import torch
        self.dist, self.torch = dist, torch
        self.rank, self.size = dist.get_rank(), dist.get_world_size()
        self._ex = L.EXCHANGE_FN(self._exchange)
        self._ar = L.ALLREDUCE_FN(self._allreduce)
        self.struct = L.NsHostTransport(None, self._ex, self._ar)
        self.calls = 0

    @staticmethod
    def _view(ptr, n):
        return np.ctypeslib.as_array(ptr, shape=(n,)) if ptr else None

    def _exchange(self, user, slo, shi, rlo, rhi, count):
        try:
            torch, dist = self.torch, self.dist
            ops = []
            bufs = []
            for sp, rp, peer in ((slo, rlo, self.rank - 1), (shi, rhi, self.rank + 1)):
                if not sp:
                    continue
                s = torch.from_numpy(self._view(sp, count).copy())
                r = torch.empty(count, dtype=torch.float64)
                ops += [dist.P2POp(dist.isend, s, peer), dist.P2POp(dist.irecv, r, peer)]
                bufs.append((rp, r))
            for w in dist.batch_isend_irecv(ops):
                w.wait()
            for rp, r in bufs:
                self._view(rp, count)[:] = r.numpy()
            self.calls += 1
            return 0
        except Exception as e:  # never raise through the C-ABI
            print("host transport exchange failed:", e, flush=True)
            return -1

    def _allreduce(self, user, buf, n, op):
        try:
            v = self._view(buf, n)
            t = self.torch.from_numpy(v.copy())
            self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN if op == 1 else self.dist.ReduceOp.SUM)
            v[:] = t.numpy()
            return 0
        except Exception as e:
            print("host transport allreduce failed:", e, flush=True)
            return -1

"""Partitioned full-batch LM over several GPUs.

BASELINE configs[4]: "2000-frame, 20-object, 500k-landmark full-batch
graph, landmark-block partitioned Schur with RCCL reduce of reduced
system". The reference solves such a graph in one GTSAM process
(RGBDBackendModule.cc:207-231); here one process per GPU holds a
dynohip handle marked as rank r of N (dynohip_set_partition). The handle
linearises and Schur-eliminates only its share of the graph; the exchange
steps are the all-reduces this module hands to the C-ABI:

  * per linear solve, the separator tiles + right-hand side rows of the
    reduced pose system (device memory, RCCL over xGMI);
  * per LM inner iteration, 8 scalars (errors and failure flags, host).

torch.distributed is the transport only. With the gloo backend (CPU tests,
or several ranks sharing one GPU) device buffers are staged through host
memory.
"""
import ctypes as C
import traceback

import numpy as np

from . import _abi
from .optimizer import LevenbergMarquardtOptimizer, Solver, _check


class _DeviceArray:
    """A raw device pointer exposed to torch.as_tensor (no copy)."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (int(n),), "typestr": "<f8", "data": (int(ptr), False),
                                         "version": 2, "strides": None}


class TorchAllReduce:
    """dynohip_allreduce_fn over torch.distributed: in-place sum over the
    group. Device buffers: with RCCL (backend "nccl") the all-reduce is
    enqueued on the solver's own stream (torch.cuda.ExternalStream), so it
    is ordered after the kernels that wrote the buffer and before the ones
    that read the result, with no host synchronisation; with gloo the stream
    is synchronised and the buffer staged through host memory."""

    def __init__(self, device, group=None, op=None):
        import torch
        import torch.distributed as dist

        self.torch, self.dist = torch, dist
        self.group = group
        self.op = dist.ReduceOp.SUM if op is None else op   # tests: a PREMUL_SUM makes the ordering visible
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.backend = dist.get_backend(group)
        self.on_gpu = self.backend == "nccl"
        self.calls = 0
        self.doubles = 0
        self.fn = _abi.ALLREDUCE_FN(self._call)

    def _call(self, _ctx, buf, n, on_device, stream):
        try:
            torch, dist = self.torch, self.dist
            self.calls += 1
            self.doubles += int(n)
            if on_device:
                ptr = C.cast(buf, C.c_void_p).value
                t = torch.as_tensor(_DeviceArray(ptr, n), device=self.device)
                ext = torch.cuda.ExternalStream(int(stream or 0), device=self.device)
                if self.on_gpu:
                    with torch.cuda.stream(ext):   # stream-ordered, returns before completion
                        dist.all_reduce(t, op=self.op, group=self.group)
                else:
                    ext.synchronize()
                    h = t.cpu()
                    dist.all_reduce(h, group=self.group)
                    t.copy_(h)
                    torch.cuda.synchronize(self.device)
            else:
                arr = np.ctypeslib.as_array(buf, shape=(int(n),))
                if self.on_gpu:
                    t = torch.from_numpy(arr.copy()).to(self.device)
                    dist.all_reduce(t, group=self.group)
                    arr[:] = t.cpu().numpy()
                else:
                    h = torch.from_numpy(arr)   # shares the C buffer
                    dist.all_reduce(h, group=self.group)
            return 0
        except Exception:  # noqa: BLE001 - reported through the C return code
            traceback.print_exc()
            return -1


class PartitionedSolver(Solver):
    """A dynohip handle that is rank `rank` of `nranks` of one partitioned
    solve. Every rank passes the same global graph and values."""

    def __init__(self, device, nranks, rank, allreduce):
        super().__init__(device)
        self.nranks, self.rank = int(nranks), int(rank)
        self._allreduce = allreduce          # keeps the ctypes callback alive
        _check(self.lib, self.h, self.lib.dynohip_set_partition(self.h, self.nranks, self.rank, allreduce.fn, None))

    def value_owner(self):
        n = self._values.keys.shape[0]
        out = np.zeros(n, dtype=np.int32)
        xd = C.c_int64()
        _check(self.lib, self.h, self.lib.dynohip_value_owner(
            self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), n, C.byref(xd)))
        return out, xd.value

    def gathered_values_data(self):
        """The global values on every rank: each rank contributes the values
        it owns (rank 0 also the replicated separator poses), summed with
        one all-reduce through the same callback."""
        owner, _ = self.value_owner()
        data = self.values_data()
        sizes = np.where(np.asarray(self._values.kinds) == _abi.POSE3, 12, 3)
        mine = (owner == self.rank) | ((owner < 0) & (self.rank == 0))
        mask = np.repeat(mine, sizes)
        part = np.where(mask, data, 0.0)
        rc = self._allreduce.fn(None, part.ctypes.data_as(C.POINTER(C.c_double)), part.shape[0], 0, None)
        if rc != 0:
            raise RuntimeError("all-reduce of the gathered values failed")
        return part


class PartitionedLevenbergMarquardtOptimizer(LevenbergMarquardtOptimizer):
    """gtsam::LevenbergMarquardtOptimizer(graph, values).optimize() split over
    the ranks of a torch.distributed group (one process per GPU). Collective:
    every rank constructs it with the same graph and values and calls the
    same methods. values() returns the full optimised values on every rank."""

    def __init__(self, graph, values, params=None, device=0, group=None):
        import torch.distributed as dist

        nranks = dist.get_world_size(group)
        rank = dist.get_rank(group)
        self.allreduce = TorchAllReduce(device, group)
        solver = PartitionedSolver(device, nranks, rank, self.allreduce)
        super().__init__(graph, values, params, device, solver=solver)

    def optimize(self):
        self._summary = self.solver.optimize(self.params)
        return self.values()

    def values(self):
        return self.solver._values.with_data(self.solver.gathered_values_data())

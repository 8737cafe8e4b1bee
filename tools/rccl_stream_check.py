"""The RCCL branch of dynosam_amd.partitioned.TorchAllReduce on a GPU, world
size 1 (tests/test_partition.py::test_rccl_device_branch_stream_ordered).

The process group (backend "nccl", i.e. RCCL) is set up before any GPU call.
A buffer is written on a stream by a kernel that is still running (a long
sleep kernel in front of it) when the dynohip_allreduce_fn callback is
called with that stream, exactly as the solver calls it (partitioned
handles, csrc/solver.cpp: no synchronisation before the call). The next
kernel on the stream reads the result. With a pre-multiplied sum (factor 2)
the order is visible in the values: 2 * src + 1 only if the reduction ran
after the write and before the read.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", str(29600 + os.getpid() % 200))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    from dynosam_amd.partitioned import TorchAllReduce

    ar = TorchAllReduce(0, op=dist._make_nccl_premul_sum(2.0))
    n = 1 << 20
    src = torch.arange(n, dtype=torch.float64, device="cuda:0")
    buf = torch.zeros(n, dtype=torch.float64, device="cuda:0")
    torch.cuda.synchronize()
    s = torch.cuda.Stream(device=0)
    res = {"backend": dist.get_backend(), "world_size": dist.get_world_size()}
    with torch.cuda.stream(s):
        torch.cuda._sleep(50_000_000)     # the producer is still running at the call
        buf.copy_(src)
    rc = ar._call(None, C.cast(buf.data_ptr(), C.POINTER(C.c_double)), n, 1, s.cuda_stream)
    res["returned_before_done"] = not s.query()
    with torch.cuda.stream(s):
        buf.add_(1.0)                     # the stream's next kernel
    s.synchronize()
    want = 2.0 * src + 1.0
    res.update(rc=rc, calls=ar.calls, doubles=ar.doubles, exact=bool(torch.equal(buf, want)),
               max_err=float((buf - want).abs().max()))
    # host branch (the 8 LM scalars per inner iteration)
    h = (C.c_double * 8)(*range(8))
    ar2 = TorchAllReduce(0)
    res["host_rc"] = ar2._call(None, h, 8, 0, s.cuda_stream)
    res["host_ok"] = list(h) == [float(i) for i in range(8)]
    dist.destroy_process_group()
    print(json.dumps(res))


if __name__ == "__main__":
    main()

"""Partitioned full-batch LM vs the single-GPU solve.

Launch one process per rank:
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P tools/partition_check.py --config C2 [--backend gloo|nccl]

Ranks use GPU local_rank % device_count, so N ranks may share one GPU (then
use --backend gloo: RCCL does not put two ranks on one device). Every rank
runs the partitioned optimize(); rank 0 then runs the ordinary single-handle
optimize() on the same graph and prints one JSON line comparing them: LM
iteration counts, the per-attempt trace (lambda, errors, accept flags) and
the final values (relative Frobenius norm). Exit code 1 on a mismatch beyond
--tol.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2")
    ap.add_argument("--backend", default="gloo")
    ap.add_argument("--tol", type=float, default=1e-6)
    ap.add_argument("--max-iterations", type=int, default=100)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    from dynosam_amd import _abi, synth
    from dynosam_amd.optimizer import LevenbergMarquardtOptimizer
    from dynosam_amd.partitioned import PartitionedLevenbergMarquardtOptimizer

    dist.init_process_group(backend=args.backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = int(os.environ.get("LOCAL_RANK", rank)) % torch.cuda.device_count()
    torch.cuda.set_device(dev)
    graph, values, _ = synth.generate(args.config)
    params = _abi.LMParams.gtsam_default()
    params.max_iterations = args.max_iterations
    t0 = time.perf_counter()
    opt = PartitionedLevenbergMarquardtOptimizer(graph, values, params, device=dev)
    t1 = time.perf_counter()
    out = opt.optimize()
    t2 = time.perf_counter()
    owner, xdoubles = opt.solver.value_owner()
    trace = opt.trace()
    summ = opt.summary()
    local_factors = None
    st = opt.solver.stats()
    local_factors = st.get("n_factor")
    counts = [None] * world
    dist.all_gather_object(counts, {"rank": rank, "factors": local_factors, "points": st.get("n_point"),
                                    "calls": opt.allreduce.calls, "doubles": opt.allreduce.doubles})
    ok = True
    if rank == 0:
        ref_opt = LevenbergMarquardtOptimizer(graph, values, params, device=dev)
        t3 = time.perf_counter()
        ref = ref_opt.optimize()
        t4 = time.perf_counter()
        rtrace = ref_opt.trace()
        rel = float(np.linalg.norm(out.data - ref.data) / np.linalg.norm(ref.data))
        n = min(len(trace), len(rtrace))
        # the error trajectory: accepted steps (a rejected trial point at a
        # small lambda is far from the solution and its error is as
        # ill-conditioned as the step; reported separately)
        def rel_err(acc):
            return max((abs(a["new_error"] - b["new_error"]) / max(abs(b["new_error"]), 1e-300)
                        for a, b in zip(trace[:n], rtrace[:n])
                        if np.isfinite(b["new_error"]) and (b["accepted"] or not acc)), default=0.0)
        err_rel = rel_err(True)
        err_rel_all = rel_err(False)
        same_accepts = [a["accepted"] for a in trace] == [b["accepted"] for b in rtrace]
        ok = (summ.iterations == ref_opt.iterations() and same_accepts and rel < args.tol and err_rel < args.tol)
        res = {"config": args.config, "ranks": world, "backend": args.backend, "ok": bool(ok),
               "iterations": [summ.iterations, ref_opt.iterations()],
               "inner": [summ.inner_iterations, ref_opt.getInnerIterations()],
               "final_error": [summ.final_error, ref_opt.summary().final_error],
               "values_rel_frobenius": rel, "trace_error_rel_max": err_rel, "trial_error_rel_max": err_rel_all, "same_accept_sequence": same_accepts,
               "exchange_doubles_per_solve": int(xdoubles),
               "replicated_values": int((owner < 0).sum()), "per_rank": counts,
               "s_setup": t1 - t0, "s_optimize_partitioned": t2 - t1, "s_optimize_single": t4 - t3}
        line = json.dumps(res)
        print(line, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(line + "\n")
    flag = torch.tensor([0 if ok else 1])
    dist.broadcast(flag, 0)
    dist.destroy_process_group()
    sys.exit(int(flag.item()))


if __name__ == "__main__":
    main()

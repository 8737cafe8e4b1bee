"""Critical path of one k_factor_persist launch from per-task timestamps.

Needs a libdynohip.so built with -DDYNOHIP_TASK_CLOCK (tools/build_variant.sh
<dir> -DDYNOHIP_TASK_CLOCK, then DYNOSAM_AMD_LIB_DIR=<dir>). Runs one LM
optimisation of a synthetic config, reads the timestamps of the last
factorisation launch (s_memrealtime, 100 MHz: dequeue, dependencies met,
factor start, factor end, done) and prints the phase totals and the chain of
tasks that ends last, each linked to the task that finished last before it
could start.

usage: python tools/task_clock.py [C2|NS] [out.json]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dynosam_amd import _native, synth  # noqa: E402
from dynosam_amd.optimizer import LevenbergMarquardtOptimizer, plan_export  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "C2"
    graph, values, _ = synth.generate(cfg)
    ft = plan_export(graph, values, "ftask").reshape(-1, 10)
    nt = ft.shape[0]
    opt = LevenbergMarquardtOptimizer(graph, values, device=0)
    opt.optimize()
    lib = _native.load("libdynohip.so")
    buf = np.zeros((32, 32768), dtype=np.uint64)
    lib.dynohip_debug_task_clock.argtypes = [C.c_void_p, C.c_int]
    assert lib.dynohip_debug_task_clock(buf.ctypes.data, nt) >= 0
    t = buf[:5, :nt].astype(np.int64)
    t0min = t[0].min()
    t = (t - t0min) / 100.0               # us
    sub = (buf[6:12, :nt].astype(np.int64) - t0min) / 100.0
    bar = (buf[12:16, :nt].astype(np.int64) - t0min) / 100.0
    worker = buf[5, :nt]
    kind, kk, ii = ft[:, 0], ft[:, 1], ft[:, 2]
    span = t[4].max()
    pan = kind == 0
    out = {"config": cfg, "tasks": int(nt), "span_us": float(span), "workers": int(worker.max() + 1)}
    for name, m in (("panel", pan), ("update", ~pan)):
        out[name] = {"n": int(m.sum()), "wait_us_mean": float((t[1] - t[0])[m].mean()),
                     "exec_us_mean": float((t[4] - t[1])[m].mean())}
    own = pan & (kk != ii)
    # the real dependency chain (Plan::fdep: the task that made the last
    # write a task waits for): each task's "ready" = its last input written
    fs = plan_export(graph, values, "fdep_start")
    fd = plan_export(graph, values, "fdep").reshape(-1, 2)
    writer, cnt = {}, {}
    for q in range(nt):
        if kind[q] == 1 or kk[q] != ii[q]:
            c = cnt.get(int(ft[q, 3]), 0) + 1
            cnt[int(ft[q, 3])] = c
            writer[(int(ft[q, 3]), c)] = q
    ready = np.zeros(nt)
    dpred = -np.ones(nt, dtype=np.int64)
    for q in range(nt):
        for j in range(fs[q], fs[q + 1]):
            w_ = writer[(int(fd[j, 0]), int(fd[j, 1]))]
            if t[4, w_] > ready[q]:
                ready[q], dpred[q] = t[4, w_], w_
    # sub-phases: early deps met (t1) -> operands waited for + loads issued +
    # rpart (P0) -> tiles in LDS (P1) -> factor start; factor end -> Linv in
    # LDS (Q0) -> y (Q1) -> TRSM (Q2) -> stores (Q3) -> done.
    # t1 is the first class of dependencies (everything but the pending
    # operand tiles, DESIGN §3 "Round 3"): the span t1 -> P0 includes the wait
    # for those operands, so it is reported as such, and the hand-off proper
    # is measured from the last input's write (the panel's `ready`)
    from_ready = sub[0] - np.maximum(t[1], ready)
    out["panel"]["sub_us_mean"] = {
        "early_deps_to_loaded (incl. the operand wait)": float((sub[0] - t[1])[pan].mean()),
        "handoff_last_input_to_loaded": float(from_ready[pan].mean()),
        "tiles_lds": float((sub[1] - sub[0])[pan].mean()),
        "pending_w0": float((t[2] - sub[1])[pan].mean()), "linv_y_sync": float((sub[2] - t[3])[own].mean()),
        "y": float((sub[3] - sub[2])[pan].mean()), "trsm": float((sub[4] - sub[3])[own].mean()),
        "store": float((sub[5] - sub[4])[own].mean()), "contrib_drain": float((t[4] - sub[5])[own].mean())}
    # factorisation block steps as wave 0 passes each barrier: stamped by the
    # diagonal tasks' factorisation (factor_tile_blk) only; an own panel
    # (factor_own) leaves its entries unwritten (zero), so only tasks whose
    # four stamps lie inside their factorisation are averaged
    raw_bar = buf[12:16, :nt].astype(np.int64)
    vb = pan & (raw_bar != 0).all(0)
    vb &= (bar[0] >= t[2]) & (bar[3] <= t[3]) & (np.diff(bar, axis=0) >= 0).all(0)
    out["panel"]["factor_steps_tasks"] = int(vb.sum())
    out["panel"]["factor_steps_us_mean"] = ([float((bar[0] - t[2])[vb].mean())] +
                                            [float((bar[j] - bar[j - 1])[vb].mean()) for j in range(1, 4)] +
                                            [float((t[3] - bar[3])[vb].mean())]) if vb.any() else None
    # per block step, cycles on the factoring wave: pivots, U row, barrier
    # wait (s_memtime; the same diagonal tasks)
    cyc = buf[16:32, :nt].astype(np.int64)
    vc = pan & (cyc != 0).all(0)
    for kb in range(4):
        a, b_, c, d = cyc[4 * kb:4 * kb + 4]
        vc &= (b_ >= a) & (c >= b_) & (d >= c)
    steps = []
    for kb in range(4):
        a, b_, c, d = cyc[4 * kb:4 * kb + 4]
        steps.append({"pivots": float((b_ - a)[vc].mean()), "u_row": float((c - b_)[vc].mean()),
                      "barrier": float((d - c)[vc].mean())} if vc.any() else None)
    out["panel"]["factor_step_cycles_tasks"] = int(vc.sum())
    out["panel"]["factor_step_cycles"] = steps
    out["panel"].update({"pre_us_mean": float((t[2] - t[1])[pan].mean()),
                         "factor_us_mean": float((t[3] - t[2])[pan].mean()),
                         "post_us_mean": float((t[4] - t[3])[pan].mean())})
    # worker occupancy
    busy = float((t[4] - t[1]).sum())
    out["busy_frac_exec"] = busy / (span * (worker.max() + 1))
    out["busy_frac_held"] = float((t[4] - t[0]).sum()) / (span * (worker.max() + 1))
    # every reported time must be a sane span of this launch
    def _walk(x):
        if isinstance(x, dict):
            for v in x.values():
                yield from _walk(v)
        elif isinstance(x, list):
            for v in x:
                yield from _walk(v)
        elif isinstance(x, float):
            yield x
    bad = [x for x in _walk({k: out[k] for k in ("panel", "update")}) if not (-1.0 <= x <= 1e6)]
    assert not bad, f"absurd task-clock fields: {bad}"
    late_pick = np.maximum(0.0, t[0] - ready)   # ready before a worker took it
    out["ready_before_pick_us"] = {"mean": float(late_pick.mean()), "max": float(late_pick.max()),
                                   "tasks_over_2us": int((late_pick > 2.0).sum())}
    # per panel, when its pending operands were written: the diagonal one
    # (pd, L(k,c)) and the own pair's first one (qa, L(i,c)); -1 if none
    pairs = plan_export(graph, values, "pairs").reshape(-1, 2)

    def operand_end(q, sl):
        for j in range(fs[q], fs[q + 1]):
            if int(fd[j, 0]) == sl:
                return float(t[4, writer[(sl, int(fd[j, 1]))]])
        return -1.0

    def operands(q):
        pd = int(pairs[ft[q, 5], 0]) if ft[q, 6] - ft[q, 5] == 1 else -1
        qa = int(pairs[ft[q, 7], 0]) if kk[q] != ii[q] and ft[q, 8] - ft[q, 7] == 1 else -1
        return {"pd_end": operand_end(q, pd) if pd >= 0 else -1.0,
                "qa_end": operand_end(q, qa) if qa >= 0 else -1.0}
    dchain = []
    cur = int(np.argmax(t[4]))
    while cur >= 0:
        dchain.append(cur)
        cur = int(dpred[cur])
    dchain.reverse()
    out["dep_chain"] = [{"q": int(q), "kind": int(kind[q]), "k": int(kk[q]), "i": int(ii[q]),
                         "pick": float(t[0, q]), "ready": float(ready[q]), "deps_met": float(t[1, q]),
                         "end": float(t[4, q]),
                         # a panel on the chain, from its predecessor's end: operands
                         # and right-hand side in (late wait included), tiles in LDS,
                         # pending diagonal block, factorisation, TRSM + stores
                         **({"to_loaded": float(sub[0, q] - ready[q]), "to_lds": float(sub[1, q] - sub[0, q]),
                             "pend": float(t[2, q] - sub[1, q]), "fac": float(t[3, q] - t[2, q]),
                             "post": float(t[4, q] - t[3, q]), **operands(q)} if kind[q] == 0 else {})}
                         for q in dchain]
    # chain ending last
    chain = []
    cur = int(np.argmax(t[4]))
    while True:
        rec = {"q": cur, "kind": int(kind[cur]), "k": int(kk[cur]), "i": int(ii[cur]),
               "t0": float(t[0, cur]), "wait": float(t[1, cur] - t[0, cur]), "exec": float(t[4, cur] - t[1, cur])}
        if kind[cur] == 0:
            rec.update(pre=float(t[2, cur] - t[1, cur]), factor=float(t[3, cur] - t[2, cur]),
                       post=float(t[4, cur] - t[3, cur]))
        chain.append(rec)
        cand = np.where(t[4] <= t[1, cur] + 0.5)[0]
        cand = cand[cand != cur]
        if cand.size == 0:
            break
        nxt = int(cand[np.argmax(t[4, cand])])
        if t[4, nxt] < t[0, cur] - 0.5:   # not waiting on anything: queue-bound from here
            rec["queue_bound"] = True
            break
        cur = nxt
    chain.reverse()
    out["chain"] = chain
    tot = {"wait": sum(c["wait"] for c in chain), "pre": sum(c.get("pre", 0) for c in chain),
           "factor": sum(c.get("factor", 0) for c in chain), "post": sum(c.get("post", 0) for c in chain),
           "update_exec": sum(c["exec"] for c in chain if c["kind"] == 1)}
    out["chain_totals_us"] = tot
    print(json.dumps({k: v for k, v in out.items() if k not in ("chain", "dep_chain")}, indent=1))
    for c in out["dep_chain"]:
        print("dep " + " ".join(f"{k}={v:.1f}" if isinstance(v, float) else f"{k}={v}" for k, v in c.items()))
    for c in chain:
        print(" ".join(f"{k}={v:.1f}" if isinstance(v, float) else f"{k}={v}" for k, v in c.items()))
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()

"""Where a sliding-window solve of the C2-shaped stream spends its time
(RGBDBackendModule.cc:343-388, backend.flags: window 10 / overlap 4).

The window problems are collected by replaying the stream through the module
with optimize off (the module builds and exports every window's graph and
values exactly as in the bench), then each is solved on one persistent handle
as the module does (set_graph, set_values, optimize, values read back), timed
per phase on the host; the handle's HIP-event phase times give the kernel
share. Usage: python tools/window_timing.py [C2] [reps]"""
import sys
import time

sys.path.insert(0, ".")
from dynosam_amd import backend, stream, synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402


def windows(config):
    c = synth.CONFIGS[config]
    cfg = stream.StreamConfig(frames=c["frames"], objects=c["objects"], static_landmarks=c["static_landmarks"],
                              dyn_slots=c["dyn_slots"], object_visible_frames=c.get("object_visible_frames", 0),
                              seed=42)
    packets, _ = stream.generate(cfg)
    m = backend.RGBDBackendModule(use_full_batch_opt=False, full_batch_frame=len(packets), optimize=False,
                                  device_id=0, post_update=False)
    out = []
    for p in packets:
        r = m.spinOnce(p)
        if r["window_end"] > r["window_start"]:
            g, v, _ = m.lastProblem()
            out.append((g, v))
    return out


def main(config="C2", reps=2):
    probs = windows(config)
    print(f"{config}: {len(probs)} windows", flush=True)
    s = Solver(0)
    for rep in range(reps):
        timed = rep == reps - 1   # HIP events only on the last pass (they add host work per phase)
        s.set_timing(timed)
        tg = tv = to = tr = 0.0
        its = tries = 0
        kern = {}
        for g, v in probs:
            t0 = time.perf_counter()
            s.set_graph(g)
            t1 = time.perf_counter()
            s.set_values(v)
            t2 = time.perf_counter()
            r = s.optimize()
            t3 = time.perf_counter()
            s.values_data()
            t4 = time.perf_counter()
            tg, tv, to, tr = tg + t1 - t0, tv + t2 - t1, to + t3 - t2, tr + t4 - t3
            its += r.iterations
            tries += r.inner_iterations
            st = s.stats()
            for k in ("ms_linearize", "ms_schur", "ms_assembly", "ms_cholesky", "ms_solve", "ms_backsub",
                      "ms_retract_error"):
                kern[k] = kern.get(k, 0.0) + st[k]
        n = len(probs)
        print(f"rep {rep}: per window set_graph {1e3 * tg / n:.3f} ms, set_values {1e3 * tv / n:.3f} ms, "
              f"optimize {1e3 * to / n:.3f} ms, values {1e3 * tr / n:.3f} ms; {its / n:.1f} iterations, "
              f"{tries / n:.1f} tries per window; optimize per try {1e6 * to / max(tries, 1):.1f} us", flush=True)
        if timed:
            print("   kernel time per try (HIP events, us): " +
                  ", ".join(f"{k[3:]} {1e3 * x / max(tries, 1):.1f}" for k, x in kern.items()), flush=True)
    s.close()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "C2", int(a[1]) if len(a) > 1 else 2)

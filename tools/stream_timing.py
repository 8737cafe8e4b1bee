"""Where the stream replay's host time goes (bench.py --mode stream): per
replay of the C2-shaped stream through RGBDBackendModule, the wall time of
the Python spinOnce calls, of the native dynob_module_spin inside them, of
the final flush (deferred windows), and the module's statistics (map update,
static / dynamic construction, window construction) in milliseconds.
usage: python tools/stream_timing.py [windows_in_flight ...]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import backend, stream, synth  # noqa: E402

cfgd = synth.CONFIGS["C2"]
cfg = stream.StreamConfig(frames=cfgd["frames"], objects=cfgd["objects"], static_landmarks=cfgd["static_landmarks"],
                          dyn_slots=cfgd["dyn_slots"], object_visible_frames=cfgd.get("object_visible_frames", 0),
                          seed=42)
packets, _ = stream.generate(cfg)


def replay(k):
    m = backend.RGBDBackendModule(use_full_batch_opt=False, optimize=True, post_update=False, windows_in_flight=k)
    lib = m._lib
    native = [0.0]
    orig = lib.dynob_module_spin

    def timed(*a):
        t = time.perf_counter()
        r = orig(*a)
        native[0] += time.perf_counter() - t
        return r

    lib_spin = timed
    t0 = time.perf_counter()
    it = 0
    for p in packets:
        m._lib = type("L", (), {"dynob_module_spin": staticmethod(lib_spin),
                                "dynob_module_last_error": lib.dynob_module_last_error})
        r = m.spinOnce(p)
        it += r["iterations"]
    m._lib = lib
    t1 = time.perf_counter()
    if k:
        it += m.flush()["iterations"]
    t2 = time.perf_counter()
    keep.append(m)   # destroyed outside the timed replays
    st = {}
    for lab in ("map.update_observations [ns]", "backend.update_static_obs [ns]", "backend.update_dynamic_obs [ns]",
                "rgbd_motion_world.sliding_window_construction [ns]", "rgbd_motion_world.sliding_window_optimise [ns]"):
        st[lab.split(" ")[0]] = float(m.statistics(lab).sum()) / 1e6
    return {"windows_in_flight": k, "lm_iterations": it, "ms_total": 1e3 * (t2 - t0), "ms_spins": 1e3 * (t1 - t0),
            "ms_native_spin": 1e3 * native[0], "ms_python_outside": 1e3 * (t1 - t0 - native[0]),
            "ms_flush": 1e3 * (t2 - t1), "stats_ms": st, "it_per_s": it / (t2 - t0)}


keep = []

if __name__ == "__main__":
    import json
    ks = [int(x) for x in sys.argv[1:]] or [0, 3]
    for k in ks:
        replay(k)
        for _ in range(2):
            print(json.dumps(replay(k)), flush=True)
        for m in keep:
            m.close()
        keep.clear()

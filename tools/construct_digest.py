"""Digest of every sliding-window problem and the full-batch problem of the
C2-shaped stream (construction only, optimize=False), plus timing."""
import sys, time, hashlib, pickle
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import numpy as np
from dynosam_amd import backend, stream, synth
c = synth.CONFIGS["C2"]
cfg = stream.StreamConfig(frames=c["frames"], objects=c["objects"], static_landmarks=c["static_landmarks"],
                          dyn_slots=c["dyn_slots"], object_visible_frames=c.get("object_visible_frames", 0), seed=42)
packets, _ = stream.generate(cfg)
def h_obj(o, hh):
    if isinstance(o, np.ndarray): hh.update(o.tobytes())
    elif isinstance(o, dict):
        for k in sorted(o, key=str): hh.update(str(k).encode()); h_obj(o[k], hh)
    elif isinstance(o, (list, tuple)):
        for x in o: h_obj(x, hh)
    else: hh.update(repr(o).encode())
for fb in (False, True):
    for formulation in ("motion", "llworld"):
        kw = dict(use_full_batch_opt=fb, full_batch_frame=len(packets), optimize=False, device_id=0, post_update=True)
        prm = backend.backend_params(formulation=backend.LL_WORLD) if formulation == "llworld" else None
        m = backend.RGBDBackendModule(params=prm, **kw)
        hh = hashlib.sha256(); t = time.perf_counter(); n = 0
        for p in packets:
            r = m.spinOnce(p)
            if r.get("window_end", 0) or (fb and p is packets[-1]):
                g, v, o = m.lastProblem(); h_obj((g.arrays(), v.keys, v.kinds, v.data), hh); n += 1
        h_obj(m.formulation.getObjectPoses(), hh)
        print(f"fb={fb} {formulation}: problems={n} digest={hh.hexdigest()[:16]} {1e3*(time.perf_counter()-t):.0f} ms")

"""Window / batch drivers (integer, bit-exact) and window sharding across
ranks (gloo, world_size 2, CPU)."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from dynosam_amd import synth
from dynosam_amd.windows import (SlidingWindow, full_batch_trigger, merge_last_writer_wins, shard,
                                 window_schedule)


class RefSlidingWindow:
    """Restatement of RGBDBackendModule::SlidingWindow::check
    (RGBDBackendModule.hpp:120-144) -- the test oracle."""

    def __init__(self, window, overlap):
        self.w, self.o, self.prev, self.first = window, overlap, overlap, -1

    def check(self, k):
        if self.first == -1:
            self.first = k
        frame = k - self.first
        cond = (self.prev - (frame - self.w)) == self.o
        if cond:
            self.prev = frame
        return cond, k - self.w, k


@pytest.mark.parametrize("window,overlap,first", [(10, 4, 0), (10, 4, 7), (5, 2, 0), (8, 0, 3), (6, 5, 1)])
def test_sliding_window_bit_exact(window, overlap, first):
    a, b = SlidingWindow(window, overlap), RefSlidingWindow(window, overlap)
    for k in range(first, first + 200):
        ca, sa, ea = a.check(k)
        cb, sb, eb = b.check(k)
        assert ca == cb
        assert ea == eb
        if ca:
            assert sa == sb


def test_shipped_window_schedule():
    # backend.flags:27-28: window 10, overlap 4 -> a window every 6 frames
    w = window_schedule(0, 50)
    assert w[0] == (0, 10)
    assert all(e2 - e1 == 6 for (_, e1), (_, e2) in zip(w, w[1:]))
    assert all(e - s == 10 for s, e in w)


def test_full_batch_trigger():
    assert full_batch_trigger(200, 199)
    assert not full_batch_trigger(200, 198)


def test_shard_partition():
    for n in range(0, 20):
        for world in (1, 2, 3, 8):
            got = sorted(i for r in range(world) for i in shard(n, r, world))
            assert got == list(range(n))


def _window_problem(i):
    g, v, _ = synth.generate("T1", seed=100 + i)
    return g, v


def _solve(i):
    from oracle_binding import Oracle
    g, v = _window_problem(i)
    o = Oracle(g, v)
    o.optimize()
    return (v.keys.copy(), v.kinds.copy(), o.values_data())


def _worker(rank, world, n_windows, port, out_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    mine = {i: _solve(i) for i in shard(n_windows, rank, world)}
    gathered = [None] * world if rank == 0 else None
    dist.gather_object(mine, gathered, dst=0)
    if rank == 0:
        allres = {}
        for d in gathered:
            allres.update(d)
        merged = merge_last_writer_wins([allres[i] for i in range(n_windows)])
        np.save(out_path, np.array([(k, *v[1]) for k, v in sorted(merged.items()) if v[0] == 1]))
    dist.barrier()
    dist.destroy_process_group()


def test_window_sharding_gloo_matches_serial(tmp_path):
    n_windows = 5
    out = str(tmp_path / "merged.npy")
    port = 29500 + os.getpid() % 1000
    mp.spawn(_worker, args=(2, n_windows, port, out), nprocs=2, join=True)
    got = np.load(out)
    serial = merge_last_writer_wins([_solve(i) for i in range(n_windows)])
    ref = np.array([(k, *v[1]) for k, v in sorted(serial.items()) if v[0] == 1])
    assert np.array_equal(got, ref)
    # last writer wins: overlapping keys take the last window's value
    last = _solve(n_windows - 1)
    keys, kinds, data = last
    assert np.array_equal(serial[int(keys[0])][1], data[:12])

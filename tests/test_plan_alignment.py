"""The reduced gather (kernels.hip k_gather_reduced) reads its operand rows
with 16-byte loads, so every block a band entry reads must start at an even
arena offset (plan.cpp "arena layout" aligns each region; the record strides,
column starts and block sizes are even). It also relies on the target
classes (Plan::red_order) covering every target once, smallest counts first,
each class in target order. Host only: the plans of single and partitioned
handles, through dynohip_plan_export."""
import sys

import numpy as np
import pytest

sys.path.insert(0, ".")
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import plan_export  # noqa: E402

K_ADD_BLOCK = 2   # plan.hpp kAddBlock


@pytest.mark.parametrize("name,nranks", [("T2", 1), ("C1", 1), ("C1", 2)])
def test_band_operands_are_16_byte_aligned(name, nranks):
    g, v, _ = synth.generate(name)
    for rank in range(nranks):
        ent = plan_export(g, v, "gRed_ent", nranks, rank).reshape(-1, 4)
        assert ent.shape[0] > 0
        a = ent[:, 0].view(np.uint32).astype(np.int64)
        b = ent[:, 1].view(np.uint32).astype(np.int64)
        k, sign = ent[:, 2], ent[:, 3]
        assert set(np.unique(k).tolist()) <= {3, 6}
        assert set(np.unique(sign).tolist()) <= {1, -1, K_ADD_BLOCK}
        assert (b % 2 == 0).all(), "odd B block offsets"
        mult = sign != K_ADD_BLOCK
        assert (a[mult] % 2 == 0).all(), "odd A block offsets"
        assert (k[~mult] == 6).all()


@pytest.mark.parametrize("name", ["T2", "C1"])
def test_reduced_target_classes(name):
    g, v, _ = synth.generate(name)
    start = plan_export(g, v, "gRed_start").view(np.int64)
    n = np.diff(start)
    order = plan_export(g, v, "red_order")
    assert sorted(order.tolist()) == list(range(n.size))
    cls = np.minimum(4, np.ceil(np.log2(np.maximum(n, 4) / 4)).astype(int))
    assert (np.diff(cls[order]) >= 0).all(), "classes out of order"
    for c in range(5):
        sel = order[cls[order] == c]
        assert (np.diff(sel) > 0).all(), "class %d not in target order" % c
        assert (n[sel] <= (4 << c)).all() or c == 4

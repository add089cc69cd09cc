"""The allocation-free reverse-play search of sokoban_gen.cpp (FastSearch: fixed arrays, 128-bit
grid keys in an open-addressing table) against the std::string-keyed search it replaces
(RMI_SOKOBAN_GEN_STRING_SEARCH=1), on rooms of every size RAGEN configures and a few more: the
same rooms, players and statuses, bit for bit.  Both follow depth_first_search
(sokoban/utils.py:440-498); the golden rooms of the reference pin the default path in
tests/test_oracle.py."""
import os

import numpy as np
import pytest

from ragen_amd import ops

CASES = [(6, 6, 1, 300, 400), (6, 6, 2, 300, 300), (8, 8, 2, 100, 200), (5, 7, 1, 50, 400),
         (10, 10, 3, 100, 40), (12, 12, 2, 60, 40), (3, 3, 1, 10, 50)]


def _gen(seeds, H, W, nb, sd, string_search):
    old = os.environ.get("RMI_SOKOBAN_GEN_STRING_SEARCH")
    os.environ["RMI_SOKOBAN_GEN_STRING_SEARCH"] = "1" if string_search else "0"
    try:
        return ops.generate_sokoban_rooms(seeds, H, W, nb, sd, 4)
    finally:
        if old is None:
            del os.environ["RMI_SOKOBAN_GEN_STRING_SEARCH"]
        else:
            os.environ["RMI_SOKOBAN_GEN_STRING_SEARCH"] = old


@pytest.mark.parametrize("H,W,nb,sd,n", CASES)
def test_fast_search_equals_string_search(H, W, nb, sd, n):
    seeds = np.arange(n, dtype=np.int64) * 7919 + 3 * H + W
    fast = _gen(seeds, H, W, nb, sd, False)
    ref = _gen(seeds, H, W, nb, sd, True)
    for a, b in zip(fast, ref):
        np.testing.assert_array_equal(a, b)


def _batch(H=6, W=6, nb=1, sd=100):
    from ragen_amd.env.configs import SokobanEnvConfig
    from ragen_amd.env.sokoban import SokobanBatch
    b = object.__new__(SokobanBatch)  # the host side of reset() only (no device tensors)
    b.config = SokobanEnvConfig(dim_x=W, dim_y=H, num_boxes=nb, search_depth=sd)
    b.H, b.W = H, W
    return b


def test_prefetched_rooms_equal_generated():
    """SokobanBatch.prefetch: the rooms a prefetch made are the ones reset() would generate; a
    reset with other seeds ignores them and generates its own."""
    from ragen_amd.env.sokoban import SokobanBatch
    b = _batch()
    seeds = np.repeat(np.arange(40, dtype=np.int64) + 5000, 4)
    want = SokobanBatch.generate_unique(seeds, 6, 6, 1, 100)
    b.prefetch(seeds)
    for x, y in zip(b._rooms(seeds.copy()), want):
        np.testing.assert_array_equal(x, y)
    assert b._prefetched is None and b.reset_prefetched
    other = seeds + 1
    b.prefetch(seeds)
    for x, y in zip(b._rooms(other), SokobanBatch.generate_unique(other, 6, 6, 1, 100)):
        np.testing.assert_array_equal(x, y)
    assert not b.reset_prefetched


@pytest.mark.parametrize("order", ["sorted", "shuffled"])
def test_generate_unique_expands_to_per_seed_rooms(order):
    """generate_unique (each distinct seed once; sorted seeds without a sort) expanded by its
    inverse = the generator run on every seed."""
    from ragen_amd.env.sokoban import SokobanBatch
    seeds = np.repeat(np.arange(30, dtype=np.int64) * 13 + 7, 3)
    if order == "shuffled":
        seeds = np.random.default_rng(0).permutation(seeds)
    f, s_, p, st = ops.generate_sokoban_rooms(seeds, 6, 6, 1, 100, 2)
    assert not st.any()
    rows, inv = SokobanBatch.generate_unique(seeds, 6, 6, 1, 100)
    assert len(rows) == 30
    for x, y in zip(SokobanBatch.generate(seeds, 6, 6, 1, 100), (f, s_, p)):
        np.testing.assert_array_equal(x, y)
    np.testing.assert_array_equal(rows[inv, :36], f)


def test_prefetch_error_raised_by_the_reset_that_takes_it():
    b = _batch()
    bad = np.array([2 ** 33], np.int64)
    b.prefetch(bad)
    with pytest.raises(ValueError):
        b._rooms(bad)
    b.prefetch(bad)  # not taken: the other seeds generate, the prefetch's error is dropped
    assert b._rooms(np.array([7], np.int64))[0].shape == (1, 74)  # fixed | state | player


def test_rooms_job_equals_the_synchronous_generator():
    """ops.RoomsJob (rmi_sokoban_generate_rooms_start / _wait: the generator on a native host
    thread) writes the rooms the synchronous call writes; a job never waited on is joined when
    it is dropped."""
    seeds = np.arange(64, dtype=np.int64) * 31 + 11
    job = ops.RoomsJob(seeds, 6, 6, 1, 100, 3)
    for x, y in zip(job.wait(), ops.generate_sokoban_rooms(seeds, 6, 6, 1, 100, 2)):
        np.testing.assert_array_equal(x, y)
    with pytest.raises(RuntimeError):
        job.wait()
    ops.RoomsJob(seeds, 6, 6, 1, 100, 2)  # dropped at once: __del__ joins it
    with pytest.raises(ValueError):
        ops.RoomsJob(np.array([-1], np.int64), 6, 6, 1, 100).wait()

"""Host-side pieces of the turn chain that run without a GPU: rmi_host_live_ids (the survivors'
env ids from a turn's read-back flags, es_manager.py:168-169) against numpy, and the formulate
chain's argument checks."""
import numpy as np
import pytest

from ragen_amd import _lib


@pytest.mark.parametrize("n,lo", [(8192, 0), (1000, 4096), (1, 7), (0, 0)])
def test_host_live_ids_equals_numpy(n, lo):
    rng = np.random.default_rng(n + lo)
    flags = rng.integers(0, 8, size=n).astype(np.uint8)
    want = lo + np.flatnonzero((flags & _lib.FLAG_DONE) == 0)
    out = np.full(max(len(want), 1), -1, np.int64)
    k = _lib.lib().rmi_host_live_ids(flags.ctypes.data, n, _lib.FLAG_DONE, lo, out.ctypes.data, len(want))
    assert k == len(want) and (out[:k] == want).all()
    if len(want):  # a cap below the count is refused, not overrun
        short = np.full(len(want), -1, np.int64)
        assert _lib.lib().rmi_host_live_ids(flags.ctypes.data, n, _lib.FLAG_DONE, lo, short.ctypes.data,
                                            len(want) - 1) == -1


def test_formulate_chain_part_refuses_bad_arguments():
    """rmi_formulate_chain_part's argument checks return before any launch (no GPU needed): a
    missing chain, a part other than 1 / 2, an early-copy count outside [0, n_copies], more than
    four copies, and a chain without its episode record are RMI_EINVAL."""
    L = _lib.lib()
    c = _lib.FormulateChain()
    assert L.rmi_formulate_chain_part(None, 1, 0, None) == _lib.RMI_EINVAL
    for part in (0, 3, -1):
        assert L.rmi_formulate_chain_part(c, part, 0, None) == _lib.RMI_EINVAL
    assert L.rmi_formulate_chain_part(c, 1, 0, None) == _lib.RMI_EINVAL  # no ep / norm / tail
    c.n_copies = 5
    assert L.rmi_formulate_chain_part(c, 2, 0, None) == _lib.RMI_EINVAL
    c.n_copies = 2
    assert L.rmi_formulate_chain_part(c, 1, 3, None) == _lib.RMI_EINVAL
    assert L.rmi_formulate_chain_part(c, 1, -1, None) == _lib.RMI_EINVAL

"""rmi_readback into host buffers whose pinned registration changes between calls: the library
looks the buffer's device mapping up on every call (capi.hip host_mapping), so a buffer that was
pinned, then released and reused as pageable memory (or pinned again under a new mapping) must
still receive exactly the device bytes — a remembered mapping would make the readback kernel
store through a stale device address."""
import ctypes

import numpy as np
import pytest
import torch

from ragen_amd import _lib
from ragen_amd.ops import _stream

pytestmark = pytest.mark.gpu


def _hip():
    return ctypes.CDLL("libamdhip64.so")


def _read(dst_ptr, src, s):
    _lib.check(_lib.lib().rmi_readback(dst_ptr, src.data_ptr(), src.numel(), s), "rmi_readback")


def test_readback_after_host_unregister_and_reregister(device):
    hip = _hip()
    hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
    hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
    s = _stream(device)
    n = 1 << 16
    host = np.zeros(n + 4096, np.uint8)
    off = (-host.ctypes.data) % 4096  # a page-aligned window of the array
    win = host[off:off + n]
    ptr = win.ctypes.data
    g = torch.Generator(device="cpu").manual_seed(3)
    for round_ in range(3):
        a = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(device)
        assert hip.hipHostRegister(ptr, n, 0) == 0
        _read(ptr, a, s)  # pinned: the kernel path through the device mapping
        np.testing.assert_array_equal(win, a.cpu().numpy())
        assert hip.hipHostUnregister(ptr) == 0
        b = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(device)
        _read(ptr, b, s)  # the same address, pageable now: the runtime copy
        np.testing.assert_array_equal(win, b.cpu().numpy())
    torch.cuda.synchronize(device)


def test_readback_into_recycled_pinned_tensors(device):
    """torch's pinned buffers released and flushed from its host cache, then allocated again
    (often at the same address, under a new mapping): every readback lands."""
    s = _stream(device)
    g = torch.Generator(device="cpu").manual_seed(5)
    n = 3 << 16
    for i in range(6):
        pin = torch.empty(n, dtype=torch.uint8, pin_memory=True)
        a = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(device)
        _read(pin.data_ptr(), a, s)
        assert torch.equal(pin, a.cpu())
        del pin
        torch.cuda.synchronize(device)
        if hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()

"""The one-shot all-gather of the per-rank episode arena (include/ragen_amd.h,
"the one-shot arena exchange").

The reference's trainer needs the WHOLE rollout batch before compute_advantage and the update,
every iteration (agent_trainer.py:514-515, 623-655).  With the env batch sharded over the ranks
of one node that is an all-gather of every rank's episode arena after every rollout.  RCCL's
ring all-gather (``distributed.gather_bytes``) moves a rank's bytes over W-1 serial hops; on the
MI355X node's full xGMI mesh one direct hop suffices: each rank stores its arena into every
rank's receive region (all links at once) and publishes an arrival count, and a rank's gather is
complete when every sender's count reached the epoch's.  ``ArenaExchange`` owns this rank's
region, maps the peers' regions once (HIP IPC handles exchanged over the process group) and runs
one kernel per exchange (``rmi_xgather``).  ``in_process`` builds W ranks' exchanges inside one
process on one device (tests: the same kernel and protocol without IPC).

Stream order is the whole contract: an exchange launched after the rollout on the same stream
reads the finished arena, and everything launched after it sees the gathered slot.  The slot of
exchange number e (1, 2, ...) is ``slot(e)``: a u8[W, nbytes] view of this rank's region, valid
until exchange e + 2 is launched on this rank (the slot is then rewritten by the senders).
"""
import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from . import _lib

HANDLE_BYTES = 64
MODES = {"uncached": _lib.XG_MEM_UNCACHED, "finegrained": _lib.XG_MEM_FINEGRAINED}


def region_bytes(world: int, nbytes: int) -> int:
    v = int(_lib.lib().rmi_xgather_region_bytes(int(world), int(nbytes)))
    if v < 0:
        raise ValueError(f"no exchange region for world {world}, {nbytes} B")
    return v


def slot_offset(world: int, nbytes: int, epoch: int) -> int:
    v = int(_lib.lib().rmi_xgather_slot_offset(int(world), int(nbytes), int(epoch)))
    if v < 0:
        raise ValueError(f"no slot for world {world}, {nbytes} B, epoch {epoch}")
    return v


def row_bytes(nbytes: int) -> int:
    """Bytes between consecutive ranks' rows of a slot (nbytes rounded up to 4096)."""
    return -(-int(nbytes) // 4096) * 4096


def plan(world: int, nbytes: int) -> dict:
    """The exchange's layout and launch shape for `world` ranks of `nbytes` each (host-side
    arithmetic of the library; identical on every rank, so no rank needs to ask another)."""
    nb = int(_lib.lib().rmi_xgather_blocks_per_peer(int(nbytes)))
    return {"world": int(world), "nbytes": int(nbytes), "row_bytes": row_bytes(nbytes),
            "region_bytes": region_bytes(world, nbytes), "slot_offsets": [slot_offset(world, nbytes, e) for e in (1, 2)],
            "blocks_per_peer": nb, "grid": int(world) * nb + 1,
            "bytes_stored_per_rank": int(world) * int(nbytes)}


def exchange_handles(handle: bytes, group=None) -> List[bytes]:
    """Every rank's 64-B region handle in rank order: one all-gather over the process group
    (gloo moves host tensors, RCCL device tensors).  Without a process group: [handle]."""
    handle = bytes(handle)
    if len(handle) != HANDLE_BYTES:
        raise ValueError(f"a region handle is {HANDLE_BYTES} bytes, got {len(handle)}")
    if not (dist.is_available() and dist.is_initialized()):
        return [handle]
    W = dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    mine = torch.tensor(list(handle), dtype=torch.uint8, device=dev)
    every = torch.empty(W * HANDLE_BYTES, dtype=torch.uint8, device=dev)
    dist.all_gather_into_tensor(every, mine, group=group)
    flat = bytes(every.cpu().tolist())
    return [flat[q * HANDLE_BYTES:(q + 1) * HANDLE_BYTES] for q in range(W)]


# ---------------------------------------------------------------- raw device memory as a tensor
class _DLDevice(ctypes.Structure):
    _fields_ = [("device_type", ctypes.c_int32), ("device_id", ctypes.c_int32)]


class _DLDataType(ctypes.Structure):
    _fields_ = [("code", ctypes.c_uint8), ("bits", ctypes.c_uint8), ("lanes", ctypes.c_uint16)]


class _DLTensor(ctypes.Structure):
    _fields_ = [("data", ctypes.c_void_p), ("device", _DLDevice), ("ndim", ctypes.c_int32), ("dtype", _DLDataType),
                ("shape", ctypes.POINTER(ctypes.c_int64)), ("strides", ctypes.POINTER(ctypes.c_int64)),
                ("byte_offset", ctypes.c_uint64)]


class _DLManagedTensor(ctypes.Structure):
    _fields_ = [("dl_tensor", _DLTensor), ("manager_ctx", ctypes.c_void_p), ("deleter", ctypes.c_void_p)]


_K_DL_ROCM, _K_DL_UINT = 10, 1


def device_bytes(ptr: int, nbytes: int, device: torch.device, keep: list) -> torch.Tensor:
    """u8[nbytes] tensor over device memory this module allocated or mapped (no copy).  The
    memory's owner must outlive the tensor; `keep` holds the DLPack structs it points at."""
    shape = (ctypes.c_int64 * 1)(int(nbytes))
    m = _DLManagedTensor()
    m.dl_tensor.data = ctypes.c_void_p(int(ptr))
    m.dl_tensor.device = _DLDevice(_K_DL_ROCM, device.index or 0)
    m.dl_tensor.ndim = 1
    m.dl_tensor.dtype = _DLDataType(_K_DL_UINT, 8, 1)
    m.dl_tensor.shape = shape
    m.dl_tensor.strides = None
    m.dl_tensor.byte_offset = 0
    m.manager_ctx = None
    m.deleter = None
    keep.extend([shape, m])
    new = ctypes.pythonapi.PyCapsule_New
    new.restype = ctypes.py_object
    new.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p]
    cap = new(ctypes.addressof(m), b"dltensor", None)
    t = torch.utils.dlpack.from_dlpack(cap)
    if t.device != device or t.numel() != nbytes:
        raise RuntimeError(f"DLPack view landed on {t.device} / {t.numel()} B, expected {device} / {nbytes} B")
    return t


def agree(ok: bool, group=None) -> bool:
    """True on every rank iff `ok` on every rank (an all-reduce MIN over the process group; the
    local value without one).  Keeps a failure on one rank from leaving the others blocked in
    a later collective of the setup."""
    if not (dist.is_available() and dist.is_initialized()):
        return bool(ok)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _stream_ptr(device, stream):
    s = stream if stream is not None else torch.cuda.current_stream(device)
    return ctypes.c_void_p(s.cuda_stream)


class ArenaExchange:
    """One rank's side of the one-shot exchange of `nbytes` per rank.

    group: the process group whose ranks exchange (None: the default group if initialised, else a
    1-rank exchange).  mode: "finegrained" (default) or "uncached" receive memory (measurement
    only: it served stale rows in one process after earlier regions were freed).  Every rank
    must construct it (collective: the handle exchange)."""

    def __init__(self, nbytes: int, device, group=None, mode: str = "finegrained", timeout_us: int = 2_000_000,
                 blocks_per_peer: int = 0, _regions=None, _rank=None, _world=None):
        self.device = torch.device(device)
        self.nbytes = int(nbytes)
        if self.nbytes < 16 or self.nbytes % 16:
            raise ValueError("the exchanged bytes must be a positive multiple of 16")
        self.mode = mode
        self._keep: list = []
        self._opened: list = []
        self._owned: Optional[int] = None
        L = _lib.lib()
        if _regions is None:  # one rank per process: own region + the peers' through IPC
            init = dist.is_available() and dist.is_initialized()
            self.world = dist.get_world_size(group) if init else 1
            self.rank = dist.get_rank(group) if init else 0
            if self.world > _lib.XG_MAX_RANKS:
                raise ValueError(f"at most {_lib.XG_MAX_RANKS} ranks")
            nreg = region_bytes(self.world, self.nbytes)
            p = ctypes.c_void_p()
            h = (ctypes.c_uint8 * HANDLE_BYTES)()
            # collective all the way: every rank learns whether every rank's step succeeded before
            # the next collective, so one rank's failure raises everywhere instead of hanging
            with torch.cuda.device(self.device):
                rc = L.rmi_xgather_alloc(nreg, MODES[mode], ctypes.byref(p), h)
                if rc == _lib.RMI_OK:
                    self._owned = p.value
                if not agree(rc == _lib.RMI_OK, group):
                    self.close()
                    raise RuntimeError(f"rmi_xgather_alloc failed on some rank (here: code {rc})")
                handles = exchange_handles(bytes(h), group)
                regions, bad = [], []
                for q, hq in enumerate(handles):
                    if q == self.rank:
                        regions.append(self._owned)
                        continue
                    r = ctypes.c_void_p()
                    buf = (ctypes.c_uint8 * HANDLE_BYTES).from_buffer_copy(hq)
                    rc = L.rmi_xgather_open(buf, ctypes.byref(r))
                    if rc == _lib.RMI_OK:
                        self._opened.append(r.value)
                    else:
                        bad.append(q)
                    regions.append(r.value)
                if not agree(not bad, group):
                    self.close()
                    raise RuntimeError(f"rmi_xgather_open failed on some rank (here: ranks {bad})")
        else:  # in_process: the caller's regions, no IPC
            self.world, self.rank, regions = int(_world), int(_rank), list(_regions)
        self.regions = regions
        self.state = torch.zeros(2, dtype=torch.int64, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        x = _lib.XGather()
        x.world, x.rank, x.nbytes = self.world, self.rank, self.nbytes
        for q, r in enumerate(regions):
            x.region[q] = r
        x.state, x.err = self.state.data_ptr(), self.err.data_ptr()
        x.timeout_us = int(timeout_us)
        x.blocks_per_peer = int(blocks_per_peer)
        self.x = x
        self.epoch = 0  # exchanges launched through run() (graph replays: advance())
        self._view = device_bytes(regions[self.rank], region_bytes(self.world, self.nbytes), self.device, self._keep)

    @classmethod
    def in_process(cls, world: int, nbytes: int, device, mode: str = "finegrained", **kw) -> List["ArenaExchange"]:
        """W ranks' exchanges in ONE process on one device (no IPC): regions allocated here, each
        rank's pointer table holding all W.  Launch every rank's PUBLISH before any WAIT when they
        share a stream (a rank's WAIT needs every sender's PUBLISH)."""
        L = _lib.lib()
        device = torch.device(device)
        nreg = region_bytes(world, nbytes)
        regs = []
        with torch.cuda.device(device):
            for _ in range(world):
                p = ctypes.c_void_p()
                h = (ctypes.c_uint8 * HANDLE_BYTES)()
                _lib.check(L.rmi_xgather_alloc(nreg, MODES[mode], ctypes.byref(p), h), "rmi_xgather_alloc")
                regs.append(p.value)
        exs = [cls(nbytes, device, mode=mode, _regions=regs, _rank=r, _world=world, **kw) for r in range(world)]
        for e, p in zip(exs, regs):
            e._owned = p
        return exs

    def run(self, src: torch.Tensor, flags: int = _lib.XG_PUBLISH | _lib.XG_WAIT, stream=None) -> None:
        """Enqueue one exchange half (or both) of src (u8, contiguous, nbytes) on the stream."""
        if flags & _lib.XG_PUBLISH:
            if src is None or src.device != self.device or not src.is_contiguous() or \
                    src.numel() * src.element_size() != self.nbytes:
                raise ValueError("src must be a contiguous device tensor of exactly nbytes on the exchange's device")
        ptr = src.data_ptr() if src is not None else None
        _lib.check(_lib.lib().rmi_xgather(ctypes.byref(self.x), ptr, int(flags), _stream_ptr(self.device, stream)),
                   "rmi_xgather")
        if flags & _lib.XG_WAIT:
            self.epoch += 1

    def sync_epoch(self) -> int:
        """Set the host mirror from the device's epoch counter (after launches that were not made
        through run(), e.g. during graph capture, which records launches without running them)."""
        torch.cuda.synchronize(self.device)
        self.epoch = int(self.state[0].item())
        return self.epoch

    def advance(self, n: int) -> None:
        """Host mirror of exchanges launched outside run() (a captured graph replayed n times)."""
        self.epoch += int(n)

    def slot(self, epoch: Optional[int] = None) -> torch.Tensor:
        """u8[W, nbytes] view of the gathered rows of exchange `epoch` (default: the last one)."""
        e = self.epoch if epoch is None else int(epoch)
        if e < 1:
            raise ValueError("no exchange has run")
        off = slot_offset(self.world, self.nbytes, e)
        rb = row_bytes(self.nbytes)
        return self._view[off:off + self.world * rb].view(self.world, rb)[:, :self.nbytes]

    def error(self) -> int:
        """RMI_XG_ERR_* bits set by any exchange so far (a device -> host read)."""
        return int(self.err.item())

    def close(self) -> None:
        L = _lib.lib()
        self._view = None
        for r in self._opened:
            L.rmi_xgather_close(ctypes.c_void_p(r))
        self._opened = []
        if self._owned:
            L.rmi_xgather_free(ctypes.c_void_p(self._owned))
            self._owned = None


def close_all(exs) -> None:
    for e in exs:
        e.close()

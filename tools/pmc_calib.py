"""PMC calibration on the Sokoban turn kernel's own access patterns (run under rocprofv3 --pmc).

    python tools/pmc_calib.py build          # hipcc tools/pmc_calib.hip -> tools/_build/libpmc_calib.so
    rocprofv3 --pmc FETCH_SIZE --kernel-trace -- python3 tools/pmc_calib.py
    rocprofv3 --pmc WRITE_SIZE --kernel-trace -- python3 tools/pmc_calib.py

Each kernel runs 3 times over buffers well past the 256 MiB Infinity Cache (B = 16 M rows of
36 B = 604 MB), so the counters see HBM traffic; the known bytes per launch are printed."""
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "_build", "libpmc_calib.so")
B = 16 << 20


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-O3",
                    os.path.join(ROOT, "tools", "pmc_calib.hip"), "-o", SO], check=True)


def main():
    import torch
    lib = ctypes.CDLL(SO)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    rows = torch.randint(0, 255, (B * 36,), dtype=torch.uint8, device=dev)
    out = torch.empty(B, dtype=torch.int32, device=dev)
    bx = torch.randint(0, 255, (4 * B,), dtype=torch.uint8, device=dev)
    bo = torch.empty_like(bx)
    f = torch.zeros(B, dtype=torch.float64, device=dev)
    for _ in range(3):
        lib.calib_rows36_read(ctypes.c_void_p(rows.data_ptr()), ctypes.c_int64(B), ctypes.c_void_p(out.data_ptr()),
                              ctypes.c_void_p(s))
        lib.calib_rows36_write(ctypes.c_void_p(rows.data_ptr()), ctypes.c_int64(B), 2, ctypes.c_void_p(s))
        lib.calib_bytes_read(ctypes.c_void_p(bx.data_ptr()), ctypes.c_int64(4 * B), ctypes.c_void_p(bo.data_ptr()),
                             ctypes.c_void_p(s))
        lib.calib_f64_rw(ctypes.c_void_p(f.data_ptr()), ctypes.c_int64(B), ctypes.c_void_p(s))
    torch.cuda.synchronize()
    print(json.dumps({"rows36_read": {"read": 36 * B, "write": 4 * B},
                      "rows36_write": {"read": 0, "write_dwords": 2 * 4 * B, "rows_touched_bytes": 36 * B},
                      "bytes_read": {"read": 4 * B, "write": 4 * B},
                      "f64_rw": {"read": 8 * B, "write": 8 * B}}))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "build":
        build()
    else:
        main()

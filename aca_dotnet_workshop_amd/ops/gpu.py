"""ctypes bindings to the gfx950 query kernels (``_ttgpu.so``) operating on torch tensors.

No silent fallback: ``GpuKernels()`` raises if the library or a HIP device is missing; the
caller (``ops.columnar``) decides whether to use the CPU path instead, explicitly.
"""
from __future__ import annotations

import ctypes
from typing import Any

from .build import LIB, build_gpu

_lib = None


def load_library(build: bool = True) -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if build:
        build_gpu()
    if not LIB.exists():
        raise RuntimeError(f"GPU kernel library {LIB} is missing; run `python -m aca_dotnet_workshop_amd.ops.build`")
    lib = ctypes.CDLL(str(LIB))
    P, I64, I32 = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32
    lib.tt_launch_scan_eval.argtypes = [P, I64, I64, P, P, I32, P, P, P, P]
    lib.tt_launch_scan_eval.restype = ctypes.c_int
    lib.tt_launch_scan_compact.argtypes = [P, P, I64, P, P]
    lib.tt_launch_scan_compact.restype = ctypes.c_int
    lib.tt_launch_group_count.argtypes = [P, P, I64, I32, P, P]
    lib.tt_launch_group_count.restype = ctypes.c_int
    lib.tt_tile_rows.restype = ctypes.c_int
    _lib = lib
    return lib


class GpuKernels:
    def __init__(self, device: Any = None) -> None:
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("no HIP device available")
        self.torch = torch
        self.lib = load_library()
        self.device = torch.device(device or "cuda")
        self.tile_rows = int(self.lib.tt_tile_rows())

    def _stream(self) -> ctypes.c_void_p:
        return ctypes.c_void_p(self.torch.cuda.current_stream(self.device).cuda_stream)

    def select(self, cols, live, nrows: int, prog, bitmaps, return_mask: bool = False):
        """Row indices (int32, ascending) of live rows satisfying ``prog``."""
        torch = self.torch
        tiles = (nrows + self.tile_rows - 1) // self.tile_rows
        if tiles == 0:
            empty = torch.empty(0, dtype=torch.int32, device=self.device)
            return (empty, None) if return_mask else empty
        assert cols.dtype == torch.int32 and cols.is_contiguous() and cols.shape[1] % self.tile_rows == 0
        assert live.dtype == torch.int32 and live.shape[0] == cols.shape[1]
        assert prog.dtype == torch.int32 and prog.ndim == 2 and prog.shape[1] == 4
        assert bitmaps.dtype == torch.int32 and bitmaps.numel() > 0
        mask = torch.empty(tiles * (self.tile_rows // 64), dtype=torch.int64, device=self.device)
        counts = torch.empty(tiles, dtype=torch.int32, device=self.device)
        rc = self.lib.tt_launch_scan_eval(cols.data_ptr(), cols.shape[1], nrows, live.data_ptr(), prog.data_ptr(),
                                          prog.shape[0], bitmaps.data_ptr(), mask.data_ptr(), counts.data_ptr(),
                                          self._stream())
        if rc != 0:
            raise RuntimeError(f"tt_scan_eval launch failed ({rc})")
        incl = torch.cumsum(counts, 0, dtype=torch.int64)
        total = int(incl[-1].item())
        offsets = incl - counts.to(torch.int64)
        out = torch.empty(max(total, 1), dtype=torch.int32, device=self.device)
        if total:
            rc = self.lib.tt_launch_scan_compact(mask.data_ptr(), offsets.data_ptr(), nrows, out.data_ptr(), self._stream())
            if rc != 0:
                raise RuntimeError(f"tt_scan_compact launch failed ({rc})")
        out = out[:total]
        return (out, mask) if return_mask else out

    def group_count(self, gcol, mask, nrows: int, ngroups: int):
        torch = self.torch
        counts = torch.zeros(max(ngroups, 1), dtype=torch.int32, device=self.device)
        rc = self.lib.tt_launch_group_count(gcol.data_ptr(), mask.data_ptr(), nrows, max(ngroups, 1), counts.data_ptr(),
                                            self._stream())
        if rc != 0:
            raise RuntimeError(f"tt_group_count launch failed ({rc})")
        return counts[:ngroups]

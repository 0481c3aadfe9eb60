"""ctypes binding of the CPU restatement (oracle/mas_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py.  Parity status: partially pinned (see
mas_oracle.h and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libmas_oracle.so")
_lib = None

_P = ctypes.c_void_p
_I = ctypes.c_int


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_create.restype = _P
        L.orc_create.argtypes = [_I, _I, _I, _I, _I]
        L.orc_destroy.argtypes = [_P]
        L.orc_set_threads.argtypes = [_P, _I]
        L.orc_allocate.argtypes = [_P, _P, _P, _P, _P, _P]
        L.orc_prepare.argtypes = [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I]
        L.orc_apply.argtypes = [_P, _P, _P]
        for name in ("orc_num_levels", "orc_natural_levels", "orc_total_clusters", "orc_capacity",
                     "orc_max_neighbors", "orc_num_stencils"):
            getattr(L, name).argtypes = [_P]
            getattr(L, name).restype = _I
        L.orc_level_size.argtypes = [_P, _P]
        L.orc_aabb.argtypes = [_P, _P, _P]
        for name in ("orc_morton", "orc_s2o", "orc_o2s", "orc_nbr_num", "orc_nbr", "orc_coarse_space_tables",
                     "orc_going_next", "orc_coarse_tables", "orc_fine_connect_mask", "orc_inv_packed",
                     "orc_stencil_index_mapped", "orc_mapped_r"):
            getattr(L, name).argtypes = [_P]
            getattr(L, name).restype = _P
        L.orc_block_matrix.argtypes = [_P, _I, _P]
        L.orc_block_inverse.argtypes = [_P, _I, _P]
        L.orc_morton_encode.argtypes = [ctypes.c_float, ctypes.c_float, ctypes.c_float]
        L.orc_morton_encode.restype = ctypes.c_uint64
        L.orc_clamp.argtypes = [ctypes.c_float] * 3
        L.orc_clamp.restype = ctypes.c_float
        for name in ("orc_min", "orc_max"):
            getattr(L, name).argtypes = [ctypes.c_float] * 2
            getattr(L, name).restype = ctypes.c_float
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _view(addr, dtype, count):
    if not addr or count == 0:
        return np.zeros(0, dtype=dtype)
    buf = (ctypes.c_char * (count * np.dtype(dtype).itemsize)).from_address(addr)
    return np.frombuffer(buf, dtype=dtype, count=count).copy()


class Oracle:
    """Mirrors the reference call order: allocate -> prepare -> apply."""

    def __init__(self, nV, nE=0, nF=0, max_levels=0, threads=1):
        self._L = lib()
        self.h = self._L.orc_create(nV, nE, nF, max_levels, threads)
        if not self.h:
            raise ValueError("orc_create failed (nV <= 0 or more than 5 levels)")
        self.nV, self.nE, self.nF = nV, nE, nF

    def __del__(self):
        if getattr(self, "h", None):
            self._L.orc_destroy(self.h)
            self.h = None

    def set_threads(self, n):
        self._L.orc_set_threads(self.h, n)

    def allocate(self, mesh):
        self._keep = (np.ascontiguousarray(mesh.pos, np.float32), np.ascontiguousarray(mesh.starts, np.int32),
                      np.ascontiguousarray(mesh.idx, np.int32), np.ascontiguousarray(mesh.edges, np.int32),
                      np.ascontiguousarray(mesh.faces, np.int32))
        rc = self._L.orc_allocate(self.h, *[_ptr(a) for a in self._keep])
        if rc:
            raise RuntimeError(f"orc_allocate rc={rc}")

    def prepare(self, mesh, ef=None, ee=None, vf=None, efC=None, eeC=None, vfC=None, fix_vf_bary=False):
        args = [np.ascontiguousarray(mesh.diag, np.float32), np.ascontiguousarray(mesh.off, np.float32),
                np.ascontiguousarray(mesh.starts, np.int32)]
        rc = self._L.orc_prepare(self.h, *[_ptr(a) for a in args], _ptr(ef), _ptr(ee), _ptr(vf),
                                 _ptr(efC), _ptr(eeC), _ptr(vfC), int(fix_vf_bary))
        if rc:
            raise RuntimeError(f"orc_prepare rc={rc}")

    def apply(self, r4):
        r4 = np.ascontiguousarray(r4, np.float32)
        z4 = np.zeros_like(r4)
        rc = self._L.orc_apply(self.h, _ptr(z4), _ptr(r4))
        if rc:
            raise RuntimeError(f"orc_apply rc={rc}")
        return z4

    # ---- introspection ----
    @property
    def num_levels(self):
        return self._L.orc_num_levels(self.h)

    @property
    def natural_levels(self):
        return self._L.orc_natural_levels(self.h)

    @property
    def total_clusters(self):
        return self._L.orc_total_clusters(self.h)

    @property
    def capacity(self):
        return self._L.orc_capacity(self.h)

    @property
    def num_stencils(self):
        return self._L.orc_num_stencils(self.h)

    def level_size(self):
        out = np.zeros(2 * (self.num_levels + 1), dtype=np.int32)
        self._L.orc_level_size(self.h, _ptr(out))
        return out.reshape(-1, 2)

    def maps(self):
        nV, L = self.nV, self.num_levels
        tc = self.total_clusters
        mx = self._L.orc_max_neighbors(self.h)
        return dict(
            morton=_view(self._L.orc_morton(self.h), np.uint64, nV),
            s2o=_view(self._L.orc_s2o(self.h), np.int32, nV),
            o2s=_view(self._L.orc_o2s(self.h), np.int32, nV),
            nbr_num=_view(self._L.orc_nbr_num(self.h), np.int32, nV),
            nbr=_view(self._L.orc_nbr(self.h), np.int32, mx * nV).reshape(mx, nV),
            coarse_space_tables=_view(self._L.orc_coarse_space_tables(self.h), np.int32, L * nV).reshape(L, nV),
            going_next=_view(self._L.orc_going_next(self.h), np.int32, tc),
            coarse_tables=_view(self._L.orc_coarse_tables(self.h), np.int32, 4 * nV).reshape(nV, 4),
            fine_connect_mask=_view(self._L.orc_fine_connect_mask(self.h), np.uint32, nV),
            level_size=self.level_size(),
        )

    def mapped_r(self):
        """m_mappedR after the last apply: [total_clusters, 4] (the residual hierarchy)."""
        return _view(self._L.orc_mapped_r(self.h), np.float32, 4 * self.total_clusters).reshape(-1, 4).copy()

    def block_matrix(self, blk):
        A = np.zeros((96, 96), dtype=np.float32)
        if self._L.orc_block_matrix(self.h, blk, _ptr(A)):
            raise IndexError(blk)
        return A

    def block_inverse(self, blk):
        B = np.zeros((96, 96), dtype=np.float32)
        if self._L.orc_block_inverse(self.h, blk, _ptr(B)):
            raise IndexError(blk)
        return B


def morton_encode(x, y, z):
    return int(lib().orc_morton_encode(x, y, z))

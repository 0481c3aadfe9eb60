"""Python binding of the MI355X MAS preconditioner C ABI (include/mas_capi.h).

Mirrors the reference plugin surface (SeSchwarzPreconditioner.h:37-178):

    P = SeSchwarzPreconditioner(max_levels=4)
    P.m_positions, P.m_neighbours, P.m_edges, P.m_faces = ...
    P.AllocatePrecoditioner(nV, nE, nF)
    P.PreparePreconditioner(diag, off, ranges, ef, ee, vf, efC, eeC, vfC)
    z = P.Preconditioning(None, r, 3 * nV)        # host arrays
    P.PreconditioningDevice(z_dev, r_dev, stream) # torch cuda tensors / raw pointers

The shared library is loaded from the package's lib/ directory; there is no
CPU fallback -- if the HIP library or a GPU is missing every call raises.
"""
from __future__ import annotations

import ctypes
import os
import warnings

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
LIB_DIR = os.path.join(PKG_ROOT, "lib")
LIB_PATH = os.path.join(LIB_DIR, os.environ.get("MAS_LIB_NAME", "libmas_amd.so"))  # dev: the probe build
FACADE_PATH = os.path.join(LIB_DIR, "libSeSchwarzPreconditioner.so")

MAS_OK = 0
STATUS = {0: "MAS_OK", -1: "MAS_ERR_ARG", -2: "MAS_ERR_HIP", -3: "MAS_ERR_CAPACITY", -4: "MAS_ERR_STATE",
          -5: "MAS_ERR_LEVELS", -6: "MAS_ERR_NOMEM", -7: "MAS_ERR_NO_DEVICE", -8: "MAS_ERR_COMM",
          -9: "MAS_ERR_NOT_SPD"}

# mas_allgather_fn(send, recv, bytes, stream, user) -> int
ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                ctypes.c_void_p)

# every entry point declared in include/mas_capi.h
EXPORTS = ["mas_version", "mas_create", "mas_destroy", "mas_last_error", "mas_allocate", "mas_prepare",
           "mas_prepare_device", "mas_apply", "mas_apply_device", "mas_set_profiling", "mas_profile_fine",
           "mas_profile_coarse", "mas_get_info",
           "mas_get_stats", "mas_get_maps", "mas_get_neighbors", "mas_get_block_matrix", "mas_get_block_inverse",
           "mas_get_packed_inverses",
           "mas_get_coarse_residual", "mas_set_prepare_shard", "mas_set_prepare_allgather", "mas_prepare_shard_rows",
           "mas_prepare_shard_complete",
           "mas_shard_plan", "mas_shard_setup", "mas_apply_shard_restrict", "mas_apply_shard_finish",
           "mas_apply_shard_fine", "mas_apply_shard_complete", "mas_shard_apply_device", "mas_allgather_loopback",
           "mas_rccl_unique_id",
           "mas_rccl_init", "mas_shard_apply_rccl",
           "mas_pcg_solve_device", "mas_pcg_solve", "mas_blob_size", "mas_save_blob", "mas_load_blob",
           "mas_blob_validate", "mas_dev_sort_pairs", "mas_dev_exclusive_scan", "mas_dev_contact_terms"]


class mas_config(ctypes.Structure):
    _fields_ = [("max_levels", ctypes.c_int), ("resort_period", ctypes.c_int), ("fix_vf_bary", ctypes.c_int),
                ("device", ctypes.c_int), ("keep_blocks", ctypes.c_int),
                ("reference_formation", ctypes.c_int), ("reference_restriction", ctypes.c_int),
                ("strict_spd", ctypes.c_int), ("host_register", ctypes.c_int),
                ("reserved", ctypes.c_int * 7)]


class mas_info(ctypes.Structure):
    _fields_ = [("num_verts", ctypes.c_int), ("num_edges", ctypes.c_int), ("num_faces", ctypes.c_int),
                ("num_levels", ctypes.c_int), ("natural_levels", ctypes.c_int), ("total_clusters", ctypes.c_int),
                ("num_blocks", ctypes.c_int), ("num_fine_blocks", ctypes.c_int), ("max_neighbors", ctypes.c_int),
                ("num_stencils", ctypes.c_int), ("level_size", ctypes.c_int * 18), ("inv_bytes", ctypes.c_int64),
                ("device_bytes", ctypes.c_int64)]


class mas_stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("allocate_ms", "prepare_ms", "prepare_levels_ms",
                                               "prepare_assemble_ms", "prepare_factor_ms")] + \
               [("apply_calls", ctypes.c_int64), ("profiled_applies", ctypes.c_int64)] + \
               [(n, ctypes.c_double) for n in ("apply_ms_avg", "pre_fine_ms_avg", "fine_ms_avg", "post_fine_ms_avg")] + \
               [("apply_mode", ctypes.c_int64), ("prepare_fine_ms", ctypes.c_double),
                ("factor_formation", ctypes.c_int64), ("hier_dirty_level", ctypes.c_int64),
                ("hier_rebuilt", ctypes.c_int64), ("prepare_fine_start_ms", ctypes.c_double),
                ("nonspd_blocks", ctypes.c_int64), ("wait_timeouts", ctypes.c_int64),
                ("prepare_complete_ms", ctypes.c_double), ("coarse_split", ctypes.c_int64),
                ("reserved", ctypes.c_int64 * 1)]


class mas_shard(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("rank", "world", "fine_block_begin", "fine_block_end", "vert_begin",
                                            "vert_end", "l1_begin", "l1_end", "seg_max")]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class mas_pcg_result(ctypes.Structure):
    _fields_ = [("iterations", ctypes.c_int), ("converged", ctypes.c_int), ("rel_residual", ctypes.c_double),
                ("true_rel_residual", ctypes.c_double), ("solve_ms", ctypes.c_double),
                ("first_pass_iterations", ctypes.c_int), ("replacements", ctypes.c_int),
                ("reserved", ctypes.c_int * 8)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "reserved"}


class MasError(RuntimeError):
    pass


class MasWarning(RuntimeWarning):
    """Prepare met a non-SPD pivot and kept going (mas_config.strict_spd = 0)."""


_lib = None


def lib():
    """Load libmas_amd.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise MasError(f"{LIB_PATH} not found: run `make -C {PKG_ROOT}` (or __graft_entry__.build())")
        # torch-ROCm ships its own libamdhip64.so.7 / libhsa-runtime64.so.  Load
        # torch first so libmas_amd.so binds to the same HIP runtime (same
        # soname) and device pointers can be shared with torch tensors.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        P, I = ctypes.c_void_p, ctypes.c_int
        L.mas_version.restype = I
        L.mas_create.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(mas_config)]
        L.mas_destroy.argtypes = [P]
        L.mas_last_error.argtypes = [P]
        L.mas_last_error.restype = ctypes.c_char_p
        L.mas_allocate.argtypes = [P, I, I, I, P, P, P, P, P]
        L.mas_prepare.argtypes = [P, P, P, P, P, P, P, P, P, P]
        L.mas_prepare_device.argtypes = [P, P, P, P, P, P, P, P, P, P, P]
        L.mas_apply.argtypes = [P, P, P]
        L.mas_apply_device.argtypes = [P, P, P, P]
        L.mas_set_profiling.argtypes = [P, I]
        L.mas_profile_fine.argtypes = [P, P, P, I, P, ctypes.POINTER(ctypes.c_double)]
        L.mas_profile_coarse.argtypes = [P, P, I, P, ctypes.POINTER(ctypes.c_double)]
        L.mas_get_info.argtypes = [P, ctypes.POINTER(mas_info)]
        L.mas_get_stats.argtypes = [P, ctypes.POINTER(mas_stats)]
        L.mas_get_maps.argtypes = [P, P, P, P, P, P, P, P]
        L.mas_get_neighbors.argtypes = [P, P, P]
        L.mas_get_block_matrix.argtypes = [P, I, P]
        L.mas_get_block_inverse.argtypes = [P, I, P]
        L.mas_get_packed_inverses.argtypes = [P, I, I, P]
        L.mas_get_coarse_residual.argtypes = [P, P]
        L.mas_set_prepare_shard.argtypes = [P, I, I]
        L.mas_set_prepare_allgather.argtypes = [P, ALLGATHER_FN, P]
        L.mas_prepare_shard_rows.argtypes = [P, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
        L.mas_prepare_shard_complete.argtypes = [P, P, P]
        L.mas_shard_plan.argtypes = [I, P, I, I, ctypes.POINTER(mas_shard)]
        L.mas_shard_setup.argtypes = [P, I, I, ctypes.POINTER(mas_shard)]
        L.mas_apply_shard_restrict.argtypes = [P, I, I, P, P, P]
        L.mas_apply_shard_finish.argtypes = [P, I, I, P, P, P, P]
        L.mas_apply_shard_fine.argtypes = [P, I, I, P, P, P]
        L.mas_apply_shard_complete.argtypes = [P, I, I, P, P, P]
        L.mas_shard_apply_device.argtypes = [P, I, I, ALLGATHER_FN, P, P, P, P]
        L.mas_rccl_unique_id.argtypes = [P]
        L.mas_rccl_init.argtypes = [P, P, I, I]
        L.mas_shard_apply_rccl.argtypes = [P, P, P, P]
        L.mas_dev_sort_pairs.argtypes = [P, P, P, P, P, I, I, I]
        L.mas_dev_exclusive_scan.argtypes = [P, P, P, I, I]
        L.mas_dev_contact_terms.argtypes = [P, P, P, P, P, I]
        F = ctypes.c_float
        L.mas_pcg_solve_device.argtypes = [P, P, P, P, P, P, I, F, I, ctypes.POINTER(mas_pcg_result), P]
        L.mas_pcg_solve.argtypes = [P, P, P, P, P, P, I, F, I, ctypes.POINTER(mas_pcg_result)]
        L.mas_blob_size.argtypes = [P, ctypes.POINTER(ctypes.c_size_t)]
        L.mas_save_blob.argtypes = [P, P, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.mas_load_blob.argtypes = [P, P, ctypes.c_size_t]
        L.mas_blob_validate.argtypes = [P, ctypes.c_size_t]
        _lib = L
    return _lib


def _ptr(a):
    if a is None:
        return None
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    if hasattr(a, "data_ptr"):  # torch tensor
        return ctypes.c_void_p(a.data_ptr())
    return a.ctypes.data_as(ctypes.c_void_p)


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def _host(a, dtype, count, width, name):
    """Host array -> C-contiguous `dtype` with exactly count*width elements
    (any shape, e.g. [n, 9] or [n, 3, 3]); raises MasError otherwise, so the
    C ABI never copies past the caller's buffer."""
    if a is None:
        raise MasError(f"{name}: missing array")
    if hasattr(a, "data_ptr"):
        raise MasError(f"{name}: host entry point given a torch tensor (use the *Device method)")
    arr = np.ascontiguousarray(a, dtype=dtype)
    if arr.size != count * width:
        raise MasError(f"{name}: expected {count} x {width} {np.dtype(dtype).name} elements, got shape {arr.shape}")
    return arr


def _dev(t, count, width, dtype_name, name):
    """Device operand: a raw pointer (int, trusted) or a torch tensor that must
    be on the GPU, C-contiguous, of the right dtype and count*width elements."""
    if t is None:
        raise MasError(f"{name}: missing device array")
    if isinstance(t, int):
        return t
    if not hasattr(t, "data_ptr"):
        raise MasError(f"{name}: expected a torch cuda tensor or a raw device pointer, got {type(t).__name__}")
    if not t.is_cuda:
        raise MasError(f"{name}: tensor is not on a GPU")
    if str(t.dtype) != "torch." + dtype_name:
        raise MasError(f"{name}: expected torch.{dtype_name}, got {t.dtype}")
    if not t.is_contiguous():
        raise MasError(f"{name}: tensor must be contiguous")
    if t.numel() != count * width:
        raise MasError(f"{name}: expected {count} x {width} elements, got shape {tuple(t.shape)}")
    return t


class SeSchwarzPreconditioner:
    """Reference-compatible surface (SE::SeSchwarzPreconditioner) on the GPU."""

    def __init__(self, max_levels: int = 0, resort_period: int = 0, fix_vf_bary: bool = False, device: int = -1,
                 keep_blocks: bool = False, reference_formation: bool = False, reference_restriction: bool = False,
                 strict_spd: bool = False, host_register: bool = False):
        self._L = lib()
        cfg = mas_config(max_levels, resort_period, int(fix_vf_bary), device, int(bool(keep_blocks)),
                         int(bool(reference_formation)), int(bool(reference_restriction)), int(bool(strict_spd)),
                         int(bool(host_register)))
        h = ctypes.c_void_p()
        rc = self._L.mas_create(ctypes.byref(h), ctypes.byref(cfg))
        if rc != MAS_OK:
            raise MasError(f"mas_create failed: {STATUS.get(rc, rc)}")
        self.h = h
        self.m_positions = None   # [nV, 4] float32
        self.m_edges = None       # [nE, 4] int32
        self.m_faces = None       # [nF, 4] int32
        self.m_neighbours = None  # (starts, idx) CSR
        self._keep = ()
        self._nV = 0              # set by AllocatePrecoditioner / load_blob
        self._nnz = 0
        self._allocated = False   # Allocate inputs present (a restored blob has none)
        self._plans = {}
        self._rows_pending = False  # a sharded Prepare's coarse-row exchange has not run yet
        self._shard_world = 1

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None and self.h.value:
                self._L.mas_destroy(self.h)
                self.h.value = None
        except Exception:  # interpreter shutdown
            pass

    def _need(self, what, allocated=False):
        """The C ABI's call-order error before any size check (sizes are known
        only after Allocate / a blob load)."""
        if not self._nV or (allocated and not self._allocated):
            raise MasError(f"{what} failed: MAS_ERR_STATE: " +
                           ("prepare before allocate" if allocated else "apply before prepare"))

    def _check(self, rc, what):
        if rc != MAS_OK:
            msg = self._L.mas_last_error(self.h)
            raise MasError(f"{what} failed: {STATUS.get(rc, rc)}: {msg.decode() if msg else ''}")

    def _warn_prepare(self, what):
        """A Prepare that met a non-SPD pivot without strict_spd keeps going, as
        the reference's void method does, with a MasWarning."""
        msg = self._L.mas_last_error(self.h)
        if msg and msg.startswith(b"warning:"):
            warnings.warn(f"{what}: {msg.decode()}", MasWarning, stacklevel=3)

    # ---- the reference's three methods ----
    def AllocatePrecoditioner(self, numVerts, numEdges, numFaces):
        if self.m_neighbours is None:
            raise MasError("AllocatePrecoditioner: m_neighbours (starts, idx) not set")
        starts, idx = self.m_neighbours
        pos = _host(self.m_positions, np.float32, numVerts, 4, "m_positions")
        starts = _host(starts, np.int32, numVerts + 1, 1, "m_neighbours starts")
        idx = _host(idx, np.int32, int(starts[-1]), 1, "m_neighbours idx")
        edges = None if self.m_edges is None else _host(self.m_edges, np.int32, numEdges, 4, "m_edges")
        faces = None if self.m_faces is None else _host(self.m_faces, np.int32, numFaces, 4, "m_faces")
        self._check(self._L.mas_allocate(self.h, numVerts, numEdges, numFaces, _ptr(pos), _ptr(starts), _ptr(idx),
                                         _ptr(edges), _ptr(faces)), "AllocatePrecoditioner")
        self._nV, self._nnz = int(numVerts), int(starts[-1])
        self._allocated = True

    AllocatePreconditioner = AllocatePrecoditioner

    def PreparePreconditioner(self, diagonal, csrOffDiagonals, csrRanges, efSets=None, eeSets=None, vfSets=None,
                              efCounts=None, eeCounts=None, vfCounts=None):
        self._need("PreparePreconditioner", allocated=True)
        nV, nnz = self._nV, self._nnz
        d = _host(diagonal, np.float32, nV, 9, "diagonal")
        o = _host(csrOffDiagonals, np.float32, nnz, 9, "csrOffDiagonals")
        r = _host(csrRanges, np.int32, nV + 1, 1, "csrRanges")
        efC, eeC, vfC = (_c(x, np.uint32) for x in (efCounts, eeCounts, vfCounts))
        for sets, cnt, name in ((efSets, efC, "ef"), (eeSets, eeC, "ee"), (vfSets, vfC, "vf")):
            n = int(cnt[-1]) if cnt is not None and cnt.size else 0
            if n and (sets is None or np.asarray(sets).nbytes < 48 * n):
                raise MasError(f"{name}Sets: {n} records of 48 B expected")
        self._plans = {}
        self._check(self._L.mas_prepare(self.h, _ptr(d), _ptr(o), _ptr(r), _ptr(efSets), _ptr(eeSets), _ptr(vfSets),
                                        _ptr(efC), _ptr(eeC), _ptr(vfC)), "PreparePreconditioner")
        self._warn_prepare("PreparePreconditioner")
        self._rows_pending = self._shard_world > 1 and self.prepare_shard_rows() is not None

    def PreparePreconditionerDevice(self, d_diag, d_off, d_ranges, efSets=None, eeSets=None, vfSets=None,
                                    efCounts=None, eeCounts=None, vfCounts=None, stream=None):
        """Device Hessian; contact records / counts may be host arrays or device
        tensors (e.g. a GPU collision pass's output buffers)."""
        efC, eeC, vfC = (x if (x is None or hasattr(x, "data_ptr") or isinstance(x, int)) else _c(x, np.uint32)
                         for x in (efCounts, eeCounts, vfCounts))
        self._need("PreparePreconditionerDevice", allocated=True)
        d_diag = _dev(d_diag, self._nV, 9, "float32", "d_diag")
        d_off = _dev(d_off, self._nnz, 9, "float32", "d_off")
        d_ranges = _dev(d_ranges, self._nV + 1, 1, "int32", "d_ranges")
        self._plans = {}
        self._check(self._L.mas_prepare_device(self.h, _ptr(d_diag), _ptr(d_off), _ptr(d_ranges), _ptr(efSets),
                                               _ptr(eeSets), _ptr(vfSets), _ptr(efC), _ptr(eeC), _ptr(vfC),
                                               _ptr(stream)), "PreparePreconditionerDevice")
        self._warn_prepare("PreparePreconditionerDevice")
        self._rows_pending = self._shard_world > 1 and self.prepare_shard_rows() is not None

    def Preconditioning(self, z, residual, dim=None):
        self._need("Preconditioning")
        nV = self._nV
        r = _host(residual, np.float32, nV, 4, "residual")
        if z is None:
            out = np.empty((nV, 4), np.float32)
        else:  # written in place: must be exactly the C layout
            if not (isinstance(z, np.ndarray) and z.dtype == np.float32 and z.flags.c_contiguous
                    and z.flags.writeable and z.size == nV * 4):
                raise MasError("Preconditioning: z must be a writable C-contiguous float32 array of nV x 4")
            out = z
        self._check(self._L.mas_apply(self.h, _ptr(out), _ptr(r)), "Preconditioning")
        return out

    def PreconditioningDevice(self, z, residual, stream=None):
        """z, residual: torch cuda float32 tensors [nV, 4] (or raw device pointers)."""
        self._need("PreconditioningDevice")
        z = _dev(z, self._nV, 4, "float32", "z")
        residual = _dev(residual, self._nV, 4, "float32", "residual")
        self._check(self._L.mas_apply_device(self.h, _ptr(z), _ptr(residual), _ptr(stream)), "PreconditioningDevice")

    # ---- the sharded coarse assembly (include/mas_capi.h, ABI 5) ----
    def prepare_shard_rows(self):
        """(device pointer, bytes) of this rank's coarse-row segment after a
        sharded Prepare, or None when no exchange is pending."""
        ptr, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc = self._L.mas_prepare_shard_rows(self.h, ctypes.byref(ptr), ctypes.byref(n))
        if rc == -4:  # MAS_ERR_STATE: nothing pending
            return None
        self._check(rc, "prepare_shard_rows")
        return int(ptr.value), int(n.value)

    def prepare_shard_complete(self, gathered, stream=None):
        """Unpack the allgathered segments ([world][bytes], device) and factor
        the blocks that needed them (synchronous)."""
        self._check(self._L.mas_prepare_shard_complete(self.h, _ptr(gathered), _ptr(stream)),
                    "prepare_shard_complete")
        self._rows_pending = False
        self._warn_prepare("prepare_shard_complete")

    def set_prepare_allgather(self, allgather):
        """allgather(send_ptr, recv_ptr, nbytes, stream_ptr) -> None, enqueued on
        that stream: a sharded Prepare then exchanges its coarse rows inside
        Prepare (mas_set_prepare_allgather); None removes it."""
        if allgather is None:
            fn = ALLGATHER_FN()
        else:
            def hook(send, recv, nbytes, strm, _user):
                try:
                    allgather(send, recv, nbytes, strm)
                    return 0
                except Exception:  # reported as MAS_ERR_COMM by the Prepare
                    return 1
            fn = ALLGATHER_FN(hook)
        self._prep_hook = fn  # the callback must outlive every Prepare that calls it
        self._check(self._L.mas_set_prepare_allgather(self.h, fn, None), "set_prepare_allgather")

    @property
    def rows_pending(self) -> bool:
        return self._rows_pending

    # ---- Morton-range sharding (include/mas_capi.h) ----
    def shard_setup(self, rank, world) -> dict:
        sh = mas_shard()
        self._check(self._L.mas_shard_setup(self.h, rank, world, ctypes.byref(sh)), "shard_setup")
        self._plans[(rank, world)] = sh.as_dict()  # valid until the next Prepare / blob load
        return dict(self._plans[(rank, world)])

    def _shard_vecs(self, rank, world, **kw):
        plan = self._plans.get((rank, world)) or self.shard_setup(rank, world)
        sizes = {"r": self._nV, "z": self._nV, "seg": plan["seg_max"], "gathered": world * plan["seg_max"]}
        return {k: _dev(v, sizes[k], 4, "float32", k) for k, v in kw.items()}

    def shard_restrict(self, rank, world, r, seg, stream=None):
        v = self._shard_vecs(rank, world, r=r, seg=seg)
        r, seg = v["r"], v["seg"]
        self._check(self._L.mas_apply_shard_restrict(self.h, rank, world, _ptr(r), _ptr(seg), _ptr(stream)),
                    "shard_restrict")

    def shard_finish(self, rank, world, gathered, r, z, stream=None):
        v = self._shard_vecs(rank, world, gathered=gathered, r=r, z=z)
        gathered, r, z = v["gathered"], v["r"], v["z"]
        self._check(self._L.mas_apply_shard_finish(self.h, rank, world, _ptr(gathered), _ptr(r), _ptr(z),
                                                   _ptr(stream)), "shard_finish")

    def shard_fine(self, rank, world, r, z, stream=None):
        """Overlapped step 3a: own level-0 blocks, z = Z0 (no coarse terms)."""
        v = self._shard_vecs(rank, world, r=r, z=z)
        r, z = v["r"], v["z"]
        self._check(self._L.mas_apply_shard_fine(self.h, rank, world, _ptr(r), _ptr(z), _ptr(stream)), "shard_fine")

    def shard_complete(self, rank, world, gathered, z, stream=None):
        """Overlapped step 3b: coarse levels from the gathered segments, z += prolongation."""
        v = self._shard_vecs(rank, world, gathered=gathered, z=z)
        gathered, z = v["gathered"], v["z"]
        self._check(self._L.mas_apply_shard_complete(self.h, rank, world, _ptr(gathered), _ptr(z), _ptr(stream)),
                    "shard_complete")

    def shard_apply(self, rank, world, z, r, allgather=None, stream=None):
        """One call per rank and apply (mas_shard_apply_device): restrict, the
        allgather hook on the library's communication stream while the own
        level-0 blocks run, then the coarse levels + prolongation.
        allgather(send_ptr, recv_ptr, nbytes, stream_ptr) -> None enqueues the
        gather on that stream (raise to fail); None only for world == 1."""
        v = self._shard_vecs(rank, world, r=r, z=z)
        r, z = v["r"], v["z"]
        err = []

        def hook(send, recv, nbytes, strm, _user):
            try:
                allgather(send, recv, nbytes, strm)
                return 0
            except Exception as e:  # reported as MAS_ERR_COMM
                err.append(e)
                return 1

        fn = ALLGATHER_FN(hook) if allgather is not None else ALLGATHER_FN()
        rc = self._L.mas_shard_apply_device(self.h, rank, world, fn, None, _ptr(z), _ptr(r), _ptr(stream))
        if err:
            raise MasError(f"shard_apply: allgather hook failed: {err[0]!r}") from err[0]
        self._check(rc, "shard_apply")

    def shard_apply_loopback(self, rank, world, z, r, stream=None):
        """mas_shard_apply_device with the library's one-process stand-in for
        the collective (mas_allgather_loopback: only this rank's slot of the
        gathered buffer is written): per-rank timing / tests on one GPU."""
        v = self._shard_vecs(rank, world, r=r, z=z)
        r, z = v["r"], v["z"]
        fn = ALLGATHER_FN(ctypes.cast(self._L.mas_allgather_loopback, ctypes.c_void_p).value)
        rk = ctypes.c_int(rank)
        self._check(self._L.mas_shard_apply_device(self.h, rank, world, fn, ctypes.cast(ctypes.pointer(rk), ctypes.c_void_p), _ptr(z), _ptr(r),
                                                   _ptr(stream)), "shard_apply_loopback")

    def rccl_init(self, unique_id: bytes, rank, world):
        """Give the handle its own RCCL communicator (mas_rccl_init)."""
        buf = ctypes.create_string_buffer(bytes(unique_id), 128)
        self._check(self._L.mas_rccl_init(self.h, buf, rank, world), "rccl_init")

    def shard_apply_rccl(self, z, r, stream=None):
        """mas_shard_apply_rccl: the one-call sharded apply over the handle's RCCL communicator."""
        z = _dev(z, self._nV, 4, "float32", "z")
        r = _dev(r, self._nV, 4, "float32", "r")
        self._check(self._L.mas_shard_apply_rccl(self.h, _ptr(z), _ptr(r), _ptr(stream)), "shard_apply_rccl")

    # ---- GPU-resident PCG (include/mas_capi.h) ----
    def pcg_solve(self, diagonal, csrOffDiagonals, csrRanges, b, x0=None, max_iters=1000, tol=1e-5,
                  precondition=True):
        """Host arrays: returns (x [nV,4] float32, result dict)."""
        self._need("pcg_solve", allocated=True)
        nV, nnz = self._nV, self._nnz
        d = _host(diagonal, np.float32, nV, 9, "diagonal")
        o = _host(csrOffDiagonals, np.float32, nnz, 9, "csrOffDiagonals")
        r = _host(csrRanges, np.int32, nV + 1, 1, "csrRanges")
        bb = _host(b, np.float32, nV, 4, "b")
        x = np.zeros_like(bb) if x0 is None else np.array(_host(x0, np.float32, nV, 4, "x0"), copy=True)
        res = mas_pcg_result()
        self._check(self._L.mas_pcg_solve(self.h, _ptr(d), _ptr(o), _ptr(r), _ptr(x), _ptr(bb), int(max_iters),
                                          float(tol), int(bool(precondition)), ctypes.byref(res)), "pcg_solve")
        return x, res.as_dict()

    def pcg_solve_device(self, d_diag, d_off, d_ranges, x, b, max_iters=1000, tol=1e-5, precondition=True,
                         stream=None) -> dict:
        """Device arrays (torch cuda tensors or raw pointers); x is updated in place."""
        self._need("pcg_solve_device", allocated=True)
        nV = self._nV
        d_diag = _dev(d_diag, nV, 9, "float32", "d_diag")
        d_off = _dev(d_off, self._nnz, 9, "float32", "d_off")
        d_ranges = _dev(d_ranges, nV + 1, 1, "int32", "d_ranges")
        x = _dev(x, nV, 4, "float32", "x")
        b = _dev(b, nV, 4, "float32", "b")
        res = mas_pcg_result()
        self._check(self._L.mas_pcg_solve_device(self.h, _ptr(d_diag), _ptr(d_off), _ptr(d_ranges), _ptr(x),
                                                 _ptr(b), int(max_iters), float(tol), int(bool(precondition)),
                                                 ctypes.byref(res), _ptr(stream)), "pcg_solve_device")
        return res.as_dict()

    # ---- fixture / wire format ----
    def save_blob(self) -> np.ndarray:
        """The prepared handle as a versioned blob (uint8 array)."""
        n = ctypes.c_size_t()
        self._check(self._L.mas_blob_size(self.h, ctypes.byref(n)), "blob_size")
        buf = np.empty(n.value, dtype=np.uint8)
        w = ctypes.c_size_t()
        self._check(self._L.mas_save_blob(self.h, _ptr(buf), n.value, ctypes.byref(w)), "save_blob")
        return buf[: w.value]

    def load_blob(self, blob):
        b = np.ascontiguousarray(np.frombuffer(blob, dtype=np.uint8) if isinstance(blob, (bytes, bytearray))
                                 else blob, dtype=np.uint8)
        self._plans = {}
        self._check(self._L.mas_load_blob(self.h, _ptr(b), b.nbytes), "load_blob")
        self._nV, self._nnz = self.info()["num_verts"], 0  # a restored handle applies; Prepare needs Allocate
        self._allocated = False

    # ---- introspection ----
    def set_profiling(self, on: bool):
        self._check(self._L.mas_set_profiling(self.h, int(on)), "set_profiling")

    def profile_fine(self, z, r, n, stream=None) -> float:
        """Average ms of the level-0 kernel alone over n back-to-back launches (mas_profile_fine)."""
        self._need("profile_fine")
        z = _dev(z, self._nV, 4, "float32", "z")
        r = _dev(r, self._nV, 4, "float32", "r")
        out = ctypes.c_double()
        self._check(self._L.mas_profile_fine(self.h, _ptr(z), _ptr(r), int(n), _ptr(stream), ctypes.byref(out)),
                    "profile_fine")
        return out.value

    def profile_coarse(self, r, n, stream=None) -> float:
        """Average ms of an apply's coarse launch(es) alone over n back-to-back applies' worth (mas_profile_coarse)."""
        self._need("profile_coarse")
        r = _dev(r, self._nV, 4, "float32", "r")
        out = ctypes.c_double()
        self._check(self._L.mas_profile_coarse(self.h, _ptr(r), int(n), _ptr(stream), ctypes.byref(out)),
                    "profile_coarse")
        return out.value

    def info(self) -> dict:
        i = mas_info()
        self._check(self._L.mas_get_info(self.h, ctypes.byref(i)), "get_info")
        d = {k: getattr(i, k) for k, _ in mas_info._fields_ if k != "level_size"}
        d["level_size"] = np.array(i.level_size[: 2 * (i.num_levels + 1)], dtype=np.int32).reshape(-1, 2)
        return d

    def stats(self) -> dict:
        s = mas_stats()
        self._check(self._L.mas_get_stats(self.h, ctypes.byref(s)), "get_stats")
        return {k: getattr(s, k) for k, _ in mas_stats._fields_ if k != "reserved"}

    def maps(self) -> dict:
        inf = self.info()
        nV, L, tc = inf["num_verts"], inf["num_levels"], inf["total_clusters"]
        out = dict(morton=np.zeros(nV, np.uint64), s2o=np.zeros(nV, np.int32), o2s=np.zeros(nV, np.int32),
                   coarse_space_tables=np.zeros((L, nV), np.int32), going_next=np.zeros(tc, np.int32),
                   coarse_tables=np.zeros((nV, 4), np.int32), fine_connect_mask=np.zeros(nV, np.uint32))
        self._check(self._L.mas_get_maps(self.h, *[_ptr(out[k]) for k in ("morton", "s2o", "o2s",
                                                                          "coarse_space_tables", "going_next",
                                                                          "coarse_tables", "fine_connect_mask")]),
                    "get_maps")
        mx = inf["max_neighbors"]
        out["nbr_num"] = np.zeros(nV, np.int32)
        out["nbr"] = np.zeros((mx, nV), np.int32)
        self._check(self._L.mas_get_neighbors(self.h, _ptr(out["nbr_num"]), _ptr(out["nbr"])), "get_neighbors")
        out["level_size"] = inf["level_size"]
        return out

    def block_matrix(self, blk):
        A = np.zeros((96, 96), np.float32)
        self._check(self._L.mas_get_block_matrix(self.h, blk, _ptr(A)), "get_block_matrix")
        return A

    def block_inverse(self, blk):
        B = np.zeros((96, 96), np.float32)
        self._check(self._L.mas_get_block_inverse(self.h, blk, _ptr(B)), "get_block_inverse")
        return B

    def set_prepare_shard(self, rank: int, world: int):
        """Later Prepares factor only the level-0 blocks of shard rank/world (mas_set_prepare_shard)."""
        self._check(self._L.mas_set_prepare_shard(self.h, int(rank), int(world)), "set_prepare_shard")
        self._shard_world = int(world)

    def packed_inverses(self, blk0: int, nblk: int) -> np.ndarray:
        """Blocks [blk0, blk0 + nblk)'s inverses as stored, [nblk, 4656] float32."""
        out = np.empty((nblk, 4656), np.float32)
        self._check(self._L.mas_get_packed_inverses(self.h, int(blk0), int(nblk), _ptr(out)), "packed_inverses")
        return out

    def coarse_residual(self):
        """R of every coarse node (ids begin_1 .. total_clusters-1) after the last apply, [n, 4] float32."""
        info = self.info()
        begin1 = int(info["level_size"].reshape(-1)[3])
        n = info["total_clusters"] - begin1
        R = np.zeros((max(n, 0), 4), np.float32)
        if n > 0:
            self._check(self._L.mas_get_coarse_residual(self.h, _ptr(R)), "get_coarse_residual")
        return R


def from_mesh(mesh, max_levels=0, contacts=None, shard=None, **kw) -> SeSchwarzPreconditioner:
    """Allocate + Prepare a preconditioner for a meshgen.Mesh (host path).
    shard=(rank, world): a sharded Prepare (only that shard's level-0 blocks)."""
    P = SeSchwarzPreconditioner(max_levels=max_levels, **kw)
    if shard is not None:
        P.set_prepare_shard(*shard)
    P.m_positions = mesh.pos
    P.m_neighbours = (mesh.starts, mesh.idx)
    P.m_edges = mesh.edges
    P.m_faces = mesh.faces
    P.AllocatePrecoditioner(mesh.nV, mesh.edges.shape[0], mesh.faces.shape[0])
    if contacts is None:
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts)
    else:
        vf, vfC = contacts
        P.PreparePreconditioner(mesh.diag, mesh.off, mesh.starts, None, None, vf, None, None, vfC)
    return P


def exchange_coarse_rows(handles, stream=None):
    """The coarse-row exchange of a world of shard-prepared handles that all
    live in this process (virtual shards on one GPU, tests and per-rank
    timing): the ranks' segments concatenated in rank order, as an allgather
    delivers them, then prepare_shard_complete on every handle.  Returns the
    gathered buffer (a torch uint8 cuda tensor)."""
    import torch
    from .distributed import device_view
    segs = [P.prepare_shard_rows() for P in handles]
    if any(sg is None for sg in segs):
        raise MasError("exchange_coarse_rows: a handle has no coarse rows pending")
    nbytes = segs[0][1]
    if any(sg[1] != nbytes for sg in segs):
        raise MasError("exchange_coarse_rows: the handles' segment sizes differ (not one world)")
    dev = torch.device("cuda", torch.cuda.current_device())
    gathered = torch.empty(len(handles) * nbytes // 4, dtype=torch.float32, device=dev)
    for g, (ptr, _) in enumerate(segs):
        gathered[g * nbytes // 4:(g + 1) * nbytes // 4].copy_(device_view(ptr, nbytes // 4, dev))
    torch.cuda.synchronize()
    for P in handles:
        P.prepare_shard_complete(gathered, stream)
    return gathered


def rccl_unique_id() -> bytes:
    """mas_rccl_unique_id: 128 bytes for rank 0 to broadcast before rccl_init."""
    buf = ctypes.create_string_buffer(128)
    rc = lib().mas_rccl_unique_id(buf)
    if rc != MAS_OK:
        raise MasError(f"mas_rccl_unique_id failed: {STATUS.get(rc, rc)}")
    return buf.raw


def blob_validate(blob) -> int:
    """mas_blob_validate: MAS_OK (0) or MAS_ERR_ARG; needs no device."""
    b = np.ascontiguousarray(np.frombuffer(blob, dtype=np.uint8) if isinstance(blob, (bytes, bytearray))
                             else blob, dtype=np.uint8)
    return lib().mas_blob_validate(_ptr(b), b.nbytes)


def shard_plan(nV, l1_first, rank, world) -> dict:
    """Host-only Morton-range shard plan (mas_shard_plan; no device needed)."""
    l1 = np.ascontiguousarray(l1_first, dtype=np.int32)
    sh = mas_shard()
    rc = lib().mas_shard_plan(nV, _ptr(l1), rank, world, ctypes.byref(sh))
    if rc != MAS_OK:
        raise MasError(f"mas_shard_plan failed: {STATUS.get(rc, rc)}")
    return sh.as_dict()

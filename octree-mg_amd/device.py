"""ctypes binding of libomg.so (the HIP library behind include/omg.h).

The product path always goes through this library: if it is missing or fails
to load, every call raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

_P, _I, _D, _LL = C.c_void_p, C.c_int, C.c_double, C.c_longlong
_IP = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_DP = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_LP = np.ctypeslib.ndpointer(dtype=np.int64, flags="C_CONTIGUOUS")

# every symbol include/omg.h declares, with its ctypes signature
SIGNATURES = {
    "omg_last_error": (C.c_char_p, []),
    "omg_get_unique_id": (_I, [C.c_char_p]),
    "omg_loopback_unique_id": (_I, [C.c_longlong, C.c_char_p]),
    "omg_host_unique_id": (_I, [C.c_char_p]),
    "omg_set_host_transport": (_I, [_P, C.c_void_p, C.c_void_p, C.c_void_p]),
    "omg_device_count": (_I, [C.POINTER(_I)]),
    "omg_plan_transfer": (_I, [_P, _I, _I, _I, _I, _IP, C.POINTER(C.c_longlong), C.POINTER(_I),
                               C.POINTER(_I)]),
    "omg_ctx_create": (_I, [C.POINTER(_P), _I, _I, _I, C.c_char_p]),
    "omg_ctx_destroy": (_I, [_P]),
    "omg_tree_setup": (_I, [_P, _I, _IP, _IP, _IP, _IP, _IP, _IP, _I, _I, _I, _I, _IP, _DP,
                            _IP, _IP, _I]),
    "omg_set_operator": (_I, [_P, _I, _D]),
    "omg_set_smoother": (_I, [_P, _I, _I, _I, _I, _D, _D]),
    "omg_set_subtract_mean": (_I, [_P, _I]),
    "omg_set_coarse_replication": (_I, [_P, _LL]),
    "omg_replicated_level": (_I, [_P, C.POINTER(_I)]),
    "omg_set_bc": (_I, [_P, _I, _I, _I, _D]),
    "omg_set_bc_faces": (_I, [_P, _I, _LP, _IP, _DP, _LL]),
    "omg_level_size": (_I, [_P, _I, C.POINTER(_I), C.POINTER(_I)]),
    "omg_upload_level": (_I, [_P, _I, _I, _DP]),
    "omg_download_level": (_I, [_P, _I, _I, _DP]),
    "omg_fas_vcycle": (_I, [_P, _I, _I, C.POINTER(_D), _I]),
    "omg_fas_fmg": (_I, [_P, _I, _I, C.POINTER(_D)]),
    "omg_apply_op": (_I, [_P, _I]),
    "omg_restrict": (_I, [_P, _I]),
    "omg_restrict_lvl": (_I, [_P, _I, _I]),
    "omg_fill_ghost_cells": (_I, [_P, _I]),
    "omg_fill_ghost_cells_lvl": (_I, [_P, _I, _I]),
    "omg_prolong": (_I, [_P, _I, _I, _I, _I]),
    "omg_smooth_boxes": (_I, [_P, _I, _I]),
    "omg_update_coarse": (_I, [_P, _I]),
    "omg_correct_children": (_I, [_P, _I]),
    "omg_residual_lvl": (_I, [_P, _I]),
    "omg_max_residual_lvl": (_I, [_P, _I, C.POINTER(_D)]),
    "omg_get_sum": (_I, [_P, _I, C.POINTER(_D)]),
    "omg_subtract_mean": (_I, [_P, _I, _I]),
    "omg_phi_bc_store": (_I, [_P]),
    "omg_set_rhs": (_I, [_P, _D, _D]),
    "omg_diffusion_solve": (_I, [_P, _I, _D, _D, _I, _D, C.POINTER(_I), C.POINTER(_D)]),
    "omg_poisson_free_3d": (_I, [_P, _I, _D, _I, _I, C.POINTER(_D), _DP, C.c_void_p]),
    "omg_free_planes": (_I, [_P, C.POINTER(_I), _IP, C.c_void_p, _LL]),
    "omg_comm_info": (_I, [_P, C.POINTER(_I), C.POINTER(_I)]),
    "omg_synchronize": (_I, [_P]),
    "omg_stream": (_P, [_P]),
    "omg_host_sync_count": (_I, [_P, C.POINTER(_LL)]),
    "omg_set_refinement_bnd": (_I, [_P, _I, _I, C.c_void_p, C.c_void_p]),
    "omg_comm_stream_priority": (_I, [_P, C.POINTER(_I)]),
    "omg_set_profiling": (_I, [_P, _I]),
    "omg_kernel_stats": (_I, [_P, C.c_char_p, C.POINTER(_LL), C.POINTER(_D), C.POINTER(_D)]),
    "omg_reset_stats": (_I, [_P]),
}


def lib_path() -> str:
    # OMG_LIB: another build of the same library (kernel A/B timing only)
    return os.environ.get("OMG_LIB") or os.path.join(_HERE, "libomg.so")


def lib():
    """Load libomg.so (raises if absent — no fallback)."""
    global _LIB
    if _LIB is None:
        p = lib_path()
        if not os.path.exists(p):
            raise RuntimeError(f"octree-mg HIP library not built: {p} (run __graft_entry__.build())")
        L = C.CDLL(p)
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("OMG_LIB") and not hasattr(L, name):
                continue   # an older build for A/B timing may lack a newer diagnostic
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _LIB = L
    return _LIB


class OmgError(RuntimeError):
    pass


def check(rc: int):
    if rc != 0:
        raise OmgError(lib().omg_last_error().decode())


def unique_id() -> bytes:
    buf = C.create_string_buffer(128)
    check(lib().omg_get_unique_id(buf))
    return buf.raw


def loopback_unique_id(tag: int) -> bytes:
    """Id of an in-process loopback group (several ranks, one GPU, one thread
    per rank): see omg_loopback_unique_id in include/omg.h."""
    buf = C.create_string_buffer(128)
    check(lib().omg_loopback_unique_id(int(tag), buf))
    return buf.raw


def host_unique_id() -> bytes:
    """Id that selects the host transport (omg_host_unique_id)."""
    buf = C.create_string_buffer(128)
    check(lib().omg_host_unique_id(buf))
    return buf.raw


def device_count() -> int:
    n = _I()
    check(lib().omg_device_count(C.byref(n)))
    return n.value


# omg_host_exchange_fn / omg_host_allgather_fn (include/omg.h)
_XCHG_FN = C.CFUNCTYPE(_I, C.c_void_p, _I, C.POINTER(_I), C.POINTER(C.c_longlong), C.POINTER(C.c_void_p),
                       _I, C.POINTER(_I), C.POINTER(C.c_longlong), C.POINTER(C.c_void_p))
_AGATH_FN = C.CFUNCTYPE(_I, C.c_void_p, C.POINTER(_D), _I, C.POINTER(_D))


def _host_view(ptr, n):
    """A float64 numpy view of n doubles of pinned host staging."""
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(_D)), shape=(int(n),))


class Context:
    """One device context (one rank, one GPU)."""

    def __init__(self, device=0, rank=0, n_ranks=1, uid: bytes | None = None):
        self.L = lib()
        h = _P()
        check(self.L.omg_ctx_create(C.byref(h), device, rank, n_ranks, uid))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            check(self.L.omg_ctx_destroy(self.h))
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    after_call = None   # e.g. re-raise what a host callback raised during the call

    def set_host_transport(self, group=None):
        """The host transport over torch.distributed (gloo, CPU tensors):
        omg_set_host_transport with an isend / irecv round and an all_gather
        (the ranks share a GPU, which RCCL refuses).  Messages of a pair keep
        their order (one group, one tag)."""
        import torch
        import torch.distributed as dist

        def exchange(user, ns, sp, sn, sb, nr, rp, rn, rb):
            try:
                reqs = [dist.irecv(torch.from_numpy(_host_view(rb[i], rn[i])), src=int(rp[i]), group=group)
                        for i in range(nr)]
                reqs += [dist.isend(torch.from_numpy(_host_view(sb[i], sn[i])), dst=int(sp[i]), group=group)
                         for i in range(ns)]
                for r in reqs:
                    r.wait()
                return 0
            except Exception:   # noqa: BLE001  (the library raises "the exchange callback failed")
                return 1

        def allgather(user, mine, n, out):
            try:
                world = dist.get_world_size(group)
                t = torch.from_numpy(np.array(_host_view(C.cast(mine, C.c_void_p), n)))
                parts = [torch.empty_like(t) for _ in range(world)]
                dist.all_gather(parts, t, group=group)
                _host_view(C.cast(out, C.c_void_p), n * world)[:] = torch.cat(parts).numpy()
                return 0
            except Exception:   # noqa: BLE001
                return 1

        self._xport = (_XCHG_FN(exchange), _AGATH_FN(allgather))   # (kept alive with the context)
        check(self.L.omg_set_host_transport(self.h, C.cast(self._xport[0], C.c_void_p),
                                            C.cast(self._xport[1], C.c_void_p), None))

    def call(self, name, *args):
        check(getattr(self.L, "omg_" + name)(self.h, *args))
        if self.after_call is not None:
            self.after_call()

    def plan_transfer(self, lvl, which, direction):
        """[(peer, key), ...] in wire order and the doubles per item of one
        transfer of the communication plan (omg_plan_transfer)."""
        n, per = _I(), _I()
        self.call("plan_transfer", lvl, which, direction, 0, np.zeros(1, np.int32),
                  np.zeros(1, np.int64).ctypes.data_as(C.POINTER(C.c_longlong)), C.byref(n), C.byref(per))
        peers = np.zeros(max(n.value, 1), np.int32)
        keys = np.zeros(max(n.value, 1), np.int64)
        self.call("plan_transfer", lvl, which, direction, n.value, peers,
                  keys.ctypes.data_as(C.POINTER(C.c_longlong)), C.byref(n), C.byref(per))
        return [(int(p), int(k)) for p, k in zip(peers[:n.value], keys[:n.value])], per.value

    def stream(self) -> int:
        return self.L.omg_stream(self.h) or 0

    def replicated_level(self):
        r = _I()
        self.call("replicated_level", C.byref(r))
        return r.value

    def level_size(self, lvl):
        n, nc = _I(), _I()
        self.call("level_size", lvl, C.byref(n), C.byref(nc))
        return n.value, nc.value

    def upload_level(self, lvl, iv, data):
        self.call("upload_level", lvl, iv, np.ascontiguousarray(data, dtype=np.float64).reshape(-1))

    def download_level(self, lvl, iv):
        n, nc = self.level_size(lvl)
        out = np.empty(n * (nc + 2) ** 3)
        if n:
            self.call("download_level", lvl, iv, out)
        return out.reshape(n, nc + 2, nc + 2, nc + 2)

    def scalar(self, name, *args):
        r = _D(0.0)
        self.call(name, *args, C.byref(r))
        return r.value

    def comm_info(self):
        """(ranks the communicator holds, transport): transport is "none",
        "rccl" (ncclCommCount) or "loopback" (omg_comm_info)."""
        n, t = _I(), _I()
        self.call("comm_info", C.byref(n), C.byref(t))
        return n.value, {0: "none", 1: "rccl", 2: "loopback", 3: "host"}[t.value]

    def host_sync_count(self):
        """Host waits on the context's streams so far (omg_host_sync_count)."""
        n = _LL(0)
        self.call("host_sync_count", C.byref(n))
        return n.value

    def comm_stream_priority(self):
        p = _I(0)
        self.call("comm_stream_priority", C.byref(p))
        return p.value

    def kernel_stats(self, name):
        n, ms, cells = _LL(0), _D(0), _D(0)
        self.call("kernel_stats", name.encode(), C.byref(n), C.byref(ms), C.byref(cells))
        return n.value, ms.value, cells.value

"""icp4r — MI355X-native drop-in for the ICP registration the reference node runs.

Host-side mirror of the PCL surface used at ``/root/reference/src/iterative_closest_point.cpp:510-521``
(``pcl::IterativeClosestPoint<PointXYZI, PointXYZI>``) over the C ABI in ``include/icp4r/icp4r.h``:

    icp = IterativeClosestPoint()
    icp.setInputSource(cloud_src_in)        # (N, >=3) float32: x, y, z[, intensity, ...]
    icp.setInputTarget(cloud_tar_in)
    Final = icp.align()                     # align(output) -> transformed source
    icp.hasConverged(), icp.getFitnessScore()
    T = icp.getFinalTransformation()        # 4x4 float32 (Eigen::Matrix4f values)

The product path is the HIP library ``icp4r/_lib/libicp4r.so`` (gfx950).  There is no CPU fallback:
if the library or a GPU is missing, calls raise :class:`ICP4RError`.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

import numpy as np

__all__ = [
    "ICP4RError", "Params", "Result", "Batch", "Context", "IterativeClosestPoint", "library_path", "load",
    "default_params", "NUMERICS_PCL", "NUMERICS_F64", "status_name", "EXPORTED_SYMBOLS", "Comm", "shard",
    "align_batch_multi",
]

HERE = os.path.dirname(os.path.abspath(__file__))
# ICP4R_LIBRARY: an alternative build of the same library (A/B experiments); default: the in-tree build
library_path = os.environ.get("ICP4R_LIBRARY") or os.path.join(HERE, "_lib", "libicp4r.so")

OK, E_INVALID, E_EMPTY, E_TOO_FEW_CORR, E_NONFINITE, E_HIP, E_RCCL, E_NOMEM, E_TOO_LARGE = 0, -1, -2, -3, -4, -5, -6, -7, -8
NUMERICS_PCL, NUMERICS_F64 = 0, 1
NO_DEVICE = -1  # icp4r_create(&ctx, ICP4R_NO_DEVICE): plan queries and plan options only
NN_AUTO, NN_BRUTE, NN_BRUTE_PACKED, NN_PRUNED = 0, 1, 2, 3
STAGE_NN, STAGE_NN_TEST, STAGE_UPDATE, STAGE_BATCH, STAGE_GICP_COV = 0, 1, 2, 3, 4
DBL_MAX = sys.float_info.max

_STATUS = {OK: "ICP4R_OK", E_INVALID: "ICP4R_E_INVALID", E_EMPTY: "ICP4R_E_EMPTY",
           E_TOO_FEW_CORR: "ICP4R_E_TOO_FEW_CORR", E_NONFINITE: "ICP4R_E_NONFINITE", E_HIP: "ICP4R_E_HIP",
           E_RCCL: "ICP4R_E_RCCL", E_NOMEM: "ICP4R_E_NOMEM", E_TOO_LARGE: "ICP4R_E_TOO_LARGE"}

# every function declared in include/icp4r/icp4r.h (tests check the library exports all of them)
EXPORTED_SYMBOLS = [
    "icp4r_version", "icp4r_abi_version", "icp4r_last_error", "icp4r_params_default", "icp4r_device_count",
    "icp4r_create", "icp4r_destroy", "icp4r_align", "icp4r_align_batch_device", "icp4r_align_batch_host",
    "icp4r_fitness", "icp4r_nearest", "icp4r_synchronize", "icp4r_kernel_time_ms", "icp4r_batch_time_ms",
    "icp4r_kernel_time_reset", "icp4r_set_kernel_timing", "icp4r_plan", "icp4r_nn_counters", "icp4r_nn_cache_hits", "icp4r_stage_time_ms",
    "icp4r_nn_stats", "icp4r_set_plan_option", "icp4r_get_plan_option", "icp4r_reset_plan_options",
]
# the plan options of icp4r_set_plan_option: A/B and diagnostic switches, never a result
PLAN_OPTIONS = (
    "nn_q", "leaf", "chunk_sb", "nn_lds", "nn_cache", "nn_tile", "tile_run", "solo", "xpad", "phase_ticks", "kd",
    "morton_mwg", "part", "src_order", "fuse_seed", "tile_own", "tile_defer", "groups", "search_cu_div",
    "fuse_test", "fuse_order", "sums_tail", "wide_update", "gather_padded", "gicp_cov_brute", "fold_keys", "gicp_spec", "gicp_grid", "gicp_knn_lanes", "res_update", "held_update", "fit_xform", "counters", "stage_sel",
)
# include/icp4r/icp4r_ego.h (radar ego velocity and the scan parse; icp4r.ego)
EGO_EXPORTED_SYMBOLS = [
    "icp4r_ego_params_default", "icp4r_radar_features", "icp4r_ego_velocity", "icp4r_ego_velocity_batch_device",
]
# include/icp4r/icp4r_gicp.h (generalized ICP; icp4r.gicp)
GICP_EXPORTED_SYMBOLS = [
    "icp4r_gicp_params_default", "icp4r_gicp_align", "icp4r_gicp_align_batch_device", "icp4r_gicp_covariances",
]
# include/icp4r/icp4r_multi.h (the batched multi-GPU mode: shards, multi-device batch, RCCL gather)
MULTI_EXPORTED_SYMBOLS = [
    "icp4r_shard", "icp4r_align_batch_multi", "icp4r_comm_unique_id", "icp4r_comm_create", "icp4r_comm_destroy",
    "icp4r_comm_rank", "icp4r_comm_check", "icp4r_gather_results", "icp4r_align_batch_sharded",
]
# include/icp4r/icp4r_map.h (scan-to-map store; icp4r.mapstore)
MAP_EXPORTED_SYMBOLS = [
    "icp4r_map_create", "icp4r_map_destroy", "icp4r_map_build", "icp4r_map_add_points", "icp4r_map_add_scan",
    "icp4r_map_size", "icp4r_map_sector_search", "icp4r_map_sector_search_device", "icp4r_map_points_device",
    "icp4r_map_time_ms", "icp4r_map_time_reset",
]


def status_name(code: int) -> str:
    return _STATUS.get(code, f"status {code}")


class ICP4RError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{status_name(code)}: {msg}")
        self.code = code


class Params(C.Structure):
    _fields_ = [
        ("max_iterations", C.c_int32),
        ("min_correspondences", C.c_int32),
        ("max_correspondence_distance", C.c_double),
        ("transformation_epsilon", C.c_double),
        ("transformation_rotation_epsilon", C.c_double),
        ("euclidean_fitness_epsilon", C.c_double),
        ("mse_threshold_absolute", C.c_double),
        ("max_iterations_similar_transforms", C.c_int32),
        ("numerics", C.c_int32),
        ("nn_mode", C.c_int32),
        ("compute_fitness", C.c_int32),
        ("huber_delta", C.c_double),
        ("fitness_max_range", C.c_double),
        ("eigen_l1_bytes", C.c_int32),
        ("eigen_gebp_mr", C.c_int32),
        ("reserved", C.c_int32 * 6),
    ]


class Result(C.Structure):
    _fields_ = [
        ("T", C.c_float * 16),
        ("fitness", C.c_double),
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("status", C.c_int32),
        ("convergence_state", C.c_int32),
        ("n_correspondences", C.c_int32),
        ("reserved", C.c_int32),
    ]

    def matrix(self) -> np.ndarray:
        """getFinalTransformation(): 4x4 float32 (stored column-major like Eigen)."""
        return np.array(self.T, np.float32).reshape(4, 4).T.copy()


class Batch(C.Structure):
    _fields_ = [
        ("src", C.c_void_p), ("tgt", C.c_void_p),
        ("src_off", C.c_void_p), ("src_n", C.c_void_p),
        ("tgt_off", C.c_void_p), ("tgt_n", C.c_void_p),
        ("guess", C.c_void_p), ("aligned", C.c_void_p),
        ("npairs", C.c_int32), ("max_src_n", C.c_int32), ("max_tgt_n", C.c_int32), ("reserved", C.c_int32),
    ]


class PlanInfo(C.Structure):
    _fields_ = [("pruned", C.c_int32), ("q", C.c_int32), ("splits", C.c_int32), ("leaf", C.c_int32),
                ("lds", C.c_int32), ("cache", C.c_int32), ("nn_blocks", C.c_int64), ("solo", C.c_int32),
                ("wide_update", C.c_int32), ("res_update", C.c_int32),
                ("held_update", C.c_int32)]


assert C.sizeof(Result) == 96
RESULT_DTYPE = np.dtype([("T", np.float32, 16), ("fitness", np.float64), ("iterations", np.int32),
                         ("converged", np.int32), ("status", np.int32), ("convergence_state", np.int32),
                         ("n_correspondences", np.int32), ("reserved", np.int32)])
assert RESULT_DTYPE.itemsize == 96

_lib = None


def load():
    """Load the HIP library (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(library_path):
        raise ICP4RError(E_HIP, f"{library_path} not built (run __graft_entry__.build() or make -C icp-4dradar_amd)")
    L = C.CDLL(library_path)
    vp, i32, i64 = C.c_void_p, C.c_int32, C.c_int64
    sig = {
        "icp4r_version": (C.c_char_p, []),
        "icp4r_abi_version": (C.c_int, []),
        "icp4r_last_error": (C.c_char_p, []),
        "icp4r_params_default": (None, [C.POINTER(Params)]),
        "icp4r_device_count": (C.c_int, [C.POINTER(C.c_int)]),
        "icp4r_create": (C.c_int, [C.POINTER(vp), C.c_int]),
        "icp4r_destroy": (C.c_int, [vp]),
        "icp4r_align": (C.c_int, [vp, vp, i32, i32, vp, i32, i32, vp, C.POINTER(Params), C.POINTER(Result), vp, i32]),
        "icp4r_align_batch_device": (C.c_int, [vp, C.POINTER(Batch), C.POINTER(Params), vp, vp]),
        "icp4r_align_batch_host": (C.c_int, [vp, vp, vp, vp, vp, vp, vp, i32, vp, C.POINTER(Params), vp]),
        "icp4r_fitness": (C.c_int, [vp, vp, i32, i32, vp, i32, i32, vp, C.c_double, C.POINTER(C.c_double)]),
        "icp4r_nearest": (C.c_int, [vp, vp, i32, i32, vp, i32, i32, vp, vp]),
        "icp4r_synchronize": (C.c_int, [vp, vp]),
        "icp4r_kernel_time_ms": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(i32)]),
        "icp4r_batch_time_ms": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(i32)]),
        "icp4r_kernel_time_reset": (C.c_int, [vp]),
        "icp4r_plan": (C.c_int, [vp, i32, i32, i32, i32, i32, C.POINTER(PlanInfo)]),
        "icp4r_set_plan_option": (C.c_int, [vp, C.c_char_p, i32]),
        "icp4r_get_plan_option": (C.c_int, [vp, C.c_char_p, C.POINTER(i32), C.POINTER(i32)]),
        "icp4r_reset_plan_options": (C.c_int, [vp]),
        "icp4r_nn_counters": (C.c_int, [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
        "icp4r_nn_cache_hits": (C.c_int, [vp, C.POINTER(C.c_uint64)]),
        "icp4r_stage_time_ms": (C.c_int, [vp, i32, C.POINTER(C.c_double), C.POINTER(i32)]),
        "icp4r_set_kernel_timing": (C.c_int, [vp, i32]),
        "icp4r_nn_stats": (C.c_int, [vp, C.POINTER(C.c_uint64 * 8)]),
        # icp4r_map.h
        "icp4r_map_create": (C.c_int, [vp, C.POINTER(vp)]),
        "icp4r_map_destroy": (C.c_int, [vp]),
        "icp4r_map_build": (C.c_int, [vp, vp, i64, i32]),
        "icp4r_map_add_points": (C.c_int, [vp, vp, i64, i32, i32]),
        "icp4r_map_add_scan": (C.c_int, [vp, vp, i64, i32, vp, vp, vp]),
        "icp4r_map_size": (C.c_int, [vp, C.POINTER(i64)]),
        "icp4r_map_sector_search": (C.c_int, [vp, vp, C.c_float, C.c_float, vp, i64, C.POINTER(i64)]),
        "icp4r_map_sector_search_device": (C.c_int, [vp, vp, C.c_float, C.c_float, vp, vp, vp]),
        "icp4r_map_points_device": (C.c_int, [vp, C.POINTER(vp), C.POINTER(i64)]),
        "icp4r_map_time_ms": (C.c_int, [vp, C.POINTER(C.c_double), C.POINTER(i32)]),
        "icp4r_map_time_reset": (C.c_int, [vp]),
        # icp4r_multi.h
        "icp4r_shard": (C.c_int, [i32, i32, i32, C.POINTER(i32), C.POINTER(i32)]),
        "icp4r_align_batch_multi": (C.c_int, [C.POINTER(vp), i32, vp, vp, vp, vp, vp, vp, i32, vp, C.POINTER(Params),
                                              vp]),
        "icp4r_comm_unique_id": (C.c_int, [C.c_char_p]),
        "icp4r_comm_create": (C.c_int, [C.POINTER(vp), vp, i32, i32, C.c_char_p]),
        "icp4r_comm_destroy": (C.c_int, [vp]),
        "icp4r_comm_rank": (C.c_int, [vp, C.POINTER(i32), C.POINTER(i32)]),
        "icp4r_comm_check": (C.c_int, [vp]),
        "icp4r_gather_results": (C.c_int, [vp, vp, i32, vp, vp]),
        "icp4r_align_batch_sharded": (C.c_int, [vp, C.POINTER(Batch), i32, C.POINTER(Params), vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def _check(rc: int, what: str):
    if rc != OK:
        raise ICP4RError(rc, f"{what}: {load().icp4r_last_error().decode()}")


def default_params(**kw) -> Params:
    p = Params()
    load().icp4r_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def _cloud(a) -> tuple[np.ndarray, int, int]:
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] < 3:
        raise ICP4RError(E_INVALID, f"cloud must be (N, >=3) float32, got {a.shape}")
    return a, a.shape[0], a.shape[1] * 4


def _ptr(a: np.ndarray):
    return a.ctypes.data if a.size else None


class Context:
    """One HIP device's stream and buffers (icp4r_create / icp4r_destroy)."""

    def __init__(self, device: int = 0, plan: dict | None = None):
        """device = NO_DEVICE: a context for plan queries and plan options only (no GPU needed).
        plan: plan options to set (icp4r_set_plan_option)."""
        self._lib = load()
        self._h = C.c_void_p()
        _check(self._lib.icp4r_create(C.byref(self._h), device), "icp4r_create")
        self.device = device
        if plan:
            self.set_plan(**plan)

    def close(self):
        if self._h:
            self._lib.icp4r_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # -- single pair, host buffers ------------------------------------------------------------
    def align(self, src, tgt, params: Params | None = None, guess=None, want_aligned: bool = False):
        s, n, ss = _cloud(src)
        t, m, ts = _cloud(tgt)
        p = params if params is not None else default_params()
        r = Result()
        g = None
        if guess is not None:
            g = np.ascontiguousarray(np.asarray(guess, np.float32).T.reshape(16))
        out = np.zeros((n, 4), np.float32) if want_aligned else None
        rc = self._lib.icp4r_align(self._h, _ptr(s), n, ss, _ptr(t), m, ts, _ptr(g) if g is not None else None,
                                   C.byref(p), C.byref(r), _ptr(out) if out is not None else None, 16)
        if rc not in (OK, E_EMPTY, E_TOO_FEW_CORR, E_NONFINITE):
            _check(rc, "icp4r_align")
        return r, out

    def align_batch_host(self, src: np.ndarray, src_off, src_n, tgt: np.ndarray, tgt_off, tgt_n,
                         params: Params | None = None, guess=None) -> np.ndarray:
        """Batch from host float4 arrays; returns a structured array of results (RESULT_DTYPE)."""
        src = np.ascontiguousarray(src, np.float32).reshape(-1, 4)
        tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 4)
        so = np.ascontiguousarray(src_off, np.int64)
        sn = np.ascontiguousarray(src_n, np.int32)
        to = np.ascontiguousarray(tgt_off, np.int64)
        tn = np.ascontiguousarray(tgt_n, np.int32)
        npairs = len(sn)
        res = np.zeros(npairs, RESULT_DTYPE)
        g = None
        if guess is not None:
            g = np.ascontiguousarray(np.asarray(guess, np.float32).transpose(0, 2, 1).reshape(npairs, 16))
        p = params if params is not None else default_params()
        _check(self._lib.icp4r_align_batch_host(self._h, _ptr(src), _ptr(so), _ptr(sn), _ptr(tgt), _ptr(to), _ptr(tn),
                                                npairs, _ptr(g) if g is not None else None, C.byref(p),
                                                res.ctypes.data), "icp4r_align_batch_host")
        return res

    def align_batch_device(self, batch: Batch, params: Params, results_ptr: int, stream: int | None = None):
        """Device-resident batch (pointers from torch.cuda tensors or hipMalloc); asynchronous."""
        _check(self._lib.icp4r_align_batch_device(self._h, C.byref(batch), C.byref(params), C.c_void_p(results_ptr),
                                                  C.c_void_p(stream) if stream else None), "icp4r_align_batch_device")

    def nearest(self, query, tgt):
        q, n, qs = _cloud(query)
        t, m, ts = _cloud(tgt)
        idx = np.empty(n, np.int32)
        d2 = np.empty(n, np.float32)
        _check(self._lib.icp4r_nearest(self._h, _ptr(q), n, qs, _ptr(t), m, ts, _ptr(idx), _ptr(d2)), "icp4r_nearest")
        return idx, d2

    def fitness(self, src, tgt, T, max_range: float = DBL_MAX) -> float:
        s, n, ss = _cloud(src)
        t, m, ts = _cloud(tgt)
        Tc = np.ascontiguousarray(np.asarray(T, np.float32).T.reshape(16))
        out = C.c_double()
        _check(self._lib.icp4r_fitness(self._h, _ptr(s), n, ss, _ptr(t), m, ts, _ptr(Tc), max_range, C.byref(out)),
               "icp4r_fitness")
        return out.value

    def synchronize(self, stream: int | None = None):
        _check(self._lib.icp4r_synchronize(self._h, C.c_void_p(stream) if stream else None), "icp4r_synchronize")

    def kernel_time_ms(self) -> tuple[float, int]:
        ms, k = C.c_double(), C.c_int32()
        _check(self._lib.icp4r_kernel_time_ms(self._h, C.byref(ms), C.byref(k)), "icp4r_kernel_time_ms")
        return ms.value, k.value

    def batch_time_ms(self) -> tuple[float, int]:
        ms, k = C.c_double(), C.c_int32()
        _check(self._lib.icp4r_batch_time_ms(self._h, C.byref(ms), C.byref(k)), "icp4r_batch_time_ms")
        return ms.value, k.value

    def set_kernel_timing(self, on: bool = True):
        """Per-kernel events for kernel_time_ms / stage_time_ms (off by default: they cost device time
        between kernels; batch_time_ms is always available)."""
        _check(self._lib.icp4r_set_kernel_timing(self._h, 1 if on else 0), "icp4r_set_kernel_timing")

    # -- plan options (icp4r_set_plan_option) -------------------------------------
    def set_plan_option(self, name: str, value: int):
        """Set one plan option (A/B and diagnostics: never changes a result) for this context's calls."""
        _check(self._lib.icp4r_set_plan_option(self._h, name.encode(), int(value)), f"plan option {name}")

    def set_plan(self, **options):
        for k, v in options.items():
            self.set_plan_option(k, v)

    def get_plan_option(self, name: str) -> tuple[int, bool]:
        """(value in effect, whether it was set)."""
        v, is_set = C.c_int32(), C.c_int32()
        _check(self._lib.icp4r_get_plan_option(self._h, name.encode(), C.byref(v), C.byref(is_set)), f"plan option {name}")
        return v.value, bool(is_set.value)

    def reset_plan_options(self):
        _check(self._lib.icp4r_reset_plan_options(self._h), "icp4r_reset_plan_options")

    def stage_time_ms(self, stage: int) -> tuple[float, int]:
        """(average ms, launches) of a stage (STAGE_NN, STAGE_NN_TEST, STAGE_UPDATE, STAGE_BATCH)."""
        ms, k = C.c_double(), C.c_int32()
        _check(self._lib.icp4r_stage_time_ms(self._h, stage, C.byref(ms), C.byref(k)), "icp4r_stage_time_ms")
        return ms.value, k.value

    def reset_timers(self):
        _check(self._lib.icp4r_kernel_time_reset(self._h), "icp4r_kernel_time_reset")

    def nn_counters(self) -> tuple[int, int]:
        """(distance evaluations, box tests) of the NN kernels since the last reset_timers()."""
        v, t = C.c_uint64(), C.c_uint64()
        _check(self._lib.icp4r_nn_counters(self._h, C.byref(v), C.byref(t)), "icp4r_nn_counters")
        return v.value, t.value

    def nn_stats(self) -> dict:
        """Every NN work counter since the last reset_timers() (icp4r_nn_stats_t)."""
        v = (C.c_uint64 * 8)()
        _check(self._lib.icp4r_nn_stats(self._h, C.byref(v)), "icp4r_nn_stats")
        keys = ("evaluations", "box_tests", "cache_hits", "cache_tested", "records_written_by_test",
                "tested_in_update", "hits_in_update", "second_chance_hits")
        return {k: int(v[i]) for i, k in enumerate(keys)}

    def nn_cache_hits(self) -> int:
        """Queries the cached-neighbour test resolved without a search since the last reset_timers()."""
        v = C.c_uint64()
        _check(self._lib.icp4r_nn_cache_hits(self._h, C.byref(v)), "icp4r_nn_cache_hits")
        return v.value

    def nn_evaluations(self) -> int:
        """Distance evaluations (query x target) of the NN kernels since the last reset_timers()."""
        return self.nn_counters()[0]


def plan(npairs: int, max_src_n: int, max_tgt_n: int, nn_mode: int = NN_AUTO, numerics: int = NUMERICS_PCL,
         ctx: "Context | None" = None) -> dict:
    """The launch plan of a batch shape (ctx: whose plan options and CU count; None: the defaults)."""
    info = PlanInfo()
    _check(load().icp4r_plan(ctx.handle if ctx is not None else None, npairs, max_src_n, max_tgt_n, nn_mode, numerics,
                             C.byref(info)), "icp4r_plan")
    return {"pruned": bool(info.pruned), "lds": bool(info.lds), "cache": bool(info.cache), "q": info.q, "splits": info.splits,
            "leaf": info.leaf, "nn_blocks": info.nn_blocks, "solo": bool(info.solo),
            "wide_update": bool(info.wide_update), "res_update": bool(info.res_update),
            "held_update": bool(info.held_update)}


_default_ctx: Context | None = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("ICP4R_DEVICE", "0")))
    return _default_ctx


class IterativeClosestPoint:
    """pcl::IterativeClosestPoint<PointXYZI, PointXYZI> surface (PCL 1.8.1 defaults)."""

    def __init__(self, context: Context | None = None):
        self._ctx = context
        self._p = default_params()
        self._src = None
        self._tgt = None
        self._result: Result | None = None

    # --- Registration setters ---
    def setInputSource(self, cloud):
        self._src = np.ascontiguousarray(cloud, np.float32)
        self._result = None

    def setInputTarget(self, cloud):
        self._tgt = np.ascontiguousarray(cloud, np.float32)
        self._result = None

    def setMaximumIterations(self, nr_iterations: int):
        self._p.max_iterations = int(nr_iterations)

    def getMaximumIterations(self) -> int:
        return self._p.max_iterations

    def setMaxCorrespondenceDistance(self, distance_threshold: float):
        self._p.max_correspondence_distance = float(distance_threshold)

    def getMaxCorrespondenceDistance(self) -> float:
        return self._p.max_correspondence_distance

    def setTransformationEpsilon(self, epsilon: float):
        self._p.transformation_epsilon = float(epsilon)

    def setTransformationRotationEpsilon(self, epsilon: float):
        self._p.transformation_rotation_epsilon = float(epsilon)

    def setEuclideanFitnessEpsilon(self, epsilon: float):
        self._p.euclidean_fitness_epsilon = float(epsilon)

    # build extensions (no PCL counterpart)
    def setHuberDelta(self, delta: float):
        self._p.huber_delta = float(delta)

    def setNumerics(self, numerics: int):
        self._p.numerics = int(numerics)

    def params(self) -> Params:
        return self._p

    # --- Registration::align ---
    def align(self, output=None, guess=None) -> np.ndarray:
        if self._tgt is None:
            raise ICP4RError(E_EMPTY, "No input target dataset was given!")
        if self._src is None:
            raise ICP4RError(E_INVALID, "No input source dataset was given!")
        ctx = self._ctx or default_context()
        r, aligned = ctx.align(self._src, self._tgt, self._p, guess=guess, want_aligned=True)
        self._result = r
        out = self._src.copy()
        out[:, :3] = aligned[:, :3]
        if output is not None:
            output[...] = out
            return output
        return out

    def hasConverged(self) -> bool:
        return bool(self._result is not None and self._result.converged)

    def getFinalTransformation(self) -> np.ndarray:
        if self._result is None:
            return np.eye(4, dtype=np.float32)
        return self._result.matrix()

    def getFitnessScore(self, max_range: float = DBL_MAX) -> float:
        if self._result is None:
            return DBL_MAX
        if max_range == self._p.fitness_max_range:
            return self._result.fitness  # computed once inside align
        return (self._ctx or default_context()).fitness(self._src, self._tgt, self.getFinalTransformation(), max_range)

    # introspection beyond PCL's getters (same information PCL keeps privately)
    def result(self) -> Result | None:
        return self._result

    def nr_iterations(self) -> int:
        return 0 if self._result is None else self._result.iterations


# ---------------------------------------------------------------------------------------------------
# Batched multi-GPU mode (include/icp4r/icp4r_multi.h).

COMM_ID_BYTES = 128


def shard(npairs: int, nranks: int, rank: int) -> range:
    """icp4r_shard: the contiguous, balanced block of global pairs rank `rank` of `nranks` owns."""
    f, c = C.c_int32(), C.c_int32()
    _check(load().icp4r_shard(npairs, nranks, rank, C.byref(f), C.byref(c)), "icp4r_shard")
    return range(f.value, f.value + c.value)


def align_batch_multi(ctxs, src, src_off, src_n, tgt, tgt_off, tgt_n, params: Params | None = None,
                      guess=None) -> np.ndarray:
    """icp4r_align_batch_multi: one process, one context per device, shard k on context k (host threads);
    returns the results of every pair in global order (RESULT_DTYPE)."""
    src = np.ascontiguousarray(src, np.float32).reshape(-1, 4)
    tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 4)
    so = np.ascontiguousarray(src_off, np.int64)
    sn = np.ascontiguousarray(src_n, np.int32)
    to = np.ascontiguousarray(tgt_off, np.int64)
    tn = np.ascontiguousarray(tgt_n, np.int32)
    npairs = len(sn)
    res = np.zeros(npairs, RESULT_DTYPE)
    g = None
    if guess is not None:
        g = np.ascontiguousarray(np.asarray(guess, np.float32).transpose(0, 2, 1).reshape(npairs, 16))
    handles = (C.c_void_p * len(ctxs))(*[c.handle.value for c in ctxs])
    p = params if params is not None else default_params()
    _check(load().icp4r_align_batch_multi(handles, len(ctxs), _ptr(src), _ptr(so), _ptr(sn), _ptr(tgt), _ptr(to),
                                          _ptr(tn), npairs, _ptr(g) if g is not None else None, C.byref(p),
                                          res.ctypes.data), "icp4r_align_batch_multi")
    return res


class Comm:
    """One rank of an RCCL communicator on a context's device (icp4r_comm_create): the one-process-per-GPU
    form of the batched mode.  Rank 0 makes the id (Comm.unique_id()) and hands it to the others."""

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(COMM_ID_BYTES)
        _check(load().icp4r_comm_unique_id(buf), "icp4r_comm_unique_id")
        return buf.raw

    def __init__(self, ctx: Context, nranks: int, rank: int, uid: bytes):
        if len(uid) != COMM_ID_BYTES:
            raise ICP4RError(E_INVALID, f"unique id must be {COMM_ID_BYTES} bytes")
        self._lib = load()
        self._h = C.c_void_p()
        self.ctx, self.nranks, self.rank = ctx, nranks, rank
        _check(self._lib.icp4r_comm_create(C.byref(self._h), ctx.handle, nranks, rank, uid), "icp4r_comm_create")

    def close(self):
        if self._h:
            self._lib.icp4r_comm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self):
        _check(self._lib.icp4r_comm_check(self._h), "icp4r_comm_check")

    def gather(self, shard_rows_ptr: int, npairs: int, gathered_ptr: int, stream: int | None = None):
        """icp4r_gather_results: this rank's rows (device) into every rank's gathered[npairs] (device)."""
        _check(self._lib.icp4r_gather_results(self._h, C.c_void_p(shard_rows_ptr), npairs, C.c_void_p(gathered_ptr),
                                              C.c_void_p(stream) if stream else None), "icp4r_gather_results")

    def align_batch_sharded(self, batch: Batch, npairs_total: int, params: Params, shard_results_ptr: int,
                            gathered_ptr: int, stream: int | None = None):
        """icp4r_align_batch_sharded: register this rank's shard, then gather every rank's rows."""
        _check(self._lib.icp4r_align_batch_sharded(self._h, C.byref(batch), npairs_total, C.byref(params),
                                                   C.c_void_p(shard_results_ptr), C.c_void_p(gathered_ptr),
                                                   C.c_void_p(stream) if stream else None),
               "icp4r_align_batch_sharded")


def env_plan(environ=None) -> dict:
    """TOOLING ONLY (A/B scripts, tests): the plan options named by ICP4R_<NAME> environment variables,
    e.g. ICP4R_GROUPS=1 -> {"groups": 1}.  Neither the library nor Context reads the environment; a
    tool applies this dict explicitly (Context.set_plan(**env_plan()))."""
    environ = os.environ if environ is None else environ
    out = {}
    for name in PLAN_OPTIONS:
        v = environ.get("ICP4R_" + name.upper())
        if v not in (None, ""):
            out[name] = int(v)
    return out

"""Scan-to-map store and sector query (include/icp4r/icp4r_map.h), mirroring the ikd-Tree API the
reference's radar_odometry node uses:

    KD_TREE<PointXYZI> ikd_Tree(0.3, 0.6, 0.5);            radar_odometry.cpp:92
    ikd_Tree.Build(src->points);                            :347
    ikd_Tree.set_downsample_param(0.5);                     :348
    pointAssociateToMap(...); ikd_Tree.Add_Points(.., false) :382-390
    ikd_Tree.Sector_Search(p_now, RADAR_RADIUS, heading, SubMap->points)   :396

Same method names; clouds are (N, >=3) float32 arrays (x, y, z[, intensity]).  Device-resident and
GPU-only: there is no CPU fallback (the library raises if it is missing).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import Context, _check, _cloud, _ptr, default_context, load

RADAR_RADIUS = 80.0  # radar_odometry.cpp:36


class KD_TREE:  # noqa: N801 — the reference's class name
    """ikd-Tree replacement for radar_odometry's map: an append-only device store (nothing is ever
    deleted on this path) with Sector_Search as a full filter in insertion order."""

    def __init__(self, delete_param: float = 0.5, balance_param: float = 0.6, box_length: float = 0.2,
                 ctx: Context | None = None):
        # delete/balance parameters steer ikd-Tree's rebalancing, which does not change query results;
        # box_length is the downsample box, unused because the node adds with downsample_on = false.
        self.delete_param, self.balance_param, self.downsample_size = delete_param, balance_param, box_length
        self._ctx = ctx or default_context()
        self._lib = load()
        self._h = C.c_void_p()
        _check(self._lib.icp4r_map_create(self._ctx.handle, C.byref(self._h)), "icp4r_map_create")

    def close(self):
        if self._h:
            self._lib.icp4r_map_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # -- the reference's method names ------------------------------------------------------------
    def Build(self, points):  # noqa: N802
        a, n, stride = _cloud(points)
        _check(self._lib.icp4r_map_build(self._h, _ptr(a), n, stride), "icp4r_map_build")

    def set_downsample_param(self, box_length: float):
        self.downsample_size = box_length

    def Add_Points(self, points, downsample_on: bool = False) -> int:  # noqa: N802
        a, n, stride = _cloud(points)
        _check(self._lib.icp4r_map_add_points(self._h, _ptr(a), n, stride, int(bool(downsample_on))),
               "icp4r_map_add_points")
        return 0  # ikd-Tree returns the downsample counter, 0 without downsampling

    def Sector_Search(self, point, radius: float, heading: float) -> np.ndarray:  # noqa: N802
        """The kept points, (K, 4) float32, insertion order (ikd-Tree: the same set, tree order)."""
        c = np.ascontiguousarray(np.asarray(point, np.float32).reshape(-1)[:3])
        cap = self.size()
        out = np.empty((max(cap, 1), 4), np.float32)
        k = C.c_int64()
        _check(self._lib.icp4r_map_sector_search(self._h, _ptr(c), float(radius), float(heading), _ptr(out), cap,
                                                 C.byref(k)), "icp4r_map_sector_search")
        return out[:k.value].copy()

    def size(self) -> int:
        n = C.c_int64()
        _check(self._lib.icp4r_map_size(self._h, C.byref(n)), "icp4r_map_size")
        return n.value

    # -- radar_odometry's insertion step ---------------------------------------------------------
    def add_scan(self, scan, R, t, want_world: bool = False):
        """pointAssociateToMap (p_w = R p + t in double, stored as float) + Add_Points(.., false)."""
        a, n, stride = _cloud(scan)
        Rd = np.ascontiguousarray(np.asarray(R, np.float64).reshape(9))
        td = np.ascontiguousarray(np.asarray(t, np.float64).reshape(3))
        out = np.empty((n, 4), np.float32) if want_world else None
        _check(self._lib.icp4r_map_add_scan(self._h, _ptr(a), n, stride, _ptr(Rd), _ptr(td),
                                            _ptr(out) if out is not None else None), "icp4r_map_add_scan")
        return out

    # -- device-resident pipeline ----------------------------------------------------------------
    def sector_search_device(self, point, radius: float, heading: float, d_out: int, d_count: int, stream=None):
        """Writes the kept points (float4) to device address d_out and their int32 count to d_count."""
        c = np.ascontiguousarray(np.asarray(point, np.float32).reshape(-1)[:3])
        _check(self._lib.icp4r_map_sector_search_device(self._h, _ptr(c), float(radius), float(heading),
                                                        C.c_void_p(d_out), C.c_void_p(d_count),
                                                        C.c_void_p(stream) if stream else None),
               "icp4r_map_sector_search_device")

    def points_device(self) -> tuple[int, int]:
        p, n = C.c_void_p(), C.c_int64()
        _check(self._lib.icp4r_map_points_device(self._h, C.byref(p), C.byref(n)), "icp4r_map_points_device")
        return p.value or 0, n.value

    def time_ms(self) -> tuple[float, int]:
        ms, k = C.c_double(), C.c_int32()
        _check(self._lib.icp4r_map_time_ms(self._h, C.byref(ms), C.byref(k)), "icp4r_map_time_ms")
        return ms.value, k.value

    def reset_timers(self):
        _check(self._lib.icp4r_map_time_reset(self._h), "icp4r_map_time_reset")

"""Synthetic 4D-radar scan pairs and the reference's ``.bin`` scan format.

The reference node reads ``radar_pointcloud_<k>.bin`` as raw float32 records
``[x, y, z, intensity, v_r]`` (``src/iterative_closest_point.cpp:64-82`` reader,
``:354-385`` parse) and feeds ``x, y, z, intensity`` of EVERY point into a ``PointXYZI`` cloud
(``:404-406``, ``:482-484``; ``USE_STATIC_POINTS`` is undefined).  There is no public dataset in
this image, so pairs are generated with a seeded sensor model:

* azimuth U(-60°, 60°), elevation U(-15°, 15°), range U(2, 80) m;
* half of the points snapped to structure (with N(0, 5 cm) jitter): half of those onto range
  shells every 10 m, half onto walls ``x = 10 k`` m — so ICP has geometry to lock onto;
* intensity U(0, 30), ``v_r`` N(0, 1) (carried for ``.bin`` fidelity, unused by ICP);
* pair: target = scene; source = the same scene seen from a moved sensor,
  ``p_src = Rᵀ (p_tgt − t) + N(0, 2 cm)`` with yaw U(±5°), pitch/roll U(±0.5°),
  ``t = (U(±1), U(±0.3), U(±0.05))`` m; 10 % of each cloud replaced by independent clutter;
* pair ``i`` uses ``numpy.random.default_rng(1000 + i)``.

The ground truth ``T_gt`` maps source coordinates into the target frame (what ICP estimates:
SURVEY.md Appendix A.7).  Everything is float32.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np

RECORD_FLOATS = 5  # x, y, z, intensity, v_r


@dataclass
class ScanPair:
    src: np.ndarray  # (N, 5) float32 records
    tgt: np.ndarray  # (M, 5) float32 records
    T_gt: np.ndarray  # (4, 4) float64, source -> target

    def src_xyzi(self) -> np.ndarray:
        return np.ascontiguousarray(self.src[:, :4])

    def tgt_xyzi(self) -> np.ndarray:
        return np.ascontiguousarray(self.tgt[:, :4])


def _rot_zyx(yaw: float, pitch: float, roll: float) -> np.ndarray:
    cy, sy = np.cos(yaw), np.sin(yaw)
    cp, sp = np.cos(pitch), np.sin(pitch)
    cr, sr = np.cos(roll), np.sin(roll)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def _sensor_points(rng: np.random.Generator, n: int, structured: bool, el_deg: float = 15.0) -> np.ndarray:
    az = np.deg2rad(rng.uniform(-60.0, 60.0, n))
    el = np.deg2rad(rng.uniform(-el_deg, el_deg, n))
    r = rng.uniform(2.0, 80.0, n)
    if structured:
        kind = rng.random(n)
        shell = kind < 0.25
        wall = (kind >= 0.25) & (kind < 0.5)
        r[shell] = np.maximum(10.0, np.round(r[shell] / 10.0) * 10.0)
        # wall x = 10k: range along the ray that hits the plane
        ce = np.cos(el[wall]) * np.cos(az[wall])
        xw = np.maximum(10.0, np.round(r[wall] * ce / 10.0) * 10.0)
        r[wall] = xw / ce
        r[shell | wall] += rng.normal(0.0, 0.05, int((shell | wall).sum()))
    x = r * np.cos(el) * np.cos(az)
    y = r * np.cos(el) * np.sin(az)
    z = r * np.sin(el)
    return np.stack([x, y, z], axis=1)


def make_pair(index: int, n_src: int = 8192, n_tgt: int | None = None, clutter: float = 0.10,
              noise: float = 0.02) -> ScanPair:
    """Pair ``index`` of the benchmark/parity corpus (seed ``1000 + index``)."""
    n_tgt = n_src if n_tgt is None else n_tgt
    rng = np.random.default_rng(1000 + index)
    n_scene = max(n_src, n_tgt)
    scene = _sensor_points(rng, n_scene, structured=True)
    yaw = np.deg2rad(rng.uniform(-5.0, 5.0))
    pitch = np.deg2rad(rng.uniform(-0.5, 0.5))
    roll = np.deg2rad(rng.uniform(-0.5, 0.5))
    t = np.array([rng.uniform(-1.0, 1.0), rng.uniform(-0.3, 0.3), rng.uniform(-0.05, 0.05)])
    R = _rot_zyx(yaw, pitch, roll)
    tgt_xyz = scene[:n_tgt].copy()
    src_xyz = (scene[:n_src] - t) @ R + rng.normal(0.0, noise, (n_src, 3))  # R^T (p - t), row form
    # independent clutter replaces 10 % of each cloud (partial overlap)
    for cloud in (tgt_xyz, src_xyz):
        k = int(round(clutter * len(cloud)))
        if k:
            sel = rng.choice(len(cloud), size=k, replace=False)
            cloud[sel] = _sensor_points(rng, k, structured=False)
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t

    def records(xyz: np.ndarray) -> np.ndarray:
        rec = np.empty((len(xyz), RECORD_FLOATS), np.float32)
        rec[:, :3] = xyz
        rec[:, 3] = rng.uniform(0.0, 30.0, len(xyz))
        rec[:, 4] = rng.normal(0.0, 1.0, len(xyz))
        return rec

    return ScanPair(src=records(src_xyz), tgt=records(tgt_xyz), T_gt=T)


def make_map_pair(index: int = 0, n_src: int = 8192, scans: int = 10, pts_per_scan: int = 6554) -> ScanPair:
    """C5 scan-to-map pair: map = ``scans`` consecutive scans posed along a straight 1 m/frame
    trajectory and concatenated (M = 65,540 at the defaults); source = the next scan."""
    rng = np.random.default_rng(5000 + index)
    world = _sensor_points(rng, 4 * scans * pts_per_scan, structured=True)
    world[:, 0] += 0.5 * scans
    parts = []
    for k in range(scans):
        sel = rng.choice(len(world), size=pts_per_scan, replace=False)
        parts.append(world[sel] + rng.normal(0.0, 0.02, (pts_per_scan, 3)))
    map_xyz = np.concatenate(parts)
    pose_x = float(scans)
    yaw = np.deg2rad(rng.uniform(-3.0, 3.0))
    R = _rot_zyx(yaw, 0.0, 0.0)
    t = np.array([pose_x, rng.uniform(-0.3, 0.3), 0.0])
    sel = rng.choice(len(world), size=n_src, replace=False)
    src_xyz = (world[sel] - t) @ R + rng.normal(0.0, 0.02, (n_src, 3))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t

    def records(xyz: np.ndarray) -> np.ndarray:
        rec = np.zeros((len(xyz), RECORD_FLOATS), np.float32)
        rec[:, :3] = xyz
        rec[:, 3] = rng.uniform(0.0, 30.0, len(xyz))
        return rec

    return ScanPair(src=records(src_xyz), tgt=records(map_xyz), T_gt=T)


def make_sequence(index: int = 0, frames: int = 5, n: int = 2048, speed: float = 5.0, dt: float = 0.1,
                  yaw_rate_deg: float = 2.0, el_deg: float = 3.0, dynamic: float = 0.1,
                  doppler_noise: float = 0.02) -> tuple[list[np.ndarray], np.ndarray]:
    """A radar sequence with Doppler (seed ``9000 + index``): the sensor moves along its own x axis at
    ``speed`` m/s, turning at ``yaw_rate_deg``/s, through a static structured scene (elevations within
    ±``el_deg``, where the node's planar sine model fits).  Static points get the radial velocity
    ``v_r = -û·v_sensor`` (+ N(0, doppler_noise)); a ``dynamic`` fraction moves on its own
    (``v_r += U(1.5, 5)`` m/s, so the node's ``delta > 0.2`` test flags it).  Returns the per-frame
    (N, 5) records and the true sensor velocity in the sensor frame — the least squares over the
    static points recovers ``-v_sensor`` (the node's Vxyz convention, K·V = v_r)."""
    rng = np.random.default_rng(9000 + index)
    world = _sensor_points(rng, 3 * n, structured=True, el_deg=el_deg)
    v_sensor = np.array([speed, 0.0, 0.0])
    t = np.zeros(3)
    yaw = 0.0
    out = []
    for _ in range(frames):
        R = _rot_zyx(yaw, 0.0, 0.0)
        sel = rng.choice(len(world), size=n, replace=False)
        p = (world[sel] - t) @ R + rng.normal(0.0, 0.02, (n, 3))  # R^T (p - t), row form
        u = p / np.linalg.norm(p, axis=1, keepdims=True)
        vr = -(u @ v_sensor) + rng.normal(0.0, doppler_noise, n)
        dyn = rng.random(n) < dynamic
        vr[dyn] += rng.uniform(1.5, 5.0, int(dyn.sum()))
        rec = np.empty((n, RECORD_FLOATS), np.float32)
        rec[:, :3] = p
        rec[:, 3] = rng.uniform(0.0, 30.0, n)
        rec[:, 4] = vr
        out.append(rec)
        t = t + R @ v_sensor * dt
        yaw += np.deg2rad(yaw_rate_deg) * dt
    return out, v_sensor


def write_sequence(folder: str | os.PathLike, frames: list[np.ndarray]) -> None:
    """The node's input layout (:303-304): ``<folder>/data/radar_pointcloud_<k>.bin``."""
    d = os.path.join(folder, "data")
    os.makedirs(d, exist_ok=True)
    for k, rec in enumerate(frames):
        write_bin(os.path.join(d, f"radar_pointcloud_{k}.bin"), rec)


def write_bin(path: str | os.PathLike, records: np.ndarray) -> None:
    """Write a scan in the reference's raw float32 5-float record format."""
    np.ascontiguousarray(records, dtype=np.float32).tofile(path)


def read_bin(path: str | os.PathLike) -> np.ndarray:
    """``read_radar_data`` (iterative_closest_point.cpp:64-82): whole file as float32; a missing
    file yields an empty scan.  Returns (N, 5) records, N = floats // 5 (the node's ``size()/5``)."""
    if not os.path.exists(path):
        return np.zeros((0, RECORD_FLOATS), np.float32)
    flat = np.fromfile(path, dtype=np.float32)
    n = flat.size // RECORD_FLOATS
    return flat[: n * RECORD_FLOATS].reshape(n, RECORD_FLOATS)


def records_to_xyzi(records: np.ndarray) -> np.ndarray:
    """The node's PointXYZI fill (``:404-406``): x, y, z, intensity; ``v_r`` is dropped."""
    return np.ascontiguousarray(records[:, :4], dtype=np.float32)

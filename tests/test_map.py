"""Scan-to-map store + Sector_Search: oracle known answers (CPU) and the HIP
store against the oracle (GPU).

Reference: radar_odometry.cpp:92, :347-348, :382-396; third_party/ikd-Tree/ikd_Tree.cpp:415-419,
1098-1140, 1427-1448.  Parity unpinned by the reference (no fixtures; ikd-Tree needs PCL headers to
build) — pinned by the known answers below.  Bar: the kept SET equals the oracle's, except points
whose heading difference sits within 1e-3 deg of a sector edge (|dh| = 60 or 300), where the
device asinf and glibc's asinf may round differently; world-frame points bit-exact.
"""
import math

import numpy as np
import pytest

EDGE_TOL_DEG = 1e-3


def _map(rng, n, extent=150.0):
    pts = np.zeros((n, 4), np.float32)
    pts[:, :3] = rng.uniform(-extent, extent, (n, 3)).astype(np.float32)
    pts[:, 2] *= 0.1
    pts[:, 3] = rng.uniform(0, 50, n).astype(np.float32)
    return pts


def _at(radius, h_deg, z=0.0):
    """A point at `radius` with calc_heading == h (0 along +y, +90 along -x) around the origin."""
    a = math.radians(h_deg)
    return [-radius * math.sin(a), radius * math.cos(a), z, 1.0]


# ------------------------------------------------------------------------------------------- oracle
def test_heading_known_answers(oracle_mod):
    c = np.zeros(3, np.float32)
    for p, h in (([0, 10, 0], 0.0), ([10, 0, 0], -90.0), ([0, -10, 0], 180.0), ([-10, 0, 0], 90.0),
                 ([-7, -7, 0], 135.0), ([7, -7, 0], -135.0)):
        assert oracle_mod.calc_heading(np.array(p, np.float32), c) == pytest.approx(h, abs=1e-5)


def test_sector_keep_known_answers_and_precedence_quirk(oracle_mod):
    pts = np.array([
        _at(10, 0),      # 0: ahead, near            -> kept
        _at(79, 50),     # 1: inside radius and cone  -> kept
        _at(81, 0),      # 2: beyond radius           -> not kept
        _at(10, 90),     # 3: outside the +-60 cone   -> not kept
        _at(10, 180),    # 4: behind                  -> not kept
        _at(500, -175),  # 5: |dh| = 345 > 300: kept at ANY distance (A && B && C || D, ikd_Tree.cpp:1114-1116)
        [0, 0, 0, 1],    # 6: the centre itself: heading NaN -> never kept
        _at(50, -59),    # 7: inside the cone (dh = 59) -> kept
    ], np.float32)
    kept = oracle_mod.sector_search(pts, [0, 0, 0], 80.0, 0.0)
    assert list(kept) == [0, 1, 7]
    kept = oracle_mod.sector_search(pts, [0, 0, 0], 80.0, 170.0)  # heading 170: point 5 has |dh| = 345
    assert 5 in kept and 4 in kept and 0 not in kept and 6 not in kept


def test_associate_to_map_is_double_then_float(oracle_mod):
    rng = np.random.default_rng(3)
    pts = _map(rng, 1000)
    yaw = 0.7
    R = np.array([[math.cos(yaw), -math.sin(yaw), 0], [math.sin(yaw), math.cos(yaw), 0], [0, 0, 1]])
    t = np.array([12.25, -3.5, 0.75])
    out = oracle_mod.associate_to_map(pts, R, t)
    p = pts[:, :3].astype(np.float64)
    ref = (((R[:, 0][None] * p[:, :1]) + R[:, 1][None] * p[:, 1:2]) + R[:, 2][None] * p[:, 2:3]) + t[None]
    assert (out[:, :3] == ref.astype(np.float32)).all() and (out[:, 3] == pts[:, 3]).all()


def test_oracle_vs_numpy_twin(oracle_mod):
    """An independent float32 numpy restatement agrees except at sector edges."""
    rng = np.random.default_rng(4)
    pts = _map(rng, 20000)
    c = np.array([3.0, -2.0, 0.5], np.float32)
    d = pts[:, :3] - c
    d2 = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    r = d[:, 0] / np.sqrt(d2)
    a = np.arcsin(r).astype(np.float32)
    h = np.where(d[:, 1] < 0, 180.0 + (a * np.float32(180.0)).astype(np.float64) / math.pi,
                 (-a * np.float32(180.0)).astype(np.float64) / math.pi).astype(np.float32)
    h = np.where((h > 180) & (h < 360), h - np.float32(360), h)
    for heading in (0.0, 37.5, -120.0, 179.0):
        dh = np.abs(h - np.float32(heading))
        twin = set(np.nonzero(((d2 <= np.float32(80.0 * 80.0)) & (dh < 60)) | (dh > 300))[0])
        orc = set(oracle_mod.sector_search(pts, c, 80.0, heading).tolist())
        for i in twin ^ orc:
            assert min(abs(dh[i] - 60), abs(dh[i] - 300)) < EDGE_TOL_DEG, i


def test_submap_order_does_not_change_registrations(oracle_mod):
    """ikd-Tree's Search_by_sector returns the kept set in its tree's pre-order
    (ikd_Tree.cpp:1114-1138); the restatement returns insertion order.  The set is the same, and the
    registrations are invariant to the target's order: the correspondences are formed and summed in
    SOURCE index order (icp.hpp / fast_gicp), each source's nearest target is the same point whatever
    the order unless two DISTINCT points tie exactly in distance (the (d², index) key then picks by
    position; identical duplicates — accumulated scans — give the same coordinates either way), and
    GICP's target covariances are k-NN sets of the same kind.  So any permutation of the submap — the
    pre-order being one — gives bit-identical ICP and GICP results; checked here on the radar_odometry
    scene (submap of the synthetic map around the pose, several seeded permutations)."""
    from icp4r import synth

    mp = synth.make_map_pair(2)
    map_pts, scan = mp.tgt_xyzi(), mp.src_xyzi()
    kept = oracle_mod.sector_search(map_pts, [0.0, 0.0, 0.0], 80.0, 0.0)
    sub = map_pts[kept]
    assert len(sub) > 1000
    ref = oracle_mod.align(scan, sub, numerics=oracle_mod.NUM_F32, max_iterations=15)
    gref = oracle_mod.gicp_align(scan[:1500], sub, k=10)
    rng = np.random.default_rng(17)
    for rep in range(3):
        perm = rng.permutation(len(sub))
        o = oracle_mod.align(scan, sub[perm], numerics=oracle_mod.NUM_F32, max_iterations=15)
        assert (o["T"] == ref["T"]).all() and o["fitness"] == ref["fitness"], rep
        assert o["iterations"] == ref["iterations"] and o["n_correspondences"] == ref["n_correspondences"], rep
        g = oracle_mod.gicp_align(scan[:1500], sub[perm], k=10)
        assert (g["T"] == gref["T"]).all() and g["iterations"] == gref["iterations"], rep


# ------------------------------------------------------------------------------------------- device
def _edge_ok(oracle_mod, pts, c, heading, idx):
    h = oracle_mod.calc_heading(pts[idx], np.asarray(c, np.float32))
    dh = abs(h - heading)
    return min(abs(dh - 60), abs(dh - 300)) < EDGE_TOL_DEG


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 1000, 300_001])
def test_sector_search_matches_oracle(gpu_ctx, oracle_mod, n):
    from icp4r.mapstore import KD_TREE

    rng = np.random.default_rng(n)
    pts = _map(rng, n)
    if n > 100:  # exact edge cases: on the radius, in the cone, behind, the centre
        pts[:8] = np.array([_at(80, 10), _at(80, 60), _at(80, -60), _at(20, 180), [0, 0, 0, 1], _at(600, 179),
                            _at(600, -179), _at(1, 0)], np.float32)
    tree = KD_TREE(0.3, 0.6, 0.5, ctx=gpu_ctx)
    tree.Build(pts[: n // 2])
    tree.Add_Points(pts[n // 2:], False)
    assert tree.size() == n
    for c, heading in (([0, 0, 0], 0.0), ([10.5, -4.0, 1.0], 75.0), ([0, 0, 0], 179.5), ([-30, 20, 0], -90.0)):
        got = tree.Sector_Search(c, 80.0, heading)
        ref = oracle_mod.sector_search(pts, c, 80.0, heading)
        gs = {tuple(p) for p in got.tolist()}
        rs = {tuple(pts[i]) for i in ref.tolist()}
        for p in gs ^ rs:
            i = int(np.nonzero((pts == np.array(p, np.float32)).all(1))[0][0])
            assert _edge_ok(oracle_mod, pts, c, heading, i), p
        if gs == rs:  # insertion order when the sets agree
            assert (got == pts[ref]).all()


@pytest.mark.gpu
def test_add_scan_bitexact_and_growth(gpu_ctx, oracle_mod):
    from icp4r.mapstore import KD_TREE

    rng = np.random.default_rng(9)
    tree = KD_TREE(ctx=gpu_ctx)
    world = []
    for k in range(40):  # 40 scans x 6554 = 262k points: several capacity doublings
        scan = _map(rng, 6554, 60.0)
        yaw = 0.05 * k
        R = np.array([[math.cos(yaw), -math.sin(yaw), 0], [math.sin(yaw), math.cos(yaw), 0], [0, 0, 1]])
        t = np.array([2.0 * k, 0.3 * k, 0.01 * k])
        w = tree.add_scan(scan, R, t, want_world=True)
        assert (w == oracle_mod.associate_to_map(scan, R, t)).all()
        world.append(w)
    allw = np.concatenate(world)
    assert tree.size() == len(allw)
    got = tree.Sector_Search([0, 0, 0], 1e9, 0.0)  # radius huge: the cone only
    ref = oracle_mod.sector_search(allw, [0, 0, 0], 1e9, 0.0)
    assert len(got) == pytest.approx(len(ref), abs=2)


@pytest.mark.gpu
def test_map_errors_and_empty(gpu_ctx):
    import icp4r
    from icp4r.mapstore import KD_TREE

    tree = KD_TREE(ctx=gpu_ctx)
    assert tree.size() == 0 and len(tree.Sector_Search([0, 0, 0], 80.0, 0.0)) == 0
    with pytest.raises(icp4r.ICP4RError):
        tree.Add_Points(np.zeros((3, 4), np.float32), True)  # the downsampling insert is not on this path
    tree.Build(np.zeros((0, 4), np.float32))
    assert tree.size() == 0


@pytest.mark.gpu
def test_scan_to_map_registration_device_resident(gpu_ctx, oracle_mod):
    """radar_odometry's loop body on the device: add the scan, sector-search the submap into device
    memory (count as a device int32), register the next scan against it with the batch API — equal
    bit for bit to the host path (sector search to host, then icp4r_align)."""
    import torch

    import icp4r
    from icp4r import synth
    from icp4r.mapstore import KD_TREE

    mp = synth.make_map_pair(2)
    map_pts, scan = mp.tgt_xyzi(), mp.src_xyzi()
    tree = KD_TREE(ctx=gpu_ctx)
    tree.Build(map_pts)
    center, heading = [0.0, 0.0, 0.0], 0.0
    host_sub = tree.Sector_Search(center, 80.0, heading)
    dev = torch.device("cuda", 0)
    d_sub = torch.zeros((tree.size(), 4), dtype=torch.float32, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()  # torch's fills run on its stream; the library uses the context's
    tree.sector_search_device(center, 80.0, heading, d_sub.data_ptr(), d_cnt.data_ptr())
    torch.cuda.synchronize()
    assert int(d_cnt.item()) == len(host_sub) and (d_sub[: len(host_sub)].cpu().numpy() == host_sub).all()
    src = torch.from_numpy(scan).to(dev)
    zero = torch.zeros(1, dtype=torch.int64, device=dev)
    sn = torch.tensor([len(scan)], dtype=torch.int32, device=dev)
    res = torch.zeros((1, 96), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    p = icp4r.default_params(max_iterations=15)
    batch = icp4r.Batch(src=src.data_ptr(), tgt=d_sub.data_ptr(), src_off=zero.data_ptr(), src_n=sn.data_ptr(),
                        tgt_off=zero.data_ptr(), tgt_n=d_cnt.data_ptr(), npairs=1, max_src_n=len(scan),
                        max_tgt_n=tree.size())
    gpu_ctx.align_batch_device(batch, p, res.data_ptr(), None)
    gpu_ctx.synchronize()
    r_dev = np.frombuffer(res.cpu().numpy().tobytes(), dtype=icp4r.RESULT_DTYPE)[0]
    r_host, _ = gpu_ctx.align(scan, host_sub, p)
    assert (r_dev["T"] == np.array(r_host.T, np.float32)).all() and r_dev["iterations"] == r_host.iterations
    o = oracle_mod.align(scan, host_sub, numerics=oracle_mod.NUM_F32, max_iterations=15)
    assert (r_host.matrix() == o["T"]).all()


@pytest.mark.gpu
@pytest.mark.parametrize("exe_name", ["map_callsite", "pcl18_map_callsite"])
def test_ikd_facade_callsite(oracle_mod, exe_name):
    """tests/cpp/map_callsite.cpp: radar_odometry's map calls through include/icp4r/ikd_compat.hpp
    (namespace-scope KD_TREE, Build, set_downsample_param, Add_Points(.., false), Sector_Search) give
    the oracle's submap, intensities included."""
    import os
    import subprocess

    from helpers import GOLDEN_DIR

    from icp4r import synth

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "cpp", "_build", exe_name)  # stand-in types / PCL-1.8-shaped tree
    a, b = (os.path.join(GOLDEN_DIR, f) for f in ("c2_pair1_8k_tgt.bin", "c2_pair1_8k_src.bin"))
    x, y, yaw = 5.0, -3.0, 30.0
    r = subprocess.run([exe, a, b, str(x), str(y), str(yaw)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    lines = r.stdout.strip().split("\n")
    head = lines[0].split()
    got = np.array([[float(v) for v in ln.split()] for ln in lines[1:]], np.float32).reshape(-1, 4)
    first = synth.records_to_xyzi(synth.read_bin(a))
    nxt = synth.records_to_xyzi(synth.read_bin(b))
    c, s_ = math.cos(math.radians(yaw)), math.sin(math.radians(yaw))
    R = np.array([[c, -s_, 0], [s_, c, 0], [0, 0, 1]])
    world = oracle_mod.associate_to_map(nxt, R, np.array([x, y, 0.0]))
    allp = np.concatenate([first, world])
    assert int(head[1]) == len(allp)
    ref = oracle_mod.sector_search(allp, [x, y, 0.0], 80.0, yaw)
    gs, rs = {tuple(p) for p in got.tolist()}, {tuple(allp[i]) for i in ref.tolist()}
    for p in gs ^ rs:
        i = int(np.nonzero((allp == np.array(p, np.float32)).all(1))[0][0])
        assert _edge_ok(oracle_mod, allp, [x, y, 0.0], yaw, i), p
    if gs == rs:
        assert (got == allp[ref]).all()  # insertion order, intensity carried through

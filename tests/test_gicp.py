"""Generalized ICP: fast_gicp's FastGICPSingleThread as the reference's
radar_odometry node calls it (src/radar_odometry.cpp:398-411) — oracle known answers on CPU, HIP
product parity on the GPU.

Parity status: unpinned by the reference (fast_gicp is not vendored and not in this image; the node
needs ROS/PCL).  The oracle (oracle/gicp_oracle.c) is pinned by known answers: covariance structure
of analytic clouds, independent numpy covariances, and pairs with a known rigid transform.  Bars
(GPU vs oracle): covariances within 1e-9 relative (same double arithmetic; the k-NN sets identical);
poses within 1e-5 (rotation rad / translation m: the Gauss-Newton sums run in a different order);
nr_iterations and hasConverged identical; the fitness within 1e-6 relative.
"""
import numpy as np
import pytest

from helpers import pose_err
from icp4r import synth

TOL_KAT_T = 0.02  # m: 2 cm point noise, 10 % clutter
TOL_KAT_R = np.deg2rad(0.2)


def _xyz(rec):
    return np.ascontiguousarray(rec[:, :3], np.float32)


def _grid_plane(n_side=20, spacing=0.1, seed=0):
    rng = np.random.default_rng(seed)
    g = np.stack(np.meshgrid(np.arange(n_side), np.arange(n_side)), -1).reshape(-1, 2) * spacing
    pts = np.zeros((len(g), 3), np.float32)
    pts[:, :2] = g + rng.uniform(-0.01, 0.01, g.shape)
    return pts


def _scene(seed, n=1500):
    """A pair with a known rigid transform: synth's structured scene, no clutter."""
    p = synth.make_pair(seed, n, clutter=0.0, noise=0.005)
    return _xyz(p.src), _xyz(p.tgt), p.T_gt


def _knn_cov_numpy(c, k):
    c = c.astype(np.float32)
    d = ((c[:, None, :] - c[None, :, :]) ** 2)
    d2 = (d[..., 0] + d[..., 1]) + d[..., 2]
    idx = np.lexsort((np.broadcast_to(np.arange(len(c)), d2.shape), d2), axis=1)[:, :k]
    out = np.zeros((len(c), 3, 3))
    for i in range(len(c)):
        nb = c[idx[i]].astype(np.float64)
        m = nb.mean(0)
        out[i] = (nb - m).T @ (nb - m) / k
    return out


# ---------------------------------------------------------------------------------------------- oracle
def test_oracle_covariance_matches_numpy(oracle_mod):
    rng = np.random.default_rng(3)
    c = rng.normal(0, 1, (300, 3)).astype(np.float32)
    for k in (5, 20):
        got = oracle_mod.gicp_covariances(c, k, oracle_mod.GICP_REG_NONE)
        np.testing.assert_allclose(got, _knn_cov_numpy(c, k), rtol=1e-10, atol=1e-12)


def test_oracle_plane_regularisation(oracle_mod):
    pts = _grid_plane()
    C = oracle_mod.gicp_covariances(pts, 20, oracle_mod.GICP_REG_PLANE)
    for M in C[::37]:
        w, V = np.linalg.eigh(M)
        np.testing.assert_allclose(w, [1e-3, 1.0, 1.0], atol=1e-9)
        assert abs(abs(V[2, 0]) - 1.0) < 1e-3  # the 1e-3 axis is the plane normal (z)
    Cm = oracle_mod.gicp_covariances(pts, 20, oracle_mod.GICP_REG_MIN_EIG)
    assert np.all(np.linalg.eigvalsh(Cm) >= 1e-3 - 1e-12)
    Cn = oracle_mod.gicp_covariances(pts, 20, oracle_mod.GICP_REG_NORMALIZED_MIN_EIG)
    np.testing.assert_allclose(np.linalg.eigvalsh(Cn)[:, -1], 1.0, atol=1e-9)
    Cf = oracle_mod.gicp_covariances(pts, 20, oracle_mod.GICP_REG_FROBENIUS)
    np.testing.assert_allclose(np.linalg.norm(np.linalg.inv(Cf), axis=(1, 2)), 1.0, rtol=1e-9)


def test_oracle_identity_converges_at_once(oracle_mod):
    src, _, _ = _scene(1, 800)
    r = oracle_mod.gicp_align(src, src, k=5)
    assert r["converged"] and r["iterations"] == 0 and not r["lm_failed"]
    assert np.abs(r["T"] - np.eye(4)).max() < 1e-9
    assert r["n_valid"] == len(src)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_oracle_recovers_known_transform(oracle_mod, seed):
    src, tgt, T = _scene(seed)
    for k in (5, 20):
        r = oracle_mod.gicp_align(src, tgt, k=k)
        assert r["converged"] and not r["lm_failed"]
        dt, dr = pose_err(r["T"], T)
        assert dt < TOL_KAT_T and dr < TOL_KAT_R, (k, dt, dr)


def test_oracle_guess_and_distance_gate(oracle_mod):
    src, tgt, T = _scene(4)
    r = oracle_mod.gicp_align(src, tgt, guess=T, k=5)
    assert r["converged"] and r["iterations"] <= 2
    # a gate shorter than every correspondence: no residual, the first LM step is the identity
    far = src + np.float32(100.0)
    r = oracle_mod.gicp_align(far, tgt, k=5, max_correspondence_distance=1.0)
    assert r["n_valid"] == 0 and r["converged"] and r["iterations"] == 0
    assert np.abs(r["T"] - np.eye(4)).max() == 0.0


# ---------------------------------------------------------------------------------------------- GPU
def _gicp():
    from icp4r import gicp

    return gicp


@pytest.mark.gpu
@pytest.mark.parametrize("reg", [0, 1, 2, 3, 4])
def test_gpu_covariances_match_oracle(gpu_ctx, oracle_mod, reg):
    gicp = _gicp()
    src, tgt, _ = _scene(5, 3000)
    for cloud in (src, _grid_plane(30)):
        for k in (5, 20, 32):
            got = gicp.covariances(cloud, k, reg, ctx=gpu_ctx)
            want = oracle_mod.gicp_covariances(cloud, k, reg)
            scale = np.abs(want).max(axis=(1, 2), keepdims=True)
            assert np.abs(got - want).max() <= 1e-9 * max(1.0, float(scale.max())), (k, reg)


@pytest.mark.gpu
def test_gpu_pruned_knn_equals_brute_force(gpu_ctx, oracle_mod, plan):
    """The Morton-pruned k-NN (clouds >= 512 points) returns exactly the brute-force neighbour sets:
    covariances bit-identical, including clouds with duplicated points (distance ties), for every
    number of lanes per query."""
    gicp = _gicp()
    src, tgt, _ = _scene(8, 6000)
    dup = np.concatenate([tgt[:1500], tgt[:1500], tgt[700:1400]])  # every point at least twice
    for cloud in (src, dup, _grid_plane(40)):
        for k in (1, 5, 20, 32):
            plan(gicp_cov_brute=1, gicp_knn_lanes=1)
            brute = gicp.covariances(cloud, k, 3, ctx=gpu_ctx)
            for mode in (1, 0):  # brute force, pruned (plan option gicp_cov_brute)
                for lanes in (1, 2, 4, 8):  # lanes per query (plan option gicp_knn_lanes)
                    plan(gicp_cov_brute=mode, gicp_knn_lanes=lanes)
                    got = gicp.covariances(cloud, k, 3, ctx=gpu_ctx)
                    np.testing.assert_array_equal(got, brute, err_msg=f"k={k} brute={mode} L={lanes}")
            plan(gicp_cov_brute=0, gicp_knn_lanes=0)
    want = oracle_mod.gicp_covariances(dup, 5, 3)
    np.testing.assert_allclose(gicp.covariances(dup, 5, 3, ctx=gpu_ctx), want, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,k", [(0, 5), (1, 5), (2, 20), (3, 20), (6, 10)])
def test_gpu_align_matches_oracle(gpu_ctx, oracle_mod, seed, k):
    gicp = _gicp()
    src, tgt, T = _scene(seed, 2000)
    p = gicp.default_params(k_correspondences=k)
    r, aligned = gicp.align(src, tgt, p, want_aligned=True, ctx=gpu_ctx)
    o = oracle_mod.gicp_align(src, tgt, k=k)
    Tg = r.matrix()
    dt, dr = pose_err(Tg, o["T"])
    assert dt < 1e-5 and dr < 1e-5, (dt, dr)
    assert r.iterations == o["iterations"] and bool(r.converged) == o["converged"]
    assert r.n_correspondences == o["n_valid"]
    # final_transformation_ = x0.cast<float>(); align's output = transformPointCloud(input, final)
    Tf = o["T"].astype(np.float32)
    dtk, drk = pose_err(Tf, T)
    assert dtk < TOL_KAT_T and drk < TOL_KAT_R
    want = np.empty_like(src)
    R, t = Tg[:3, :3], Tg[:3, 3]
    for rr in range(3):
        v = R[rr, 0] * src[:, 0]
        v = v + R[rr, 1] * src[:, 1]
        v = v + R[rr, 2] * src[:, 2]
        want[:, rr] = v + t[rr]
    np.testing.assert_array_equal(aligned[:, :3], want)
    # getFitnessScore(): mean NN d² of the aligned cloud (float L2_Simple), keys in double
    d = aligned[:, None, :3] - tgt[None, :, :]
    d2 = ((d[..., 0] * d[..., 0]) + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
    fit = float(np.mean(d2.min(1).astype(np.float64)))
    assert abs(r.fitness - fit) <= 1e-6 * max(fit, 1e-12)


@pytest.mark.gpu
def test_gpu_align_guess_gate_and_errors(gpu_ctx, oracle_mod):
    import icp4r

    gicp = _gicp()
    src, tgt, T = _scene(4, 1500)
    r, _ = gicp.align(src, tgt, gicp.default_params(k_correspondences=5), guess=T, ctx=gpu_ctx)
    o = oracle_mod.gicp_align(src, tgt, guess=T, k=5)
    assert r.iterations == o["iterations"] and r.converged
    assert max(pose_err(r.matrix(), o["T"])) < 1e-5
    far = src + np.float32(100.0)
    r, _ = gicp.align(far, tgt, gicp.default_params(k_correspondences=5, max_correspondence_distance=1.0), ctx=gpu_ctx)
    assert r.converged and r.iterations == 0 and r.n_correspondences == 0
    np.testing.assert_array_equal(r.matrix(), np.eye(4, dtype=np.float32))
    r, _ = gicp.align(src, tgt[:0], ctx=gpu_ctx)
    assert r.status == icp4r.E_EMPTY and not r.converged
    with pytest.raises(icp4r.ICP4RError):
        gicp.align(src, tgt, gicp.default_params(k_correspondences=33), ctx=gpu_ctx)
    with pytest.raises(icp4r.ICP4RError):
        gicp.covariances(src, 0, ctx=gpu_ctx)


@pytest.mark.gpu
def test_gpu_small_clouds_fewer_points_than_k(gpu_ctx, oracle_mod):
    gicp = _gicp()
    src, tgt, _ = _scene(7, 200)
    s, t = src[:12], tgt[:15]
    got = gicp.covariances(s, 20, 3, ctx=gpu_ctx)
    np.testing.assert_allclose(got, oracle_mod.gicp_covariances(s, 20, 3), rtol=1e-9, atol=1e-12)
    r, _ = gicp.align(s, t, gicp.default_params(k_correspondences=20), ctx=gpu_ctx)
    o = oracle_mod.gicp_align(s, t, k=20)
    assert r.iterations == o["iterations"] and bool(r.converged) == o["converged"]
    assert max(pose_err(r.matrix(), o["T"])) < 1e-4


@pytest.mark.gpu
def test_gpu_lm_trials_speculative_equals_one_by_one(gpu_ctx, oracle_mod, plan):
    """The iteration evaluates its first LM trials together (plan option gicp_spec, default 2) and any
    further trial one by one, each summed slice by slice in the same order: every gicp_spec gives
    bit-identical results, and so does every spread of the slices over workgroups (gicp_grid). Cases: far initial poses (rejected trials), lm_max_iterations = 1 and 0,
    a large initial damping (lm_init_lambda_factor 1e-2), and a source of 17k points (512-point slices)."""
    gicp = _gicp()
    cases = []
    for seed in (0, 3):
        src, tgt, _ = _scene(seed, 2000)
        c, s_ = np.cos(0.6), np.sin(0.6)
        guess = np.eye(4, dtype=np.float32)
        guess[:2, :2] = [[c, -s_], [s_, c]]
        guess[:3, 3] = [0.8, -0.5, 0.3]
        for lm in (10, 1, 0):
            cases.append((src, tgt, guess, gicp.default_params(k_correspondences=5, lm_max_iterations=lm)))
        # a damping large enough to change every step: the first λ must be the same whether the trials
        # are solved up front (gicp_spec > 0) or one by one (gicp_spec = 0)
        cases.append((src, tgt, guess, gicp.default_params(k_correspondences=5, lm_init_lambda_factor=1e-2)))
    src, tgt, _ = _scene(9, 17000)
    cases.append((src, tgt, None, gicp.default_params(k_correspondences=5)))
    for src, tgt, guess, p in cases:
        runs = []
        for spec, grid in ((0, 2048), (1, 3), (2, 1), (2, 2048)):
            plan(gicp_spec=spec, gicp_grid=grid)
            r, aligned = gicp.align(src, tgt, p, guess=guess, want_aligned=True, ctx=gpu_ctx)
            runs.append((r.matrix(), r.iterations, r.converged, r.fitness, r.status, aligned))
        plan(gicp_spec=2, gicp_grid=2048)
        for other in runs[:3]:
            np.testing.assert_array_equal(other[0], runs[3][0])
            assert other[1:5] == runs[3][1:5]
            np.testing.assert_array_equal(other[5], runs[3][5])
    o = oracle_mod.gicp_align(src, tgt, k=5)
    r = runs[3]
    assert r[1] == o["iterations"] and bool(r[2]) == o["converged"]
    assert max(pose_err(r[0], o["T"])) < 1e-5


@pytest.mark.gpu
def test_gpu_batch_device_equals_single(gpu_ctx):
    import torch

    import icp4r

    gicp = _gicp()
    pairs = [_scene(s, 600 + 150 * s) for s in range(6)]
    src = np.concatenate([np.pad(p[0], ((0, 0), (0, 1))) for p in pairs]).astype(np.float32)
    tgt = np.concatenate([np.pad(p[1], ((0, 0), (0, 1))) for p in pairs]).astype(np.float32)
    sn = np.array([len(p[0]) for p in pairs], np.int32)
    tn = np.array([len(p[1]) for p in pairs], np.int32)
    so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
    to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
    dev = torch.device("cuda:0")
    ts = {k: torch.from_numpy(v).to(dev) for k, v in dict(src=src, tgt=tgt, sn=sn, tn=tn, so=so, to=to).items()}
    res = torch.zeros(len(pairs) * icp4r.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    b = icp4r.Batch()
    b.src, b.tgt = ts["src"].data_ptr(), ts["tgt"].data_ptr()
    b.src_off, b.src_n, b.tgt_off, b.tgt_n = ts["so"].data_ptr(), ts["sn"].data_ptr(), ts["to"].data_ptr(), ts["tn"].data_ptr()
    b.npairs, b.max_src_n, b.max_tgt_n = len(pairs), int(sn.max()), int(tn.max())
    p = gicp.default_params(k_correspondences=5)
    gicp.align_batch_device(b, p, res.data_ptr(), ctx=gpu_ctx)
    gpu_ctx.synchronize()
    out = np.frombuffer(res.cpu().numpy().tobytes(), icp4r.RESULT_DTYPE)
    for i, (s, t, _) in enumerate(pairs):
        r, _ = gicp.align(s, t, p, ctx=gpu_ctx)
        np.testing.assert_array_equal(out[i]["T"], np.array(r.T, np.float32))
        assert out[i]["iterations"] == r.iterations and out[i]["converged"] == r.converged
        assert out[i]["fitness"] == r.fitness


@pytest.mark.gpu
def test_gpu_device_calls_back_to_back(gpu_ctx):
    """Two device-API calls on one context with no synchronisation between them (the API returns with
    its work queued): the second must not read the first's late active-pair check — each check carries
    a sequence number — and both equal the same pairs registered alone."""
    import torch

    import icp4r

    gicp = _gicp()
    dev = torch.device("cuda:0")

    def batch(pairs):
        src = np.concatenate([np.pad(p[0], ((0, 0), (0, 1))) for p in pairs]).astype(np.float32)
        tgt = np.concatenate([np.pad(p[1], ((0, 0), (0, 1))) for p in pairs]).astype(np.float32)
        sn = np.array([len(p[0]) for p in pairs], np.int32)
        tn = np.array([len(p[1]) for p in pairs], np.int32)
        so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
        to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
        ts = {k: torch.from_numpy(v).to(dev) for k, v in dict(src=src, tgt=tgt, sn=sn, tn=tn, so=so, to=to).items()}
        b = icp4r.Batch()
        b.src, b.tgt = ts["src"].data_ptr(), ts["tgt"].data_ptr()
        b.src_off, b.src_n, b.tgt_off, b.tgt_n = ts["so"].data_ptr(), ts["sn"].data_ptr(), ts["to"].data_ptr(), ts["tn"].data_ptr()
        b.npairs, b.max_src_n, b.max_tgt_n = len(pairs), int(sn.max()), int(tn.max())
        return b, ts

    # the first batch stops early (identical clouds converge at once) while the second needs many
    # iterations: a late check of the first would read "0 active" and stop the second
    first = [(p[1].copy(), p[1], None) for p in (_scene(s, 1200) for s in range(3))]
    second = [_scene(10 + s, 1500) for s in range(3)]
    p1 = gicp.default_params(k_correspondences=5)
    p2 = gicp.default_params(k_correspondences=5, max_iterations=40)
    b1, keep1 = batch(first)
    b2, keep2 = batch(second)
    r1 = torch.zeros(len(first) * icp4r.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    r2 = torch.zeros(len(second) * icp4r.RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    for _ in range(3):
        gicp.align_batch_device(b1, p1, r1.data_ptr(), ctx=gpu_ctx)
        gicp.align_batch_device(b2, p2, r2.data_ptr(), ctx=gpu_ctx)
    gpu_ctx.synchronize()
    for res, pairs, p in ((r1, first, p1), (r2, second, p2)):
        out = np.frombuffer(res.cpu().numpy().tobytes(), icp4r.RESULT_DTYPE)
        for i, (s, t, _) in enumerate(pairs):
            r, _ = gicp.align(s, t, p, ctx=gpu_ctx)
            np.testing.assert_array_equal(out[i]["T"], np.array(r.T, np.float32))
            assert out[i]["iterations"] == r.iterations and out[i]["converged"] == r.converged


@pytest.mark.gpu
def test_gpu_fast_gicp_facade(gpu_ctx):
    gicp = _gicp()
    src, tgt, T = _scene(2, 1200)
    reg = gicp.FastGICPSingleThread(gpu_ctx)
    reg.clearTarget()
    reg.clearSource()
    reg.setInputTarget(tgt)
    reg.setInputSource(src)
    reg.setCorrespondenceRandomness(5)
    out = reg.align()
    assert reg.hasConverged() and out.shape == src.shape
    dt, dr = pose_err(reg.getFinalTransformation(), T)
    assert dt < TOL_KAT_T and dr < TOL_KAT_R
    assert 0.0 <= reg.getFitnessScore() < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("exe_name", ["gicp_callsite", "pcl18_gicp_callsite"])
def test_gpu_fast_gicp_cpp_callsite(gpu_ctx, oracle_mod, tmp_path, exe_name):
    """tests/cpp/gicp_callsite.cpp: radar_odometry's GICP block (radar_odometry.cpp:398-411) through
    include/icp4r/fast_gicp_compat.hpp — the same bits as the Python facade on the same inputs, and the
    oracle's pose within the GICP bar."""
    import os
    import subprocess

    gicp = _gicp()
    src, tgt, T = _scene(4, 1500)
    rec = lambda xyz: np.concatenate([xyz, np.ones((len(xyz), 1), np.float32), np.zeros((len(xyz), 1), np.float32)], 1)
    a, b = tmp_path / "scan_map.bin", tmp_path / "submap.bin"
    synth.write_bin(a, rec(src))
    synth.write_bin(b, rec(tgt))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "tests", "cpp", "_build", exe_name)  # stand-in types / PCL-1.8-shaped tree
    r = subprocess.run([exe, str(a), str(b)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    head, tl = r.stdout.strip().split("\n")[:2]
    conv, score, iters, nout = head.split()
    Tc = np.array([float(v) for v in tl.split()], np.float32).reshape(4, 4).T  # column-major
    res, _ = gicp.align(src, tgt, gicp.default_params(k_correspondences=5), ctx=gpu_ctx)
    assert (Tc == res.matrix()).all()
    assert int(conv) == int(res.converged) and int(iters) == res.iterations and int(nout) == len(src)
    assert float(score) == res.fitness
    o = oracle_mod.gicp_align(src, tgt, k=5)
    dt, dr = pose_err(Tc, o["T"])
    assert dt < 1e-5 and dr < 1e-5, (dt, dr)

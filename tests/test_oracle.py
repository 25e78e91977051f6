"""The C oracle (oracle/icp_oracle.c) against the golden fixtures and analytic known answers.

The oracle is the checker of the HIP product; these tests pin it before it is trusted (the
reference has no tests of its own: SURVEY.md §4, §8c).  CPU only.
"""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN_DIR, TOL_R, TOL_T, load_case_clouds, pose_err


def _digest(idx, d2):
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(idx, np.int32).tobytes())
    h.update(np.ascontiguousarray(d2, np.float32).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("which", [0, 1])
def test_nn_iteration0_matches_golden(oracle_mod, golden, which):
    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    for nn in (oracle_mod.NN_BRUTE, oracle_mod.NN_KDTREE):
        idx, d2 = oracle_mod.nearest(src, tgt, nn)
        assert _digest(idx, d2) == case["nn0_sha256"], f"nn mode {nn}"
        rows = np.array(case["nn0_rows"])
        assert (idx[rows] == np.array(case["nn0_idx_rows"])).all()
        assert (d2[rows] == np.array(case["nn0_d2_rows"], np.float32)).all()
        if "nn0_idx" in case:
            assert (idx == np.array(case["nn0_idx"])).all()


@pytest.mark.parametrize("which", [0, 1])
def test_icp_f64_matches_numpy_twin(oracle_mod, golden, which):
    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    r = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F64, max_iterations=case["max_iterations"], trace=True)
    assert r["status"] == 0
    assert r["iterations"] == case["iterations"]
    assert r["converged"] == case["converged"]
    assert r["convergence_state"] == case["convergence_state"]
    # same arithmetic up to double summation order: identical to ~float rounding
    for k, Tk in enumerate(case["T_final_trace"]):
        dt, dr = pose_err(r["trace"]["T_final"][k], Tk)
        assert dt < 2e-6 and dr < 2e-6, (k, dt, dr)
    np.testing.assert_allclose(r["trace"]["mu_src"][0], case["mu_src0"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(r["trace"]["mu_dst"][0], case["mu_dst0"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(r["trace"]["sigma"][0], case["sigma0"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(r["trace"]["mse"], case["mse_trace"], rtol=1e-9)
    assert abs(r["fitness"] - case["fitness"]) <= 1e-9 * max(1.0, case["fitness"])


@pytest.mark.parametrize("which", [0, 1])
def test_pcl_float_sigma_matches_numpy_twin(oracle_mod, golden, which):
    """The oracle's float Umeyama moments of the first iteration — sequential centroids and Eigen's
    depth-blocked sigma GEMM (13 panels of 632 at 8k, 4 of 520 at 2k) — equal an independent numpy
    restatement bit for bit.  Also the unblocked form (eigen_l1_bytes < 0: one chain of n)."""
    import sys
    sys.path.insert(0, GOLDEN_DIR)
    import numpy_twin as tw

    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    idx, _ = tw.nearest(src[:, :3], tgt[:, :3])
    n = len(src)
    assert tw.eigen_gemm_kc(n) == {2048: 520, 8192: 632}[n]
    for l1, kc in ((0, None), (-1, n)):
        r = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=1, trace=True,
                             eigen_l1_bytes=l1)
        sigma, ms, md = tw.umeyama_sigma_f32(src[:, :3], tgt[idx, :3], kc=kc)
        assert (r["trace"]["sigma"][0].astype(np.float32) == sigma).all(), l1
        assert (r["trace"]["mu_src"][0].astype(np.float32) == ms).all()
        assert (r["trace"]["mu_dst"][0].astype(np.float32) == md).all()


@pytest.mark.parametrize("which", [0, 1])
def test_pcl_float_icp_matches_numpy_twin(oracle_mod, golden, which):
    """The oracle's whole float registration equals an independent numpy restatement bit for bit at
    every iteration: sequential float centroids, Eigen's blocked sigma GEMM, Eigen 3.3's
    JacobiSVD<Matrix3f> and umeyama product order, the float transformCloud and composition, the
    convergence expressions in float, and the sequential double MSE / fitness sums."""
    import sys
    sys.path.insert(0, GOLDEN_DIR)
    import numpy_twin as tw

    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    it = case["max_iterations"]
    t = tw.icp(src, tgt, max_iterations=it, numerics="f32")
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=it, trace=True)
    assert o["iterations"] == t["iterations"] and o["convergence_state"] == t["state"]
    for k, tk in enumerate(t["trace"]):
        assert (o["trace"]["T_inc"][k] == tk["T_inc"]).all(), k
        assert (o["trace"]["T_final"][k] == tk["T_final"]).all(), k
        assert o["trace"]["mse"][k] == tk["mse"], k
    assert (o["T"] == t["T"]).all() and o["fitness"] == t["fitness"]


def _sigma_cases(rng, count):
    """3x3 float32 matrices of the shapes a registration meets and of the SVD's edge cases."""
    out = []
    for t in range(count):
        S = rng.normal(0, 100, (3, 3)).astype(np.float32)
        if t % 8 == 1:
            S[2] = S[1] * np.float32(0.5)  # rank 2
        elif t % 8 == 2:
            S = (np.eye(3) * 500 + 0.01 * S).astype(np.float32)  # near identity
        elif t % 8 == 3:
            a = rng.uniform(-0.2, 0.2)
            Rz = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
            S = (Rz @ np.diag([400.0, 90.0, 0.5 + t % 3]) + rng.normal(0, 0.01, (3, 3))).astype(np.float32)
        elif t % 8 == 4:
            S = (S * np.float32(2.0 ** rng.integers(-20, 20))).astype(np.float32)
        elif t % 8 == 5:
            S = np.diag(rng.normal(0, 5, 3)).astype(np.float32)  # diagonal, signs, order
        elif t % 8 == 6:
            S = np.outer(rng.normal(size=3), rng.normal(size=3)).astype(np.float32)  # rank 1
        elif t % 16 == 7:
            S = np.zeros((3, 3), np.float32)
        out.append(S)
    return out


def test_eigen_svd_rotation_matches_numpy_twin(oracle_mod):
    """PCL's float rotation (Eigen 3.3 JacobiSVD<Matrix3f> + umeyama): the C oracle and the numpy
    restatement agree bit for bit over registration-shaped and edge-case sigmas."""
    import sys
    sys.path.insert(0, GOLDEN_DIR)
    import numpy_twin as tw

    rng = np.random.default_rng(11)
    for k, S in enumerate(_sigma_cases(rng, 600)):
        Ro = oracle_mod.rot_f32(S)
        Rt = tw.umeyama_rotation_f32(S)
        assert (Ro.view(np.uint32) == Rt.view(np.uint32)).all(), (k, S, Ro, Rt)


def test_eigen_svd_known_answers():
    """JacobiSVD<Matrix3f> semantics on inputs with known decompositions: singular values
    descending, U S V^T reproduces the input, U and V orthonormal; a diagonal input keeps its
    axes (with U's column sign fixes); R of a rotated diagonal spread is that rotation."""
    import sys
    sys.path.insert(0, GOLDEN_DIR)
    import numpy_twin as tw

    U, S, V = tw.eigen_jacobi_svd3_f32(np.diag([2.0, -7.0, 3.0]).astype(np.float32))
    assert list(S) == [7.0, 3.0, 2.0]
    assert np.allclose(U @ np.diag(S) @ V.T, np.diag([2.0, -7.0, 3.0]), atol=1e-6)
    rng = np.random.default_rng(2)
    for _ in range(50):
        A = rng.normal(0, 10, (3, 3)).astype(np.float32)
        U, S, V = tw.eigen_jacobi_svd3_f32(A)
        assert S[0] >= S[1] >= S[2] >= 0
        assert np.allclose(U @ np.diag(S) @ V.T, A, atol=2e-5 * np.abs(A).max())
        assert np.allclose(U.T @ U, np.eye(3), atol=2e-6) and np.allclose(V.T @ V, np.eye(3), atol=2e-6)
    a = 0.1
    R0 = np.array([[np.cos(a), -np.sin(a), 0], [np.sin(a), np.cos(a), 0], [0, 0, 1]])
    R = tw.umeyama_rotation_f32((R0 @ np.diag([300.0, 80.0, 2.0])).astype(np.float32))
    assert np.abs(R - R0).max() < 1e-6


@pytest.mark.parametrize("which", [0, 1])
def test_icp_pcl_float_within_bar_of_f64(oracle_mod, golden, which):
    """PCL's float Umeyama vs the exact solve: the reference's own float noise (documented)."""
    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    a = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=case["max_iterations"])
    dt, dr = pose_err(a["T"], case["T"])
    assert dt < 3 * TOL_T and dr < TOL_R, (dt, dr)


def test_kdtree_equals_bruteforce_including_ties(oracle_mod):
    rng = np.random.default_rng(3)
    tgt = rng.uniform(-50, 50, (3000, 4)).astype(np.float32)
    tgt[1500:1600] = tgt[100:200]  # exact duplicates -> ties must resolve to the lowest index
    q = np.concatenate([rng.uniform(-60, 60, (2000, 4)).astype(np.float32), tgt[100:200]])
    i1, d1 = oracle_mod.nearest(q, tgt, oracle_mod.NN_BRUTE)
    i2, d2 = oracle_mod.nearest(q, tgt, oracle_mod.NN_KDTREE)
    assert (i1 == i2).all() and (d1 == d2).all()
    assert (i1[2000:] == np.arange(100, 200)).all()


@pytest.mark.parametrize("num", [0, 1])
def test_known_answers(oracle_mod, golden, num):
    for kat in golden["kat"]:
        src = np.array(kat["src"], np.float32)
        tgt = np.array(kat["tgt"], np.float32)
        r = oracle_mod.align(src, tgt, numerics=num, max_iterations=20)
        dt, dr = pose_err(r["T"], kat["T_expect"])
        assert dt < kat["tol_t"] and dr < kat["tol_r"], (kat["name"], dt, dr)


def test_error_paths(oracle_mod):
    rng = np.random.default_rng(5)
    c = rng.uniform(-5, 5, (100, 4)).astype(np.float32)
    # empty target: Registration::initCompute fails -> identity, not converged
    r = oracle_mod.align(c, np.zeros((0, 4), np.float32))
    assert r["status"] == -2 and not r["converged"] and np.allclose(r["T"], np.eye(4))
    # fewer than 3 correspondences
    r = oracle_mod.align(c[:2], c)
    assert r["status"] == -3 and not r["converged"] and r["convergence_state"] == 5
    # rejection by max correspondence distance -> too few
    far = c.copy()
    far[:, :3] += 1000
    r = oracle_mod.align(far, c, max_correspondence_distance=1.0)
    assert r["status"] == -3 and r["iterations"] == 0
    # non-finite input rejected up front
    bad = c.copy()
    bad[7, 1] = np.nan
    assert oracle_mod.align(bad, c)["status"] == -4


def test_convergence_criteria(oracle_mod, golden):
    case = golden["cases"][0]
    src, tgt = load_case_clouds(case)
    r = oracle_mod.align(src, tgt, max_iterations=1)
    assert r["iterations"] == 1 and r["converged"] and r["convergence_state"] == 1
    # max_iterations = 0: PCL's do/while still runs one iteration
    r = oracle_mod.align(src, tgt, max_iterations=0)
    assert r["iterations"] == 1 and r["converged"]
    # identical clouds (the node's order-0 frame): exact solve -> X unchanged -> |ΔMSE| = 0 < 1e-12
    # stops at iteration 2 with CONVERGENCE_CRITERIA_ABS_MSE.  The float solve's rounding instead
    # moves X by ~1e-7 per iteration (MSE 0 -> 4e-11 -> ...), so it runs to the cap; T stays I.
    r = oracle_mod.align(tgt, tgt, max_iterations=10, numerics=oracle_mod.NUM_F64)
    assert r["converged"] and r["iterations"] == 2 and r["convergence_state"] == 3
    r = oracle_mod.align(tgt, tgt, max_iterations=10, numerics=oracle_mod.NUM_F32)
    assert r["converged"] and np.abs(r["T"] - np.eye(4)).max() < 1e-5


def test_guess_applied(oracle_mod, golden):
    case = golden["cases"][0]
    src, tgt = load_case_clouds(case)
    G = np.array(case["T"], np.float32)
    r0 = oracle_mod.align(src, tgt, max_iterations=10)
    r1 = oracle_mod.align(src, tgt, guess=G, max_iterations=10)
    dt, dr = pose_err(r0["T"], r1["T"])
    assert dt < 5e-3 and dr < 5e-3


def test_sanitizer_build_runs():
    """The oracle under ASan/UBSan (host-only sanitizers) on a small pair."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    od = os.path.join(root, "oracle")
    r = subprocess.run(["make", "-s", "-C", od, "_build/oracle_asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([os.path.join(od, "_build", "oracle_asan")], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout

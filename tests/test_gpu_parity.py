"""Parity of the HIP product (through the C ABI) with the oracle — needs a real MI355X.

Bars (north_star): NN indices and d² bit-exact (integer/index work); per-pair transforms within
1e-4 m / 1e-4 rad of the reference-faithful oracle on identical inputs; batch, split and repeated
runs bit-identical to each other.
"""
import os
import subprocess

import numpy as np
import pytest

from helpers import GOLDEN_DIR, TOL_R, TOL_T, load_case_clouds, pose_err

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _pair(i, n, m=None):
    from icp4r import synth

    p = synth.make_pair(i, n, m)
    return p.src_xyzi(), p.tgt_xyzi()


# ---------------------------------------------------------------------------------------------- NN
@pytest.mark.parametrize("which", [0, 1])
def test_nn_bitexact_golden(gpu_ctx, oracle_mod, golden, which):
    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    gi, gd = gpu_ctx.nearest(src, tgt)
    oi, od = oracle_mod.nearest(src, tgt, oracle_mod.NN_BRUTE)
    assert (gi == oi).all() and (gd == od).all()
    rows = np.array(case["nn0_rows"])
    assert (gi[rows] == np.array(case["nn0_idx_rows"])).all()


@pytest.mark.parametrize("n,m", [(1, 1), (5, 3), (7, 1001), (1000, 4099), (4097, 8190), (3, 65540), (20000, 511),
                                 (9000, 70001)])
def test_nn_bitexact_shapes_and_ties(gpu_ctx, oracle_mod, n, m):
    rng = np.random.default_rng(n * 31 + m)
    tgt = rng.uniform(-80, 80, (m, 4)).astype(np.float32)
    if m > 10:
        tgt[m // 2: m // 2 + 5] = tgt[:5]  # duplicates: ties -> lowest index
    q = rng.uniform(-90, 90, (n, 4)).astype(np.float32)
    k = min(n, m, 5)
    q[:k] = tgt[:k]
    gi, gd = gpu_ctx.nearest(q, tgt)
    oi, od = oracle_mod.nearest(q, tgt, oracle_mod.NN_BRUTE)
    assert (gi == oi).all() and (gd == od).all()


def _lattice(rng, side, spacing=0.5):
    g = np.stack(np.meshgrid(*[np.arange(side, dtype=np.float32) * spacing] * 3, indexing="ij"), -1).reshape(-1, 3)
    g = g[rng.permutation(len(g))]  # lowest index is not the first visited in Morton order
    return np.concatenate([g, np.zeros((len(g), 1), np.float32)], 1)


@pytest.mark.parametrize("side", [9, 16])
def test_nn_lattice_ties_lowest_index(gpu_ctx, oracle_mod, side):
    """Integer lattices: most queries sit at exactly equal distance from 2, 4 or 8 targets (exact
    float ties) — the pruned search must still return the lowest target index."""
    rng = np.random.default_rng(side)
    tgt = _lattice(rng, side)
    q = tgt.copy()
    q[:, :3] += np.float32(0.25)  # equidistant from 8 lattice points in the interior
    q[::3, 0] += np.float32(-0.25)  # 4-way ties
    q[::5, 1] += np.float32(-0.25)  # 2-way ties
    gi, gd = gpu_ctx.nearest(q, tgt)
    oi, od = oracle_mod.nearest(q, tgt, oracle_mod.NN_BRUTE)
    assert (gd == od).all() and (gi == oi).all()


# ---------------------------------------------------------------------------------------------- ICP
@pytest.mark.parametrize("which", [0, 1])
def test_icp_pcl_numerics_vs_oracle(gpu_ctx, oracle_mod, golden, which):
    import icp4r

    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    it = case["max_iterations"]
    r, _ = gpu_ctx.align(src, tgt, icp4r.default_params(max_iterations=it))
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=it)
    assert r.status == 0 and r.iterations == o["iterations"] and bool(r.converged) == o["converged"]
    # PCL numerics are a bit-exact restatement of the float oracle: equal bits, not a tolerance
    assert (r.matrix() == o["T"]).all()
    assert r.fitness == o["fitness"]
    dt, dr = pose_err(r.matrix(), o["T"])
    assert dt <= TOL_T and dr <= TOL_R, (dt, dr)
    # and against the independent numpy twin's golden answer
    dt, dr = pose_err(r.matrix(), case["T"])
    assert dt <= 3 * TOL_T and dr <= TOL_R, (dt, dr)


@pytest.mark.parametrize("which", [0, 1])
def test_icp_f64_numerics_vs_oracle_f64(gpu_ctx, oracle_mod, golden, which):
    import icp4r

    case = golden["cases"][which]
    src, tgt = load_case_clouds(case)
    it = case["max_iterations"]
    r, _ = gpu_ctx.align(src, tgt, icp4r.default_params(max_iterations=it, numerics=icp4r.NUMERICS_F64))
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F64, max_iterations=it)
    assert r.iterations == o["iterations"] == case["iterations"]
    dt, dr = pose_err(r.matrix(), o["T"])
    assert dt <= 2e-6 and dr <= 2e-6, (dt, dr)
    dt, dr = pose_err(r.matrix(), case["T"])
    assert dt <= 2e-6 and dr <= 2e-6, (dt, dr)
    assert abs(r.fitness - case["fitness"]) <= 1e-6 * case["fitness"]


@pytest.mark.parametrize("i", range(6))
def test_icp_random_pairs_pcl_defaults(gpu_ctx, oracle_mod, i):
    """PCL defaults (10 iterations, |ΔMSE| early stop live) on assorted shapes."""
    import icp4r

    n = [2048, 8192, 1000, 3001, 513, 6000][i]
    m = [2048, 8192, 1500, 2999, 700, 8191][i]
    src, tgt = _pair(100 + i, n, m)
    r, out = gpu_ctx.align(src, tgt, icp4r.default_params(), want_aligned=True)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, aligned=True)
    assert r.iterations == o["iterations"] and bool(r.converged) == o["converged"]
    assert r.convergence_state == o["convergence_state"]
    assert (r.matrix() == o["T"]).all() and r.fitness == o["fitness"]
    assert (out == o["aligned"]).all()
    assert (out[:, 3] == src[:, 3]).all()


# The sigma GEMM's depth blocking (Eigen 3.3: panels of kc correspondences): one panel
# up to 680 correspondences, 2-13 panels at the benchmark sizes, more than one panel group (> 14
# panels) past ~9k, panel starts counted in accepted correspondences when some are rejected, Huber
# products, the unblocked form, and every plan (solo, multi-launch, batched).
@pytest.mark.parametrize("n,m,kw", [
    (681, 700, {}),                                          # 2 panels of 344 / 337
    (2048, 2048, {"max_iterations": 20}),                    # 4 panels (C1 shape)
    (8192, 8192, {"max_iterations": 20}),                    # 13 panels (C2 shape)
    (16384, 8192, {"max_iterations": 6}),                    # 25 panels: two panel groups
    (4096, 4096, {"max_correspondence_distance": 0.6}),      # rejected correspondences: ranked starts
    (20000, 6000, {"max_correspondence_distance": 0.5, "max_iterations": 5}),  # ... over two groups
    (3000, 3000, {"huber_delta": 0.4}),                      # Huber products, 5 panels
    (8192, 8192, {"eigen_l1_bytes": -1}),                    # unblocked: one chain of |C|
    (8192, 8192, {"eigen_l1_bytes": 49152, "eigen_gebp_mr": 16}),  # other host facts
])
@pytest.mark.parametrize("wide", [1, 0])
def test_sigma_panels_vs_oracle(gpu_ctx, oracle_mod, n, m, kw, wide, plan):
    """Both single-pair updates on the multi-launch plan (solo = 0): fold_update_wide_kernel (the
    panels side by side) and, with plan option wide_update = 0, fold_update_kernel's sequential pass B
    over correspondence records (test_sigma_panels_batch_and_solo covers solo_kernel)."""
    import icp4r

    plan(wide_update=wide, solo=0)
    pl = icp4r.plan(1, n, m, ctx=gpu_ctx)
    assert pl["wide_update"] == bool(wide) and not pl["solo"]
    src, tgt = _pair(700 + n % 97, n, m)
    r, out = gpu_ctx.align(src, tgt, icp4r.default_params(**kw), want_aligned=True)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, aligned=True, **kw)
    assert r.status == o["status"] == 0
    assert r.iterations == o["iterations"] and r.convergence_state == o["convergence_state"]
    assert r.n_correspondences == o["n_correspondences"]
    if "max_correspondence_distance" in kw:
        assert 0 < r.n_correspondences < n  # the ranked panel starts were exercised
    assert (r.matrix() == o["T"]).all() and r.fitness == o["fitness"]
    assert (out == o["aligned"]).all()


@pytest.mark.parametrize("solo,wide", [("0", 1), ("0", 0), ("1", 1)])
def test_sigma_panels_batch_and_solo(gpu_ctx, oracle_mod, solo, wide, plan):
    """Panels in the one-workgroup registration (solo_kernel, forced up to 16k sources) and in a
    batch of ragged pairs (either update kernel), against the oracle pair by pair."""
    import icp4r

    plan(solo=int(solo), wide_update=wide)
    shapes = [(1024, 1024), (2048, 1500), (700, 2048), (5000, 4000), (681, 681)]
    pairs = [_pair(800 + k, n, m) for k, (n, m) in enumerate(shapes)]
    p = icp4r.default_params(max_iterations=12)
    res = gpu_ctx.align_batch_host(*_batch(pairs), params=p)
    for k, (s, t) in enumerate(pairs):
        o = oracle_mod.align(s, t, numerics=oracle_mod.NUM_F32, max_iterations=12)
        T = np.array(res[k]["T"], np.float32).reshape(4, 4).T
        assert res[k]["iterations"] == o["iterations"], k
        assert (T == o["T"]).all(), k
        assert res[k]["fitness"] == o["fitness"], k


def test_device_eigen_svd_rotation_matches_oracle(gpu_ctx, oracle_mod):
    """The device's float Umeyama rotation (icp4r_math.hpp: Eigen 3.3 JacobiSVD<Matrix3f> + umeyama,
    the solve of every PCL-numerics update) equals the oracle's bit for bit, one thread per matrix."""
    import ctypes as C

    import icp4r
    from test_oracle import _sigma_cases

    S = np.stack(_sigma_cases(np.random.default_rng(11), 4096)).reshape(-1, 9).astype(np.float32)
    R = np.zeros_like(S)
    L = icp4r.load()
    assert L.icp4r__test_rot_f32(gpu_ctx.handle, C.c_void_p(S.ctypes.data), C.c_void_p(R.ctypes.data), len(S)) == 0
    Ro = np.stack([oracle_mod.rot_f32(s) for s in S]).reshape(-1, 9)
    bad = (R.view(np.uint32) != Ro.view(np.uint32)).any(1)
    assert not bad.any(), f"{int(bad.sum())} of {len(S)} rotations differ"


def test_known_answers(gpu_ctx, golden):
    import icp4r

    for kat in golden["kat"]:
        r, _ = gpu_ctx.align(np.array(kat["src"], np.float32), np.array(kat["tgt"], np.float32),
                             icp4r.default_params(max_iterations=20))
        dt, dr = pose_err(r.matrix(), kat["T_expect"])
        assert dt < kat["tol_t"] and dr < kat["tol_r"], (kat["name"], dt, dr)


# ---------------------------------------------------------------------------------------------- paths
def _batch(pairs):
    src = np.concatenate([p[0] for p in pairs]).astype(np.float32)
    tgt = np.concatenate([p[1] for p in pairs]).astype(np.float32)
    sn = np.array([len(p[0]) for p in pairs], np.int32)
    tn = np.array([len(p[1]) for p in pairs], np.int32)
    so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
    to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
    return src, so, sn, tgt, to, tn


def test_batch_equals_single_calls(gpu_ctx):
    import icp4r

    shapes = [(8192, 8192), (2048, 2048), (1000, 1200), (37, 4000), (4096, 64), (8000, 8100), (3, 3), (700, 650)]
    pairs = [_pair(200 + k, n, m) for k, (n, m) in enumerate(shapes)]
    p = icp4r.default_params(max_iterations=15)
    res = gpu_ctx.align_batch_host(*_batch(pairs), params=p)
    for k, (s, t) in enumerate(pairs):
        r, _ = gpu_ctx.align(s, t, p)
        assert (np.array(r.T, np.float32) == res[k]["T"]).all(), k
        assert r.iterations == res[k]["iterations"] and r.fitness == res[k]["fitness"]


def test_target_split_equals_unsplit(gpu_ctx):
    """Brute force: a single pair runs with the target split across workgroups (atomicMin merge of
    the keys); a 64-pair batch does not."""
    import icp4r

    s, t = _pair(300, 8192)
    assert icp4r.plan(1, 8192, 8192, icp4r.NN_BRUTE, ctx=gpu_ctx)["splits"] > 1
    assert icp4r.plan(64, 8192, 8192, icp4r.NN_BRUTE, ctx=gpu_ctx)["splits"] == 1
    p = icp4r.default_params(max_iterations=20, nn_mode=icp4r.NN_BRUTE)
    r, _ = gpu_ctx.align(s, t, p)
    res = gpu_ctx.align_batch_host(*_batch([(s, t)] * 64), params=p)
    for k in range(64):
        assert (res[k]["T"] == np.array(r.T, np.float32)).all()


@pytest.mark.parametrize("lds,cache,tile,solo", [("0", "1", "1", "1"), ("0", "1", "1", "0"), ("0", "1", "0", "0"),
                                                ("1", "0", "1", "1"), ("1", "1", "1", "1")])
@pytest.mark.parametrize("case", ["c2", "ragged", "far_guess", "lattice", "map", "dup_map", "big_src", "huge_src"])
def test_nn_modes_identical(gpu_ctx, case, lds, cache, tile, solo, plan):
    """Pruned (the whole registration per workgroup, LDS target tiles x query parts, the scalar-cache
    stream, or with the target set in LDS and per-query work lists, with or without the
    cached-neighbour test), brute-force and packed searches produce bit-identical registrations (T,
    fitness, iterations, aligned cloud) — the pruned index changes only which targets are evaluated.
    dup_map: every target twice, the copies in different tiles of a > 8192-point target, so ties
    resolve across tiles (lowest index).  big_src: a batch mixing sources of more than 8192 points
    (their own index) with ones ordered by the target's tree."""
    import icp4r

    plan(nn_lds=int(lds))  # 1: force nn_lds_kernel whenever the targets fit
    plan(nn_cache=int(cache))
    plan(nn_tile=int(tile))  # 0: the scalar-cache stream for the unbatched plan
    plan(solo=int(solo))  # 0: the multi-launch unbatched plan (solo_kernel off)
    guess = None
    if case == "c2":
        pairs = [_pair(310, 8192)]
    elif case == "ragged":
        shapes = [(8192, 8192), (2048, 600), (1000, 1200), (37, 4000), (4096, 64), (8000, 8100), (3, 700)]
        pairs = [_pair(320 + k, n, m) for k, (n, m) in enumerate(shapes)]
    elif case == "far_guess":  # iteration-0 seeds far from the answer
        pairs = [_pair(330, 4096)]
        g = np.eye(4, dtype=np.float32)
        g[:3, 3] = [7.0, -5.0, 1.0]
        c, sn = np.cos(0.4), np.sin(0.4)
        g[:2, :2] = [[c, -sn], [sn, c]]
        guess = g
    elif case == "lattice":
        rng = np.random.default_rng(7)
        t = _lattice(rng, 14)
        sr = t.copy()
        sr[:, :3] += np.float32(0.25)
        pairs = [(sr, t)]
    elif case == "map":
        from icp4r import synth

        mp = synth.make_map_pair(1)
        pairs = [(mp.src_xyzi()[:4096], mp.tgt_xyzi())]
    elif case == "big_src":  # sources beyond one kd build (own index, not the target's tree) beside small ones
        shapes = [(12000, 8000), (16384, 4096), (9000, 8192), (8192, 8192), (500, 300)]
        pairs = [_pair(350 + k, n, m) for k, (n, m) in enumerate(shapes)]
    elif case == "huge_src":  # sources past the batched search's 14-bit query records (tiled search)
        shapes = [(20000, 8000), (16385, 4096), (16384, 8192), (700, 300)]
        pairs = [_pair(360 + k, n, m) for k, (n, m) in enumerate(shapes)]
        assert not icp4r.plan(len(pairs), 20000, 8192, ctx=gpu_ctx)["lds"]
    else:
        sp, tp = _pair(340, 3000, 6000)
        pairs = [(sp, np.concatenate([tp, tp]))]
    p = dict(max_iterations=12, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    if len(pairs) == 1:
        s, t = pairs[0]
        out = {}
        for mode in (icp4r.NN_PRUNED, icp4r.NN_BRUTE, icp4r.NN_BRUTE_PACKED):
            r, al = gpu_ctx.align(s, t, icp4r.default_params(nn_mode=mode, **p), guess=guess, want_aligned=True)
            out[mode] = (bytes(r), al.tobytes())
        assert out[icp4r.NN_PRUNED] == out[icp4r.NN_BRUTE] == out[icp4r.NN_BRUTE_PACKED]
    else:
        res = {mode: gpu_ctx.align_batch_host(*_batch(pairs), params=icp4r.default_params(nn_mode=mode, **p))
               for mode in (icp4r.NN_PRUNED, icp4r.NN_BRUTE)}
        assert res[icp4r.NN_PRUNED].tobytes() == res[icp4r.NN_BRUTE].tobytes()


@pytest.mark.parametrize("numerics,huber", [(0, float("inf")), (1, float("inf")), (0, 0.5), (1, 0.5)])
def test_cached_neighbour_batch(gpu_ctx, oracle_mod, numerics, huber, plan):
    """The batched LDS search with the cached-neighbour test: bit-identical to the same search
    without it (every numerics / weighting), to the oracle (PCL numerics), and it resolves most
    queries of the late iterations without a search."""
    import icp4r

    npairs, n = 256, 8192
    pairs = [_pair(700 + k, n) for k in range(npairs)]
    args = _batch(pairs)
    assert icp4r.plan(npairs, n, n, ctx=gpu_ctx)["lds"] and icp4r.plan(npairs, n, n, ctx=gpu_ctx)["cache"]
    p = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0,
                             numerics=numerics, huber_delta=huber)
    plan(nn_cache=0, counters=1)  # (the work counters are opt-in diagnostics)
    gpu_ctx.reset_timers()
    plain = gpu_ctx.align_batch_host(*args, params=p)
    ev_plain, _ = gpu_ctx.nn_counters()
    plan(nn_cache=1)
    gpu_ctx.reset_timers()
    cached = gpu_ctx.align_batch_host(*args, params=p)
    ev_cached, _ = gpu_ctx.nn_counters()
    hits = gpu_ctx.nn_cache_hits()
    assert cached.tobytes() == plain.tobytes()
    assert (cached["status"] == 0).all() and (cached["iterations"] == 20).all()
    queries = npairs * n * 21  # 20 iterations + the fitness pass
    assert hits > 0.5 * queries, (hits, queries)
    assert ev_cached < ev_plain
    if numerics == 0:
        for k in (0, 131, 255):
            o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=20,
                                 mse_threshold_absolute=-1.0, transformation_epsilon=-1.0, huber_delta=huber)
            assert (cached[k]["T"].reshape(4, 4).T == o["T"]).all() and cached[k]["fitness"] == o["fitness"]


def test_tile_run_lengths_identical(gpu_ctx, plan):
    """nn_tile_kernel's queries per wave run (plan option tile_run 64 / 32 / 16 / 8: 1024 / 512 / 256 / 128 queries per
    workgroup, the single-pair plans' default picks the length whose grid covers the CUs), and the
    update's transform deferred into the one-tile search or not (tile_defer): bit-identical
    registrations, one target tile (C2's and C1's shapes) and several (a scan-to-map target), fixed
    iterations and PCL's defaults, aligned clouds included."""
    import icp4r

    cases = [_pair(41, 8192), _pair(42, 5000, 20000), _pair(43, 2048)]
    for params in (icp4r.default_params(max_iterations=12, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0),
                   icp4r.default_params()):
        for s, t in cases:
            out = {}
            # (tile_defer = 0: the update transforms the cloud itself instead of the next search)
            for run, defer in (("64", "1"), ("32", "1"), ("16", "1"), ("8", "1"), ("16", "0")):
                plan(tile_run=int(run))
                plan(tile_defer=int(defer))
                pl = icp4r.plan(1, len(s), len(t), ctx=gpu_ctx)
                assert pl["pruned"] and not pl["lds"] and not pl["solo"]
                r, al = gpu_ctx.align(s, t, params, want_aligned=True)
                out[run + defer] = (bytes(r), al.tobytes())
            assert out["641"] == out["321"] == out["161"] == out["81"] == out["160"]


@pytest.mark.parametrize("early", [False, True])
def test_fused_cache_test_identical(gpu_ctx, oracle_mod, early, plan):
    """The cached-neighbour test run in the tail of fold_update_kernel (default) instead of its own
    nn_cache_test_kernel launch: bit-identical batches, with fixed iterations and with PCL's early
    stops live (pairs converging at different iterations, so some skip the fused tail), over ragged
    shapes; the oracle on sampled pairs."""
    import icp4r

    shapes = [(8192, 8192)] * 200 + [(8000, 8100), (4096, 8192), (2048, 600), (1000, 1200), (37, 4000)] * 12
    pairs = [_pair(1300 + k, n, m) for k, (n, m) in enumerate(shapes)]
    args = _batch(pairs)
    assert icp4r.plan(len(pairs), 8192, 8192, ctx=gpu_ctx)["lds"] and icp4r.plan(len(pairs), 8192, 8192, ctx=gpu_ctx)["cache"]
    kw = {} if early else dict(mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    p = icp4r.default_params(max_iterations=20, **kw)
    out = {}
    # (fuse_order = 1, the default: the update's last workgroup also builds the next search's
    # work list from the words the other workgroups publish; 0: nn_order_kernel does)
    plan(counters=1)
    for fuse, order in (("0", "1"), ("1", "0"), ("1", "1")):
        plan(fuse_test=int(fuse))
        plan(fuse_order=int(order))
        gpu_ctx.reset_timers()
        out[fuse + order] = gpu_ctx.align_batch_host(*args, params=p)
        st = gpu_ctx.nn_stats()
        assert (st["tested_in_update"] > 0) == (fuse == "1")
    assert out["10"].tobytes() == out["01"].tobytes()
    assert out["11"].tobytes() == out["01"].tobytes()
    out["1"] = out["11"]
    assert (out["1"]["status"] == 0).all()
    if early:
        assert len(set(out["1"]["iterations"].tolist())) > 1  # pairs stop at different iterations
    for k in (0, 199, 203, 204):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=20, **kw)
        assert (out["1"][k]["T"].reshape(4, 4).T == o["T"]).all() and out["1"][k]["fitness"] == o["fitness"]
        assert out["1"][k]["iterations"] == o["iterations"]


@pytest.mark.parametrize("cache", [0, 1])
def test_batched_update_panels_with_rejections(gpu_ctx, oracle_mod, cache, plan):
    """fold_update_kernel, the batched plan's update (more pairs than CUs), with rejected
    correspondences: the sigma panels then start at ranked positions counted in accepted
    correspondences (fold_bounds).  cache = 0 takes the correspondence records (no cached-neighbour
    test, nothing fused); cache = 1 reads X and nn_t.  Sampled pairs bit-equal to the oracle, and
    every one of them really rejected some correspondences."""
    import icp4r

    plan(nn_cache=cache)
    shapes = [(2048, 2048)] * 290 + [(3000, 2500), (1400, 3000)] * 5
    pairs = [_pair(2500 + k, n, m) for k, (n, m) in enumerate(shapes)]
    pl = icp4r.plan(len(pairs), 3000, 3000, ctx=gpu_ctx)
    assert pl["lds"] and pl["cache"] == bool(cache) and not pl["wide_update"]
    kw = dict(max_iterations=10, max_correspondence_distance=0.45)
    res = gpu_ctx.align_batch_host(*_batch(pairs), params=icp4r.default_params(**kw))
    for k in (0, 7, 145, 289, 290, 291, 299):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, **kw)
        assert 0 < o["n_correspondences"] < len(pairs[k][0]), k
        assert res[k]["n_correspondences"] == o["n_correspondences"], k
        assert res[k]["iterations"] == o["iterations"], k
        assert (res[k]["T"].reshape(4, 4).T == o["T"]).all() and res[k]["fitness"] == o["fitness"], k


@pytest.mark.parametrize("kw", [{}, {"max_correspondence_distance": 1.0}, {"huber_delta": 0.5}])
def test_sums_tail_identical(gpu_ctx, oracle_mod, kw, plan):
    """The fused tail folding the next pass A's source centroid sums (plan option sums_tail, eligible
    registrations: every correspondence kept, unweighted, no MSE criterion; the other two
    parametrisations are ineligible and must take the normal pass A): bit-identical batches either
    way, and the oracle on sampled pairs."""
    import icp4r

    shapes = [(2048, 2048)] * 240 + [(3000, 2500), (700, 2048), (2048, 900)] * 8
    pairs = [_pair(1700 + k, n, m) for k, (n, m) in enumerate(shapes)]
    args = _batch(pairs)
    assert icp4r.plan(len(pairs), 3000, 2500, ctx=gpu_ctx)["lds"]
    fixed = dict(max_iterations=15, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0, **kw)
    p = icp4r.default_params(**fixed)
    out = {}
    for on in ("0", "1"):
        plan(sums_tail=int(on))
        out[on] = gpu_ctx.align_batch_host(*args, params=p)
    assert out["1"].tobytes() == out["0"].tobytes()
    for k in (0, 239, 240, 242):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, **fixed)
        assert (out["1"][k]["T"].reshape(4, 4).T == o["T"]).all() and out["1"][k]["fitness"] == o["fitness"]


@pytest.mark.parametrize("npairs", [1, 300])
def test_source_order_identical(gpu_ctx, npairs, plan):
    """Sources ordered by descending their target's kd tree (src_order_kernel; the batched plan's default) or by their
    own kd tree (plan option src_order = 0): the order and the first-pass seeds change, the registrations do
    not — bit-identical on the single-pair pruned kernel and the batched LDS search, ragged shapes,
    a lattice (ties) and targets over 8192 points (their sources keep the own-tree path)."""
    import icp4r

    rng = np.random.default_rng(5)
    lat = _lattice(rng, 13)
    ls = lat.copy()
    ls[:, :3] += np.float32(0.25)
    if npairs == 1:
        pairs = [_pair(1600, 8192)]
    else:
        shapes = [(8192, 8192)] * (npairs - 8) + [(8000, 8100), (4096, 8192), (2048, 600), (1000, 1200),
                                                   (37, 4000), (3, 700), (8192, 9000)]
        pairs = [_pair(1600 + k, n, m) for k, (n, m) in enumerate(shapes)] + [(ls, lat)]
    args = _batch(pairs)
    p = icp4r.default_params(max_iterations=15)
    out = {}
    for so in ("0", "1"):
        plan(src_order=int(so))
        out[so] = gpu_ctx.align_batch_host(*args, params=p)
    assert out["0"].tobytes() == out["1"].tobytes()
    assert (out["1"]["status"] == 0).all()


def test_work_item_parts_identical(gpu_ctx, oracle_mod, plan):
    """The batched search's work list cuts a heavy pair's misses into parts of at least `part`
    misses (round 6 default 2048): any part size — none, small, the default — gives bit-identical
    registrations, equal to the oracle."""
    import icp4r

    pairs = [_pair(2600 + k, 8192 if k % 7 == 0 else 2048) for k in range(260)]
    args = _batch(pairs)
    assert icp4r.plan(len(pairs), 8192, 8192, ctx=gpu_ctx)["lds"]
    p = icp4r.default_params(max_iterations=8)
    out = {}
    for part in (0, 256, 2048):
        plan(part=part)
        out[part] = gpu_ctx.align_batch_host(*args, params=p)
    assert out[0].tobytes() == out[256].tobytes() == out[2048].tobytes()
    for k in (0, 7, 259):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=8)
        assert (np.array(out[2048][k]["T"], np.float32).reshape(4, 4).T == o["T"]).all(), k


def test_stage_sel_identical(gpu_ctx, oracle_mod, plan):
    """Small ranked work items stage only the superblocks their queries can reach (plan option
    stage_sel: items of at most that many misses): off, tiny, the default and every item give
    bit-identical registrations and fitness, equal to the oracle — a superblock the search needed and
    the mask left out would be read as the previous item's targets."""
    import icp4r

    pairs = [_pair(2900 + k, 8192 if k % 5 == 0 else 4096) for k in range(300)]
    args = _batch(pairs)
    assert icp4r.plan(len(pairs), 8192, 8192, ctx=gpu_ctx)["lds"]
    p = icp4r.default_params(max_iterations=12)
    out = {}
    for sel in (0, 16, 128, 1 << 20):
        plan(stage_sel=sel)
        out[sel] = gpu_ctx.align_batch_host(*args, params=p)
    assert out[0].tobytes() == out[16].tobytes() == out[128].tobytes() == out[1 << 20].tobytes()
    for k in (0, 3, 299):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=12)
        assert (np.array(out[128][k]["T"], np.float32).reshape(4, 4).T == o["T"]).all(), k
        assert out[128][k]["fitness"] == o["fitness"], k


def test_pruned_evaluates_fewer_pairs(gpu_ctx, plan):
    """The evaluation counter: brute force evaluates exactly n*m per pass; pruning far fewer; and the
    counters are opt-in (zero without plan option counters = 1 or per-kernel timing)."""
    import icp4r

    s, t = _pair(340, 8192)
    p = dict(max_iterations=5, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0, compute_fitness=0)
    gpu_ctx.reset_timers()
    gpu_ctx.align(s, t, icp4r.default_params(nn_mode=icp4r.NN_PRUNED, **p))
    assert gpu_ctx.nn_counters() == (0, 0)
    plan(counters=1)
    gpu_ctx.reset_timers()
    gpu_ctx.align(s, t, icp4r.default_params(nn_mode=icp4r.NN_BRUTE, **p))
    brute, brute_tests = gpu_ctx.nn_counters()
    assert brute == 5 * len(s) * len(t) and brute_tests == 0
    gpu_ctx.reset_timers()
    gpu_ctx.align(s, t, icp4r.default_params(nn_mode=icp4r.NN_PRUNED, **p))
    pruned, tests = gpu_ctx.nn_counters()
    assert 0 < pruned < 0.3 * brute and tests > 0


def test_repeatable_and_target_permutation_invariant(gpu_ctx):
    import icp4r

    s, t = _pair(400, 8192)
    p = icp4r.default_params(max_iterations=20, mse_threshold_absolute=-1.0)
    a, _ = gpu_ctx.align(s, t, p)
    b, _ = gpu_ctx.align(s, t, p)
    assert bytes(a) == bytes(b)
    perm = np.random.default_rng(1).permutation(len(t))
    c, _ = gpu_ctx.align(s, t[perm], p)
    assert (np.array(a.T) == np.array(c.T)).all()  # same matched coordinates, same fold order


# ---------------------------------------------------------------------------------------------- edges
def test_error_and_option_paths(gpu_ctx, oracle_mod):
    import icp4r

    s, t = _pair(500, 2000)
    r, _ = gpu_ctx.align(s, np.zeros((0, 4), np.float32))
    assert r.status == icp4r.E_EMPTY and not r.converged and np.allclose(r.matrix(), np.eye(4))
    r, _ = gpu_ctx.align(s[:2], t)
    assert r.status == icp4r.E_TOO_FEW_CORR and not r.converged and r.convergence_state == 5
    bad = s.copy()
    bad[3, 2] = np.inf
    r, _ = gpu_ctx.align(bad, t)
    assert r.status == icp4r.E_NONFINITE
    # correspondence rejection, max_iterations 0/1, guess, Huber (F64 vs oracle F64)
    for kw in ({"max_correspondence_distance": 1.0}, {"max_iterations": 0}, {"max_iterations": 1},
               {"transformation_epsilon": 1e-8}, {"euclidean_fitness_epsilon": 1e-3}):
        r, _ = gpu_ctx.align(s, t, icp4r.default_params(**kw))
        o = oracle_mod.align(s, t, numerics=oracle_mod.NUM_F32, **kw)
        assert r.iterations == o["iterations"] and r.convergence_state == o["convergence_state"], kw
        assert r.n_correspondences == o["n_correspondences"], kw
        assert (r.matrix() == o["T"]).all() and r.fitness == o["fitness"], kw
    G = np.eye(4, dtype=np.float32)
    G[:3, 3] = [0.3, -0.2, 0.05]
    r, _ = gpu_ctx.align(s, t, icp4r.default_params(), guess=G)
    o = oracle_mod.align(s, t, guess=G, numerics=oracle_mod.NUM_F32)
    assert r.iterations == o["iterations"] and (r.matrix() == o["T"]).all()
    # Huber weighting (build extension; parity unpinned vs the reference, pinned vs the oracle)
    r, _ = gpu_ctx.align(s, t, icp4r.default_params(huber_delta=0.5, numerics=icp4r.NUMERICS_PCL))
    o = oracle_mod.align(s, t, huber_delta=0.5, numerics=oracle_mod.NUM_F32)
    assert (r.matrix() == o["T"]).all() and r.iterations == o["iterations"]
    r, _ = gpu_ctx.align(s, t, icp4r.default_params(huber_delta=0.5, numerics=icp4r.NUMERICS_F64))
    o = oracle_mod.align(s, t, huber_delta=0.5, numerics=oracle_mod.NUM_F64)
    dt, dr = pose_err(r.matrix(), o["T"])
    assert dt <= 2e-6 and dr <= 2e-6, (dt, dr)


def test_fitness_entry_point(gpu_ctx, oracle_mod):
    s, t = _pair(600, 3000)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = [0.1, 0.2, -0.1]
    for mr in (np.finfo(np.float64).max, 0.5):
        g = gpu_ctx.fitness(s, t, T, mr)
        o = oracle_mod.fitness(s, t, T, mr)
        assert g == o


# ---------------------------------------------------------------------------------------------- facade
@pytest.mark.parametrize("exe_name", ["callsite", "pcl18_callsite"])
def test_pcl_facade_callsite(oracle_mod, golden, exe_name):
    """The node's call sequence compiled against pcl_compat.hpp, on the golden C1 scans — with the
    facade's stand-in types, and against the PCL-1.8-shaped include tree (boost::shared_ptr clouds)."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    case = golden["cases"][0]
    exe = os.path.join(ROOT, "tests", "cpp", "_build", exe_name)
    out = subprocess.run([exe, os.path.join(GOLDEN_DIR, case["src_bin"]), os.path.join(GOLDEN_DIR, case["tgt_bin"])],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    lines = {l.split()[0]: l for l in out.stdout.splitlines() if l.split()}
    kv = dict(tok.split("=") for tok in lines["RESULT"].split()[1:])
    T = np.array([float(v) for v in lines["T"].split()[1:]]).reshape(4, 4)
    src, tgt = load_case_clouds(case)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32)
    assert int(kv["converged"]) == 1 and int(kv["iterations"]) == o["iterations"] == 10
    assert int(kv["points"]) == len(src)
    assert (T.astype(np.float32) == o["T"]).all()  # printed with %.9g: float32 round-trips exactly
    assert float(kv["score"]) == o["fitness"]


@pytest.mark.parametrize("solo", ["1", "0"])
def test_kernel_timing_api(gpu_ctx, solo, plan):
    """The NN kernel timer counts one launch per NN pass (5 iterations + the fitness pass) on the
    multi-launch plan, and the one solo_kernel launch of the whole registration on the solo plan."""
    import icp4r

    plan(solo=int(solo))
    s, t = _pair(700, 2048)
    p = icp4r.default_params(max_iterations=5, mse_threshold_absolute=-1)
    gpu_ctx.reset_timers()  # per-kernel timing off (the default): only the whole call is timed
    gpu_ctx.align(s, t, p)
    assert gpu_ctx.kernel_time_ms()[1] == 0 and gpu_ctx.batch_time_ms()[1] == 1
    gpu_ctx.set_kernel_timing(True)
    try:
        gpu_ctx.reset_timers()
        gpu_ctx.align(s, t, p)
        ms, k = gpu_ctx.kernel_time_ms()
        bms, bk = gpu_ctx.batch_time_ms()
    finally:
        gpu_ctx.set_kernel_timing(False)
    assert k == (1 if solo == "1" else 6) and ms > 0 and bk == 1 and bms >= ms


def _brute_nn(q, t):
    """Exact 1-NN with FLANN's L2_Simple float order, lowest index on ties (numpy)."""
    q = q[:, :3].astype(np.float32)
    t = t[:, :3].astype(np.float32)
    idx = np.empty(len(q), np.int32)
    d2o = np.empty(len(q), np.float32)
    for s in range(0, len(q), 256):
        d = q[s:s + 256, None, :] - t[None, :, :]
        d2 = (d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1]) + d[..., 2] * d[..., 2]
        i = np.argmin(d2, axis=1)  # first minimum = lowest index
        idx[s:s + 256] = i
        d2o[s:s + 256] = d2[np.arange(len(i)), i]
    return idx, d2o


@pytest.mark.parametrize("shape", ["identical", "collinear", "duplicates", "lattice", "slab", "clustered"])
@pytest.mark.parametrize("m", [512, 513, 1000, 4097, 8191, 8192])
def test_kd_index_degenerate_clouds(gpu_ctx, shape, m):
    """The kd-tree index (index_kernel, clouds <= 8192 points) on degenerate targets: every point the
    same, all on a line, many exact duplicates, an integer lattice (ties everywhere), a flat slab, tight
    clusters — the pruned search over it returns brute force's keys exactly (lowest index on ties)."""
    rng = np.random.default_rng(m * 7 + len(shape))
    if shape == "identical":
        t = np.tile(np.array([[3.0, -2.0, 1.0]], np.float32), (m, 1))
    elif shape == "collinear":
        t = np.outer(rng.uniform(-50, 50, m), [0.6, 0.8, 0.0]).astype(np.float32)
    elif shape == "duplicates":
        base = rng.uniform(-20, 20, (max(m // 8, 1), 3)).astype(np.float32)
        t = base[rng.integers(0, len(base), m)]
    elif shape == "lattice":
        g = np.stack(np.meshgrid(np.arange(16), np.arange(16), np.arange(40)), -1).reshape(-1, 3)
        t = g[rng.permutation(len(g))[:m]].astype(np.float32)
    elif shape == "slab":
        t = np.concatenate([rng.uniform(-60, 60, (m, 2)), np.zeros((m, 1))], 1).astype(np.float32)
    else:
        c = rng.uniform(-40, 40, (5, 3))
        t = (c[rng.integers(0, 5, m)] + rng.normal(0, 0.01, (m, 3))).astype(np.float32)
    tgt = np.concatenate([t, np.zeros((m, 1), np.float32)], 1)
    q = (t[rng.integers(0, m, 700)] + rng.normal(0, 0.5, (700, 3))).astype(np.float32)
    q = np.concatenate([q, t[:50]])  # exact hits
    src = np.concatenate([q, np.zeros((len(q), 1), np.float32)], 1)
    gi, gd = gpu_ctx.nearest(src, tgt)
    bi, bd = _brute_nn(src, tgt)
    assert (gd.view(np.uint32) == bd.view(np.uint32)).all()
    assert (gi == bi).all()


def test_c3_full_size_bench_workload(gpu_ctx, oracle_mod, plan):
    """BASELINE.json configs[2] at its own size, exactly as bench.py runs it: 1024 pairs of 8192/8192
    points (pair i seeded 1000 + i), 20 fixed iterations + the fitness pass, device-resident, the
    default plan (two pair groups on two streams, cached-neighbour test fused into the update).
    All 1024 result rows must be bit-identical to the same batch on one group without the
    cached-neighbour test, and 16 pairs spread over both groups bit-equal to the oracle."""
    import torch

    import icp4r

    P, n, iters = 1024, 8192, 20
    src_h = np.empty((P, n, 4), np.float32)
    tgt_h = np.empty((P, n, 4), np.float32)
    for k in range(P):
        src_h[k], tgt_h[k] = _pair(1000 + k, n)
    dev = torch.device("cuda", 0)
    src = torch.from_numpy(src_h.reshape(-1, 4)).to(dev)
    tgt = torch.from_numpy(tgt_h.reshape(-1, 4)).to(dev)
    off = torch.arange(P, dtype=torch.int64, device=dev) * n
    cnt = torch.full((P,), n, dtype=torch.int32, device=dev)
    batch = icp4r.Batch(src=src.data_ptr(), tgt=tgt.data_ptr(), src_off=off.data_ptr(), src_n=cnt.data_ptr(),
                        tgt_off=off.data_ptr(), tgt_n=cnt.data_ptr(), guess=None, aligned=None, npairs=P,
                        max_src_n=n, max_tgt_n=n)
    params = icp4r.default_params(max_iterations=iters, mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    pl = icp4r.plan(P, n, n, ctx=gpu_ctx)
    assert pl["lds"] and pl["cache"]
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run():
        out = torch.zeros((P, 96), dtype=torch.uint8, device=dev)
        gpu_ctx.align_batch_device(batch, params, out.data_ptr(), stream)
        torch.cuda.synchronize(dev)
        return np.frombuffer(out.cpu().numpy().tobytes(), dtype=icp4r.RESULT_DTYPE)

    gpu_ctx.reset_plan_options()
    default = run()
    assert (default["status"] == 0).all() and (default["iterations"] == iters).all()
    plan(groups=1, nn_cache=0)
    plain = run()
    assert default.tobytes() == plain.tobytes()
    picks = [0, 1, 100, 255, 384, 510, 511, 512, 513, 640, 777, 900, 1000, 1021, 1022, 1023]
    for k in picks:
        o = oracle_mod.align(src_h[k], tgt_h[k], numerics=oracle_mod.NUM_F32, max_iterations=iters,
                             mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
        assert (default[k]["T"].reshape(4, 4).T == o["T"]).all(), k
        assert default[k]["fitness"] == o["fitness"], k


@pytest.mark.parametrize("fixed", [True, False])
def test_c5_full_size_scan_to_map(gpu_ctx, oracle_mod, fixed):
    """BASELINE.json configs[4] at its own size (the scan-to-map registration of
    /root/reference/src/radar_odometry.cpp:386-411): an 8,192-point scan against a 65,540-point map
    (10 accumulated scans, synth.make_map_pair(0)), 20 iterations (fixed as the bench runs it, and
    with PCL's early stops live) plus the fitness pass, through icp4r_align — the tiled search over
    9 target tiles.  T, fitness, iteration count, convergence state and the aligned cloud bit-equal
    to the oracle."""
    import icp4r
    from icp4r import synth

    mp = synth.make_map_pair(0)
    src, tgt = mp.src_xyzi(), mp.tgt_xyzi()
    assert (len(src), len(tgt)) == (8192, 65540)
    pl = icp4r.plan(1, len(src), len(tgt), ctx=gpu_ctx)
    assert pl["pruned"] and not pl["lds"]
    kw = dict(mse_threshold_absolute=-1.0, transformation_epsilon=-1.0) if fixed else {}
    r, al = gpu_ctx.align(src, tgt, icp4r.default_params(max_iterations=20, **kw), want_aligned=True)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=20, aligned=True, **kw)
    assert r.status == 0 and r.iterations == o["iterations"]
    if fixed:
        assert r.iterations == 20
    assert r.convergence_state == o["convergence_state"] and bool(r.converged) == o["converged"]
    assert (r.matrix() == o["T"]).all()
    assert r.fitness == o["fitness"]
    assert r.n_correspondences == o["n_correspondences"]
    assert (al[:, :3].view(np.uint32) == o["aligned"][:, :3].view(np.uint32)).all()


@pytest.mark.parametrize("huber", [False, True])
def test_fold_keys_identical(gpu_ctx, oracle_mod, huber, plan):
    """The multi-tile single pair (targets over one 8192-point tile: the scan-to-map call) with the
    wide update forming the correspondence records in its pass A from X and the merged keys (plan
    option fold_keys = 1, the default) or corr_kernel writing them after every search (fold_keys = 0):
    bit-identical registrations (T, fitness, iterations, correspondences, the aligned cloud), PCL's
    early stops live, unweighted and Huber-weighted, and bit-equal to the oracle."""
    import icp4r

    src, tgt = _pair(2300, 4096, 30001)
    pl = icp4r.plan(1, len(src), len(tgt), ctx=gpu_ctx)
    assert pl["pruned"] and not pl["lds"] and pl["wide_update"]
    kw = dict(huber_delta=0.5) if huber else {}
    p = icp4r.default_params(max_iterations=12, **kw)
    out = {}
    for fk in (0, 1):
        plan(fold_keys=fk)
        r, al = gpu_ctx.align(src, tgt, p, want_aligned=True)
        out[fk] = (r.matrix().copy(), r.fitness, r.iterations, r.n_correspondences, r.status, al.copy())
    a, b = out[0], out[1]
    assert (a[0] == b[0]).all() and a[1:5] == b[1:5]
    assert (a[5].view(np.uint32) == b[5].view(np.uint32)).all()
    assert b[4] == 0
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=12, **kw)
    assert (b[0] == o["T"]).all() and b[2] == o["iterations"] and b[1] == o["fitness"]


@pytest.mark.parametrize("npairs", [1, 5, 40])
def test_morton_multi_workgroup_identical(gpu_ctx, oracle_mod, npairs, plan):
    """Targets too large for the in-LDS kd build (the C5 submap class): their Morton sort on one
    workgroup per 8192-point chunk (index_mo_hist_kernel / index_mo_scatter_kernel, the default for
    few pairs) or on one workgroup per target (plan option morton_mwg = 0) — the order changes, the
    registrations do not: bit-identical, ragged targets (8193 .. 40000 points, a partial last chunk,
    a lattice with ties, a small target in the same batch), and bit-equal to the oracle."""
    import icp4r

    rng = np.random.default_rng(11)
    if npairs == 1:
        pairs = [_pair(2100, 4096, 30001)]
    elif npairs == 40:  # a larger batch: 40 pairs x 3 chunk rows of histograms and 40 cell tables
        pairs = [_pair(2200 + k, 1024 + 97 * k, 8193 + 311 * k) for k in range(npairs)]
    else:
        lat = _lattice(rng, 22)  # 22^3 = 10648 points: ties everywhere
        ls = lat[rng.permutation(len(lat))[:3000]].copy()
        ls[:, :3] += np.float32(0.25)
        pairs = [_pair(2100 + k, n, m) for k, (n, m) in enumerate([(4096, 8193), (1000, 40000), (2048, 600),
                                                                     (8192, 16384)])] + [(ls, lat)]
    args = _batch(pairs)
    p = icp4r.default_params(max_iterations=12)
    out = {}
    for mwg in ("0", "1"):
        plan(morton_mwg=int(mwg))
        out[mwg] = gpu_ctx.align_batch_host(*args, params=p)
    assert out["0"].tobytes() == out["1"].tobytes()
    assert (out["1"]["status"] == 0).all()
    for k in (0, len(pairs) - 1):
        s, t = pairs[k]
        o = oracle_mod.align(s, t, numerics=oracle_mod.NUM_F32, max_iterations=12)
        T = out["1"]["T"][k].reshape(4, 4).T
        assert (T == o["T"]).all()
        assert out["1"]["iterations"][k] == o["iterations"]


def test_fitness_exact_and_sequential_forms(gpu_ctx, oracle_mod):
    """finish_kernel's fitness sum: the exact integer form (terms within 53 bits of the total) and the
    sequential fold it falls back to (a term whose last bit lies more than 53 bits below the total: a
    point 1e-15 off its target, d² = 1e-30), an all-zero sum (the source on the target), a single
    point, far points beyond max_range, and a source over 8192 points (keys re-read, not in registers) — every case bit-equal to the oracle's sequential loop."""
    s, t = _pair(601, 4096)
    T = np.eye(4, dtype=np.float32)
    T[:3, 3] = [0.05, -0.02, 0.01]
    tiny_t = t.copy()
    tiny_t[7, :3] = [1e-15, 0.0, 0.0]
    tiny_s = s.copy()
    tiny_s[3, :3] = [0.0, 0.0, 0.0]
    wide = s.copy()
    wide[::97, :3] *= np.float32(1000.0)  # a few distant points: large terms beside the small ones
    bs, bt = _pair(602, 9000, 3000)  # over 8192 sources: the keys re-read per pass, not held in registers
    cases = [(s, t, T), (tiny_s, tiny_t, np.eye(4, dtype=np.float32)), (t.copy(), t, np.eye(4, dtype=np.float32)),
             (s[:1].copy(), t, T), (wide, t, T), (bs, bt, T)]
    for k, (cs, ct, cT) in enumerate(cases):
        for mr in (np.finfo(np.float64).max, 0.5, 1e-3):
            g = gpu_ctx.fitness(cs, ct, cT, mr)
            o = oracle_mod.fitness(cs, ct, cT, mr)
            assert g == o, (k, mr, g, o)


@pytest.mark.parametrize("n", [700, 2048, 8192])
@pytest.mark.parametrize("tiny", [False, True])
def test_mse_exact_and_sequential_forms(gpu_ctx, oracle_mod, n, tiny):
    """Pass A's MSE sum under PCL's default criteria (live): its exact parallel form, and the sequential
    chain it falls back to when the terms span more than 53 bits (tiny: a source point 1e-15 off a
    target, d² = 1e-30 in the first iteration) — single pairs (solo_kernel at 700 sources, the
    multi-launch update above) and a batch; T, iterations, convergence state and fitness bit-equal
    to the oracle."""
    import icp4r

    s, t = _pair(610 + n, n)
    if tiny:
        t = t.copy()
        s = s.copy()
        t[5, :3] = [1e-15, 0.0, 0.0]
        s[9, :3] = [0.0, 0.0, 0.0]
    p = icp4r.default_params()
    o = oracle_mod.align(s, t, numerics=oracle_mod.NUM_F32)
    r, _ = gpu_ctx.align(s, t, p)
    assert r.status == 0 and r.iterations == o["iterations"]
    assert r.convergence_state == o["convergence_state"]
    assert (r.matrix() == o["T"]).all()
    assert r.fitness == o["fitness"]
    res = gpu_ctx.align_batch_host(*_batch([(s, t), _pair(620, 3000)]), params=p)
    assert (res[0]["T"] == np.array(r.T, np.float32)).all() and res[0]["iterations"] == r.iterations

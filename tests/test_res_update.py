"""fold_update_res_kernel (round 6): the batched update with each pair held on chip (registers + LDS)
across pass A, pass B and the fused cached-neighbour test — needs a real MI355X.

Every registration must be bit-identical to the streaming fold_update_kernel (plan option
res_update = 0) and, on sampled pairs, to the oracle: ragged sources (whole and partial 256-point
columns, a handful of points), PCL's early stops live (pairs converging at different iterations,
the MSE sum's exact form), fixed iterations, the MSE sum's sequential fallback (terms spanning more
than 53 bits), and the parametrisations the kernel leaves to fold_update_kernel (Huber, a distance
threshold).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(i, n, m=None):
    from icp4r import synth

    p = synth.make_pair(i, n, m)
    return p.src_xyzi(), p.tgt_xyzi()


def _batch(pairs):
    src = np.concatenate([p[0] for p in pairs]).astype(np.float32)
    tgt = np.concatenate([p[1] for p in pairs]).astype(np.float32)
    sn = np.array([len(p[0]) for p in pairs], np.int32)
    tn = np.array([len(p[1]) for p in pairs], np.int32)
    so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
    to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
    return src, so, sn, tgt, to, tn


def _run_both(gpu_ctx, plan, args, params):
    out = {}
    plan(counters=1)
    for on in (0, 1):
        plan(res_update=on)
        gpu_ctx.reset_timers()
        out[on] = gpu_ctx.align_batch_host(*args, params=params)
        st = gpu_ctx.nn_stats()
        out[f"st{on}"] = st
    plan(res_update=1)
    return out


@pytest.mark.parametrize("early", [False, True])
def test_res_update_identical(gpu_ctx, oracle_mod, early, plan):
    """Ragged batch (8192, 8191, 8000, 4097, 4096, 2048, 1000, 300, 256, 37, 5 sources): the on-chip
    update equals the streaming one bit for bit — results, and the cached-neighbour test's tested
    counts (its hits within 1 %: L is held rounded down) — and sampled pairs equal the oracle."""
    import icp4r

    shapes = [(8192, 8192)] * 200 + [(8191, 8000), (8000, 8100), (4097, 5000), (4096, 8192), (2048, 600),
                                     (1000, 1200), (300, 4000), (256, 256), (37, 4000), (5, 300)] * 8
    pairs = [_pair(3100 + k, n, m) for k, (n, m) in enumerate(shapes)]
    args = _batch(pairs)
    plan(res_update=1)
    assert icp4r.plan(len(pairs), 8192, 8192, ctx=gpu_ctx)["res_update"]
    kw = {} if early else dict(mse_threshold_absolute=-1.0, transformation_epsilon=-1.0)
    p = icp4r.default_params(max_iterations=20, **kw)
    out = _run_both(gpu_ctx, plan, args, p)
    assert out[1].tobytes() == out[0].tobytes()
    # (the on-chip kernel holds L rounded down to half precision: a few more misses, searched exactly —
    # the same queries tested, within 1 % of the hits)
    for key in ("cache_tested", "tested_in_update"):
        assert out["st1"][key] == out["st0"][key], key
    for key in ("cache_hits", "hits_in_update"):
        assert abs(out["st1"][key] - out["st0"][key]) <= 0.01 * out["st0"][key], key
    assert out["st1"]["tested_in_update"] > 0
    res = out[1]
    assert (res["status"] == 0).all()
    if early:
        assert len(set(res["iterations"].tolist())) > 1
    for k in (0, 199, 200, 201, 202, 203, 205, 206, 207, 208, 209, 279):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=20, **kw)
        assert (res[k]["T"].reshape(4, 4).T == o["T"]).all(), k
        assert res[k]["fitness"] == o["fitness"], k
        assert res[k]["iterations"] == o["iterations"], k
        assert res[k]["n_correspondences"] == o["n_correspondences"], k


def test_res_update_mse_sequential_fallback(gpu_ctx, oracle_mod, plan):
    """PCL's default criteria with a pair whose MSE terms span more than 53 bits (a source point 1e-15
    off a target: d² = 1e-30 next to ~1 m² terms) — the kernel's exact per-thread MSE sums saturate
    and it runs PCL's sequential double chain over the re-read points instead; bit-identical to the
    streaming update and the oracle."""
    import icp4r

    pairs = [_pair(3400 + k, 8192) for k in range(260)]
    s, t = pairs[3]
    s, t = s.copy(), t.copy()
    t[5, :3] = [1e-15, 0.0, 0.0]
    s[9, :3] = [0.0, 0.0, 0.0]
    pairs[3] = (s, t)
    p = icp4r.default_params(max_iterations=12)
    out = _run_both(gpu_ctx, plan, _batch(pairs), p)
    assert out[1].tobytes() == out[0].tobytes()
    for k in (3, 4):
        o = oracle_mod.align(*pairs[k], numerics=oracle_mod.NUM_F32, max_iterations=12)
        assert (out[1][k]["T"].reshape(4, 4).T == o["T"]).all(), k
        assert out[1][k]["iterations"] == o["iterations"], k
        assert out[1][k]["fitness"] == o["fitness"], k


@pytest.mark.parametrize("kw", [{"huber_delta": 0.5}, {"max_correspondence_distance": 0.5}])
def test_res_update_ineligible_parametrisations(gpu_ctx, oracle_mod, kw, plan):
    """Huber weights and a distance threshold stay on fold_update_kernel (the on-chip kernel keeps
    every correspondence unweighted): the option changes nothing."""
    import icp4r

    pairs = [_pair(3600 + k, 2048) for k in range(260)]
    p = icp4r.default_params(max_iterations=10, **kw)
    out = _run_both(gpu_ctx, plan, _batch(pairs), p)
    assert out[1].tobytes() == out[0].tobytes()
    o = oracle_mod.align(*pairs[7], numerics=oracle_mod.NUM_F32, max_iterations=10, **kw)
    assert (out[1][7]["T"].reshape(4, 4).T == o["T"]).all()

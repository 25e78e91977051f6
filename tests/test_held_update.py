"""fold_update_held_kernel (round 6): the wide update with the correspondence records held in the
fillers' registers from pass A to pass B (sources of at most 8960 points: 3 records per filler up to
2112 — the node's C1 scan; 11 filler waves, the fold wave alone on its SIMD — and 10 for the 8k scans
of C2 / C5) — needs a real MI355X.

Every registration must be bit-identical to fold_update_wide_kernel (plan option held_update = 0)
and to the oracle: sources across the 896-point slot boundaries (a handful of points, one slot, a
partial second slot, C1's 2048, both forms' maxima and one past each), PCL's early stops live (the MSE
sum's exact form and its sequential fallback), and the forms whose pass B takes the wide kernel's
global path (a distance threshold: panels by rank; Huber weights) or whose records come from the
merged keys (the multi-tile target, plan option fold_keys).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pair(i, n, m=None):
    from icp4r import synth

    p = synth.make_pair(i, n, m)
    return p.src_xyzi(), p.tgt_xyzi()


def _both(gpu_ctx, plan, src, tgt, p):
    out = {}
    for held in (0, 1):
        plan(held_update=held)
        r, al = gpu_ctx.align(src, tgt, p, want_aligned=True)
        out[held] = (r.matrix().copy(), r.fitness, r.iterations, r.n_correspondences, r.status,
                     r.convergence_state, al.view(np.uint32).copy())
    a, b = out[0], out[1]
    assert (a[0] == b[0]).all() and a[1:6] == b[1:6]
    assert (a[6] == b[6]).all()
    return b


@pytest.mark.parametrize("n,m,kw", [
    (5, 300, {}),
    (700, 2048, {}),                                      # one slot, one panel (global pass B)
    (896, 896, {"max_iterations": 20}),                   # exactly one slot, 2 panels
    (1000, 1200, {}),                                     # a partial second slot
    (2048, 2048, {}),                                     # C1: PCL defaults, 4 panels
    (2048, 2048, {"max_iterations": 20, "mse_threshold_absolute": -1.0, "transformation_epsilon": -1.0}),
    (2112, 3000, {"max_iterations": 15}),                 # the largest 3-record source (11 filler waves)
    (2113, 3000, {"max_iterations": 8}),                  # one past it: the 10-record form
    (8192, 8192, {"max_iterations": 20}),                 # C2: 13 panels
    (8192, 8192, {}),                                     # PCL defaults (MSE live) at 8k
    (8960, 9000, {"max_iterations": 6}),                  # the largest held source: 15 panels, pass B's global path
    (8961, 9000, {"max_iterations": 6}),                  # one past it: the wide kernel
    (6000, 7000, {"eigen_l1_bytes": 49152, "eigen_gebp_mr": 16}),  # other panel widths
    (2048, 2048, {"eigen_l1_bytes": 1024, "max_iterations": 5}),  # narrow panels: more than one group (global path)
    (8192, 8192, {"eigen_l1_bytes": 2048, "max_iterations": 4}),
    (2048, 2048, {"max_correspondence_distance": 0.6}),   # rejections: pass B's global ranked path
    (2400, 2048, {"huber_delta": 0.4}),                   # Huber: the same
])
def test_held_update_identical(gpu_ctx, oracle_mod, plan, n, m, kw):
    import icp4r

    plan(solo=0)
    pl = icp4r.plan(1, n, m, ctx=gpu_ctx)
    assert pl["wide_update"] and pl["held_update"] == (n <= 8960)
    src, tgt = _pair(4100 + n % 89, n, m)
    p = icp4r.default_params(**kw)
    b = _both(gpu_ctx, plan, src, tgt, p)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, aligned=True, **kw)
    assert b[4] == o["status"] == 0
    assert (b[0] == o["T"]).all() and b[1] == o["fitness"] and b[2] == o["iterations"]
    assert b[3] == o["n_correspondences"]
    if "max_correspondence_distance" in kw:
        assert 0 < b[3] < n


def test_held_update_mse_sequential_fallback(gpu_ctx, oracle_mod, plan):
    """PCL's default criteria with MSE terms spanning more than 53 bits: the held records restaged
    for the sequential double chain."""
    plan(solo=0)
    src, tgt = _pair(4300, 2048)
    src, tgt = src.copy(), tgt.copy()
    tgt[5, :3] = [1e-15, 0.0, 0.0]
    src[9, :3] = [0.0, 0.0, 0.0]
    import icp4r

    p = icp4r.default_params(max_iterations=12)
    b = _both(gpu_ctx, plan, src, tgt, p)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=12)
    assert (b[0] == o["T"]).all() and b[2] == o["iterations"] and b[1] == o["fitness"]


@pytest.mark.parametrize("huber", [False, True])
def test_held_update_fold_keys(gpu_ctx, oracle_mod, plan, huber):
    """The multi-tile target (scan-to-map): pass A forms the records from X and the merged keys and
    writes them for the global path."""
    import icp4r

    src, tgt = _pair(4400, 2500, 30001)
    kw = dict(huber_delta=0.5) if huber else {}
    p = icp4r.default_params(max_iterations=10, **kw)
    b = _both(gpu_ctx, plan, src, tgt, p)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, max_iterations=10, **kw)
    assert (b[0] == o["T"]).all() and b[2] == o["iterations"] and b[1] == o["fitness"]


def test_held_update_small_batch(gpu_ctx, oracle_mod, plan):
    """A ragged batch of fewer pairs than CUs (one held workgroup per pair, an 8k source beside
    them: the launch takes the form its largest source needs)."""
    import icp4r

    shapes = [(2048, 2048), (37, 500), (1409, 1800), (2112, 2000), (900, 4000), (8192, 6000)]
    pairs = [_pair(4500 + k, n, m) for k, (n, m) in enumerate(shapes)]
    src = np.concatenate([s for s, _ in pairs]).astype(np.float32)
    tgt = np.concatenate([t for _, t in pairs]).astype(np.float32)
    sn = np.array([len(s) for s, _ in pairs], np.int32)
    tn = np.array([len(t) for _, t in pairs], np.int32)
    so = np.concatenate([[0], np.cumsum(sn)[:-1]]).astype(np.int64)
    to = np.concatenate([[0], np.cumsum(tn)[:-1]]).astype(np.int64)
    p = icp4r.default_params(max_iterations=12)
    out = {}
    for held in (0, 1):
        plan(held_update=held, solo=0)
        out[held] = gpu_ctx.align_batch_host(src, so, sn, tgt, to, tn, params=p)
    assert out[0].tobytes() == out[1].tobytes()
    for k, (s, t) in enumerate(pairs):
        o = oracle_mod.align(s, t, numerics=oracle_mod.NUM_F32, max_iterations=12)
        assert (np.array(out[1][k]["T"], np.float32).reshape(4, 4).T == o["T"]).all(), k
        assert out[1][k]["iterations"] == o["iterations"], k


@pytest.mark.parametrize("n,m,kw", [(2048, 2048, {}), (8192, 8192, {"max_iterations": 20}),
                                    (3000, 5000, {"huber_delta": 0.5})])
def test_fitness_transform_in_search_identical(gpu_ctx, oracle_mod, plan, n, m, kw):
    """Round 6: on the one-tile plan the fitness pass' search forms X := final * input itself (plan
    option fit_xform, the default) instead of fitness_prep_kernel: fitness, the aligned cloud and the
    result bit-identical to fit_xform = 0 and to the oracle."""
    import icp4r

    src, tgt = _pair(4700 + n % 83, n, m)
    p = icp4r.default_params(**kw)
    out = {}
    for fx in (0, 1):
        plan(fit_xform=fx, solo=0)
        r, al = gpu_ctx.align(src, tgt, p, want_aligned=True)
        out[fx] = (r.matrix().copy(), r.fitness, r.iterations, al.view(np.uint32).copy())
    assert (out[0][0] == out[1][0]).all() and out[0][1:3] == out[1][1:3]
    assert (out[0][3] == out[1][3]).all()
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, aligned=True, **kw)
    assert out[1][1] == o["fitness"] and (out[1][0] == o["T"]).all()
    assert (out[1][3] == o["aligned"].view(np.uint32)).all()


def test_aligned_without_fitness_keeps_prep(gpu_ctx, oracle_mod, plan):
    """compute_fitness = 0 with the aligned cloud asked for: no fitness pass to form X := final *
    input in, so fitness_prep_kernel runs (fit_xform applies only with the fitness pass) — the aligned
    cloud still equals the oracle's."""
    import icp4r

    src, tgt = _pair(4800, 2048)
    p = icp4r.default_params(compute_fitness=0)
    r, al = gpu_ctx.align(src, tgt, p, want_aligned=True)
    o = oracle_mod.align(src, tgt, numerics=oracle_mod.NUM_F32, aligned=True)
    assert (r.matrix() == o["T"]).all()
    assert (al.view(np.uint32) == o["aligned"].view(np.uint32)).all()

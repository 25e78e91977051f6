"""The C-ABI library: it loads without a GPU, exports every entry point include/icp4r/icp4r.h declares,
and its host-only helpers behave (no GPU compute calls here)."""
import ctypes as C
import math
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "icp4r", "icp4r.h")
MAP_HEADER = os.path.join(ROOT, "include", "icp4r", "icp4r_map.h")
EGO_HEADER = os.path.join(ROOT, "include", "icp4r", "icp4r_ego.h")
GICP_HEADER = os.path.join(ROOT, "include", "icp4r", "icp4r_gicp.h")
MULTI_HEADER = os.path.join(ROOT, "include", "icp4r", "icp4r_multi.h")


def header_functions(path=None):
    paths = [path] if path else [HEADER, MAP_HEADER, EGO_HEADER, GICP_HEADER, MULTI_HEADER]
    names = set()
    for p in paths:
        names |= set(re.findall(r"^\s*(?:const\s+char\s*\*|int|void)\s+(icp4r_\w+)\s*\(", open(p).read(), re.M))
    return sorted(names)


def test_library_exports_every_declared_symbol():
    import icp4r

    L = icp4r.load()
    decl = header_functions()
    assert len(decl) >= 26
    for name in decl:
        assert hasattr(L, name), f"{name} declared in include/icp4r/*.h but not exported"
    assert sorted(icp4r.EXPORTED_SYMBOLS) == header_functions(HEADER)
    assert sorted(icp4r.MAP_EXPORTED_SYMBOLS) == header_functions(MAP_HEADER)
    assert sorted(icp4r.EGO_EXPORTED_SYMBOLS) == header_functions(EGO_HEADER)
    assert sorted(icp4r.GICP_EXPORTED_SYMBOLS) == header_functions(GICP_HEADER)
    assert sorted(icp4r.MULTI_EXPORTED_SYMBOLS) == header_functions(MULTI_HEADER)


def test_shard_ranges_match_split_even():
    """icp4r_shard (C ABI) is the contiguous balanced split of icp4r.dist.split_even, every pair once."""
    import icp4r
    from icp4r import dist as idist

    for P, N in ((8192, 8), (7, 3), (3, 5), (0, 2), (1024, 1)):
        blocks = [icp4r.shard(P, N, r) for r in range(N)]
        assert blocks == [idist.split_even(P, r, N) for r in range(N)]
        assert [i for b in blocks for i in b] == list(range(P))
    with pytest.raises(icp4r.ICP4RError):
        icp4r.shard(8, 2, 2)


def test_nm_shows_c_linkage():
    import icp4r

    out = subprocess.run(["nm", "-D", "--defined-only", icp4r.library_path], capture_output=True, text=True).stdout
    for name in header_functions():
        assert re.search(rf"\bT {name}$", out, re.M), name


def test_params_default_matches_pcl():
    import icp4r

    p = icp4r.default_params()
    assert p.max_iterations == 10
    assert p.min_correspondences == 3
    assert p.max_correspondence_distance == math.sqrt(sys.float_info.max)
    assert p.transformation_epsilon == 0.0
    assert p.transformation_rotation_epsilon == 0.0
    assert p.euclidean_fitness_epsilon == -sys.float_info.max
    assert p.mse_threshold_absolute == 1e-12
    assert p.numerics == icp4r.NUMERICS_PCL
    assert p.compute_fitness == 1
    assert math.isinf(p.huber_delta)
    assert p.fitness_max_range == sys.float_info.max
    L = icp4r.load()
    assert L.icp4r_abi_version() == 6
    assert b"gfx950" in L.icp4r_version()


def test_struct_layouts():
    import icp4r

    assert C.sizeof(icp4r.Result) == 96
    assert C.sizeof(icp4r.Batch) == 8 * 8 + 16
    assert icp4r.Result.fitness.offset == 64


def test_plan_geometry():
    import icp4r

    ctx = icp4r.Context(icp4r.NO_DEVICE)  # plan options without a GPU
    plan = lambda *a, **k: icp4r.plan(*a, ctx=ctx, **k)  # noqa: E731
    try:
        big = plan(1024, 8192, 8192)  # C3: pruned search, targets in LDS, one workgroup per pair
        assert big["pruned"] and big["lds"] and big["q"] == 2 and big["leaf"] == 16 and big["nn_blocks"] == 1024
        assert big["cache"] and plan(1024, 16384, 8192)["lds"]
        # the batched search's query records hold 14-bit source indices: larger sources take the tiled search
        assert not plan(1024, 16385, 8192)["lds"] and not plan(1024, 16385, 8192)["cache"]
        ctx.set_plan_option("nn_lds", 1)
        assert not plan(8, 20000, 8192)["lds"]  # ... even when forced
        ctx.reset_plan_options()
        assert not plan(1024, 8192, 8193)["lds"]  # target set larger than LDS: streamed kernel
        assert not plan(1024, 8192, 65540)["lds"] and plan(1024, 8192, 65540)["pruned"]
        c1 = plan(1, 2048, 2048)  # C1: the multi-launch plan, one tile x 16 query parts of 128
        assert c1["pruned"] and not c1["lds"] and not c1["solo"] and c1["nn_blocks"] == 16
        small = plan(1, 1024, 2048)  # up to 1024 sources: the whole registration in one workgroup
        assert small["pruned"] and not small["lds"] and small["solo"] and small["nn_blocks"] == 1
        assert plan(200, 1024, 8192)["solo"] and not plan(200, 1025, 8192)["solo"]
        assert not big["solo"] and not plan(1, 2048, 8193)["solo"]
        single = plan(1, 8192, 8192)  # C2: the multi-launch plan, one target tile x 64 query parts of 128
        assert single["pruned"] and not single["lds"] and not single["solo"] and single["nn_blocks"] == 64
        ctx.set_plan_option("tile_run", 64)  # runs of 64 queries: parts of 1024
        assert plan(1, 8192, 8192)["nn_blocks"] == 8 and plan(1, 8192, 65540)["nn_blocks"] == 72
        ctx.reset_plan_options()
        assert plan(64, 8192, 8192)["nn_blocks"] == 64 * 8  # a small batch already covers the CUs
        ctx.set_plan_option("solo", 1)  # forced: up to the cached-neighbour test's 16384 sources
        assert plan(1, 8192, 8192)["solo"] and plan(200, 16384, 8192)["solo"]
        assert not plan(200, 16385, 8192)["solo"]
        ctx.set_plan_option("solo", 0)
        assert not plan(1, 2048, 2048)["solo"] and plan(1, 2048, 2048)["nn_blocks"] == 16
        ctx.reset_plan_options()
        c5 = plan(1, 8192, 65540)  # C5: 9 target tiles of <= 8192 x 32 query parts
        assert c5["pruned"] and not c5["lds"] and not c5["solo"] and c5["nn_blocks"] == 32 * 9
        ctx.set_plan_option("nn_tile", 0)  # the streamed kernel instead
        single = plan(1, 8192, 8192)  # one query per lane, the target in 4 chunks
        assert single["pruned"] and not single["lds"] and single["q"] == 1 and single["nn_blocks"] == 32 * 4
        c5 = plan(1, 8192, 65540)  # 513 superblocks in 9 chunks of <= 64
        assert c5["pruned"] and not c5["lds"] and c5["nn_blocks"] == 32 * 9
        ctx.reset_plan_options()
        brute = plan(1024, 8192, 8192, icp4r.NN_BRUTE)
        assert not brute["pruned"] and brute["q"] == 4 and brute["splits"] == 1
        bsingle = plan(1, 8192, 8192, icp4r.NN_BRUTE)
        assert bsingle["splits"] > 1 and bsingle["nn_blocks"] >= 512
        tiny = plan(1, 10, 7)  # small target: brute force
        assert not tiny["pruned"] and tiny["q"] == 1 and tiny["splits"] == 1
        assert plan(1, 10, 7, icp4r.NN_PRUNED)["pruned"]
        # the wide update: PCL numerics only, at most one pair per CU, not with the fused cache test
        assert plan(1, 8192, 8192)["wide_update"] and plan(200, 8192, 8192)["wide_update"]
        assert not plan(1, 8192, 8192, numerics=icp4r.NUMERICS_F64)["wide_update"]
        assert not plan(1024, 8192, 8192)["wide_update"]
        # ... with the records held in registers for sources of at most 8960 points
        assert plan(1, 8960, 8192)["held_update"] and not plan(1, 8961, 8192)["held_update"]
        assert not plan(1024, 2048, 2048)["held_update"]
        ctx.set_plan_option("held_update", 0)
        assert not plan(1, 2048, 2048)["held_update"] and plan(1, 2048, 2048)["wide_update"]
        ctx.set_plan_option("held_update", 1)
        ctx.set_plan_option("wide_update", 0)
        assert not plan(1, 8192, 8192)["wide_update"]
        # the on-chip batched update: the batched plan with its fused test, sources <= 8192
        ctx.set_plan_option("res_update", 1)
        assert plan(1024, 8192, 8192)["res_update"] and not plan(1024, 8193, 8192)["res_update"]
        assert not plan(1, 8192, 8192)["res_update"]
        assert not plan(1024, 8192, 8192, numerics=icp4r.NUMERICS_F64)["res_update"]
        ctx.set_plan_option("res_update", 0)
        assert not plan(1024, 8192, 8192)["res_update"]
        # without a context: the defaults
        assert icp4r.plan(1, 8192, 8192) == icp4r.plan(1, 8192, 8192, ctx=icp4r.Context(icp4r.NO_DEVICE))
    finally:
        ctx.close()


def test_plan_options_api():
    """icp4r_set_plan_option / get / reset: every documented name is known, unknown
    names and a group count that would share a hardware queue are refused, reset restores the
    defaults, and a context without a device holds options but fails every device call."""
    import numpy as np

    import icp4r

    ctx = icp4r.Context(icp4r.NO_DEVICE)
    try:
        for name in icp4r.PLAN_OPTIONS:
            v, is_set = ctx.get_plan_option(name)
            assert not is_set, name
        assert ctx.get_plan_option("groups") == (2, False) and ctx.get_plan_option("leaf") == (16, False)
        # round-6 options: held update and in-search fitness transform on, counters opt-in
        assert ctx.get_plan_option("held_update") == (1, False)
        assert ctx.get_plan_option("fit_xform") == (1, False)
        assert ctx.get_plan_option("counters") == (0, False)
        assert ctx.get_plan_option("stage_sel") == (32, False)
        ctx.set_plan(held_update=0, counters=1)
        assert ctx.get_plan_option("held_update") == (0, True) and ctx.get_plan_option("counters") == (1, True)
        ctx.reset_plan_options()
        ctx.set_plan(groups=1, nn_cache=0)
        assert ctx.get_plan_option("groups") == (1, True) and ctx.get_plan_option("nn_cache") == (0, True)
        for bad in (("groups", 4), ("groups", 0), ("no_such_option", 1), ("xpad", -1)):
            with pytest.raises(icp4r.ICP4RError):
                ctx.set_plan_option(*bad)
        ctx.reset_plan_options()
        assert ctx.get_plan_option("groups") == (2, False)
        with pytest.raises(icp4r.ICP4RError):
            ctx.align(np.zeros((8, 4), np.float32), np.zeros((8, 4), np.float32))
    finally:
        ctx.close()
    assert icp4r.env_plan({"ICP4R_GROUPS": "1", "ICP4R_NN_CACHE": "0", "ICP4R_OTHER": "3"}) == {"groups": 1, "nn_cache": 0}


def test_library_reads_no_environment():
    """Plan choices come from icp4r_set_plan_option only: the shipped library imports no getenv
    (deployment behaviour cannot depend on the process environment)."""
    import icp4r

    out = subprocess.run(["nm", "-D", "--undefined-only", icp4r.library_path], capture_output=True, text=True).stdout
    assert "getenv" not in out, [l for l in out.splitlines() if "getenv" in l]
    assert out.strip(), "nm printed nothing"


def test_fails_loudly_without_library(tmp_path, monkeypatch):
    import icp4r

    monkeypatch.setattr(icp4r, "_lib", None)
    monkeypatch.setattr(icp4r, "library_path", str(tmp_path / "missing.so"))
    with pytest.raises(icp4r.ICP4RError):
        icp4r.load()


def test_cpp_facade_compiles():
    """include/icp4r/pcl_compat.hpp, ikd_compat.hpp and fast_gicp_compat.hpp + the reference's call
    blocks (ICP, the radar_odometry map calls and its GICP) compile and link against the library (running them needs the GPU:
    tests/test_gpu_parity.py, tests/test_map.py)."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    for exe in ("callsite", "map_callsite", "gicp_callsite"):
        assert os.access(os.path.join(ROOT, "tests", "cpp", "_build", exe), os.X_OK), exe


def test_device_float_umeyama_matches_oracle_on_host():
    """icp4r_math.hpp's float SVD/rotation compiled for the host == the oracle's, bit for bit."""
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "_build", "svd_host_check")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout

"""pytest setup: the `gpu` marker and import paths.

-m "not gpu": oracle vs golden fixtures, host logic, C-ABI library loading/exports (no GPU calls).
-m gpu:       parity of the HIP product (through the C ABI) against the oracle on a real MI355X.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for sub in ("icp-4dradar_amd", "oracle", os.path.join("tests", "golden")):
    p = os.path.join(ROOT, sub)
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN_DIR = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C ABI)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    """A context on cuda:0.  Fails (never skips) when the HIP library or the GPU is missing.

    torch's HIP runtime is brought up first (as bench.py does): tests that hand torch device tensors
    to the library need torch's runtime to be the process's first HIP initialisation."""
    import torch

    import icp4r

    torch.zeros(1, device="cuda:0")
    torch.cuda.synchronize()
    ctx = icp4r.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture
def plan(gpu_ctx):
    """Plan options (icp4r_set_plan_option) on the session's GPU context for one test: plan(groups=1,
    ...) sets them; every option is back at its default afterwards."""
    gpu_ctx.reset_plan_options()
    yield gpu_ctx.set_plan
    gpu_ctx.reset_plan_options()
